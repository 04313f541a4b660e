"""MI355X-native outer-loop sync for Evolutionary Distributed Training / DiLoCo.

Replaces the reference's Python/PyTorch-CPU hot path (BarryFutureman/EvolutionaryDistributedTraining):
  * DiLoCo outer step          EDT_LM/diloco.py:238-289           -> diloco.outer_step / OuterSync
  * EDT pairwise SGD merge     EDT_LM/train/crossover.py:150-333  -> lm_crossover
  * SLERP crossover            EDT_RL/crossover.py, EDT_EVOMERGE/train/crossover.py
                                                                   -> rl_crossover, evomerge_crossover
with fused HIP kernels for gfx950 behind the C ABI in include/edt_sync.h (libedt_sync.so).
"""
from ._lib import EdtError, load_library
from .diloco import DILOCO_DEFAULTS, DILOCO_SIM_DEFAULTS, OuterState, OuterSync, outer_step
from .params import ParamArena, ParamLayout, arena_of_module, bind_module_

__all__ = [
    "EdtError", "load_library", "OuterState", "OuterSync", "outer_step", "DILOCO_DEFAULTS",
    "DILOCO_SIM_DEFAULTS", "ParamArena", "ParamLayout", "arena_of_module", "bind_module_",
]
__version__ = "0.1.0"
