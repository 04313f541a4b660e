"""Drop-in replacement for EDT_RL/crossover.py: EDT_RL/edt.py:6 does `from crossover import crossover`
and calls it in-process (:290). Same functions (slerp, lerp, normalize, interpolate_t,
run_slerp_merge_from_config, run_slerp_merge, crossover); the SLERP runs on the MI355X.
Copy this file over the reference's; the repo root must be on PYTHONPATH or in EDT_SYNC_ROOT."""
import os
import sys

try:                                   # the package on sys.path already, or EDT_SYNC_ROOT = the repo root
    import evolutionarydistributedtraining_amd  # noqa: F401
except ImportError:
    _root = os.environ.get("EDT_SYNC_ROOT")
    if not _root:
        raise ImportError("edt-sync-mi355x not importable: put the repo root on PYTHONPATH or set EDT_SYNC_ROOT")
    sys.path.insert(0, _root)
from evolutionarydistributedtraining_amd.rl_crossover import *  # noqa: E402,F401,F403
