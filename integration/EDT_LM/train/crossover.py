"""Drop-in replacement for EDT_LM/train/crossover.py (worker side of EDT_LM/edt.py and
edt_sim.py, which run `python crossover.py --model1_path A --model2_path B --output_path O` in
the worker's train/ dir). Same CLI, same functions; the merge runs on the MI355X.
Copy this file over the reference's; the repo root must be on PYTHONPATH or in EDT_SYNC_ROOT
(see INTEGRATION.md)."""
import os
import sys

try:                                   # the package on sys.path already, or EDT_SYNC_ROOT = the repo root
    import evolutionarydistributedtraining_amd  # noqa: F401
except ImportError:
    _root = os.environ.get("EDT_SYNC_ROOT")
    if not _root:
        raise ImportError("edt-sync-mi355x not importable: put the repo root on PYTHONPATH or set EDT_SYNC_ROOT")
    sys.path.insert(0, _root)
from evolutionarydistributedtraining_amd.lm_crossover import *  # noqa: E402,F401,F403
from evolutionarydistributedtraining_amd.lm_crossover import main  # noqa: E402

if __name__ == "__main__":
    main()
