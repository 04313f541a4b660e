"""Drop-in replacement for EDT_EVOMERGE/train/crossover.py (worker side of EDT_EVOMERGE/edt.py:262-280).
Same CLI and functions; the SLERP runs on the MI355X. Requires the repo root on PYTHONPATH."""
from evolutionarydistributedtraining_amd.evomerge_crossover import *  # noqa: F401,F403
from evolutionarydistributedtraining_amd.evomerge_crossover import main

if __name__ == "__main__":
    main()
