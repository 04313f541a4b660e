"""Drop-in replacement for EDT_LM/train/crossover.py (worker side of EDT_LM/edt.py and
edt_sim.py, which run `python crossover.py --model1_path A --model2_path B --output_path O` in
the worker's train/ dir). Same CLI, same functions; the merge runs on the MI355X.
Requires the repo root on PYTHONPATH."""
from evolutionarydistributedtraining_amd.lm_crossover import *  # noqa: F401,F403
from evolutionarydistributedtraining_amd.lm_crossover import main

if __name__ == "__main__":
    main()
