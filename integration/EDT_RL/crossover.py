"""Drop-in replacement for EDT_RL/crossover.py: EDT_RL/edt.py:6 does `from crossover import crossover`
and calls it in-process (:290). Same functions; the SLERP runs on the MI355X.
Requires the repo root on PYTHONPATH."""
from evolutionarydistributedtraining_amd.rl_crossover import *  # noqa: F401,F403
