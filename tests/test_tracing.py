"""roctx ranges (tracing.py): the library loads on this host, ranges nest and pop, and the
decorated shim functions still return their results; EDT_ROCTX=0 turns them into no-ops."""
import subprocess
import sys

from evolutionarydistributedtraining_amd import tracing


def test_roctx_ranges_nest():
    assert tracing.available()
    with tracing.trange("edt/test/outer"):
        with tracing.trange("edt/test/inner"):
            pass

    @tracing.traced("edt/test/fn")
    def f(x):
        return x + 1
    assert f(1) == 2 and f.__name__ == "f"


def test_roctx_can_be_disabled():
    code = ("import os; os.environ['EDT_ROCTX']='0'; from evolutionarydistributedtraining_amd import tracing as t; "
            "assert not t.available()\nwith t.trange('x'): pass\nprint('ok')")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.stdout.strip() == "ok", p.stderr
