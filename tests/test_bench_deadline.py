"""bench.py's multi-GPU safety net (ExtrasDeadline): the line is printed exactly once, by rank 0,
with the value and every extra that finished, whether the extras complete or hang past the
deadline; other ranks print nothing; the deadline makes every rank exit with a non-zero status
(a hang must read as a failed run)."""
import io
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _line(buf):
    lines = [l for l in buf.getvalue().splitlines() if l.strip()]
    assert len(lines) == 1, lines
    return json.loads(lines[0])


def test_deadline_fires_once_with_the_value_and_finished_extras():
    out = {"value": 123.0, "cpu_baseline": {"value": 1.0}, "weak_scaling": {"ms_per_step": 2.0}}
    buf, exited, codes = io.StringIO(), threading.Event(), []
    d = bench.ExtrasDeadline(0.2, 0, out, buf, exit_fn=lambda code: (codes.append(code), exited.set()))
    assert exited.wait(5)
    assert codes == [3]
    line = _line(buf)
    assert line["value"] == 123.0 and line["weak_scaling"] == {"ms_per_step": 2.0}
    assert line["extras_deadline"]["unfinished_or_skipped"] == ["parity", "other_schedules", "baseline_configs",
                                                                "population_slerp_7b"]
    assert d.emit() is False            # the main thread arriving later prints nothing more
    assert len(buf.getvalue().splitlines()) == 1


def test_extras_in_time_print_one_line_and_cancel():
    out = {"value": 1.0}
    buf, exited = io.StringIO(), threading.Event()
    d = bench.ExtrasDeadline(0.3, 0, out, buf, exit_fn=lambda code: exited.set())
    out["other_schedules"] = {}
    assert d.emit() is True
    d.cancel()
    time.sleep(0.5)
    assert not exited.is_set()
    line = _line(buf)
    assert "extras_deadline" not in line and line["other_schedules"] == {}


def test_other_ranks_never_print_but_exit_on_the_deadline():
    buf, exited, codes = io.StringIO(), threading.Event(), []
    d = bench.ExtrasDeadline(0.1, 3, None, buf, exit_fn=lambda code: (codes.append(code), exited.set()))
    assert exited.wait(5)
    assert codes == [3]
    assert d.emit() is False and buf.getvalue() == ""


def test_no_deadline():
    buf = io.StringIO()
    d = bench.ExtrasDeadline(0, 0, {"value": 2.0}, buf, exit_fn=lambda code: None)
    assert d.timer is None
    assert d.emit() and _line(buf)["value"] == 2.0
