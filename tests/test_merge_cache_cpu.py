"""merge_models_into_'s binding cache: an entry holds the last references to memory its
last merge read (model_2's tensors, model_1's previous buffer), so it is dropped only after the event
recorded behind that merge — on whatever stream and device the merge ran — has completed. Host
logic only: a stand-in event records the order."""
from evolutionarydistributedtraining_amd import merge


class _Ev:
    def __init__(self, log):
        self.log = log

    def synchronize(self):
        self.log.append("sync")


class _Entry:
    def __init__(self, log):
        self.done = _Ev(log)
        self.hold2 = object()


def test_evict_waits_for_the_last_merge_then_drops():
    log = []
    cache = {"k": _Entry(log)}

    class _Watch(dict):
        def pop(self, key, default=None):
            log.append(("pop", key))
            return super().pop(key, default)
    cache = _Watch(cache)
    merge._evict(cache, "k")
    assert log == [("pop", "k"), "sync"] and "k" not in cache


def test_evict_of_an_absent_or_unlaunched_entry():
    merge._evict({}, "missing")                       # nothing to wait for
    cache = {"k": object()}                           # an entry without a recorded merge
    merge._evict(cache, "k")
    assert cache == {}


def test_evict_survives_a_runtime_that_is_gone():
    class _Dead:
        def synchronize(self):
            raise RuntimeError("HIP runtime shut down")

    class _E:
        done = _Dead()
    cache = {"k": _E()}
    merge._evict(cache, "k")                          # interpreter exit: no exception escapes
    assert cache == {}
