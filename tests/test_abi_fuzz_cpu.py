"""Fuzz of the C ABI's argument validation (include/edt_sync.h), host side only: every call carries
exactly one invalid argument — an unknown dtype code, an unsupported dtype pair, a worker / partial /
child count out of range, a negative chunk or segment count, a null buffer where data is due — and
must come back with a negative code and the matching message in edt_last_error(), before any HIP
call (pointers are host addresses that are never dereferenced). The reference raises at the same
points (Python exceptions: EDT_LM/diloco.py:238-289 would fail on mismatched tensors,
EDT_LM/train/crossover.py:227 on a missing momentum). Runs without a GPU."""
import ctypes

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

FUZZ = settings(max_examples=150, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
P = ctypes.c_void_p
F32, BF16 = 0, 1


@pytest.fixture(scope="module")
def lib():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host-pointer fuzz: CPU-only (a device run would launch on host addresses)")
    from evolutionarydistributedtraining_amd import _lib
    return _lib.load_library()


_host = (ctypes.c_uint8 * 65536)()
_base = ctypes.addressof(_host)


def fake(i):
    return P(_base + 64 * (i + 1))            # distinct, 16-byte aligned, never dereferenced


def arr(ptrs):
    return (P * max(1, len(ptrs)))(*ptrs)


def _expect(lib, rc, needle):
    msg = lib.edt_last_error().decode()
    assert rc < 0, (rc, msg)
    assert needle in msg, (needle, msg)


bad_dtype = st.one_of(st.integers(2, 1000), st.integers(-1000, -1))


@FUZZ
@given(kind=st.sampled_from(["gdt", "wdt", "pair", "K_low", "K_high", "theta", "worker", "momentum"]),
       K=st.integers(1, 64), n=st.integers(1, 1 << 40), bad=bad_dtype, mu=st.floats(0.01, 0.99),
       which=st.integers(0, 63))
def test_outer_step_rejects(lib, kind, K, n, bad, mu, which):
    gdt, wdt, theta, mom = F32, BF16, fake(0), fake(1)
    ws = [fake(2 + k) for k in range(K)]
    needle = "dtype"
    if kind == "gdt":
        gdt = bad
    elif kind == "wdt":
        wdt = bad
    elif kind == "pair":
        gdt, wdt = BF16, F32                       # bf16 master with fp32 replicas: not a reference regime
    elif kind == "K_low":
        K, needle = -abs(which), "worker count"
    elif kind == "K_high":
        K, needle = 65 + which, "worker count"
        ws = [fake(2 + k) for k in range(K)]
    elif kind == "theta":
        theta, needle = None, "theta_g is null"
    elif kind == "worker":
        ws[which % K], needle = None, f"theta_k[{which % K}] is null"
    else:
        mom, needle = None, "momentum buffer is null"
    rc = lib.edt_outer_step(theta, gdt, arr(ws), wdt, K, mom, 1, n, 0.7, mu, 1, None)
    _expect(lib, rc, needle)


@FUZZ
@given(kind=st.sampled_from(["gdt", "nacc_low", "nacc_high", "theta", "acc", "acc_entry", "momentum"]),
       nacc=st.integers(1, 64), n=st.integers(1, 1 << 36), bad=bad_dtype, which=st.integers(0, 63))
def test_sgd_apply_sum_rejects(lib, kind, nacc, n, bad, which):
    gdt, theta, mom = F32, fake(0), fake(1)
    accs = [fake(2 + r) for r in range(nacc)]
    acc_arr = arr(accs)
    needle = "dtype"
    if kind == "gdt":
        gdt = bad
    elif kind == "nacc_low":
        nacc, needle = -which, "partial count"
    elif kind == "nacc_high":
        nacc, needle = 65 + which, "partial count"
        acc_arr = arr([fake(2 + r) for r in range(nacc)])
    elif kind == "theta":
        theta, needle = None, "null buffer"
    elif kind == "acc":
        acc_arr, needle = None, "null buffer"
    elif kind == "acc_entry":
        accs[which % nacc] = None
        acc_arr, needle = arr(accs), f"acc_f32[{which % nacc}] is null"
    else:
        mom, needle = None, "momentum buffer is null"
    rc = lib.edt_sgd_apply_sum(theta, gdt, ctypes.cast(acc_arr, ctypes.POINTER(P)) if acc_arr is not None else None,
                               nacc, mom, 1, n, 0.7, 0.9, 1, None)
    _expect(lib, rc, needle)


@FUZZ
@given(kind=st.sampled_from(["in_dt", "out_dt", "negative", "null"]), entry=st.sampled_from(["stats", "blend", "merge"]),
       nchunks=st.integers(1, 1 << 30), neg=st.integers(-(1 << 40), -1), bad=bad_dtype)
def test_slerp_passes_reject(lib, kind, entry, nchunks, neg, bad):
    in_dt, out_dt, v0 = BF16, BF16, fake(0)
    needle = "dtype"
    if kind == "in_dt":
        in_dt = bad
    elif kind == "out_dt":
        if entry == "stats":
            in_dt = bad                           # stats has no output dtype
        else:
            out_dt = bad
    elif kind == "negative":
        nchunks, needle = neg, "negative"
    else:
        v0, needle = None, "null buffer"
    if entry == "stats":
        rc = lib.edt_slerp_stats(v0, fake(1), in_dt, fake(2), nchunks, fake(3), None)
    elif entry == "blend":
        rc = lib.edt_slerp_blend(v0, fake(1), in_dt, fake(2), out_dt, fake(3), nchunks, fake(4), None)
    else:
        rc = lib.edt_slerp_merge(v0, fake(1), in_dt, fake(2), out_dt, fake(3), nchunks, fake(4), 1, fake(5),
                                 0.9995, 1e-8, fake(6), fake(7), None, None)
    _expect(lib, rc, needle)


@FUZZ
@given(kind=st.sampled_from(["wdt", "pair", "null_b1", "null_out", "momentum", "momentum_in"]),
       n=st.integers(1, 1 << 36), bad=bad_dtype)
def test_pair_merge_rejects(lib, kind, n, bad):
    wdt, gdt = BF16, BF16
    b1, out, mom, mom_in = fake(0), fake(4), fake(5), fake(6)
    needle = "dtype"
    if kind == "wdt":
        wdt = bad
    elif kind == "pair":
        wdt, gdt = F32, BF16
    elif kind == "null_b1":
        b1, needle = None, "null buffer"
    elif kind == "null_out":
        out, needle = None, "null buffer"
    elif kind == "momentum":
        mom, needle = None, "momentum buffer is null"
    else:
        mom_in, needle = None, "carried momentum is null"
    rc = lib.edt_pair_merge_to(b1, fake(1), fake(2), fake(3), wdt, out, gdt, mom_in, mom, 1, n, 0.7, 0.9, 1, None)
    _expect(lib, rc, needle)


def test_success_clears_the_message(lib):
    """edt_last_error() is cleared by the next call that succeeds (an empty call returns 0)."""
    _expect(lib, lib.edt_outer_step(fake(0), 7, arr([fake(1)]), F32, 1, fake(2), 1, 8, 0.7, 0.9, 1, None), "dtype")
    assert lib.edt_outer_step(None, F32, arr([None]), F32, 1, None, 0, 0, 0.7, 0.0, 0, None) == 0
    assert lib.edt_last_error() == b""


def _table(lib, ptrs0, ptrs1, ptrso, sizes, apart, in_dt=F32, out_dt=F32):
    n = len(sizes)
    arr = lambda xs: (ctypes.c_void_p * max(1, n))(*xs)
    numel = (ctypes.c_uint64 * max(1, n))(*sizes)
    host = (ctypes.c_uint64 * max(1, 3 * n))()
    rc = lib.edt_slerp_seg_table(arr(ptrs0), arr(ptrs1), arr(ptrso), n, numel, in_dt, out_dt, apart,
                                 ctypes.cast(host, ctypes.c_void_p))
    return rc, list(host)


def test_seg_table_host_checks(lib):
    """edt_slerp_seg_table (a host function): the {v0, v1, out} image in order; a misaligned tensor
    refused; with apart = 1 every output byte range checked against every parent's (sorted spans):
    an output inside ANOTHER tensor's parent, a partial overlap or an output equal to its own parent
    refused, disjoint outputs accepted, empty tensors ignored."""
    base = 1 << 40
    p0, p1, po = [base, base + 4096], [base + 8192, base + 12288], [base + 16384, base + 20480]
    sizes = [1000, 1000]                                   # 4000 bytes each (fp32)
    rc, host = _table(lib, p0, p1, po, sizes, 1)
    assert rc == 0 and host == [p0[0], p1[0], po[0], p0[1], p1[1], po[1]]
    assert _table(lib, [base + 4], p1[:1], po[:1], [10], 0)[0] < 0              # not 16-byte aligned
    assert _table(lib, p0, p1, [p0[0], po[1]], sizes, 1)[0] < 0                   # out == own parent
    assert _table(lib, p0, p1, [po[0], p1[0]], sizes, 1)[0] < 0                   # out = another's parent
    assert _table(lib, p0, p1, [po[0], p1[1] + 2048], sizes, 1)[0] < 0             # partial overlap
    assert b"overlaps a parent" in lib.edt_last_error()
    assert _table(lib, p0, p1, [p0[0], po[1]], sizes, 0)[0] == 0                  # two-pass: allowed
    assert _table(lib, p0, p1, [p1[0], po[1]], [0, 1000], 1)[0] == 0              # empty spans ignored
    # bf16 outputs are half the bytes: one right after the last parent's end, the next right after it
    assert _table(lib, p0, p1, [p1[1] + 4000, p1[1] + 6000], [1000, 1000], 1, F32, BF16)[0] == 0
    assert _table(lib, p0, p1, [p1[1] + 3984, p1[1] + 6000], [1000, 1000], 1, F32, BF16)[0] < 0


def test_abi_version_matches_the_binding(lib):
    from evolutionarydistributedtraining_amd import _lib as L
    assert lib.edt_abi_version() == L.EDT_ABI_VERSION == 6
