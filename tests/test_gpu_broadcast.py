"""edt_outer_step_bcast (ops.outer_step(..., broadcast=...)): the DiLoCo step fused with the
broadcast of EDT_LM/diloco.py:302-308 — theta and the momentum bit-identical to the plain fused
step, and every broadcast buffer equal to the new theta rounded to the worker dtype (torch
copy_, RNE), whether the buffers are the workers themselves (read, then overwritten) or separate
arenas; vector and scalar (misaligned) bodies."""
import pytest
import torch

from evolutionarydistributedtraining_amd import ops
from evolutionarydistributedtraining_amd._lib import EdtError
from evolutionarydistributedtraining_amd.diloco import OuterSync
from evolutionarydistributedtraining_amd.params import ParamArena, ParamLayout

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int16)


def _data(n, K, tdt, wdt, off=0):
    g = torch.Generator().manual_seed(n + K)
    th = (torch.randn(n + off, generator=g) * 0.02).to(tdt).to(DEV)[off:]
    ws = [(th.float().cpu() + torch.randn(n, generator=g) * 1e-3).to(wdt).to(DEV) for _ in range(K)]
    if off:
        ws = [torch.cat([torch.zeros(off, dtype=wdt, device=DEV), w])[off:] for w in ws]
    mom = (torch.randn(n + off, generator=g) * 1e-3).to(tdt).to(DEV)[off:]
    return th, ws, mom


@pytest.mark.parametrize("tdt,wdt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("K", [1, 3, 8, 16])
@pytest.mark.parametrize("n,off", [(1_000_003, 0), (40_961, 1)])
@pytest.mark.parametrize("into", ["workers", "separate"])
def test_step_bcast_matches_step_then_copy(tdt, wdt, K, n, off, into):
    th, ws, mom = _data(n, K, tdt, wdt, off)
    th2, ws2, mom2 = th.clone(), [w.clone() for w in ws], mom.clone()
    ops.outer_step(th2, ws2, mom2, True, 0.7, 0.9, True)
    want = th2.to(wdt)
    dst = ws if into == "workers" else [torch.full_like(w, float("nan")) for w in ws[:max(1, K // 2)]]
    ops.outer_step(th, ws, mom, True, 0.7, 0.9, True, broadcast=dst)
    torch.cuda.synchronize()
    assert torch.equal(_bits(th), _bits(th2))
    assert torch.equal(_bits(mom), _bits(mom2))
    for d in dst:
        assert torch.equal(_bits(d), _bits(want))


def test_outer_sync_step_broadcast_two_generations():
    """OuterSync.step(broadcast=True) == step() + broadcast_(), carried momentum, two steps."""
    lay = ParamLayout([(257, 33), (5,), (4097,)])
    a = [ParamArena(lay, torch.float32, DEV), [ParamArena(lay, torch.bfloat16, DEV) for _ in range(4)]]
    b = [ParamArena(lay, torch.float32, DEV), [ParamArena(lay, torch.bfloat16, DEV) for _ in range(4)]]
    g = torch.Generator(device=DEV).manual_seed(3)
    th0 = torch.randn(lay.total, generator=g, device=DEV) * 0.02
    s1, s2 = OuterSync(a[0], a[1]), OuterSync(b[0], b[1])
    for x in (a, b):
        x[0].flat.copy_(th0)
    for gen in range(2):
        noise = [torch.randn(lay.total, generator=g, device=DEV) * 1e-3 for _ in range(4)]
        for x in (a, b):
            for w, nz in zip(x[1], noise):
                w.flat.copy_((x[0].flat + nz) if gen == 0 else (w.flat.float() + nz))
        s1.step(broadcast=True)
        s2.step()
        s2.broadcast_()
        torch.cuda.synchronize()
        assert torch.equal(_bits(a[0].flat), _bits(b[0].flat))
        for w1, w2 in zip(a[1], b[1]):
            assert torch.equal(_bits(w1.flat), _bits(w2.flat))


def test_bcast_rejects_theta_overlap():
    th, ws, mom = _data(4096, 2, torch.float32, torch.float32)
    with pytest.raises(EdtError, match="overlaps"):
        ops.outer_step(th, ws, mom, True, 0.7, 0.9, True, broadcast=[th])
