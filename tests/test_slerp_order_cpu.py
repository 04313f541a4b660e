"""oracle.canonical_chunk_sums (the checker tests/test_gpu_slerp_order.py holds the kernels to):
its sums are the true dot products to fp64 accuracy, and its order is the one documented — a
hand-built case where the order is visible in the last bit."""
import numpy as np
import torch


def test_canonical_sums_are_the_dot_products(oracle):
    g = torch.Generator().manual_seed(3)
    n = 200003
    x, y = torch.randn(n, generator=g), torch.randn(n, generator=g)
    chunks = [(0, 65536, 0), (65536, 65536, 0), (131072, 65536, 0), (196608, 3395, 0), (3, 77, 1)]
    got = oracle.canonical_chunk_sums(x, y, chunks)
    xd, yd = x.double().numpy(), y.double().numpy()
    for (s, ln, _), row in zip(chunks, got):
        want = [xd[s:s + ln] @ xd[s:s + ln], yd[s:s + ln] @ yd[s:s + ln], xd[s:s + ln] @ yd[s:s + ln]]
        assert np.allclose(row, want, rtol=1e-12, atol=1e-12)


def test_canonical_order_is_lane_chain_then_butterfly_then_tile_tree(oracle):
    """1.0 in element 0 of lane 0 of tile 0 and 2^-53 spread so that only the documented order
    keeps or drops them: lane 1 of tile 0 holds eight 2^-54 (its chain sums them exactly to
    2^-51, then the butterfly adds that to lane 0's 1.0 at level 1: kept); element 512 (tile 1)
    holds 2^-27 (square 2^-54, added to tile 0's sum in the tree: dropped by rounding)."""
    x = np.zeros(1024, np.float32)
    x[0] = 1.0
    x[8:16] = np.float32(2.0 ** -27)                  # lane 1 of tile 0: squares 2^-54 each
    x[512] = np.float32(2.0 ** -27)                   # tile 1, lane 0
    got = oracle.canonical_chunk_sums(torch.from_numpy(x), torch.from_numpy(x), [(0, 1024, 0)])
    assert got[0, 0] == 1.0 + 2.0 ** -51              # lane 1's chain 8 x 2^-54 = 2^-51 survives
