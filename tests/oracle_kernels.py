"""Test-only stand-in for the HIP kernels: the CPU oracle behind the same call surface as
`evolutionarydistributedtraining_amd.ops` (the product default). Used to exercise the
multi-rank host logic (gloo, CPU) and as the checker of the GPU runs."""
import torch


class OracleKernels:
    def __init__(self, oracle):
        self.o = oracle

    def make_slerp_plan(self, offsets, device):
        return list(offsets)

    def slerp_arena(self, plan, v0, v1, out, t, thr, eps):
        for s in range(len(plan) - 1):
            a, b = plan[s], plan[s + 1]
            out[a:b] = self.o.slerp(float(t[s]), v0[a:b], v1[a:b], thr, eps).to(out.dtype)

    def slerp_population(self, plan, members, pairs, outs, t, thr, eps, speculate=None):
        for (i, j), out in zip(pairs, outs):
            self.slerp_arena(plan, members[i], members[j], out, t, thr, eps)

    def pair_merge(self, b1, b2, m1, m2, out, mom, has, lr, mu, nesterov, momentum_in=None):
        if momentum_in is not None and mom is not None:
            mom.copy_(momentum_in)
        self.o.pair_merge(b1, b2, m1, m2, out, mom, has, lr, mu, nesterov)

    def pair_merge_population(self, children, lr, mu, nesterov):
        for ch in children:
            self.pair_merge(ch["b1"], ch["b2"], ch["m1"], ch["m2"], ch["out"], ch["momentum"], ch["has_momentum"],
                            lr, mu, nesterov, momentum_in=ch["momentum_in"])

    def outer_step(self, theta, workers, mom, has, lr, mu, nesterov):
        self.o.outer_step(theta, workers, mom, has, lr, mu, nesterov)

    def delta_partial(self, theta, workers, k_total, acc, accumulate=False):
        self.o.delta_partial(theta, workers, k_total, acc, accumulate)

    def sgd_apply(self, theta, acc, mom, has, lr, mu, nesterov):
        self.o.sgd_apply(theta, acc, mom, has, lr, mu, nesterov)


class ChunkGramKernels(OracleKernels):
    """CPU stand-in for the split population-SLERP passes (edt_slerp_needed_sums / _needed_coef /
    _blend_children) with the same chunk-table semantics: per-chunk fp64 sums (torch, one fixed
    order per chunk), per-segment sums over the chunks in order, the reference's scalar formula,
    fp32 blends. Used to test the sharded schedule's data movement on CPU (gloo / virtual ranks):
    a sharded run must equal this same arithmetic on the whole population, bit for bit.
    slerp_gram / slerp_gram_coef are the whole-population form of that arithmetic (every pair's
    sums; the library's triangle layout is a mode of the needed-sums pass since r6)."""

    def make_slerp_plan(self, offsets, device, chunk_elems=1 << 16):
        import types

        import numpy as np
        rows, first = [], []
        for s in range(len(offsets) - 1):
            first.append(len(rows))
            for x in range(offsets[s], offsets[s + 1], chunk_elems):
                rows.append((x, min(chunk_elems, offsets[s + 1] - x), s))
        first.append(len(rows))
        host = np.asarray(rows, dtype=np.int64).reshape(-1, 3)
        return types.SimpleNamespace(seg_offsets=list(offsets), chunks=torch.from_numpy(host), chunks_host=host,
                                     seg_first=first, nseg=len(offsets) - 1, nchunks=len(rows), chunk_elems=chunk_elems)

    def slerp_gram(self, members, chunks, nchunks, gram=None):
        M = len(members)
        NT = M * (M + 1) // 2
        out = torch.zeros((max(1, nchunks), NT), dtype=torch.float64) if gram is None else gram
        for c in range(nchunks):
            a, n = int(chunks[c, 0]), int(chunks[c, 1])
            xs = [m[a:a + n].double() for m in members]
            q = 0
            for i in range(M):
                for j in range(i, M):
                    out[c, q] = (xs[i] * xs[j]).sum()
                    q += 1
        return out

    def slerp_gram_coef(self, plan, gram, M, pairs, t, thr=0.9995, eps=1e-8):
        import math
        tri = {}
        q = 0
        for i in range(M):
            for j in range(i, M):
                tri[(i, j)] = q
                q += 1
        coef = torch.empty((len(pairs), plan.nseg, 2), dtype=torch.float32)
        dots = torch.empty((len(pairs), plan.nseg), dtype=torch.float32)
        for p, (i, j) in enumerate(pairs):
            lo, hi = min(i, j), max(i, j)
            for s in range(plan.nseg):
                rows = gram[plan.seg_first[s]:plan.seg_first[s + 1]]
                s00 = float(rows[:, tri[(i, i)]].sum())
                s11 = float(rows[:, tri[(j, j)]].sum())
                s01 = float(rows[:, tri[(lo, hi)]].sum())
                n0, n1 = math.sqrt(s00), math.sqrt(s11)
                d = s01 / ((n0 if n0 > eps else 1.0) * (n1 if n1 > eps else 1.0))
                tt = float(t[s])
                if abs(d) > thr:
                    c0, c1 = 1 - tt, tt
                else:
                    th = math.acos(max(-1.0, min(1.0, d)))
                    c0, c1 = math.sin(th - th * tt) / math.sin(th), math.sin(th * tt) / math.sin(th)
                coef[p, s, 0], coef[p, s, 1], dots[p, s] = c0, c1, d
        return coef, dots

    def needed_table(self, pairs, nmembers, nchunks):
        """The library's own layout (edt_slerp_needed_table is host only)."""
        from evolutionarydistributedtraining_amd import ops
        return ops.needed_table(pairs, nmembers, nchunks)

    def slerp_needed_sums(self, members, layout, chunks, nchunks, table, row0, scratch=None):
        """edt_slerp_needed_sums' contract: every used column of every block, rows [row0, row0 +
        nchunks), the same per-chunk sums as slerp_gram."""
        for b, (off, nt) in enumerate(layout.blocks):
            for c in range(nchunks):
                a, n = int(chunks[c, 0]), int(chunks[c, 1])
                for x, (i, j) in enumerate(layout.columns[b]):
                    if i >= 0:
                        table[off + (row0 + c) * nt + x] = (members[i][a:a + n].double()
                                                            * members[j][a:a + n].double()).sum()
        return table

    def slerp_needed_coef(self, plan, table, layout, t, thr=0.9995, eps=1e-8):
        """slerp_gram_coef's arithmetic on the needed table: each child's two norms and dot found
        by their members in the layout's columns."""
        where = {}
        for b, (off, nt) in enumerate(layout.blocks):
            for x, (i, j) in enumerate(layout.columns[b]):
                if i >= 0:
                    where.setdefault((i, j), (off, nt, x))
                    where.setdefault((j, i), (off, nt, x))
        col = lambda i, j: table[where[(i, j)][0]:where[(i, j)][0] + layout.nchunks * where[(i, j)][1]].view(
            layout.nchunks, where[(i, j)][1])[:, where[(i, j)][2]]
        M = layout.nmembers
        gram = torch.zeros((max(1, layout.nchunks), M * (M + 1) // 2), dtype=torch.float64)
        tri = {}
        q = 0
        for i in range(M):
            for j in range(i, M):
                tri[(i, j)] = q
                q += 1
        for (i, j) in where:
            if i <= j:
                gram[:layout.nchunks, tri[(i, j)]] = col(i, j)
        return self.slerp_gram_coef(plan, gram, M, list(layout.pairs), t, thr, eps)

    def slerp_blend_children(self, members, pairs, outs, chunks, nchunks, coef, nseg):
        for c in range(nchunks):
            a, n, s = (int(x) for x in chunks[c])
            for q, (i, j) in enumerate(pairs):
                outs[q][a:a + n] = (coef[q, s, 0] * members[i][a:a + n].float()
                                    + coef[q, s, 1] * members[j][a:a + n].float()).to(outs[q].dtype)

    def slerp_refdot(self, v0, v1, chunks, seg_first, nseg, chunk_elems, flag, ref, eps=1e-8):
        """edt_slerp_refdot's contract: the reference's fp32 dot (oracle.ref_slerp_dot, the pinned
        BLAS / numpy restatement) of each flagged segment, its elements gathered from the chunk rows."""
        val = torch.zeros(max(1, nseg), dtype=torch.float32)
        for s in range(nseg):
            if not int(flag[s]):
                continue
            rows = chunks[int(seg_first[s]):int(seg_first[s + 1])]
            a = torch.cat([v0[int(r[0]):int(r[0]) + int(r[1])] for r in rows]) if len(rows) else v0[:0]
            b = torch.cat([v1[int(r[0]):int(r[0]) + int(r[1])] for r in rows]) if len(rows) else v1[:0]
            val[s] = float(self.o.ref_slerp_dot(a.contiguous(), b.contiguous(), ref.threads, eps)[0])
        return val
