"""Test-only stand-in for the HIP kernels: the CPU oracle behind the same call surface as
`evolutionarydistributedtraining_amd.ops` (the product default). Used to exercise the
multi-rank host logic (gloo, CPU) and as the checker of the GPU runs."""


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
