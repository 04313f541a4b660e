"""Rank-resident EDT generations: the population stays in HBM across
generations; selection, parent exchange and the merge never touch a disk.

The reference moves every individual through the shared disk each generation: the master
selects pairs from genome.json fitness values (EDT_LM/edt_sim.py:177-240, EDT_RL/edt.py:
221-272), then each worker's crossover.py loads both parents' base and trained checkpoints,
merges, and saves the child (EDT_LM/edt_sim.py:244-256 -> EDT_LM/train/crossover.py:240-315;
EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:173-201). Here:

  * members live in flat parameter arenas, `members_per_rank` of them on each rank (one process
    per GPU; every member on one GPU when the world is 1);
  * the selection runs on rank 0 with the reference's own selection functions (schedule.py,
    draw for draw) and the replicated host state (genomes, momentum flags) is broadcast;
  * child c replaces member c and is built on member c's rank; the parents it needs arrive by
    grouped point-to-point transfers (schedule.exchange_plan, RCCL send/recv over xGMI: one
    transfer per (member, destination rank));
  * the merge is the single-GPU kernel: kind="sgd" is the EDT-LM child (edt_pair_merge:
    lerp(0.5) of the bases + SGD step along the mean pseudo-gradient with the donor's outer
    momentum, EDT_LM/train/crossover.py:150-232), kind="slerp" the EDT-RL / EVOMERGE child
    (edt_slerp_merge with per-tensor t, EDT_RL/crossover.py:84-135);
  * children are written into spare arenas and swapped in after every transfer of the
    generation has completed (a parent may feed several children).

The inner loop (SFT / PPO) and fitness evaluation are the caller's: `trained(m)` / `params(m)`
are the arenas it updates (params.bind_module_ points a model's parameters into one).
"""
from __future__ import annotations

import json
import os
import random

import numpy as np
import torch
import torch.distributed as dist

from . import ops as _ops
from . import schedule
from ._lib import EdtError
from .merge import uniform_dna_crossover
from .params import ParamLayout
from .tracing import traced


class ResidentPopulation:
    """kind="sgd":   member m holds base (the generation's start weights, GenN), trained (after
                     the inner loop, the genome's mutation_path) and its outer momentum.
       kind="slerp": member m holds params (its Policy+Value keys, one segment per key) and the
                     per-segment t of the merge (`seg_t`, e.g. merge.merge_plan's t values).

    genomes: the initial genome dicts in member order (EDT-LM: {"dna": [...]};
    EDT-RL: {"env": {"env_name", "reward_dna", "agents"}}); "fitness" and "model_path" are
    filled in here ("model_path" = a per-member, per-generation id)."""

    def __init__(self, layout: ParamLayout, dtype: torch.dtype, device, genomes: list[dict],
                 kind: str = "sgd", momentum_dtype: torch.dtype | None = None, seg_t=None,
                 lr: float = 0.7, momentum: float = 0.9, nesterov: bool = True,
                 dot_threshold: float = 0.9995, eps: float = 1e-8, elitism: int = 0,
                 group=None, kernels=None, keep_previous: bool = False, slerp_chunk: int | None = None,
                 comm=None, exchange: str = "per_child", exchange_groups: int = 1, ref_dot=None):
        if kind not in ("sgd", "slerp"):
            raise ValueError(kind)
        if kind == "sgd":
            from .diloco import check_sgd_hparams
            check_sgd_hparams(lr, momentum, nesterov)
        self.kind = kind
        self.slerp_chunk = slerp_chunk          # SLERP plan chunk (elements per workgroup); None: default
        self.layout = layout
        self.dtype = dtype
        self.device = torch.device(device)
        self.kernels = kernels or _ops
        # the communicator seam (collectives.py): given, or torch.distributed when initialised
        if comm is None and dist.is_available() and dist.is_initialized():
            from .collectives import TorchCollectives
            comm = TorchCollectives(group)
        self.comm = comm
        self.distributed = comm is not None
        self.world = comm.world if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.P = len(genomes)
        if self.P == 0 or self.P % self.world:
            raise EdtError(f"population {self.P} does not split over {self.world} ranks")
        self.M = self.P // self.world
        # exchange="sharded": one member per rank, the generation's data path link-balanced
        # (distributed.ShardedPopulationCrossover: chunk-range shards of every member, children
        # gathered back) instead of shipping each child's two parents whole
        if exchange not in ("per_child", "sharded"):
            raise ValueError(exchange)
        if exchange == "sharded" and (self.M != 1 or keep_previous or comm is None):
            raise EdtError("exchange='sharded' needs one member per rank, a communicator, no keep_previous")
        self.exchange = exchange
        self.exchange_groups = exchange_groups      # sharded SLERP: exchanges pipelined over chunk groups
        self._sharded = None
        self.lr, self.momentum, self.nesterov = lr, momentum, nesterov
        self.dot_threshold, self.eps = dot_threshold, eps
        # SLERP: ops.RefDot = the reference host's own dots and coefficients (bit for bit, band < 0)
        self.ref_dot = ref_dot
        self.elitism = elitism
        self.generation = 0
        self.genomes = [dict(g) for g in genomes]
        self.has_momentum = [False] * self.P
        self._fitness = None
        # keep_previous: generation N-1 stays resident as members P..2P-1, so the selection can
        # draw parents from it (EDT_LM/edt.py:226-247: tournament over current + previous)
        self.keep_previous = keep_previous
        self.prev_genomes = None
        self.prev_has_momentum = [False] * self.P
        n = layout.total
        mdt = momentum_dtype or dtype
        if mdt != dtype:
            # the pair merge writes the child momentum in the child's dtype (edt_pair_merge,
            # ops.pair_merge checks it), so a separate momentum dtype could never cross over
            raise EdtError(f"momentum_dtype {mdt} must equal the member dtype {dtype}")

        def arena(dt):
            return torch.zeros(n, dtype=dt, device=self.device)

        self._slot = {m: m - self.rank * self.M for m in self.local_members()}
        if kind == "sgd":
            self._base = [arena(dtype) for _ in range(self.M)]
            self._trained = [arena(dtype) for _ in range(self.M)]
            self._mom = [arena(mdt) if momentum else None for _ in range(self.M)]
            self._child = [arena(dtype) for _ in range(self.M)]
            self._child_mom = [arena(mdt) if momentum else None for _ in range(self.M)]
            if keep_previous:
                self._pbase = [arena(dtype) for _ in range(self.M)]
                self._ptrained = [arena(dtype) for _ in range(self.M)]
                self._pmom = [arena(mdt) if momentum else None for _ in range(self.M)]
        else:
            if seg_t is None or len(seg_t) != len(layout):
                raise EdtError("kind='slerp' needs one t per tensor of the layout (seg_t)")
            self._params = [arena(dtype) for _ in range(self.M)]
            self._child = [arena(dtype) for _ in range(self.M)]   # RN to the member dtype (bf16: :142)
            if keep_previous:
                self._pparams = [arena(dtype) for _ in range(self.M)]
            self._t = torch.tensor([float(t) for t in seg_t], dtype=torch.float64).to(self.device)
            self._plan = None
        self._recv = {}

    # ---- member access ---------------------------------------------------------------------
    def local_members(self) -> list[int]:
        return list(range(self.rank * self.M, (self.rank + 1) * self.M))

    def owner(self, m: int) -> int:
        """Rank holding member m (m >= P: member m - P of the previous generation)."""
        return (m % self.P) // self.M

    def _local(self, m):
        if m % self.P not in self._slot or (m >= self.P and not self.keep_previous):
            raise EdtError(f"member {m} lives on rank {self.owner(m)}, not {self.rank}")
        return self._slot[m % self.P]

    def base(self, m: int) -> torch.Tensor:
        return self._base[self._local(m)]

    def trained(self, m: int) -> torch.Tensor:
        return self._trained[self._local(m)]

    def outer_momentum(self, m: int) -> torch.Tensor | None:
        return self._mom[self._local(m)]

    def params(self, m: int) -> torch.Tensor:
        return self._params[self._local(m)]

    def begin_inner(self) -> None:
        """Start every local member's inner loop from its base (mutation.py trains a copy of
        GenN; at generation 0 the reference copies Gen0000 to Gen0000_mutated)."""
        if self.kind == "sgd":
            for b, t in zip(self._base, self._trained):
                t.copy_(b)

    def model_path(self, m: int, generation: int | None = None) -> str:
        g = self.generation if generation is None else generation
        return f"member{m}/Gen{g:04d}"

    # ---- selection (rank 0, broadcast) -----------------------------------------------------
    def _sync_host(self, obj):
        if self.world == 1:
            return obj
        return self.comm.broadcast_object(obj, src=0)

    @traced("edt/ResidentPopulation.select")
    def select(self, fitness: list[float], method: str | None = None, scale: float | None = None):
        """Parent pairs (member indices) for the next generation, chosen on rank 0.

        sgd:   edt_sim.py:233-240: rank_based_selection of P - elitism pairs, then (elite,
               elite) pairs for the top `elitism` genomes; a population of one pairs with itself.
        slerp: EDT_RL/edt.py:267-272: roulette_wheel_selection of P pairs with
               scale = roulette_scale(generation, max_generations) (pass `scale`).
        method="tournament_pool" (EDT_LM/edt.py:213-247, the distributed master): tournament
               selection over this generation and the previous one (needs keep_previous=True;
               pair indices >= P name previous-generation members), elites from this one."""
        if len(fitness) != self.P:
            raise EdtError(f"{len(fitness)} fitness values for {self.P} members")
        pairs = None
        if self.rank == 0:
            genomes = []
            for m, (g, f) in enumerate(zip(self.genomes, fitness)):
                g = dict(g)
                g["fitness"] = f
                g["model_path"] = self.model_path(m)
                genomes.append(g)
            method = method or ("rank" if self.kind == "sgd" else "roulette")
            if method == "tournament_pool" and not self.keep_previous:
                raise EdtError("tournament_pool selection needs keep_previous=True")
            if self.P == 1:
                sel = [(genomes[0], genomes[0])]
            elif method == "rank":
                sel = schedule.rank_based_selection(genomes, self.P - self.elitism)
                ranked = sorted(genomes, key=lambda g: g["fitness"], reverse=True)
                sel += [(e, e) for e in ranked[:self.elitism]]
            elif method == "roulette":
                sel = schedule.roulette_wheel_selection(genomes, self.P, 1.0 if scale is None else scale)
            elif method == "tournament":
                sel = schedule.tournament_selection(genomes, self.P)
            elif method == "tournament_pool":
                # EDT_LM/edt.py:226-247: tournament over this generation + the previous one, then
                # (elite, elite) pairs from this generation
                pool = genomes + (list(self.prev_genomes) if self.prev_genomes is not None else [])
                sel = schedule.tournament_selection(pool, self.P - self.elitism)
                ranked = sorted(genomes, key=lambda g: g["fitness"], reverse=True)
                sel += [(e, e) for e in ranked[:self.elitism]]
                genomes = pool
            else:
                raise ValueError(method)
            pairs = schedule.pair_indices(sel, genomes)
            self._fitness = list(fitness)
        pairs = self._sync_host(pairs)
        return [tuple(p) for p in pairs]

    # ---- crossover -------------------------------------------------------------------------
    def _donors(self, pairs):
        """Whose outer momentum child c inherits (EDT_LM/train/crossover.py:183-227): parent 1's
        when it has one, else parent 2's; none at generation 0; otherwise an error."""
        out = []
        has = self.has_momentum + self.prev_has_momentum
        for i, j in pairs:
            if has[i]:
                out.append(i)
            elif has[j]:
                out.append(j)
            elif self.generation == 0 or self.momentum == 0:
                out.append(None)
            else:
                raise NotImplementedError(f"What, no outer_optim.pt for {self.model_path(i)} or {self.model_path(j)}?")
        return out

    def _payload(self, m, with_state):
        s, prev = self._local(m), m >= self.P
        if self.kind == "slerp":
            return [(self._pparams if prev else self._params)[s]]
        out = [(self._pbase if prev else self._base)[s], (self._ptrained if prev else self._trained)[s]]
        if with_state:
            out.append((self._pmom if prev else self._mom)[s])
        return out

    def _recv_like(self, key, like):
        buf = self._recv.get(key)
        if buf is None or buf.dtype != like.dtype or buf.numel() != like.numel():
            buf = self._recv[key] = torch.empty_like(like)
        return buf

    def _exchange(self, pairs, donors):
        """Grouped send/recv of every parent a local child needs; {member: [tensors]}."""
        nmem = 2 * self.P if self.prev_genomes is not None else self.P
        owner = [self.owner(m) for m in range(nmem)]
        child_rank = [self.owner(c) for c in range(self.P)]
        have = [m for m in range(nmem) if owner[m] == self.rank]
        if self.world == 1:
            return {m: self._payload(m, True) for m in have}
        plan = schedule.exchange_plan(pairs, owner, child_rank)
        mine = plan.get(self.rank, {"send": [], "recv": []})

        def with_state(m, dst):
            return self.kind == "sgd" and any(donors[c] == m and child_rank[c] == dst for c in range(self.P))

        p2p = []
        for m, dst in mine["send"]:
            for t in self._payload(m, with_state(m, dst)):
                p2p.append(("send", t, dst))
        got = {m: self._payload(m, True) for m in have}
        like = self._payload(self.local_members()[0], self.kind == "sgd")
        for slot, (m, src) in enumerate(mine["recv"]):
            n = len(like) if with_state(m, self.rank) else (1 if self.kind == "slerp" else 2)
            bufs = [self._recv_like((slot, k), like[k]) for k in range(n)]
            p2p.extend(("recv", b, src) for b in bufs)
            got[m] = bufs
        self.comm.p2p(p2p)
        return got

    @traced("edt/ResidentPopulation.crossover")
    def crossover(self, pairs, child_hook=None) -> None:
        """Build child c of pairs[c] = (i, j) on member c's rank, for every c, then make the
        children the population (generation + 1). child_hook(c, genome), on rank 0 right after
        child c's genome is made (in child order), is where a master does its per-child host work
        in the reference's draw order — e.g. EDT_RL/edt.py:290-294 sets genome["env"]["agents"]
        with random.sample after each crossover() call."""
        pairs = [tuple(p) for p in pairs]
        if len(pairs) != self.P:
            raise EdtError(f"{len(pairs)} pairs for a population of {self.P}")
        donors = self._donors(pairs) if self.kind == "sgd" else [None] * self.P
        if self.exchange == "sharded":
            self._sharded_children(pairs)
        else:
            got = self._exchange(pairs, donors)
            if self.kind == "slerp":
                self._slerp_children(pairs, got)
            else:
                self._sgd_children(pairs, got, donors)
        # every transfer and merge of this generation is enqueued/complete: swap the children in
        # (keep_previous: the current generation becomes the previous one, whose arenas are
        # recycled for the next children)
        if self.kind == "sgd" and self.keep_previous:
            self._pbase, self._base, self._child = self._base, self._child, self._pbase
            self._ptrained, self._trained = self._trained, self._ptrained
            if self.momentum:
                self._pmom, self._mom, self._child_mom = self._mom, self._child_mom, self._pmom
        elif self.kind == "sgd":
            self._base, self._child = self._child, self._base
            if self.momentum:
                self._mom, self._child_mom = self._child_mom, self._mom
        elif self.keep_previous:
            self._pparams, self._params, self._child = self._params, self._child, self._pparams
        else:
            self._params, self._child = self._child, self._params
        if self.keep_previous:
            self.prev_has_momentum = list(self.has_momentum)
        self._genomes_after(pairs, child_hook)
        if self.kind == "sgd" and self.momentum:
            self.has_momentum = [True] * self.P
        self.generation += 1

    def _sgd_children(self, pairs, got, donors):
        """EDT-LM merge of every local child: the donor's momentum buffer is read in place (it may
        feed other children; has = False at generation 0: the first step writes buf =
        grad.clone() without reading). Up to 16 local children go in ONE launch whose
        workgroups share an XCD per chunk, so a parent that feeds several children crosses HBM
        once (ops.pair_merge_population); bit-identical to one pair_merge per child."""
        k = self.kernels
        local = self.local_members()
        children = []
        for c in local:
            i, j = pairs[c]
            s = self._local(c)
            has = donors[c] is not None and self.momentum != 0
            children.append({"b1": got[i][0], "b2": got[j][0], "m1": got[i][1], "m2": got[j][1],
                             "out": self._child[s], "momentum": self._child_mom[s],
                             "momentum_in": got[donors[c]][2] if has else None, "has_momentum": has})
        if hasattr(k, "pair_merge_population") and len(children) <= 16:
            k.pair_merge_population(children, self.lr, self.momentum, self.nesterov)
            return
        for ch in children:
            k.pair_merge(ch["b1"], ch["b2"], ch["m1"], ch["m2"], ch["out"], ch["momentum"], ch["has_momentum"],
                         self.lr, self.momentum, self.nesterov, momentum_in=ch["momentum_in"])

    def _slerp_children(self, pairs, got):
        """SLERP every local child in one population call (ops.slerp_population, bit-identical to
        one edt_slerp_merge per child): shared parents are read once per pass — by the Gram stats
        pass (<= 8 distinct parents) or the speculative co-located pass, which ops picks from the
        previous generation's dots (parents of one lineage take the lerp branch: one pass). More
        than 8 distinct parents: the speculative form (<= 16 local children), else per child."""
        k = self.kernels
        if self._plan is None:
            self._plan = k.make_slerp_plan(self.layout.offsets, self.device,
                                           **({"chunk_elems": self.slerp_chunk} if self.slerp_chunk else {}))
        local = self.local_members()
        srcs = sorted({m for c in local for m in pairs[c]})
        where = {m: q for q, m in enumerate(srcs)}
        args = (self._plan, [got[m][0] for m in srcs], [(where[pairs[c][0]], where[pairs[c][1]]) for c in local],
                [self._child[self._local(c)] for c in local], self._t, self.dot_threshold, self.eps)
        rd = {"ref_dot": self.ref_dot} if self.ref_dot is not None else {}
        if hasattr(k, "slerp_population") and len(srcs) <= 8:
            k.slerp_population(*args, **rd)
            return
        if hasattr(k, "slerp_population") and len(local) <= 16:
            k.slerp_population(*args, speculate=True, **rd)
            return
        for c in local:
            i, j = pairs[c]
            k.slerp_arena(self._plan, got[i][0], got[j][0], self._child[self._local(c)], self._t,
                          self.dot_threshold, self.eps, **rd)

    def _sharded_children(self, pairs):
        """This rank's child through the link-balanced schedule (bit-identical to the per-child
        kernels)."""
        from .distributed import ShardedPopulationCrossover
        if self._sharded is None:
            self._sharded = ShardedPopulationCrossover(self.layout, self.dtype, self.device, kind=self.kind,
                                                       comm=self.comm, kernels=self.kernels,
                                                       chunk_elems=self.slerp_chunk or (1 << 16),
                                                       groups=self.exchange_groups)
        m = self.rank
        if self.kind == "slerp":
            self._sharded.slerp_step(self._params[0], pairs, self._t, self._child[0], self.dot_threshold, self.eps,
                                     ref_dot=self.ref_dot)
            return
        has = self.has_momentum[m] and self.momentum != 0
        self._sharded.pair_merge_step(self._base[0], self._trained[0], self._mom[0] if has else None, pairs,
                                      self._child[0], self._child_mom[0], self.lr, self.momentum, self.nesterov,
                                      has_momentum=has, generation=self.generation)

    def _pool_genome(self, m):
        """Genome of member m as the master sees it at selection time: current members with this
        generation's fitness and model path, previous members (m >= P) as recorded then."""
        if m >= self.P:
            return dict(self.prev_genomes[m - self.P])
        g = dict(self.genomes[m])
        g["model_path"] = self.model_path(m)
        if self._fitness is not None:
            g["fitness"] = self._fitness[m]
        return g

    def _genomes_after(self, pairs, child_hook=None):
        """Child genomes (rank 0, numpy's global RNG, child order; broadcast): EDT-LM
        {"fitness": 0, "dna", "p1", "p2"} with the parents' own p1/p2 dropped
        (EDT_LM/train/crossover.py:296-309; EDT_EVOMERGE/train/crossover.py:214-227 for SLERP
        children of DNA genomes); EDT-RL {"env": {env_name, reward_dna, agents: []},
        "p1", "p2"} (EDT_RL/crossover.py:186-201; parents' p1/p2 dropped here too, so the record
        stays one level deep). keep_previous: this generation's genomes (with fitness) become
        the previous generation's."""
        new = None
        if self.rank == 0:
            children = []
            for c, (i, j) in enumerate(pairs):
                g1, g2 = self._pool_genome(i), self._pool_genome(j)
                for g in (g1, g2):
                    g.pop("p1", None)
                    g.pop("p2", None)
                if "env" not in g1:         # EDT-LM and EVOMERGE (SLERP children, DNA genomes)
                    child = {"fitness": 0.0, "model_path": self.model_path(c, self.generation + 1),
                             "dna": uniform_dna_crossover(g1["dna"], g2["dna"]), "p1": g1, "p2": g2}
                else:                           # EDT-RL: reward DNA in the env record
                    env = g1["env"]
                    child = {"model_path": self.model_path(c, self.generation + 1),
                             "env": {"env_name": env["env_name"],
                                     "reward_dna": uniform_dna_crossover(env["reward_dna"], g2["env"]["reward_dna"]),
                                     "agents": []},
                             "p1": g1, "p2": g2}
                if child_hook is not None:
                    child_hook(c, child)
                children.append(child)
            prev = [self._pool_genome(m) for m in range(self.P)] if self.keep_previous else None
            new = (children, prev)
        self.genomes, prev = self._sync_host(new)
        if self.keep_previous:
            self.prev_genomes = prev

    # ---- persistence (resume a resident run) ------------------------------------------------
    def _member_tensors(self, m):
        s = self._local(m)
        if self.kind == "slerp":
            out = [("params", self._params[s])]
            if self.keep_previous and self.prev_genomes is not None:
                out.append(("prev_params", self._pparams[s]))
            return out
        out = [("base", self._base[s]), ("trained", self._trained[s])]
        if self._mom[s] is not None:
            out.append(("outer_momentum", self._mom[s]))
        if self.keep_previous and self.prev_genomes is not None:
            out += [("prev_base", self._pbase[s]), ("prev_trained", self._ptrained[s])]
            if self._pmom[s] is not None:
                out.append(("prev_outer_momentum", self._pmom[s]))
        return out

    def _names(self):
        return self.layout.names or [f"param.{i}" for i in range(len(self.layout))]

    def save(self, path: str, rng: bool = True) -> None:
        """Every local member's arenas as safetensors checkpoints under
        path/member{m}/{base,trained,outer_momentum | params}/model.safetensors, and (rank 0)
        path/population.json: generation, genomes, momentum flags and, with rng=True, the
        states of the host RNGs the selection and DNA crossover draw from (python `random`,
        numpy's global RNG), so a resumed run continues draw for draw. The reference keeps
        this state in RAM and on the shared disk between its scripts (genome.json per dir,
        outer_optim.pt per individual)."""
        from concurrent.futures import ThreadPoolExecutor
        from .checkpoint import write_from_arena
        names = self._names()
        tasks = []
        for m in self.local_members():
            for tag, t in self._member_tensors(m):
                d = os.path.join(path, f"member{m}", tag)
                os.makedirs(d, exist_ok=True)
                tasks.append((os.path.join(d, "model.safetensors"), t))
        # one writer thread per file (the page cache takes one file at ~11-12 GB/s, several at
        # once far faster: profiles/r06_e2e_sharded_write.jsonl), each ordered after the caller's
        # current stream, which produced the arenas
        dev = tasks[0][1].device if tasks else None
        caller = torch.cuda.current_stream(dev) if dev is not None and dev.type == "cuda" else None

        def one(task):
            target, t = task
            if caller is not None:
                with torch.cuda.device(t.device), torch.cuda.stream(caller):
                    write_from_arena(target, self.layout, t, names)
            else:
                write_from_arena(target, self.layout, t, names)
        with ThreadPoolExecutor(max_workers=max(1, min(8, len(tasks)))) as ex:
            list(ex.map(one, tasks))
        if self.rank == 0:
            meta = {"kind": self.kind, "population": self.P, "generation": self.generation,
                    "genomes": self.genomes, "has_momentum": self.has_momentum,
                    "prev_genomes": self.prev_genomes, "prev_has_momentum": self.prev_has_momentum}
            if rng:
                st = random.getstate()
                ns = np.random.get_state()
                meta["rng"] = {"python": [st[0], list(st[1]), st[2]],
                               "numpy": [ns[0], ns[1].tolist(), int(ns[2]), int(ns[3]), float(ns[4])]}
            os.makedirs(path, exist_ok=True)
            with open(os.path.join(path, "population.json.tmp"), "w") as f:
                json.dump(meta, f)
            os.replace(os.path.join(path, "population.json.tmp"), os.path.join(path, "population.json"))
        if self.world > 1:
            self.comm.barrier()

    def load(self, path: str, rng: bool = True) -> None:
        """Restore what save() wrote (same layout, kind and population; any world size that
        divides the population: each rank reads its own members)."""
        from .checkpoint import read_into_arena
        with open(os.path.join(path, "population.json")) as f:
            meta = json.load(f)
        if meta["kind"] != self.kind or meta["population"] != self.P:
            raise EdtError(f"{path} holds a {meta['kind']} population of {meta['population']}")
        self.generation = meta["generation"]
        self.genomes = meta["genomes"]
        self.has_momentum = list(meta["has_momentum"])
        if self.keep_previous:
            self.prev_genomes = meta.get("prev_genomes")
            self.prev_has_momentum = list(meta.get("prev_has_momentum") or [False] * self.P)
        names = self._names()
        for m in self.local_members():
            for tag, t in self._member_tensors(m):
                read_into_arena(os.path.join(path, f"member{m}", tag), self.layout, t, names)
        if rng and "rng" in meta and self.rank == 0:
            py = meta["rng"]["python"]
            random.setstate((py[0], tuple(py[1]), py[2]))
            ns = meta["rng"]["numpy"]
            np.random.set_state((ns[0], np.asarray(ns[1], dtype=np.uint32), ns[2], ns[3], ns[4]))

    # ---- mutation schedule (host) ----------------------------------------------------------
    def mutation_flags(self, probability: float = 0.5) -> list[bool]:
        """Which children mutate their DNA this generation (EDT_LM/edt_sim.py:282-296: shuffle
        the machines with `random.shuffle`, flag the first round(p * P)); chosen on rank 0."""
        flags = None
        if self.rank == 0:
            order = list(range(self.P))
            random.shuffle(order)
            k = max(1, int(round(probability * self.P)))
            chosen = set(order[:k])
            flags = [m in chosen for m in range(self.P)]
        flags = self._sync_host(flags)
        for g, f in zip(self.genomes, flags):
            g["dna_mutated"] = f
        return flags

    def step(self, fitness: list[float], child_hook=None, **select_kw):
        """One generation's data path: select -> exchange -> merge -> swap. Returns the pairs."""
        pairs = self.select(fitness, **select_kw)
        self.crossover(pairs, child_hook)
        return pairs
