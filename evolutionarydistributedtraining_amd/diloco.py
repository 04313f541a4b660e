"""DiLoCo outer step on MI355X — the drop-in for EDT_LM/diloco.py:238-289 (== diloco_sim.py:233-299).

Reference behaviour (per parameter tensor i, worker-major, torch CPU ops):
    acc_i = 0;  for k in trained_models: acc_i += (theta_k,i - theta_g,i) / K
    p.grad = -acc_i
    torch.optim.SGD(lr, momentum, nesterov).step()          # single-tensor path
with the SGD object carried across generations by `load_state_dict` (diloco.py:258-286), so the
momentum buffer survives the base model being reloaded. Defaults: diloco.py lr 0.7, momentum 0.9,
nesterov True (:253-255); diloco_sim.py lr 1.0, momentum 0.0, nesterov False (:248-250).

Here the whole step is ONE fused HIP launch over flat parameter arenas (see `ops.outer_step`).
`outer_step()` keeps the reference's tensor-list surface; `OuterSync` is the arena-native form
the benchmark and the multi-GPU path use.
"""
from __future__ import annotations

import os

import torch

from . import ops
from ._lib import EDT_MAX_WORKERS as L_MAX, EdtError
from .params import ParamArena, ParamLayout, flat_view, pack, unpack_
from .tracing import traced

DILOCO_DEFAULTS = dict(lr=0.7, momentum=0.9, nesterov=True)        # EDT_LM/diloco.py:253-255


def check_sgd_hparams(lr: float, momentum: float, nesterov: bool) -> None:
    """The argument checks torch.optim.SGD's constructor makes (the reference builds one per outer
    step, EDT_LM/diloco.py:253-257, EDT_LM/train/crossover.py:185-230), with its messages."""
    if lr < 0.0:
        raise ValueError(f"Invalid learning rate: {lr}")
    if momentum < 0.0:
        raise ValueError(f"Invalid momentum value: {momentum}")
    if nesterov and momentum <= 0:
        raise ValueError("Nesterov momentum requires a momentum and zero dampening")
DILOCO_SIM_DEFAULTS = dict(lr=1.0, momentum=0.0, nesterov=False)   # EDT_LM/diloco_sim.py:248-250


class OuterState:
    """The outer optimiser's state across generations: one flat momentum buffer in
    `parameters()` order — what the reference keeps in the master's `outer_optimizer`
    (EDT_LM/diloco.py:100,258-289). Also serialises to the torch `SGD.state_dict()` format
    (`outer_optim.pt`, as EDT_LM/train/crossover.py:231-232 writes per individual)."""

    def __init__(self, place_momentum: int = 0):
        self.momentum: torch.Tensor | None = None   # flat, dtype of theta_g
        self.has_momentum = False                   # False until the first momentum step
        self.hparams = dict(DILOCO_DEFAULTS)
        self.steps = 0
        # > 1: when outer_step creates the buffer over flat arenas (parameters bound with
        # params.arena_of_module, so they stay where they are across generations), choose its HBM
        # placement among this many candidates by measurement first (placement.place_momentum,
        # as OuterSync.place_momentum / DirOuterSync do). The tensor-list form skips it: reloaded
        # parameter tensors move, so no placement can hold.
        self.place_momentum = int(place_momentum)
        self.placement: dict | None = None

    def buffer_for(self, theta: torch.Tensor, numel: int | None = None) -> torch.Tensor:
        """The flat momentum for parameters like `theta` (numel: total count when theta is
        only the first of a tensor list)."""
        numel = theta.numel() if numel is None else numel
        if self.momentum is None:
            self.momentum = torch.zeros(numel, dtype=theta.dtype, device=theta.device)
            self.has_momentum = False
        elif self.momentum.numel() != numel:
            raise EdtError("outer-optimizer state does not match the parameter count "
                           f"({self.momentum.numel()} vs {numel})")
        elif self.momentum.dtype != theta.dtype or self.momentum.device != theta.device:
            # torch's load_state_dict casts state to the param's dtype/device
            self.momentum = self.momentum.to(dtype=theta.dtype, device=theta.device)
        return self.momentum

    # --- torch.optim.SGD state_dict interop (index-keyed, as load_state_dict carries it) ---
    def state_dict(self, layout: ParamLayout) -> dict:
        state = {}
        if self.momentum is not None and self.has_momentum:
            for i, v in enumerate(layout.views(self.momentum)):
                state[i] = {"momentum_buffer": v.detach().to("cpu", copy=True)}
        group = dict(lr=self.hparams["lr"], momentum=self.hparams["momentum"], dampening=0,
                     weight_decay=0, nesterov=self.hparams["nesterov"], maximize=False,
                     foreach=None, differentiable=False, fused=None,
                     params=list(range(len(layout))))
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd: dict, layout: ParamLayout, dtype: torch.dtype, device) -> None:
        group = sd["param_groups"][0]
        self.hparams = dict(lr=group["lr"], momentum=group["momentum"], nesterov=group["nesterov"])
        bufs = [sd["state"].get(i, {}).get("momentum_buffer") for i in range(len(layout))]
        if all(b is None for b in bufs):
            self.momentum, self.has_momentum = None, False
            return
        if any(b is None for b in bufs):
            raise EdtError("partial momentum state is not supported (every parameter needs a buffer)")
        flat = torch.empty(layout.total, dtype=dtype, device=device)
        for v, b in zip(layout.views(flat), bufs):
            v.copy_(b)
        self.momentum, self.has_momentum = flat, True

    def save(self, path: str, layout: ParamLayout) -> None:
        torch.save(self.state_dict(layout), path)

    @classmethod
    def load(cls, path: str, layout: ParamLayout, dtype, device) -> "OuterState":
        st = cls()
        st.load_state_dict(torch.load(path, map_location="cpu", weights_only=True), layout, dtype, device)
        return st


def _tail_bits(cpu_tails, numels, device, state=None, per_tensor=False):
    """cpu_tails = (vec_elems, num_threads) of the reference's host -> the device bitmask of its
    torch scalar-tail elements (torchcompat), or None. per_tensor: the tensor-list form's masks
    ((bits, byte offsets), each tensor's from a byte boundary). With `state` the mask is kept on it
    for the next generation (it depends only on the sizes and the host model; building it walks
    every element once on the CPU)."""
    if cpu_tails is None:
        return None
    key = (tuple(int(n) for n in numels), tuple(cpu_tails), str(device), per_tensor)
    cached = getattr(state, "_tail_cache", None) if state is not None else None
    if cached is not None and cached[0] == key:
        return cached[1]
    from .torchcompat import torch_cpu_tail_bits, torch_cpu_tail_bits_per_tensor
    vec, threads = cpu_tails
    if per_tensor:
        got = torch_cpu_tail_bits_per_tensor(numels, vec_elems=vec, num_threads=threads, device=device)
    else:
        got = torch_cpu_tail_bits(numels, vec_elems=vec, num_threads=threads, device=device)
    if state is not None:
        state._tail_cache = (key, got)
    return got


def _step_flat(theta: torch.Tensor, workers: list[torch.Tensor], state: OuterState, lr: float,
               momentum: float, nesterov: bool, broadcast: list[torch.Tensor] | None = None,
               tail_bits: torch.Tensor | None = None) -> None:
    check_sgd_hparams(lr, momentum, nesterov)
    state.hparams = dict(lr=lr, momentum=momentum, nesterov=nesterov)
    fresh = state.momentum is None
    mom = state.buffer_for(theta) if momentum != 0 else None
    if mom is not None and fresh and getattr(state, "place_momentum", 0) > 1 and theta.is_cuda:
        from .placement import place_momentum
        try:
            state.momentum, state.placement = place_momentum(theta, workers, mom, state.place_momentum)
            mom = state.momentum
        except EdtError as e:                   # e.g. operands the probe cannot stream (alignment)
            state.placement = {"candidates": 1, "probe_ms": [], "chosen": 0, "skipped": str(e)}
    has = state.has_momentum if momentum != 0 else False
    if tail_bits is not None and broadcast:              # the tail form has no fused broadcast
        ops.outer_step(theta, workers, mom, has, lr, momentum, nesterov, tail_bits=tail_bits)
        for b in broadcast:
            b.copy_(theta)
    else:
        ops.outer_step(theta, workers, mom, has, lr, momentum, nesterov, broadcast, tail_bits=tail_bits)
    if momentum != 0:
        state.has_momentum = True
    state.steps += 1


def _step_list(thetas: list[torch.Tensor], workers: list[list[torch.Tensor]], state: OuterState,
               lr: float, momentum: float, nesterov: bool, tails=None) -> None:
    check_sgd_hparams(lr, momentum, nesterov)
    state.hparams = dict(lr=lr, momentum=momentum, nesterov=nesterov)
    moms = None
    if momentum != 0:
        flat = state.buffer_for(thetas[0], sum(t.numel() for t in thetas))
        shapes = [t.shape for t in thetas]
        cached = getattr(state, "_list_views", None)      # the per-tensor views of the buffer,
        if cached is not None and cached[0] is flat and cached[1] == shapes:   # kept across calls
            moms = cached[2]
        else:
            moms = ParamLayout.of(thetas).views(flat)
            state._list_views = (flat, shapes, moms)
    ops.outer_step_list(thetas, workers, moms, state.has_momentum if momentum != 0 else False,
                        lr, momentum, nesterov, tails=tails)
    if momentum != 0:
        state.has_momentum = True
    state.steps += 1


def outer_step(base_params, worker_params, state: OuterState | None = None, lr: float = 0.7,
               momentum: float = 0.9, nesterov: bool = True, cpu_tails: tuple[int, int] | None = None) -> OuterState:
    """Drop-in for EDT_LM/diloco.py:238-289 on device-resident parameters.

    base_params:   list of the global model's parameters (`list(base_model.parameters())`),
                   updated in place.
    worker_params: K lists of the trained replicas' parameters, same order.
    state:         the carried outer-optimiser state (None on the first generation).
    One launch either way: over the flat arenas when each list is a run of views of one arena
    (`params.arena_of_module`), else over the tensor lists themselves (`ops.outer_step_list`,
    no packing). Only populations above 64 workers with separate tensors are packed first.
    cpu_tails = (Vec::size(), torch threads) of the reference's master, e.g. (32, 8): bf16 results
    bit-exact with the reference run there, torch's scalar tails included (torchcompat; r5: the
    tensor-list form reads per-tensor masks, edt_outer_step_list_tail, so nothing is packed; the
    masks are kept on `state` across generations).
    """
    state = state or OuterState()
    base_params = list(base_params)
    worker_params = [list(w) for w in worker_params]
    if not worker_params:
        raise EdtError("no trained models")
    shapes = [p.shape for p in base_params]
    for w in worker_params:
        if [a.shape for a in w] != shapes:
            raise EdtError("trained model parameters do not match the base model")
    with torch.no_grad():
        theta = flat_view(base_params)
        flats = [flat_view(w) for w in worker_params]
        if theta is None or any(f is None for f in flats):
            bf16_master = base_params and base_params[0].dtype == torch.bfloat16
            if (cpu_tails is None or bf16_master) and len(worker_params) <= L_MAX and base_params \
                    and all(p.is_cuda for p in base_params):
                if len({w[0].dtype for w in worker_params}) != 1:
                    raise EdtError("all trained models must share one dtype")
                tails = _tail_bits(cpu_tails, [p.numel() for p in base_params], base_params[0].device, state,
                                   per_tensor=True)
                _step_list(base_params, worker_params, state, lr, momentum, nesterov, tails=tails)
                return state
        copied = theta is None
        if copied:
            theta = pack(base_params)
        flats = [f if f is not None else pack(w) for f, w in zip(flats, worker_params)]
        wdt = {f.dtype for f in flats}
        if len(wdt) != 1:
            raise EdtError("all trained models must share one dtype")
        _step_flat(theta, flats, state, lr, momentum, nesterov,
                   tail_bits=_tail_bits(cpu_tails, [p.numel() for p in base_params], theta.device, state))
        if copied:
            unpack_(theta, base_params)
    return state


class OuterSync:
    """Arena-native DiLoCo outer step for a population resident in HBM.

    theta:   global parameters (master) — float32 or bfloat16 arena
    workers: K replica arenas (bfloat16 or float32) the inner loops trained
    """

    def __init__(self, theta: ParamArena, workers: list[ParamArena], lr: float = 0.7,
                 momentum: float = 0.9, nesterov: bool = True, state: OuterState | None = None,
                 cpu_tails: tuple[int, int] | None = None):
        self.theta = theta
        self.workers = workers
        self.lr, self.momentum, self.nesterov = lr, momentum, nesterov
        self.state = state or OuterState()
        # (Vec::size(), threads) of the reference's host: its bf16 scalar tails (outer_step's doc)
        self.tail_bits = _tail_bits(cpu_tails, theta.layout.numels, theta.flat.device)

    @traced("edt/OuterSync.step")
    def step(self, broadcast: bool = False) -> None:
        """One outer step. broadcast=True also starts every worker from the new global weights
        (EDT_LM/diloco.py:302-308) in the same pass: each worker arena is overwritten with theta
        rounded to its dtype right after the kernel has read it (edt_outer_step_bcast)."""
        ws = [w.flat for w in self.workers]
        _step_flat(self.theta.flat, ws, self.state, self.lr, self.momentum, self.nesterov,
                   ws if broadcast else None, tail_bits=self.tail_bits)

    def place_momentum(self, candidates: int = 8) -> dict:
        """Choose where the outer momentum lives in HBM by measurement, once, for the life of
        the run (placement.place_momentum: the step's two read-modify-write streams conflict
        or not depending on their relative physical placement). Creates the buffer if the
        first step has not run yet; contents and semantics are unchanged."""
        if self.momentum == 0:
            return {"candidates": 0, "probe_ms": [], "chosen": None}
        from .placement import place_momentum
        mom = self.state.buffer_for(self.theta.flat)
        self.state.momentum, rep = place_momentum(self.theta.flat, [w.flat for w in self.workers], mom,
                                                  candidates)
        return rep

    def place_arenas(self, draws: int = 3, candidates: int = 8) -> dict:
        """Choose where the whole operand set lives — θ, the workers and the outer momentum — by
        measurement, once, for the life of the run (placement.place_set: `draws` regions of HBM,
        the momentum placed inside each). The arenas are re-pointed at the chosen buffers with
        their contents unchanged; a module bound to an arena (params.bind_module_) must be bound
        again afterwards. With draws = 1 this is place_momentum."""
        if self.momentum == 0:
            return {"draws": [], "chosen_draw": None}
        from .placement import place_set
        mom = self.state.buffer_for(self.theta.flat)
        th, ws, m, rep = place_set(self.theta.flat, [w.flat for w in self.workers], mom, draws, candidates)
        self.theta.flat = th
        for w, f in zip(self.workers, ws):
            w.flat = f
        self.state.momentum = m
        return rep

    def broadcast_(self) -> None:
        """Start every worker from the new global weights (what saving base_model to every
        worker dir does, EDT_LM/diloco.py:302-308) as K device copies; step(broadcast=True) does
        the same inside the step's pass."""
        for w in self.workers:
            w.flat.copy_(self.theta.flat)

    @property
    def bytes_reduced(self) -> int:
        """Metric bytes of one step: K x P x bytes per worker element."""
        return sum(w.flat.numel() * w.flat.element_size() for w in self.workers)

    def traffic_bytes(self) -> int:
        """Algorithmic HBM bytes of one fused step: every operand read once / written once."""
        n = self.theta.flat.numel()
        b = self.bytes_reduced + 2 * n * self.theta.flat.element_size()
        if self.momentum != 0:
            b += (2 if self.state.has_momentum else 1) * n * self.theta.flat.element_size()
        return b


class DirOuterSync:
    """The whole outer step of EDT_LM/diloco.py:224-308 on checkpoint directories, with no HF
    model objects: the base (GenN of worker 0) and the K trained replicas (GenN+1) are read
    straight into HBM arenas (checkpoint.read_into_arena), the fused kernel runs, and the new
    global weights are written to every worker's GenN+1 dir (checkpoint.save_to_dirs) together
    with the base dir's config/tokenizer files. Arenas and the outer state persist across
    generations, so the momentum carry of diloco.py:258-286 needs no state_dict round trip.

    names: parameter names in `model.parameters()` order (e.g. `ParamLayout.of_module(model).names`)
    — the index order of the momentum; default: the checkpoint's own tensor order.
    state_path: the outer optimiser's state file (torch `SGD.state_dict()` format, as
    `outer_optim.pt`): loaded before the first step when it exists and rewritten after every step,
    so a restarted master resumes the momentum carry (the reference keeps it in RAM only,
    EDT_LM/diloco.py:100).
    carry_inner_state: EDT_LM/diloco.py:295-300 — before the new weights are written, each
    worker's previous-generation `optimizer.pt` / `scheduler.pt` (step(prev_dirs=...), GenN of
    every machine) is copied over the one its inner loop left in its GenN+1 dir, where it exists,
    so the next inner loop resumes the inner optimiser as the reference's does — into the dirs the
    new weights go to (out_dirs; the reference writes them over worker_dirs, its default here).
    place_momentum: after the first step, choose the outer momentum's HBM placement by measurement
    once among this many candidates (OuterSync.place_momentum; 0 or 1 = keep the first allocation).
    The θ and worker arenas stay resident across generations here (the checkpoints are read into
    them), so the choice holds for the rest of the run. On by default (r4): the first
    allocation ran the step 8-11 % slower in about half of the bench runs, and the search costs
    0.19 s once at 1.3B x 8 bf16. place_draws > 1 (r6): also draw the whole resident set (θ, the
    worker arenas, the momentum) in that many regions of HBM (placement.place_set). Off by default
    here: a generation through checkpoint files takes ~1 s, of which the step is 12 ms, and three
    draws cost 1.79 s once (profiles/r06_e2e_checkpoint_publish.jsonl) — OuterSync.place_arenas is
    the resident kernel loop's form."""

    INNER_STATE_FILES = ("optimizer.pt", "scheduler.pt")

    def __init__(self, device=None, theta_dtype=None, worker_dtype=None, names=None,
                 lr=0.7, momentum=0.9, nesterov=True, state: OuterState | None = None,
                 state_path: str | None = None, carry_inner_state: bool = False, place_momentum: int = 8,
                 place_draws: int = 1):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.theta_dtype, self.worker_dtype, self.names = theta_dtype, worker_dtype, names
        self.lr, self.momentum, self.nesterov = lr, momentum, nesterov
        self.state = state or OuterState()
        self.layout = None
        self.theta = None
        self.workers: list[ParamArena] = []
        self._written: set[str] = set()     # dirs holding the resident theta (last step's output)
        self.state_path = state_path
        self.carry_inner_state = carry_inner_state
        self.place_candidates = place_momentum
        self.place_draws = place_draws
        self.placement = None             # the placement search's report, once it has run

    def _layout_from(self, model_dir):
        from .checkpoint import checkpoint_files, read_header, _ST_DTYPES
        files = checkpoint_files(model_dir)
        metas = {}
        for path in set(files.values()):
            h, base = read_header(path)
            for k, v in h.items():
                if k != "__metadata__":
                    metas[k] = (path, v)
        names = self.names or sorted(metas, key=lambda k: (metas[k][0], metas[k][1]["data_offsets"][0]))
        dt = _ST_DTYPES[metas[names[0]][1]["dtype"]]
        return ParamLayout([tuple(metas[n][1]["shape"]) for n in names], names), dt

    @traced("edt/DirOuterSync.step")
    def step(self, base_dir: str, worker_dirs: list[str], out_dirs: list[str] | None = None,
             prev_dirs: list[str] | None = None) -> OuterState:
        """base_dir: GenN of worker 0 (the base); worker_dirs: GenN+1 of every worker (trained);
        out_dirs: where the new weights go (default: worker_dirs, as the reference); prev_dirs:
        GenN of every worker, whose inner optimiser / scheduler files are carried into
        worker_dirs when carry_inner_state is set (EDT_LM/diloco.py:295-300)."""
        import shutil
        from .checkpoint import copy_file, read_many, save_to_dirs
        if self.carry_inner_state and (prev_dirs is None or len(prev_dirs) != len(worker_dirs)):
            raise ValueError("carry_inner_state needs prev_dirs: the previous generation dir of every worker")
        if self.layout is None:
            self.layout, ckpt_dt = self._layout_from(base_dir)
            self.theta_dtype = self.theta_dtype or ckpt_dt
            self.worker_dtype = self.worker_dtype or ckpt_dt
            self.theta = ParamArena(self.layout, self.theta_dtype, self.device)
            if self.state_path and os.path.exists(self.state_path) and self.state.momentum is None:
                self.state = OuterState.load(self.state_path, self.layout, self.theta_dtype, self.device)
        while len(self.workers) < len(worker_dirs):
            self.workers.append(ParamArena(self.layout, self.worker_dtype, self.device))
        items = [(d, arena.flat) for d, arena in zip(worker_dirs, self.workers)]
        if os.path.abspath(base_dir) not in self._written:   # else theta is already resident
            items.insert(0, (base_dir, self.theta.flat))
        read_many(items, self.layout, self.names)        # the K + 1 checkpoints read in parallel
        workers = [w.flat for w in self.workers[:len(worker_dirs)]]
        _step_flat(self.theta.flat, workers, self.state, self.lr, self.momentum, self.nesterov)
        if self.place_candidates > 1 and self.placement is None and self.momentum != 0 \
                and self.theta.flat.device.type == "cuda":
            import time
            from .placement import place_set
            t0 = time.perf_counter()
            th, ws, m, self.placement = place_set(self.theta.flat, workers, self.state.momentum,
                                                  max(1, self.place_draws), self.place_candidates)
            torch.cuda.synchronize(th.device)
            self.placement["seconds"] = round(time.perf_counter() - t0, 3)     # once per run
            self.theta.flat, self.state.momentum = th, m
            for arena, flat in zip(self.workers, ws):
                arena.flat = flat
            workers = ws
        out_dirs = worker_dirs if out_dirs is None else out_dirs
        if self.carry_inner_state:          # diloco.py:295-300, before the model write as there
            # beside the weights the next inner loop loads: out_dirs (== worker_dirs in the reference)
            for source, target in zip(prev_dirs, out_dirs):
                os.makedirs(target, exist_ok=True)
                for fname in self.INNER_STATE_FILES:
                    src = os.path.join(source, fname)
                    if os.path.exists(src):
                        copy_file(src, os.path.join(target, fname))
        save_to_dirs(out_dirs, self.layout, self.theta.flat)
        if self.state_path:                  # durable carry: write-then-rename
            self.state.save(self.state_path + ".tmp", self.layout)
            os.replace(self.state_path + ".tmp", self.state_path)
        self._written = {os.path.abspath(d) for d in out_dirs}
        for d in out_dirs:                  # config / generation config / tokenizer of the base
            for f in os.listdir(base_dir):
                src = os.path.join(base_dir, f)
                if os.path.isfile(src) and not f.startswith("model.safetensors") and f not in (
                        "genome.json", "optimizer.pt", "scheduler.pt", "outer_optim.pt"):
                    if os.path.abspath(src) != os.path.abspath(os.path.join(d, f)):
                        shutil.copyfile(src, os.path.join(d, f))
        return self.state
