"""Fused Adam / SGD over a flat parameter arena (drop-ins for torch.optim.Adam / SGD,
main.py:114-120).

On first use the optimizer moves every parameter of each group into one fp32 arena
(``p.data`` becomes a view, same shape and strides, so modules and ``state_dict`` are
unchanged), points ``p.grad`` at views of a flat gradient buffer, and keeps exp_avg /
exp_avg_sq flat too.  One ``rtsds_adam_step`` launch then updates a whole group and, in the
same pass, refreshes the bf16 weight shadows the bf16 convs read.  With
``torch.distributed`` initialised (world > 1) the flat gradients are all-reduced over RCCL
(one collective per arena) before the update and scaled by 1/world inside the kernel --
this replaces the reference's nn.DataParallel grad reduce (utils.py:104-105).

SGD (momentum / dampening / nesterov / weight decay as torch.optim.SGD) shares the arena
with its momentum buffer in the first-moment slot.  Checkpoints use torch.optim's
state_dict format (interchangeable with the reference's optimizers both ways).

Semantics match torch.optim.Adam(amsgrad=False, maximize=False): L2 weight decay added to the
gradient, per-parameter step counts, parameters whose gradient was not produced in a step
are skipped (tracked with post-accumulate-grad hooks instead of ``grad is None``).
``zero_grad`` zeroes the arena rather than dropping ``.grad`` tensors.
"""
import ctypes
import warnings

import torch
import torch.distributed as dist

from ._lib import ConvDesc, lib
from .runtime import bump_params_epoch, collective, dp_world, stream


_ALLREDUCE = {"dtype": torch.float32}


def set_allreduce_dtype(dtype):
    """Wire dtype of the gradient all-reduce: float32 (exact, default) or float16 / bfloat16
    (half the xGMI bytes; BASELINE configs[4] runs fp16).  The fp32 gradients are cast into the
    arena's persistent wire buffer (one rtsds_cast launch per bucket), summed there, and the
    optimizer kernel reads the summed wire copy directly (no cast back into the fp32 arena,
    which keeps the rank's local gradients)."""
    if dtype not in (torch.float32, torch.float16, torch.bfloat16):
        raise ValueError("all-reduce dtype must be float32, float16 or bfloat16")
    _ALLREDUCE["dtype"] = dtype


_DCODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def wire_active():
    """The gradients are all-reduced over a reduced-precision wire (the optimizer then reads
    the arenas' summed wire copies)."""
    return _ALLREDUCE["dtype"] != torch.float32 and dp_world() > 1 and dist.is_available() and dist.is_initialized()


def _to_wire(buffers, wires):
    """The tensors to sum: the fp32 gradient slices themselves, or (reduced-precision wire)
    their casts into the matching slices of the arenas' wire buffers (one rtsds_cast launch
    each); the optimizer then reads the sums there.  Without ``wires`` (a caller outside the
    optimizer, e.g. the gloo CPU tests) the buffers are cast by torch and the sums copied back
    into them after the reduction: returns [(tensor to sum, buffer to copy it back into)]."""
    if _ALLREDUCE["dtype"] == torch.float32:
        return [(b, None) for b in buffers]
    if wires is None:
        return [(b.to(_ALLREDUCE["dtype"]), b) for b in buffers]
    out = []
    for b, w in zip(buffers, wires):
        lib.rtsds_cast(b.data_ptr(), 0, w.data_ptr(), _DCODE[w.dtype], b.numel(), stream())
        out.append((w, None))
    return out


def allreduce_flat(buffers, wires=None):
    """Sum flat gradient buffers over the data-parallel group (RCCL over xGMI for HIP
    tensors, gloo for CPU tests) -- one collective per buffer, replacing DataParallel's
    per-module reduce (utils.py:104-105).  The rtsds losses are already normalised by the
    global batch (runtime.dp_world), so the SUM is the single-device gradient; returns the
    gradient scale the Adam kernel applies (1.0).  ``wires``: the buffers' slices of the
    arenas' wire buffers (reduced-precision wire): the sum lands there."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    if dp_world() > 1:
        for t, back in _to_wire(buffers, wires):
            collective(lambda t=t: dist.all_reduce(t))  # a graph-segment break under capture
            if back is not None:
                back.copy_(t)
    return 1.0


_OVERLAP = {"on": True}
# gradient-arrival generation: every gradient write into an arena records the current value;
# begin_grad_phase() advances it, so a partial all-reduce can select the parameters that received
# their gradient in the current backward phase (DA iteration: the adversarial backward through G
# after the source backward already touched every parameter)
_GEN = [0]


def begin_grad_phase():
    """Start a new gradient-arrival generation; returns its number (start_grad_allreduce's
    ``since``)."""
    _GEN[0] += 1
    return _GEN[0]


def set_overlap_allreduce(on):
    """Early (overlapped) gradient all-reduce in the DA iteration on (default) / off (serial,
    inside step())."""
    _OVERLAP["on"] = bool(on)


def allreduce_start(buffers, wires=None):
    """Start the SUM all-reduce of flat gradient buffers now, asynchronously (RCCL on its own
    stream, overlapping whatever the caller enqueues next), and return a finisher that makes
    the current stream wait for them; None when there is nothing to reduce.  ``wires``: as
    allreduce_flat.  Under runtime.GraphedStep capture the start and the wait are graph-segment
    breaks re-issued between replays, so a replayed iteration overlaps the same way (DA
    iteration: G's all-reduce runs beside the discriminator phase)."""
    if not (dist.is_available() and dist.is_initialized()) or dp_world() <= 1:
        return None
    pending, pairs = [], _to_wire(buffers, wires)
    for t, _ in pairs:
        collective(lambda t=t: pending.append(dist.all_reduce(t, async_op=True)))

    def wait_all():
        for h in pending:
            h.wait()
        pending.clear()

    def finish():
        collective(wait_all)
        for t, back in pairs:
            if back is not None:
                back.copy_(t)
    return finish


class _Arena:
    """One parameter group's flat fp32 buffers: parameters, gradients, first moment (Adam's
    exp_avg / SGD's momentum buffer), second moment (Adam only) and the bf16 shadow."""

    def __init__(self, params, second=True):
        dev = params[0].device
        self.params = params
        self.offsets = []
        total = 0
        for p in params:
            if p.dtype != torch.float32 or not p.is_cuda:
                raise RuntimeError("rtsds_amd.optim: fp32 HIP parameters required")
            if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                p.data = p.data.contiguous()
            self.offsets.append(total)
            total += (p.numel() + 63) // 64 * 64  # 256-B aligned segments
        self.total = total
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.gflat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(total, dtype=torch.float32, device=dev) if second else None
        self.shadow = torch.empty(total, dtype=torch.bfloat16, device=dev)
        self.gwire = None  # reduced-precision all-reduce wire: the summed gradients (wire())
        self.steps = [0] * len(params)
        self.touched = [False] * len(params)
        self.gen = [0] * len(params)  # generation of the last gradient write (_GEN)
        # per parameter: its gradient's all-reduce has been started (optimizer.start_grad_allreduce
        # with partial=True); a later gradient write would be missing from the reduced sum
        self.reduced = None
        self.dpacks = []  # conv weights whose packed dgrad copy this arena refreshes (functional._dgrad_weight)
        with torch.no_grad():
            for i, p in enumerate(params):
                off, n = self.offsets[i], p.numel()
                view = self.flat[off:off + n].as_strided(p.shape, p.stride())
                view.copy_(p.data)
                p.data = view
                p.grad = self.gflat[off:off + n].as_strided(p.shape, p.stride())
        lib.rtsds_cast(self.flat.data_ptr(), 0, self.shadow.data_ptr(), 1, total, stream())
        for i, p in enumerate(params):
            off, n = self.offsets[i], p.numel()
            if p.dim() == 4:
                p._rt_shadow = self.shadow[off:off + n].as_strided(p.shape, p.stride())
                p._rt_shadow_key = (p.data_ptr(), p._version)
            p._rt_arena = (self, i)
            if p.requires_grad:
                p.register_post_accumulate_grad_hook(self._hook(i))

    def wire(self):
        """The persistent gradient wire buffer in the current wire dtype (allocated once)."""
        dt = _ALLREDUCE["dtype"]
        if self.gwire is None or self.gwire.dtype != dt:
            self.gwire = torch.zeros(self.total, dtype=dt, device=self.gflat.device)
        return self.gwire

    def reduced_grad(self):
        """The all-reduced gradients the optimizer applies (fp32): the arena itself, or the
        summed reduced-precision wire copy."""
        return self.gwire.float() if wire_active() and self.gwire is not None else self.gflat

    def _hook(self, i):
        def mark(_p):
            self._check_open(i)
            self.touched[i] = True
            self.gen[i] = _GEN[0]
        return mark

    def _check_open(self, i):
        if self.reduced is not None and self.reduced[i]:
            raise RuntimeError(f"rtsds_amd.optim: a gradient of parameter {i} ({tuple(self.params[i].shape)}) arrived "
                               "after its all-reduce started (start_grad_allreduce(partial=True)): the backward cut "
                               "must separate the parameters of the two phases")

    def repack(self):
        """Refresh the packed data-gradient copies of the registered conv weights from the bf16
        shadows just updated (one rtsds_conv2d_dgrad_pack_many launch per 16 segments)."""
        live = [p for p in self.dpacks if p._rt_dpack.arena is self and getattr(p, "_rt_shadow", None) is not None]
        if not live:
            return
        n = len(live)
        descs = (ConvDesc * n)(*[p._rt_dpack.desc for p in live])
        src = (ctypes.c_void_p * n)(*[p._rt_shadow.data_ptr() for p in live])
        dst = (ctypes.c_void_p * n)(*[p._rt_dpack.buf.data_ptr() for p in live])
        lib.rtsds_conv2d_dgrad_pack_many(n, descs, src, dst, stream())
        for p in live:
            p._rt_dpack.valid = p._rt_shadow_key

    def sink(self, i):
        """Gradient view a backward kernel may accumulate into directly (marks the parameter
        as having received a gradient this step); None if .grad left the arena."""
        if not self.grad_ptr_ok(i):
            return None
        self._check_open(i)
        self.touched[i] = True
        self.gen[i] = _GEN[0]
        return self.params[i].grad

    def grad_ptr_ok(self, i):
        p = self.params[i]
        return p.grad is not None and p.grad.data_ptr() == self.gflat.data_ptr() + 4 * self.offsets[i]

    def rebind_grad(self, i):
        """AccumulateGrad replaced .grad out of place: fold it back into the arena."""
        p = self.params[i]
        off, n = self.offsets[i], p.numel()
        view = self.gflat[off:off + n].as_strided(p.shape, p.stride())
        if p.grad is not None:
            view.copy_(p.grad)
        p.grad = view


class _FlatOptimizer(torch.optim.Optimizer):
    """Flat-arena optimizer core shared by Adam and SGD: the arenas, gradient sinks,
    zero_grad, the per-step runs of touched parameters, the data-parallel all-reduce, the
    hipGraph hyperparameter buffer, and torch-format state_dict / load_state_dict.
    Subclasses name their per-parameter state (``_STATE``: arena buffer -> torch key) and
    launch the update kernel for one run (``_launch``) / fill its hyper slots (``_hyper3``)."""

    _STATE = ()       # ((arena attribute, torch state key), ...)
    _NAME = "optimizer"

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._arenas = None
        self._warned = False
        # hipGraph mode (runtime.GraphedStep): lr (and bias corrections) from a device buffer
        self._graph = False      # launch the _dev kernel variant
        self._capturing = False  # inside stream capture: the hyper values are staged outside
        self._runs = None        # [(group, i, j)] of the last step
        self._hyper = None       # device fp32 [runs][3]
        self._ring = [[None, None] for _ in range(8)]  # pinned staging buffers + their copy events
        self._ring_pos = 0
        self._finish = []        # pending early gradient all-reduces (start_grad_allreduce)
        self._reduced = None     # per arena: parameters whose all-reduce has been started

    # ------------------------------------------------------------------ arena
    def _ensure(self):
        if self._arenas is None:
            # trainable parameters first: frozen ones (DeepLab's BatchNorm affines, deeplabv2.py:
            # requires_grad = False) would otherwise split the update into one launch per conv
            self._arenas = [_Arena(sorted(g["params"], key=lambda p: not p.requires_grad),
                                   second=len(self._STATE) > 1) for g in self.param_groups]
            self._import_state()
        return self._arenas

    def arenas(self):
        return self._ensure()

    # ------------------------------------------------------------------ checkpoints
    # torch.optim's state_dict format ({"state": {index: {...}}, "param_groups": [...]}), so
    # optimizer checkpoints interchange with the reference's torch.optim.Adam / SGD
    # (main.py:116-120) in both directions.
    def _view(self, a, i, attr):
        p, off = a.params[i], a.offsets[i]
        return getattr(a, attr)[off:off + p.numel()].as_strided(p.shape, p.stride())

    def _import_state(self):
        """Move per-parameter state loaded by load_state_dict into the flat arenas."""
        if not self.state:
            return
        with torch.no_grad():
            for a in self._arenas:
                for i, p in enumerate(a.params):
                    st = self.state.get(p)
                    if not st:
                        continue
                    for attr, key in self._STATE:
                        if st.get(key) is not None:
                            self._view(a, i, attr).copy_(st[key])
                    a.steps[i] = self._imported_steps(st)
        self.state.clear()

    def _imported_steps(self, st):
        return int(float(st["step"]))

    def _exported(self, a, i):
        st = {key: self._view(a, i, attr).detach().clone() for attr, key in self._STATE}
        st["step"] = torch.tensor(float(a.steps[i]))
        return st

    def state_dict(self):
        if self._arenas is not None:
            for a in self._arenas:
                for i, p in enumerate(a.params):
                    if a.steps[i] > 0:
                        self.state[p] = self._exported(a, i)
        try:
            return super().state_dict()
        finally:
            if self._arenas is not None:
                self.state.clear()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        if self._arenas is not None:
            self._import_state()

    def zero_grad(self, set_to_none=True):
        for a in self._ensure():
            a.gflat.zero_()
            for i in range(len(a.params)):
                a.touched[i] = False
                if not a.grad_ptr_ok(i):
                    a.rebind_grad(i)
                    a.gflat[a.offsets[i]:a.offsets[i] + a.params[i].numel()].zero_()

    # ------------------------------------------------------------------ step
    def _fix_grads(self, arenas):
        for a in arenas:
            for i in range(len(a.params)):
                if a.touched[i] and not a.grad_ptr_ok(i):
                    if not self._warned:
                        warnings.warn(f"rtsds_amd.{self._NAME}: gradient left the arena; copying back")
                        self._warned = True
                    a.rebind_grad(i)

    @staticmethod
    def _ranges(a, idx):
        """Contiguous arena ranges [lo, hi) covering the parameters ``idx`` (sorted)."""
        out = []
        for i in idx:
            lo, hi = a.offsets[i], a.offsets[i] + a.params[i].numel()
            if out and out[-1][2] == i - 1:
                out[-1] = (out[-1][0], hi, i)
            else:
                out.append((lo, hi, i))
        return [(lo, hi) for lo, hi, _ in out]

    @torch.no_grad()
    def start_grad_allreduce(self, partial=False, since=None):
        """Data parallelism: the gradients are final now -- start their all-reduce so it overlaps
        the work enqueued before step(), which then only waits for it.  ``partial``: only the
        parameters that have received their gradients so far (a backward pass split at a cut,
        train.seg_step: the later phase writes only the others), as contiguous arena ranges;
        the rest follow at step() (or a later call).  ``since`` (with ``partial``): only the
        parameters whose last gradient write belongs to generation >= since (begin_grad_phase):
        a phased backward after an earlier one that touched every parameter.  No-op at world 1."""
        if not _OVERLAP["on"] or dp_world() <= 1 or not (dist.is_available() and dist.is_initialized()):
            return
        arenas = self._ensure()
        self._fix_grads(arenas)
        if self._reduced is None:
            self._reduced = [[False] * len(a.params) for a in arenas]
            for a, red in zip(arenas, self._reduced):
                a.reduced = red
        bufs, wires = [], []
        for a, red in zip(arenas, self._reduced):
            idx = [i for i in range(len(a.params)) if not red[i] and
                   (not partial or (a.touched[i] and (since is None or a.gen[i] >= since)))]
            for i in idx:
                red[i] = True
            rng = self._ranges(a, idx)
            bufs += [a.gflat[lo:hi] for lo, hi in rng]
            if wire_active():
                wires += [a.wire()[lo:hi] for lo, hi in rng]
        if bufs:
            fin = allreduce_start(bufs, wires if wire_active() else None)
            if fin is not None:
                self._finish.append(fin)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        from .functional import flush_wgrad_reduce
        flush_wgrad_reduce()  # normally done at the end of each backward already
        arenas = self._ensure()
        bump_params_epoch()  # the update writes the arenas through raw pointers
        if self._finish:
            self.start_grad_allreduce()  # whatever a partial start left
            for fin in self._finish:
                fin()
            self._finish, self._reduced = [], None
            for a in arenas:
                a.reduced = None
            gscale = 1.0
        else:
            self._fix_grads(arenas)
            gscale = allreduce_flat([a.gflat for a in arenas], [a.wire() for a in arenas] if wire_active() else None)
        # contiguous runs of touched parameters with equal step counts -> one launch each
        runs = []
        for gi, a in enumerate(arenas):
            i, n = 0, len(a.params)
            while i < n:
                if not a.touched[i]:
                    i += 1
                    continue
                j = i
                while j + 1 < n and a.touched[j + 1] and a.steps[j + 1] == a.steps[i]:
                    j += 1
                runs.append((gi, i, j))
                i = j + 1
        if self._capturing:
            if runs != self._runs or self._hyper is None:
                raise RuntimeError(f"rtsds_amd.{self._NAME}: step structure changed under graph capture")
        else:
            self._runs = runs
            if self._graph:
                self.stage_hyper()
        for r, (gi, i, j) in enumerate(runs):
            g, a = self.param_groups[gi], arenas[gi]
            lo = a.offsets[i]
            hi = a.offsets[j] + a.params[j].numel()
            hyper = self._hyper.data_ptr() + 12 * r if self._graph else None
            self._launch(g, a, lo, hi, a.steps[i] + 1, hyper, gscale)
            for k in range(i, j + 1):
                a.steps[k] += 1
        for a in arenas:
            if a.shadow is not None:
                a.repack()
        return loss

    # ------------------------------------------------------------------ hipGraph support
    def set_graph_mode(self, on=True):
        self._graph = bool(on)

    def stage_hyper(self):
        """Write the hyperparameters of the NEXT step of every run of the last step into the
        device hyper buffer (stream-ordered H2D copy from pinned memory)."""
        runs = self._runs or []
        arenas = self._ensure()
        flat = []
        for gi, i, _ in runs:
            flat.extend(self._hyper3(self.param_groups[gi], arenas[gi].steps[i] + 1))
        n = max(1, len(flat))
        if self._hyper is None or self._hyper.numel() < n:
            self._hyper = torch.empty(n, dtype=torch.float32, device=arenas[0].flat.device)
        # A ring of pinned staging buffers, each reused only after its previous copy has
        # completed (its event).  A fresh pinned tensor per replay -- round 2 -- hit the host
        # allocator whenever the host ran ahead of the GPU (the cached block's copy still
        # pending), and the new pinned allocation waited for the device: enqueue ~= step time.
        slot = self._ring[self._ring_pos]
        self._ring_pos = (self._ring_pos + 1) % len(self._ring)
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(n, dtype=torch.float32, pin_memory=True)
            slot[1] = torch.cuda.Event()
        else:
            slot[1].synchronize()
        buf = slot[0][:n]
        if flat:
            buf.numpy()[:] = flat
        self._hyper[:n].copy_(buf, non_blocking=True)
        slot[1].record()

    def steps_snapshot(self):
        return [list(a.steps) for a in self._ensure()]

    def restore_steps(self, snap):
        for a, st in zip(self._ensure(), snap):
            a.steps[:] = st

    def advance_steps(self, by=1):
        """Host step counters after a replayed step (the graph does not run Python)."""
        arenas = self._ensure()
        for gi, i, j in self._runs or []:
            for k in range(i, j + 1):
                arenas[gi].steps[k] += by


def _ptrs(a, lo, hi, *attrs):
    return tuple(getattr(a, at).data_ptr() + 4 * lo for at in attrs)


def _grad(a, lo):
    """(pointer, dtype code) of the gradients the update reads from arena offset lo: the fp32
    arena, or the summed reduced-precision wire copy."""
    if wire_active() and a.gwire is not None:
        return a.gwire.data_ptr() + a.gwire.element_size() * lo, _DCODE[a.gwire.dtype]
    return a.gflat.data_ptr() + 4 * lo, 0


class Adam(_FlatOptimizer):
    """torch.optim.Adam (main.py:116-117) as one rtsds_adam_step launch per run."""

    _STATE = (("m", "exp_avg"), ("v", "exp_avg_sq"))
    _NAME = "Adam"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("rtsds_amd.optim.Adam: amsgrad")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    def _launch(self, g, a, lo, hi, t, hyper, gscale):
        b1, b2 = g["betas"]
        gp, gd = _grad(a, lo)
        ptrs = _ptrs(a, lo, hi, "flat") + (gp,) + _ptrs(a, lo, hi, "m", "v") + (a.shadow.data_ptr() + 2 * lo, hi - lo)
        if hyper is not None:
            lib.rtsds_adam_step_dev(*ptrs, hyper, float(b1), float(b2), float(g["eps"]),
                                    float(g["weight_decay"]), gscale, gd, stream())
        else:
            lib.rtsds_adam_step(*ptrs, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                float(g["weight_decay"]), t, gscale, gd, stream())

    def _hyper3(self, g, t):
        # betas rounded to fp32 first, exactly as rtsds_adam_step receives them (eager and
        # replayed steps then update bit-identically)
        b1, b2 = (float(torch.tensor(b, dtype=torch.float32)) for b in g["betas"])
        return [float(g["lr"]), 1.0 - b1 ** t, (1.0 - b2 ** t) ** 0.5]


class SGD(_FlatOptimizer):
    """torch.optim.SGD (main.py:118-120: lr, momentum; weight_decay, dampening and nesterov
    as torch) as one rtsds_sgd_step launch per run.  The momentum buffer is the arena's
    first-moment buffer; a parameter's first step initialises it with the gradient (torch's
    ``momentum_buffer is None`` branch)."""

    _STATE = (("m", "momentum_buffer"),)
    _NAME = "SGD"

    def __init__(self, params, lr=1e-3, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 maximize=False):
        if maximize:
            raise NotImplementedError("rtsds_amd.optim.SGD: maximize")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov))

    def _launch(self, g, a, lo, hi, t, hyper, gscale):
        gp, gd = _grad(a, lo)
        lib.rtsds_sgd_step(*_ptrs(a, lo, hi, "flat"), gp, *_ptrs(a, lo, hi, "m"), a.shadow.data_ptr() + 2 * lo, hi - lo,
                           hyper, float(g["lr"]), float(g["momentum"]), float(g["dampening"]),
                           float(g["weight_decay"]), int(bool(g["nesterov"])), int(t == 1), gscale, gd, stream())

    def _hyper3(self, g, t):
        return [float(g["lr"]), 1.0 if t == 1 else 0.0, 0.0]

    def _exported(self, a, i):
        # torch.optim.SGD keeps no step count; momentum_buffer only when momentum != 0
        st = {}
        if self.param_groups[self._arenas.index(a)]["momentum"] != 0:
            st["momentum_buffer"] = self._view(a, i, "m").detach().clone()
        st["step"] = torch.tensor(float(a.steps[i]))  # extra key, ignored by torch.optim.SGD
        return st

    def _imported_steps(self, st):
        if "step" in st:
            return int(float(st["step"]))
        return 1 if st.get("momentum_buffer") is not None else 0
