"""Process-wide runtime settings and helpers for the HIP path.

* compute dtype: ``float32`` (default; exact-f32 MFMA, the parity mode) or ``bfloat16``
  (bf16 activations / weight shadows, fp32 accumulation, statistics and master weights).
* tensor helpers: NHWC ("channels_last") allocation, stream handle, HIP-only guard.
"""
import contextlib
import os
import time
import warnings

import torch

_state = {"dtype": torch.float32}


def set_compute_dtype(dtype):
    if dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
    _state["dtype"] = dtype


def compute_dtype():
    return _state["dtype"]


@contextlib.contextmanager
def precision(dtype):
    old = _state["dtype"]
    set_compute_dtype(dtype)
    try:
        yield
    finally:
        _state["dtype"] = old


def dp_world():
    """Size of the data-parallel group (1 when torch.distributed is not initialised).

    Under data parallelism the rtsds losses are normalised by the GLOBAL batch (the
    reference's DataParallel computes each loss once over the gathered batch): CE divides
    by the all-reduced valid-pixel count, BCE by world * local batch, and the optimizer
    SUMS the gradients (optim.allreduce_flat) -- so a sharded step equals the single-device
    step on the concatenated batch (with per-replica BatchNorm statistics, as DataParallel)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def dcode(t):
    """torch dtype -> RTSDS_F32 / RTSDS_BF16."""
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise RuntimeError(f"rtsds_amd: unsupported dtype {t.dtype}")


def stream():
    return torch.cuda.current_stream().cuda_stream


def require_hip(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("rtsds_amd: ops run only on HIP (MI355X) tensors; "
                               "there is no CPU fallback (move the model / data to 'cuda')")


# Parameter epoch: advanced by every rtsds writer that updates parameters / BatchNorm running
# statistics through raw device pointers (which torch's tensor versions do not see): the
# optimizer step, a replayed training iteration, a train-mode BatchNorm forward.  Caches of
# values derived from parameters (the eval-mode BatchNorm folds) are keyed on it.
_epoch = [0]


def bump_params_epoch():
    _epoch[0] += 1


def params_epoch():
    return _epoch[0]


CL = torch.channels_last
# hipGraph captures are thread-local: under the default global mode a HIP call from ANY thread
# during a capture -- RCCL's process-group watchdog polling its events -- is rejected
# ("operation not permitted when stream is capturing") and aborts the process; seen on the
# one-rank RCCL test of the data-parallel graph segments.
CAPTURE_MODE = "thread_local"


def empty_nhwc(n, c, h, w, dtype, device):
    return torch.empty((n, c, h, w), dtype=dtype, device=device, memory_format=CL)


def is_nhwc(t):
    return t.dim() == 4 and t.is_contiguous(memory_format=CL)


def nhwc(t):
    """Return ``t`` with NHWC memory (no copy when it already is)."""
    if is_nhwc(t):
        return t
    return t.contiguous(memory_format=CL)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ----------------------------------------------------------------------------- backward cuts
# Data parallelism (train.seg_step): the backward pass runs in two phases split at a cut tensor
# (the context path's layer-3 output), so that the all-reduce of the gradients finished in the
# first phase (the late layers: ResNet layer4, attention / fusion modules, heads, spatial path --
# ~75 % of BiSeNet-R18's parameters) is started from the host between the phases and overlaps
# the second (layer3 .. stem).  A cut returns a detached leaf copy of its input for the
# downstream consumers; phase 2 is torch.autograd.backward(cut inputs, their leaf gradients).
_cuts = []


@contextlib.contextmanager
def collect_cuts(on=True):
    """Models' grad_cut() calls inside the block record (tensor, detached leaf) pairs here."""
    if not on:
        yield None
        return
    lst = []
    _cuts.append(lst)
    try:
        yield lst
    finally:
        _cuts.pop()


def grad_cut(x):
    """Identity, or -- inside collect_cuts() with autograd on -- a detached leaf copy of ``x``
    whose gradient phase 1 of the backward accumulates."""
    if not _cuts or not (torch.is_grad_enabled() and x.requires_grad):
        return x
    xd = x.detach().requires_grad_()
    _cuts[-1].append((x, xd))
    return xd


# ----------------------------------------------------------------------------- side stream
# Weight gradients run on a second HIP stream, concurrently with the data-gradient chain of
# the backward pass (dgrad GEMMs, BatchNorm backward passes and the small reduction /
# finalize kernels that leave most CUs idle).  A conv's wgrad forks off the main stream once
# its output gradient is ready and writes only into the optimizer's flat gradient arena;
# the tensors it reads are kept alive here, and the main stream joins the side stream at
# the end of the backward pass (an autograd engine callback, so code that reads gradients
# after backward() -- optimizer, all-reduce, tests -- sees them complete).  Under hipGraph
# capture the fork / join become graph edges.  Off by default (RTSDS_OVERLAP=1 enables it):
# on the BiSeNet-R18 bs8 step it measured 1196 img/s vs 1250 serial, and 1155-1194 when
# restricted to the small late-stage convs (RTSDS_OVERLAP_MAXROWS) -- the concurrent GEMMs
# and the cross-stream graph edges cost more than the idle CUs it fills.
_side = {"stream": None, "main": None, "keep": [], "armed": False,
         "on": os.environ.get("RTSDS_OVERLAP", "0") == "1",
         "max_rows": int(os.environ.get("RTSDS_OVERLAP_MAXROWS", "0"))}


def side_enabled(rows=0):
    """Side-stream weight gradients on (for a conv with ``rows`` output pixels: only
    convs up to RTSDS_OVERLAP_MAXROWS when that is set)."""
    return _side["on"] and (_side["max_rows"] <= 0 or rows <= _side["max_rows"])


def set_side_enabled(on):
    _side["on"] = bool(on)


def side_fork(*keep):
    """Side stream ordered after everything enqueued so far on the current stream; ``keep``
    (inputs / workspaces of the side work) stay referenced until the join."""
    main = torch.cuda.current_stream()
    s = _side["stream"]
    if s is None or s.device != main.device:
        s = _side["stream"] = torch.cuda.Stream(device=main.device)
    s.wait_stream(main)
    _side["keep"].extend(keep)
    if not _side["armed"]:
        _side["armed"] = True
        _side["main"] = main  # the stream the backward pass runs on (callbacks may not)
        torch.autograd.Variable._execution_engine.queue_callback(side_join)
    return s


def side_join():
    """Main stream waits for the side stream; release the kept tensors."""
    if _side["stream"] is not None and _side["armed"]:
        _side["main"].wait_stream(_side["stream"])
    _side["keep"].clear()
    _side["main"] = None
    _side["armed"] = False


# ----------------------------------------------------------------------------- branch streams
# Independent branches of one network (BiSeNet's spatial path beside its ResNet context path)
# run on a second stream: forward forks after the shared input and joins before the first op
# that reads both; autograd runs each backward op on its forward op's stream, so the backward
# branches overlap too, and an engine callback queued by the branch's first backward op joins
# the branch back into the ambient stream at the end of backward (its weight gradients go
# straight into optimizer arenas, which autograd does not see).  Under hipGraph capture the
# fork / joins are graph edges.
_branch = {}


_branch_off = {"depth": 0}


@contextlib.contextmanager
def branches_serial():
    """Modules issue their branches on the current stream (already a concurrent branch: a
    fork nested in it measured no gain and broke hipGraph capture of the DA iteration)."""
    _branch_off["depth"] += 1
    try:
        yield
    finally:
        _branch_off["depth"] -= 1


def branches_enabled():
    """Branch streams in use: not inside branches_serial(), and not while side-stream weight
    gradients are on -- the two overlap schemes are alternatives (a side fork from a branch
    stream would be joined only into the first forking stream, leaving the branch un-joined,
    which breaks hipGraph capture)."""
    return _branch_off["depth"] == 0 and not _side["on"]


def branch_stream(device, name="spatial"):
    s = _branch.get((device, name))
    if s is None:
        s = _branch[(device, name)] = torch.cuda.Stream(device=device)
    return s


class BranchOut(torch.autograd.Function):
    """Identity on a branch's output (applied on the branch stream); its backward -- the
    branch's first backward op -- queues the end-of-backward join of ``side`` into ``main``."""

    @staticmethod
    def forward(ctx, x, main, side):
        ctx.main, ctx.side = main, side
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g.record_stream(ctx.side)
        main, side = ctx.main, ctx.side
        torch.autograd.Variable._execution_engine.queue_callback(lambda: main.wait_stream(side))
        return g, None, None


# Submission of captured graphs.  hipGraphLaunch of a graph captured from several streams (the
# branch streams) takes the runtime's multi-queue path and enqueues node by node: ~4.7 ms of
# host time per BiSeNet bs-8 step (~330 nodes) -- hidden while the GPU needs 5.7 ms, but a
# ceiling once the kernels get faster -- whereas a linear (single-stream) graph goes out as
# one pre-recorded packet batch (~0.2 ms).  Measured on the bs-8 step (round 3,
# profiles/r3_graph_submit.txt): multi-stream graph 5.67 ms wall / 4.7 ms host, the same
# iteration captured serially 5.85 / 0.23, and the multi-stream capture replayed as per-stream
# linear segment graphs joined by events (rtsds_graph_split, csrc/graph.hip) 6.11 / 0.41 -- each
# segment launch and cross-queue wait costs ~20 us of GPU idle time.  GraphedStep therefore
# captures both the branch-stream and the serial variant, adds the split replay of the branch
# capture, and keeps whichever runs fastest (submit="auto").
SUBMIT = {"mode": "auto", "max_lanes": 4, "trial_calls": 3, "host_frac": 0.5}


def capture_nodes(stream):
    """Nodes captured so far by the capture ``stream`` records into (None if it is not capturing)."""
    from ._lib import load
    n = load().rtsds_capture_nodes(stream.cuda_stream)
    return n if n >= 0 else None


def graph_nodes(graph):
    """Nodes of a captured graph (0 = empty capture)."""
    import ctypes
    from ._lib import load
    n = load().rtsds_graph_nodes(ctypes.c_void_p(graph.raw_cuda_graph()))
    if n < 0:
        raise RuntimeError(f"rtsds_amd: rtsds_graph_nodes failed (status {-n})")
    return n


def graph_lanes(graph):
    """Stream chains of a captured graph (1 = linear)."""
    import ctypes
    from ._lib import load
    n = load().rtsds_graph_lanes(ctypes.c_void_p(graph.raw_cuda_graph()), int(SUBMIT["max_lanes"]))
    if n < 1:
        raise RuntimeError(f"rtsds_amd: rtsds_graph_lanes failed (status {-n})")
    return n


class GraphRunner:
    """Replays one captured torch.cuda.CUDAGraph(keep_graph=True) -- as lane-split linear
    segments (rtsds_graph_split) when ``split`` and the capture forked streams, else the graph
    itself.  Keeps the graph (and its memory pool) alive."""

    def __init__(self, graph, split=False):
        import ctypes
        from ._lib import load
        self.graph, self.handle, self.segments = graph, None, 1
        self.lanes = graph_lanes(graph)
        if split and self.lanes > 1:
            lib = load()
            h, ns, nl = ctypes.c_void_p(), ctypes.c_int(0), ctypes.c_int(0)
            rc = lib.rtsds_graph_split(ctypes.c_void_p(graph.raw_cuda_graph()), int(SUBMIT["max_lanes"]),
                                       ctypes.byref(h), ctypes.byref(ns), ctypes.byref(nl))
            if rc == 0:
                self.handle, self.segments = h, ns.value
            elif rc != 2:  # RTSDS_ERR_UNSUPPORTED node type: replay the graph itself
                raise RuntimeError(f"rtsds_amd: rtsds_graph_split failed (status {rc})")
        if self.handle is None:
            graph.instantiate()

    def replay(self):
        if self.handle is not None:
            from ._lib import lib
            lib.rtsds_graph_split_launch(self.handle, stream())
        else:
            self.graph.replay()

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h is not None:
            try:
                from ._lib import load
                load().rtsds_graph_split_destroy(h)
            except Exception:  # interpreter shutdown
                pass


class GraphedForward:
    """hipGraph capture of a fixed-shape inference forward (torch.cuda.CUDAGraph is a hipGraph
    on ROCm): every rtsds kernel of ``module(x)`` is recorded once on a side stream and the
    whole launch sequence is replayed with one call, removing the per-kernel host launch cost
    that dominates small-batch inference.  ``x`` fixes shape / dtype / device; replays copy the
    new batch into the captured input buffer and return the captured output buffer (valid
    until the next replay)."""

    def __init__(self, module, x, warmup=2, packed=None):
        """``packed``: the module's forward starts with ``nn.to_input`` (the reference-layout
        NCHW fp32 batch -> the packed compute-dtype input): the graph is captured from the packed
        tensor and each replay packs the new batch straight into it (one pass over the batch
        instead of a copy into a captured fp32 buffer plus the pack).  Default: on when the
        module says so (``accepts_packed_input``)."""
        self.module = module
        if packed is None:
            packed = bool(getattr(module, "accepts_packed_input", False)) and x.dtype == torch.float32
        self.packed = packed
        if packed:
            from .functional import pack_input
            self.in_shape, self.in_dtype = tuple(x.shape), x.dtype
            self.static_in = pack_input(x.detach(), compute_dtype())
            if self.static_in.data_ptr() == x.data_ptr():
                self.static_in = self.static_in.clone()
        else:
            self.static_in = x.detach().clone()
        side = torch.cuda.Stream(device=x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(warmup):  # settle lazy allocations (bf16 shadows, workspaces)
                module(self.static_in)
        torch.cuda.current_stream(x.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        _fold_capture.append([])
        try:
            with torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
                self.static_out = module(self.static_in)
        finally:
            self.folds = _fold_capture.pop()
        self.runner = GraphRunner(self.graph)

    def __call__(self, x):
        if self.packed:
            if tuple(x.shape) != self.in_shape or x.dtype != self.in_dtype:
                raise RuntimeError("GraphedForward: input shape/dtype differs from the captured one")
            from .functional import pack_input_into
            pack_input_into(x, self.static_in)
        else:
            if x.shape != self.static_in.shape or x.dtype != self.static_in.dtype:
                raise RuntimeError("GraphedForward: input shape/dtype differs from the captured one")
            self.static_in.copy_(x)
        for refresh in self.folds:  # BatchNorm folds the graph reads (recomputed if stale)
            refresh()
        self.runner.replay()
        return self.static_out


_capture = {"step": None}  # the GraphedStep currently capturing, if any
# GraphedForward captures in progress: each collects the refresh callables of the cached
# BatchNorm folds its graph reads (functional.conv_bn_eval)
_fold_capture = []


def register_fold(refresh):
    if _fold_capture:
        _fold_capture[-1].append(refresh)


def collective(fn):
    """Run ``fn`` (a collective on device tensors, e.g. ``dist.all_reduce(t)``) -- eagerly, or,
    while a GraphedStep is capturing, as a break between two captured graph segments: the
    collective is not captured but re-issued between the segments' replays (RCCL's own launch
    path, stream-ordered with the graphs)."""
    cap = _capture["step"]
    if cap is None:
        return fn()
    cap._break(fn)
    return None


class GraphedStep:
    """hipGraph of a whole training iteration (zero_grad, forward, losses, backward, optimizer
    step).  ``fn()`` runs one iteration on fixed input buffers and returns device tensors; the
    rtsds optimizers in ``optimizers`` switch to device-side hyperparameters
    (optim.Adam.set_graph_mode) so that every replay applies the current learning rate
    (``param_groups[..]["lr"]``, e.g. set by utils.poly_lr_scheduler before the call) and the
    advancing Adam step count, staged by a stream-ordered H2D copy before the replay.  The
    iteration must keep its launch structure (same shapes, same parameters receiving
    gradients); no host synchronisation may happen inside ``fn``.

    Data parallelism: every collective of the iteration goes through ``runtime.collective``
    (the global valid-pixel count of each loss, the gradient all-reduce); under capture each
    one ends the current graph segment and starts the next in the same memory pool, and a
    replay runs segment, collective, segment, ... -- so a data-parallel step is replayed too,
    with its RCCL calls issued eagerly between the graphs."""

    def __init__(self, fn, optimizers, warmup=2, submit=None):
        """``submit``: "auto" (default, SUBMIT["mode"]): capture the iteration with its branch
        streams and, if it forked, a second time serially, and also replay the branch capture as
        per-stream segment graphs ("split"); the first trial_calls replays of each are timed
        (host submission time and GPU time, HIP events) and the faster variant -- max(host, GPU)
        per step -- is kept.  Both compute bit-identical results, so the trial
        replays are ordinary training steps.  "branches" / "serial" / "split": that variant only."""
        self.fn = fn
        self.optimizers = list(optimizers)
        mode = submit or SUBMIT["mode"]
        if mode not in ("auto", "branches", "serial", "split"):
            raise ValueError(f"GraphedStep: unknown submit mode {mode!r}")
        for o in self.optimizers:
            o.set_graph_mode(True)
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream(device=cur.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side), (branches_serial() if mode == "serial" else contextlib.nullcontext()):
            for _ in range(warmup):
                fn()
        cur.wait_stream(side)
        for o in self.optimizers:
            if o._runs is None:
                raise RuntimeError("GraphedStep: run one eager iteration before capturing")
            o.stage_hyper()  # allocates the device hyper buffer outside the capture
        torch.cuda.synchronize()
        self._pool = torch.cuda.graph_pool_handle()  # shared by the variants (never run concurrently)
        self.variants = []  # [(name, segments [(graph or None, [collectives])], runners, outputs)]
        first = "serial" if mode == "serial" else ("split" if mode == "split" else "branches")
        self._add_variant(first, fn, serial=first == "serial", split=first == "split")
        if mode == "auto" and max((r.lanes for r, _ in self.variants[0][2] if r is not None), default=1) > 1:
            self._add_variant("serial", fn, serial=True, split=False)
            # the branch capture also replayed as per-stream segment graphs (no second capture):
            # ~GPU time of the branch graph at the serial graph's host cost where it has few
            # segments (DeepLab DA: 54.8 ms GPU / 0.9 ms host vs 54.3 / 52 host-bound)
            name, segs, _, outs = self.variants[0]
            self.variants.append(("split", segs, [(GraphRunner(g, split=True) if g is not None else None, colls)
                                                  for g, colls in segs], outs))
        self._use(0)
        self._trial = [[] for _ in self.variants] if len(self.variants) > 1 else None
        self._calls = 0
        self.submit_choice = self.variants[0][0] if self._trial is None else None
        self.submit_trials = {}
        self.host_launch_s = 0.0  # host time spent submitting replays (bench.py)

    def _add_variant(self, name, fn, serial, split):
        cur = torch.cuda.current_stream()
        self.segments = []  # [(graph or None, [collectives run after it])]
        cap_stream = torch.cuda.Stream(device=cur.device)
        cap_stream.wait_stream(cur)
        # the capture runs the optimizers' Python bookkeeping (step counters) without executing
        # a step: their counters are restored afterwards, also when the capture fails part-way
        saved = [o.steps_snapshot() for o in self.optimizers]
        for o in self.optimizers:
            o._capturing = True
        try:
            with torch.cuda.stream(cap_stream), (branches_serial() if serial else contextlib.nullcontext()):
                self._graph = torch.cuda.CUDAGraph(keep_graph=True)
                self._graph.capture_begin(pool=self._pool, capture_error_mode=CAPTURE_MODE)
                _capture["step"] = self
                self._cap_stream = cap_stream
                try:
                    outputs = fn()
                finally:
                    _capture["step"] = None
                    empty = capture_nodes(cap_stream) == 0
                    with warnings.catch_warnings():
                        if empty:  # a collective ended the iteration: dropped below, no warning
                            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
                        self._graph.capture_end()
                if graph_nodes(self._graph) > 0 or not self.segments:
                    self.segments.append((self._graph, []))
        finally:
            for o, st in zip(self.optimizers, saved):
                o._capturing = False
                o.restore_steps(st)
        cur.wait_stream(cap_stream)
        runners = [(GraphRunner(g, split=split) if g is not None else None, colls) for g, colls in self.segments]
        self.variants.append((name, self.segments, runners, outputs))

    def _use(self, i):
        self.variant = self.variants[i][0]
        self.segments, self.runners, self.outputs = self.variants[i][1], self.variants[i][2], self.variants[i][3]
        self.graph = next((g for g, _ in self.segments if g is not None), None)

    def _break(self, coll):
        """End the current segment at a collective.  Nothing captured since the last break (two
        collectives back to back, or one at the very start): the capture stays open and the
        collective joins the previous segment's list, so no empty graph is captured or launched."""
        if capture_nodes(self._cap_stream) == 0:
            if self.segments:
                self.segments[-1][1].append(coll)
            else:
                self.segments.append((None, [coll]))
            return
        self._graph.capture_end()
        if graph_nodes(self._graph) > 0:
            self.segments.append((self._graph, [coll]))
        elif self.segments:
            self.segments[-1][1].append(coll)
        else:
            self.segments.append((None, [coll]))
        self._graph = torch.cuda.CUDAGraph(keep_graph=True)
        self._graph.capture_begin(pool=self._pool, capture_error_mode=CAPTURE_MODE)

    def __call__(self):
        for o in self.optimizers:
            o.stage_hyper()
            o.advance_steps()
        bump_params_epoch()
        trial = self._trial is not None
        if trial:  # trial replays: trial_calls per variant, timed
            vi = self._calls // int(SUBMIT["trial_calls"])
            self._use(vi)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # drained queues: the host time below is the submission's own CPU work, not the
            # back-pressure of a previous replay still filling the hardware queues
            torch.cuda.synchronize()
            e0.record()
        t0 = time.perf_counter()
        for r, colls in self.runners:
            if r is not None:
                r.replay()
            for coll in colls:
                coll()
        dt = time.perf_counter() - t0
        self.host_launch_s += dt
        outputs = self.outputs  # of the variant just replayed (_decide may switch)
        if trial:
            e1.record()
            self._trial[vi].append((dt, e0, e1))
            self._calls += 1
            if self._calls == int(SUBMIT["trial_calls"]) * len(self.variants):
                self._decide()
        return outputs

    def _decide(self):
        """Keep the multi-stream graph ("branches") unless its host submission takes more than
        half its GPU time (SUBMIT["host_frac"]); otherwise the variant with the smallest
        max(host submission, GPU) time per step (the first trial replay of each is a warm-up).
        Each trial replay starts on drained queues, so its host time is the submission's CPU
        work: back to back, the node-by-node submission of a multi-stream graph fills the
        hardware queues and then waits for the GPU (DeepLab DA: 41.8 of 50.3 ms "host" per step
        in round 4, nearly all of it that wait), which says nothing about whether the host can
        keep up -- under data parallelism it is the CPU work that delays the collectives issued
        between segments.  The trials replay each variant in isolation; sustained, consecutive
        branch-graph replays overlap each other's head and tail, which the per-stream segment
        graphs of "split" do not (bench: BiSeNet seg 5.45 ms/step branches vs 5.66 split with
        near-equal trials)."""
        torch.cuda.synchronize()
        costs, hosts, names = [], [], []
        for (name, *_), rec in zip(self.variants, self._trial):
            use = rec[1:] if len(rec) > 1 else rec
            host = 1e3 * sum(r[0] for r in use) / len(use)
            gpu = sum(r[1].elapsed_time(r[2]) for r in use) / len(use)
            self.submit_trials[name] = {"host_ms": round(host, 3), "gpu_ms": round(gpu, 3)}
            costs.append(max(host, gpu))
            hosts.append(host)
            names.append(name)
        bi = names.index("branches") if "branches" in names else -1
        if bi >= 0 and hosts[bi] <= float(SUBMIT["host_frac"]) * costs[bi]:
            best = bi
        else:
            best = min(range(len(costs)), key=costs.__getitem__)
        # drop the variants not chosen: their graphs, split-replay clones and the captured
        # collectives' closures (with a reduced-precision wire, an arena-sized copy each)
        # would otherwise stay referenced for the whole run ("split" keeps the branch
        # capture's graphs through its own segment list)
        self.variants = [self.variants[best]]
        self._use(0)
        self.submit_choice = self.variants[0][0]
        self._trial = None
