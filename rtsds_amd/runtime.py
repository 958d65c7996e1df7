"""Process-wide runtime settings and helpers for the HIP path.

* compute dtype: ``float32`` (default; exact-f32 MFMA, the parity mode) or ``bfloat16``
  (bf16 activations / weight shadows, fp32 accumulation, statistics and master weights).
* tensor helpers: NHWC ("channels_last") allocation, stream handle, HIP-only guard.
"""
import contextlib
import os

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


class GraphedForward:
    """hipGraph capture of a fixed-shape inference forward (torch.cuda.CUDAGraph is a hipGraph
    on ROCm): every rtsds kernel of ``module(x)`` is recorded once on a side stream and the
    whole launch sequence is replayed with one call, removing the per-kernel host launch cost
    that dominates small-batch inference.  ``x`` fixes shape / dtype / device; replays copy the
    new batch into the captured input buffer and return the captured output buffer (valid
    until the next replay)."""

    def __init__(self, module, x, warmup=2):
        self.module = module
        self.static_in = x.detach().clone()
        side = torch.cuda.Stream(device=x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(warmup):  # settle lazy allocations (bf16 shadows, workspaces)
                module(self.static_in)
        torch.cuda.current_stream(x.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
            self.static_out = module(self.static_in)

    def __call__(self, x):
        if x.shape != self.static_in.shape or x.dtype != self.static_in.dtype:
            raise RuntimeError("GraphedForward: input shape/dtype differs from the captured one")
        self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out


_capture = {"step": None}  # the GraphedStep currently capturing, if any


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

    def __init__(self, fn, optimizers, warmup=2):
        self.fn = fn
        self.optimizers = list(optimizers)
        for o in self.optimizers:
            o.set_graph_mode(True)
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream(device=cur.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        cur.wait_stream(side)
        for o in self.optimizers:
            if o._runs is None:
                raise RuntimeError("GraphedStep: run one eager iteration before capturing")
            o.stage_hyper()  # allocates the device hyper buffer outside the capture
        torch.cuda.synchronize()
        self.segments = []  # [(graph, collective run after it or None)]
        self._pool = torch.cuda.graph_pool_handle()
        cap_stream = torch.cuda.Stream(device=cur.device)
        # the capture runs the optimizers' Python bookkeeping (step counters) without executing
        # a step: their counters are restored afterwards, also when the capture fails part-way
        saved = [o.steps_snapshot() for o in self.optimizers]
        for o in self.optimizers:
            o._capturing = True
        try:
            with torch.cuda.stream(cap_stream):
                self._graph = torch.cuda.CUDAGraph()
                self._graph.capture_begin(pool=self._pool, capture_error_mode=CAPTURE_MODE)
                _capture["step"] = self
                try:
                    self.outputs = fn()
                finally:
                    _capture["step"] = None
                    self._graph.capture_end()
                self.segments.append((self._graph, None))
        finally:
            for o, st in zip(self.optimizers, saved):
                o._capturing = False
                o.restore_steps(st)
        cur.wait_stream(cap_stream)
        self.graph = self.segments[0][0]

    def _break(self, coll):
        self._graph.capture_end()
        self.segments.append((self._graph, coll))
        self._graph = torch.cuda.CUDAGraph()
        self._graph.capture_begin(pool=self._pool, capture_error_mode=CAPTURE_MODE)

    def __call__(self):
        for o in self.optimizers:
            o.stage_hyper()
            o.advance_steps()
        for g, coll in self.segments:
            g.replay()
            if coll is not None:
                coll()
        return self.outputs
