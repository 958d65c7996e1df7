"""Which BatchNorm backwards of one BiSeNet train step take the separate statistics pass:
wraps rtsds_bn_bwd / rtsds_bn_bwd_part / the dgrad entry points and prints (rows, c, residual)."""
import sys
import torch
sys.path.insert(0, ".")
import bench  # noqa: E402
from rtsds_amd import _lib  # noqa: E402

lib = _lib.load()
log = []
for name in ("rtsds_bn_bwd", "rtsds_bn_bwd_part", "rtsds_conv2d_dgrad", "rtsds_conv2d_dgrad_bnstats", "rtsds_conv2d_dgrad_act"):
    f = getattr(lib, name)
    def wrap(*a, _f=f, _n=name):
        if _n == "rtsds_bn_bwd":
            log.append((_n, a[7], a[8], a[4] is not None and bool(a[4])))
        elif _n == "rtsds_bn_bwd_part":
            log.append((_n, a[5], a[6]))
        else:
            d = a[0]._obj
            log.append((_n, d.n, d.h, d.w, d.c, "->", d.k, "k%d s%d" % (d.kh, d.sh)))
        return _f(*a)
    setattr(lib, name, wrap)

from rtsds_amd import functional as Fn  # noqa: E402
_cb = Fn.ConvFn.backward
def cb(ctx, dy):
    l = ctx.bn_link
    log.append(("convbwd", tuple(ctx.d.__getattribute__(k) for k in ("n", "h", "w", "c", "k")),
                "link" if l is not None else "-", "src" if (l is not None and l.src is not None) else "-",
                ctx.join is not None and ctx.join.buf is not None, dy.dtype))
    return _cb(ctx, dy)
Fn.ConvFn.backward = staticmethod(cb)
sys.argv = ["bench.py"]
args = bench.parse()
args.batch = bench.WORKLOADS[args.workload][2]
from rtsds_amd import set_compute_dtype  # noqa: E402
set_compute_dtype(torch.bfloat16)
net, x, set_lr, core, opts = bench.build(args, torch.device("cuda"), 0)
core()
torch.cuda.synchronize()
log.clear()
core()
torch.cuda.synchronize()
for e in log:
    print(*e)
