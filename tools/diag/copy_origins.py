"""Diagnostic: where do the device-to-device copies (hipMemcpyAsync -> __amd_rocclr_copyBuffer
graph nodes) of one bench iteration come from?  Runs the bench workload eagerly for two
warm-up iterations, then logs every aten copy_/clone/contiguous-materialising op of the third
under a TorchDispatchMode with the innermost repo frames of its Python stack.
usage: copy_origins.py [bisenet-seg|bisenet-da|deeplab-seg|deeplab-da] [batch] [infer]"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from rtsds_amd import set_compute_dtype  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
WATCH = ("copy_", "clone", "_to_copy", "copy", "cat", "stack", "index_put_")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        base = str(func.overloadpacket.__name__) if hasattr(func, "overloadpacket") else name
        if any(base == w or base.startswith(w) for w in WATCH):
            t = next((a for a in args if isinstance(a, torch.Tensor)), None)
            dev = t.device.type if t is not None else "-"
            if dev == "cuda":
                fr = [f for f in traceback.extract_stack()[:-1] if f.filename.startswith(ROOT) and "copy_origins" not in f.filename]
                where = " <- ".join(f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in fr[::-1][:4])
                shape = tuple(t.shape) if t is not None else ()
                self.sites[(base, str(t.dtype) if t is not None else "", shape, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "bisenet-seg"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else None
    infer = len(sys.argv) > 3 and sys.argv[3] == "infer"
    sys.argv = [sys.argv[0], "--workload", wl] + (["--batch", str(batch)] if batch else [])
    args = bench.parse()
    if args.batch is None:
        args.batch = bench.WORKLOADS[wl][2]
    set_compute_dtype(torch.bfloat16)
    torch.manual_seed(42)
    dev = torch.device("cuda", 0)
    net, x, set_lr, core, opts = bench.build(args, dev, 0)
    if infer:
        net.eval()

        def core():  # noqa: F811
            with torch.no_grad():
                return net(x)
    for i in range(2):
        set_lr(i) if not infer else None
        core()
    torch.cuda.synchronize()
    log = Log()
    with log:
        if not infer:
            set_lr(2)
        core()
    torch.cuda.synchronize()
    total = sum(log.sites.values())
    print(f"{wl} batch {args.batch} {'inference' if infer else 'train'}: {total} watched ops on cuda tensors")
    for (op, dt, shape, where), n in log.sites.most_common():
        print(f"{n:4d}  {op:12s} {dt:15s} {str(shape):24s} {where}")


if __name__ == "__main__":
    main()
