"""Where do the per-step device copies (__amd_rocclr_copyBuffer) of the bench's seg step come
from?  Runs the bench workload eagerly under torch.profiler and prints every copy / fill op of
one step with its Python call site.  Usage (GPU box): python tools/diag_copies.py [workload]"""
import collections
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "bisenet-seg"
    args = types.SimpleNamespace(workload=wl, batch=bench.WORKLOADS[wl][2], da_unfused=False)
    dev = torch.device("cuda:0")
    net, x, set_lr, core, opts = bench.build(args, dev, 0)
    for i in range(3):
        set_lr(i)
        core()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        set_lr(3)
        core()
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::clone", "aten::to", "aten::_to_copy",
                    "aten::cat", "aten::contiguous", "aten::index_put_", "aten::add_", "aten::mul",
                    "aten::add", "aten::sum", "aten::div", "aten::mul_", "aten::zeros", "aten::ones",
                    "aten::full"):
            stack = [s for s in (ev.stack or []) if "rtsds_amd" in s or "bench.py" in s]
            sites[(name, " <- ".join(stack[:3]))] += 1
    for (name, st), n in sites.most_common(60):
        print(f"{n:4d} {name:20s} {st}")
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
