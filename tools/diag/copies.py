"""Which torch-side copies / elementwise kernels run inside one eager seg step (bisenet, bs8):
torch.profiler over the 3rd eager step, memcpy / non-rtsds kernels with their Python stacks."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torch.profiler import ProfilerActivity, profile

import bench
from rtsds_amd import set_compute_dtype

set_compute_dtype(torch.bfloat16)
wl = sys.argv.pop(1) if len(sys.argv) > 1 else "bisenet-seg"
args = bench.parse()
args.workload, args.batch, args.da_unfused = wl, bench.WORKLOADS[wl][2], False
dev = torch.device("cuda", 0)
net, x, set_lr, core, opts = bench.build(args, dev, 0)
for i in range(2):
    set_lr(i)
    core()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    set_lr(2)
    core()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ka if e.device_type.name == "CUDA" or "Memcpy" in e.key or "Memset" in e.key]
for e in prof.events():
    pass
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=40))
for e in prof.key_averages(group_by_input_shape=True):
    if any(k in e.key for k in ("copy", "Memcpy", "Memset", "fill", "elementwise", "zero", "Copy")):
        print(f"{e.key[:70]:70s} n={e.count:3d} cuda_us={e.self_device_time_total:8.1f} shapes={str(e.input_shapes)[:120]}")
# aten ops that launch device work, with stacks
for e in prof.key_averages(group_by_stack_n=8):
    if e.key.startswith("aten::") and e.key in ("aten::copy_", "aten::zero_", "aten::fill_", "aten::zeros", "aten::add_",
                                                  "aten::mul", "aten::div", "aten::add", "aten::sum", "aten::clone",
                                                  "aten::contiguous", "aten::cat", "aten::to", "aten::_to_copy",
                                                  "aten::item", "aten::index", "aten::masked_fill_", "aten::where"):
        print(f"{e.key:22s} n={e.count:3d} shapes={e.input_shapes}")
        for s in e.stack[:8]:
            print("      ", s)
