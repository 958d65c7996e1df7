"""Host cost and wall time of a replayed training iteration per graph-submission variant of
runtime.GraphedStep: "branches" (the multi-stream capture, hipGraphLaunch),
"serial" (captured without branch streams), "split" (multi-stream capture replayed as lane-split
linear segments, rtsds_graph_split) and "auto" (both captures, the faster kept after timed trial
replays).

usage: python tools/diag/enqueue.py [--workload bisenet-seg] [--steps 40] [--modes auto,branches,serial,split]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="bisenet-seg")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--modes", default="auto,branches,serial,split")
    a = ap.parse_args()
    import bench
    from rtsds_amd import runtime, set_compute_dtype
    set_compute_dtype(torch.bfloat16)
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload=a.workload, batch=bench.WORKLOADS[a.workload][2], da_unfused=False)
    for mode in a.modes.split(","):
        torch.manual_seed(42)
        net, x, set_lr, core, opts = bench.build(args, dev, 0)
        for i in range(3):
            set_lr(i)
            core()
        g = runtime.GraphedStep(core, opts, warmup=1, submit=mode)
        for i in range(8):  # trial replays of "auto"
            set_lr(3 + i)
            g()
        torch.cuda.synchronize()
        g.host_launch_s = 0.0
        t0 = time.perf_counter()
        for i in range(a.steps):
            set_lr(20 + i)
            g()
        enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        lanes = max(r.lanes for r, _ in g.runners)
        print(f"{a.workload} {mode}: kept {g.variant} ({len(g.segments)} capture segments, "
              f"{[r.segments for r, _ in g.runners]} launch units, {lanes} stream lanes), "
              f"wall {1e3 * wall / a.steps:.3f} ms/step, host loop {1e3 * enq / a.steps:.3f}, "
              f"host launch {1e3 * g.host_launch_s / a.steps:.3f} ms/step; trials {g.submit_trials}", flush=True)
        del g, net, opts, core
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
