"""Host cost of a replayed training iteration: time the pieces of
runtime.GraphedStep.__call__ -- stage_hyper, advance_steps, graph replays -- over K steps with
the GPU kept busy, for the graph captured with and without branch streams.

usage: python tools/diag/enqueue.py [--workload bisenet-seg] [--steps 40]
"""
import argparse
import contextlib
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
    a = ap.parse_args()
    import bench
    from rtsds_amd import runtime, set_compute_dtype
    set_compute_dtype(torch.bfloat16)
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(workload=a.workload, batch=bench.WORKLOADS[a.workload][2], da_unfused=False)
    for mode in ("branches", "serial"):
        torch.manual_seed(42)
        net, x, set_lr, core, opts = bench.build(args, dev, 0)
        ctx = runtime.branches_serial() if mode == "serial" else contextlib.nullcontext()
        with ctx:
            for i in range(3):
                set_lr(i)
                core()
            g = runtime.GraphedStep(core, opts, warmup=1)
        torch.cuda.synchronize()
        nodes = []
        for gr, _ in g.segments:
            try:
                nodes.append(gr.raw_cuda_graph().num_nodes() if hasattr(gr, "raw_cuda_graph") else -1)
            except Exception:
                nodes.append(-1)
        t = {"set_lr": 0.0, "stage": 0.0, "advance": 0.0, "replay": 0.0}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            s = time.perf_counter()
            set_lr(10 + i)
            s1 = time.perf_counter()
            for o in g.optimizers:
                o.stage_hyper()
            s2 = time.perf_counter()
            for o in g.optimizers:
                o.advance_steps()
            s3 = time.perf_counter()
            for gr, coll in g.segments:
                gr.replay()
            s4 = time.perf_counter()
            t["set_lr"] += s1 - s
            t["stage"] += s2 - s1
            t["advance"] += s3 - s2
            t["replay"] += s4 - s3
        enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"{a.workload} {mode}: segments {len(g.segments)}, wall {1e3 * wall / a.steps:.3f} ms/step, "
              f"enqueue {1e3 * enq / a.steps:.3f} ms/step: " +
              ", ".join(f"{k} {1e3 * v / a.steps:.3f}" for k, v in t.items()), flush=True)
        del g, net, opts, core
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
