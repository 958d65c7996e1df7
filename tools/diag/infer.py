"""Eval-mode BiSeNet-R18 forward at 1024x512 (bench.py's inference_fps_bs8 path): hipGraph
replays of runtime.GraphedForward, for rocprofv3 kernel traces of the inference path.

usage: python tools/diag/infer.py [--batch 8] [--reps 20]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from rtsds_amd import set_compute_dtype
    from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
    from rtsds_amd.runtime import GraphedForward
    set_compute_dtype(torch.bfloat16)
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    net = BiSeNet(19, "resnet18").to(dev).eval()
    x, _ = bench.synthetic_batch(a.batch, 42, dev)
    with torch.no_grad():
        fwd = GraphedForward(net, x)
        for _ in range(3):
            fwd(x)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            fwd(x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"bs {a.batch}: {a.reps} replays, {1e3 * dt / a.reps:.3f} ms/batch, {a.batch * a.reps / dt:.1f} FPS", flush=True)


if __name__ == "__main__":
    main()
