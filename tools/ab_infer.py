"""Inference A/B inside one process: BiSeNet-R18 eval forward at 1024x512 (bench.py's
inference path, GraphedForward replays), alternating between settings of a model class
attribute.  usage: python tools/ab_infer.py ATTR V1 V2 ... [--batch 8] [--reps 200] [--rounds 4]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("attr")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=4)
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
    fwds, outs = {}, {}
    with torch.no_grad():
        for v in a.values:
            setattr(BiSeNet, a.attr, eval(v))
            fwds[v] = GraphedForward(net, x)
            outs[v] = fwds[v](x).clone()
        ref = outs[a.values[0]]
        for v in a.values[1:]:
            print(f"{a.attr}={v}: output bit-identical to {a.values[0]}: {torch.equal(outs[v], ref)}", flush=True)
        for r in range(a.rounds):
            for v in a.values:
                f = fwds[v]
                for _ in range(5):
                    f(x)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(a.reps):
                    f(x)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                print(f"{a.attr}={v} bs {a.batch}: {1e3 * dt / a.reps:.4f} ms/batch, {a.batch * a.reps / dt:.1f} FPS", flush=True)


if __name__ == "__main__":
    main()
