"""RTSDS MI355X benchmark -- BASELINE.json metric on configs[1]:
BiSeNet ResNet-18, 19 classes, 1024x512, batch 8 per GPU, bf16, seg-only train.py step.

One "step" = one train.train iteration body (train.py:65-113): zero_grad, poly LR,
forward (3 heads), 3x cross-entropy(ignore 19), backward, Adam step, pixel-accuracy count --
``rtsds_amd.train.seg_step`` on synthetic, HBM-resident inputs.  N GPUs = one process per GPU
(torchrun), each with its own batch of 8 (weak scaling); gradients all-reduced over RCCL
inside the optimizer step.  Prints ONE JSON line on rank 0.

``--workload`` selects the other BASELINE.json configs as separate bench lines (the default is
configs[1]): ``bisenet-da`` (configs[3] per GPU: adversarial_train iteration, 8 source + 8
target 1024x512 images, TinyDomainDiscriminator), ``deeplab-seg`` (configs[2]: DeepLabV2
ResNet-101 + ASPP seg step, bs 4, 1024x512), ``deeplab-da`` (configs[4] per GPU: DeepLabV2 DA
iteration, 2 + 2 images at 1280x720).  Unit: source images/s (one DA unit = a source image
with its paired target image).

Extra fields: inference FPS (eval forward, bs 8 and bs 1), the live conv roofline
(HIP events around every implicit-GEMM launch over one extra step after the timed
region), and the CPU baseline (the oracle's restatement of the reference step on the host
cores, bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)
NC = 19
# north_star's inference roofline: BiSeNet-R18 eval forward at 1024x512 is
# 51.26 GFLOP per image; at bs 8 the per-layer roofline sum_i max(flop_i / 2.5 PF, bytes_i /
# 8 TB/s) is t_roof = 0.266 ms (conv traffic >= 1.72 GB), the MFMA-only time 0.164 ms
INFER_GFLOP_PER_IMG = 51.26
INFER_T_ROOF_MS_BS8 = 0.266
# default timed steps per workload: >= ~2.4 s of timed work at the round-2 step times, so the
# driver's own wall clock and GPU-busy sampler can corroborate the measured window
DEFAULT_STEPS = {"bisenet-seg": 400, "bisenet-da": 160, "deeplab-seg": 70, "deeplab-da": 40}
# workload -> (model, DA?, default per-GPU batch, H, W, conv GFLOP per unit, BASELINE config)
WORKLOADS = {
    "bisenet-seg": ("bisenet", False, 8, 512, 1024, 151.6, "configs[1]: BiSeNet-R18 seg-only train step (train.py:65-113)"),
    "bisenet-da": ("bisenet", True, 8, 512, 1024, 333.8,
                   "configs[3] per GPU: BiSeNet-R18 + TinyD adversarial_train iteration (train.py:172-284)"),
    "deeplab-seg": ("deeplab", False, 4, 512, 1024, 2239.5,
                    "configs[2]: DeepLabV2-R101 + ASPP seg-only train step (train.py:65-113)"),
    "deeplab-da": ("deeplab", True, 2, 720, 1280, 7881.3,
                   "configs[4] per GPU: DeepLabV2-R101 + TinyD adversarial_train iteration (train.py:172-284)"),
}
H, W = 512, 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: the workload's, >= 2 s of timed work)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="bisenet-seg", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the workload's)")
    ap.add_argument("--allreduce-dtype", default="fp32", choices=["fp32", "fp16", "bf16"],
                    help="gradient all-reduce wire dtype (N>1)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-infer", action="store_true")
    ap.add_argument("--conv-report", action="store_true")
    ap.add_argument("--da-unfused", action="store_true",
                    help="A/B: discriminator input through interpolate + softmax (no fused upsample_softmax)")
    ap.add_argument("--no-conv-profile", action="store_true", help="skip the event-timed roofline step")
    ap.add_argument("--submit", default="auto", choices=["auto", "branches", "serial", "split"],
                    help="graph submission variant (runtime.GraphedStep; auto = time both captures, keep the faster)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the iteration as hipGraph segments (auto = on; under data parallelism "
                         "the RCCL collectives run between the segments, runtime.GraphedStep)")
    return ap.parse_args()


def synthetic_batch(n, seed, device, h=H, w=W):
    """ImageNet-normalised 0-255 images + labels in [0, 19] (19 = ignore), SURVEY 8(d)."""
    H, W = h, w
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 256, (n, 3, H, W), generator=g).float()
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    x = (x - mean) / std
    y = torch.randint(0, NC + 1, (n, H, W), generator=g)
    return x.to(device), y.to(device)


def host_cpus():
    """CPUs this process may actually run on: the affinity mask, further capped by a cgroup
    CPU quota when one is set (the GPU box gives a job a share of a larger machine, and
    os.cpu_count() reports the whole machine there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = period = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2
            quota, period = f.read().split()[:2]
    except (OSError, ValueError):
        try:  # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                quota = f.read().strip()
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = f.read().strip()
        except OSError:
            pass
    try:
        if quota not in (None, "max", "-1"):
            n = min(n, max(1, -(-int(quota) // int(period))))
    except ValueError:
        pass
    return max(1, n)


def cpu_baseline(seconds=15.0):
    """Oracle (plain-PyTorch CPU restatement of the reference, pinned to the reference's
    golden captures) timed on the host: train step at 1024x512, batch 2, with one intra-op
    thread per CPU available to the process (host_cpus)."""
    from oracle import models as om
    from oracle import steps as osteps
    from oracle.weights import apply_recipe, synthetic_images, synthetic_labels
    threads = host_cpus()
    torch.set_num_threads(threads)
    net = apply_recipe(om.BiSeNet(NC, "resnet18"), seed=1).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    ce = torch.nn.CrossEntropyLoss(ignore_index=NC)
    x = synthetic_images(2, H, W, seed=42)
    y = synthetic_labels(2, H, W, seed=43)
    osteps.seg_step(net, opt, ce, x, y)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        osteps.seg_step(net, opt, ce, x, y)
        n += 1
        if time.perf_counter() - t0 > seconds or n >= 20:
            break
    dt = time.perf_counter() - t0
    return {"value": round(2 * n / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "host_cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "sample": f"oracle BiSeNet-R18 train step (fwd+3xCE+bwd+Adam), fp32, 2x3x512x1024, "
                      f"{n} timed steps after 1 warm-up ({dt:.1f} s)"}


def conv_traffic(args, dtype):
    """HBM bytes per step of the conv kernels, from the newest committed rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this same workload at its default batch in bf16
    (tools/profile_all.sh -> profiles/r<NN>_<workload>_pmc_traffic.json; gfx950 FETCH_SIZE x2)."""
    import glob
    if args.batch != WORKLOADS[args.workload][2] or dtype != torch.bfloat16:
        return None
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{args.workload}_pmc_traffic.json")))
    if not paths:
        return None
    with open(paths[-1]) as f:
        return json.load(f)["conv_gemm_kernel_bytes_per_step"]


def build(args, dev, rank):
    """Model(s), optimizer(s), synthetic resident inputs and the step closure of the workload."""
    from rtsds_amd import losses, optim
    from rtsds_amd.train import da_step, seg_step
    from rtsds_amd.utils import poly_lr_scheduler
    model, da, _, h, w, _, _ = WORKLOADS[args.workload]
    if model == "bisenet":
        from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
        net = BiSeNet(NC, "resnet18").to(dev).train()
    else:
        from rtsds_amd.models.deeplabv2.deeplabv2 import get_deeplab_v2
        net = get_deeplab_v2(NC, pretrain=False).to(dev).train()
    opt = optim.Adam(net.parameters(), lr=1e-4)
    crit = losses.CrossEntropyLoss(ignore_index=NC)
    x, y = synthetic_batch(args.batch, 42 + 2 * rank, dev, h, w)
    max_iter = 1000
    if not da:
        def set_lr(i):
            poly_lr_scheduler(opt, 1e-4, i, 1, max_iter, 0.9)

        def core():
            return seg_step(net, crit, opt, x, y)
        return net, x, set_lr, core, [opt]
    from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator
    disc = TinyDomainDiscriminator(NC).to(dev).train()
    if args.da_unfused:
        disc.accepts_padded_probs = False
    dopt = optim.Adam(disc.parameters(), lr=1e-4, weight_decay=1e-4)
    bce = losses.BCEWithLogitsLoss()
    xt, _ = synthetic_batch(args.batch, 43 + 2 * rank, dev, h, w)
    poly_lr_scheduler(dopt, 1e-4, 0, 1, 10, 0.05)  # per epoch (train.py:167)

    def set_lr(i):
        poly_lr_scheduler(opt, 1e-4, i, 1, max_iter, 0.9)

    def core():
        out = da_step(net, disc, opt, dopt, crit, bce, x, y, xt, 0.1, 100)  # lambda, iterations: config.yaml
        return out[0], out[-1]
    return net, x, set_lr, core, [opt, dopt]


def launch_ranks(args):
    """``--gpus N`` (N > 1) without a torchrun environment: start N ranks (one process per
    GPU) under torch.distributed.run as a CHILD process -- nothing here has touched the GPU
    yet -- and exit with its status; rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    env_world = int(os.environ.get("WORLD_SIZE", "0"))
    if env_world == 0 and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world and env_world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)
    if args.steps is None:
        args.steps = DEFAULT_STEPS[args.workload]
    from rtsds_amd import functional as F
    from rtsds_amd import optim, set_compute_dtype
    from rtsds_amd.utils import init_distributed

    wl = WORKLOADS[args.workload]
    if args.batch is None:
        args.batch = wl[2]
    rank, local, world = init_distributed()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:  # the ranks the collective backend actually formed
        world = dist.get_world_size()
        backend = dist.get_backend()
    else:
        backend = None
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    set_compute_dtype(dtype)
    optim.set_allreduce_dtype({"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[args.allreduce_dtype])
    torch.manual_seed(42)
    net, x, set_lr, core, opts = build(args, dev, rank)
    use_graph = args.graph in ("on", "auto")

    def step(i):
        set_lr(i)
        return core()

    for i in range(args.warmup):
        step(i)
    if use_graph:
        # the whole iteration as hipGraph replays (runtime.GraphedStep): same kernels, no
        # per-kernel host launches; lr / Adam step advance through a device buffer; under data
        # parallelism the collectives run between the graph segments
        from rtsds_amd.runtime import GraphedStep
        try:
            graphed = GraphedStep(core, opts, warmup=1, submit=args.submit)
        except Exception as e:  # keep the measurement alive on the eager path
            print(f"bench: hipGraph capture failed ({e!r}); timing eager iterations", file=sys.stderr)
            for o in opts:
                o.set_graph_mode(False)
            use_graph = False
    if use_graph:
        def step(i):
            set_lr(i)
            return graphed()
        # untimed replays until GraphedStep has timed its submission variants and kept one
        j = args.warmup
        while True:
            step(j)
            j += 1
            if graphed.submit_choice is not None:
                break
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if use_graph:
        graphed.host_launch_s = 0.0
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss, corr = step(args.warmup + i)
    t_enqueue = time.perf_counter() - t0
    t_launch = graphed.host_launch_s if use_graph else t_enqueue
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / args.steps
    imgs = args.batch * world * args.steps / elapsed
    final_loss = float(loss.item())

    # ---- live conv roofline: one more step with HIP events around each implicit-GEMM launch
    recs = []
    if not args.no_conv_profile:
        # a GPU-bound spacer ahead of the profiled step lets the host run ahead, so the step's
        # launches queue back to back and each conv's events bracket GPU time rather than the
        # host launch gaps of an eager step (~40 ms of bf16 GEMMs vs ~8 ms of host enqueue)
        spacer = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
        torch.cuda.synchronize()
        for _ in range(40):
            torch.mm(spacer, spacer)
        F.CONV_PROFILE = []
        set_lr(args.warmup + args.steps)
        core()  # eager: HIP events around each conv launch
        torch.cuda.synchronize()
        recs, F.CONV_PROFILE = F.CONV_PROFILE, None
        del spacer
    conv_ms = sum(r[0].elapsed_time(r[1]) for r in recs) or float("nan")
    conv_flop = sum(r[2] for r in recs)

    def conv_report(recs):
        rows = []
        for e0, e1, fl, tag, d in recs:
            ms_ = e0.elapsed_time(e1)
            rows.append((ms_, tag, f"n{d.n} {d.h}x{d.w}x{d.c} -> {d.ho}x{d.wo}x{d.k} k{d.kh} s{d.sh} d{d.dh}",
                         fl / 1e9, fl / (ms_ * 1e-3) / 1e12))
        rows.sort(reverse=True)
        for r in rows:
            print(f"{r[0]*1000:8.1f} us  {r[1]:5s} {r[2]:45s} {r[3]:7.2f} GF {r[4]:7.1f} TF/s", file=sys.stderr)
        for tag in ("fwd", "dgrad", "wgrad"):
            sel = [r for r in rows if r[1] == tag]
            print(f"total {tag:5s} {sum(r[0] for r in sel):8.3f} ms over {len(sel)} convs", file=sys.stderr)
        print(f"total conv  {sum(r[0] for r in rows):8.3f} ms, {sum(r[3] for r in rows):.1f} GF", file=sys.stderr)
    if args.conv_report and rank == 0:
        conv_report(recs)
    achieved = conv_flop / (conv_ms * 1e-3) / 1e12

    # ---- inference FPS (eval forward, no grad)
    # Eval-mode forward (BN folded into the conv epilogues), replayed as one hipGraph per batch
    # size (runtime.GraphedForward); each replay copies the batch into the captured input.
    infer = {}
    if not args.no_infer and args.workload == "bisenet-seg":
        from rtsds_amd.runtime import GraphedForward
        net.eval()
        with torch.no_grad():
            for bs in (args.batch, 1):
                xb = x[:bs].contiguous()
                fwd = GraphedForward(net, xb)
                for _ in range(3):
                    fwd(xb)
                torch.cuda.synchronize()
                k = 50 if bs > 1 else 200
                t1 = time.perf_counter()
                for _ in range(k):
                    fwd(xb)
                torch.cuda.synchronize()
                infer[f"inference_fps_bs{bs}"] = round(bs * k * world / (time.perf_counter() - t1), 2)
                # eager (no graph) for reference
                t1 = time.perf_counter()
                for _ in range(k // 5):
                    net(xb)
                torch.cuda.synchronize()
                infer[f"inference_fps_bs{bs}_eager"] = round(bs * (k // 5) * world / (time.perf_counter() - t1), 2)
                if bs == 8 and dtype == torch.bfloat16:
                    # north_star's headline: fraction of the MFMA roofline of the bs-8 forward
                    # (whole forward, graph replay), plus the event-timed conv family of one
                    # eager eval forward queued behind a GPU spacer (as the train roofline)
                    fps = infer["inference_fps_bs8"] / world
                    t_ms = 1000.0 * bs / fps
                    spacer = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
                    for _ in range(20):
                        torch.mm(spacer, spacer)
                    F.CONV_PROFILE = []
                    net(xb)
                    torch.cuda.synchronize()
                    irecs, F.CONV_PROFILE = F.CONV_PROFILE, None
                    if args.conv_report and rank == 0:
                        print("-- eval forward (bs 8):", file=sys.stderr)
                        conv_report(irecs)
                    del spacer
                    ims = sum(r[0].elapsed_time(r[1]) for r in irecs)
                    ifl = sum(r[2] for r in irecs)
                    infer["inference_roofline"] = {
                        "batch": bs, "gflop_per_image": INFER_GFLOP_PER_IMG, "ms_per_batch": round(t_ms, 4),
                        "mfma_achieved_tflops": round(INFER_GFLOP_PER_IMG * bs / t_ms, 2),
                        "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
                        "mfma_frac": round(INFER_GFLOP_PER_IMG * bs / t_ms / MFMA_BF16_PEAK_TFLOPS, 4),
                        "t_roof_ms": INFER_T_ROOF_MS_BS8,
                        "roofline_frac": round(INFER_T_ROOF_MS_BS8 / t_ms, 4),
                        "conv_family_ms": round(ims, 4), "conv_family_gflop": round(ifl / 1e9, 2),
                        "conv_family_frac": round(ifl / (ims * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4) if ims else None,
                        "conv_launches": len(irecs),
                        "note": "mfma_frac = 51.26 GFLOP/img x FPS / 2.5 PF; roofline_frac = t_roof / t_measured "
                                "(SURVEY.md 8(d)); conv_family_* from HIP events around each conv call of one "
                                "eager eval forward"}
                del fwd
        net.train()

    out = {
        "metric": "images/sec/node (train step) + inference FPS@1024x512, BiSeNet 19-cls",
        "value": round(imgs, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (ImageNet-normalised 0-255 images, labels 0..19, 19=ignore; random-init weights)",
        "config": {"workload": wl[6], "model": "BiSeNet-ResNet18" if wl[0] == "bisenet" else "DeepLabV2-ResNet101",
                   "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                   "image": f"3x{wl[3]}x{wl[4]}", "num_classes": NC, "parallelism": f"dp{world}",
                   **({"discriminator": "TinyDomainDiscriminator", "target_batch_per_gpu": args.batch} if wl[1] else {}),
                   **({"grad_allreduce_dtype": args.allreduce_dtype} if world > 1 else {})},
        **infer,
        "roofline": {"bound": "mfma", "kernel": "conv_gemm_kernel (implicit-GEMM conv fwd/dgrad/wgrad, "
                                                "incl. dgrad repack + wgrad split-reduce launches)",
                     "achieved": round(achieved, 2), "peak": MFMA_BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else 157.3,
                     "unit": "TFLOP/s", "frac": round(achieved / (MFMA_BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else 157.3), 4),
                     "traffic": conv_traffic(args, dtype), "traffic_unit": "HBM bytes per step, all conv launches",
                     "launches_per_step": len(recs),
                     "conv_ms_per_step": round(conv_ms, 3),
                     "conv_gflop_per_step": round(conv_flop / 1e9, 1)},
        "whole_step_conv_flop_rate_tflops": round(wl[5] * args.batch / ms, 2),
        "final_loss": round(final_loss, 4),
        # host time submitting the iteration (graph segment launches + collectives), and the
        # host loop's total per step (includes waiting once it runs 8 steps ahead of the GPU)
        "host_launch_ms_per_step": round(1000.0 * t_launch / args.steps, 3),
        "host_enqueue_ms_per_step": round(1000.0 * t_enqueue / args.steps, 3),
        "hip_graph": use_graph,
        **({"graph_submit": graphed.submit_choice, "graph_submit_trials": graphed.submit_trials,
            "graph_segments": len(graphed.segments)} if use_graph else {}),
        "timed_s": round(elapsed, 3),
        **({"ranks": world, "backend": backend} if backend else {}),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "bisenet-seg":
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
