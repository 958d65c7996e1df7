"""Vendor-library reference points for the conv suite shapes (diagnostic only, never on the
product path): MIOpen conv2d forward (torch, bf16 channels_last) and, for 1x1 convs, the
hipBLASLt GEMM of the same [M, K] x [K, N] (torch.mm), timed like tools/bench_conv.py.
usage: vendor_ref.py  (shapes: tools/conv_suite.sh's list)"""
import time

import torch
import torch.nn.functional as TF

torch.backends.cudnn.benchmark = True
SHAPES = """8 64 128 256 64 3 1 1
8 128 64 128 128 3 1 1
8 256 32 64 256 3 1 1
8 512 16 32 512 3 1 1
4 1024 65 129 256 1 1 0
4 256 65 129 1024 1 1 0
4 256 65 129 256 3 1 2 2
4 512 65 129 512 3 1 4 4
4 2048 65 129 512 1 1 0
8 1024 64 128 1024 3 1 1"""
dev = "cuda"


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


for line in SHAPES.splitlines():
    v = [int(a) for a in line.split()]
    n, c, h, w, k, kh, s, p = v[:8]
    dil = v[8] if len(v) > 8 else 1
    x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(k, c, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ho = (h + 2 * p - dil * (kh - 1) - 1) // s + 1
    wo = (w + 2 * p - dil * (kh - 1) - 1) // s + 1
    flop = 2.0 * n * ho * wo * k * c * kh * kh
    t = timeit(lambda: TF.conv2d(x, wt, None, s, p, dil))
    out = f"{line:28s} miopen fwd {t * 1e6:8.1f} us {flop / t / 1e12:7.1f} TF/s"
    if kh == 1:
        a = x.permute(0, 2, 3, 1).reshape(-1, c)
        b = wt.reshape(k, c).t()
        t2 = timeit(lambda: torch.mm(a, b))
        out += f" | hipblaslt mm {t2 * 1e6:8.1f} us {flop / t2 / 1e12:7.1f} TF/s"
    print(out, flush=True)
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
t = timeit(lambda: torch.mm(a, b), 10)
print(f"hipblaslt 8192^3 {t * 1e6:.1f} us {2 * 8192 ** 3 / t / 1e12:.1f} TF/s")
