"""How a multi-stream hipGraph replay schedules a side branch: main = a chain of 20 spin
kernels, side = 5 spin kernels depending only on main's first kernel.  Captured with the side
branch issued early (right after the fork) or late (after the whole main chain), plus a serial
capture.  Replay time shows whether the side chain overlaps the main chain."""
import torch

torch.cuda.init()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
cyc = 20000
for _ in range(3):
    e0.record(); torch.cuda._sleep(cyc); e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3
cyc = int(cyc * 50.0 / us)  # ~50 us per spin kernel
e0.record(); torch.cuda._sleep(cyc); e1.record(); torch.cuda.synchronize()
print(f"spin kernel: {e0.elapsed_time(e1) * 1e3:.1f} us", flush=True)


def body(mode, main, side):
    torch.cuda._sleep(cyc)
    ev = torch.cuda.Event()
    ev.record(main)
    if mode == "early":
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for _ in range(5):
                torch.cuda._sleep(cyc)
    for _ in range(19):
        torch.cuda._sleep(cyc)
    if mode == "serial":
        for _ in range(5):
            torch.cuda._sleep(cyc)
    if mode == "late":
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for _ in range(5):
                torch.cuda._sleep(cyc)
    if mode != "serial":
        main.wait_stream(side)


for mode in ("serial", "early", "late"):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    side = torch.cuda.Stream()
    with torch.cuda.stream(cap):
        side.wait_stream(cap)
        with torch.cuda.graph(g, stream=cap):
            body(mode, cap, side)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for lock in (False, True):
        e0.record()
        for _ in range(20):
            g.replay()
            if lock:
                torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        print(f"{mode:6s} {'lockstep' if lock else 'queued  '}: {e0.elapsed_time(e1) * 1e3 / 20:8.1f} us per replay "
              f"(serial sum {25 * 50} us, overlapped {20 * 50} us)", flush=True)
