"""Data-parallel plumbing on CPU (gloo, world size 2): environment-driven init and the flat
gradient all-reduce (a plain SUM: the losses are normalised by the global batch,
rtsds_amd/runtime.py dp_world)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtsds_amd.optim import allreduce_flat


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, wire="fp32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from rtsds_amd.utils import init_distributed
    r, local, w = init_distributed("gloo")
    assert (r, w) == (rank, world)
    from rtsds_amd.optim import set_allreduce_dtype
    set_allreduce_dtype({"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[wire])
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    scale = allreduce_flat([g])
    q.put((rank, g.tolist(), scale))
    dist.barrier()
    dist.destroy_process_group()


def _async_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from rtsds_amd.utils import init_distributed
    init_distributed("gloo")
    from rtsds_amd.optim import allreduce_start
    a = torch.arange(6, dtype=torch.float32) * (rank + 1)
    b = torch.ones(3) * (rank + 10)
    finish = allreduce_start([a, b])
    finish()
    q.put((rank, a.tolist(), b.tolist(), finish is not None))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_async_allreduce_start_finish():
    """optim.allreduce_start (the DA iteration's early, overlapped gradient all-reduce):
    after finish() every buffer holds the SUM over ranks, exactly as the serial path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_async_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, a, b, started in res:
        assert started
        assert a == [float(3 * i) for i in range(6)]
        assert b == [21.0] * 3


@pytest.mark.parametrize("wire", ["fp32", "fp16"])
@pytest.mark.parametrize("world", [2])
def test_gloo_flat_allreduce(world, wire):
    """Exact for small integers in every wire dtype (fp16 represents 0..27 exactly)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, wire)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = [float(i * sum(r + 1 for r in range(world))) for i in range(10)]
    for rank, vals, scale in res:
        assert vals == want
        assert scale == 1.0


def test_single_process_is_identity():
    g = torch.ones(4)
    assert allreduce_flat([g]) == 1.0
    assert g.tolist() == [1.0] * 4
