"""CPU, gloo, world_size 2: the multi-GPU harness (sharding, MAX timing, result gather) that bench.py
and damvsnet_amd.dist use, exercised with a pure-CPU stand-in for the per-sample forward."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from damvsnet_amd import dist as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world_size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        n = 7
        out = D.run_sharded(lambda i: torch.full((2, 3), float(i * 10 + 1)), n)
        t = D.max_over_ranks(1.5 + rank)
        if rank == 0:
            q.put(("maps", [float(m[0, 0]) for m in out]))
            q.put(("max", t))
        else:
            q.put(("other", out is None))
    finally:
        dist.destroy_process_group()


def test_shard_indices_partition():
    for n in (0, 1, 7, 16):
        for ws in (1, 2, 3, 8):
            seen = sorted(i for r in range(ws) for i in D.shard_indices(n, r, ws))
            assert seen == list(range(n))


def test_single_process_passthrough():
    assert D.world() == (0, 1)
    assert D.max_over_ranks(3.0) == 3.0
    maps = D.run_sharded(lambda i: torch.tensor([i]), 3)
    assert [int(m) for m in maps] == [0, 1, 2]


@pytest.mark.timeout(120)
def test_gloo_world2_shard_gather_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(90)
        assert p.exitcode == 0
    got = dict(q.get(timeout=10) for _ in range(3))
    assert got["maps"] == [float(i * 10 + 1) for i in range(7)]
    assert got["max"] == 2.5
    assert got["other"] is True
