"""bench.py's N > 1 path as a CPU gloo job (tests/test_bench_multirank.py launches it under torch.distributed.run).

Everything bench.main() does across ranks runs for real -- the process group, the barriers around the timed steps,
the max-over-ranks timing, rank 0's JSON line, the timer guard around the depth-sharded blocks and the all_reduce
failure flag after each block -- while the GPU work is replaced by CPU stand-ins: a stub model whose forward sleeps
a few milliseconds, HIP events as host clocks, and sharded blocks whose behaviour DAMVS_DRYRUN selects:
  ok    both sharded blocks succeed on every rank
  fail  rank 1 raises inside the "gather" block after its last exchange (the flag must mark it failed on every rank)
  hang  rank 1 sleeps in the first block past the guard (rank 0's line must go out, exit status 3)
No GPU, no HIP library: the product path is not exercised here (tests/test_gpu_*.py do that).
"""
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import damvsnet_amd.dist as D  # noqa: E402

MODE = os.environ.get("DAMVS_DRYRUN", "ok")


class _Event:
    def __init__(self, enable_timing=True):
        self.t = None
        self.cuda_event = 0

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class _DepthNet:
    probe = None

    def check_range(self):
        pass


class _Net:
    """Stand-in for CascadeMVSNet: 2 ms per forward, stage hooks and probes called as the real one calls them."""

    def __init__(self):
        self.DepthNet = _DepthNet()

    def __call__(self, imgs, proj, dv, ins=None, stage_hook=None, streams=1, check_range=True, depthnet=None):
        hook = stage_hook or (lambda n: None)
        hook("features")
        for s in range(3):
            hook("stage%d.depthnet" % (s + 1))
            if self.DepthNet.probe is not None:
                for e in self.DepthNet.probe(s):
                    e.record()
                    time.sleep(0.0002)
            time.sleep(0.0007)
        hook("end")
        return {}


def _sharded(net, H, W, N, device, comm=None, emulate=1, warp="depth", steps=5, warmup=2):
    rank = dist.get_rank()
    if MODE == "hang" and rank == 1:
        time.sleep(60)
    el = D.max_over_ranks(0.01, device=bench.coll_device(device))
    if MODE == "fail" and warp == "gather" and rank == 1:  # after the block's last exchange: only the flag tells rank 0
        raise RuntimeError("dry-run failure on rank 1")
    return {"ms_per_map": round(el * 1e3, 3), "ranks": dist.get_world_size(), "warp": warp, "transport": "gloo dry run"}


def main():
    torch.cuda.set_device = lambda *a, **k: None
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.Event = _Event
    _init = dist.init_process_group
    dist.init_process_group = lambda backend=None, device_id=None, **k: _init("gloo", **k)
    bench.SHARD_GUARD_S = 8
    bench.build_model = lambda *a, **k: (_Net(), None)
    bench.make_inputs = lambda B, N, H, W, device=None, seed=0: (torch.zeros(B, N, 3, 8, 8), {}, torch.zeros(B, 2), {})
    bench.latency_b1 = lambda *a, **k: {"ms_per_map": 0.0, "ms_per_stage": {}}
    bench.warp_roofline = lambda *a, **k: (1.0, 1)
    bench.hot_path_roofline = lambda *a, **k: {"dry_run": True}
    bench.pmc_traffic = lambda *a, **k: None
    bench.pmc_mfma = lambda *a, **k: None
    bench.sharded_latency = _sharded
    bench.main()


if __name__ == "__main__":
    main()
