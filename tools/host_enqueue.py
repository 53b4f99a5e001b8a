"""Host enqueue time of the bench forward (GPU box): wall time of the Python call that enqueues one step (no
synchronisation inside) against the step's GPU time, for 1 and 2 streams. If the enqueue time reaches the step
time the host, not the GPU, sets the rate.

  python tools/host_enqueue.py [--config cfgC] [--batch 4]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4)
    args = ap.parse_args()
    import bench
    H, W, N, nd, dt, _ = bench.CONFIGS[args.config]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dt, dev)
    imgs, proj, dv, ins = bench.make_inputs(args.batch, N, H, W, dev, seed=0)
    with torch.no_grad():
        for streams in (1, 2, 1, 2):
            for _ in range(3):
                net(imgs, proj, dv, ins, streams=streams)
            torch.cuda.synchronize()
            enq, tot = [], []
            for _ in range(10):
                t0 = time.perf_counter()
                net(imgs, proj, dv, ins, streams=streams)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                enq.append((t1 - t0) * 1e3)
                tot.append((t2 - t0) * 1e3)
            enq.sort(); tot.sort()
            print("streams %d: enqueue %.2f ms (median), enqueue+drain %.2f ms" % (streams, enq[5], tot[5]), flush=True)


if __name__ == "__main__":
    main()
