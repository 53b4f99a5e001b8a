"""A/B: the B=4 cfgC forward as one batch on one stream vs S sub-batches on S concurrent HIP streams.

The sub-batches are independent reference views (results are per-sample identical, batch composition does
not enter any kernel), so concurrent streams let kernels with different bounds overlap (the TA-bound
warp of one sub-batch beside the HBM/MFMA-bound U-Net or front-end of another).
  python tools/streams_ab.py [--streams 1,2,4] [--steps 10]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import bench
    H, W, N, nd, dtype, _ = bench.CONFIGS[args.config]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    imgs, proj, dv, ins = bench.make_inputs(args.batch, N, H, W, dev)
    main_s = torch.cuda.current_stream()
    ref = None
    for S in [int(x) for x in args.streams.split(",")]:
        streams = [torch.cuda.Stream() for _ in range(S)]
        cb = args.batch // S
        chunks = [(imgs[i * cb:(i + 1) * cb], {k: v[i * cb:(i + 1) * cb] for k, v in proj.items()},
                   dv[i * cb:(i + 1) * cb]) for i in range(S)]

        def step():
            outs = []
            for st, (im, pr, d) in zip(streams, chunks):
                st.wait_stream(main_s)
                with torch.cuda.stream(st):
                    outs.append(net(im, pr, d))
            for st in streams:
                main_s.wait_stream(st)
            return outs

        with torch.no_grad():
            for _ in range(3):
                outs = step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                outs = step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
        depth = torch.cat([o["depth"] for o in outs])
        with torch.no_grad():  # the same sub-batches one after another on one stream; and the concurrent run again
            seq_outs = [net(im, pr, d) for im, pr, d in chunks]
            seq = torch.cat([o["depth"] for o in seq_outs])
            torch.cuda.synchronize()
            again = [torch.cat([o["depth"] for o in step()]) for _ in range(5)]
        torch.cuda.synchronize()
        for st_name in ("stage1", "stage2", "stage3"):
            for key in ("depth", "photometric_confidence", "prob_volume"):
                a_ = torch.cat([o[st_name][key] for o in outs])
                b_ = torch.cat([o[st_name][key] for o in seq_outs])
                if not torch.equal(a_, b_):
                    print("  first difference concurrent vs sequential: %s %s (%d elements)" % (
                        st_name, key, int((a_ != b_).sum())), flush=True)
                    break
            else:
                continue
            break
        print("  concurrent runs bitwise equal to the sequential sub-batches: %d of %d; sequential vs streams=1: %s" % (
            sum(torch.equal(x, seq) for x in again + [depth]), len(again) + 1,
            torch.equal(seq, ref) if ref is not None else True), flush=True)
        if ref is None:
            ref = depth
        print("streams %d (B=%d each): %.3f ms per %d maps = %.2f maps/s; depth bitwise equal to the same "
              "sub-batches on one stream: %s, to streams=%s: %s (max rel %.2e)"
              % (S, cb, dt * 1e3, args.batch, args.batch / dt, torch.equal(depth, seq), args.streams.split(",")[0],
                 torch.equal(depth, ref), ((depth - ref).abs() / ref.abs().clamp_min(1e-6)).max().item()), flush=True)


if __name__ == "__main__":
    main()
