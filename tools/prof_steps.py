"""Per-kernel time inside the timed bench steps from a rocprofv3 kernel trace (csv).

Steps are delimited by the regression kernels (one prob_regress / prob_mfma / head launch per stage, 3 per
forward). Also prints the average of the last `roofline_iters` launches of the roofline kernel
(bench.py's warp_roofline loop runs last), to check against the bench line's roofline.ms_per_launch."""
import collections
import csv
import sys


ROOFLINE_KERNEL = "warp_split_kernel<unsigned short, 16,"  # stage 2 (C = 16), bf16, channel-split form


def main(path, warmup=2, steps=5, top=40, roofline_iters=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    reg = [i for i, r in enumerate(rows) if any(k in r["Kernel_Name"] for k in ("regress_kernel", "prob_mfma_kernel", "head_kernel"))]
    ends = reg[2::3]  # last regress of each forward
    first = ends[warmup - 1] + 1
    last = ends[warmup + steps - 1]
    sel = rows[first:last + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += d
    busy = sum(a[1] for a in agg.values()) / steps
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / steps
    print("per step: kernel-busy %.1f us, wall %.1f us, %d launches" % (busy, wall, len(sel) // steps))
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print("%9.1f us/step %4d/step avg %8.1f us  %5.1f%%  %s" % (t / steps, n // steps, t / n, 100 * t / steps / busy,
                                                                   name[:100]))
    rl = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if ROOFLINE_KERNEL in r["Kernel_Name"]]
    if len(rl) >= roofline_iters:
        print("roofline kernel (%s...): last %d launches avg %.4f ms" % (ROOFLINE_KERNEL, roofline_iters,
                                                                       sum(rl[-roofline_iters:]) / roofline_iters))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
