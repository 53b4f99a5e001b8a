"""Per-kernel time inside the timed bench steps from a rocprofv3 kernel trace (csv).

Steps are delimited by the stage-3 regression kernel (3 regress launches per forward)."""
import collections
import csv
import sys


def main(path, warmup=2, steps=5, top=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    reg = [i for i, r in enumerate(rows) if "regress_kernel" in r["Kernel_Name"]]
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


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
