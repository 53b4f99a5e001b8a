"""Launch segments of the roofline kernel in a rocprofv3 kernel trace of `python bench.py`.

The bench launches the stage-2 warp with three grid sizes: the timed steps run the batch as sub-batches on
concurrent streams, the attribution pass runs the whole batch on one stream (bench.py's
`roofline.ms_per_launch` is this pass's launch time, from HIP events around it), and the isolated loop
(`roofline.isolated_ms_per_launch`) repeats the whole-batch launch back to back. This prints the launches in
time order as segments of equal grid, each with its count and mean duration, so the bench line can be
checked against the trace.
  python tools/prof_roofline_kernel.py <run_kernel_trace.csv> [kernel-name prefix]
"""
import csv
import sys


def main(path, prefix="warp_split_kernel<unsigned short, 16,"):
    rows = sorted((r for r in csv.DictReader(open(path)) if prefix in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    segs = []
    for r in rows:
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if segs and segs[-1][0] == grid:
            segs[-1][1].append(d)
        else:
            segs.append((grid, [d]))
    print("kernel %s... launch segments in time order" % prefix)
    for grid, v in segs:
        print("  grid %-9s %3d launches, mean %.4f ms (min %.4f, max %.4f)" % (grid, len(v), sum(v) / len(v), min(v),
                                                                            max(v)))


if __name__ == "__main__":
    main(*sys.argv[1:])
