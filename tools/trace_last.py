"""Print the damvs kernels of the last iteration of a rocprofv3 kernel trace (tools/kbench.py runs
3 warmup + N timed iterations; pass the number of iterations in total)."""
import csv
import sys

path, iters = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "damvs" in r["Kernel_Name"]]
n = len(rows) // iters
tot = 0.0
for r in rows[-n:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    nm = r["Kernel_Name"]
    nm = nm.split("(")[0] if not nm.startswith("void") else nm[5:]
    nm = nm.replace("damvs::(anonymous namespace)::", "")[:60]
    grid = r.get("Grid_Size") or r.get("Grid_Size_X")
    print("  %7.1f us  grid %9s  vgpr %3s  lds %6s  %s" % (d, grid, r.get("VGPR_Count", ""), r.get("LDS_Block_Size", ""), nm))
print("  total %.1f us" % tot)
