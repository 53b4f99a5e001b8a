"""Per-launch durations of the damvs kernels in one forward of a rocprofv3 kernel trace
(argv[2] = forward index, default the last).

  python tools/prof_damvs_launches.py run_kernel_trace.csv [forward]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# one regression launch per stage (prob_mfma_kernel or prob_regress_kernel), 3 per forward
reg = [i for i, r in enumerate(rows) if "regress_kernel" in r["Kernel_Name"] or "prob_mfma_kernel" in r["Kernel_Name"]]
ends = reg[2::3]
step = int(sys.argv[2]) if len(sys.argv) > 2 else len(ends) - 1
sel = rows[ends[step - 1] + 1:ends[step] + 1]
tot = 0.0


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0].replace("void ", "").replace("damvs::", "").replace(" ", "")[:60]


for r in sel:
    n = r["Kernel_Name"]
    if "damvs" in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print("%8.1f us  grid %9s x %2s  vgpr %3s lds %6s  %s" % (d, r["Grid_Size_X"], r["Grid_Size_Y"], r["VGPR_Count"],
                                                               r["LDS_Block_Size"], short(n)))
print("damvs total %.1f us" % tot)
