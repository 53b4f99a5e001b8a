"""Per-kernel table of every counter in a PMC output dir (first dispatch per kernel name+grid)."""
import collections
import csv
import glob
import sys

res = collections.OrderedDict()
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "damvs" not in r["Kernel_Name"]:
            continue
        nm = r["Kernel_Name"]
        nm = (nm[5:] if nm.startswith("void ") else nm).replace("damvs::(anonymous namespace)::", "").split("(")[0][:48]
        key = nm + " " + r["Grid_Size"]
        e = res.setdefault(key, {})
        e.setdefault(r["Counter_Name"], float(r["Counter_Value"]))
for k, v in res.items():
    w = max(1.0, v.get("SQ_WAVES", 1))
    clk = v.get("GRBM_GUI_ACTIVE", 0) / 8 or 1
    print(k)
    print("   " + "  ".join("%s=%.3g" % (c, x / w if c.startswith("SQ_INSTS") or c in ("SQ_LDS_BANK_CONFLICT",) else x)
                           for c, x in sorted(v.items())))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        print("   mfma_util=%.2f valu_busy=%.2f lds_busy=%.2f occ=%.1f" % (
            v["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / clk, v.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / clk,
            v.get("SQ_ACTIVE_INST_LDS", 0) * 4 / 1024 / clk, v.get("SQ_WAVE_CYCLES", 0) * 4 / 1024 / clk))
