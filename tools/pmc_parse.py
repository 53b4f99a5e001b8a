"""Summarise tools/pmc_run.sh output: per kernel (first dispatch of each name/grid), counters per wave."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
res = collections.OrderedDict()
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "damvs" not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        e = res.setdefault(key, {"name": r["Kernel_Name"].split("(")[0].split("::")[-1][:40] + " " + r["Grid_Size"],
                                 "vgpr": r["VGPR_Count"], "lds": r["LDS_Block_Size"]})
        e.setdefault(r["Counter_Name"], float(r["Counter_Value"]))
        e.setdefault("dur", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
seen = set()
for k, v in res.items():
    if v["name"] in seen:
        continue
    seen.add(v["name"])
    w = max(1.0, v.get("SQ_WAVES", 1))
    clk = v.get("GRBM_GUI_ACTIVE", 0) / 8
    print("%-52s dur %7.1f  vgpr %3s  VALU/w %6.0f  SALU/w %5.0f  MFMA/w %5.0f  VMEM_RD/w %5.1f  LDS/w %5.0f  occ %.1f  "
          "fetchMB %6.0f  writeMB %6.0f  TA %.2f" % (
              v["name"], v.get("dur", 0), v["vgpr"], v.get("SQ_INSTS_VALU", 0) / w, v.get("SQ_INSTS_SALU", 0) / w,
              v.get("SQ_INSTS_MFMA", 0) / w, v.get("SQ_INSTS_VMEM_RD", 0) / w, v.get("SQ_INSTS_LDS", 0) / w,
              v.get("SQ_WAVE_CYCLES", 0) * 4 / 1024 / max(1, clk), v.get("FETCH_SIZE", 0) * 2 / 1e3,
              v.get("WRITE_SIZE", 0) / 1e3, v.get("TA_BUSY_avr", 0) / max(1, clk)))
