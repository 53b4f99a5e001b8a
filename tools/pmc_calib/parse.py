"""Summarise tools/pmc_calib/run.sh: per calibration kernel, mean counters per dispatch and FETCH_SIZE bytes
against the 1 GiB each dispatch must read."""
import collections
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
TABLE = 1 << 30
res = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("fetch", "rdreq", "bubble"):
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            k = (int(row["Dispatch_Id"]), row["Counter_Name"])
            per[k] += float(row["Counter_Value"])
            names[int(row["Dispatch_Id"])] = row["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        for (d, c), v in per.items():
            res[names[d]][c].append(v)
summary = {}
for kname, cs in res.items():
    s = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in s:
        s["fetch_bytes"] = s["FETCH_SIZE"] * 1024
        s["fetch_over_table"] = s["fetch_bytes"] / TABLE
    if "TCC_EA0_RDREQ_sum" in s and "TCC_EA0_RDREQ_64B_sum" in s:
        n32, n64 = s["TCC_EA0_RDREQ_32B_sum"], s["TCC_EA0_RDREQ_64B_sum"]
        n128 = s["TCC_EA0_RDREQ_sum"] - n32 - n64  # requests that are neither 32- nor 64-byte
        s["req_bytes_by_size"] = 128 * n128 + 64 * n64 + 32 * n32
        s["req_bytes_over_table"] = s["req_bytes_by_size"] / TABLE
    summary[kname] = s
timing = [json.loads(l) for l in open(os.path.join(out, "calib_timing.jsonl")) if l.strip()]
print(json.dumps({"table_bytes": TABLE, "per_kernel": summary, "timing": timing}, indent=1))
