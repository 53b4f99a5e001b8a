"""The stage-2 warp as the pipeline runs it against the same launch in bench.py's isolated loop, from rocprofv3 PMC
counters (GPU box): per group, mean duration, effective clock (GRBM_GUI_ACTIVE / duration), TA / TD busy, L2 hit
rate, L1 -> L2 requests and fabric fetch bytes.

  python tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe

One `rocprofv3 --pmc ... --kernel-trace` pass per counter group over `bench.py --streams 1 --warmup 1 --steps 2`
(the B=4 stage-2 warp runs 1 + 2 times in the steps and 2 times in the attribution pass: 5 in-pipeline launches;
then bench.py's isolated loop re-launches it on the pipeline's features but with the stage-1-style linear hypotheses
from depth_values, the same for every pixel, so its gathers are far more coherent than the pipeline's).
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [["GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD"],
          ["TA_BUSY_avr", "TD_BUSY_avr"],
          ["TCC_HIT_sum", "TCC_MISS_sum"],
          ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"],
          ["FETCH_SIZE"],
          ["WRITE_SIZE"]]
KERNEL = os.environ.get("PMC_WARP_KERNEL", "warp_aggregate_kernel<unsigned short, 16")
N_PIPE = 5


def run_pass(i, counters, out):
    d = os.path.join(out, "p%d" % i)
    cmd = ["rocprofv3", "--pmc"] + counters + ["--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
                                              sys.executable, os.path.join(REPO, "bench.py"), "--streams", "1",
                                              "--warmup", "1", "--steps", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        raise RuntimeError("pass %d failed:\n%s" % (i, r.stderr[-2000:]))
    disp = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KERNEL not in row["Kernel_Name"] or int(row.get("Grid_Size", 0) or 0) != 1894400:
                continue
            k = int(row["Dispatch_Id"])
            e = disp.setdefault(k, {"start": int(row["Start_Timestamp"]),
                                    "ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
            e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    rows = sorted(disp.values(), key=lambda e: e["start"])
    return rows[:N_PIPE], rows[N_PIPE:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/pmc_inpipe")
    ap.add_argument("--passes", default="", help="comma-separated pass indices (default: all)")
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)
    res = {"pipeline": collections.defaultdict(list), "isolated": collections.defaultdict(list)}
    sel = [int(x) for x in args.passes.split(",")] if args.passes else list(range(len(PASSES)))
    for i, counters in enumerate(PASSES):
        if i not in sel:
            continue
        pipe, iso = run_pass(i, counters, out)
        for name, grp in (("pipeline", pipe), ("isolated", iso)):
            for e in grp:
                for k, v in e.items():
                    if k != "start":
                        res[name][k].append(v)
        print("pass %d: %d in-pipeline, %d isolated launches" % (i, len(pipe), len(iso)), flush=True)
    summary = {}
    for name, d in res.items():
        m = {k: sum(v) / len(v) for k, v in d.items() if v}
        if "ns" not in m:
            continue
        s = {"launches_per_pass": len(d.get("ns", [])) // len(sel), "ms": m["ns"] / 1e6}
        if "GRBM_GUI_ACTIVE" in m:
            s["effective_clock_GHz"] = m["GRBM_GUI_ACTIVE"] / m["ns"]
        for k in ("TA_BUSY_avr", "TD_BUSY_avr"):
            if k in m and "GRBM_GUI_ACTIVE" in m:
                s[k.replace("_avr", "") + "_frac"] = m[k] / m["GRBM_GUI_ACTIVE"]
        if "TCC_HIT_sum" in m:
            s["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        for k in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VALU", "SQ_WAVES"):
            if k in m:
                s[k] = m[k]
        if "FETCH_SIZE" in m:  # KB units; MI355X_MICROARCH.md: x2 for 128-B requests (calibrated on streaming reads)
            s["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
            s["fetch_bytes_x2_gfx950"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            s["write_bytes"] = m["WRITE_SIZE"] * 1024
        summary[name] = s
    json.dump({"kernel": KERNEL, "grid": 1894400, "counters": PASSES, "summary": summary},
              open(os.path.join(out, "pmc_warp_inpipe.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
