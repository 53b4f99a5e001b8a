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
          ["GRBM_GUI_ACTIVE", "TA_TA_BUSY_sum", "TA_BUFFER_READ_WAVEFRONTS_sum"],
          ["TCC_HIT_sum", "TCC_MISS_sum"],
          ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"],
          ["FETCH_SIZE"],
          ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum"],
          ["WRITE_SIZE"]]
# the stage-2 warp: the channel-split kernel (default) or the one-lane-per-voxel kernel (DAMVS_WARP_SPLIT=0)
# PMC_DTYPE=f32: the fp32 parity path's stage-2 warp (warp_split_kernel<float, 16>: 4 lanes per voxel; the kernel name
# identifies stage 2 there; 4 lanes per voxel: twice the bf16 kernel's grid)
DTYPE = os.environ.get("PMC_DTYPE", "bf16")
KERNEL = os.environ.get("PMC_WARP_KERNEL", ("warp_split_kernel<float, 16" if DTYPE == "f32" else "warp_split_kernel<unsigned short, 16")
                        if os.environ.get("DAMVS_WARP_SPLIT", "1") != "0" else "warp_aggregate_kernel<unsigned short, 16")
GRID = int(os.environ.get("PMC_WARP_GRID", "7577600" if DTYPE == "f32" else "3788800" if "split" in KERNEL else "1894400"))
N_PIPE = 5


def run_pass(i, counters, out):
    d = os.path.join(out, "p%d" % i)
    cmd = ["rocprofv3", "--pmc"] + counters + ["--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
                                              sys.executable, os.path.join(REPO, "bench.py"), "--streams", "1",
                                              "--warmup", "1", "--steps", "2", "--no-cpu-baseline", "--no-parity-path",
                                              "--dtype", DTYPE]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        raise RuntimeError("pass %d failed:\n%s" % (i, r.stderr[-2000:]))
    disp = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KERNEL not in row["Kernel_Name"] or (GRID and int(row.get("Grid_Size", 0) or 0) != GRID):
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
        if "GRBM_GUI_ACTIVE" in m:  # summed over the 8 XCDs (MI355X_MICROARCH.md): cycles = GRBM / 8
            cyc = m["GRBM_GUI_ACTIVE"] / 8.0
            s["effective_clock_GHz"] = cyc / m["ns"]
            if "TA_TA_BUSY_sum" in m:  # one TA per CU: busy fraction = sum / 256 CUs / cycles
                s["TA_busy_frac"] = m["TA_TA_BUSY_sum"] / 256.0 / cyc
        if "TA_TA_BUSY_sum" in m and "TA_BUFFER_READ_WAVEFRONTS_sum" in m:
            s["TA_cycles_per_buffer_read_instr"] = m["TA_TA_BUSY_sum"] / max(1.0, m["TA_BUFFER_READ_WAVEFRONTS_sum"])
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in m and "TA_BUFFER_READ_WAVEFRONTS_sum" in m:
            s["l1_tag_lookups_per_read_instr"] = m["TCP_TOTAL_CACHE_ACCESSES_sum"] / max(1.0, m["TA_BUFFER_READ_WAVEFRONTS_sum"])
        if "TCC_HIT_sum" in m:
            s["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        for k in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VALU", "SQ_WAVES",
                  "TA_BUFFER_READ_WAVEFRONTS_sum"):
            if k in m:
                s[k] = m[k]
        if "FETCH_SIZE" in m:
            # KB units. profiles/r03/pmc_fetch_calibration.json (tools/pmc_calib): on gfx950 every L2 -> fabric read
            # request is a 128-byte line fill (TCC_EA0_RDREQ_32B / _64B ~ 0) and FETCH_SIZE counts 64 bytes per
            # request, for streaming reads AND for 16 / 32 / 64-byte record gathers in random order: x2 is the
            # calibrated byte count for the warp's gathers too
            s["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
            s["fetch_bytes_x2_gfx950"] = m["FETCH_SIZE"] * 1024 * 2
        if "TCC_EA0_RDREQ_sum" in m:
            n32, n64 = m.get("TCC_EA0_RDREQ_32B_sum", 0.0), m.get("TCC_EA0_RDREQ_64B_sum", 0.0)
            s["read_requests"] = m["TCC_EA0_RDREQ_sum"]
            s["read_bytes_by_request_size"] = 128 * (m["TCC_EA0_RDREQ_sum"] - n32 - n64) + 64 * n64 + 32 * n32
        if "WRITE_SIZE" in m:
            s["write_bytes"] = m["WRITE_SIZE"] * 1024
        summary[name] = s
    json.dump({"kernel": KERNEL, "grid": GRID, "counters": PASSES, "summary": summary},
              open(os.path.join(out, "pmc_warp_inpipe.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
