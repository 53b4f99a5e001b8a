"""MFMA utilisation per kernel family of the bench forward from rocprofv3 PMC counters (GPU box).

  python tools/pmc_mfma.py --config cfgC --batch 4 --out profiles/r02

One `rocprofv3 --pmc ... --kernel-trace` pass (SQ and GRBM counters only, within the per-pass slot limits of
MI355X_MICROARCH.md) over a short bench.py run; counters that `rocprofv3 -L` does not list on this device are
dropped. Per kernel family (U-Net conv3d, front-end conv2d, prob conv + regression, warp):
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)   (issued MFMA cycles per
               SIMD-cycle of the kernels' wall time, padding rows / zero taps included)
  valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA (when both exist)
Writes <out>/pmc_mfma_<config>_b<batch>[_f32].json (bench.py reports it as "mfma_utilisation"; --dtype f32: the
fp32 parity path, whose mfma_busy counts the three split-f16 MFMAs of every product).
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
WANT = ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_BUSY_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"]
FAMILIES = (("unet_conv3d", ("conv3d", "deconv_", "conv_s2_c8", "conv_s1_c16")), ("frontend_conv2d", ("conv2d", "fpn_top")),
            ("prob_regress", ("prob_mfma", "prob_regress", "prob_conv", "regress_kernel")),
            ("warp_aggregate", ("warp_aggregate", "warp_split", "warp_pair")))


def family(name):
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return None


def available(tmp):
    r = subprocess.run(["rocprofv3", "-L"], capture_output=True, text=True, timeout=120, cwd="/tmp",
                       env=dict(os.environ, TMPDIR="/tmp"))
    text = r.stdout + r.stderr
    with open(os.path.join(tmp, "rocprofv3_L.txt"), "w") as f:
        f.write(text)
    return [c for c in WANT if c in text]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05"))
    ap.add_argument("--tmp", default=os.path.join(REPO, "gpurun_out", "pmc_mfma"))
    args = ap.parse_args()
    args.tmp, args.out = os.path.abspath(args.tmp), os.path.abspath(args.out)  # rocprofv3 runs with cwd /tmp
    os.makedirs(args.tmp, exist_ok=True)
    counters = available(args.tmp)
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in counters or "GRBM_GUI_ACTIVE" not in counters:
        raise SystemExit("required counters missing; listed: %s" % counters)
    d = os.path.join(args.tmp, "pass")
    cmd = ["rocprofv3", "--pmc"] + counters + ["--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
                                               sys.executable, os.path.join(REPO, "bench.py"), "--config", args.config,
                                               "--batch", str(args.batch), "--steps", "2", "--warmup", "1",
                                               "--dtype", args.dtype, "--no-parity-path",
                                               "--no-cpu-baseline", "--no-shard-latency"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        raise SystemExit("rocprofv3 failed:\n" + r.stderr[-3000:])
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    per_dispatch = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            fam = family(row["Kernel_Name"])
            if fam is None:
                continue
            key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), fam)
            per_dispatch[key][row["Counter_Name"]] = float(row["Counter_Value"])
            per_dispatch[key]["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    if not per_dispatch:  # say what the pass produced instead of writing an empty summary
        files = glob.glob(os.path.join(d, "**", "*"), recursive=True)
        raise SystemExit("no counter rows for any kernel family; files: %s\nstdout tail:\n%s\nstderr tail:\n%s"
                         % (files[:20], r.stdout[-1500:], r.stderr[-1500:]))
    for (_, fam), cs in per_dispatch.items():
        a = acc[fam]
        a["dispatches"] += 1
        for k, v in cs.items():
            a[k] += v
    summary = {}
    for fam, a in acc.items():
        cyc = a["GRBM_GUI_ACTIVE"] / 8.0
        e = {"dispatches": int(a["dispatches"]), "kernel_ms": round(a["_ns"] / 1e6, 3),
             "mfma_busy": round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0), 4) if cyc else None,
             "effective_clock_GHz": round(cyc / a["_ns"], 3) if a["_ns"] else None}
        if a.get("SQ_INSTS_MFMA") and a.get("SQ_INSTS_VALU"):
            e["valu_per_mfma"] = round(a["SQ_INSTS_VALU"] / a["SQ_INSTS_MFMA"], 2)
        summary[fam] = e
    res = {"config": args.config, "batch": args.batch, "dtype": args.dtype, "counters": counters, "summary": summary,
           "totals": {f: dict(a) for f, a in acc.items()},
           "formula": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); profiled pass "
                      "(3 forwards incl. warm-up and the B=1 latency block), clocks lower than unprofiled"}
    os.makedirs(args.out, exist_ok=True)
    path = os.path.join(args.out, "pmc_mfma_%s_b%d%s.json" % (args.config, args.batch, "_f32" if args.dtype == "f32" else ""))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
