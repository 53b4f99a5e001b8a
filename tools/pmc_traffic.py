"""Per-launch HBM traffic of one hot-path kernel from rocprofv3 PMC counters (GPU box).

  python tools/pmc_traffic.py --kernel warp --stage 2 --config cfgC --out profiles/r01

Runs tools/kbench.py under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes,
kernel trace only), averages over the launches of the named kernel and applies the gfx950
correction of MI355X_MICROARCH.md (FETCH_SIZE reads 1/2 of a wide coalesced stream's bytes:
doubled; WRITE_SIZE exact for 16-B stores). Writes <out>/pmc_<name>_<config>.json.
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
KNAME = {"warp": "warp_aggregate", "unet": "conv3d", "probreg": "prob_regress"}


def run_pass(counter, args, tmp):
    d = os.path.join(tmp, counter)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(REPO, "tools", "kbench.py"), "--kernel", args.kernel, "--stage",
           str(args.stage), "--config", args.config, "--iters", "3", "--batch", str(args.batch)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                       env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        raise RuntimeError("rocprofv3 pass %s failed:\n%s" % (counter, r.stderr[-3000:]))
    vals, durs = [], []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KNAME[args.kernel] in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if not vals:
        raise RuntimeError("no %s samples for %s" % (counter, KNAME[args.kernel]))
    return sum(vals) / len(vals), sum(durs) / len(durs), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="warp", choices=sorted(KNAME))
    ap.add_argument("--stage", type=int, default=2)
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4, help="reference views per launch (bench.py's default batch)")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r01"))
    ap.add_argument("--tmp", default=os.path.join(REPO, "gpurun_out", "pmc_traffic"))
    args = ap.parse_args()
    fetch_kb, d1, n1 = run_pass("FETCH_SIZE", args, args.tmp)
    write_kb, d2, n2 = run_pass("WRITE_SIZE", args, args.tmp)
    hbm = (2.0 * fetch_kb + write_kb) * 1024.0
    res = {"kernel": KNAME[args.kernel], "stage": args.stage, "config": args.config, "batch": args.batch,
           "FETCH_SIZE_kb_raw": fetch_kb, "WRITE_SIZE_kb": write_kb, "launches": [n1, n2],
           "hbm_bytes_per_launch": hbm, "profiled_duration_ns": [d1, d2],
           "correction": "FETCH_SIZE x2 (gfx950: reads 1/2 of wide coalesced stream bytes), WRITE_SIZE as is"}
    os.makedirs(args.out, exist_ok=True)
    path = os.path.join(args.out, "pmc_%s_%s_b%d.json" % (KNAME[args.kernel], args.config, args.batch))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
