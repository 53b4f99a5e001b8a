"""Scan a kernel's gfx950 assembly for LDS reads whose wait could be released by an out-of-order SMEM return.

  python tools/lgkm_hazard.py <file.s> <kernel-name-substring> [--show N]

lgkmcnt counts LDS (ds_*), scalar memory (s_load / s_buffer_load) and message operations. LDS operations return in
issue order, SMEM operations in any order (ISA: a partial lgkmcnt(N) is only meaningful for LDS when no SMEM is
outstanding). The scan walks the kernel's instructions in text order (loops and branches are read as straight-line
code, so it lists candidates, not proofs), keeps the queue of outstanding lgkm operations (kind, line, text) and at every
`s_waitcnt lgkmcnt(N)` with N > 0 reports the LDS reads that must have completed (all but the N youngest) while an
SMEM load is also outstanding: if that SMEM load returns first, the counter reaches N with the LDS read's data
still in flight, and the wave reads the destination registers early. A full wait (N = 0) clears the queue.
"""
import argparse
import re
import sys


def instructions(path, kernel):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*%s\S*:" % re.escape(kernel), l) or (kernel in l and l.rstrip().endswith(":") and
                                                               l.startswith("_Z")):
            start = i
            break
    if start is None:
        sys.exit("kernel %s not found" % kernel)
    for j in range(start + 1, len(lines)):
        l = lines[j]
        if l.startswith("\t.size") or re.match(r"^_Z\S*:", l):
            break
        t = l.split(";")[0].strip()
        if t and not t.startswith("."):
            yield j + 1, t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--show", type=int, default=20)
    a = ap.parse_args()
    queue = []  # (kind, line, text)
    hazards = []
    n_wait = n_partial = n_ds = n_smem = 0
    for ln, t in instructions(a.asm, a.kernel):
        op = t.split()[0]
        if op.startswith("ds_") and not op.startswith(("ds_write", "ds_store", "ds_swizzle", "ds_bpermute",
                                                      "ds_permute")) or op.startswith(("ds_swizzle", "ds_bpermute",
                                                                                      "ds_permute")):
            queue.append(("LDS", ln, t))
            n_ds += 1
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            queue.append(("LDSW", ln, t))
        elif op.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime")):
            queue.append(("SMEM", ln, t))
            n_smem += 1
        elif op.startswith("s_sendmsg"):
            queue.append(("MSG", ln, t))
        elif op == "s_waitcnt" or op == "s_waitcnt_lgkmcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if op == "s_waitcnt_lgkmcnt":
                m2 = re.search(r",\s*(0x[0-9a-f]+|\d+)", t)
                cnt = int(m2.group(1), 0) if m2 else None
            else:
                cnt = int(m.group(1)) if m else None
            if cnt is None:
                continue
            n_wait += 1
            if cnt == 0:
                queue = []
                continue
            n_partial += 1
            must = queue[:max(0, len(queue) - cnt)]
            smem_out = [q for q in queue if q[0] == "SMEM"]
            lds_must = [q for q in must if q[0] == "LDS"]
            if smem_out and lds_must:
                hazards.append((ln, t, lds_must, smem_out))
            queue = queue[max(0, len(queue) - cnt):]
    print("kernel %s: %d LDS reads, %d SMEM loads, %d lgkm waits (%d partial), %d partial waits with SMEM outstanding "
          "and an LDS read to complete" % (a.kernel, n_ds, n_smem, n_wait, n_partial, len(hazards)))
    for ln, t, lds, smem in hazards[:a.show]:
        print("line %d: %s" % (ln, t))
        for q in lds:
            print("    waits for  %s line %d: %s" % (q[0], q[1], q[2]))
        for q in smem:
            print("    SMEM out   line %d: %s" % (q[1], q[2]))


if __name__ == "__main__":
    main()
