"""CPU: the instruction stream of every kernel in the built library equals the one the GPU stream tests last
validated (tests/isa_pins.json).

Round 4 found that a warp kernel's lanes 48-63 computed wrong voxels while MFMA / LDS-heavy U-Net kernels of another
stream shared its CU, depending only on the warp's instruction selection (a source change that respelled multiply-adds
as fmaf; DESIGN.md section 4 "Concurrent streams"). The trigger is not isolated, so any change of any kernel's
instructions must go through the GPU stream tests (tests/test_gpu_streams.py: every product warp kernel beside U-Net
layers, the whole forward on 2 and 4 streams, both dtypes) before the two-stream bench numbers are trusted. This test
makes such a change fail on the CPU until that has happened:
  1. run the GPU suite (tests/test_gpu_streams.py at least) on the new build and commit its log under profiles/;
  2. python tools/isa.py --update-pins --validated-by <that log>.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def _llvm_ok():
    return os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")


@pytest.mark.skipif(not _llvm_ok(), reason="no llvm-objdump")
def test_kernel_instruction_streams_are_the_validated_ones():
    import isa
    from damvsnet_amd import build
    build.build()
    with open(isa.PINS) as f:
        pins = json.load(f)
    assert os.path.exists(os.path.join(REPO, pins["validated_by"])), pins["validated_by"]
    if pins["compiler"] != isa.compiler():
        pytest.skip("different compiler (%s): instruction streams are not comparable" % isa.compiler())
    got = isa.hashes()
    changed = sorted(k for k in got if pins["kernels"].get(k) != got[k])
    gone = sorted(k for k in pins["kernels"] if k not in got)
    assert not changed and not gone, (
        "instruction streams differ from the stream-test-validated build (%d changed, %d removed): run "
        "tests/test_gpu_streams.py on the GPU, commit the log, then tools/isa.py --update-pins --validated-by <log>.\n"
        "changed: %s\nremoved: %s" % (len(changed), len(gone), changed[:20], gone[:20]))


@pytest.mark.skipif(not _llvm_ok(), reason="no llvm-objdump")
def test_warp_kernels_carry_no_packed_fp32_ops():
    """Round 5 located the concurrent-stream fault in the warp's packed-FP32 VALU ops: a warp build whose sampling
    path used v_pk_fma_f32 / v_pk_mul_f32 computed wrong sample coordinates in lanes 48-63 beside MFMA kernels of
    another stream, and the same source built without them (-fno-slp-vectorize) passed every stream case
    (profiles/r05/diag_streams/r05w). build.py compiles k_warp.hip that way (FILE_FLAGS); this keeps it so."""
    import re
    import isa
    from damvsnet_amd import build
    assert "-fno-slp-vectorize" in build.FILE_FLAGS.get("k_warp.hip", [])
    build.build()
    ks = isa.disassemble()
    warp = {k: b for k, b in ks.items() if "warp_split_kernel" in k or "warp_aggregate_kernel" in k}
    assert len(warp) >= 40, sorted(ks)[:10]
    pk = re.compile(r"v_pk_(fma|mul|add|mov)_f32\b")
    bad = sorted(k for k, b in warp.items() if any(pk.match(t) for t in b))
    assert not bad, "warp kernels with packed-FP32 VALU ops: %s" % bad[:10]


@pytest.mark.skipif(not _llvm_ok(), reason="no llvm-objdump")
def test_valu_kernels_carry_no_packed_fp32_ops():
    """Round 6 extends the warp's rule to every kernel without MFMA instructions: in the two-stream forward any of them
    can share a CU with the other sub-batch's MFMA kernels, the condition under which the warp's packed-FP32 results
    came back wrong in lanes 48-63 ("Concurrent streams"). The VALU-only units are built without
    the SLP and loop vectorizers (build.py FILE_FLAGS) and write no explicit float2 arithmetic; kernels with MFMA
    instructions (the co-runners in every measured case, never the victims) keep theirs."""
    import re
    import isa
    from damvsnet_amd import build
    for f in ("k_warp.hip", "k_planes.hip", "k_geometry.hip", "k_regress.hip", "k_fusion.hip"):
        assert "-fno-slp-vectorize" in build.FILE_FLAGS.get(f, []), f
    build.build()
    ks = isa.disassemble()
    pk = re.compile(r"v_pk_(fma|mul|add|mov)_f32\b")
    valu = {k: b for k, b in ks.items() if not any(t.startswith("v_mfma") for t in b)}
    assert len(valu) >= 100, len(valu)
    bad = sorted(k for k, b in valu.items() if any(pk.match(t) for t in b))
    assert not bad, "kernels without MFMA carrying packed-FP32 VALU ops: %s" % bad[:10]
