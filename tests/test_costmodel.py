"""CPU: the roofline cost model (damvsnet_amd/costmodel.py) reproduces SURVEY.md section 8(d)'s numbers."""
import pytest

from damvsnet_amd import costmodel as CM


def test_cfgC_totals_match_survey():
    """cfgC (1600x1184, 5 views, 48/32/8, bf16): 7.09 GB, 504.6 GFLOP, 0.89 ms per map at the roofline;
    stage-1 conv0 78.6 GFLOP."""
    c = CM.cascade_cost(1184, 1600, 5, (48, 32, 8), 2)
    nbytes = sum(v[0] for st in c for v in st.values())
    flops = sum(v[1] for st in c for v in st.values())
    assert nbytes / 1e9 == pytest.approx(7.09, abs=0.01)
    assert flops / 1e9 == pytest.approx(504.6, abs=0.1)
    t = sum(CM.roofline_time(*v) for st in c for v in st.values())
    assert t * 1e3 == pytest.approx(0.886, abs=0.002)
    V = 48 * 296 * 400
    assert 54 * 32 * 8 * V / 1e9 == pytest.approx(78.6, abs=0.05)
    assert c[0]["warp"][0] / 1e6 == pytest.approx(424.3, abs=0.1)  # 413 MB with bf16 hypotheses + fp32 ones


def test_unet_flops_per_stage():
    """U-Net + prob conv GFLOP per stage at cfgC: 115.4 / 203.0 / 150.6."""
    c = CM.cascade_cost(1184, 1600, 5, (48, 32, 8), 2)
    for s, ref in enumerate((115.4, 203.0, 150.6)):
        D, h, w = (48, 32, 8)[s], 1184 >> (2 - s), 1600 >> (2 - s)
        prob = 54 * 8 * D * h * w
        assert (c[s]["unet"][1] + prob) / 1e9 == pytest.approx(ref, abs=0.1)


def test_roofline_time_bound():
    assert CM.roofline_time(8e12, 1.0) == pytest.approx(1.0)
    assert CM.roofline_time(1.0, 2.5e15) == pytest.approx(1.0)
    assert CM.roofline_time(1.0, 2.5e15 / 3, "f32") == pytest.approx(1.0)
    assert CM.roofline_time(1.0, 157.3e12, "f32_exact") == pytest.approx(1.0)


def _cfgD_b1_times():
    """One-GPU cfgD (1600x1184, 7 views, 64/32/8, bf16) times at B = 1 from the committed bench record: the B = 1
    latency pass's phases, each stage's DepthNet split into warp / U-Net / regression by the B = 4 in-pipeline
    probes of the same record."""
    import json
    import os
    rec = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r05",
                       "bench_cfgD_r05O.json")
    d = json.loads(open(rec).read().strip().splitlines()[-1])
    ph = d["latency_b1"]["ms_per_stage"]
    hp = d["hot_path_roofline"]["per_stage"]
    stages = []
    for s in (1, 2, 3):
        k = hp["stage%d" % s]["kernels"]
        tot = sum(k[g]["ms"] for g in ("warp", "unet", "regress"))
        dn = ph["stage%d.depthnet" % s]
        stages.append({g: dn * k[g]["ms"] / tot for g in ("warp", "unet", "regress")})
    replicated = sum(v for n, v in ph.items() if not n.endswith(".depthnet"))
    return {"replicated": replicated, "stages": stages}, d["latency_b1"]["ms_per_map"]


CFGD_STAGES = [(64, 296, 400, 32), (32, 592, 800, 16), (8, 1184, 1600, 8)]


def test_sharded_latency_model_cfgD():
    """DESIGN.md section 7's prediction for one cfgD depth map over P = 2 / 4 / 8 GPUs (unmeasured on hardware):
    P = 1 reproduces the one-GPU time; more GPUs never cost more warp time; the replicated front end (3.7 of the
    7.4 ms) bounds both modes, so neither reaches 2x at P = 8; the H-slab mode ("depth") divides the U-Net too and
    beats the volume all-gather ("gather") from P = 4 on."""
    t1, b1 = _cfgD_b1_times()
    one = CM.sharded_latency(t1, 1, "gather", CFGD_STAGES)["total"]
    assert one == pytest.approx(b1, rel=0.01)
    res = {}
    for mode in ("gather", "depth"):
        for P in (2, 4, 8):
            r = CM.sharded_latency(t1, P, mode, CFGD_STAGES)
            res[mode, P] = r["total"]
            print("cfgD B=1 %-6s P=%d: %.2f ms per map (comm %.2f ms)" % (mode, P, r["total"], r["comm"]))
    for mode in ("gather", "depth"):
        assert res[mode, 2] < one and res[mode, 8] > t1["replicated"]
        assert res[mode, 8] > one / 2  # the replicated front end caps the speed-up below 2x
    assert res["depth", 4] < res["gather", 4] and res["depth", 8] < res["gather", 8]
    # xGMI at a third of SURVEY's all-gather figure: the gather mode's volume transfer dominates its stage time
    slow = CM.sharded_latency(t1, 8, "gather", CFGD_STAGES, all_bw=CM.XGMI_ALL / 3)
    assert slow["comm"] > CM.sharded_latency(t1, 8, "gather", CFGD_STAGES)["comm"] * 2
