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
