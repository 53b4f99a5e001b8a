"""Algorithmic bytes and FLOPs of the hot path and the gfx950 peaks they are priced
against -- the roofline model bench.py reports with its measured kernel times.

Per depth map and stage (V = D*h*w voxels, e = storage bytes: 2 bf16 / 4 fp32, hypotheses and maps fp32):

* warp + aggregation (models/cas_mvsnet.py:26-87, one fused kernel): bytes = e*(N*C*h*w + C*V) + 4*V,
  FLOPs = (N-1)*V*(16*C + 2)
* CostRegNet (models/module.py:510-541): bytes = e * sum over layers of (Cin*V_in + Cout*V_out
  [+ Cout*V_out skip read]) + weights, FLOPs = sum of 2*27*Cin*Cout*V (V = V_out for Conv3d, V_in for the
  transposed convs)
* prob conv + regression (models/module.py:541, models/cas_mvsnet.py:105-124): bytes = e*base*V (U-Net output)
  + 4*V (hypotheses) + 4*V (probability volume) + 12*h*w (three maps), FLOPs = 54*base*V + 12*V
"""
from __future__ import annotations

HBM_PEAK = 8.0e12              # B/s, MI355X HBM3E (MI355X_MICROARCH.md chip table, spec)
MFMA_PEAK = {"bf16": 2.5e15,   # FLOP/s dense bf16 MFMA (spec, no sparsity)
             # the fp32 path computes every conv product as three f16 MFMAs (split operands, DESIGN.md "The fp32
             # path"): its instruction ceiling is a third of the dense f16 rate, not the exact-f32 MFMA's
             "f32": 2.5e15 / 3,
             "f32_exact": 157.3e12}  # FLOP/s exact-f32 MFMA (= the FP32 vector rate), reported beside it


def unet_layers(C: int, base: int = 8):
    """(name, cin, cout, level_in, level_out, transposed, skip) of CostRegNet (models/module.py:513-530)."""
    b = base
    return (("conv0", C, b, 0, 0, False, False), ("conv1", b, 2 * b, 0, 1, False, False),
            ("conv2", 2 * b, 2 * b, 1, 1, False, False), ("conv3", 2 * b, 4 * b, 1, 2, False, False),
            ("conv4", 4 * b, 4 * b, 2, 2, False, False), ("conv5", 4 * b, 8 * b, 2, 3, False, False),
            ("conv6", 8 * b, 8 * b, 3, 3, False, False), ("conv7", 8 * b, 4 * b, 3, 2, True, True),
            ("conv9", 4 * b, 2 * b, 2, 1, True, True), ("conv11", 2 * b, b, 1, 0, True, True))


def stage_cost(N: int, C: int, D: int, h: int, w: int, e: int, base: int = 8):
    """{"warp" | "unet" | "regress": (bytes, flops)} for ONE depth map of one stage."""
    V = D * h * w
    hw = h * w
    warp = (e * (N * C * hw + C * V) + 4 * V, (N - 1) * V * (16 * C + 2))
    ub = uf = 0
    for name, cin, cout, li, lo, tr, skip in unet_layers(C, base):
        vin, vout = V >> (3 * li), V >> (3 * lo)
        ub += e * (cin * vin + cout * vout * (2 if skip else 1) + 27 * cin * cout)
        uf += 2 * 27 * cin * cout * (vin if tr else vout)
    regress = (e * base * V + 8 * V + 12 * hw + 4 * 27 * base, 54 * base * V + 12 * V)
    return {"warp": warp, "unet": (ub, uf), "regress": regress}


def cascade_cost(H: int, W: int, N: int, ndepths, e: int, channels=(32, 16, 8)):
    """Per stage (list of stage_cost dicts) for one depth map of an H x W cascade (stages at 1/4, 1/2, 1)."""
    return [stage_cost(N, channels[s], ndepths[s], H >> (2 - s), W >> (2 - s), e) for s in range(3)]


def roofline_time(nbytes: float, flops: float, dtype: str = "bf16") -> float:
    """Seconds at the roofline: max(bytes / HBM peak, FLOPs / MFMA peak)."""
    return max(nbytes / HBM_PEAK, flops / MFMA_PEAK[dtype])
