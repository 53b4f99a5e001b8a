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


# ------------------------------------------------------------------------------- multi-GPU latency model
# One depth map over P GPUs (damvsnet_amd/sharded.py), predicted from measured one-GPU kernel times and the xGMI
# figures of SURVEY.md section 5 (8 fully connected MI355X, 7 links x ~153 GB/s per GPU; all-gather / all-to-all can
# use all 7 links, ~1 TB/s per GPU; ring collectives per-link bound). Nothing here is measured on several GPUs: the
# model is the prediction a SCALE record would test.
XGMI_LINK = 153e9       # B/s per link and direction
XGMI_ALL = 7 * XGMI_LINK  # B/s per GPU when every link carries traffic (all-gather / all-to-all)
P2P_LATENCY = 15e-6     # s per RCCL point-to-point group (one halo exchange of a batch half)
COLL_LATENCY = 25e-6    # s per collective (all-gather / all-to-all launch and ring start)
LAUNCH_FLOOR = 6e-6     # s: no kernel finishes faster, however small its share of the work


def slab_factor(h: int, P: int, halo: int = 8) -> float:
    """Rows a rank's U-Net layer computes (its tallest slab, multiple of 8, plus 2 x 8 halo rows) over h / P."""
    n8 = h // 8
    tallest = 8 * (n8 // P + (1 if n8 % P else 0))
    return (tallest + 2 * halo) / (h / P)


def sharded_latency(t1: dict, P: int, mode: str, stages, es: int = 2, link=XGMI_LINK, all_bw=XGMI_ALL):
    """Predicted ms per depth map (B = 1) of the cascade on P GPUs.

    t1      measured one-GPU times in ms at B = 1: t1["replicated"] (front end + hypotheses + GeoFF: every rank
            runs them whole) and per stage s t1["stages"][s] = {"warp", "unet", "regress"} (ms)
    stages  per stage (D, h, w, C) of the volume
    mode    "gather" (north_star's literal form: D-sharded warp, one all-gather of the volume, U-Net and
            regression replicated) or "depth" (D-sharded warp, all-to-all to H-slabs, U-Net on slabs with a halo
            exchange after each of its 10 layers, regression on slabs, one all-gather of the output rows)
    Returns {"total", "per_stage": [...], "comm": ms of communication on the critical path}."""
    if P == 1:
        tot = t1["replicated"] + sum(sum(st.values()) for st in t1["stages"])
        return {"total": tot, "per_stage": [sum(st.values()) for st in t1["stages"]], "comm": 0.0}
    per, comm = [], 0.0
    for (D, h, w, C), st in zip(stages, t1["stages"]):
        vol = D * h * w * C * es
        warp = max(st["warp"] / P, LAUNCH_FLOOR * 1e3)
        if mode == "gather":
            c = (COLL_LATENCY + vol * (P - 1) / P / all_bw) * 1e3
            t = warp + c + st["unet"] + st["regress"]
        elif mode == "depth":
            f = slab_factor(h, P)
            a2a = (COLL_LATENCY + vol * 1.4 * (P - 1) / P / P / all_bw) * 1e3  # x1.4: the slab's halo rows
            # 10 layers, two batch halves each: a P2P group per half and layer; the exchange of one half overlaps
            # the other half's layer, so per layer the exposed cost is one group's latency + its bytes on one link
            halo_bytes = 0.0
            for l, cl in ((0, 8), (1, 16), (1, 16), (2, 32), (2, 32), (3, 64), (3, 64), (2, 32), (1, 16), (0, 8)):
                halo_bytes += 2 * (8 >> l) * (w >> l) * (D >> l) * cl * es
            halos = (10 * P2P_LATENCY + halo_bytes / link) * 1e3
            unet = max(st["unet"] * f / P, 10 * LAUNCH_FLOOR * 1e3)
            reg = max(st["regress"] * f / P, LAUNCH_FLOOR * 1e3)
            rows = (COLL_LATENCY + 3 * h * w * 4 * (P - 1) / P / all_bw) * 1e3  # depth / conf / var rows
            c = a2a + halos + rows
            t = warp + unet + reg + c
        else:
            raise ValueError(mode)
        per.append(t)
        comm += c
    return {"total": t1["replicated"] + sum(per), "per_stage": per, "comm": comm}
