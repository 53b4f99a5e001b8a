"""Where the stage-2 warp's volume differs when it runs beside U-Net layers on another stream.

  python tools/diag_warp_streams.py [--layout cblock|nhwc] [--layer 0]

Prints, for solo repeats and for runs beside the layer: the number of differing voxels, the batch elements, planes,
rows and lane positions (pixel index mod 64 within the warp's pixel blocks) they fall on, and the largest difference.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="cblock", choices=["cblock", "nhwc"])
    ap.add_argument("--layer", type=int, default=0)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--stage", type=int, default=1, choices=[0, 1])
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    from common import model_state
    from test_gpu_streams import _perturb
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import hypotheses, block_channels, proj_prepare
    from damvsnet_amd import _capi, synth
    DEV = "cuda"
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dt)
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    net = net.to(DEV).eval()
    B, N, H, W, s = 2, 5, 1184, 1600, a.stage
    C, D, scale = (32, 48, 4) if s == 0 else (16, 32, 2)
    h, w = H // scale, W // scale
    proj, _, dv = synth.cameras(B, N, H, W)
    P = _perturb(torch.from_numpy(proj["stage%d" % (s + 1)])).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(0)
    pd = 600 + 100 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
    pv = 5 + 20 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
    hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale, pd, pv) if s else \
        hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale)
    feats = [torch.randn(B, h, w, C, generator=g, device=DEV).to(dt) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], torch.device(DEV))

    es = feats[0].element_size()
    S = C * es // 16 if (C * es) in (32, 64, 128) else 1  # lanes per voxel of the split kernel (NHWC maps, odd N)
    ppb = 256 // S
    tc = ppb // 8  # 8-row pixel tiles (warp_pixel, DAMVS_WARP_TILE default)

    def waves(d):
        """Per wave instance (batch, tile, wave) whose voxels differ: planes hit, pixels per (wave, plane), lanes."""
        badc = (d > 0)  # [B][D][h][w][C]
        idx = badc.any(-1).nonzero()
        if not len(idx):
            return {}
        b, z, y, x = idx[:, 0], idx[:, 1], idx[:, 2], idx[:, 3]
        i = (y % 8) * tc + (x % tc)
        t = i * S
        wave = t // 64
        lane0 = t % 64
        key = ((b * 1000 + y // 8) * 1000 + x // tc) * 8 + wave
        chunks = badc[b, z, y, x].reshape(len(idx), S, -1).any(-1).sum(-1)  # bad 16-byte chunks per bad voxel
        per = {}
        for k, zz, ln in zip(key.tolist(), z.tolist(), lane0.tolist()):
            e = per.setdefault(k, {"planes": {}, "lanes": set()})
            e["planes"][zz] = e["planes"].get(zz, 0) + 1
            e["lanes"].add(ln)
        nplanes = [len(e["planes"]) for e in per.values()]
        suffix = sum(1 for e in per.values() if sorted(e["planes"]) == list(range(min(e["planes"]), D)))
        full_q = sum(1 for e in per.values() for c in e["planes"].values() if c == 16 // S)
        events = sum(len(e["planes"]) for e in per.values())
        return {"waves": len(per), "planes_per_wave_hist": torch.bincount(torch.tensor(nplanes), minlength=D + 1).tolist(),
                "suffix_shaped": suffix, "wave_plane_events": events, "events_whole_quarter": full_q,
                "min_lane": min(min(e["lanes"]) for e in per.values()),
                "bad_chunks_per_voxel_hist": torch.bincount(chunks.cpu(), minlength=S + 1).tolist()}

    lib = _capi.load_library()

    def take():
        """Diagnostic builds (-DDAMVS_DIAG): the records the warp kernels appended since the last take, by kind."""
        if not hasattr(lib, "damvs_diag_take_warp"):
            return None
        import ctypes
        buf = (ctypes.c_uint * (8 + 8 * 64))()
        lib.damvs_diag_take_warp(buf, len(buf))
        kinds = {}
        for r in range(min(buf[0], 64)):
            k = buf[8 + 8 * r]
            kinds[k] = kinds.get(k, 0) + 1
        first = [{"kind": buf[8 + 8 * r], "lane": buf[10 + 8 * r] >> 8, "view": buf[10 + 8 * r] & 255,
                  "seen": "0x%08x" % buf[11 + 8 * r], "want": "0x%08x" % buf[12 + 8 * r]} for r in range(min(buf[0], 4))]
        return {"count": int(buf[0]), "kinds_in_first_64": kinds, "first": first}

    def report(tag, outs, ref):
        rec_diag = take()
        if rec_diag is not None:
            print(json.dumps({"case": tag, "diag_records": rec_diag}), flush=True)
        for i, o in enumerate(outs):
            d = (o.float() - ref.float()).abs()
            bad = (d > 0).any(-1)  # [B][D][h][w]
            nb = int(bad.sum())
            rec = {"case": tag, "rep": i, "voxels": nb}
            if nb and S > 1 and a.layout == "nhwc":
                rec["wave_analysis"] = waves(d)
            if nb:
                idx = bad.nonzero()
                rec["batch"] = sorted(set(idx[:, 0].tolist()))
                rec["planes"] = sorted(set(idx[:, 1].tolist()))[:12]
                rec["rows"] = [int(idx[:, 2].min()), int(idx[:, 2].max())]
                rec["cols"] = [int(idx[:, 3].min()), int(idx[:, 3].max())]
                rec["col_mod_32_hist"] = torch.bincount(idx[:, 3] % 32, minlength=32).tolist()
                rec["row_mod_8_hist"] = torch.bincount(idx[:, 2] % 8, minlength=8).tolist()
                rec["maxdiff"] = float(d.max())
                rec["nan"] = int(torch.isnan(o.float()).sum())
            print(json.dumps(rec), flush=True)

    with torch.no_grad():
        rt = proj_prepare(P)
        if a.layout == "cblock":
            fb = block_channels(feats)
            warp = lambda: eng.warp_aggregate(fb, None, hyps, rt=rt, layout=_capi.DAMVS_LAYOUT_CBLOCK)
        else:
            warp = lambda: eng.warp_aggregate(feats, None, hyps, rt=rt)
        vol = warp()
        bufs = eng.unet_buffers(B, D, h, w)
        torch.cuda.synchronize()
        ref = vol.clone()
        report("solo", [warp() for _ in range(a.reps)], ref)
        torch.cuda.synchronize()
        sa, sb, main = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()
        layer = a.layer
        src = vol if layer == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[layer]]
        dst = bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[layer]]
        for it in range(2):
            sa.wait_stream(main)
            sb.wait_stream(main)
            with torch.cuda.stream(sa):
                for _ in range(a.reps):
                    eng.unet_layer(layer, D, h, w, src, dst)
            with torch.cuda.stream(sb):
                outs = [warp() for _ in range(a.reps)]
            torch.cuda.synchronize()
            report("beside layer %d (iteration %d)" % (layer, it), outs, ref)
        # same stream, interleaved (no concurrency)
        outs = []
        for _ in range(a.reps):
            eng.unet_layer(layer, D, h, w, src, dst)
            outs.append(warp())
        torch.cuda.synchronize()
        report("interleaved on one stream", outs, ref)


if __name__ == "__main__":
    main()
