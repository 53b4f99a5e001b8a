"""How do the stage-2 warp's volumes differ when U-Net kernels run on another stream? (follow-up of
tools/diag_streams.py: the LDS camera copy is never altered, yet the outputs differ.)

Stream A repeats a U-Net layer; stream B runs the warp through the C ABI into output buffers that are first
filled with a sentinel (0xFFFF bf16 words = NaN) on stream B, so unwritten voxels show as the sentinel. For each
differing output: number of differing voxels / bf16 words, whether they hold the sentinel, the (d, y, x) box
they span, and whether they still differ after a cache scrub (a 2 GiB copy on the main stream) and when read back
by a host copy (DMA) instead of a kernel.

    DAMVS_LIB=... python tools/diag_streams2.py [layers...]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from damvsnet_amd.engine import hypotheses, proj_prepare
    from damvsnet_amd import _capi
    from damvsnet_amd._capi import check, ptr
    lib = _capi.load_library()
    H, W, N, nd, dtype, _ = bench.CONFIGS["cfgC"]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    s, C, scale, B = 1, 16, 2, 2
    h, w, D = H // scale, W // scale, nd[s]
    g = torch.Generator(device=dev).manual_seed(0)
    imgs, proj, dv, _ = bench.make_inputs(B, N, H, W, dev)
    pd = 600 + 100 * torch.rand(B, H // 4, W // 4, device=dev, generator=g)
    pv = 5 + 20 * torch.rand(B, H // 4, W // 4, device=dev, generator=g)
    hyps = hypotheses(dv, D, H, W, scale, pd, pv)
    feats = [torch.randn(B, h, w, C, generator=g, device=dev).to(dtype) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
    rt = proj_prepare(proj["stage2"])
    fptrs = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats])
    nout = 8
    outs = [torch.empty(B, D, h, w, C, device=dev, dtype=dtype) for _ in range(nout)]
    scrub_a = torch.empty(1 << 30, dtype=torch.int16, device=dev)
    scrub_b = torch.empty_like(scrub_a)

    def warp_into(o):
        o.view(torch.int16).fill_(-1)  # sentinel on the warp's stream
        check(lib.damvs_warp_aggregate(eng.handle, _capi.stream_ptr(dev), B, N, D, h, w, fptrs, _capi.DAMVS_LAYOUT_NHWC,
                                       ptr(rt), ptr(hyps), ptr(o)))

    with torch.no_grad():
        ref = torch.empty_like(outs[0])
        warp_into(ref)
        bufs = eng.unet_buffers(B, D, h, w)
        torch.cuda.synchronize()
        ref_host = ref.view(torch.int16).cpu()
        layers = sys.argv[1:] or ["0", "unet", "1", "7"]
        for which in layers:
            def other():
                if which == "unet":
                    eng.costreg_logits(ref)
                else:
                    k = int(which)
                    src = ref if k == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[k]]
                    eng.unet_layer(k, D, h, w, src, bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[k]])

            sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
            main_s = torch.cuda.current_stream()
            summary = {"layer": which, "trials": 0, "outputs": 0, "differ_kernel_compare": 0, "details": []}
            for trial in range(int(os.environ.get("DIAG_TRIALS", "4"))):
                sa.wait_stream(main_s)
                sb.wait_stream(main_s)
                with torch.cuda.stream(sa):
                    for _ in range(nout):
                        other()
                with torch.cuda.stream(sb):
                    for o in outs:
                        warp_into(o)
                torch.cuda.synchronize()
                summary["trials"] += 1
                for i, o in enumerate(outs):
                    summary["outputs"] += 1
                    if torch.equal(o, ref):
                        continue
                    summary["differ_kernel_compare"] += 1
                    if len(summary["details"]) >= 6:
                        continue
                    d = {"trial": trial, "out": i}
                    oi = o.view(torch.int16)
                    diff = (oi != ref.view(torch.int16))
                    d["words_differ"] = int(diff.sum())
                    vox = diff.any(-1)  # (B, D, h, w)
                    d["voxels_differ"] = int(vox.sum())
                    d["sentinel_words"] = int(((oi == -1) & diff).sum())
                    idx = vox.nonzero()
                    if idx.numel():
                        mn, mx = idx.min(0).values.tolist(), idx.max(0).values.tolist()
                        d["box_bdyx_min"], d["box_bdyx_max"] = mn, mx
                        f = idx[0].tolist()
                        d["first_voxel"] = f
                        d["first_got"] = o[tuple(f)].float().tolist()[:4]
                        d["first_ref"] = ref[tuple(f)].float().tolist()[:4]
                    # shape of the differing set: whole pixel columns (all D planes)? whole 64-pixel waves?
                    pix = vox.any(1)  # (B, h, w)
                    d["pixels_differ"] = int(pix.sum())
                    d["pixels_all_planes_differ"] = int(vox.all(1).sum())
                    flat = pix.reshape(B, -1)
                    waves = flat.reshape(B, -1, 64).sum(-1)  # affected pixels per 64-pixel wave (256 | h*w)
                    nz = waves[waves > 0]
                    d["waves_touched"] = int(nz.numel())
                    d["pixels_per_touched_wave"] = [int(nz.min()), float(nz.float().mean()), int(nz.max())] if nz.numel() else []
                    lanes = flat.nonzero()[:, 1] % 64  # lane of each differing pixel in its wave
                    d["lane_group_hist"] = torch.bincount(lanes // 16, minlength=4).tolist()
                    d["lane_in_group_hist"] = torch.bincount(lanes % 16, minlength=16).tolist()
                    d["wave_in_block_hist"] = torch.bincount((flat.nonzero()[:, 1] % 256) // 64, minlength=4).tolist()
                    blocks = flat.reshape(B, -1, 256).sum(-1)
                    d["blocks_touched"] = int((blocks > 0).sum())
                    # host copy (DMA engine), then again after a 2 GiB copy on the main stream
                    d["differ_host_copy"] = int((oi.cpu() != ref_host).sum())
                    scrub_b.copy_(scrub_a)
                    torch.cuda.synchronize()
                    d["differ_after_scrub_kernel"] = int((o.view(torch.int16) != ref.view(torch.int16)).sum())
                    summary["details"].append(d)
            if hasattr(lib, "damvs_diag_take_warp"):
                buf = (ctypes.c_uint * (8 + 8 * 64))()
                lib.damvs_diag_take_warp(buf, len(buf))
                summary["diag_records"] = int(buf[0])
                summary["diag_first"] = [list(buf[8 + 8 * i: 16 + 8 * i]) for i in range(min(int(buf[0]), 6))]
            print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
