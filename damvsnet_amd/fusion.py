"""Depth-map fusion on the GPU: the reference's dynamic-consistency
filter (filter/dypcd.py, `dypcd_filter` / `filter_depth`) with the per-pixel reprojection checks in
one HIP kernel per reference view (damvs_fusion_view, k_fusion.hip).

`fuse_view` is the per-view primitive (device tensors in, averaged depth / masks / world points
out); `filter_depth` mirrors filter/dypcd.py:179-326 over a scene directory written by the test
path (cams/, images/, depth_est/, confidence/ PFMs; see mvsio.save_stage_outputs) and writes the
masks and the PLY point cloud. The reference's defaults (test_uni.py:104-109): conf (0.1, 0.15, 0.9),
dist_base 1/4, rel_diff_base 1/1300.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _capi, mvsio
from ._capi import check


def fusion_cams(K_ref, E_ref, srcs):
    """Camera products as the reference forms them: float32 numpy inverses and float32 4x4 products
    (filter/dypcd.py:104-123), packed into damvs_fusion_cams."""
    c = _capi.DamvsFusionCams()
    f32 = lambda a: np.asarray(a, dtype=np.float32)
    K_ref, E_ref = f32(K_ref), f32(E_ref)
    put = lambda dst, a: ctypes.memmove(dst, np.ascontiguousarray(f32(a)).ctypes.data, f32(a).size * 4)
    put(c.kinv_ref, np.linalg.inv(K_ref))
    put(c.k_ref, K_ref)
    put(c.einv_ref, np.linalg.inv(E_ref))
    if len(srcs) > _capi.FUSION_MAX_SRC:
        raise ValueError("at most %d source views (the reference's masks run to i = 10)" % _capi.FUSION_MAX_SRC)
    for v, (K_src, E_src) in enumerate(srcs):
        K_src, E_src = f32(K_src), f32(E_src)
        put(c.t_sr[v], np.matmul(E_src, np.linalg.inv(E_ref)))
        put(c.k_src[v], K_src)
        put(c.kinv_src[v], np.linalg.inv(K_src))
        put(c.t_rs[v], np.matmul(E_ref, np.linalg.inv(E_src)))
    return c


def fuse_view(depth_ref, K_ref, E_ref, srcs, confs=None, conf_thr=(0.1, 0.15, 0.9), dist_base=0.25,
              rel_diff_base=1 / 1300, want_xyz=True):
    """One reference view. depth_ref (H, W) fp32 CUDA tensor; srcs [(depth (H, W) CUDA, K, E)];
    confs: (final, stage-2, stage-1) confidence maps at (H, W) or None.
    -> {'depth_avg', 'photo', 'geo', 'final' (bool), 'xyz' (H, W, 3) world points (0 off-mask)}."""
    for t in [depth_ref] + [s[0] for s in srcs] + list(confs or []):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.shape == depth_ref.shape):
            raise ValueError("fusion maps must be contiguous (H, W) float32 CUDA tensors of one size")
    lib = _capi.load_library()
    H, W = depth_ref.shape
    dev = depth_ref.device
    cams = fusion_cams(K_ref, E_ref, [(K, E) for _, K, E in srcs])
    n = len(srcs)
    dsrc = (ctypes.c_void_p * n)(*[s[0].data_ptr() for s in srcs])
    cptr = (ctypes.c_void_p * 3)(*[c.data_ptr() for c in confs]) if confs is not None else None
    thr = (ctypes.c_float * 3)(*conf_thr)
    depth_avg = torch.empty(H, W, device=dev, dtype=torch.float32)
    mask = torch.empty(H, W, device=dev, dtype=torch.uint8)
    xyz = torch.empty(H, W, 3, device=dev, dtype=torch.float32) if want_xyz else None
    check(lib.damvs_fusion_view(_capi.stream_ptr(dev), H, W, n, depth_ref.data_ptr(), dsrc, cptr, thr, ctypes.byref(cams),
                                dist_base, rel_diff_base, depth_avg.data_ptr(), mask.data_ptr(),
                                xyz.data_ptr() if xyz is not None else None))
    return {"depth_avg": depth_avg, "photo": (mask & 1).bool(), "geo": (mask & 2).bool(), "final": (mask & 4).bool(),
            "xyz": xyz}


def _save_mask(path, m):
    from PIL import Image
    Image.fromarray(m.astype(np.uint8) * 255).save(path)


def filter_depth(pair_folder, scan_folder, out_folder, plyfilename, conf=(0.1, 0.15, 0.9), dist_base=0.25,
                 rel_diff_base=1 / 1300, device="cuda"):
    """filter/dypcd.py:179-326 for one scene: per reference view of pair.txt, load its cams, image,
    depth and three confidences (and the sources' depths), run the fusion kernel, save the photo /
    geo / final masks, collect coloured world points; write the PLY. Returns the point count."""
    pairs = mvsio.read_pair_file(os.path.join(pair_folder, "pair.txt"))
    cam = lambda v: mvsio.read_camera_parameters(os.path.join(scan_folder, "cams", "%08d_cam.txt" % v))
    pfm = lambda kind, v, sfx="": torch.from_numpy(np.ascontiguousarray(
        mvsio.read_pfm(os.path.join(out_folder, kind, "%08d%s.pfm" % (v, sfx)))[0])).to(device)
    os.makedirs(os.path.join(out_folder, "mask"), exist_ok=True)
    verts, cols = [], []
    for ref_view, src_views in pairs:
        K_ref, E_ref = cam(ref_view)
        img = mvsio.read_img(os.path.join(scan_folder, "images", "%08d.jpg" % ref_view))
        confs = (pfm("confidence", ref_view), pfm("confidence", ref_view, "_stage2"),
                 pfm("confidence", ref_view, "_stage1"))
        srcs = [(pfm("depth_est", v),) + cam(v) for v in src_views]
        r = fuse_view(pfm("depth_est", ref_view), K_ref, E_ref, srcs, confs, conf, dist_base, rel_diff_base)
        fin = r["final"].cpu().numpy()
        for kind in ("photo", "geo", "final"):
            _save_mask(os.path.join(out_folder, "mask", "%08d_%s.png" % (ref_view, kind)), r[kind].cpu().numpy())
        verts.append(r["xyz"][r["final"]].cpu().numpy())
        cols.append((img[fin] * 255).astype(np.uint8))
    xyz = np.concatenate(verts) if verts else np.zeros((0, 3), np.float32)
    rgb = np.concatenate(cols) if cols else np.zeros((0, 3), np.uint8)
    mvsio.write_ply(plyfilename, xyz, rgb)
    return len(xyz)
