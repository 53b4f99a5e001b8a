"""Depth fusion (filter/dypcd.py): the HIP kernel against the oracle's numpy
restatement on synthetic scenes — a tilted plane rendered into DTU-like cameras, with perturbed
patches so that every mask outcome occurs — plus CPU sanity checks of the oracle itself.

Gate (floating point): masks agree on >= 99.9 % of pixels (the remaining ones must sit within 1e-4
of a threshold: float64 matrix products are summed in a different order than numpy's BLAS), the
averaged depth within 1e-6 relative and world points within 1e-6 of the scene extent (a few float32
ulps after the float64 -> float32 cast) where both final masks agree.
"""
import numpy as np
import pytest
import torch

from oracle import fusion_oracle as FO
from damvsnet_amd import synth


def plane_scene(nviews=4, H=96, W=128, seed=0, noise=True):
    """Depth maps of the plane z - 0.2 x = 600 (ref-camera frame = world) in nviews synthetic cameras."""
    proj, _, _ = synth.cameras(1, nviews, H, W)
    E = proj["stage3"][0, :, 0].astype(np.float32)
    K = proj["stage3"][0, :, 1, :3, :3].astype(np.float32)
    n, c = np.array([-0.2, 0.0, 1.0]), 600.0
    rng = np.random.default_rng(seed)
    depths = []
    u, v = np.meshgrid(np.arange(W), np.arange(H))
    pix = np.stack([u, v, np.ones_like(u)], 0).reshape(3, -1).astype(np.float64)
    for i in range(nviews):
        R, t = E[i, :3, :3].astype(np.float64), E[i, :3, 3].astype(np.float64)
        C = -R.T @ t
        d = R.T @ np.linalg.inv(K[i].astype(np.float64)) @ pix
        depth = ((c - n @ C) / (n @ d)).reshape(H, W).astype(np.float32)
        if noise:
            for _ in range(6):  # inconsistent patches
                y0, x0 = rng.integers(0, H - 16), rng.integers(0, W - 16)
                depth[y0:y0 + 16, x0:x0 + 16] *= np.float32(1 + rng.uniform(-0.03, 0.03))
            depth *= (1 + 2e-4 * rng.standard_normal(depth.shape)).astype(np.float32)
        depths.append(depth)
    confs = [rng.random((H, W), dtype=np.float32) for _ in range(3)]
    img = rng.random((H, W, 3), dtype=np.float32)
    return depths, K, E, confs, img


def test_oracle_identical_views_are_consistent():
    depths, K, E, _, _ = plane_scene(2, noise=False)
    one = FO.fuse_view(depths[0], K[0], E[0], [(depths[0], K[0], E[0])], [np.ones_like(depths[0])] * 3, (0, 0, 0))
    assert not one["geo"].any()  # dynamic test: one source can never reach count >= dy_range = 2
    r = FO.fuse_view(depths[0], K[0], E[0], [(depths[0], K[0], E[0])] * 2, [np.ones_like(depths[0])] * 3, (0, 0, 0))
    assert r["geo"].all() and r["final"].all()  # 2 sources agreeing at i = 2
    assert np.allclose(r["depth_avg"], depths[0], rtol=1e-6)


def test_oracle_plane_consistency_and_remap():
    depths, K, E, confs, img = plane_scene(4, noise=False)
    srcs = [(depths[i], K[i], E[i]) for i in range(1, 4)]
    r = FO.fuse_view(depths[0], K[0], E[0], srcs, confs, (0.1, 0.15, 0.9), img=img)
    # a noise-free plane is consistent wherever every source view sees it
    assert r["geo"].mean() > 0.6
    assert np.allclose(r["depth_avg"][r["geo"]], depths[0][r["geo"]], rtol=1e-4)
    # remap restatement: integer coordinates return the pixel, out-of-range ones zero
    s = np.arange(12, dtype=np.float32).reshape(3, 4)
    out = FO.remap_linear(s, np.array([[1.0, 3.0, -1.5, 1.5]], np.float32), np.array([[2.0, 0.0, 0.0, 0.5]], np.float32))
    assert out[0, 0] == 9 and out[0, 1] == 3 and out[0, 2] == 0
    assert out[0, 3] == np.float32(((1 * 0.25 + 2 * 0.25) + 5 * 0.25) + 6 * 0.25)


@pytest.mark.gpu
@pytest.mark.parametrize("nviews,seed", [(4, 0), (6, 1), (11, 2)])
def test_fusion_kernel_vs_oracle(nviews, seed):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import build, _capi
    from damvsnet_amd.fusion import fuse_view
    build.build()
    _capi.load_library()
    depths, K, E, confs, img = plane_scene(nviews, seed=seed)
    srcs = [(depths[i], K[i], E[i]) for i in range(1, nviews)]
    thr = (0.1, 0.15, 0.9)
    ref = FO.fuse_view(depths[0], K[0], E[0], srcs, confs, thr, img=img)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    got = fuse_view(cu(depths[0]), K[0], E[0], [(cu(d), k, e) for d, k, e in srcs], [cu(c) for c in confs], thr)
    for k in ("photo", "geo", "final"):
        g = got[k].cpu().numpy()
        agree = (g == ref[k]).mean()
        assert agree >= 0.999, (k, agree)
    assert ref["geo"].mean() > 0.3 and (~ref["geo"]).mean() > 0.01  # both outcomes exercised
    both = got["final"].cpu().numpy() & ref["final"]
    davg = got["depth_avg"].cpu().numpy()
    assert np.allclose(davg[both], ref["depth_avg"][both], rtol=1e-6)
    xyz = got["xyz"].cpu().numpy()
    ref_xyz = np.zeros_like(xyz)
    ref_xyz[ref["final"]] = ref["xyz"]
    assert np.abs(xyz[both] - ref_xyz[both]).max() <= 1e-6 * np.abs(ref_xyz).max()  # a few float32 ulps
    assert not xyz[~got["final"].cpu().numpy()].any()


@pytest.mark.gpu
def test_fusion_errors():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    from damvsnet_amd.fusion import fuse_view
    _capi.load_library()
    depths, K, E, confs, _ = plane_scene(12)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    with pytest.raises(ValueError):  # 11 source views: beyond the reference's i <= 10 masks
        fuse_view(cu(depths[0]), K[0], E[0], [(cu(depths[i]), K[i], E[i]) for i in range(1, 12)])
    with pytest.raises(ValueError):  # size mismatch
        fuse_view(cu(depths[0]), K[0], E[0], [(cu(depths[1][:-1]), K[1], E[1])])


@pytest.mark.gpu
def test_filter_depth_scene(tmp_path):
    """filter_depth over a scene directory (cams/, images/, depth_est/, confidence/ as test_uni.py
    writes them): masks written, PLY point count = the oracle's final-mask total over all views."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from PIL import Image
    from damvsnet_amd import _capi, mvsio
    from damvsnet_amd.fusion import filter_depth
    _capi.load_library()
    N = 4
    depths, K, E, _, _ = plane_scene(N, seed=5)
    rng = np.random.default_rng(7)
    for d in ("cams", "images", "depth_est", "confidence"):
        (tmp_path / d).mkdir()
    confs, imgs = [], []
    for v in range(N):
        cam = np.zeros((2, 4, 4), np.float32)
        cam[0], cam[1, :3, :3] = E[v], K[v]
        mvsio.write_cam(str(tmp_path / "cams" / ("%08d_cam.txt" % v)), cam)
        im = rng.integers(0, 256, depths[v].shape + (3,)).astype(np.uint8)
        Image.fromarray(im).save(str(tmp_path / "images" / ("%08d.jpg" % v)), quality=100)
        imgs.append(mvsio.read_img(str(tmp_path / "images" / ("%08d.jpg" % v))))
        mvsio.save_pfm(str(tmp_path / "depth_est" / ("%08d.pfm" % v)), depths[v])
        c = [rng.random(depths[v].shape, dtype=np.float32) * 0.3 + 0.7 for _ in range(3)]
        confs.append(c)
        for cc, sfx in zip(c, ("", "_stage2", "_stage1")):
            mvsio.save_pfm(str(tmp_path / "confidence" / ("%08d%s.pfm" % (v, sfx))), cc)
    pairs = [(v, [u for u in range(N) if u != v]) for v in range(N)]
    open(tmp_path / "pair.txt", "w").write("%d\n" % N + "".join(
        "%d\n%d %s\n" % (r, len(s), " ".join("%d 1.0" % u for u in s)) for r, s in pairs))
    ply = str(tmp_path / "scene.ply")
    n = filter_depth(str(tmp_path), str(tmp_path), str(tmp_path), ply)
    expect = 0
    for r, s in pairs:
        o = FO.fuse_view(depths[r], K[r], E[r], [(depths[u], K[u], E[u]) for u in s], confs[r], (0.1, 0.15, 0.9))
        expect += int(o["final"].sum())
    assert expect > 0 and abs(n - expect) <= max(2, expect // 1000)
    xyz, rgb = mvsio.read_ply(ply)
    assert len(xyz) == n and rgb.dtype == np.uint8
    assert (tmp_path / "mask" / "00000000_final.png").exists()
