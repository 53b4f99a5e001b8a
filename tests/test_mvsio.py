"""CPU: scene I/O — PFM, cam.txt, pair.txt, input scaling, eval samples, PLY.

The first tests check hand-derived values written out from the reference's definitions (datasets/data_io.py:6-71,
datasets/general_eval.py:35-193, filter/dypcd.py:70-95, test_uni.py:182-199). The tests at the end pin the PFM,
cam.txt, pair.txt, eval-sample and write_cam paths bit-exactly to the reference's own functions, run on a seeded
scene with stand-ins for its absent cv2 / plyfile / yacs imports (tests/golden/make_f3.py). Image resizing (cv2) and
the PLY writer stay parity unpinned.
"""
import os

import numpy as np
import pytest

from damvsnet_amd import mvsio

CAM_TXT = """extrinsic
0.970263 0.00747983 0.241939 -191.02
-0.0147429 0.999493 0.0282234 3.28832
-0.241605 -0.030951 0.969881 22.5401
0.0 0.0 0.0 1.0

intrinsic
2892.33 0 823.205
0 2883.18 619.071
0 0 1

425.0 2.5
"""


def test_pfm_roundtrip_and_bytes(tmp_path):
    img = np.arange(15, dtype=np.float32).reshape(3, 5) * 0.5 + 0.25
    p = str(tmp_path / "d.pfm")
    mvsio.save_pfm(p, img)
    raw = open(p, "rb").read()
    hdr = b"Pf\n5 3\n-1.000000\n"
    assert raw[:len(hdr)] == hdr
    assert raw[len(hdr):] == np.flipud(img).astype("<f4").tobytes()  # rows stored bottom-up
    back, scale = mvsio.read_pfm(p)
    assert scale == 1.0 and back.dtype == np.float32 and np.array_equal(back, img)
    col = np.random.default_rng(0).random((4, 6, 3), dtype=np.float32)
    mvsio.save_pfm(p, col)
    assert open(p, "rb").read(3) == b"PF\n"
    assert np.array_equal(mvsio.read_pfm(p)[0], col)
    # big-endian file (positive scale)
    with open(p, "wb") as f:
        f.write(b"Pf\n2 2\n2.000000\n")
        f.write(np.array([[1, 2], [3, 4]], dtype=">f4").tobytes())
    d, s = mvsio.read_pfm(p)
    assert s == 2.0 and np.array_equal(d, np.array([[3, 4], [1, 2]], np.float32))
    with pytest.raises(ValueError):
        mvsio.save_pfm(p, img.astype(np.float64))


def test_cam_file_eval_and_fusion_readers(tmp_path):
    p = str(tmp_path / "00000000_cam.txt")
    open(p, "w").write(CAM_TXT)
    K, E = mvsio.read_camera_parameters(p)
    assert K.dtype == np.float32 and E.shape == (4, 4)
    assert K[0, 0] == np.float32(2892.33) and E[0, 3] == np.float32(-191.02)
    K4, E4, dmin, dint = mvsio.read_cam_file(p, ndepths=192, interval_scale=1.06)
    assert np.array_equal(K4[:2], K[:2] / np.float32(4.0)) and np.array_equal(K4[2], K[2])
    assert dmin == 425.0 and dint == pytest.approx(2.5 * 1.06)
    # a third field redefines the interval: (depth_max - depth_min) / ndepths, depth_max = min + int(n) * interval
    open(p, "w").write(CAM_TXT.replace("425.0 2.5", "425.0 2.5 192 935.0"))
    _, _, dmin, dint = mvsio.read_cam_file(p, ndepths=48, interval_scale=1.0)
    assert dint == pytest.approx(192 * 2.5 / 48)
    # writer (test_uni.py:182-199) -> reader
    cam = np.zeros((2, 4, 4), np.float32)
    cam[0], cam[1, :3, :3] = E, K
    cam[1, 3, :2] = 425.0, 2.5
    q = str(tmp_path / "w_cam.txt")
    mvsio.write_cam(q, cam)
    K2, E2 = mvsio.read_camera_parameters(q)
    assert np.array_equal(K2, K) and np.array_equal(E2, E)
    assert open(q).read().rstrip().split("\n")[-1] == "425.0 2.5 0.0 0.0"
    # the written depth line has 4 fields, so the eval reader takes num_depth = 0 (interval 0), as
    # the reference's would: written cams are for the fusion reader (filter/dypcd.py:70-80) only
    assert mvsio.read_cam_file(q, 192, 1.0)[2:] == (425.0, 0.0)


def test_pair_file(tmp_path):
    p = str(tmp_path / "pair.txt")
    open(p, "w").write("3\n0\n3 10 2.5 5 1.0 7 0.3\n1\n0\n2\n1 4 9.0\n")
    assert mvsio.read_pair_file(p) == [(0, [10, 5, 7]), (2, [4])]  # view 1 has no source: dropped
    assert mvsio.read_pair_file(p, nviews=4) == [(0, [10, 5, 7, 10]), (2, [4, 4, 4, 4])]


def test_scale_mvs_input_rules():
    K = np.array([[2892.33, 0, 823.2], [0, 2883.18, 619.07], [0, 0, 1]], np.float32)
    img = np.random.default_rng(1).random((1200, 1600, 3), dtype=np.float32)
    out, K2 = mvsio.scale_mvs_input(img, K, max_w=1600, max_h=1184)
    assert out.shape == (1184, 1568, 3)  # 1200 -> 1184 (x 0.98667), 1578.7 -> 1568 (multiple of 32)
    assert np.allclose(K2[0], K[0] * 1568 / 1600) and np.allclose(K2[1], K[1] * 1184 / 1200)
    small = img[:100, :130]
    out, K3 = mvsio.scale_mvs_input(small, K, max_w=1600, max_h=1184)
    assert out.shape == (96, 128, 3)  # no upscaling: round down to multiples of 32
    # bilinear, half-pixel centres: a linear ramp stays linear away from the clamped border
    ramp = np.tile(np.arange(64, dtype=np.float32), (4, 1))
    r = mvsio.resize_bilinear(ramp, 32, 4)
    assert np.allclose(r[0, 1:-1], np.arange(1, 31) * 2 + 0.5)


def test_resize_nearest_matches_inter_nearest_rule():
    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    r = mvsio.resize_nearest(a, 8, 6)
    assert np.array_equal(r, a[np.arange(6) // 2][:, np.arange(8) // 2])


def test_eval_scenes_sample(tmp_path):
    from PIL import Image
    from damvsnet_amd import synth
    scan = tmp_path / "scan1"
    (scan / "cams").mkdir(parents=True)
    (scan / "images").mkdir()
    N, H, W = 3, 128, 160
    proj, _, _ = synth.cameras(1, N, H, W)
    E, K = proj["stage1"][0, :, 0], proj["stage1"][0, :, 1, :3, :3]
    for v in range(N):
        cam = np.zeros((2, 4, 4), np.float32)
        cam[0] = E[v]
        cam[1, :3, :3] = K[v] * np.array([[4], [4], [1]], np.float32)  # files hold full-resolution K
        cam[1, 3, :2] = 425.0, 2.65
        cp = str(scan / "cams" / ("%08d_cam.txt" % v))
        mvsio.write_cam(cp, cam)
        lines = open(cp).read().rstrip().split("\n")
        open(cp, "w").write("\n".join(lines[:-1] + ["425.0 2.65"]) + "\n")  # DTU cams: min, interval
        Image.fromarray(np.full((H, W, 3), 40 * v, np.uint8)).save(str(scan / "images" / ("%08d.jpg" % v)))
    open(scan / "pair.txt", "w").write("3\n0\n2 1 9.0 2 8.0\n1\n2 0 9.0 2 8.0\n2\n1 0 9.0\n")
    ds = mvsio.EvalScenes(str(tmp_path), ["scan1"], nviews=3, ndepths=48, interval_scale=1.0, max_h=H, max_w=W)
    assert len(ds) == 3 and ds.metas[2] == ("scan1", 2, [0, 0, 0])  # filled to nviews entries
    s = ds[0]
    assert s["imgs"].shape == (3, 3, H, W) and s["imgs"].dtype == np.float32
    p = s["proj_matrices"]
    assert p["stage1"].shape == (3, 2, 4, 4)
    assert np.allclose(p["stage2"][:, 1, :2], p["stage1"][:, 1, :2] * 2)
    assert np.allclose(p["stage3"][:, 1, :2], p["stage1"][:, 1, :2] * 4)
    assert np.allclose(p["stage1"][:, 1, :3, :3], K, rtol=1e-6)  # K/4 of the full-resolution K
    dv = s["depth_values"]
    assert dv.shape == (48,) and dv[0] == 425.0 and np.isclose(dv[1] - dv[0], 2.65)
    assert s["filename"].format("depth_est", ".pfm") == "scan1/depth_est/00000000.pfm"


def test_ply_roundtrip(tmp_path):
    rng = np.random.default_rng(2)
    xyz = rng.random((100, 3), dtype=np.float32) * 100
    rgb = rng.integers(0, 256, (100, 3)).astype(np.uint8)
    p = str(tmp_path / "p.ply")
    mvsio.write_ply(p, xyz, rgb)
    head = open(p, "rb").read(200)
    assert head.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 100\n")
    x2, c2 = mvsio.read_ply(p)
    assert np.array_equal(x2, xyz) and np.array_equal(c2, rgb)
    assert os.path.getsize(p) == len(head[:head.index(b"end_header\n") + 11]) + 100 * 15


# ------------------------------------------------------------------- pinned to the reference's own parsers
# tests/golden/scene_io.npz holds what the reference's readers / writers return on the seeded scene of
# tests/scene_fixture.py (tests/golden/make_f3.py, build container: datasets/data_io.py:6-71,
# datasets/general_eval.py:26-199, filter/dypcd.py:70-96, test_uni.py:182-199). Bit-exact comparisons.
def _f3():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import scene_fixture
    return scene_fixture, np.load(os.path.join(here, "golden", "scene_io.npz"))


def test_pfm_matches_reference_writer_and_reader(tmp_path):
    SF, g = _f3()
    for name, arr in SF.pfm_arrays().items():
        p = str(tmp_path / (name + ".pfm"))
        mvsio.save_pfm(p, arr)
        assert open(p, "rb").read() == g["pfm_%s_bytes" % name].tobytes(), name
        data, scale = mvsio.read_pfm(p)
        assert np.array_equal(data, g["pfm_%s_read" % name]) and data.shape == g["pfm_%s_read" % name].shape, name
        assert scale == float(g["pfm_%s_scale" % name])
    p = str(tmp_path / "be.pfm")
    with open(p, "wb") as f:
        f.write(b"Pf\n3 2\n2.000000\n" + np.arange(6, dtype=">f4").tobytes())
    data, scale = mvsio.read_pfm(p)
    assert np.array_equal(data, g["pfm_be_read"]) and scale == float(g["pfm_be_scale"])


def test_cam_and_pair_readers_match_reference(tmp_path):
    SF, g = _f3()
    SF.make_scene(str(tmp_path))
    scan = tmp_path / "scan1"
    for v in range(SF.NV):
        cam = str(scan / "cams" / ("%08d_cam.txt" % v))
        K, E, dmin, dint = mvsio.read_cam_file(cam, ndepths=192, interval_scale=1.06)
        assert np.array_equal(K, g["cam_eval_%d_K" % v]) and np.array_equal(E, g["cam_eval_%d_E" % v])
        assert (dmin, dint) == tuple(g["cam_eval_%d_depth" % v]), v
        K, E = mvsio.read_camera_parameters(cam)
        assert np.array_equal(K, g["cam_fusion_%d_K" % v]) and np.array_equal(E, g["cam_fusion_%d_E" % v])

    def enc(pairs):
        out = np.full((len(pairs), 9), -1, dtype=np.int64)
        for i, (ref, src) in enumerate(pairs):
            out[i, 0] = ref
            out[i, 1:1 + len(src)] = src
        return out
    assert np.array_equal(enc(mvsio.read_pair_file(str(scan / "pair.txt"))), g["pairs_fusion"])
    assert np.array_equal(enc(mvsio.read_pair_file(str(scan / "pair.txt"), SF.NV)), g["metas"])


def test_eval_samples_match_reference_dataset(tmp_path):
    SF, g = _f3()
    SF.make_scene(str(tmp_path))
    ds = mvsio.EvalScenes(str(tmp_path), ["scan1"], SF.NV, ndepths=192, interval_scale=1.06, max_h=1184, max_w=1600)
    assert len(ds) == g["metas"].shape[0]
    for i in range(len(ds)):
        item = ds[i]
        want = g["item%d_imgs_u8" % i].astype(np.float32) / np.float32(255.0)
        assert item["imgs"].dtype == np.float32 and np.array_equal(item["imgs"], want), i
        assert np.array_equal(item["depth_values"], g["item%d_depth_values" % i]), i
        for s in ("stage1", "stage2", "stage3"):
            assert np.array_equal(item["proj_matrices"][s], g["item%d_proj_%s" % (i, s)]), (i, s)
            assert np.array_equal(item["intrinsics_matrices"][s], g["item%d_ins_%s" % (i, s)]), (i, s)
        assert item["filename"] == str(g["item%d_filename" % i])


def test_write_cam_matches_reference(tmp_path):
    _, g = _f3()
    p = str(tmp_path / "cam.txt")
    mvsio.write_cam(p, g["write_cam_in"])
    assert open(p).read() == str(g["write_cam_text"])
