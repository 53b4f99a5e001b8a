"""Scene-I/O fixtures from the reference's own parsers (build container only).

Run from the repo root:  ``PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_f3.py``  -> tests/golden/scene_io.npz

The reference modules that hold the parsers import OpenCV, plyfile and yacs at module level, none of which is installed
here; their parsers themselves are numpy / PIL only. Empty stand-ins for those three modules are put in sys.modules
before the import (as make_golden.py does for torchvision), so the reference's own functions run:
  * datasets/data_io.py:6-71      read_pfm / save_pfm
  * datasets/general_eval.py      MVSDataset.build_list (:26-52), read_cam_file (:59-79), scale_mvs_input (:89-109),
                                  __getitem__ (:111-199)
  * filter/dypcd.py:70-96         read_camera_parameters / read_pair_file
  * test_uni.py:182-199           write_cam (the module is imported with an empty argv, its parser's defaults)
The stand-in cv2.resize only accepts a call that keeps the image size (then OpenCV returns a copy); the scene of
tests/scene_fixture.py keeps every image at a multiple of 32 inside max_h x max_w, so no real resize is needed.
Resizing itself (cv2.INTER_LINEAR / INTER_NEAREST) and cv2.remap stay "parity unpinned".
The scene is written into a temporary directory from seeds by tests/scene_fixture.py; only the reference's outputs
(and the bytes its writers produce) are stored.
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import scene_fixture as SF  # noqa: E402

REF = "/root/reference"


def stub_modules():
    cv2 = types.ModuleType("cv2")

    def resize(img, size, *a, **k):
        w, h = size
        if img.shape[:2] != (h, w):
            raise RuntimeError("stub cv2.resize: only the size-preserving call is exact without OpenCV")
        return img.copy()

    cv2.resize = resize
    cv2.INTER_LINEAR, cv2.INTER_NEAREST = 1, 0
    ply = types.ModuleType("plyfile")
    ply.PlyData = type("PlyData", (), {})
    ply.PlyElement = type("PlyElement", (), {})
    yacs = types.ModuleType("yacs")
    yc = types.ModuleType("yacs.config")
    yc.CfgNode = type("CfgNode", (), {})
    yacs.config = yc
    tv = types.ModuleType("torchvision")
    tv.utils = types.ModuleType("torchvision.utils")
    for name, m in (("cv2", cv2), ("plyfile", ply), ("yacs", yacs), ("yacs.config", yc), ("torchvision", tv),
                    ("torchvision.utils", tv.utils)):
        sys.modules.setdefault(name, m)
    sys.path.insert(0, REF)


def main():
    stub_modules()
    import datasets.data_io as dio
    import datasets.general_eval as ge
    import filter.dypcd as dy
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        # PFM: the reference writer's bytes and its reader's arrays
        for name, arr in SF.pfm_arrays().items():
            p = os.path.join(tmp, name + ".pfm")
            dio.save_pfm(p, arr)
            out["pfm_%s_bytes" % name] = np.frombuffer(open(p, "rb").read(), dtype=np.uint8)
            data, scale = dio.read_pfm(p)
            out["pfm_%s_read" % name] = np.ascontiguousarray(data)
            out["pfm_%s_scale" % name] = np.float64(scale)
        p = os.path.join(tmp, "be.pfm")  # big-endian (positive scale) file, written by hand
        with open(p, "wb") as f:
            f.write(b"Pf\n3 2\n2.000000\n" + np.arange(6, dtype=">f4").tobytes())
        data, scale = dio.read_pfm(p)
        out["pfm_be_read"], out["pfm_be_scale"] = np.ascontiguousarray(data), np.float64(scale)

        SF.make_scene(tmp)
        scan = os.path.join(tmp, "scan1")
        ds = ge.MVSDataset(tmp, ["scan1"], "test", SF.NV, ndepths=192, interval_scale=1.06, max_h=1184, max_w=1600)
        metas = np.full((len(ds.metas), 1 + 8), -1, dtype=np.int64)
        for i, (_, ref, src, _) in enumerate(ds.metas):
            metas[i, 0] = ref
            metas[i, 1:1 + len(src)] = src
        out["metas"] = metas
        for v in range(SF.NV):
            cam = os.path.join(scan, "cams", "%08d_cam.txt" % v)
            K, E, dmin, dint = ds.read_cam_file(cam, interval_scale=1.06)
            out["cam_eval_%d_K" % v], out["cam_eval_%d_E" % v] = K, E
            out["cam_eval_%d_depth" % v] = np.array([dmin, dint], dtype=np.float64)
            K, E = dy.read_camera_parameters(cam)
            out["cam_fusion_%d_K" % v], out["cam_fusion_%d_E" % v] = K, E
        pairs = dy.read_pair_file(os.path.join(scan, "pair.txt"))
        enc = np.full((len(pairs), 1 + 8), -1, dtype=np.int64)
        for i, (ref, src) in enumerate(pairs):
            enc[i, 0] = ref
            enc[i, 1:1 + len(src)] = src
        out["pairs_fusion"] = enc
        for i in range(len(ds)):
            item = ds[i]
            # float32 pixels / 255 of 8-bit images: stored as the 8-bit values, checked to rebuild bit-exactly
            u8 = np.round(item["imgs"] * 255.0).astype(np.uint8)
            assert np.array_equal(u8.astype(np.float32) / np.float32(255.0), item["imgs"])
            out["item%d_imgs_u8" % i] = u8
            out["item%d_depth_values" % i] = item["depth_values"]
            for s in ("stage1", "stage2", "stage3"):
                out["item%d_proj_%s" % (i, s)] = item["proj_matrices"][s]
                out["item%d_ins_%s" % (i, s)] = item["intrinsics_matrices"][s]
            out["item%d_filename" % i] = np.array(item["filename"])

        argv = sys.argv
        sys.argv = ["test_uni.py"]
        try:
            import test_uni
        finally:
            sys.argv = argv
        cam = np.zeros((2, 4, 4), dtype=np.float32)
        cam[0] = out["cam_eval_1_E"]
        cam[1, :3, :3] = out["cam_eval_1_K"]
        cam[1, 3] = [425.0, 2.65, 192, 933.8]
        p = os.path.join(tmp, "w_cam.txt")
        test_uni.write_cam(p, cam)
        out["write_cam_in"] = cam
        out["write_cam_text"] = np.array(open(p).read())
    path = os.path.join(HERE, "scene_io.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024), len(out), "arrays")


if __name__ == "__main__":
    main()
