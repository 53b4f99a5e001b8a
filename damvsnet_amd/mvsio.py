"""MVS scene I/O around the engine: the file formats the reference's
test path reads and writes, so DTU / Tanks&Temples scenes run through `CascadeMVSNet` and the depth
maps reach fusion (`damvsnet_amd.fusion`).

Mirrors (reference paths relative to the reference repo):
  * PFM read / write ............ datasets/data_io.py:6-71 (flipped rows, negative scale = little endian)
  * cam.txt ..................... datasets/general_eval.py:62-81 (eval: K rows 0-1 / 4, depth range
                                  and interval rules) and filter/dypcd.py:70-80 (fusion: K as is);
                                  writer test_uni.py:182-199
  * pair.txt .................... datasets/general_eval.py:35-50 (fill to nviews with the first source)
                                  and filter/dypcd.py:84-95 (fusion: as listed)
  * input scaling ............... datasets/general_eval.py:89-108 (multiple-of-32 resize, K scaled)
  * per-stage projections ....... datasets/general_eval.py:158-193 (stage2 = K x2, stage3 = K x4)
  * confidence upsampling ....... test_uni.py:257-259 (cv2.INTER_NEAREST)
  * PLY point cloud ............. filter/dypcd.py:306-326 (vertex x,y,z f4 + red,green,blue u1)

The reference resizes with OpenCV (absent here): `resize_bilinear` is the half-pixel-centre
bilinear map cv2.INTER_LINEAR defines for float images (torch's align_corners=False form, borders
clamped) and `resize_nearest` cv2.INTER_NEAREST's floor(dst * src / dst) source index — restated, not
checked against cv2 itself.
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------------------- PFM
def read_pfm(filename):
    """-> (data float32 (H, W) or (H, W, 3), scale). datasets/data_io.py:6-41."""
    with open(filename, "rb") as f:
        header = f.readline().decode("utf-8").rstrip()
        if header == "PF":
            color = True
        elif header == "Pf":
            color = False
        else:
            raise ValueError("Not a PFM file: %r" % filename)
        m = re.match(r"^(\d+)\s(\d+)\s$", f.readline().decode("utf-8"))
        if not m:
            raise ValueError("Malformed PFM header: %r" % filename)
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        scale = abs(scale)
        data = np.fromfile(f, endian + "f")
    shape = (height, width, 3) if color else (height, width)
    return np.flipud(np.reshape(data, shape)), scale


def save_pfm(filename, image, scale=1):
    """datasets/data_io.py:44-71: rows bottom-up, '%f' scale, negative for little-endian data."""
    image = np.asarray(image)
    if image.dtype != np.float32:
        raise ValueError("Image dtype must be float32.")
    if image.ndim == 3 and image.shape[2] == 3:
        color = True
    elif image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1):
        color = False
    else:
        raise ValueError("Image must have H x W x 3, H x W x 1 or H x W dimensions.")
    image = np.flipud(image)
    endian = image.dtype.byteorder
    if endian == "<" or (endian == "=" and sys.byteorder == "little"):
        scale = -scale
    with open(filename, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(("%d %d\n" % (image.shape[1], image.shape[0])).encode("utf-8"))
        f.write(("%f\n" % scale).encode("utf-8"))
        image.tofile(f)


# ------------------------------------------------------------------------------------- cameras
def _cam_lines(filename):
    with open(filename) as f:
        return [line.rstrip() for line in f.readlines()]


def read_camera_parameters(filename):
    """-> (intrinsics (3,3), extrinsics (4,4)) float32, K unscaled (filter/dypcd.py:70-80)."""
    lines = _cam_lines(filename)
    extrinsics = np.array(" ".join(lines[1:5]).split(), dtype=np.float32).reshape(4, 4)
    intrinsics = np.array(" ".join(lines[7:10]).split(), dtype=np.float32).reshape(3, 3)
    return intrinsics, extrinsics


def read_cam_file(filename, ndepths=192, interval_scale=1.06):
    """-> (intrinsics with rows 0-1 / 4, extrinsics, depth_min, depth_interval) as the eval dataset
    reads them (datasets/general_eval.py:62-81): a third field on line 11 (num_depth) redefines the
    interval as (depth_max - depth_min) / ndepths with depth_max = depth_min + int(num_depth) *
    interval; the interval is then scaled by interval_scale."""
    lines = _cam_lines(filename)
    intrinsics, extrinsics = read_camera_parameters(filename)
    intrinsics[:2, :] /= 4.0
    fields = lines[11].split()
    depth_min, depth_interval = float(fields[0]), float(fields[1])
    if len(fields) >= 3:
        depth_max = depth_min + int(float(fields[2])) * depth_interval
        depth_interval = (depth_max - depth_min) / ndepths
    return intrinsics, extrinsics, depth_min, depth_interval * interval_scale


def write_cam(filename, cam):
    """cam (2, 4, 4): [0] extrinsic, [1][:3,:3] intrinsic, [1][3] depth params (test_uni.py:182-199)."""
    with open(filename, "w") as f:
        f.write("extrinsic\n")
        for i in range(4):
            for j in range(4):
                f.write(str(cam[0][i][j]) + " ")
            f.write("\n")
        f.write("\n")
        f.write("intrinsic\n")
        for i in range(3):
            for j in range(3):
                f.write(str(cam[1][i][j]) + " ")
            f.write("\n")
        f.write("\n" + " ".join(str(cam[1][3][k]) for k in range(4)) + "\n")


def read_pair_file(filename, nviews=None):
    """-> [(ref_view, [src_view, ...]), ...]; views without sources are dropped. With nviews, the
    source list is filled to nviews entries with its first element, as the eval dataset does
    (datasets/general_eval.py:38-50); without, as listed (filter/dypcd.py:84-95)."""
    data = []
    with open(filename) as f:
        num_viewpoint = int(f.readline())
        for _ in range(num_viewpoint):
            ref_view = int(f.readline().rstrip())
            src_views = [int(x) for x in f.readline().rstrip().split()[1::2]]
            if not src_views:
                continue
            if nviews is not None and len(src_views) < nviews:
                src_views = src_views + [src_views[0]] * (nviews - len(src_views))
            data.append((ref_view, src_views))
    return data


# ------------------------------------------------------------------------------------ resizing
def resize_bilinear(img, new_w, new_h):
    """(H, W[, C]) float32 -> (new_h, new_w[, C]); cv2.INTER_LINEAR on float images."""
    t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.float32))
    chw = t[None, None] if t.ndim == 2 else t.permute(2, 0, 1)[None]
    out = F.interpolate(chw, size=(int(new_h), int(new_w)), mode="bilinear", align_corners=False)[0]
    return (out[0] if t.ndim == 2 else out.permute(1, 2, 0)).contiguous().numpy()


def resize_nearest(img, new_w, new_h):
    """cv2.INTER_NEAREST: destination (y, x) takes source (floor(y * H / new_h), floor(x * W / new_w))."""
    h, w = img.shape[:2]
    ys = np.minimum(np.floor(np.arange(new_h) * (h / new_h)).astype(np.int64), h - 1)
    xs = np.minimum(np.floor(np.arange(new_w) * (w / new_w)).astype(np.int64), w - 1)
    return img[ys][:, xs]


def scale_mvs_input(img, intrinsics, max_w, max_h, base=32):
    """datasets/general_eval.py:89-108: shrink to fit (max_w, max_h) keeping the aspect ratio, round
    both sides down to a multiple of `base`, scale K's rows accordingly."""
    h, w = img.shape[:2]
    if h > max_h or w > max_w:
        scale = 1.0 * max_h / h
        if scale * w > max_w:
            scale = 1.0 * max_w / w
        new_w, new_h = scale * w // base * base, scale * h // base * base
    else:
        new_w, new_h = 1.0 * w // base * base, 1.0 * h // base * base
    intrinsics = intrinsics.copy()
    intrinsics[0, :] *= 1.0 * new_w / w
    intrinsics[1, :] *= 1.0 * new_h / h
    return resize_bilinear(img, int(new_w), int(new_h)), intrinsics


def read_img(filename):
    """RGB image as float32 in [0, 1] (datasets/general_eval.py:83-87)."""
    from PIL import Image
    return np.array(Image.open(filename), dtype=np.float32) / 255.0


# ------------------------------------------------------------------------------ eval samples
def stage_projections(proj_matrices):
    """(N, 2, 4, 4) stage-1 projections -> {'stage1', 'stage2', 'stage3'} with K rows 0-1 x1/x2/x4
    (datasets/general_eval.py:172-186)."""
    s2 = proj_matrices.copy()
    s2[:, 1, :2, :] = proj_matrices[:, 1, :2, :] * 2
    s3 = proj_matrices.copy()
    s3[:, 1, :2, :] = proj_matrices[:, 1, :2, :] * 4
    return {"stage1": proj_matrices, "stage2": s2, "stage3": s3}


class EvalScenes:
    """The reference's eval dataset (datasets/general_eval.py:8-199) over a DTU-style tree
    <datapath>/<scan>/{pair.txt, cams/%08d_cam.txt, images[_post]/%08d.jpg}: item i is the sample
    dict CascadeMVSNet.forward consumes (imgs (N,3,H,W), proj_matrices per stage, depth_values,
    intrinsics_matrices per stage, filename pattern)."""

    def __init__(self, datapath, scans, nviews, ndepths=192, interval_scale=1.06, max_h=1184, max_w=1600,
                 fix_res=False):
        self.datapath, self.nviews, self.ndepths = datapath, nviews, ndepths
        self.max_h, self.max_w = max_h, max_w
        self.fix_res, self.fix_wh, self._s = fix_res, False, None
        self.interval_scale = {s: (interval_scale if isinstance(interval_scale, float) else interval_scale[s])
                               for s in scans}
        self.metas = [(scan, ref, src) for scan in scans
                      for ref, src in read_pair_file(os.path.join(datapath, scan, "pair.txt"), nviews)]

    def __len__(self):
        return len(self.metas)

    def _img_path(self, scan, vid):
        p = os.path.join(self.datapath, scan, "images_post", "%08d.jpg" % vid)
        return p if os.path.exists(p) else os.path.join(self.datapath, scan, "images", "%08d.jpg" % vid)

    def __getitem__(self, idx):
        scan, ref_view, src_views = self.metas[idx]
        view_ids = [ref_view] + src_views[:self.nviews - 1]
        imgs, projs, depth_values, K = [], [], None, None
        for i, vid in enumerate(view_ids):
            img = read_img(self._img_path(scan, vid))
            K, E, dmin, dint = read_cam_file(os.path.join(self.datapath, scan, "cams", "%08d_cam.txt" % vid),
                                             self.ndepths, self.interval_scale[scan])
            img, K = scale_mvs_input(img, K, self.max_w, self.max_h)
            if self.fix_res:  # one standard size for the whole scene (general_eval.py:133-137)
                self._s = img.shape[:2]
                self.fix_res, self.fix_wh = False, True
            if i == 0 and not self.fix_wh:
                self._s = img.shape[:2]
            s_h, s_w = self._s
            c_h, c_w = img.shape[:2]
            if (c_h, c_w) != (s_h, s_w):
                img = resize_bilinear(img, s_w, s_h)
                K[0, :] *= 1.0 * s_w / c_w
                K[1, :] *= 1.0 * s_h / c_h
            imgs.append(img)
            pm = np.zeros((2, 4, 4), dtype=np.float32)
            pm[0] = E
            pm[1, :3, :3] = K
            projs.append(pm)
            if i == 0:
                depth_values = np.arange(dmin, dint * (self.ndepths - 0.5) + dmin, dint, dtype=np.float32)
        projs = np.stack(projs)
        ins = {"stage1": K, "stage2": K.copy(), "stage3": K.copy()}  # K of the last view, as the reference
        ins["stage2"][:2, :] = K[:2, :] * 2.0
        ins["stage3"][:2, :] = K[:2, :] * 4.0
        return {"imgs": np.stack(imgs).transpose(0, 3, 1, 2), "proj_matrices": stage_projections(projs),
                "depth_values": depth_values, "intrinsics_matrices": ins,
                "filename": scan + "/{}/" + "%08d" % view_ids[0] + "{}"}


# ------------------------------------------------------------------------------------- outputs
def save_stage_outputs(outdir, filename, outputs, b=0):
    """Depth / confidence PFMs of one reference view as test_uni.py:246-282 writes them (stage-1/2
    confidences nearest-upsampled to the final resolution)."""
    def path(kind, suffix):
        p = os.path.join(outdir, filename.format(kind, suffix))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        return p
    npy = lambda t: t[b].detach().float().cpu().numpy() if torch.is_tensor(t) else np.asarray(t[b], np.float32)
    conf = npy(outputs["photometric_confidence"])
    h, w = conf.shape
    save_pfm(path("depth_est", ".pfm"), npy(outputs["depth"]))
    save_pfm(path("depth_est", "_stage2.pfm"), npy(outputs["stage2"]["depth"]))
    save_pfm(path("depth_est", "_stage1.pfm"), npy(outputs["stage1"]["depth"]))
    save_pfm(path("confidence", ".pfm"), conf)
    save_pfm(path("confidence", "_stage2.pfm"), resize_nearest(npy(outputs["stage2"]["photometric_confidence"]), w, h))
    save_pfm(path("confidence", "_stage1.pfm"), resize_nearest(npy(outputs["stage1"]["photometric_confidence"]), w, h))


def write_ply(filename, xyz, rgb):
    """Binary little-endian PLY of vertices (x, y, z float32; red, green, blue uint8), the element
    layout filter/dypcd.py:306-326 writes through plyfile."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8).reshape(-1, 3)
    v = np.empty(len(xyz), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("red", "u1"), ("green", "u1"),
                                  ("blue", "u1")])
    v["x"], v["y"], v["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    v["red"], v["green"], v["blue"] = rgb[:, 0], rgb[:, 1], rgb[:, 2]
    header = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
              "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n"
              % len(v))
    with open(filename, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(v.tobytes())


def read_ply(filename):
    """Inverse of write_ply -> (xyz float32 (n,3), rgb uint8 (n,3))."""
    with open(filename, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    n = int(re.search(rb"element vertex (\d+)", data[:end]).group(1))
    v = np.frombuffer(data[end:], dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("red", "u1"), ("green", "u1"),
                                         ("blue", "u1")], count=n)
    return np.stack([v["x"], v["y"], v["z"]], 1), np.stack([v["red"], v["green"], v["blue"]], 1)
