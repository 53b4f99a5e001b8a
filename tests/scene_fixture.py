"""A small DTU-style scene tree written from seeds (no reference code): the input of the f3 scene-I/O fixtures.

``make_scene(root)`` writes <root>/scan1/{pair.txt, cams/%08d_cam.txt, images[_post]/%08d.jpg} and returns the arrays it
wrote. Both tests/golden/make_f3.py (which runs the reference's parsers on the tree, build container only) and
tests/test_mvsio.py (which runs damvsnet_amd.mvsio on the same tree) call it, so the two see byte-identical files.

Coverage, following the reference readers (datasets/general_eval.py:35-193, filter/dypcd.py:70-95):
* pair.txt: a view without sources (dropped), views with fewer sources than nviews (filled with the first source);
* cam.txt: depth lines of 2 fields (min, interval), 3 fields (min, interval, num_depth: the interval redefined) and
  4 fields (min, interval, num_depth, max);
* images: sizes that are multiples of 32 and inside max_h x max_w (the reference's cv2.resize is then a copy, so the
  stubbed cv2 of make_f3.py is exact), one view under images_post/ (preferred over images/);
* the files are PNG data under .jpg names (PIL reads by content): lossless, so pixels are exact on any box.
"""
from __future__ import annotations

import os

import numpy as np

H, W, NV = 32, 64, 5

# ref view -> (source view, score) pairs as pair.txt lists them
PAIRS = [(0, [(1, 820.5), (2, 700.25), (3, 512.0), (4, 300.75)]),
         (1, [(0, 810.0), (2, 640.5)]),          # fewer than nviews: filled with the first source
         (2, []),                                 # no source: dropped
         (3, [(4, 900.0), (2, 450.5), (1, 120.25), (0, 10.0)]),
         (4, [(3, 777.0), (0, 555.5), (1, 333.25), (2, 111.0)])]

DEPTH_LINES = ["425.0 2.5", "425.0 2.5 192", "430.5 2.65 256 1108.9", "425.0 2.5", "600.25 1.75 128"]


def _cam_text(v, rng):
    yaw = 0.08 * v
    c, s = np.cos(yaw), np.sin(yaw)
    E = np.array([[c, 0, s, -40.0 * v + rng.uniform(-1, 1)], [0, 1, 0, 5.0 * v], [-s, 0, c, 2.0 * v], [0, 0, 0, 1]])
    K = np.array([[2892.33, 0, 823.205 + v], [0, 2883.18, 619.071 - v], [0, 0, 1]])
    lines = ["extrinsic"] + [" ".join("%.6f" % x for x in row) for row in E] + ["", "intrinsic"]
    lines += [" ".join("%g" % x for x in row) for row in K] + ["", DEPTH_LINES[v]]
    return "\n".join(lines) + "\n"


def make_scene(root, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    scan = os.path.join(root, "scan1")
    for d in ("cams", "images", "images_post"):
        os.makedirs(os.path.join(scan, d), exist_ok=True)
    with open(os.path.join(scan, "pair.txt"), "w") as f:
        f.write("%d\n" % len(PAIRS))
        for ref, src in PAIRS:
            f.write("%d\n%d %s\n" % (ref, len(src), " ".join("%d %g" % p for p in src)))
    imgs = []
    for v in range(NV):
        with open(os.path.join(scan, "cams", "%08d_cam.txt" % v), "w") as f:
            f.write(_cam_text(v, rng))
        img = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
        sub = "images_post" if v == 3 else "images"
        Image.fromarray(img).save(os.path.join(scan, sub, "%08d.jpg" % v), format="PNG")
        imgs.append(img)
    return {"imgs": np.stack(imgs)}


def pfm_arrays(seed=1):
    """Arrays the PFM fixtures round-trip: a grey map, a colour image, a single-channel (H, W, 1) map."""
    rng = np.random.default_rng(seed)
    return {"grey": (rng.random((7, 11), dtype=np.float32) * 900 + 100),
            "colour": rng.random((5, 6, 3), dtype=np.float32),
            "single": rng.random((4, 3, 1), dtype=np.float32)}
