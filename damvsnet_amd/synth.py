"""Synthetic, seeded inputs shaped like the reference's DTU test samples.

The reference builds one test sample in ``datasets/general_eval.py:111-199``:

* ``imgs``            float32 (N, 3, H, W) in [0, 1]          (``:81-86,168``)
* ``proj_matrices``   dict stage1..3 -> float32 (N, 2, 4, 4)  (``:158-175``)
  ``[v, 0]`` = 4x4 world->camera extrinsic, ``[v, 1, :3, :3]`` = K of that stage
  (stage1 = K/4 of the input resolution, x2 / x4 for stages 2 / 3).
* ``depth_values``    float32 (192,) ascending                 (``:163-165``)
* ``intrinsics_matrices`` dict stage1..3 -> (3, 3)             (``:176-193``)

There is no dataset in this environment, so every benchmark and parity test uses
this generator: DTU-like intrinsics (fx 2892.33, fy 2883.18,
cx 823.2, cy 619.07 at 1600x1200) rescaled to W x H, extrinsics with a yaw of
0.08*v rad and a translation of (-40v, 5v, 2v) mm for view v, depth_values
425 + 2.65*arange(192) mm, images U[0,1) from numpy PCG64.
"""
from __future__ import annotations

import math

import numpy as np

DTU_K = np.array([[2892.33, 0.0, 823.2],
                  [0.0, 2883.18, 619.07],
                  [0.0, 0.0, 1.0]], dtype=np.float64)
DTU_RES = (1200, 1600)  # (H, W) the DTU intrinsics refer to
DEPTH_MIN = 425.0
DEPTH_INTERVAL = 2.65
NUM_DEPTH_VALUES = 192


def _rng(seed, *stream):
    return np.random.Generator(np.random.PCG64([int(seed)] + [int(s) for s in stream]))


def view_extrinsic(v: int) -> np.ndarray:
    """World->camera 4x4 for view ``v`` (view 0 is the identity reference camera)."""
    a = 0.08 * v
    R = np.array([[math.cos(a), 0.0, math.sin(a)],
                  [0.0, 1.0, 0.0],
                  [-math.sin(a), 0.0, math.cos(a)]])
    E = np.eye(4)
    E[:3, :3] = R
    E[:3, 3] = (-40.0 * v, 5.0 * v, 2.0 * v)
    return E


def stage1_intrinsics(H: int, W: int) -> np.ndarray:
    """K at stage-1 (quarter) resolution of an H x W input, as general_eval.py:66,105-107 builds it."""
    K = DTU_K.copy()
    K[0, :] *= W / DTU_RES[1]
    K[1, :] *= H / DTU_RES[0]
    K[:2, :] /= 4.0
    return K


def cameras(B: int, N: int, H: int, W: int):
    """Return (proj_matrices dict, intrinsics dict, depth_values) as float32 numpy arrays.

    Shapes follow the reference collate: proj (B, N, 2, 4, 4), intrinsics (B, 3, 3),
    depth_values (B, 192).
    """
    K1 = stage1_intrinsics(H, W)
    proj = np.zeros((N, 2, 4, 4), dtype=np.float64)
    for v in range(N):
        proj[v, 0] = view_extrinsic(v)
        proj[v, 1, :3, :3] = K1
    proj = proj.astype(np.float32)
    p2 = proj.copy()
    p2[:, 1, :2, :] = proj[:, 1, :2, :] * 2
    p3 = proj.copy()
    p3[:, 1, :2, :] = proj[:, 1, :2, :] * 4
    K1f = K1.astype(np.float32)
    ins = {"stage1": K1f, "stage2": K1f.copy(), "stage3": K1f.copy()}
    ins["stage2"][:2, :] = K1f[:2, :] * 2.0
    ins["stage3"][:2, :] = K1f[:2, :] * 4.0
    dv = (DEPTH_MIN + DEPTH_INTERVAL * np.arange(NUM_DEPTH_VALUES, dtype=np.float64)).astype(np.float32)
    rep = lambda a: np.ascontiguousarray(np.broadcast_to(a, (B,) + a.shape))
    return ({k: rep(v) for k, v in (("stage1", proj), ("stage2", p2), ("stage3", p3))},
            {k: rep(v) for k, v in ins.items()},
            rep(dv))


def images(B: int, N: int, H: int, W: int, seed: int = 0) -> np.ndarray:
    """Seeded images U[0,1) of shape (B, N, 3, H, W), float32."""
    return _rng(seed, 1).random((B, N, 3, H, W), dtype=np.float32)


def features(B: int, N: int, C: int, h: int, w: int, seed: int = 0) -> np.ndarray:
    """Seeded feature maps (N, B, C, h, w) ~ N(0, 1) for DepthNet-only cases."""
    return _rng(seed, 2, C, h).standard_normal((N, B, C, h, w), dtype=np.float32)


def stage_hypotheses(B: int, D: int, h: int, w: int, seed: int = 0, dmin=DEPTH_MIN, span=None) -> np.ndarray:
    """Per-pixel ascending hypotheses (B, D, h, w) for DepthNet-only cases.

    A smooth depth surface plus a per-pixel interval, the shape stage 2/3 sampling produces.
    """
    span = span if span is not None else DEPTH_INTERVAL * NUM_DEPTH_VALUES
    r = _rng(seed, 3, D, h)
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    centre = dmin + span * (0.35 + 0.25 * np.sin(3.0 * xx + 2.0 * yy) * np.cos(2.0 * yy))
    half = (0.02 + 0.02 * r.random((h, w))) * span
    t = np.linspace(-1.0, 1.0, D)
    hyp = centre[None] + t[:, None, None] * half[None]
    return np.ascontiguousarray(np.broadcast_to(hyp, (B, D, h, w))).astype(np.float32)
