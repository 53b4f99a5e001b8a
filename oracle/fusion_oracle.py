"""TEST INFRASTRUCTURE — CPU restatement of the reference's dynamic-consistency depth fusion
(filter/dypcd.py) for one reference view, used only by tests/ and tools/bench_fusion.py as the checker
and CPU baseline. Never imported by the product path (damvsnet_amd/fusion.py runs the HIP kernel).

Follows, line by line:
  reproject_with_depth ........ filter/dypcd.py:98-136 (float64 projections, float32 casts where the
                                reference casts, cv2.remap INTER_LINEAR on the source depth)
  check_geometric_consistency . filter/dypcd.py:139-159 (masks for i = 2..10: dist < i*dist_base and
                                relative depth difference < i*rel_diff_base; the i = 10 mask zeroes
                                the reprojected depth)
  filter_depth (per view) ..... filter/dypcd.py:184-297 (photo mask from three confidences, dynamic
                                geometric mask, averaged depth, world points + colours)

cv2 is not installed here: `remap_linear` restates OpenCV's documented INTER_LINEAR remap for float
images with float maps — coordinates quantised to 1/32 pixel (INTER_BITS = 5, cvRound), bilinear
weights from the 32x32 table (1 - t, t) products, BORDER_CONSTANT 0 for taps outside the image —
so parity with cv2 itself is unpinned; the GPU kernel is checked against this restatement.
"""
import numpy as np

INTER_BITS = 5
INTER_TAB = 1 << INTER_BITS


def remap_linear(src, mapx, mapy):
    """cv2.remap(src float32 (H,W), mapx, mapy float32, INTER_LINEAR, BORDER_CONSTANT 0)."""
    H, W = src.shape
    X = np.rint(mapx.astype(np.float32) * np.float32(INTER_TAB))
    Y = np.rint(mapy.astype(np.float32) * np.float32(INTER_TAB))
    big = np.float64(2 ** 31 - 1)
    X = np.clip(np.nan_to_num(X.astype(np.float64), nan=0.0), -big - 1, big).astype(np.int64)
    Y = np.clip(np.nan_to_num(Y.astype(np.float64), nan=0.0), -big - 1, big).astype(np.int64)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    fx = (X & (INTER_TAB - 1)).astype(np.float32) * np.float32(1.0 / INTER_TAB)
    fy = (Y & (INTER_TAB - 1)).astype(np.float32) * np.float32(1.0 / INTER_TAB)
    cx = [np.float32(1) - fx, fx]
    cy = [np.float32(1) - fy, fy]
    w = [cy[0] * cx[0], cy[0] * cx[1], cy[1] * cx[0], cy[1] * cx[1]]
    out = np.zeros(mapx.shape, np.float32)
    vals = []
    for k in range(4):
        xx, yy = sx + (k & 1), sy + (k >> 1)
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = np.where(ok, src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)], np.float32(0))
        vals.append(v.astype(np.float32))
    out = ((vals[0] * w[0] + vals[1] * w[1]) + vals[2] * w[2]) + vals[3] * w[3]
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
    return np.where(outside, np.float32(0), out).astype(np.float32)


def reproject_with_depth(depth_ref, K_ref, E_ref, depth_src, K_src, E_src):
    """filter/dypcd.py:98-136."""
    height, width = depth_ref.shape
    x_ref, y_ref = np.meshgrid(np.arange(0, width), np.arange(0, height))
    x_ref, y_ref = x_ref.reshape([-1]), y_ref.reshape([-1])
    xyz_ref = np.matmul(np.linalg.inv(K_ref), np.vstack((x_ref, y_ref, np.ones_like(x_ref))) * depth_ref.reshape([-1]))
    xyz_src = np.matmul(np.matmul(E_src, np.linalg.inv(E_ref)), np.vstack((xyz_ref, np.ones_like(x_ref))))[:3]
    K_xyz_src = np.matmul(K_src, xyz_src)
    xy_src = K_xyz_src[:2] / K_xyz_src[2:3]
    x_src = xy_src[0].reshape([height, width]).astype(np.float32)
    y_src = xy_src[1].reshape([height, width]).astype(np.float32)
    sampled = remap_linear(depth_src, x_src, y_src)
    xyz_src = np.matmul(np.linalg.inv(K_src), np.vstack((xy_src, np.ones_like(x_ref))) * sampled.reshape([-1]))
    xyz_rep = np.matmul(np.matmul(E_ref, np.linalg.inv(E_src)), np.vstack((xyz_src, np.ones_like(x_ref))))[:3]
    depth_rep = xyz_rep[2].reshape([height, width]).astype(np.float32)
    K_xyz_rep = np.matmul(K_ref, xyz_rep)
    K_xyz_rep[2:3][K_xyz_rep[2:3] == 0] += 0.00001
    xy_rep = K_xyz_rep[:2] / K_xyz_rep[2:3]
    x_rep = xy_rep[0].reshape([height, width]).astype(np.float32)
    y_rep = xy_rep[1].reshape([height, width]).astype(np.float32)
    return depth_rep, x_rep, y_rep, x_src, y_src


def check_geometric_consistency(depth_ref, K_ref, E_ref, depth_src, K_src, E_src, dist_base, rel_diff_base):
    """filter/dypcd.py:139-159 -> (masks for i = 2..10, mask at i = 10, reprojected depth)."""
    height, width = depth_ref.shape
    x_ref, y_ref = np.meshgrid(np.arange(0, width), np.arange(0, height))
    depth_rep, x_rep, y_rep, _, _ = reproject_with_depth(depth_ref, K_ref, E_ref, depth_src, K_src, E_src)
    dist = np.sqrt((x_rep - x_ref) ** 2 + (y_rep - y_ref) ** 2)
    rel = np.abs(depth_rep - depth_ref) / depth_ref
    masks = [np.logical_and(dist < i * dist_base, rel < i * rel_diff_base) for i in range(2, 11)]
    mask = masks[-1]
    depth_rep[~mask] = 0
    return masks, mask, depth_rep


def fuse_view(depth_ref, K_ref, E_ref, srcs, confs, conf_thr, dist_base=0.25, rel_diff_base=1 / 1300, img=None):
    """One reference view of filter_depth (filter/dypcd.py:196-297). srcs: [(depth, K, E)],
    confs: (stage3, stage2, stage1) confidence maps, conf_thr = args.conf (stage1, stage2, stage3).
    -> dict photo, geo, final masks, depth_avg (float64), xyz (n,3) float64 world points, rgb."""
    photo = np.logical_and(np.logical_and(confs[0] > conf_thr[2], confs[1] > conf_thr[1]), confs[2] > conf_thr[0])
    reps = []
    geo_sum = 0
    dy_range = len(srcs) + 1
    geo_sums = [0] * (dy_range - 2)
    for depth_src, K_src, E_src in srcs:
        masks, geo_mask, depth_rep = check_geometric_consistency(depth_ref, K_ref, E_ref, depth_src, K_src, E_src,
                                                                 dist_base, rel_diff_base)
        geo_sum += geo_mask.astype(np.int32)
        for i in range(2, dy_range):
            geo_sums[i - 2] += masks[i - 2].astype(np.int32)
        reps.append(depth_rep)
    depth_avg = (sum(reps) + depth_ref) / (geo_sum + 1)
    geo = geo_sum >= dy_range
    for i in range(2, dy_range):
        geo = np.logical_or(geo, geo_sums[i - 2] >= i)
    final = np.logical_and(photo, geo)
    height, width = depth_avg.shape[:2]
    x, y = np.meshgrid(np.arange(0, width), np.arange(0, height))
    x, y, depth = x[final], y[final], depth_avg[final]
    xyz_ref = np.matmul(np.linalg.inv(K_ref), np.vstack((x, y, np.ones_like(x))) * depth)
    xyz_world = np.matmul(np.linalg.inv(E_ref), np.vstack((xyz_ref, np.ones_like(x))))[:3].T
    rgb = (img[final] * 255).astype(np.uint8) if img is not None else None
    return {"photo": photo, "geo": geo, "final": final, "depth_avg": depth_avg, "xyz": xyz_world, "rgb": rgb}
