"""Scenes that stress tight binning's predicate (preprocess.hip cull_data + col_spans) where its
float margins are thinnest; shared by the CPU brute force (test_tight_model.py) and the GPU pin
(test_gpu_tight_pin.py).  Camera: the static view at (0, 0, 4), 1280x720 unless noted.

  needles     -- one long axis (logU(0.004, 0.06)) and two ~zero ones (logU(1e-7, 1e-4)): the
                 2D covariance is rank-1 + 0.3 I, so det / (a c) -> ~1e-7 (near-singular conics)
  faint       -- opacity in [0.97, 1.05] / 255, a slice exactly float32(1/255): the alpha
                 threshold's log L = ln(255 o) at or just above 0 (ellipses of ~zero size)
  off_centre  -- centres projected 0..300 px outside the frame with radii 60..260 px: getRect
                 clips the rect to <= 8 columns / <= 15 rows at the edge, so huge splats whose
                 centre lies far from every tile of the rect are span-coded
  rect_limits -- radii 48..80 px: rects of 7, 8 (the span code's limit), 9 and 10 columns
and `conics_2d`, a direct fuzz of upstream's 2D stage (cov2D = J W S W^T J^T + 0.3 I restated
from its eigen-form, conic and radius in upstream's float32 order) for the CPU model check.
"""
from __future__ import annotations

import numpy as np

from gaussiansplattingviewer_amd.camera import Camera, static_camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians

W, H = 1280, 720
KINDS = ("needles", "faint", "off_centre", "rect_limits")


def _focal_and_tan():
    cam = Camera(H, W)
    tx, ty, _ = cam.get_htanfovxy_focal()
    return H / (2.0 * ty), tx, ty


def _place(rng, n, ndc_lo, ndc_hi, depth_lo, depth_hi):
    """Points at view depth U(depth_lo, depth_hi) whose NDC x / y magnitude is U(ndc_lo, ndc_hi)
    on a random side (camera at (0,0,4) looking down -z, up +y)."""
    _, tx, ty = _focal_and_tan()
    depth = rng.uniform(depth_lo, depth_hi, n)
    nx = rng.uniform(ndc_lo, ndc_hi, n) * rng.choice([-1.0, 1.0], n)
    ny = rng.uniform(-ndc_hi, ndc_hi, n)
    swap = rng.random(n) < 0.5  # half of them off the top / bottom edge instead
    nx2 = np.where(swap, rng.uniform(-ndc_hi, ndc_hi, n), nx)
    ny2 = np.where(swap, rng.uniform(ndc_lo, ndc_hi, n) * rng.choice([-1.0, 1.0], n), ny)
    return np.stack([nx2 * tx * depth, ny2 * ty * depth, 4.0 - depth], axis=1)


def scene(kind: str, P: int, seed: int):
    """(GaussianData, Camera) of one stress scene."""
    rng = np.random.default_rng(1000 + seed)
    g = synthetic_gaussians(P, 3, seed)
    f, _, _ = _focal_and_tan()
    if kind == "needles":
        g.scale[:, 0] = np.exp(rng.uniform(np.log(0.004), np.log(0.06), P))
        g.scale[:, 1:] = np.exp(rng.uniform(np.log(1e-7), np.log(1e-4), (P, 2)))
        g.opacity[:] = rng.uniform(0.05, 0.999, (P, 1))
    elif kind == "faint":
        g.scale[:] = np.exp(rng.uniform(-5.0, -3.0, (P, 3)))
        g.opacity[:] = rng.uniform(0.97 / 255, 1.05 / 255, (P, 1))
        g.opacity[::5] = np.float32(1.0 / 255.0)
    elif kind == "off_centre":
        g.xyz[:] = _place(rng, P, 1.0, 1.5, 2.0, 5.0)
        depth = 4.0 - g.xyz[:, 2]
        r = rng.uniform(60.0, 260.0, P)  # target radius in pixels
        s = r * depth / (3.0 * f)
        g.scale[:] = s[:, None] * rng.uniform(0.5, 1.0, (P, 3))
        g.opacity[:] = rng.uniform(0.3, 0.999, (P, 1))
    elif kind == "rect_limits":
        g.xyz[:] = _place(rng, P, 0.0, 0.95, 3.0, 5.0)
        depth = 4.0 - g.xyz[:, 2]
        r = rng.uniform(48.0, 80.0, P)
        s = r * depth / (3.0 * f)
        g.scale[:] = s[:, None] * rng.uniform(0.3, 1.0, (P, 3))
        g.scale[:, 0] = s  # the longest axis sets the radius
        g.opacity[:] = rng.uniform(0.02, 0.999, (P, 1))
    else:
        raise KeyError(kind)
    g.scale[:] = g.scale.astype(np.float32)
    g.opacity[:] = g.opacity.astype(np.float32)
    return g, static_camera(W, H)


def conics_2d(n: int, seed: int, w: int = W, h: int = H):
    """Random 2D splats in upstream's form: cov2D = R diag(s1, s2) R^T + 0.3 I with s1, s2 ~
    logU(1e-6, 3e3) px^2 (rank-1 when one is ~0: det / (a c) -> 0), then upstream's float32
    conic (det, 1/det, (c, -b, a) / det) and radius ceil(3 sqrt(max(lambda1, lambda2))), and
    centres over [-400, w + 400] x [-400, h + 400].  Returns (means2D, conic_opacity, radii)."""
    rng = np.random.default_rng(seed)
    f32 = np.float32
    s1 = np.exp(rng.uniform(np.log(1e-6), np.log(3e3), n))
    s2 = np.exp(rng.uniform(np.log(1e-6), np.log(3e3), n))
    th = rng.uniform(0.0, np.pi, n)
    c, s = np.cos(th), np.sin(th)
    a = (c * c * s1 + s * s * s2).astype(f32) + f32(0.3)
    cc = (s * s * s1 + c * c * s2).astype(f32) + f32(0.3)
    b = (c * s * (s1 - s2)).astype(f32)
    det = a * cc - b * b
    ok = det != f32(0.0)
    det_inv = f32(1.0) / np.where(ok, det, f32(1.0))
    conic = np.stack([cc * det_inv, -b * det_inv, a * det_inv], axis=1).astype(f32)
    mid = f32(0.5) * (a + cc)
    l1 = mid + np.sqrt(np.maximum(f32(0.1), mid * mid - det))
    l2 = mid - np.sqrt(np.maximum(f32(0.1), mid * mid - det))
    radius = np.ceil(f32(3.0) * np.sqrt(np.maximum(l1, l2))).astype(np.int64)
    radius = np.where(ok, np.minimum(radius, 2**31 - 1), 0).astype(np.int32)
    means = np.stack([rng.uniform(-400, w + 400, n), rng.uniform(-400, h + 400, n)],
                     axis=1).astype(f32)
    op = rng.uniform(0.9 / 255, 1.0, n)
    op[::4] = rng.uniform(1.0 / 255, 1.1 / 255, len(op[::4]))
    op[::9] = 1.0 / 255
    co = np.concatenate([conic, op.astype(f32)[:, None]], axis=1).astype(f32)
    return means, np.ascontiguousarray(co), radius
