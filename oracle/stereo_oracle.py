"""TEST INFRASTRUCTURE -- CPU restatements for the COLMAP pose, disparity and frame-packing rows
(SURVEY.md §8(f) rows 1, 3, 4).  Never imported by the product path.

* `colmap_view_f64` -- the reference's pose -> view chain in float64: create_look_at_from_colmap
  (main.py:196-215) with quaternion_to_rotation_matrix (main.py:165-181), then the reference's
  own numpy `look_at` (main.py:218-243, mathematically glm.lookAtRH), then T(-0.5) . view
  (main.py:376-380).  The product restates glm.lookAtRH in float32; parity is within float32
  rounding of this float64 chain.  glm itself is absent: PyGLM's float32
  rounding is not pinned.
* `disparity_f32` -- gau_vert.glsl:182-207 in float32, in the kernel's operation order
  (row-wise left-to-right sums, no FMA): bit-exact parity with gsr_disparity_colors.  Against a
  GL driver's shader compiler the order is unpinned.
* `pack_f32` -- the frame packers: round(clamp(v,0,1)*255) for RGB8 (GL unorm conversion;
  ties to even as np.rint), numpy's float32 -> uint16 astype for the disparity PNG
  (main.py:873-874; out-of-range values follow x86's truncate-through-int32-and-wrap, the
  packer's documented behaviour), HWC RGBA float with alpha 1 (renderer_cuda.py:226-228).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def quat_to_rot_f64(qw, qx, qy, qz):
    q = np.array([qw, qx, qy, qz], dtype=np.float64)
    qw, qx, qy, qz = q / np.linalg.norm(q)
    return np.array([
        [1 - 2 * qy ** 2 - 2 * qz ** 2, 2 * qx * qy - 2 * qz * qw, 2 * qx * qz + 2 * qy * qw],
        [2 * qx * qy + 2 * qz * qw, 1 - 2 * qx ** 2 - 2 * qz ** 2, 2 * qy * qz - 2 * qx * qw],
        [2 * qx * qz - 2 * qy * qw, 2 * qy * qz + 2 * qx * qw, 1 - 2 * qx ** 2 - 2 * qy ** 2]])


def look_at_f64(eye, center, up):
    """main.py:218-243 (returned here untransposed: math layout)."""
    forward = center - eye
    forward = forward / np.linalg.norm(forward)
    up = up / np.linalg.norm(up)
    right = np.cross(forward, up)
    right = right / np.linalg.norm(right)
    up = np.cross(right, forward)
    m = np.eye(4)
    m[0, :3], m[1, :3], m[2, :3] = right, up, -forward
    m[:3, 3] = -m[:3, :3] @ eye
    return m


def colmap_view_f64(pose_fields, baseline=-0.5):
    """One images.txt entry -> (view_left, view_right, cam_left, cam_right) in float64."""
    qw, qx, qy, qz, tx, ty, tz = (float(pose_fields[i]) for i in range(1, 8))
    eye = np.array([-tx, -ty, -tz])
    rot = quat_to_rot_f64(qw, qx, qy, qz).T @ np.diag([1.0, 1.0, -1.0])
    center = eye + rot @ np.array([0.0, 0.0, -1.0])
    up = rot @ np.array([0.0, -1.0, 0.0])
    vl = look_at_f64(eye, center, up)
    t = np.eye(4)
    t[0, 3] = baseline
    vr = t @ vl
    return vl, vr, eye, np.linalg.inv(vr)[:, 3]


def disparity_f32(xyz, view, proj, baseline=-0.5):
    """(P,) float32 disparity of gau_vert.glsl:182-207, kernel operation order."""
    xyz = np.asarray(xyz, F32)
    v = np.asarray(view, F32)
    p = np.asarray(proj, F32)
    b = F32(baseline)

    def ndc_x(x, y, z):
        pv = [((v[i, 0] * x + v[i, 1] * y) + v[i, 2] * z) + v[i, 3] for i in range(4)]
        sx = ((p[0, 0] * pv[0] + p[0, 1] * pv[1]) + p[0, 2] * pv[2]) + p[0, 3] * pv[3]
        sw = ((p[3, 0] * pv[0] + p[3, 1] * pv[1]) + p[3, 2] * pv[2]) + p[3, 3] * pv[3]
        return (sx / sw).astype(F32)

    x, y, z = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    one, two = F32(1.0), F32(2.0)
    xl = (ndc_x(x, y, z) + one) / two
    xr = (ndc_x(x + b, y + F32(0.0), z + F32(0.0)) + one) / two
    return np.abs(xl - xr).astype(F32)


def _u16_wrap(v):
    v = np.asarray(v, F32)
    ok = (v == v) & (v < F32(2147483648.0)) & (v >= F32(-2147483648.0))
    out = np.zeros(v.shape, np.uint16)
    out[ok] = (np.trunc(v[ok]).astype(np.int64) & 0xFFFF).astype(np.uint16)
    return out


def pack_f32(chw, fmt, flip_rows=False):
    img = np.asarray(chw, F32)
    if flip_rows:
        img = img[:, ::-1, :]
    if fmt == "rgb8":
        c = np.clip(np.nan_to_num(img, nan=0.0), F32(0.0), F32(1.0)) * F32(255.0)
        return np.ascontiguousarray(np.rint(c).astype(np.uint8).transpose(1, 2, 0))
    if fmt == "r16":
        return _u16_wrap(img[0] * F32(65535.0))
    if fmt == "rgba_f32":
        hwc = img.transpose(1, 2, 0)
        return np.ascontiguousarray(np.concatenate([hwc, np.ones_like(hwc[..., :1])], -1))
    raise ValueError(fmt)
