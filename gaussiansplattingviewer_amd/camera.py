"""Camera math that produces the rasterizer's inputs (util.py:10-116 of the viewer), headless.

The viewer builds every camera input from `util.Camera` with PyGLM: `get_view_matrix`
(util.py:58-70, glm.lookAt), `perspective` / `get_project_matrix` (util.py:72-105) and
`get_htanfovxy_focal` (util.py:107-113).  PyGLM is not available to this framework, so the
view matrix is restated with glm's lookAtRH in float32; the projection and tan-fov are plain
numpy like the original.  Matrices are math layout (translation in [:3, 3]), as every viewer
consumer reads them (renderer_ogl.py:14, renderer_cuda.py:189-194).

`cuda_camera_inputs` restates renderer_cuda.py:181-203: negate rows 0 and 2 of the view,
projmatrix = P @ view, both transposed (upstream reads column-major).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def _dot(a, b):
    return F32(F32(a[0] * b[0]) + F32(a[1] * b[1])) + F32(a[2] * b[2])


def _normalize(v):
    return (v * (F32(1.0) / np.sqrt(_dot(v, v)))).astype(F32)


def _cross(x, y):
    return np.array([x[1] * y[2] - y[1] * x[2], x[2] * y[0] - y[2] * x[0],
                     x[0] * y[1] - y[0] * x[1]], dtype=F32)


def look_at(eye, center, up) -> np.ndarray:
    """glm::lookAtRH in float32, returned in math layout (rows s, u, -f)."""
    eye = np.asarray(eye, dtype=F32)
    center = np.asarray(center, dtype=F32)
    up = np.asarray(up, dtype=F32)
    f = _normalize((center - eye).astype(F32))
    s = _normalize(_cross(f, up))
    u = _cross(s, f)
    m = np.eye(4, dtype=F32)
    m[0, :3] = s
    m[1, :3] = u
    m[2, :3] = -f
    m[0, 3] = -_dot(s, eye)
    m[1, 3] = -_dot(u, eye)
    m[2, 3] = _dot(f, eye)
    return m


class Camera:
    """Headless counterpart of util.Camera: same attributes and matrix methods."""

    def __init__(self, h: int, w: int):
        self.znear = 0.1
        self.zfar = 100
        self.h = h
        self.w = w
        self.fovy = 2 * math.atan(2088.0 / (3443.915946 * 2))
        self.position = np.array([0.0, 0.0, 3.0]).astype(np.float32)
        self.target = np.array([0.0, 0.0, 0.0]).astype(np.float32)
        self.up = np.array([0.0, -1.0, 0.0]).astype(np.float32)
        self.camera_up = np.array([0.0, -1.0, 0.0], dtype=F32)
        self.camera_front = np.array([0.0, 0.0, -1.0], dtype=F32)
        self.camera_position = np.array([-3.0, 0.0, 1.5], dtype=F32)
        self.is_pose_dirty = True
        self.is_intrin_dirty = True

    def get_view_matrix(self, arcball=True, front=None, pos=None, up=None, view=None):
        if arcball:
            if front is not None:
                if view is not None:
                    return np.array(view)
                pos = np.asarray(pos, dtype=F32)
                return look_at(pos, pos + np.asarray(front, dtype=F32), up)
            target = self.camera_position + self.camera_front
            return look_at(self.camera_position, target, self.camera_up)
        return look_at(self.position, self.target, self.up)

    @staticmethod
    def perspective(fov, aspect, near, far):
        f = 1 / np.tan(fov / 2.0)
        mat = np.zeros((4, 4))
        mat[0, 0] = f / aspect
        mat[1, 1] = f
        mat[2, 2] = -(far + near) / (far - near)
        mat[2, 3] = -(2.0 * far * near) / (far - near)
        mat[3, 2] = -1.0
        return mat

    def get_project_matrix(self):
        aspect = self.w / self.h
        return np.array(self.perspective(self.fovy, aspect, 0.1, 100.0)).astype(np.float32)

    def get_htanfovxy_focal(self):
        htany = np.tan(self.fovy / 2)
        htanx = htany * (self.w / self.h)
        focal = self.h / (2 * htany)
        return [htanx, htany, focal]

    def get_focal(self):
        return self.h / (2 * np.tan(self.fovy / 2))

    def look_from(self, eye, center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)):
        """Place the arcball camera at `eye` looking at `center` (bench / harness helper)."""
        self.camera_position = np.asarray(eye, dtype=F32)
        self.position = np.asarray(eye, dtype=F32)  # campos source (renderer_cuda.py:192)
        self.camera_front = (np.asarray(center, dtype=F32) - self.camera_position).astype(F32)
        self.camera_up = np.asarray(up, dtype=F32)
        self.is_pose_dirty = True


def cuda_camera_inputs(camera: Camera, view_mat: np.ndarray | None = None):
    """renderer_cuda.py:181-203 as host numpy: returns (viewmatrix, projmatrix, campos,
    tanfovx, tanfovy) with both matrices already transposed to upstream's column-major."""
    view = np.array(camera.get_view_matrix() if view_mat is None else view_mat, dtype=np.float32)
    view[[0, 2], :] = -view[[0, 2], :]
    proj = camera.get_project_matrix() @ view
    hfovx, hfovy, _ = camera.get_htanfovxy_focal()
    campos = np.array(camera.position, dtype=np.float32)  # renderer_cuda.py:192 uses .position
    return (np.ascontiguousarray(view.T), np.ascontiguousarray(proj.T), campos,
            float(hfovx), float(hfovy))


def static_camera(w: int, h: int, eye=(0.0, 0.0, 4.0)) -> Camera:
    """The static view of the benchmark configs: lookAtRH(eye, 0, +y)."""
    cam = Camera(h, w)
    cam.look_from(eye)
    return cam


def orbit_eye(i: int, n: int = 1000, radius: float = 4.0, height: float = 0.5):
    """Config C5 orbit: eye_i = (r sin t, 0.5, r cos t), t = 2 pi i / n (cf. main_test.py:392-426)."""
    t = 2.0 * math.pi * i / n
    return (radius * math.sin(t), height, radius * math.cos(t))
