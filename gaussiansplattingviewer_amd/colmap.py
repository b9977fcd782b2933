"""COLMAP pose ingestion and the viewer's pose -> view math.

The viewer reads a COLMAP text model (main.py:602-632) and turns each image pose into a left /
right stereo pair of pose dicts (`load_camera_positions`, main.py:275-407) that the renderers'
`update_camera_pose(camera, use_file=True, pose=...)` consume (renderer_cuda.py:181-194,
renderer_ogl.py:160-168).  This module restates that host logic without PyGLM (absent here):

* `read_images_txt` -- main.py:602-620: comment lines skipped, then every other remaining line
  is an image line (the odd ones are the POINTS2D lines), split on whitespace into exactly ten
  fields IMAGE_ID QW QX QY QZ TX TY TZ CAMERA_ID NAME (anything else raises ValueError, as the
  reference's tuple unpacking does).  The fields stay strings, like the reference's list.
* `read_cameras_txt` -- main.py:622-630 (id, model, width, height, fx, fy, cx, cy).  The viewer
  then overrides the window to `VIEWER_RESOLUTION` = 1160 x 522 regardless (main.py:632-633).
* `load_camera_positions` -- main.py:275-407 with `create_look_at_from_colmap`
  (main.py:196-215), `quaternion_to_rotation_matrix` (main.py:165-181) and glm.lookAtRH in
  float32.  The reference uses -t as the camera position (not -R^T t) and builds the view from
  a z-flipped transposed rotation; both quirks are kept, since the rendered datasets depend on
  them.  The right view is T(-0.5) . view (main.py:376-380), i.e. the left view with its x
  translation reduced by 0.5; the right pose's camera_position is column 3 of its inverse, a
  4-vector as in the reference (only its xyz reach the rasterizer).

Matrices are float32 math layout (translation in [:3, 3]), what `np.array(glm.mat4)` gives
every consumer (camera.py).  `getWorld2View2` (main.py:34-45) is computed and discarded by the
reference (main.py:336-338) and so is not restated.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .camera import look_at

F32 = np.float32

BASELINE = -0.5                 # main.py:279, the stereo baseline in world units
VIEWER_RESOLUTION = (1160, 522)  # (width, height) forced at main.py:632-633
FRONT_VECTOR = np.array([0.0, 0.0, 1.0], dtype=F32)  # global front_vector (main.py:160)


@dataclass(frozen=True)
class ColmapCamera:
    """One cameras.txt line (main.py:626-630 reads exactly these fields)."""
    camera_id: int
    model: str
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float


def read_images_txt(path: str) -> list[list[str]]:
    """main.py:602-620.  `path` is images.txt or the directory holding it."""
    if os.path.isdir(path):
        path = os.path.join(path, "images.txt")
    poses = []
    line_no = 0
    with open(path, "r") as f:
        for line in f.readlines():
            if line.startswith("#"):
                continue
            if line_no % 2 == 1:      # the POINTS2D line that follows every image line
                line_no += 1
                continue
            elements = line.split()
            if len(elements) != 10:
                raise ValueError(
                    f"{path}: image line {line_no} has {len(elements)} fields, expected 10 "
                    "(IMAGE_ID QW QX QY QZ TX TY TZ CAMERA_ID NAME)")
            poses.append(elements)
            line_no += 1
    return poses


def read_cameras_txt(path: str) -> list[ColmapCamera]:
    """main.py:622-630 (the reference keeps only the last line's values; all are returned
    here, in file order).  `path` is cameras.txt or the directory holding it."""
    if os.path.isdir(path):
        path = os.path.join(path, "cameras.txt")
    cams = []
    with open(path, "r") as f:
        for line in f.readlines():
            if line.startswith("#"):
                continue
            e = line.split()
            cams.append(ColmapCamera(int(e[0]), e[1], int(e[2]), int(e[3]), float(e[4]),
                                     float(e[5]), float(e[6]), float(e[7])))
    return cams


def quaternion_to_rotation_matrix(qw, qx, qy, qz) -> np.ndarray:
    """main.py:165-181: unit-normalise (float64), then the usual rotation matrix."""
    q = np.array([qw, qx, qy, qz], dtype=np.float64)
    norm = np.linalg.norm(q)
    if norm == 0:
        raise ValueError("Cannot normalize a zero-norm quaternion.")
    qw, qx, qy, qz = q / norm
    return np.array([
        [1 - 2 * qy ** 2 - 2 * qz ** 2, 2 * qx * qy - 2 * qz * qw, 2 * qx * qz + 2 * qy * qw],
        [2 * qx * qy + 2 * qz * qw, 1 - 2 * qx ** 2 - 2 * qz ** 2, 2 * qy * qz - 2 * qx * qw],
        [2 * qx * qz - 2 * qy * qw, 2 * qy * qz + 2 * qx * qw, 1 - 2 * qx ** 2 - 2 * qy ** 2],
    ])


def create_look_at_from_colmap(tx, ty, tz, qw, qx, qy, qz):
    """main.py:196-215 -> (camera_pos, center_point, world_up), float64 3-vectors."""
    camera_pos = np.array([-tx, -ty, -tz], dtype=np.float64)
    rot = quaternion_to_rotation_matrix(qw, qx, qy, qz).T @ np.diag([1.0, 1.0, -1.0])
    world_forward = rot @ np.array([0.0, 0.0, -1.0])
    world_up = rot @ np.array([0.0, -1.0, 0.0])
    return camera_pos, camera_pos + world_forward, world_up


def _inverse_column3(view: np.ndarray) -> np.ndarray:
    """Column 3 of inverse(view) as a float32 4-vector (glm.inverse(m)[3], main.py:403).
    Computed in float64 and rounded: glm's float32 cofactor inverse is not restated, so this
    can differ from the reference in the last bit (it only feeds the SH view direction)."""
    return np.linalg.inv(view.astype(np.float64))[:, 3].astype(F32)


def load_camera_positions(camera_pose, bounding_box=None, center=(0.0, 0.0, 0.0),
                          camera_bb=(0, 1, 0, 1, 0, 1)):
    """main.py:275-407: one images.txt entry -> (pose_left, pose_right) pose dicts.

    `bounding_box`, `center` and `camera_bb` are accepted for signature parity; the
    reference's use of them is commented out (main.py:284-309)."""
    qw, qx, qy, qz = (float(camera_pose[i]) for i in range(1, 5))
    x, y, z = (float(camera_pose[i]) for i in range(5, 8))
    camera_pos, center_point, up_vector = create_look_at_from_colmap(x, y, z, qw, qx, qy, qz)
    # glm.vec3(numpy float64) rounds each component to float32 before lookAtRH (main.py:343).
    view_left = look_at(camera_pos.astype(F32), center_point.astype(F32), up_vector.astype(F32))
    view_right = view_left.copy()
    view_right[0, 3] = view_left[0, 3] + F32(BASELINE)  # T(baseline) . view, exact (see doc)
    pose_left = {
        "camera_front": FRONT_VECTOR.copy(),
        "camera_up": up_vector,
        "camera_position": camera_pos,
        "camera_view": view_left,
    }
    pose_right = {
        "camera_front": FRONT_VECTOR.copy(),
        "camera_up": up_vector,
        "camera_position": _inverse_column3(view_right),
        "camera_view": view_right,
    }
    return pose_left, pose_right


def load_colmap_poses(colmap_dir: str):
    """The viewer's start-up ingestion (main.py:602-633): (poses, cameras, (width, height))."""
    poses = read_images_txt(colmap_dir)
    cam_path = os.path.join(colmap_dir, "cameras.txt")
    cameras = read_cameras_txt(cam_path) if os.path.exists(cam_path) else []
    return poses, cameras, VIEWER_RESOLUTION


def read_camera_poses_from_csv(csv_file_path: str) -> list[dict]:
    """main.py:529-562: rows of camera_front(3), camera_up(3), camera_position(3) saved by the
    middle-mouse handler (main.py:418-434) -> pose dicts.  Rows with fewer than 9 columns are
    skipped, rows that do not parse are reported and skipped, as in the reference.  The dicts
    carry "camera_view": None so `update_camera_pose` takes the lookAt(pos, pos + front, up)
    branch of get_view_matrix (util.py:60-64); the reference's dicts lack the key, which its
    renderers index (renderer_cuda.py:184), so it never rendered these."""
    import csv
    poses = []
    with open(csv_file_path, "r") as f:
        for row in csv.reader(f):
            if len(row) < 9:
                continue
            try:
                v = [float(c) for c in row[:9]]
            except ValueError as e:
                print(f"Error converting row to float: {row}. Error: {e}")
                continue
            poses.append({"camera_front": np.array(v[0:3], dtype=F32),
                          "camera_up": np.array(v[3:6], dtype=F32),
                          "camera_position": np.array(v[6:9], dtype=F32),
                          "camera_view": None})
    return poses


def camera_marker_gaussians(camera_poses):
    """main.py:729-745: one zero-opacity Gaussian per pose at (TX, TY, TZ) (scale 0.03, identity
    rotation, SH all ones, 48 coefficients) that the viewer appends to the scene.  Returns
    (xyz, rot, scale, opacity, sh) float32 arrays; opacity 0 makes them invisible."""
    n = len(camera_poses)
    xyz = np.array([[float(p[5]), float(p[6]), float(p[7])] for p in camera_poses],
                   dtype=np.float64).reshape(n, 3).astype(F32)
    rot = np.tile(np.array([1, 0, 0, 0], dtype=F32), (n, 1))
    scale = np.full((n, 3), 0.03, dtype=F32)
    opacity = np.zeros((n, 1), dtype=F32)
    sh = np.ones((n, 48), dtype=F32)
    return xyz, rot, scale, opacity, sh
