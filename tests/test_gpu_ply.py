"""GPU: the PLY reader's direct device upload equals its host load, and a scene loaded from
PLY renders exactly as the same Gaussians uploaded from host arrays."""
import numpy as np
import pytest
import torch

import ply_oracle
from gaussiansplattingviewer_amd import ply
from gaussiansplattingviewer_amd.camera import static_camera
from gaussiansplattingviewer_amd.renderer import HIPRenderer, gaus_hip_from_cpu

pytestmark = pytest.mark.gpu


def _raw(P, seed):
    rng = np.random.default_rng(seed)
    v = {"x": rng.uniform(-2, 2, P), "y": rng.uniform(-2, 2, P), "z": rng.uniform(-2, 2, P)}
    for c in range(3):
        v[f"f_dc_{c}"] = rng.normal(0, 0.6, P)
    for i in range(45):
        v[f"f_rest_{i}"] = rng.normal(0, 0.05, P)
    v["opacity"] = rng.normal(0, 1.5, P)
    for i in range(3):
        v[f"scale_{i}"] = rng.uniform(-5.5, -3.5, P)
    for i in range(4):
        v[f"rot_{i}"] = rng.normal(0, 1, P)
    return {k: np.asarray(a, np.float32) for k, a in v.items()}


@pytest.mark.parametrize("P,fmt,types", [
    (600_000, "binary_little_endian", None),          # pipelined upload: 3 chunks, ragged tail
    (70_000, "binary_big_endian", None),
    (30_000, "binary_little_endian", {"x": "double", "y": "double", "z": "double"}),
    (5_000, "ascii", None),                           # host conversion, then upload
])
def test_device_load_equals_host_load(tmp_path, gpu, P, fmt, types):
    path = tmp_path / "scene.ply"
    raw = _raw(P, 12)
    if types:
        raw = {k: (v.astype(np.float64) if k in types else v) for k, v in raw.items()}
    ply_oracle.write_ply(path, raw, fmt=fmt, types=types)
    host, bbox_h, center_h = ply.load_ply(str(path))
    dev, bbox_d, center_d = ply.load_ply(str(path), device=gpu)
    torch.cuda.synchronize()
    for name in ("xyz", "rot", "scale", "opacity"):
        np.testing.assert_array_equal(getattr(dev, name).cpu().numpy(), getattr(host, name))
    np.testing.assert_array_equal(dev.sh.cpu().numpy().reshape(-1, 48), host.sh)
    np.testing.assert_array_equal(bbox_d, bbox_h)
    np.testing.assert_array_equal(center_d, center_h)


def test_device_load_equals_host_load_and_renders(tmp_path, gpu):
    path = tmp_path / "scene.ply"
    ply_oracle.write_ply(path, _raw(200_000, 11))
    host, bbox_h, center_h = ply.load_ply(str(path))
    dev, bbox_d, center_d = ply.load_ply(str(path), device=gpu)
    torch.cuda.synchronize()
    for name in ("xyz", "rot", "scale", "opacity"):
        np.testing.assert_array_equal(getattr(dev, name).cpu().numpy(), getattr(host, name))
    np.testing.assert_array_equal(dev.sh.cpu().numpy().reshape(-1, 48), host.sh)
    np.testing.assert_array_equal(bbox_d, bbox_h)
    np.testing.assert_array_equal(center_d, center_h)

    cam = static_camera(640, 480)
    r1 = HIPRenderer(640, 480, device=gpu)
    r1.update_gaussian_data(dev)
    r1.update_camera_intrin(cam)
    r1.update_camera_pose(cam)
    img1 = r1.draw().clone()
    r2 = HIPRenderer(640, 480, device=gpu)
    r2.update_gaussian_data(host)
    r2.update_camera_intrin(cam)
    r2.update_camera_pose(cam)
    img2 = r2.draw()
    assert float(img1.abs().sum()) > 0
    torch.testing.assert_close(img1, img2, rtol=0, atol=0)
