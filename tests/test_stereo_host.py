"""Host side of the stereo rows on CPU: the restated disparity / packers against closed forms,
and the device-only entry points refusing host tensors (there is no CPU path)."""
import numpy as np
import pytest
import torch

import stereo_oracle
from gaussiansplattingviewer_amd import colmap
from gaussiansplattingviewer_amd.camera import Camera


def test_disparity_closed_form():
    # identity-rotation view: ndc_x shifts by P00 * b / (-z_view), d = |shift| / 2
    left, _ = colmap.load_camera_positions(["1", "1", "0", "0", "0", "0", "0", "4", "1", "a"])
    cam = Camera(522, 1160)
    proj = cam.get_project_matrix()
    rng = np.random.default_rng(3)
    xyz = rng.uniform(-2, 2, size=(1000, 3)).astype(np.float32)
    d = stereo_oracle.disparity_f32(xyz, left["camera_view"], proj)
    zv = (left["camera_view"].astype(np.float64) @ np.c_[xyz, np.ones(1000)].T)[2]
    want = np.abs(proj[0, 0] * 0.5 / zv) / 2
    np.testing.assert_allclose(d, want, rtol=2e-5, atol=1e-6)


def test_pack_reference_values():
    img = np.zeros((3, 2, 4), np.float32)
    img[0, 0] = [0.0, 1.0, 0.5, -1.0]
    img[0, 1] = [2.0, 1.0 / 65535 * 3, np.nan, 0.25]
    rgb = stereo_oracle.pack_f32(img, "rgb8")
    assert rgb.shape == (2, 4, 3) and rgb.dtype == np.uint8
    np.testing.assert_array_equal(rgb[0, :, 0], [0, 255, 128, 0])
    np.testing.assert_array_equal(rgb[1, :, 0], [255, 0, 0, 64])
    r16 = stereo_oracle.pack_f32(img, "r16")
    np.testing.assert_array_equal(r16[0], [0, 65535, 32767, 0xFFFF & -65535])
    assert r16[1, 0] == (131070 & 0xFFFF) and r16[1, 2] == 0  # wrap; NaN -> 0
    np.testing.assert_array_equal(stereo_oracle.pack_f32(img, "r16", True), r16[::-1])
    rgba = stereo_oracle.pack_f32(img, "rgba_f32")
    assert rgba.shape == (2, 4, 4) and (rgba[..., 3] == 1).all()


def test_device_entry_points_refuse_host_tensors():
    from gaussiansplattingviewer_amd.stereo import disparity_colors, pack_image
    with pytest.raises(RuntimeError):
        disparity_colors(torch.zeros(4, 3), np.eye(4), np.eye(4))
    with pytest.raises(RuntimeError):
        pack_image(torch.zeros(3, 4, 4), "rgb8")
    with pytest.raises(ValueError):
        pack_image(torch.zeros(3, 4, 4), "bgr8")
