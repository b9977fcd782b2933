"""GPU: tight binning (GSR_OPT_TIGHT_BINNING, the default for every forward without n_contrib)
renders the same bits as upstream's full 3-sigma lists.

Tight binning pairs a Gaussian only with the tiles its alpha >= 1/255 ellipse reaches (per-column
tile-row spans, preprocess.hip col_spans); upstream's blend skips it on the others (`alpha <
1/255: continue`), so each tile list is a subsequence of upstream's holding every splat that can
change a pixel of the tile, in upstream's order.  Bar: color and final_T bit-identical to the
full lists' forward (which the parity suite pins against the oracle), in both blend arithmetic
modes, with and without the blend's quadrant cull, on strips, and num_rendered unchanged.
"""
import ctypes

import numpy as np
import pytest

from gaussiansplattingviewer_amd import _lib
from gaussiansplattingviewer_amd.camera import static_camera
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians
from gaussiansplattingviewer_amd.rasterizer import tile_row_pairs

from gpu_helpers import run_hip, scene_inputs, set_option, tight_binning

pytestmark = pytest.mark.gpu

TIGHT = ("final_T",)               # no n_contrib: tight binning
FULL = ("final_T", "n_contrib")    # n_contrib: upstream's lists


def _scene(name):
    if name == "dense_720p":
        return scene_inputs(synthetic_gaussians(200_000, 3, 17), static_camera(1280, 720), 3)
    if name == "elongated_close":  # strongly anisotropic splats seen up close
        g = synthetic_gaussians(20_000, 3, 20)
        rng = np.random.default_rng(20)
        g.scale[:] = np.exp(rng.uniform(-7.0, -1.5, g.scale.shape)).astype(np.float32)
        return scene_inputs(g, static_camera(960, 540, (0.2, 0.1, 1.2)), 3)
    if name == "needles":  # one long axis: thin diagonal ellipses across several tile columns
        g = synthetic_gaussians(30_000, 3, 31)
        rng = np.random.default_rng(31)
        g.scale[:] = np.float32(0.002)
        g.scale[:, 0] = rng.uniform(0.02, 0.08, len(g.scale)).astype(np.float32)
        return scene_inputs(g, static_camera(1024, 768), 3)
    if name == "huge_and_faint":  # rects past the span code (w > 8) and opacities near 1/255
        g = synthetic_gaussians(3_000, 3, 32)
        rng = np.random.default_rng(32)
        g.scale[:] = rng.uniform(0.01, 0.4, g.scale.shape).astype(np.float32)
        g.opacity[:] = rng.uniform(0.0, 0.02, g.opacity.shape).astype(np.float32)
        g.opacity[::3] = np.float32(0.999)
        return scene_inputs(g, static_camera(800, 600, (0.0, 0.0, 2.5)), 3)
    if name == "clustered_300k":  # the capture-like generator (c3r) at a third of its size
        return scene_inputs(clustered_scene(300_000, 7), static_camera(1920, 1080), 3)
    if name == "oblique_inside":
        return scene_inputs(synthetic_gaussians(40_000, 3, 5), static_camera(1160, 522, (0.3, -0.2, 0.5)), 3)
    raise KeyError(name)


SCENES = ["dense_720p", "elongated_close", "needles", "huge_and_faint", "clustered_300k",
          "oblique_inside"]


def _same(a, b, keys=("color", "final_T")):
    for k in keys:
        np.testing.assert_array_equal(a[k].view(np.uint32), b[k].view(np.uint32), err_msg=k)
    assert a["num_rendered"] == b["num_rendered"]


@pytest.mark.parametrize("scene", SCENES)
def test_tight_equals_full_lists(gpu, scene):
    s = _scene(scene)
    full = run_hip(s, gpu, extras=FULL, binning=False)
    tight = run_hip(s, gpu, extras=TIGHT, binning=False)
    assert full["num_rendered"] > 0
    _same(tight, full)
    np.testing.assert_array_equal(tight["radii"], full["radii"])
    with tight_binning(gpu, 0):
        off = run_hip(s, gpu, extras=TIGHT, binning=False)
    _same(off, full)


@pytest.mark.parametrize("fast", [0, 1])
@pytest.mark.parametrize("cull", [0, 1])
@pytest.mark.parametrize("scene", ["elongated_close", "needles", "huge_and_faint"])
def test_tight_in_every_blend_mode(gpu, scene, fast, cull):
    """Tight binning does not lean on the blend's cull or on its arithmetic mode."""
    s = _scene(scene)
    set_option(gpu, _lib.GSR_OPT_BLEND_FAST, fast)
    set_option(gpu, _lib.GSR_OPT_BLEND_CULL, cull)
    try:
        full = run_hip(s, gpu, extras=FULL, binning=False)
        tight = run_hip(s, gpu, extras=TIGHT, binning=False)
    finally:
        set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 1)
        set_option(gpu, _lib.GSR_OPT_BLEND_CULL, 1)
    _same(tight, full)


def test_tight_lists_are_shorter_and_exported(gpu):
    s = _scene("dense_720p")
    gy = (s["H"] + 15) // 16
    with tight_binning(gpu, 0):
        run_hip(s, gpu, extras=(), binning=False)
        full_rows = tile_row_pairs(gy).cpu().numpy().view(np.uint32).astype(np.int64)
    res = run_hip(s, gpu, extras=(), binning=False)
    rows = tile_row_pairs(gy).cpu().numpy().view(np.uint32).astype(np.int64)
    assert full_rows.sum() == res["num_rendered"]  # upstream's K either way
    assert np.all(rows <= full_rows) and rows.sum() < 0.8 * full_rows.sum(), (rows.sum(), full_rows.sum())
    # gsr_get_binning exports the tight lists the blend read (their total, not upstream's K)
    lib = _lib.load_library()
    K = ctypes.c_int64()
    T = ctypes.c_int32()
    rc = lib.gsr_get_binning(_lib.context(gpu.index or 0), None, None, None, ctypes.byref(K),
                             ctypes.byref(T), None)
    assert rc == 0 and K.value == rows.sum() and T.value == gy * ((s["W"] + 15) // 16)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tight_strips_equal_full_frame_rows(gpu, world):
    from gaussiansplattingviewer_amd.strips import strip_layout, strip_pixel_rows
    s = _scene("clustered_300k")
    H = s["H"]
    full = run_hip(s, gpu, extras=FULL, binning=False)
    for rows in strip_layout((H + 15) // 16, world):
        y0, n = strip_pixel_rows(rows, H)
        for radii in (True, False):  # False: the bench's strip call
            part = run_hip(s, gpu, tile_rows=rows, extras=TIGHT, binning=False, radii=radii)
            np.testing.assert_array_equal(part["color"].view(np.uint32),
                                          full["color"][:, y0:y0 + n].view(np.uint32))
            np.testing.assert_array_equal(part["final_T"].view(np.uint32),
                                          full["final_T"][y0:y0 + n].view(np.uint32))
