"""CPU: pin the oracle against vectors captured from the reference (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from gaussiansplattingviewer_amd.camera import Camera, cuda_camera_inputs, static_camera
from gaussiansplattingviewer_amd.gaussian_data import naive_gaussian, synthetic_gaussians

SORT_CASES = ["10k_front", "10k_oblique", "10k_viewer_default", "100k_front", "ties_front"]


def _xyz(g, case):
    return g["xyz_" + case.split("_")[0]]


@pytest.mark.parametrize("case", SORT_CASES)
def test_view_depth_bit_exact_vs_reference(golden, oracle_mod, case):
    g = golden("sort_backend.npz")
    d = oracle_mod.view_depth(_xyz(g, case), g[case + "__view"])
    ref = g[case + "__depth"]
    assert d.dtype == np.float32
    np.testing.assert_array_equal(d.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("case", SORT_CASES)
def test_stable_argsort_and_reference_order(golden, oracle_mod, case):
    """The reference uses np.argsort's default (unstable) kind: its order must equal the
    stable order on the sorted depth sequence and everywhere outside tie groups."""
    g = golden("sort_backend.npz")
    depth = g[case + "__depth"]
    ref_idx = g[case + "__index"][:, 0]
    ours = oracle_mod.argsort_stable(depth)
    np.testing.assert_array_equal(ours, np.argsort(depth, kind="stable"))
    np.testing.assert_array_equal(depth[ours], depth[ref_idx])
    ds = depth[ours]
    tie = np.zeros(len(ds), bool)
    eq = ds[1:] == ds[:-1]
    tie[1:] |= eq
    tie[:-1] |= eq
    np.testing.assert_array_equal(ours[~tie], ref_idx[~tie])


@pytest.mark.parametrize("case", SORT_CASES)
def test_cpu_baseline_restatement_matches_reference(golden, oracle_mod, case):
    g = golden("sort_backend.npz")
    idx = oracle_mod.sort_gaussian_cpu(_xyz(g, case), g[case + "__view"])
    assert idx.dtype == np.int32 and idx.shape == (len(_xyz(g, case)), 1)
    np.testing.assert_array_equal(idx, g[case + "__index"])


@pytest.mark.parametrize("wh", ["640x480", "1920x1080", "3840x2160", "1160x522"])
def test_camera_matches_reference(golden, wh):
    g = golden("camera.npz")
    w, h = map(int, wh.split("x"))
    cam = Camera(h, w)
    np.testing.assert_array_equal(cam.get_project_matrix(), g[wh + "__proj"])
    np.testing.assert_array_equal(np.array(cam.get_htanfovxy_focal()), g[wh + "__htanfovxy_focal"])
    assert cam.fovy == float(g[wh + "__fovy"])


def test_naive_gaussian_matches_reference(golden):
    g = golden("naive_gaussian.npz")
    ours = naive_gaussian()
    for k in ("xyz", "rot", "scale", "opacity", "sh"):
        np.testing.assert_array_equal(getattr(ours, k), g[k])
    np.testing.assert_array_equal(ours.flat(), g["flat"])


def test_oracle_c1_regression(golden, oracle_mod):
    """Regression pin of the restatement at config C1 (10k, 640x480, SH3, seed 0)."""
    ref = golden("oracle_c1.npz")
    gs = synthetic_gaussians(10_000, 3, seed=0)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(640, 480))
    r = oracle_mod.forward(gs.xyz, gs.opacity, view, proj, campos, tx, ty, 640, 480, shs=gs.sh,
                           sh_degree=3, scales=gs.scale, rotations=gs.rot)
    assert r["num_rendered"] == int(ref["num_rendered"])
    for k in ("radii", "tiles_touched", "point_list", "point_keys", "ranges", "n_contrib"):
        np.testing.assert_array_equal(r[k], ref[k])
    assert abs(r["color"].astype(np.float64).sum() - float(ref["color_sum"])) < 1e-3
