"""GPU: the tight tile lists themselves, pinned against the oracle's (upstream's) lists.

The default forward (no n_contrib output) bins tightly (include/gsr.h GSR_OPT_TIGHT_BINNING):
each Gaussian is paired only with the tiles its alpha >= 1/255 ellipse reaches, where upstream's
duplicateWithKeys (reached via renderer_cuda.py:211-224) pairs it with every tile of its getRect
rect and its renderCUDA then skips it wherever alpha < 1/255.  gsr_get_binning exports the lists
the blend read; for every tile, oracle/tight_check.c checks
  - the tight list is an in-order subsequence of the oracle's list (so every pixel composites
    the kept splats in upstream's order), and
  - every pair it dropped is skipped at all 256 pixel centres of the tile in the oracle's
    arithmetic (power > 0 or alpha < 1/255): it could not have changed any pixel.
Scenes: C3 and c3r at full size, the stress scenes of tests/tight_scenes.py (near-singular
conics, opacity at 1/255, huge off-centre splats clipped to <= 8 columns, rects of 7-10
columns).  The 18 reference viewer poses get the same check in test_gpu_viewer_poses.py.
"""
import numpy as np
import pytest

from gaussiansplattingviewer_amd.camera import static_camera
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians

import tight_scenes
from gpu_helpers import run_hip, run_oracle, scene_inputs

pytestmark = pytest.mark.gpu


def pin_tight_lists(oracle_mod, orc, hip, W, H):
    """The check above for one frame: orc = the oracle's binning (stages "bin"), hip = a tight
    forward's exported lists (run_hip without n_contrib).  Returns the check's statistics."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    if hip["num_rendered"] is not None:  # (the viewer's draw does not return it)
        assert hip["num_rendered"] == orc["num_rendered"]  # num_rendered stays upstream's K
    np.testing.assert_array_equal(hip["radii"], orc["radii"])
    st = oracle_mod.check_tight(gx, gy, orc["ranges"], orc["point_list"], hip["ranges"],
                                hip["point_list"], orc["means2D"], orc["conic_opacity"])
    assert st["not_subsequence"] == 0 and st["dropped_reaching"] == 0, st
    assert st["kept"] == len(hip["point_list"]) and st["kept"] + st["dropped"] == orc["num_rendered"]
    # the exported tile ids agree with the exported ranges
    rg = hip["ranges"].reshape(-1, 2).astype(np.int64)
    tiles = np.repeat(np.arange(gx * gy), rg[:, 1] - rg[:, 0])
    np.testing.assert_array_equal(hip["point_tiles"], tiles)
    return st


def _run(gpu, oracle_mod, s):
    orc = run_oracle(oracle_mod, s, stages="bin")
    hip = run_hip(s, gpu, extras=())
    return pin_tight_lists(oracle_mod, orc, hip, s["W"], s["H"])


@pytest.mark.parametrize("name", ["c3", "c3r"])
def test_headline_frames(gpu, oracle_mod, name):
    g = synthetic_gaussians(1_000_000, 3, 2) if name == "c3" else clustered_scene(1_000_000, 7)
    st = _run(gpu, oracle_mod, scene_inputs(g, static_camera(1920, 1080), 3))
    assert st["dropped"] > 0.25 * (st["kept"] + st["dropped"]), st  # tight binning is on


@pytest.mark.parametrize("kind", tight_scenes.KINDS)
def test_stress_scenes(gpu, oracle_mod, kind):
    g, cam = tight_scenes.scene(kind, 100_000, 5)
    st = _run(gpu, oracle_mod, scene_inputs(g, cam, 3))
    assert st["dropped"] > 50_000, st
