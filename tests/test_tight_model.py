"""CPU: the brute force behind tight binning (DESIGN.md decision 11), committed.

Tight binning (include/gsr.h GSR_OPT_TIGHT_BINNING) pairs a Gaussian only with the tiles of its
getRect rect that its alpha >= 1/255 ellipse reaches (preprocess.hip cull_data + col_spans).
Upstream's renderCUDA skips a splat at a pixel where power > 0 or alpha < 1/255 (oracle_render;
twin shaders/gau_frag.glsl:21-27), so a dropped tile must be skipped at all 256 of its pixel
centres.  oracle/tight_check.c restates the HIP predicate in C (correctly rounded where the
kernel uses v_log / v_rcp / v_sqrt) and checks every tile it drops at every pixel centre, on the
oracle's own preprocess outputs for:
  - the C3 and c3r scenes (1M Gaussians, 1080p) -- the headline frames;
  - the stress scenes of tests/tight_scenes.py (near-singular conics, opacity at 1/255, huge
    off-centre splats clipped to <= 8 columns, rects of 7-10 columns);
  - a direct fuzz of upstream's 2D stage (tight_scenes.conics_2d).
Bar: no dropped tile reaches alpha >= 1/255 anywhere.  The mutation check shows the brute force
has teeth: the predicate without its margins and with its log-threshold 0.5 % low is caught.
The device lists themselves are pinned against the oracle's in tests/test_gpu_tight_pin.py.
"""
import numpy as np
import pytest

from gaussiansplattingviewer_amd.camera import static_camera
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians

import tight_scenes
from gpu_helpers import scene_inputs


def _preprocess(oracle_mod, s):
    g = s["g"]
    return oracle_mod.forward(g.xyz, g.opacity, s["view"], s["proj"], s["campos"], s["tx"],
                              s["ty"], s["W"], s["H"], shs=g.sh, sh_degree=s["sh_degree"],
                              scales=g.scale, rotations=g.rot, stages="preprocess")


def _check(oracle_mod, o, W, H, min_dropped):
    st = oracle_mod.tight_model_check(o["means2D"], o["conic_opacity"], o["radii"], W, H)
    assert st["dropped_reaching"] == 0, st
    assert st["dropped"] >= min_dropped, st
    # the closest call: a dropped tile's largest alpha stays below the 1/255 threshold
    assert st["max_dropped_alpha_e9"] < 1e9 / 255.0, st
    return st


@pytest.mark.parametrize("name", ["c3", "c3r"])
def test_headline_frames(oracle_mod, name):
    g = synthetic_gaussians(1_000_000, 3, 2) if name == "c3" else clustered_scene(1_000_000, 7)
    s = scene_inputs(g, static_camera(1920, 1080), 3)
    st = _check(oracle_mod, _preprocess(oracle_mod, s), 1920, 1080, 2_000_000)
    assert st["span_coded"] > 500_000


@pytest.mark.parametrize("kind", tight_scenes.KINDS)
def test_stress_scenes(oracle_mod, kind):
    g, cam = tight_scenes.scene(kind, 100_000, 5)
    s = scene_inputs(g, cam, 3)
    st = _check(oracle_mod, _preprocess(oracle_mod, s), cam.w, cam.h, 100_000)
    if kind in ("rect_limits", "off_centre"):
        assert st["eight_columns"] > 1000 and st["too_large"] > 1000, st  # both sides of the limit


@pytest.mark.parametrize("seed", [3, 4])
def test_fuzzed_2d_splats(oracle_mod, seed):
    m, co, r = tight_scenes.conics_2d(400_000, seed)
    _check(oracle_mod, dict(means2D=m, conic_opacity=co, radii=r), tight_scenes.W, tight_scenes.H,
           500_000)


def test_mutation_is_caught(oracle_mod):
    """Without its margins and with L 0.5 % low, the predicate drops tiles the splat reaches --
    and the brute force finds them."""
    m, co, r = tight_scenes.conics_2d(400_000, 3)
    st = oracle_mod.tight_model_check(m, co, r, tight_scenes.W, tight_scenes.H, shrink=5e-3)
    assert st["dropped_reaching"] > 10, st


def test_subsequence_checker_catches_reordering_and_reaching_drops(oracle_mod):
    """oracle_check_tight itself: a list out of order, a pair not in upstream's list, and a
    dropped pair that reaches its tile are each reported."""
    means = np.array([[8.0, 8.0], [100.0, 100.0], [8.0, 8.0]], np.float32)
    co = np.array([[0.1, 0.0, 0.1, 0.9], [0.1, 0.0, 0.1, 0.9], [0.1, 0.0, 0.1, 0.9]], np.float32)
    full_r = np.array([[0, 3]], np.uint32)
    full = np.array([0, 1, 2], np.uint32)
    ok = oracle_mod.check_tight(1, 1, full_r, full, np.array([[0, 2]], np.uint32),
                                np.array([0, 2], np.uint32), means, co)
    assert ok["not_subsequence"] == 0 and ok["dropped"] == 1 and ok["dropped_reaching"] == 0
    swapped = oracle_mod.check_tight(1, 1, full_r, full, np.array([[0, 2]], np.uint32),
                                     np.array([2, 0], np.uint32), means, co)
    assert swapped["not_subsequence"] == 1
    reach = oracle_mod.check_tight(1, 1, full_r, full, np.array([[0, 1]], np.uint32),
                                   np.array([1], np.uint32), means, co)
    assert reach["dropped_reaching"] == 2 and reach["first_tile"] == 0
