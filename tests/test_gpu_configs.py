"""GPU parity at the two BASELINE configs the other suites do not reach at full size.

C5 (BASELINE.json configs[4]): 1M Gaussians, SH3, 1920x1080, orbit camera with a per-frame
re-sort.  Four frames of the 1000-frame orbit (i = 0, 250, 500, 750; SURVEY.md §8(d), cf.
main_test.py:392-426) are rendered through `FramePipeline` -- the two-frames-in-flight path the
bench times -- and each is checked against the oracle with the full parity bar (integer outputs,
sort order and tile ranges bit-exact; image within the SURVEY.md §8(c) tolerance).

C4 (configs[3]): 6M Gaussians, SH3, 3840x2160 -- ~178M (Gaussian, tile) pairs, a 47-bit
upstream sort key, 135 tile rows (8 bits of packed row), a 32.8k-cell difference array.  The
full frame on one GPU is checked against the oracle, and every strip of the 8-GPU partition
(rendered here one after another on one device, as each rank of `bench.py --gpus 8` renders
it) is checked bit-identical to the same rows of the full frame, with its point list equal to
the full frame's pairs of those tile rows.  The oracle frame takes ~50 s on one host core.
"""
import numpy as np
import pytest
import torch

from gaussiansplattingviewer_amd.camera import orbit_eye, static_camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians
from gaussiansplattingviewer_amd.pipeline import FramePipeline
from gaussiansplattingviewer_amd.rasterizer import binning_state
from gaussiansplattingviewer_amd.strips import strip_pixel_rows, strip_rows

from gpu_helpers import (ALL_EXTRAS, assert_parity, run_hip, run_oracle, scene_inputs,
                         tight_binning, to_dev)
from gaussiansplattingviewer_amd.rasterizer import rasterize_gaussians_native

pytestmark = pytest.mark.gpu

C5_FRAMES = (0, 250, 500, 750)


@pytest.fixture(scope="module")
def c5_scene():
    return synthetic_gaussians(1_000_000, 3, 2)


def _collect(res, dev, slot):
    out = {"num_rendered": res.num_rendered, "color": res.color.cpu().numpy(),
           "radii": res.radii.cpu().numpy()}
    for k, v in res.extras.items():
        out[k] = v.cpu().numpy()
    out["tiles_touched"] = out["tiles_touched"].view(np.uint32)
    out["n_contrib"] = out["n_contrib"].view(np.uint32)
    pl, pt, rg = binning_state(dev.index or 0, slot=slot)
    out["point_list"] = pl.cpu().numpy().view(np.uint32)
    out["point_tiles"] = pt.cpu().numpy().view(np.uint32)
    out["ranges"] = rg.cpu().numpy().view(np.uint32)
    return out


@pytest.mark.parametrize("depth", [2, 4])
def test_c5_orbit_frames_through_pipeline(gpu, oracle_mod, c5_scene, depth):
    """C5 frames through FramePipeline: depth 4 is the bench's timed mode (four frames in
    flight, one stream each).  Each frame is rendered twice on its slot: as the viewer calls it
    (no per-Gaussian extras: tight binning, the paired-slot blend) and with every extra, which
    is checked against the oracle; the viewer call's image is bit-identical to the extras
    call's and within the image tolerance of the oracle's."""
    g = c5_scene
    P = len(g.xyz)
    dg = dict(xyz=to_dev(g.xyz, gpu), rot=to_dev(g.rot, gpu), scale=to_dev(g.scale, gpu),
              opacity=to_dev(g.opacity, gpu),
              sh=to_dev(g.sh, gpu).reshape(P, -1, 3).contiguous())
    Ks = []
    with FramePipeline(depth, gpu) as pipe:
        assert pipe.second_stream == (depth < 3)
        for i in C5_FRAMES:
            s = scene_inputs(g, static_camera(1920, 1080, orbit_eye(i, 1000)), 3)
            args = (to_dev(s["bg"], gpu), dg["xyz"], None, dg["opacity"], dg["scale"], dg["rot"],
                    1.0, None, to_dev(s["view"], gpu), to_dev(s["proj"], gpu), s["tx"], s["ty"],
                    s["H"], s["W"], dg["sh"], 3, to_dev(s["campos"], gpu), False, False)
            with pipe.frame() as slot:
                viewer = rasterize_gaussians_native(*args, slot=slot)
                res = rasterize_gaussians_native(*args, slot=slot, extras=ALL_EXTRAS)
                hip = _collect(res, gpu, slot)
            orc = run_oracle(oracle_mod, s)
            assert orc["num_rendered"] > 5_000_000, (i, orc["num_rendered"])
            assert_parity(hip, orc)
            assert viewer.num_rendered == hip["num_rendered"]
            np.testing.assert_array_equal(viewer.color.cpu().numpy().view(np.uint32),
                                          hip["color"].view(np.uint32))
            Ks.append(hip["num_rendered"])
    assert len(set(Ks)) == len(Ks)  # the camera really moved (different binning per frame)


@pytest.fixture(scope="module")
def c4(oracle_mod):
    """6M Gaussians, 3840x2160, static camera (seed 3): inputs and the oracle frame."""
    s = scene_inputs(synthetic_gaussians(6_000_000, 3, 3), static_camera(3840, 2160), 3)
    return s, run_oracle(oracle_mod, s)


@pytest.fixture(scope="module")
def c4_hip(gpu, c4):
    s, _ = c4
    out = run_hip(s, gpu)
    torch.cuda.empty_cache()
    return out


def test_c4_full_frame_vs_oracle(c4, c4_hip):
    s, orc = c4
    assert orc["num_rendered"] > 100_000_000
    # the regimes this config exists for: > 2^27 pairs, 47-bit upstream keys, 8-bit rows
    assert int(orc["point_keys"][-1] >> np.uint64(32)) > 2 ** 14
    assert_parity(c4_hip, orc)


@pytest.mark.parametrize("rank", range(8))
def test_c4_strips_equal_full_frame_rows(gpu, c4, c4_hip, rank):
    s, _ = c4
    full = c4_hip
    W, H = s["W"], s["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    rows = strip_rows(gy, 8, rank)
    part = run_hip(s, gpu, tile_rows=rows)
    y0, n = strip_pixel_rows(rows, H)
    np.testing.assert_array_equal(part["color"].view(np.uint32),
                                  full["color"][:, y0:y0 + n].view(np.uint32))
    np.testing.assert_array_equal(part["n_contrib"], full["n_contrib"][y0:y0 + n])
    np.testing.assert_array_equal(part["final_T"].view(np.uint32),
                                  full["final_T"][y0:y0 + n].view(np.uint32))
    np.testing.assert_array_equal(part["radii"], full["radii"])
    t0, t1 = rows[0] * gx, rows[1] * gx
    lo = int(np.searchsorted(full["point_tiles"], t0))
    hi = int(np.searchsorted(full["point_tiles"], t1))
    assert part["num_rendered"] == hi - lo
    np.testing.assert_array_equal(part["point_list"], full["point_list"][lo:hi])
    np.testing.assert_array_equal(part["point_tiles"], full["point_tiles"][lo:hi])
    nonempty = full["ranges"][t0:t1, 1] > full["ranges"][t0:t1, 0]
    np.testing.assert_array_equal(part["ranges"][t0:t1][nonempty],
                                  full["ranges"][t0:t1][nonempty] - lo)


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_c4_strips_without_radii(gpu, c4, c4_hip, rank):
    """A strip rank without the radii output (gsr_outputs.radii NULL, the multi-GPU bench's
    call) skips the Gaussians whose footprint bound misses its strip -- here with the C4 strips'
    compaction and colour-id path: image and binning stay bit-identical to the full frame."""
    s, _ = c4
    full = c4_hip
    W, H = s["W"], s["H"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    rows = strip_rows(gy, 8, rank)
    part = run_hip(s, gpu, tile_rows=rows, extras=("final_T", "n_contrib"), radii=False)
    assert part["radii"] is None
    y0, n = strip_pixel_rows(rows, H)
    np.testing.assert_array_equal(part["color"].view(np.uint32),
                                  full["color"][:, y0:y0 + n].view(np.uint32))
    np.testing.assert_array_equal(part["n_contrib"], full["n_contrib"][y0:y0 + n])
    t0, t1 = rows[0] * gx, rows[1] * gx
    lo = int(np.searchsorted(full["point_tiles"], t0))
    hi = int(np.searchsorted(full["point_tiles"], t1))
    assert part["num_rendered"] == hi - lo
    np.testing.assert_array_equal(part["point_list"], full["point_list"][lo:hi])


# ---- C3 with a capture-like scene (gaussian_data.clustered_scene) ----------------------------
# BASELINE configs[2] quotes "bicycle PLY scale"; no PLY exists offline, so this scene stands in
# for one: clustered centres, a ground plane under and behind the camera, a far background
# shell, floaters in front of the lens.  Depths span ~0.25..44 (D = 31 key bits: all three
# depth-sort passes), tile rows carry 4-5x different pair counts, tile lists reach ~4k splats.

@pytest.fixture(scope="module")
def c3r(oracle_mod):
    from gaussiansplattingviewer_amd.gaussian_data import clustered_scene
    s = scene_inputs(clustered_scene(1_000_000, 7), static_camera(1920, 1080), 3)
    return s, run_oracle(oracle_mod, s)


@pytest.fixture(scope="module")
def c3r_hip(gpu, c3r):
    return run_hip(c3r[0], gpu)


def test_c3r_clustered_scene_vs_oracle(c3r, c3r_hip):
    s, orc = c3r
    d = orc["depths"][orc["radii"] > 0]
    keys = d.view(np.uint32)
    assert int(np.bitwise_or.reduce(keys) ^ np.bitwise_and.reduce(keys)).bit_length() > 24
    assert d.max() / d.min() > 32  # >= 5 float exponents
    assert_parity(c3r_hip, orc)


def test_c3r_balanced_strips_bit_identical(gpu, c3r, c3r_hip):
    """The 8-GPU strips of this scene, split by strips.StripBalancer's rule from the frame's own
    per-row pair counts (gsr_tile_row_pairs): the heaviest strip carries fewer pairs than in the
    equal split, and every strip is bit-identical to the same rows of the full frame."""
    from gaussiansplattingviewer_amd.rasterizer import tile_row_pairs
    from gaussiansplattingviewer_amd.strips import balanced_layout, strip_layout
    s, _ = c3r
    full = c3r_hip
    W, H = s["W"], s["H"]
    gy, gx = (H + 15) // 16, (W + 15) // 16
    with tight_binning(gpu, 0):  # the context's last forward: the full frame, upstream's lists
        run_hip(s, gpu, binning=False, extras=())
    rp = tile_row_pairs(gy).cpu().numpy().view(np.uint32).astype(np.int64)
    rg = full["ranges"].astype(np.int64).reshape(gy, gx, 2)
    np.testing.assert_array_equal(rp, (rg[..., 1] - rg[..., 0]).sum(axis=1))
    layout = balanced_layout(rp + 64 * gx, 8)
    loads = [int(rp[b:e].sum()) for b, e in layout]
    equal = [int(rp[b:e].sum()) for b, e in strip_layout(gy, 8)]
    assert max(loads) < 0.9 * max(equal), (loads, equal)
    for rows in layout:
        part = run_hip(s, gpu, tile_rows=rows, binning=False)
        y0, n = strip_pixel_rows(rows, H)
        np.testing.assert_array_equal(part["color"].view(np.uint32),
                                      full["color"][:, y0:y0 + n].view(np.uint32))
        np.testing.assert_array_equal(part["n_contrib"], full["n_contrib"][y0:y0 + n])
        # the bench's strip call: no radii, Gaussians that miss the strip skipped (near
        # floaters, the ground plane and the background shell stress the footprint bound)
        lean = run_hip(s, gpu, tile_rows=rows, extras=("final_T", "n_contrib"), radii=False)
        np.testing.assert_array_equal(lean["color"].view(np.uint32),
                                      part["color"].view(np.uint32))
        np.testing.assert_array_equal(lean["n_contrib"], part["n_contrib"])
        assert lean["num_rendered"] == part["num_rendered"]
