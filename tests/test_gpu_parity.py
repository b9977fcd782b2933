"""GPU parity: the HIP rasterizer (libgsr.so through its C ABI) against the CPU oracle.

Bit-exact: radii, tiles_touched, depths, means2D, conic_opacity, rgb, num_rendered, the
sorted point list, its tile ids, and the tile ranges.  Image (color, final_T, n_contrib): the
tolerance in gpu_helpers.py -- the blend is the only stage that is not bit-exact (exp, and in
the default fast arithmetic the fused multiply-adds of the staged quadratic; see there).  The
viewer's own call requests no per-pixel extras, which selects the blend's paired-slot variant:
every forward case is also rendered that way and must be bit-identical to the frame rendered
with the extras."""
import numpy as np
import pytest
import torch

from gaussiansplattingviewer_amd import _lib
from gaussiansplattingviewer_amd.camera import Camera, static_camera
from gaussiansplattingviewer_amd.gaussian_data import (GaussianData, naive_gaussian,
                                                       synthetic_gaussians)

from gpu_helpers import (assert_image_close, assert_parity, run_hip, run_oracle, scene_inputs)

pytestmark = pytest.mark.gpu


def _set_option(dev, opt, value):
    lib = _lib.load_library()
    _lib.check(lib.gsr_set_option(_lib.context(dev.index or 0), opt, int(value)), "gsr_set_option")


def _set_cull(dev, on):
    _set_option(dev, _lib.GSR_OPT_BLEND_CULL, on)


@pytest.fixture
def exact_blend(gpu):
    """Upstream per-pixel operation order (GSR_OPT_BLEND_FAST = 0; the default is 1)."""
    _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 0)
    yield
    _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 1)


CASES = {
    # name: (P, W, H, sh_degree, seed, eye)
    "C1_10k_640x480_sh3": (10_000, 640, 480, 3, 0, (0.0, 0.0, 4.0)),
    "C2_100k_1080p_sh0": (100_000, 1920, 1080, 0, 1, (0.0, 0.0, 4.0)),
    "oblique_30k_800x600_sh3": (30_000, 800, 600, 3, 4, (2.5, 1.0, -3.0)),
    "inside_cloud_20k_1160x522_sh3": (20_000, 1160, 522, 3, 5, (0.3, -0.2, 0.5)),
    # image shapes that change the tile-sort plan: one tile (0 bits), one tile row, > 256
    # tile columns, a narrow ragged image
    "one_tile_5k_16x16_sh3": (5_000, 16, 16, 3, 6, (0.0, 0.0, 4.0)),
    "one_row_8k_1000x12_sh3": (8_000, 1000, 12, 3, 7, (0.0, 0.0, 4.0)),
    "wide_20k_4200x64_sh3": (20_000, 4200, 64, 3, 8, (0.0, 0.0, 4.0)),
    "narrow_10k_33x700_sh3": (10_000, 33, 700, 3, 9, (0.0, 0.0, 4.0)),
}


@pytest.mark.parametrize("name", list(CASES))
def test_forward_parity(gpu, oracle_mod, name):
    P, W, H, deg, seed, eye = CASES[name]
    s = scene_inputs(synthetic_gaussians(P, deg, seed), static_camera(W, H, eye), deg)
    orc = run_oracle(oracle_mod, s)
    hip = run_hip(s, gpu)
    assert orc["num_rendered"] > 0
    assert_parity(hip, orc)
    _assert_plain_call_identical(gpu, s, hip)


def _assert_plain_call_identical(gpu, s, hip):
    """The viewer's call (no extras: the blend's n_contrib-free, paired-slot variant) renders the
    same bits as the call with every extra output."""
    plain = run_hip(s, gpu, extras=(), binning=False)
    np.testing.assert_array_equal(plain["color"].view(np.uint32), hip["color"].view(np.uint32))
    np.testing.assert_array_equal(plain["radii"], hip["radii"])
    assert plain["num_rendered"] == hip["num_rendered"]


def test_naive_scene_viewer_window(gpu, oracle_mod):
    """The viewer's default 4-Gaussian scene (util_gau.py:25-60) in its 1160x522 window."""
    cam = Camera(522, 1160)
    cam.look_from((0.4, 0.3, 3.0))
    s = scene_inputs(naive_gaussian(), cam, 0)
    assert_parity(run_hip(s, gpu), run_oracle(oracle_mod, s))


@pytest.mark.parametrize("deg", [1, 2])
def test_lower_sh_degree_with_degree3_storage(gpu, oracle_mod, deg):
    s = scene_inputs(synthetic_gaussians(8000, 3, 12), static_camera(512, 384), deg)
    assert_parity(run_hip(s, gpu), run_oracle(oracle_mod, s))


def test_background_and_scale_modifier(gpu, oracle_mod):
    s = scene_inputs(synthetic_gaussians(15_000, 3, 13), static_camera(700, 500, (1, 1, 3.5)), 3,
                     bg=(0.25, 0.5, 1.0), scale_modifier=1.7)
    assert_parity(run_hip(s, gpu), run_oracle(oracle_mod, s))


def test_precomputed_colors_and_covariance(gpu, oracle_mod):
    g = synthetic_gaussians(6000, 0, 14)
    rng = np.random.default_rng(14)
    colors = rng.uniform(0, 1, (len(g), 3)).astype(np.float32)
    A = rng.normal(0, 0.03, (len(g), 3, 3))
    cov = np.einsum("pij,pkj->pik", A, A)
    cov6 = np.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2],
                     cov[:, 2, 2]], -1).astype(np.float32)
    s = scene_inputs(g, static_camera(480, 360), 0)
    orc = run_oracle(oracle_mod, s, colors_precomp=colors, cov3D_precomp=cov6)
    hip = run_hip(s, gpu, colors_precomp=colors, cov3D_precomp=cov6)
    orc["rgb"] = np.zeros_like(orc["rgb"])  # not computed on either side with precomp colors
    assert_parity(hip, orc)


def test_large_splats_many_tiles(gpu, oracle_mod):
    """A few huge Gaussians close to the camera: each touches most of the frame's tiles."""
    g = synthetic_gaussians(300, 3, 15)
    g.scale[:] = np.float32(0.4)
    s = scene_inputs(g, static_camera(640, 480, (0, 0, 2.2)), 3)
    orc = run_oracle(oracle_mod, s)
    assert orc["num_rendered"] > 300 * 100
    assert_parity(run_hip(s, gpu), orc)


def test_empty_and_fully_culled(gpu, oracle_mod):
    # P = 0: upstream returns a zero image (not the background)
    empty = GaussianData(*(np.zeros((0, k), np.float32) for k in (3, 4, 3, 1, 3)))
    s = scene_inputs(empty, static_camera(64, 48), 0, bg=(0.3, 0.3, 0.3))
    hip = run_hip(s, gpu, extras=(), binning=False)
    assert hip["num_rendered"] == 0 and hip["radii"].shape == (0,)
    assert np.all(hip["color"] == 0)
    # everything behind the camera: no pairs, background everywhere
    g = synthetic_gaussians(1000, 0, 16)
    g.xyz[:, 2] = g.xyz[:, 2] + 10.0
    s = scene_inputs(g, static_camera(100, 70), 0, bg=(0.1, 0.2, 0.3))
    orc = run_oracle(oracle_mod, s)
    hip = run_hip(s, gpu)
    assert orc["num_rendered"] == 0
    assert_parity(hip, orc)
    assert np.all(hip["color"][1] == np.float32(0.2))


@pytest.mark.parametrize("fast", [0, 1])
@pytest.mark.parametrize("scene", ["dense_720p", "elongated_close"])
def test_cull_is_exact(gpu, fast, scene):
    """The blend's ellipse-vs-quadrant cull changes nothing: bit-identical image either way,
    in both arithmetic modes, including strongly anisotropic splats seen up close."""
    if scene == "dense_720p":
        g = synthetic_gaussians(200_000, 3, 17)
        cam = static_camera(1280, 720)
    else:
        g = synthetic_gaussians(20_000, 3, 20)
        rng = np.random.default_rng(20)
        g.scale[:] = np.exp(rng.uniform(-7.0, -1.5, g.scale.shape)).astype(np.float32)
        cam = static_camera(960, 540, (0.2, 0.1, 1.2))
    s = scene_inputs(g, cam, 3)
    _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, fast)
    try:
        _set_cull(gpu, False)
        try:
            off = run_hip(s, gpu, binning=False)
        finally:
            _set_cull(gpu, True)
        on = run_hip(s, gpu, binning=False)
    finally:
        _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 1)
    for k in ("color", "final_T", "n_contrib"):
        np.testing.assert_array_equal(on[k].view(np.uint32), off[k].view(np.uint32), err_msg=k)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("name", ["C1_10k_640x480_sh3", "C2_100k_1080p_sh0",
                                  "inside_cloud_20k_1160x522_sh3"])
def test_blend_mode_parity(gpu, oracle_mod, name, mode):
    """Both blend arithmetic modes (GSR_OPT_BLEND_FAST: 0 = upstream operation order, 1 = fused):
    binning bit-exact, image within the tolerance."""
    P, W, H, deg, seed, eye = CASES[name]
    s = scene_inputs(synthetic_gaussians(P, deg, seed), static_camera(W, H, eye), deg)
    _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, mode)
    try:
        hip = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 1)
    assert_parity(hip, run_oracle(oracle_mod, s))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_strips_equal_full_frame_rows(gpu, world):
    """Each strip of the multi-GPU partition is bit-identical to the same rows of the 1-GPU
    frame (here rendered one strip after another on one device)."""
    from gaussiansplattingviewer_amd.strips import strip_pixel_rows, strip_rows
    W, H = 1920, 1080
    s = scene_inputs(synthetic_gaussians(150_000, 3, 18), static_camera(W, H), 3)
    full = run_hip(s, gpu)
    gy = (H + 15) // 16
    K_sum = 0
    for r in range(world):
        rows = strip_rows(gy, world, r)
        part = run_hip(s, gpu, tile_rows=rows)
        y0, n = strip_pixel_rows(rows, H)
        np.testing.assert_array_equal(part["color"].view(np.uint32),
                                      full["color"][:, y0:y0 + n].view(np.uint32))
        np.testing.assert_array_equal(part["n_contrib"], full["n_contrib"][y0:y0 + n])
        np.testing.assert_array_equal(part["radii"], full["radii"])
        t0, t1 = rows[0] * 120, rows[1] * 120
        before = int((full["point_tiles"] < t0).sum())
        nonempty = full["ranges"][t0:t1, 1] > full["ranges"][t0:t1, 0]
        np.testing.assert_array_equal(part["ranges"][t0:t1][nonempty],
                                      full["ranges"][t0:t1][nonempty] - before)
        assert np.all(part["ranges"][t0:t1][~nonempty] == 0)
        assert np.all(part["ranges"][:t0] == 0) and np.all(part["ranges"][t1:] == 0)
        sel = (full["point_tiles"] >= t0) & (full["point_tiles"] < t1)
        np.testing.assert_array_equal(part["point_list"], full["point_list"][sel])
        np.testing.assert_array_equal(part["point_tiles"], full["point_tiles"][sel])
        K_sum += part["num_rendered"]
        # without radii (a strip rank's call): Gaussians that miss the strip are skipped
        lean = run_hip(s, gpu, tile_rows=rows, extras=("final_T", "n_contrib"), radii=False)
        for k in ("color", "n_contrib", "final_T", "point_list", "ranges"):
            np.testing.assert_array_equal(lean[k], part[k], err_msg=k)
    assert K_sum == full["num_rendered"]


def test_cost_weighted_strips_on_a_crowded_scene(gpu):
    """Strips split by the blend work of a scene crowded into the upper left of the image
    (the pair counts per tile row from gsr_tile_row_pairs of the full frame, as
    strips.StripBalancer uses them): the per-row counts equal the full frame's ranges, the
    weighted split differs from the equal one, and every strip is bit-identical to the rows of
    the full frame."""
    import torch
    from gaussiansplattingviewer_amd.rasterizer import tile_row_pairs
    from gaussiansplattingviewer_amd.strips import (balanced_layout, strip_layout,
                                                    strip_pixel_rows)
    W, H, world = 1280, 720, 8
    g = synthetic_gaussians(200_000, 3, 25)
    rng = np.random.default_rng(25)
    crowd = rng.random(len(g.xyz)) < 0.8  # 80% of the splats in one corner
    g.xyz[crowd, 0] = g.xyz[crowd, 0] * np.float32(0.3) - np.float32(0.6)
    g.xyz[crowd, 1] = g.xyz[crowd, 1] * np.float32(0.3) + np.float32(0.5)
    s = scene_inputs(g, static_camera(W, H), 3)
    full = run_hip(s, gpu)
    gy, gx = (H + 15) // 16, (W + 15) // 16
    rp = tile_row_pairs(gy).cpu().numpy().view(np.uint32).astype(np.int64)
    rg = full["ranges"].astype(np.int64).reshape(gy, gx, 2)
    np.testing.assert_array_equal(rp, (rg[..., 1] - rg[..., 0]).sum(axis=1))
    layout = balanced_layout(rp + 64 * gx, world)
    assert layout != strip_layout(gy, world)
    loads = [int(rp[b:e].sum()) for b, e in layout]
    equal = [int(rp[b:e].sum()) for b, e in strip_layout(gy, world)]
    assert max(loads) < max(equal)
    for rows in layout:
        part = run_hip(s, gpu, tile_rows=rows, binning=False)
        y0, n = strip_pixel_rows(rows, H)
        np.testing.assert_array_equal(part["color"].view(np.uint32),
                                      full["color"][:, y0:y0 + n].view(np.uint32))
        np.testing.assert_array_equal(part["n_contrib"], full["n_contrib"][y0:y0 + n])
        sub = tile_row_pairs(rows[1] - rows[0]).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(sub, rp[rows[0]:rows[1]])


def test_debug_mode_and_repeatability(gpu):
    s = scene_inputs(synthetic_gaussians(50_000, 3, 19), static_camera(960, 540), 3)
    a = run_hip(s, gpu, debug=True)
    b = run_hip(s, gpu)
    for k in ("color", "point_list", "ranges", "radii"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.fixture(scope="module")
def c3_oracle(oracle_mod):
    s = scene_inputs(synthetic_gaussians(1_000_000, 3, 2), static_camera(1920, 1080), 3)
    return s, run_oracle(oracle_mod, s)


@pytest.mark.parametrize("fast", [0, 1])
def test_headline_config_c3(gpu, c3_oracle, fast):
    """Config C3 at full size: 1M Gaussians, 1920x1080, SH degree 3, static camera."""
    s, orc = c3_oracle
    _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, fast)
    try:
        hip = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_BLEND_FAST, 1)
    assert orc["num_rendered"] > 5_000_000
    assert_parity(hip, orc)
    if fast:
        _assert_plain_call_identical(gpu, s, hip)


VARIANTS = {  # [(option, alternative value, default), ...]
    "no_cull": [(_lib.GSR_OPT_BLEND_CULL, 0, 1)],
    "lsd_sort": [(_lib.GSR_OPT_DEPTH_SORT, 0, -1)],
    "compact_sort": [(_lib.GSR_OPT_DEPTH_SORT, 1, -1)],
    "msd_sort": [(_lib.GSR_OPT_DEPTH_SORT, 2, -1)],
    "compact_msd": [(_lib.GSR_OPT_DEPTH_SORT, 3, -1)],
}


class _options:
    """Set a VARIANTS entry's options for the duration of a with-block."""

    def __init__(self, gpu, opts):
        self.gpu, self.opts = gpu, opts

    def __enter__(self):
        for opt, val, _ in self.opts:
            _set_option(self.gpu, opt, val)

    def __exit__(self, *exc):
        for opt, _, default in self.opts:
            _set_option(self.gpu, opt, default)


@pytest.mark.parametrize("variant", list(VARIANTS))
@pytest.mark.parametrize("size", [(1920, 1080), (16, 16), (4200, 64)])
def test_sort_implementations_agree(gpu, variant, size):
    """The defaults (the blend's quadrant cull, the depth sort dropping the off-strip keys in
    its first pass) and the alternatives -- no cull, a compacting depth sort -- give identical
    binning and images.  Sizes: 1 tile (tbits = 0), a column-first frame and > 256 tile columns
    (the per-pair binning form, which api.hip picks for such frames)."""
    w, h = size
    P = 300_000 if w * h > 10_000 else 20_000
    s = scene_inputs(synthetic_gaussians(P, 3, 21), static_camera(w, h, (0.5, 0.2, 3.5)), 3)
    ref = run_hip(s, gpu)
    with _options(gpu, VARIANTS[variant]):
        alt = run_hip(s, gpu)
    assert ref["num_rendered"] > 0
    for k in ("point_list", "point_tiles", "ranges", "color", "n_contrib"):
        np.testing.assert_array_equal(alt[k], ref[k], err_msg=k)


@pytest.mark.parametrize("variant", ["default", "per_pair", "lsd_sort", "compact_sort", "msd_sort",
                                     "compact_msd"])
def test_long_tile_lists_and_depth_ties(gpu, oracle_mod, variant):
    """Tiles covered by more than 2048 splats (multi-chunk digit runs in the tile sort, long
    blend lists) and half of the Gaussians at one depth (ties: upstream orders them by
    Gaussian index, so the stable depth sort must keep index order).  per_pair: the same scene
    in a 4128-px-wide frame (258 tile columns), which api.hip bins in the per-pair form."""
    g = synthetic_gaussians(15000, 3, 23)
    g.scale[:] = np.float32(0.3)
    g.xyz[:7000, 2] = np.float32(0.25)  # one depth for half of them
    w = 4128 if variant == "per_pair" else 320
    s = scene_inputs(g, static_camera(w, 240, (0, 0, 3.0)), 3)
    orc = run_oracle(oracle_mod, s)
    counts = orc["ranges"][:, 1] - orc["ranges"][:, 0]
    assert counts.max() > 2048 and (counts > 2048).sum() > 10, counts.max()
    with _options(gpu, VARIANTS.get(variant, [])):
        hip = run_hip(s, gpu)
    assert_parity(hip, orc)


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("spread", [0.0, 2e-4, 0.05, 1.5, 60.0])
def test_depth_sort_pass_regimes(gpu, oracle_mod, spread, form):
    """The depth sort (depth_sort.hip) sorts only the key bits that differ between the kept
    Gaussians' depths (D = bits of OR ^ AND): all depths equal (D = 0), within 2^12 ulps, within
    2^24 (2.5..2.55, and 2.5..4 across a float exponent) and 2.5..62.5 (five exponents, D > 24).
    25k Gaussians = 4 sort tiles; off-screen ones are dropped.  GSR_OPT_DEPTH_SORT forms: 0 LSD
    passes of 12 bits decided on the device, 1 the same after compacting the kept keys, 2 one MSD
    pass over the top 12 of the D bits then every bucket sorted in LDS (its slow path for buckets
    past 4096 keys included: at D <= 12 or with few distinct depths the buckets are crowded), 3
    the MSD form on the compacted keys."""
    g = synthetic_gaussians(25000, 3, 31)
    rng = np.random.default_rng(31)
    _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, form)
    g.xyz[:, 2] = (np.float32(0.5) - rng.random(25000, dtype=np.float32) * np.float32(spread))
    g.xyz[::5, 2] = g.xyz[1::5, 2]  # ties across tiles
    s = scene_inputs(g, static_camera(320, 240, (0, 0, 3.0)), 3)
    orc = run_oracle(oracle_mod, s)
    assert orc["num_rendered"] > 0
    try:
        hip = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, -1)
    assert_parity(hip, orc)


@pytest.mark.parametrize("form", [2, 3])
@pytest.mark.parametrize("n", [5000, 60000])
def test_msd_sort_crowded_bucket(gpu, oracle_mod, n, form):
    """The MSD sort's slow path: most kept Gaussians in one bucket of the top 12 varying key bits
    (depths within 2^-13 relative of each other, a few far ones widen D to 24), so one bucket
    holds more keys than the in-LDS sort (4096) and the block sorts it through global memory."""
    g = synthetic_gaussians(n, 3, 33)
    rng = np.random.default_rng(33)
    g.xyz[:, :2] = rng.uniform(-0.5, 0.5, (n, 2)).astype(np.float32)  # all in view
    g.xyz[:, 2] = np.float32(0.5) + rng.random(n, dtype=np.float32) * np.float32(1e-4)
    g.xyz[:50, 2] = np.float32(-1.5)  # widen the key bits
    g.scale[:] = np.float32(0.01)
    s = scene_inputs(g, static_camera(320, 240, (0, 0, 3.0)), 3)
    orc = run_oracle(oracle_mod, s)
    d = orc["depths"][orc["radii"] > 0].view(np.uint32)
    D = int(np.bitwise_or.reduce(d) ^ np.bitwise_and.reduce(d)).bit_length()
    top = (d >> np.uint32(D - 12)) & np.uint32(4095)
    assert D == 24 and np.bincount(top).max() > 4096, (D, np.bincount(top).max())
    _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, form)
    try:
        hip = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, -1)
    assert_parity(hip, orc)


def test_tile_lists_of_one_depth(gpu, oracle_mod):
    """Every Gaussian at the same depth: each tile's list is already in upstream's order."""
    g = synthetic_gaussians(3000, 3, 24)
    g.xyz[:, 2] = np.float32(-0.5)
    s = scene_inputs(g, static_camera(160, 120, (0, 0, 3.0)), 1)
    assert_parity(run_hip(s, gpu), run_oracle(oracle_mod, s))


@pytest.mark.parametrize("form", [1, 3])
def test_compacted_strip_colour_path(gpu, form):
    """Compacted strip frames (GSR_OPT_DEPTH_SORT 1 or 3: auto on strips of >= 4M Gaussians,
    forced here, with the LSD passes or the MSD form) colour only the compacted kept ids (k_color_ids, handed from the main stream's
    compaction to the second stream by an event) when no rgb output is requested -- the bench's
    and the viewer's call.  Every strip must be bit-identical to the same rows of the full frame
    rendered without compaction (k_color over every Gaussian)."""
    from gaussiansplattingviewer_amd.strips import strip_pixel_rows, strip_rows
    W, H = 1920, 1080
    s = scene_inputs(synthetic_gaussians(300_000, 3, 26), static_camera(W, H, (0.3, 0.2, 3.8)), 3)
    pix = ("final_T", "n_contrib")  # no "rgb": the compacted-id colour pass is allowed
    full = run_hip(s, gpu, extras=pix)
    gy = (H + 15) // 16
    _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, form)
    try:
        for r in range(8):
            rows = strip_rows(gy, 8, r)
            part = run_hip(s, gpu, tile_rows=rows, extras=pix)
            y0, n = strip_pixel_rows(rows, H)
            for k, v in (("color", full["color"][:, y0:y0 + n]), ("final_T", full["final_T"][y0:y0 + n]),
                         ("n_contrib", full["n_contrib"][y0:y0 + n])):
                np.testing.assert_array_equal(part[k].view(np.uint32), v.view(np.uint32), err_msg=k)
            np.testing.assert_array_equal(part["radii"], full["radii"])
            lean = run_hip(s, gpu, tile_rows=rows, extras=pix, radii=False)
            for k in ("color", "final_T", "n_contrib", "point_list"):
                np.testing.assert_array_equal(lean[k], part[k], err_msg=k)
    finally:
        _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, -1)


def test_msd_local_sort_tier_boundaries(gpu, oracle_mod):
    """k_ds_local sorts a bucket with 2, 4, 8 or 16 keys per lane by its size (<= 128, <= 256,
    <= 512, <= 1024 keys with GSR_LOCAL_WAVE_KEYS 1024; larger ones by the whole block): buckets of the MSD pass's top 12 key bits are
    built with sizes on both sides of every boundary (depths 2..8: D = 24, bucket = key bits
    12..23), then the frame must match the oracle."""
    rng = np.random.default_rng(41)
    sizes = [1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 700, 1023, 1024, 1025,
             2000, 4000]
    keys = [np.uint32(0x40000000 | (4095 << 12) | 2048)]  # the deepest key: bit 23 set, D = 24
    for i, n in enumerate(sizes):
        b = 16 + 211 * i  # well-separated buckets below 4095
        low = rng.integers(256, 3840, n).astype(np.uint32)  # away from the bucket's edges
        keys.append(np.uint32(0x40000000) | np.uint32(b << 12) | low)
    keys = np.concatenate([np.atleast_1d(k) for k in keys]).astype(np.uint32)
    P = len(keys)
    g = synthetic_gaussians(P, 3, 41)
    g.xyz[:, :2] = rng.uniform(-0.15, 0.15, (P, 2)).astype(np.float32)
    g.xyz[:, 2] = np.float32(3.0) - keys.view(np.float32)  # view depth 3 - z from (0, 0, 3)
    g.scale[:] = np.float32(0.005)
    g.opacity[:] = np.float32(3.0)
    s = scene_inputs(g, static_camera(320, 240, (0, 0, 3.0)), 3)
    orc = run_oracle(oracle_mod, s)
    d = orc["depths"][orc["radii"] > 0].view(np.uint32)
    D = int(np.bitwise_or.reduce(d) ^ np.bitwise_and.reduce(d)).bit_length()
    counts = np.bincount((d >> np.uint32(D - 12)) & np.uint32(4095), minlength=4096)
    assert D == 24, D
    for edge in (128, 256, 512, 1024):  # sizes on both sides of every tier boundary
        assert ((counts > 0) & (counts <= edge) & (counts > edge - 3)).any(), (edge, counts[counts > 0])
        assert ((counts > edge) & (counts < edge + 3)).any(), (edge, counts[counts > 0])
    _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, 2)
    try:
        hip = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, -1)
    assert_parity(hip, orc)


def test_msd_local_sort_lds_slices(gpu, oracle_mod):
    """k_ds_local's waves sort buckets of <= 1024 keys in slices of the block's 4096 LDS slots
    (wave_slice): the buckets of <= 512 keys first, then the larger ones while slots remain, the
    rest by the whole block.  Groups of 8 buckets with eight ~900-key buckets (four fit), three
    ~1000-key and five ~300-key ones (one fits), and a mix across the 512 / 1024 edges.  The
    first frame's crowded groups switch the context to the 8192-slot form (all fit) for the
    next frames: both forms must match the oracle."""
    rng = np.random.default_rng(43)
    groups = {100: [900] * 8, 101: [1000, 1000, 1000, 300, 300, 300, 300, 300],
              102: [1024, 1025, 513, 512, 1, 0, 1023, 129]}
    keys = [np.uint32(0x40000000), np.uint32(0x40000000 | (4095 << 12) | 2048)]  # min, max: D = 24
    for gi, sizes in groups.items():
        for j, n in enumerate(sizes):
            b = gi * 8 + j
            low = rng.integers(1, 4096, n).astype(np.uint32)
            low[1::3] = low[0::3][: len(low[1::3])]  # ties
            keys.append(np.uint32(0x40000000) | np.uint32(b << 12) | low)
    keys = np.concatenate([np.atleast_1d(k) for k in keys]).astype(np.uint32)
    P = len(keys)
    g = synthetic_gaussians(P, 3, 43)
    g.xyz[:, :2] = rng.uniform(-0.15, 0.15, (P, 2)).astype(np.float32)
    g.xyz[:, 2] = np.float32(3.0) - keys.view(np.float32)
    g.scale[:] = np.float32(0.005)
    g.opacity[:] = np.float32(3.0)
    s = scene_inputs(g, static_camera(320, 240, (0, 0, 3.0)), 3)
    orc = run_oracle(oracle_mod, s)
    d = orc["depths"][orc["radii"] > 0].view(np.uint32)
    kmin = d.min()
    Dr = int(d.max() - kmin).bit_length()
    counts = np.bincount((d - kmin) >> np.uint32(Dr - 12), minlength=4096)
    assert Dr == 24, Dr
    assert (counts[800:808] > 512).sum() >= 6 and (counts[816:824] > 1024).any(), counts[800:824]
    _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, 2)
    try:
        for _ in range(3):
            assert_parity(run_hip(s, gpu), orc)
    finally:
        _set_option(gpu, _lib.GSR_OPT_DEPTH_SORT, -1)


def test_one_stream_forward_outputs(gpu, oracle_mod):
    """GSR_OPT_SECOND_STREAM 0: the second stream's kernels run in order on the frame's stream.
    Every output -- image, radii, the rgb extra, the lists -- equals the two-stream forward's, and
    matches the oracle."""
    s = scene_inputs(synthetic_gaussians(20_000, 3, 51), static_camera(320, 240, (0.2, 0.1, 3.5)), 3)
    two = run_hip(s, gpu)
    _set_option(gpu, _lib.GSR_OPT_SECOND_STREAM, 0)
    try:
        one = run_hip(s, gpu)
    finally:
        _set_option(gpu, _lib.GSR_OPT_SECOND_STREAM, 1)
    assert one.keys() == two.keys()
    for k in two:
        if isinstance(two[k], np.ndarray):
            np.testing.assert_array_equal(one[k], two[k], err_msg=k)
        else:
            assert one[k] == two[k], k
    assert_parity(one, run_oracle(oracle_mod, s))
