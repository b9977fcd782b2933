"""CPU: pin the oracle's SH colour, 3D covariance and per-pixel alpha to the reference's own GLSL
twins of upstream's formulas.

The upstream CUDA forward (diff-gaussian-rasterization) is not vendored in the reference, so the
oracle's restatement of it cannot be checked against its outputs.  What the
reference does hold is a GLSL restatement of three of the same formulas, which its OpenGL backend
runs:

  * gau_vert.glsl:3-18 + :213-250 -- the SH basis constants and the degree 0..3 SH -> colour
    formula (upstream computeColorFromSH, before its clamp at 0);
  * gau_vert.glsl:73-93 -- computeCov3D (Sigma = (S R)^T (S R), the quaternion unnormalised);
  * gau_frag.glsl:21-27 -- the per-pixel alpha: power = -0.5 (a dx^2 + c dy^2) - b dx dy,
    skip if power > 0, alpha = min(0.99, opacity exp(power)), skip if alpha < 1/255.

Their numeric literals are parsed from the shader text into tests/golden/glsl_twins.npz
(tests/golden/make_golden.py --only glsl).  Each test evaluates the GLSL formula in float64
with those literals (as float32, their `f` suffix) and compares the oracle's float32 result.
(The EWA covariance, gau_vert.glsl:95-120, is checked in test_oracle_restatement.py.)  The
steps of upstream's forward that have no reference-held twin stay parity-unpinned and are
listed in DESIGN.md §4.
"""
import numpy as np
import pytest

from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera


@pytest.fixture(scope="module")
def glsl(golden):
    z = golden("glsl_twins.npz")
    return {k: float(z[k]) for k in z.files}


def _c(glsl, name):  # a GLSL float literal (`...f`): its float32 value
    return float(np.float32(glsl[name]))


def glsl_sh(glsl, dirs, sh, deg):
    """gau_vert.glsl:213-250 in float64 (render_mod = deg, sh_dim = 48): colour before any clamp."""
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    g = lambda i: sh[:, i, :]  # noqa: E731  (get_vec3(sh_start + 3 i))
    color = _c(glsl, "SH_C0") * g(0)
    if deg >= 1:
        c1 = _c(glsl, "SH_C1")
        color = color - c1 * y * g(1) + c1 * z * g(2) - c1 * x * g(3)
        if deg >= 2:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            color = (color + _c(glsl, "SH_C2_0") * xy * g(4) + _c(glsl, "SH_C2_1") * yz * g(5) +
                     _c(glsl, "SH_C2_2") * (2.0 * zz - xx - yy) * g(6) +
                     _c(glsl, "SH_C2_3") * xz * g(7) + _c(glsl, "SH_C2_4") * (xx - yy) * g(8))
            if deg >= 3:
                color = (color +
                         _c(glsl, "SH_C3_0") * y * (3.0 * xx - yy) * g(9) +
                         _c(glsl, "SH_C3_1") * xy * z * g(10) +
                         _c(glsl, "SH_C3_2") * y * (4.0 * zz - xx - yy) * g(11) +
                         _c(glsl, "SH_C3_3") * z * (2.0 * zz - 3.0 * xx - 3.0 * yy) * g(12) +
                         _c(glsl, "SH_C3_4") * x * (4.0 * zz - xx - yy) * g(13) +
                         _c(glsl, "SH_C3_5") * z * (xx - yy) * g(14) +
                         _c(glsl, "SH_C3_6") * x * (xx - 3.0 * yy) * g(15))
    return color + 0.5


def test_glsl_literals_parsed(glsl):
    """The parse found every literal, and they are the values upstream's forward.cu writes
    (its SH_C* float literals, the 1.3 clamp, the 0.3 low-pass, 0.99 and 1/255)."""
    assert sum(k.startswith("SH_C") for k in glsl) == 14
    assert glsl["SH_C2_1"] == -glsl["SH_C2_0"] and glsl["SH_C2_3"] == -glsl["SH_C2_0"]
    assert glsl["SH_C3_6"] == glsl["SH_C3_0"] and glsl["SH_C3_4"] == glsl["SH_C3_2"]
    assert glsl["COV2D_CLAMP"] == 1.3 and glsl["COV2D_LOWPASS"] == 0.3
    assert glsl["ALPHA_EXP_COEF"] == -0.5 and glsl["ALPHA_CAP"] == 0.99
    assert glsl["ALPHA_MIN"] == 1.0 / 255.0


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_colour_matches_glsl(oracle_mod, glsl, deg):
    """100k directions over the whole sphere (upstream's dir = (mean - campos) / |...|),
    3DGS-like coefficients (DC of order 1, the rest of order 0.1-0.3): the oracle's colour
    equals the GLSL formula within 2e-6 where it is not clamped, and clamped channels are the
    ones the GLSL formula puts below 0 (up to the same rounding)."""
    rng = np.random.default_rng(100 + deg)
    n = 100_000
    campos = rng.normal(size=3).astype(np.float32)
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    means = (campos + dirs * rng.uniform(0.3, 30.0, size=(n, 1))).astype(np.float32)
    sh = np.empty((n, 16, 3), np.float32)
    sh[:, 0] = rng.uniform(-2.5, 2.5, size=(n, 3))
    sh[:, 1:] = rng.normal(scale=0.25, size=(n, 15, 3))
    rgb, clamped = oracle_mod.color_from_sh(means, campos, sh, deg)
    # the direction as upstream / the GLSL compute it, from the float32 inputs
    d = means.astype(np.float64) - campos.astype(np.float64)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ref = glsl_sh(glsl, d, sh.astype(np.float64), deg)
    free = ~clamped
    assert free.mean() > 0.5
    err = np.abs(rgb[free] - ref[free])
    assert err.max() <= 2e-6, (err.max(), np.argmax(err))
    assert np.all(rgb[clamped] == 0.0)
    assert np.all(ref[clamped] <= 2e-6)


@pytest.mark.parametrize("normalised", [True, False])
@pytest.mark.parametrize("mod", [1.0, 0.7])
def test_cov3d_matches_glsl(oracle_mod, normalised, mod):
    """gau_vert.glsl:73-93 computeCov3D(g_scale * scale_modifier, g_rot) in float64 against the
    oracle's upstream computeCov3D (S = diag(mod * scale)): within 1e-6 of the largest entry.
    Both use the quaternion as given (neither normalises it), so unnormalised ones are checked
    too."""
    rng = np.random.default_rng(7 if normalised else 8)
    n = 20_000
    scales = np.exp(rng.normal(-3.5, 1.2, size=(n, 3))).astype(np.float32)
    q = rng.normal(size=(n, 4))
    if normalised:
        q /= np.linalg.norm(q, axis=1, keepdims=True)
    else:
        q *= rng.uniform(0.3, 2.0, size=(n, 1)) / np.linalg.norm(q, axis=1, keepdims=True)
    q = q.astype(np.float32)
    ours = oracle_mod.cov3d(scales, q, mod).astype(np.float64)
    s = scales.astype(np.float64) * np.float64(np.float32(mod))
    r, x, y, z = (q[:, i].astype(np.float64) for i in range(4))
    # GLSL mat3(...) takes columns; R[col][row]
    cols = np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        np.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        np.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], 1)
    Rm = np.transpose(cols, (0, 2, 1))            # row-major matrix of the GLSL R
    Sm = np.zeros((n, 3, 3))
    Sm[:, 0, 0], Sm[:, 1, 1], Sm[:, 2, 2] = s[:, 0], s[:, 1], s[:, 2]
    M = Sm @ Rm                                    # GLSL `S * R`
    Sig = np.transpose(M, (0, 2, 1)) @ M           # transpose(M) * M
    ref = np.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2],
                    Sig[:, 2, 2]], -1)
    scale = np.abs(ref).max(axis=1, keepdims=True)
    rel = np.abs(ours - ref) / scale
    assert rel.max() <= 1e-6, rel.max()


def glsl_alpha(glsl, conic, opacity, dx, dy):
    """gau_frag.glsl:21-27 in float64: alpha, or 0 where the fragment is discarded."""
    power = (_c(glsl, "ALPHA_EXP_COEF") * (conic[0] * dx * dx + conic[2] * dy * dy) -
             conic[1] * dx * dy)
    alpha = np.minimum(_c(glsl, "ALPHA_CAP"), opacity * np.exp(power))
    keep = (power <= 0.0) & (alpha >= np.float32(1.0) / np.float32(255.0))
    return np.where(keep, alpha, 0.0), power


@pytest.mark.parametrize("case", range(6))
def test_alpha_matches_glsl_fragment(oracle_mod, glsl, case):
    """One splat per frame, white colour, black background: the oracle's pixel value is
    upstream's alpha (T = 1 before it).  On every pixel of the tiles the splat is binned to, it
    equals the GLSL fragment's alpha (0 where the fragment discards) within 1e-6; the only
    pixels allowed to disagree on keep / skip lie within 1e-6 of the 1/255 floor.  Opacities
    span the floor, the middle and the 0.99 cap."""
    rng = np.random.default_rng(300 + case)
    W, H = 160, 128
    opac = [0.0045, 0.02, 0.3, 0.75, 0.995, 1.0][case]
    xyz = np.array([[rng.uniform(-0.3, 0.3), rng.uniform(-0.2, 0.2), rng.uniform(-0.5, 0.5)]],
                   np.float32)
    scale = np.exp(rng.normal(-2.8, 0.5, size=(1, 3))).astype(np.float32)
    q = rng.normal(size=(1, 4))
    rot = (q / np.linalg.norm(q)).astype(np.float32)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H, eye=(0.0, 0.0, 2.5)))
    r = oracle_mod.forward(xyz, np.array([[opac]], np.float32), view, proj, campos, tx, ty, W, H,
                           scales=scale, rotations=rot,
                           colors_precomp=np.ones((1, 3), np.float32))
    assert r["radii"][0] > 0
    gx = (W + 15) // 16
    binned = np.zeros((H, W), bool)
    for t in np.nonzero(r["ranges"][:, 1] > r["ranges"][:, 0])[0]:
        ty_, tx_ = divmod(int(t), gx)
        binned[ty_ * 16:(ty_ + 1) * 16, tx_ * 16:(tx_ + 1) * 16] = True
    assert binned.sum() >= 256
    ys, xs = np.nonzero(binned)
    mx, my = r["means2D"][0].astype(np.float64)
    conic = r["conic_opacity"][0, :3].astype(np.float64)
    ref, power = glsl_alpha(glsl, conic, np.float64(np.float32(opac)), mx - xs, my - ys)
    ours = r["color"][0, ys, xs].astype(np.float64)
    # the outside of the binned tiles stays background
    assert np.all(r["color"][:, ~binned] == 0.0)
    both = (ours > 0) & (ref > 0)
    assert np.abs(ours[both] - ref[both]).max(initial=0.0) <= 1e-6
    differ = (ours > 0) != (ref > 0)
    edge = (np.abs(ref - 1.0 / 255.0) <= 1e-6) | (np.abs(np.minimum(opac * np.exp(power), 0.99)
                                                          - 1.0 / 255.0) <= 1e-6)
    assert np.all(edge[differ]), int(differ.sum())
    capped = opac * np.exp(power) >= 0.99 + 1e-6  # the 0.99 cap binds on these pixels
    assert np.all(ours[capped] == np.float32(0.99))
    if opac == 1.0:
        assert capped.any()
