"""CPU: check the C oracle against an independent pure-Python float32 restatement of the same
upstream functions (small sizes), against the reference's GLSL twin formulas, and for the
structural invariants of upstream's binning."""
import math

import numpy as np
import pytest

from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, look_at, static_camera, Camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians

f32 = np.float32


# ---- pure-Python float32 restatement (upstream forward.cu / auxiliary.h) -----------------
def mat3_cols(*a):
    return [[f32(a[3 * c + r]) for r in range(3)] for c in range(3)]  # m[col][row]


def mat3_mul(A, B):
    R = [[f32(0)] * 3 for _ in range(3)]
    for j in range(3):
        for i in range(3):
            s = f32(A[0][i] * B[j][0])
            s = f32(s + f32(A[1][i] * B[j][1]))
            s = f32(s + f32(A[2][i] * B[j][2]))
            R[j][i] = s
    return R


def transpose(A):
    return [[A[i][j] for i in range(3)] for j in range(3)]


def tp43(p, M):
    return [f32(f32(f32(f32(M[k] * p[0]) + f32(M[4 + k] * p[1])) + f32(M[8 + k] * p[2])) + M[12 + k])
            for k in range(3)]


def tp44(p, M):
    return [f32(f32(f32(f32(M[k] * p[0]) + f32(M[4 + k] * p[1])) + f32(M[8 + k] * p[2])) + M[12 + k])
            for k in range(4)]


def f2i(v):
    if math.isnan(v):
        return 0
    return int(max(min(math.trunc(float(v)), 2**31 - 1), -2**31))


def py_preprocess(i, g, view, proj, campos, tx, ty, W, H, D):
    M_ = 16 if g.sh.shape[1] == 48 else 1
    p = [f32(v) for v in g.xyz[i]]
    pv = tp43(p, view)
    if not pv[2] > f32(0.2):
        return None
    ph = tp44(p, proj)
    pw = f32(f32(1) / f32(ph[3] + f32(1e-7)))
    pp = [f32(ph[0] * pw), f32(ph[1] * pw)]
    s = g.scale[i]
    S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1)
    S[0][0], S[1][1], S[2][2] = f32(f32(1) * s[0]), f32(f32(1) * s[1]), f32(f32(1) * s[2])
    r, x, y, z = [f32(v) for v in g.rot[i]]
    two, one = f32(2), f32(1)
    R = mat3_cols(one - two * f32(y * y + z * z), two * f32(x * y - r * z), two * f32(x * z + r * y),
                  two * f32(x * y + r * z), one - two * f32(x * x + z * z), two * f32(y * z - r * x),
                  two * f32(x * z - r * y), two * f32(y * z + r * x), one - two * f32(x * x + y * y))
    Mm = mat3_mul(S, R)
    Sig = mat3_mul(transpose(Mm), Mm)
    c = [Sig[0][0], Sig[0][1], Sig[0][2], Sig[1][1], Sig[1][2], Sig[2][2]]
    fy = f32(f32(H) / f32(f32(2) * f32(ty)))
    fx = f32(f32(W) / f32(f32(2) * f32(tx)))
    t = list(pv)
    limx, limy = f32(f32(1.3) * f32(tx)), f32(f32(1.3) * f32(ty))
    txtz, tytz = f32(t[0] / t[2]), f32(t[1] / t[2])
    t[0] = f32(min(limx, max(-limx, txtz)) * t[2])
    t[1] = f32(min(limy, max(-limy, tytz)) * t[2])
    tz2 = f32(t[2] * t[2])
    J = mat3_cols(f32(fx / t[2]), 0, f32(-f32(fx * t[0]) / tz2), 0, f32(fy / t[2]),
                  f32(-f32(fy * t[1]) / tz2), 0, 0, 0)
    Wm = mat3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10])
    T = mat3_mul(Wm, J)
    Vrk = mat3_cols(c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5])
    cov = mat3_mul(mat3_mul(transpose(T), transpose(Vrk)), T)
    a, b, cc = f32(cov[0][0] + f32(0.3)), cov[0][1], f32(cov[1][1] + f32(0.3))
    det = f32(f32(a * cc) - f32(b * b))
    if det == 0:
        return None
    di = f32(f32(1) / det)
    conic = (f32(cc * di), f32(-b * di), f32(a * di))
    mid = f32(f32(0.5) * f32(a + cc))
    l1 = f32(mid + np.sqrt(max(f32(0.1), f32(f32(mid * mid) - det)), dtype=f32))
    l2 = f32(mid - np.sqrt(max(f32(0.1), f32(f32(mid * mid) - det)), dtype=f32))
    rad = f32(math.ceil(f32(f32(3) * np.sqrt(max(l1, l2), dtype=f32))))
    px = f32(((float(pp[0]) + 1.0) * W - 1.0) * 0.5)
    py = f32(((float(pp[1]) + 1.0) * H - 1.0) * 0.5)
    ri = f2i(rad)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    rect = (min(gx, max(0, f2i(f32(f32(px - f32(ri)) / f32(16))))),
            min(gy, max(0, f2i(f32(f32(py - f32(ri)) / f32(16))))),
            min(gx, max(0, f2i(f32(f32(f32(f32(px + f32(ri)) + f32(16)) - f32(1)) / f32(16))))),
            min(gy, max(0, f2i(f32(f32(f32(f32(py + f32(ri)) + f32(16)) - f32(1)) / f32(16))))))
    if (rect[2] - rect[0]) * (rect[3] - rect[1]) == 0:
        return None
    # SH (deg <= 3), upstream computeColorFromSH
    pos = [f32(v) for v in g.xyz[i]]
    d = [f32(pos[k] - f32(campos[k])) for k in range(3)]
    ln = np.sqrt(f32(f32(f32(d[0] * d[0]) + f32(d[1] * d[1])) + f32(d[2] * d[2])), dtype=f32)
    d = [f32(v / ln) for v in d]
    sh = g.sh[i].reshape(M_, 3).astype(f32)
    C0, C1 = f32(0.28209479177387814), f32(0.4886025119029199)
    C2 = [f32(v) for v in (1.0925484305920792, -1.0925484305920792, 0.31539156525252005,
                           -1.0925484305920792, 0.5462742152960396)]
    C3 = [f32(v) for v in (-0.5900435899266435, 2.890611442640554, -0.4570457994644658,
                           0.3731763325901154, -0.4570457994644658, 1.445305721320277,
                           -0.5900435899266435)]
    res = [f32(C0 * sh[0][k]) for k in range(3)]
    if D > 0:
        x, y, z = d
        a1, a2, a3 = f32(C1 * y), f32(C1 * z), f32(C1 * x)
        res = [f32(f32(f32(res[k] - f32(a1 * sh[1][k])) + f32(a2 * sh[2][k])) - f32(a3 * sh[3][k]))
               for k in range(3)]
        if D > 1:
            xx, yy, zz = f32(x * x), f32(y * y), f32(z * z)
            xy, yz, xz = f32(x * y), f32(y * z), f32(x * z)
            b = [f32(C2[0] * xy), f32(C2[1] * yz), f32(C2[2] * f32(f32(f32(2) * zz - xx) - yy)),
                 f32(C2[3] * xz), f32(C2[4] * f32(xx - yy))]
            for k in range(3):
                acc = res[k]
                for m in range(5):
                    acc = f32(acc + f32(b[m] * sh[4 + m][k]))
                res[k] = acc
            if D > 2:
                e = [f32(f32(C3[0] * y) * f32(f32(f32(3) * xx) - yy)),
                     f32(f32(C3[1] * xy) * z),
                     f32(f32(C3[2] * y) * f32(f32(f32(f32(4) * zz) - xx) - yy)),
                     f32(f32(C3[3] * z) * f32(f32(f32(f32(2) * zz) - f32(f32(3) * xx)) - f32(f32(3) * yy))),
                     f32(f32(C3[4] * x) * f32(f32(f32(f32(4) * zz) - xx) - yy)),
                     f32(f32(C3[5] * z) * f32(xx - yy)),
                     f32(f32(C3[6] * x) * f32(xx - f32(f32(3) * yy)))]
                for k in range(3):
                    acc = res[k]
                    for m in range(7):
                        acc = f32(acc + f32(e[m] * sh[9 + m][k]))
                    res[k] = acc
    rgb = [max(f32(v + f32(0.5)), f32(0)) for v in res]
    return dict(depth=pv[2], radius=ri, xy=(px, py), conic=conic, rgb=rgb,
                tiles=(rect[2] - rect[0]) * (rect[3] - rect[1]))


@pytest.mark.parametrize("sh_degree,seed", [(3, 5), (0, 6)])
def test_oracle_preprocess_matches_python_restatement(oracle_mod, sh_degree, seed):
    W, H = 160, 120
    g = synthetic_gaussians(400, sh_degree, seed=seed)
    cam = static_camera(W, H, eye=(0.3, -0.2, 3.0))
    view, proj, campos, tx, ty = cuda_camera_inputs(cam)
    r = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                           sh_degree=sh_degree, scales=g.scale, rotations=g.rot)
    vflat, pflat = view.reshape(-1), proj.reshape(-1)
    nvis = 0
    for i in range(len(g)):
        e = py_preprocess(i, g, vflat, pflat, campos, tx, ty, W, H, sh_degree)
        if e is None:
            assert r["radii"][i] == 0 and r["tiles_touched"][i] == 0
            continue
        nvis += 1
        assert r["radii"][i] == e["radius"]
        assert r["tiles_touched"][i] == e["tiles"]
        assert r["depths"][i] == e["depth"]
        assert tuple(r["means2D"][i]) == e["xy"]
        assert tuple(r["conic_opacity"][i, :3]) == e["conic"]
        assert tuple(r["rgb"][i]) == tuple(e["rgb"])
    assert nvis > 50


def py_render_pixel(r, px, py, W):
    gx = (W + 15) // 16
    t = (py // 16) * gx + px // 16
    s, e = r["ranges"][t]
    T, C, last = f32(1), [f32(0)] * 3, 0
    for j in range(s, e):
        gid = r["point_list"][j]
        x, y = r["means2D"][gid]
        co = r["conic_opacity"][gid]
        dx, dy = f32(x - f32(px)), f32(y - f32(py))
        power = f32(f32(f32(-0.5) * f32(f32(f32(co[0] * dx) * dx) + f32(f32(co[2] * dy) * dy)))
                    - f32(f32(co[1] * dx) * dy))
        if power > 0:
            continue
        alpha = min(f32(0.99), f32(co[3] * np.exp(power, dtype=f32)))
        if alpha < f32(1) / f32(255):
            continue
        test_T = f32(T * f32(1 - alpha))
        if test_T < f32(0.0001):
            break
        C = [f32(C[k] + f32(f32(r["rgb"][gid][k] * alpha) * T)) for k in range(3)]
        T = test_T
        last = j - s + 1
    return C, T, last


def test_oracle_render_matches_python_restatement(oracle_mod):
    W, H = 96, 80
    g = synthetic_gaussians(3000, 3, seed=11)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H, eye=(0, 0, 2.5)))
    r = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                           sh_degree=3, scales=g.scale, rotations=g.rot)
    rng = np.random.default_rng(0)
    for _ in range(150):
        px, py = int(rng.integers(0, W)), int(rng.integers(0, H))
        C, T, last = py_render_pixel(r, px, py, W)
        np.testing.assert_allclose(r["color"][:, py, px], C, rtol=0, atol=2e-6)
        assert abs(r["final_T"][py, px] - T) <= 2e-6
        assert r["n_contrib"][py, px] == last


def test_binning_invariants_c1(oracle_mod):
    W, H = 640, 480
    g = synthetic_gaussians(10_000, 3, seed=0)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H))
    r = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                           sh_degree=3, scales=g.scale, rotations=g.rot)
    K = r["num_rendered"]
    assert K == int(r["tiles_touched"].sum()) and K == len(r["point_list"])
    keys = r["point_keys"]
    assert np.all(keys[1:] >= keys[:-1])
    tiles = (keys >> np.uint64(32)).astype(np.int64)
    depth_bits = (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    np.testing.assert_array_equal(depth_bits, r["depths"][r["point_list"]].view(np.uint32))
    # within equal keys the Gaussian ids ascend (stable sort of index-ordered input)
    same = keys[1:] == keys[:-1]
    assert np.all(r["point_list"][1:][same] > r["point_list"][:-1][same])
    gx = (W + 15) // 16
    counts = np.bincount(tiles, minlength=gx * ((H + 15) // 16))
    nonempty = counts > 0
    np.testing.assert_array_equal(r["ranges"][nonempty, 1] - r["ranges"][nonempty, 0], counts[nonempty])
    assert np.all(r["ranges"][~nonempty] == 0)


def test_conic_matches_glsl_twin_formula(oracle_mod):
    """shaders/gau_vert.glsl:95-120 computes Sigma2D with the GL view (z < 0); the CUDA view
    negates rows 0 and 2, which flips the sign of the off-diagonal term only."""
    W, H = 320, 240
    g = synthetic_gaussians(500, 0, seed=3)
    cam = static_camera(W, H, eye=(0.5, 0.2, 3.5))
    view, proj, campos, tx, ty = cuda_camera_inputs(cam)
    r = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                           sh_degree=0, scales=g.scale, rotations=g.rot)
    Vgl = cam.get_view_matrix().astype(np.float64)
    focal = cam.get_htanfovxy_focal()[2]
    htx, hty = cam.get_htanfovxy_focal()[:2]
    checked = 0
    for i in np.nonzero(r["radii"] > 0)[0][:200]:
        q = g.rot[i].astype(np.float64)
        rr, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - rr * z), 2 * (x * z + rr * y)],
                      [2 * (x * y + rr * z), 1 - 2 * (x * x + z * z), 2 * (y * z - rr * x)],
                      [2 * (x * z - rr * y), 2 * (y * z + rr * x), 1 - 2 * (x * x + y * y)]]).T
        S = np.diag(g.scale[i].astype(np.float64))
        Mm = S @ R
        Sig = Mm.T @ Mm
        t = Vgl @ np.append(g.xyz[i].astype(np.float64), 1.0)
        t[0] = min(1.3 * htx, max(-1.3 * htx, t[0] / t[2])) * t[2]
        t[1] = min(1.3 * hty, max(-1.3 * hty, t[1] / t[2])) * t[2]
        J = np.array([[focal / t[2], 0, -(focal * t[0]) / (t[2] * t[2])],
                      [0, focal / t[2], -(focal * t[1]) / (t[2] * t[2])], [0, 0, 0]])
        Wv = Vgl[:3, :3]
        T = Wv.T @ J.T  # GLSL: mat3 W = transpose(mat3(view)); T = W * J (column-major)
        cov = T.T @ Sig.T @ T
        a, b, c = cov[0, 0] + 0.3, cov[0, 1], cov[1, 1] + 0.3
        det = a * c - b * b
        glsl_conic = np.array([c / det, -b / det, a / det])
        ours = r["conic_opacity"][i, :3].astype(np.float64)
        scale = np.abs(glsl_conic).max()
        assert abs(ours[0] - glsl_conic[0]) <= 1e-3 * scale
        assert abs(ours[2] - glsl_conic[2]) <= 1e-3 * scale
        assert abs(ours[1] + glsl_conic[1]) <= 1e-3 * scale  # y flip: off-diagonal sign
        checked += 1
    assert checked > 50
