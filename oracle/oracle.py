"""TEST INFRASTRUCTURE ONLY -- Python side of the CPU oracle (liboracle.so from gsr_oracle.c).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package (gaussiansplattingviewer_amd/) never imports it.

Contents:
  forward(...)            -- upstream diff-gaussian-rasterization forward, restated in C
                             (preprocess -> InclusiveSum -> duplicateWithKeys -> stable 64-bit
                             SortPairs -> identifyTileRanges -> renderCUDA).  PARITY UNPINNED:
                             no output of the real upstream CUDA forward exists to check it
                             against (see gsr_oracle.c header and DESIGN.md).
  view_depth / argsort    -- the reference's own sort backend (renderer_ogl.py:10-19),
                             PINNED against tests/golden/ vectors captured from the reference.
  sort_gaussian_cpu(...)  -- numpy restatement of renderer_ogl.py:10-19 (the CPU baseline).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class _OracleIn(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int64), ("D", ctypes.c_int), ("M", ctypes.c_int),
        ("scale_modifier", ctypes.c_float),
        ("means3D", ctypes.c_void_p), ("scales", ctypes.c_void_p), ("rotations", ctypes.c_void_p),
        ("opacities", ctypes.c_void_p), ("shs", ctypes.c_void_p),
        ("colors_precomp", ctypes.c_void_p), ("cov3D_precomp", ctypes.c_void_p),
        ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
        ("campos", ctypes.c_void_p), ("bg", ctypes.c_void_p),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
        ("W", ctypes.c_int), ("H", ctypes.c_int),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.oracle_preprocess.restype = i64
        L.oracle_preprocess.argtypes = [ctypes.POINTER(_OracleIn)] + [vp] * 8
        L.oracle_bin.restype = ctypes.c_int
        L.oracle_bin.argtypes = [ctypes.POINTER(_OracleIn), vp, vp, vp, vp, i64, vp, vp, vp]
        L.oracle_render.restype = None
        L.oracle_render.argtypes = [ctypes.POINTER(_OracleIn)] + [vp] * 8
        L.oracle_view_depth.restype = None
        L.oracle_view_depth.argtypes = [vp, i64, vp, vp]
        L.oracle_argsort_f32.restype = ctypes.c_int
        L.oracle_argsort_f32.argtypes = [vp, i64, vp]
        L.oracle_set_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_check_tight.restype = i64
        L.oracle_check_tight.argtypes = [ctypes.c_uint32, ctypes.c_uint32] + [vp] * 7
        L.oracle_tight_model_check.restype = i64
        L.oracle_tight_model_check.argtypes = [i64, vp, vp, vp, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_float, vp]
        L.oracle_color_from_sh.restype = None
        L.oracle_color_from_sh.argtypes = [i64, ctypes.c_int, ctypes.c_int] + [vp] * 5
        L.oracle_cov3d.restype = None
        L.oracle_cov3d.argtypes = [i64, vp, ctypes.c_float, vp, vp]
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the oracle's parallel loops (n < 1: the default, OMP_NUM_THREADS or
    the core count).  Results do not depend on it.  Returns the thread count in effect."""
    return int(lib().oracle_set_threads(int(n)))


def _c(a, dtype=np.float32):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def _p(a):
    return None if a is None else a.ctypes.data


def forward(means3D, opacities, viewmatrix, projmatrix, campos, tanfovx, tanfovy, W, H,
            shs=None, sh_degree=0, scales=None, rotations=None, scale_modifier=1.0,
            colors_precomp=None, cov3D_precomp=None, bg=(0.0, 0.0, 0.0),
            stages="all") -> dict:
    """Full forward on the CPU.  Matrices are upstream's column-major layout (the row-major
    bytes of view.T / (P @ view).T).  Returns every intermediate and output.  stages:
    "preprocess" or "bin" stop after that stage (only its outputs are returned)."""
    L = lib()
    means3D = _c(means3D).reshape(-1, 3)
    P = len(means3D)
    shs = _c(shs)
    M = 0
    if shs is not None:
        shs = shs.reshape(P, -1, 3)
        M = shs.shape[1]
    keep = dict(means3D=means3D, opac=_c(opacities).reshape(-1), shs=shs,
                scales=_c(scales), rot=_c(rotations), cp=_c(colors_precomp),
                cov=_c(cov3D_precomp), view=_c(viewmatrix).reshape(-1),
                proj=_c(projmatrix).reshape(-1), campos=_c(campos).reshape(-1),
                bg=_c(bg).reshape(-1))
    inp = _OracleIn(P=P, D=int(sh_degree), M=M, scale_modifier=float(scale_modifier),
                    means3D=_p(keep["means3D"]), scales=_p(keep["scales"]),
                    rotations=_p(keep["rot"]), opacities=_p(keep["opac"]), shs=_p(keep["shs"]),
                    colors_precomp=_p(keep["cp"]), cov3D_precomp=_p(keep["cov"]),
                    viewmatrix=_p(keep["view"]), projmatrix=_p(keep["proj"]),
                    campos=_p(keep["campos"]), bg=_p(keep["bg"]), tanfovx=float(tanfovx),
                    tanfovy=float(tanfovy), W=int(W), H=int(H))
    depths = np.zeros(P, np.float32)
    radii = np.zeros(P, np.int32)
    means2D = np.zeros((P, 2), np.float32)
    conic = np.zeros((P, 4), np.float32)
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    tiles = np.zeros(P, np.uint32)
    cov3d = np.zeros((P, 6), np.float32)
    K = L.oracle_preprocess(ctypes.byref(inp), _p(depths), _p(radii), _p(means2D), _p(conic),
                            _p(rgb), _p(clamped), _p(tiles), _p(cov3d))
    out = dict(num_rendered=int(K), depths=depths, radii=radii, means2D=means2D,
               conic_opacity=conic, rgb=rgb, clamped=clamped, tiles_touched=tiles, cov3D=cov3d)
    if stages == "preprocess":
        return out
    gx, gy = (W + 15) // 16, (H + 15) // 16
    keys = np.zeros(max(K, 1), np.uint64)
    vals = np.zeros(max(K, 1), np.uint32)
    ranges = np.zeros((gx * gy, 2), np.uint32)
    rc = L.oracle_bin(ctypes.byref(inp), _p(depths), _p(radii), _p(means2D), _p(tiles), K,
                      _p(keys), _p(vals), _p(ranges))
    if rc != 0:
        raise RuntimeError(f"oracle_bin failed: {rc}")
    keys, vals = keys[:K], vals[:K]
    out.update(point_keys=keys, point_list=vals, ranges=ranges)
    if stages == "bin":
        return out
    color = np.zeros((3, H, W), np.float32)
    final_T = np.zeros((H, W), np.float32)
    n_contrib = np.zeros((H, W), np.uint32)
    features = rgb if colors_precomp is None else keep["cp"]
    if P > 0:
        L.oracle_render(ctypes.byref(inp), _p(ranges), _p(vals), _p(means2D), _p(features),
                        _p(conic), _p(color), _p(final_T), _p(n_contrib))
    out.update(color=color, final_T=final_T, n_contrib=n_contrib)
    return out


_TIGHT_KEYS = ("not_subsequence", "kept", "dropped", "dropped_reaching", "first_tile",
               "first_id", "max_dropped_alpha_e9", "_")
_MODEL_KEYS = ("span_coded", "rect_tiles", "dropped", "dropped_reaching", "first_id",
               "max_dropped_alpha_e9", "too_large", "eight_columns")


def check_tight(gx, gy, ranges_full, list_full, ranges_tight, list_tight, means2D,
                conic_opacity) -> dict:
    """Tight tile lists (the HIP path's GSR_OPT_TIGHT_BINNING) against the oracle's lists:
    per tile, an in-order subsequence, and every dropped pair skipped (power > 0 or alpha <
    1/255, the oracle's arithmetic) at all 256 pixel centres (tight_check.c)."""
    rf = _c(ranges_full, np.uint32).reshape(-1)
    rt = _c(ranges_tight, np.uint32).reshape(-1)
    assert len(rf) == len(rt) == 2 * gx * gy
    lf = _c(list_full, np.uint32).reshape(-1)
    lt = _c(list_tight, np.uint32).reshape(-1)
    m2 = _c(means2D).reshape(-1)
    co = _c(conic_opacity).reshape(-1)
    stats = np.zeros(8, np.int64)
    lib().oracle_check_tight(int(gx), int(gy), _p(rf), _p(lf) if len(lf) else None, _p(rt),
                             _p(lt) if len(lt) else None, _p(m2), _p(co), _p(stats))
    return dict(zip(_TIGHT_KEYS, (int(v) for v in stats)))


def tight_model_check(means2D, conic_opacity, radii, W, H, shrink=0.0) -> dict:
    """The HIP tight-binning predicate restated in C (preprocess.hip cull_data + col_spans) on
    the oracle's preprocess outputs: every tile it drops from a rect is checked at all 256
    pixel centres (tight_check.c).  shrink > 0: the predicate without its rounding margins and
    with its log-threshold scaled by (1 - shrink) -- a mutation the check must catch."""
    m2 = _c(means2D).reshape(-1)
    co = _c(conic_opacity).reshape(-1)
    r = _c(radii, np.int32).reshape(-1)
    stats = np.zeros(8, np.int64)
    lib().oracle_tight_model_check(len(r), _p(m2), _p(co), _p(r), int(W), int(H), float(shrink),
                                   _p(stats))
    return dict(zip(_MODEL_KEYS, (int(v) for v in stats)))


def color_from_sh(means3D, campos, shs, sh_degree):
    """upstream computeColorFromSH for every Gaussian: (rgb [P,3] clamped >= 0, clamped flags
    [P,3] bool).  shs [P,M,3] or [P,3M]."""
    means3D = _c(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    shs = _c(shs).reshape(P, -1)
    M = shs.shape[1] // 3
    rgb = np.zeros((P, 3), np.float32)
    clamped = np.zeros((P, 3), np.uint8)
    lib().oracle_color_from_sh(P, int(sh_degree), M, _p(means3D), _p(_c(campos).reshape(3)),
                               _p(shs), _p(rgb), _p(clamped))
    return rgb, clamped.astype(bool)


def cov3d(scales, rotations, scale_modifier=1.0) -> np.ndarray:
    """upstream computeCov3D for every Gaussian: [P,6] upper triangle xx xy xz yy yz zz."""
    scales = _c(scales).reshape(-1, 3)
    rotations = _c(rotations).reshape(-1, 4)
    out = np.zeros((scales.shape[0], 6), np.float32)
    lib().oracle_cov3d(scales.shape[0], _p(scales), float(scale_modifier), _p(rotations), _p(out))
    return out


def view_depth(xyz, view) -> np.ndarray:
    """Depth of the reference sort backend, in the operation order the reference's numpy
    produced in the build container (bit-exact against tests/golden/)."""
    xyz = _c(xyz).reshape(-1, 3)
    view = _c(view).reshape(-1)
    out = np.empty(len(xyz), np.float32)
    lib().oracle_view_depth(_p(xyz), len(xyz), _p(view), _p(out))
    return out


def argsort_stable(d) -> np.ndarray:
    d = _c(d).reshape(-1)
    out = np.empty(len(d), np.int32)
    if lib().oracle_argsort_f32(_p(d), len(d), _p(out)) != 0:
        raise RuntimeError("oracle_argsort_f32 failed")
    return out


def sort_gaussian_cpu(xyz, view_mat) -> np.ndarray:
    """numpy restatement of the reference's CPU sort backend (renderer_ogl.py:10-19): depth
    from one stacked (1,3,3) @ (P,3,1) matmul plus the z translation, then np.argsort with
    numpy's default (unstable) kind, as int32 (P, 1).  Timed as the CPU baseline."""
    xyz = np.asarray(xyz)
    view_mat = np.asarray(view_mat)
    rot = view_mat[:3, :3][np.newaxis]
    z = np.matmul(rot, xyz[:, :, np.newaxis])[:, 2, 0] + view_mat[2, 3]
    return np.argsort(z).astype(np.int32)[:, np.newaxis]
