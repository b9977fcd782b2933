"""CPU, property-based (hypothesis): invariants of the oracle's binning and sort on random
scenes, cameras and image sizes -- the CPU tier SURVEY.md §4 recommends.  The GPU tests check
the HIP path against the oracle bit-exactly, so these invariants carry over to it.

- num_rendered = sum(tiles_touched); radii > 0 exactly where a Gaussian touches a tile;
- every Gaussian's pairs sit in tiles_touched distinct tiles forming a rectangle;
- tile ranges partition [0, K) in tile order, each range holding exactly that tile's pairs;
- within a tile, pairs are ordered by (depth, Gaussian index) -- upstream's stable sort;
- the oracle's stable float argsort equals numpy's stable argsort (ties, -0, NaN, huge).
"""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians

SETTINGS = dict(max_examples=25, deadline=None,
                suppress_health_check=[HealthCheck.function_scoped_fixture])


def _scene(P, seed, W, H, eye, scale_mul, tie_frac):
    g = synthetic_gaussians(P, 3, seed)
    g.scale[:] = (g.scale * np.float32(scale_mul)).astype(np.float32)
    if P and tie_frac > 0:  # a share of the Gaussians at one depth plane (ties)
        g.xyz[:int(P * tie_frac), 2] = np.float32(0.125)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H, eye))
    return g, view, proj, campos, tx, ty


@settings(**SETTINGS)
@given(P=st.integers(1, 400), seed=st.integers(0, 10_000), W=st.integers(8, 200),
       H=st.integers(8, 150), ex=st.floats(-1.5, 1.5), ey=st.floats(-1.5, 1.5),
       ez=st.floats(2.5, 6.0), scale_mul=st.sampled_from([1.0, 10.0, 60.0]),
       tie_frac=st.sampled_from([0.0, 0.5]))
def test_binning_invariants(oracle_mod, P, seed, W, H, ex, ey, ez, scale_mul, tie_frac):
    g, view, proj, campos, tx, ty = _scene(P, seed, W, H, (ex, ey, ez), scale_mul, tie_frac)
    r = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                           sh_degree=3, scales=g.scale, rotations=g.rot)
    K = r["num_rendered"]
    gx = (W + 15) // 16
    tiles = r["tiles_touched"].astype(np.int64)
    assert K == int(tiles.sum())
    np.testing.assert_array_equal(r["radii"] > 0, tiles > 0)
    pl = r["point_list"].astype(np.int64)
    tile_of = (r["point_keys"] >> np.uint64(32)).astype(np.int64)
    assert pl.shape == (K,) and tile_of.shape == (K,)
    # the ranges partition [0, K) in tile order
    rg = r["ranges"].astype(np.int64)
    nonempty = rg[:, 1] > rg[:, 0]
    assert np.all(rg[~nonempty] == 0)
    if K:
        starts, ends = rg[nonempty, 0], rg[nonempty, 1]
        assert starts[0] == 0 and ends[-1] == K
        np.testing.assert_array_equal(starts[1:], ends[:-1])
    for t in np.flatnonzero(nonempty):
        s, e = rg[t]
        assert np.all(tile_of[s:e] == t)
        ids = pl[s:e]
        # (depth, index) non-decreasing: upstream's stable sort of index-ordered pairs
        np.testing.assert_array_equal(np.lexsort((ids, r["depths"][ids])), np.arange(e - s))
    # each Gaussian: tiles_touched distinct tiles, forming its rect
    np.testing.assert_array_equal(np.bincount(pl, minlength=P)[:P], tiles)
    for i in np.flatnonzero(tiles)[:40]:
        t_i = tile_of[pl == i]
        xs, ys = t_i % gx, t_i // gx
        w = xs.max() - xs.min() + 1
        h = ys.max() - ys.min() + 1
        assert len(np.unique(t_i)) == tiles[i] == w * h


@settings(**SETTINGS)
@given(n=st.integers(0, 3000), seed=st.integers(0, 10_000),
       kind=st.sampled_from(["normal", "ties", "signed_zero", "nan", "huge"]))
def test_stable_argsort_matches_numpy(oracle_mod, n, seed, kind):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        d = rng.normal(0, 3, n).astype(np.float32)
    elif kind == "ties":
        d = rng.integers(-5, 5, n).astype(np.float32)
    elif kind == "signed_zero":
        d = rng.choice(np.array([-0.0, 0.0, 1.0, -1.0], np.float32), n)
    elif kind == "nan":
        d = rng.choice(np.array([np.nan, 0.5, -2.0, np.inf, -np.inf], np.float32), n)
    else:
        d = (rng.normal(0, 1, n) * 1e30).astype(np.float32)
    np.testing.assert_array_equal(oracle_mod.argsort_stable(d), np.argsort(d, kind="stable"))


def test_oracle_threads_do_not_change_results(oracle_mod):
    """The oracle's OpenMP loops (bench.py's host-cores CPU baseline) give bit-identical results
    at 1 and at 8 threads."""
    g, view, proj, campos, tx, ty = _scene(120_000, 3, 400, 300, (0.4, -0.2, 3.5), 10.0, 0.25)
    out = []
    for n in (1, 8):
        oracle_mod.set_threads(n)
        out.append(oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, 400, 300,
                                      shs=g.sh, sh_degree=3, scales=g.scale, rotations=g.rot))
    oracle_mod.set_threads(0)
    a, b = out
    assert a["num_rendered"] > 100_000
    for k, v in a.items():
        if isinstance(v, np.ndarray):
            np.testing.assert_array_equal(np.asarray(b[k]).view(np.uint8), v.view(np.uint8), err_msg=k)
        else:
            assert b[k] == v, k
