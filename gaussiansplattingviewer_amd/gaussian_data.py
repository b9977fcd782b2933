"""The Gaussian input contract and the synthetic scenes of the benchmark configs.

`GaussianData` mirrors the viewer's container (util_gau.py:6-22): SoA float32 arrays
xyz (P,3), rot (P,4) quaternion (r,x,y,z), scale (P,3), opacity (P,1), sh (P, 3*M) with the
DC triple first, already activated by the loader (util_gau.py:114-124).  The renderer accepts
any object with these attributes, so the viewer's own GaussianData drops in unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class GaussianData:
    xyz: np.ndarray
    rot: np.ndarray
    scale: np.ndarray
    opacity: np.ndarray
    sh: np.ndarray

    def flat(self) -> np.ndarray:
        """AoS (P, 11 + sh_dim) array, the OpenGL SSBO layout (util_gau.py:13-15)."""
        return np.ascontiguousarray(
            np.concatenate([self.xyz, self.rot, self.scale, self.opacity, self.sh], axis=-1))

    def __len__(self) -> int:
        return len(self.xyz)

    @property
    def sh_dim(self) -> int:
        return self.sh.shape[-1]


def activate(xyz, raw_rot, raw_log_scale, raw_opacity, f_dc, f_rest_ply=None) -> GaussianData:
    """Apply the loader's activations exactly as util_gau.py:114-124 does (float64 math,
    then float32): unit quaternion, exp scale, sigmoid opacity, SH rows [DC, rest].

    f_rest_ply is in PLY property order f_rest_0..44 (channel-major, util_gau.py:92-100);
    it is reordered to coefficient-major / channel-minor like the loader."""
    xyz = np.asarray(xyz).astype(np.float32)
    rots = np.asarray(raw_rot, dtype=np.float64)
    rots = (rots / np.linalg.norm(rots, axis=-1, keepdims=True)).astype(np.float32)
    scales = np.exp(np.asarray(raw_log_scale, dtype=np.float64)).astype(np.float32)
    opac = np.asarray(raw_opacity, dtype=np.float64).reshape(-1, 1)
    opac = (1 / (1 + np.exp(-opac))).astype(np.float32)
    dc = np.asarray(f_dc, dtype=np.float64).reshape(-1, 3)
    if f_rest_ply is None:
        shs = dc.astype(np.float32)
    else:
        rest = np.asarray(f_rest_ply, dtype=np.float64)
        n = rest.shape[1] // 3
        rest = rest.reshape(len(rest), 3, n).transpose(0, 2, 1).reshape(len(rest), -1)
        shs = np.concatenate([dc, rest], axis=-1).astype(np.float32)
    return GaussianData(xyz, rots, scales, opac, np.ascontiguousarray(shs))


def synthetic_gaussians(P: int, sh_degree: int = 3, seed: int = 0) -> GaussianData:
    """The benchmark scene of SURVEY.md §8(d): rng = default_rng(seed), drawn in this order:
    xyz ~ U(-2,2)^3, log-scale ~ U(-5.5,-3.5)^3, quat ~ N(0,1)^4, opacity ~ N(0,1.5),
    f_dc ~ N(0,0.6)^3, f_rest ~ N(0,0.05)^45 (degree 3 only); then the loader activations."""
    if sh_degree not in (0, 3):
        raise ValueError("the loader (util_gau.py:94) only produces SH degree 3; degree 0 is the "
                         "DC-only scene of config C2")
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-2.0, 2.0, (P, 3))
    log_scale = rng.uniform(-5.5, -3.5, (P, 3))
    quat = rng.standard_normal((P, 4))
    opacity = rng.normal(0.0, 1.5, (P, 1))
    f_dc = rng.normal(0.0, 0.6, (P, 3))
    f_rest = rng.normal(0.0, 0.05, (P, 45)) if sh_degree == 3 else None
    return activate(xyz, quat, log_scale, opacity, f_dc, f_rest)


def clustered_scene(P: int, seed: int = 0) -> GaussianData:
    """A capture-like scene at "bicycle PLY scale" (BASELINE.json configs[2]) for the static
    camera at (0, 0, 4): no PLY is available offline, so this stands in for the structure the
    uniform cube of SURVEY.md §8(d) lacks -- clustered centres, a ground plane running under and
    behind the camera, a far background shell and floaters right in front of the lens; flat,
    anisotropic splats with mostly high opacity.  View depths span ~0.2 to ~45 (8 float
    exponents, so the depth sort needs all three of its passes), tile rows carry very different
    work (the strip balancer has something to balance), and near splats cover many tiles.

    rng = default_rng(seed); shares: 55 % clusters, 20 % ground, 20 % background, 5 % floaters;
    drawn in this order: cluster centres ~ N(0, 0.8^2)^3 (48), cluster weights ~ lognormal(0,1),
    cluster axes (std ~ logU(0.04, 0.5)^3, rotation from N(0,1)^4), cluster members; ground x, z
    ~ U(-6, 6), y ~ -1 + N(0, 0.02^2); background direction ~ N(0,1)^3 normalised, radius ~
    U(15, 40); floater depth ~ U(0.25, 1.2) in front of the camera within its field of view; then
    per Gaussian log-scale ~ U(-6, -3.8) + log(size), one axis x U(0.05, 0.3) (flat), one x
    U(0.3, 1); quat ~ N(0,1)^4; opacity ~ N(1, 2^2); f_dc ~ N(0, 0.8^2) + a per-cluster offset;
    f_rest ~ N(0, 0.08^2); the loader activations of util_gau.py:114-124 last."""
    rng = np.random.default_rng(seed)
    n_cl = int(P * 0.55)
    n_gr = int(P * 0.20)
    n_bg = int(P * 0.20)
    n_fl = P - n_cl - n_gr - n_bg
    C = 48
    centres = np.clip(rng.normal(0.0, 0.8, (C, 3)), -1.6, 1.6)
    w = rng.lognormal(0.0, 1.0, C)
    axes = np.exp(rng.uniform(np.log(0.04), np.log(0.5), (C, 3)))
    q = rng.standard_normal((C, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    r, x, y, z = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                  2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                  2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)],
                 axis=1).reshape(C, 3, 3)
    member = rng.choice(C, size=n_cl, p=w / w.sum())
    local = rng.standard_normal((n_cl, 3)) * axes[member]
    xyz_cl = centres[member] + np.einsum("pij,pj->pi", R[member], local)
    gx_ = rng.uniform(-6.0, 6.0, n_gr)
    gz_ = rng.uniform(-6.0, 6.0, n_gr)
    gy_ = -1.0 + rng.normal(0.0, 0.02, n_gr)
    xyz_gr = np.stack([gx_, gy_, gz_], axis=1)
    d = rng.standard_normal((n_bg, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    xyz_bg = d * rng.uniform(15.0, 40.0, (n_bg, 1))
    depth = rng.uniform(0.25, 1.2, n_fl)
    fx_ = rng.uniform(-0.5, 0.5, n_fl) * depth
    fy_ = rng.uniform(-0.28, 0.28, n_fl) * depth
    xyz_fl = np.stack([fx_, fy_, 4.0 - depth], axis=1)
    xyz = np.concatenate([xyz_cl, xyz_gr, xyz_bg, xyz_fl])
    size = np.concatenate([np.full(n_cl, 1.0), np.full(n_gr, 2.0),
                           np.linalg.norm(xyz_bg, axis=1) / 4.0, np.full(n_fl, 0.5)])
    log_scale = rng.uniform(-6.0, -3.8, (P, 3)) + np.log(size)[:, None]
    log_scale[:, 0] += np.log(rng.uniform(0.05, 0.3, P))
    log_scale[:, 1] += np.log(rng.uniform(0.3, 1.0, P))
    quat = rng.standard_normal((P, 4))
    opacity = rng.normal(1.0, 2.0, (P, 1))
    tint = np.concatenate([rng.normal(0.0, 0.6, (C, 3))[member], np.zeros((P - n_cl, 3))])
    f_dc = rng.normal(0.0, 0.8, (P, 3)) + tint
    f_rest = rng.normal(0.0, 0.08, (P, 45))
    return activate(xyz, quat, log_scale, opacity, f_dc, f_rest)


def naive_gaussian() -> GaussianData:
    """The viewer's 4-Gaussian default scene (util_gau.py:25-60): origin + unit axes."""
    xyz = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1], dtype=np.float32).reshape(-1, 3)
    rot = np.tile(np.array([1, 0, 0, 0], dtype=np.float32), (4, 1))
    scale = np.array([0.03, 0.03, 0.03, 0.2, 0.03, 0.03, 0.03, 0.2, 0.03, 0.03, 0.03, 0.2],
                     dtype=np.float32).reshape(-1, 3)
    col = np.array([1, 0, 1, 1, 0, 0, 0, 1, 0, 0, 0, 1], dtype=np.float32).reshape(-1, 3)
    sh = (col - 0.5) / 0.28209
    opacity = np.ones((4, 1), dtype=np.float32)
    return GaussianData(xyz, rot, scale, opacity, sh.astype(np.float32))
