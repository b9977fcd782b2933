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
