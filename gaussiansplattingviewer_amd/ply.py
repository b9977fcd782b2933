"""PLY loading through the native reader.

Drop-in for the reference's `util_gau.load_ply(path)` (util_gau.py:63-125): same return value
`(GaussianData, bounding_box, center)` with the same activated float32 arrays, parsed by the
C++ reader in libgsr.so (csrc/ply_loader.hip: memory-mapped, multi-threaded) instead of
plyfile and per-property numpy loops.  `device=` loads straight into HIP device tensors (the
`GaussianDataHIP` the renderer consumes) through pinned staging, without building the numpy
arrays first.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from .gaussian_data import GaussianData


def _probe(path: str) -> _lib.GsrPlyInfo:
    lib = _lib.load_library()
    info = _lib.GsrPlyInfo()
    _lib.check(lib.gsr_ply_probe(os.fsencode(path), ctypes.byref(info)), "gsr_ply_probe")
    return info


def _bbox_center(info: _lib.GsrPlyInfo):
    bbox = np.array([list(info.bbox_min), list(info.bbox_max)], dtype=np.float32)
    return bbox, np.array(list(info.center), dtype=np.float32)


def load_ply(path: str, device=None):
    """util_gau.load_ply: returns (gaussians, bounding_box (2, 3), center (3,)).

    device=None: a host `GaussianData` (numpy float32: xyz (P,3), rot (P,4), scale (P,3),
    opacity (P,1), sh (P,48)).  device="cuda:i" (or a torch.device): a `GaussianDataHIP` whose
    tensors are filled on that device; sh is (P, 16, 3) as the renderer reshapes it."""
    info = _probe(path)
    P = int(info.P)
    lib = _lib.load_library()
    if device is None:
        xyz = np.empty((P, 3), np.float32)
        rot = np.empty((P, 4), np.float32)
        scale = np.empty((P, 3), np.float32)
        opacity = np.empty((P, 1), np.float32)
        sh = np.empty((P, 48), np.float32)
        ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in (xyz, rot, scale, opacity, sh)]
        _lib.check(lib.gsr_ply_load(os.fsencode(path), ctypes.byref(info), *ptrs, 0, None),
                   "gsr_ply_load")
        bbox, center = _bbox_center(info)
        return GaussianData(xyz, rot, scale, opacity, sh), bbox, center

    import torch
    from .renderer import GaussianDataHIP
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("device must be a HIP device (torch 'cuda:i') or None")
    t = {k: torch.empty(shape, dtype=torch.float32, device=dev) for k, shape in
         (("xyz", (P, 3)), ("rot", (P, 4)), ("scale", (P, 3)), ("opacity", (P, 1)),
          ("sh", (P, 16, 3)))}
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.gsr_ply_load(os.fsencode(path), ctypes.byref(info),
                                    *[ctypes.c_void_p(t[k].data_ptr() if P else 0)
                                      for k in ("xyz", "rot", "scale", "opacity", "sh")],
                                    1, ctypes.c_void_p(stream)), "gsr_ply_load")
    bbox, center = _bbox_center(info)
    return GaussianDataHIP(t["xyz"], t["rot"], t["scale"], t["opacity"], t["sh"]), bbox, center
