"""Drop-in replacement for the `diff_gaussian_rasterization` Python API the viewer imports.

renderer_cuda.py:13 does `from diff_gaussian_rasterization import GaussianRasterizationSettings,
GaussianRasterizer` and renderer_cuda.py:211-224 calls

    GaussianRasterizer(raster_settings=GaussianRasterizationSettings(**settings))(
        means3D=..., means2D=None, shs=..., colors_precomp=None, opacities=...,
        scales=..., rotations=..., cov3D_precomp=None)  ->  (color [3,H,W], radii [P])

The names, field order, argument checks and return values below follow that third-party API
(upstream `diff_gaussian_rasterization/__init__.py` and `_C.rasterize_gaussians` in
rasterize_points.cu); the work is done by libgsr.so (HIP, gfx950) through `_lib`.
Forward only: the viewer never differentiates (renderer_cuda.py:214 `torch.no_grad()`).
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple

import torch

from . import _lib


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _device_of(t: torch.Tensor) -> torch.device:
    if not t.is_cuda:
        raise RuntimeError("means3D must be a device (HIP) tensor")
    return t.device


def _as_dev(t, device, shape_hint: str):
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    if t.numel() == 0:
        return None
    if t.device != device:
        t = t.to(device)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


class ForwardResult(NamedTuple):
    """Everything one native forward produced (color/radii plus optional intermediates)."""
    num_rendered: int
    color: torch.Tensor
    radii: torch.Tensor
    extras: dict


def rasterize_gaussians_native(bg, means3D, colors_precomp, opacities, scales, rotations,
                               scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx,
                               tanfovy, image_height, image_width, sh, degree, campos, prefiltered,
                               debug, *, tile_rows=None, extras=(), stream=None, slot=0,
                               out_color=None, radii=True) -> ForwardResult:
    """Same arguments, order and validation as upstream `_C.rasterize_gaussians`.

    Extensions (keyword-only, for the strip partition and the parity tests):
      tile_rows -- (begin, end) 16-px tile rows to render; the image is then strip-local;
      extras    -- names of intermediates to return: depths, means2D, conic_opacity, rgb,
                   tiles_touched, final_T, n_contrib;
      stream    -- HIP stream handle (default: torch's current stream);
      slot      -- context slot (`_lib.context`): forwards in different slots may overlap;
      out_color -- preallocated contiguous f32 (3, rows, W) output (e.g. a gather buffer);
      radii     -- False (strips only, no per-Gaussian extras): no radii output
                   (ForwardResult.radii is None); Gaussians whose footprint bound misses the
                   strip skip the per-Gaussian work (a multi-GPU strip rank needs its image only).
    """
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    if not radii and (tile_rows is None or any(
            n in extras for n in ("depths", "means2D", "conic_opacity", "rgb", "tiles_touched"))):
        raise RuntimeError("radii=False needs tile_rows and no per-Gaussian extras")
    device = _device_of(means3D)
    dev_index = device.index if device.index is not None else torch.cuda.current_device()
    P = int(means3D.size(0))
    H, W = int(image_height), int(image_width)
    means3D = _as_dev(means3D, device, "P,3")
    opacities = _as_dev(opacities, device, "P,1")
    scales = _as_dev(scales, device, "P,3")
    rotations = _as_dev(rotations, device, "P,4")
    cov3D_precomp = _as_dev(cov3D_precomp, device, "P,6")
    colors_precomp = _as_dev(colors_precomp, device, "P,3")
    sh = _as_dev(sh, device, "P,M,3")
    bg = _as_dev(bg, device, "3")
    viewmatrix = _as_dev(viewmatrix, device, "4,4")
    projmatrix = _as_dev(projmatrix, device, "4,4")
    campos = _as_dev(campos, device, "3")

    M = 0
    if sh is not None:
        M = int(sh.size(1)) if sh.ndimension() == 3 else int(sh.numel() // max(P, 1) // 3)

    gy = (H + 15) // 16
    if tile_rows is None:
        rb, re = 0, 0
        y0, rows = 0, H
    else:
        rb, re = int(tile_rows[0]), int(tile_rows[1])
        y0 = rb * 16
        rows = min(H, re * 16) - y0
        if not (0 <= rb < re <= gy):
            raise RuntimeError(f"tile_rows {tile_rows} outside [0, {gy}]")

    f32 = dict(dtype=torch.float32, device=device)
    if out_color is None:
        color = torch.empty((3, rows, W), **f32)
    else:
        if (out_color.dtype != torch.float32 or not out_color.is_contiguous() or
                tuple(out_color.shape) != (3, rows, W) or out_color.device != device):
            raise RuntimeError(f"out_color must be a contiguous float32 (3, {rows}, {W}) tensor "
                               f"on {device}")
        color = out_color
    radii = torch.empty((P,), dtype=torch.int32, device=device) if radii else None
    ext = {}
    for name in extras:
        if name == "depths":
            ext[name] = torch.zeros((P,), **f32)
        elif name == "means2D":
            ext[name] = torch.zeros((P, 2), **f32)
        elif name == "conic_opacity":
            ext[name] = torch.zeros((P, 4), **f32)
        elif name == "rgb":
            ext[name] = torch.zeros((P, 3), **f32)
        elif name == "tiles_touched":
            ext[name] = torch.zeros((P,), dtype=torch.int32, device=device)
        elif name == "final_T":
            ext[name] = torch.zeros((rows, W), **f32)
        elif name == "n_contrib":
            ext[name] = torch.zeros((rows, W), dtype=torch.int32, device=device)
        else:
            raise ValueError(f"unknown extra output {name!r}")

    g = _lib.GsrGaussians(P=P, D=int(degree), M=M, scale_modifier=float(scale_modifier),
                          means3D=_lib.ptr(means3D), scales=_lib.ptr(scales),
                          rotations=_lib.ptr(rotations), opacities=_lib.ptr(opacities),
                          shs=_lib.ptr(sh), colors_precomp=_lib.ptr(colors_precomp),
                          cov3D_precomp=_lib.ptr(cov3D_precomp))
    st = _lib.GsrRasterSettings(image_width=W, image_height=H, tanfovx=float(tanfovx),
                                tanfovy=float(tanfovy), viewmatrix=_lib.ptr(viewmatrix),
                                projmatrix=_lib.ptr(projmatrix), campos=_lib.ptr(campos),
                                bg=_lib.ptr(bg), tile_row_begin=rb, tile_row_end=re,
                                prefiltered=int(bool(prefiltered)), debug=int(bool(debug)))
    out = _lib.GsrOutputs(color=color.data_ptr(),
                          radii=radii.data_ptr() if P and radii is not None else None)
    for name, t in ext.items():
        setattr(out, name, t.data_ptr())
    if stream is None:
        stream = torch.cuda.current_stream(device).cuda_stream
    lib = _lib.load_library()
    ctx = _lib.context(dev_index, slot)
    with torch.cuda.device(dev_index):
        _lib.check(lib.gsr_forward(ctx, ctypes.byref(g), ctypes.byref(st), ctypes.byref(out),
                                   ctypes.c_void_p(stream)), "gsr_forward")
    return ForwardResult(int(out.num_rendered), color, radii, ext)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings: GaussianRasterizationSettings):
    """upstream rasterize_gaussians(...) -> (color, radii), through _RasterizeGaussians."""
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales,
                                     rotations, cov3Ds_precomp, raster_settings)


# upstream's debug dump (diff-gaussian-rasterization __init__.py; the reference ignores the file
# in /root/reference/.gitignore:7)
SNAPSHOT_FILE = "snapshot_fw.dump"


def _cpu_copy(args):
    """The `_C.rasterize_gaussians` argument tuple with every tensor copied to the host."""
    return tuple(a.detach().cpu().clone() if isinstance(a, torch.Tensor) else a for a in args)


def replay_snapshot(path: str = SNAPSHOT_FILE, device=None):
    """Re-run a forward from a debug snapshot (the 19 `_C.rasterize_gaussians` arguments, tensors
    on the host) on `device` (default: the current HIP device); returns upstream's 6-tuple.
    Loaded with weights_only=True: the file holds tensors and plain numbers only."""
    from . import _C
    args = torch.load(path, weights_only=True)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    args = tuple(a.to(dev) if isinstance(a, torch.Tensor) and a.numel() else a for a in args)
    return _C.rasterize_gaussians(*args)


class _RasterizeGaussians(torch.autograd.Function):
    """upstream `_RasterizeGaussians`: packs the settings into `_C.rasterize_gaussians`'s
    argument tuple and keeps (color, radii) of its 6-tuple.  Forward only (the viewer renders
    under `torch.no_grad()`, renderer_cuda.py:214)."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings):
        from . import _C
        del means2D  # only carries screen-space gradients upstream
        rs = raster_settings
        # absent inputs travel as empty tensors, as upstream's __init__.py passes them
        none = lambda t: torch.empty(0) if t is None else t  # noqa: E731
        args = (rs.bg, means3D, none(colors_precomp), opacities, none(scales), none(rotations),
                rs.scale_modifier, none(cov3Ds_precomp), rs.viewmatrix, rs.projmatrix,
                rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, none(sh), rs.sh_degree,
                rs.campos, rs.prefiltered, rs.debug)
        # debug (upstream __init__.py): the arguments are copied to the host first, and a
        # forward that raises leaves them in SNAPSHOT_FILE for replay_snapshot()
        cpu_args = _cpu_copy(args) if rs.debug else None
        try:
            if _lib._native_shares_library():
                num_rendered, color, radii, geom, binning, img = _C.rasterize_gaussians(*args)
            else:  # GSR_LIB (an A/B build): `_C` links the in-tree library, so render by ctypes
                num_rendered, color, radii, _ = rasterize_gaussians_native(*args)
        except Exception:
            if cpu_args is not None:
                torch.save(cpu_args, SNAPSHOT_FILE)
                print(f"\nThe forward raised; its arguments are in {SNAPSHOT_FILE} "
                      "(gaussiansplattingviewer_amd.rasterizer.replay_snapshot re-runs them).")
            raise
        ctx.num_rendered = num_rendered
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_color, grad_radii):
        raise RuntimeError("gaussiansplattingviewer_amd renders forward only (the viewer never "
                           "differentiates, renderer_cuda.py:214)")


class GaussianRasterizer(torch.nn.Module):
    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions: torch.Tensor) -> torch.Tensor:
        """Frustum-cull test per point: view-space z > 0.2 (upstream markVisible, through
        `_C.mark_visible`)."""
        from . import _C
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or '
                            'precomputed 3D covariance!')
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales,
                                   rotations, cov3D_precomp, rs)


def binning_state(device_index: int = 0, slot: int = 0):
    """(point_list, point_tiles, ranges [T,2]) of the last forward on a device's context slot,
    as device int32 tensors holding the uint32 values (test / debug helper)."""
    lib = _lib.load_library()
    ctx = _lib.context(device_index, slot)
    K = ctypes.c_int64()
    T = ctypes.c_int32()
    stream = ctypes.c_void_p(torch.cuda.current_stream(device_index).cuda_stream)
    _lib.check(lib.gsr_get_binning(ctx, None, None, None, ctypes.byref(K), ctypes.byref(T),
                                   stream), "gsr_get_binning")
    dev = torch.device("cuda", device_index)
    pl = torch.empty((K.value,), dtype=torch.int32, device=dev)
    pt = torch.empty((K.value,), dtype=torch.int32, device=dev)
    rg = torch.empty((T.value, 2), dtype=torch.int32, device=dev)
    _lib.check(lib.gsr_get_binning(ctx, _lib.ptr(pl), _lib.ptr(pt), _lib.ptr(rg), None, None,
                                   stream), "gsr_get_binning")
    return pl, pt, rg


def tile_row_pairs(n_rows: int, device_index: int = 0, slot: int = 0, out=None,
                   stream=None) -> torch.Tensor:
    """Pair count of every tile row of the last forward's strip on a device's context slot
    (gsr_tile_row_pairs), as a device int32 tensor of n_rows uint32 values, written on `stream`
    (default: the current stream) without synchronising.  strips.StripBalancer weights the
    next frame's strip boundaries by these counts."""
    lib = _lib.load_library()
    ctx = _lib.context(device_index, slot)
    if out is None:
        out = torch.empty((n_rows,), dtype=torch.int32, device=torch.device("cuda", device_index))
    s = stream if stream is not None else torch.cuda.current_stream(device_index)
    _lib.check(lib.gsr_tile_row_pairs(ctx, _lib.ptr(out), int(n_rows),
                                      ctypes.c_void_p(s.cuda_stream)), "gsr_tile_row_pairs")
    return out
