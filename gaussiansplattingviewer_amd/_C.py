"""The native-entry shape of upstream `diff_gaussian_rasterization._C`.

Upstream's Python package calls one C++ entry per forward (rasterize_points.cu
`RasterizeGaussiansCUDA`, bound as `_C.rasterize_gaussians`; its caller is
`_RasterizeGaussians.forward` in `diff_gaussian_rasterization/__init__.py`, which the viewer
reaches through renderer_cuda.py:211-224):

    num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = \\
        _C.rasterize_gaussians(bg, means3D, colors_precomp, opacities, scales, rotations,
                               scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx,
                               tanfovy, image_height, image_width, sh, sh_degree, campos,
                               prefiltered, debug)

Same arguments, order, checks and return arity here; the work is `gsr_forward` in libgsr.so.
The three buffers are upstream's scratch (geometry, binning and image state, kept for the
backward pass).  This rasterizer is forward only and keeps that state inside its
`gsr_context` (reused across frames, never reallocated per call), so they are returned as
empty uint8 device tensors; the binning of the last forward is available from
`rasterizer.binning_state()`.
"""
from __future__ import annotations

import torch

from .rasterizer import rasterize_gaussians_native


def rasterize_gaussians(bg, means3D, colors_precomp, opacities, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy,
                        image_height, image_width, sh, sh_degree, campos, prefiltered, debug):
    res = rasterize_gaussians_native(bg, means3D, colors_precomp, opacities, scales, rotations,
                                     scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                                     tanfovx, tanfovy, image_height, image_width, sh, sh_degree,
                                     campos, prefiltered, debug)
    dev = res.color.device
    empty = lambda: torch.empty((0,), dtype=torch.uint8, device=dev)  # noqa: E731
    return res.num_rendered, res.color, res.radii, empty(), empty(), empty()
