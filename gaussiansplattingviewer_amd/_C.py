"""upstream `diff_gaussian_rasterization._C`: the native entry points, from the PyTorch-ROCm
extension `_native.so` (csrc/torch_ext.cpp) over libgsr.so.

Upstream's Python package calls one C++ entry per forward (rasterize_points.cu
`RasterizeGaussiansCUDA`, bound as `_C.rasterize_gaussians`; its caller is
`_RasterizeGaussians.forward` in `diff_gaussian_rasterization/__init__.py`, which the viewer
reaches through renderer_cuda.py:211-224):

    num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer = \\
        _C.rasterize_gaussians(bg, means3D, colors_precomp, opacities, scales, rotations,
                               scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx,
                               tanfovy, image_height, image_width, sh, sh_degree, campos,
                               prefiltered, debug)

    visible = _C.mark_visible(means3D, viewmatrix, projmatrix)

Same arguments, order and return arity; absent optional inputs are empty tensors, as upstream
passes them.  The work is `gsr_forward` / `gsr_mark_visible` in libgsr.so, on torch's current
HIP stream, with one `gsr_context` per device held by the extension.  The three buffers are
upstream's scratch (geometry, binning and image state, kept for the backward pass); this
rasterizer is forward only and keeps that state inside its context (reused across frames), so
they are returned as empty uint8 device tensors.

No fallback: importing this module fails when `_native.so` is not built
(`python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

try:
    from ._native import abi_version, mark_visible, rasterize_gaussians  # noqa: F401
except ImportError as e:  # pragma: no cover - a build problem, reported loudly
    raise ImportError(f"gaussiansplattingviewer_amd._native is not built or does not load ({e}); "
                      "run __graft_entry__.build()") from e
