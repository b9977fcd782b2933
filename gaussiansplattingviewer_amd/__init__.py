"""MI355X-native forward Gaussian-splat rasterizer behind the Gaussian Splatting Viewer's
renderer backend interface (renderer_cuda.py / renderer_ogl.py of the reference).

    from gaussiansplattingviewer_amd import GaussianRasterizationSettings, GaussianRasterizer
    from gaussiansplattingviewer_amd import HIPRenderer, _sort_gaussian_hip

Compute runs in hand-written HIP kernels for gfx950 (libgsr.so, C ABI in include/gsr.h);
there is no CPU fallback.
"""
from .rasterizer import (ForwardResult, GaussianRasterizationSettings, GaussianRasterizer,
                         binning_state, rasterize_gaussians, rasterize_gaussians_native)
from .renderer import (GaussianDataHIP, GaussianRenderBase, HIPRenderer, _sort_gaussian_hip,
                       depth_argsort, gaus_hip_from_cpu)
from .gaussian_data import GaussianData, naive_gaussian, synthetic_gaussians
from .camera import Camera, cuda_camera_inputs, look_at, orbit_eye, static_camera
from .strips import strip_rows, render_strips

__all__ = [
    "GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians",
    "rasterize_gaussians_native", "ForwardResult", "binning_state", "HIPRenderer",
    "GaussianRenderBase", "GaussianDataHIP", "gaus_hip_from_cpu", "_sort_gaussian_hip",
    "depth_argsort", "GaussianData", "naive_gaussian", "synthetic_gaussians", "Camera",
    "cuda_camera_inputs", "look_at", "orbit_eye", "static_camera", "strip_rows",
    "render_strips",
]
