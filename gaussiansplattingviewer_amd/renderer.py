"""Viewer backend on MI355X: `HIPRenderer` and the `_sort_gaussian_hip` sort backend.

`HIPRenderer` mirrors `CUDARenderer` (renderer_cuda.py:101-258) method for method, so the
viewer's frame loop (main.py:824-837: update_camera_intrin -> sort_and_update ->
update_camera_pose -> draw) drives it unchanged.  The GL texture interop of the CUDA backend
(renderer_cuda.py:118-133, 148-179, 226-258) has no counterpart: the MI355X box is headless,
so `draw()` leaves the frame in `self.image` (3,H,W) and `rgba()` gives the HWC+alpha layout
the GL path uploads (renderer_cuda.py:226-228).

`_sort_gaussian_hip(gaus, view_mat)` has the contract of the viewer's sort backends
(renderer_ogl.py:10-53): ascending view-space depth -> int32 index array (P, 1) on the host.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians_native


class GaussianRenderBase:
    """Same interface as the viewer's base class (renderer_ogl.py:75-101)."""

    def __init__(self):
        self.gaussians = None

    def update_gaussian_data(self, gaus):
        raise NotImplementedError()

    def sort_and_update(self, camera, use_file=False, pose=None):
        raise NotImplementedError()

    def set_scale_modifier(self, modifier: float):
        raise NotImplementedError()

    def set_render_mod(self, mod: int):
        raise NotImplementedError()

    def update_camera_pose(self, camera, use_file=False, pose=None):
        raise NotImplementedError()

    def update_camera_intrin(self, camera):
        raise NotImplementedError()

    def draw(self):
        raise NotImplementedError()

    def set_render_reso(self, w, h):
        raise NotImplementedError()


@dataclass
class GaussianDataHIP:
    """Device copy of the Gaussians (renderer_cuda.py:55-68 GaussianDataCUDA)."""
    xyz: torch.Tensor
    rot: torch.Tensor
    scale: torch.Tensor
    opacity: torch.Tensor
    sh: torch.Tensor

    def __len__(self):
        return len(self.xyz)

    @property
    def sh_dim(self):
        return self.sh.shape[-2]


def gaus_hip_from_cpu(gau, device="cuda") -> GaussianDataHIP:
    """renderer_cuda.py:87-98: one H2D copy per array; sh reshaped to (P, M, 3)."""
    def up(a):
        return torch.as_tensor(np.ascontiguousarray(a)).float().to(device).requires_grad_(False)

    g = GaussianDataHIP(xyz=up(gau.xyz), rot=up(gau.rot), scale=up(gau.scale),
                        opacity=up(gau.opacity), sh=up(gau.sh))
    g.sh = g.sh.reshape(len(g), -1, 3).contiguous()
    return g


class HIPRenderer(GaussianRenderBase):
    """CUDARenderer's behaviour on the MI355X rasterizer (no GL)."""

    def __init__(self, w, h, device="cuda", tile_rows=None):
        super().__init__()
        self.device = torch.device(device)
        self.raster_settings = {
            "image_height": int(h),
            "image_width": int(w),
            "tanfovx": 1,
            "tanfovy": 1,
            "bg": torch.Tensor([0., 0., 0]).float().to(self.device),
            "scale_modifier": 1.,
            "viewmatrix": None,
            "projmatrix": None,
            "sh_degree": 3,
            "campos": None,
            "prefiltered": False,
            "debug": False,
        }
        self.tile_rows = tile_rows  # optional (begin, end) strip of 16-px tile rows
        self.render_mod = 3
        self._warned_mod = False
        self._view_gl = None   # the last pose's GL view (math layout), for the disparity mode
        self._proj_gl = None
        self.image = None
        self.radii = None

    def update_gaussian_data(self, gaus):
        """renderer_cuda.py:135-137 (host GaussianData -> device); a GaussianDataHIP already on
        the device (e.g. ply.load_ply(path, device=...)) is used as is."""
        self.gaussians = gaus if isinstance(gaus, GaussianDataHIP) else gaus_hip_from_cpu(gaus, self.device)
        self.raster_settings["sh_degree"] = int(np.round(np.sqrt(self.gaussians.sh_dim))) - 1

    def sort_and_update(self, camera, use_file=False, pose=None):
        pass  # the rasterizer sorts on the device every frame

    def set_scale_modifier(self, modifier):
        self.raster_settings["scale_modifier"] = float(modifier)

    def set_render_mod(self, mod: int):
        """Render modes of the GL backend (gau_vert.glsl / gau_frag.glsl; the viewer passes
        g_render_mode - 3, main.py:1010-1014).  The CUDA backend ignores them
        (renderer_cuda.py:145-146); this backend implements the two the stereo capture uses:
        mod >= 0 caps the SH degree at mod ("SH:0~k", gau_vert.glsl:217-247) and mod == -1
        renders the disparity image (per-Gaussian disparity grey, Gaussians scaled by 1.2,
        gau_vert.glsl:152-156, 182-207).  The ball / billboard modes (-2, -3, -4) render as the
        default mode, as in the CUDA backend, with a one-time warning."""
        mod = int(mod)
        if mod < -1 and not self._warned_mod:
            import warnings
            warnings.warn(f"render mode {mod} (ball / billboard shading) is GL-only; "
                          "rendering the default SH colours", stacklevel=2)
            self._warned_mod = True
        self.render_mod = mod

    def set_render_reso(self, w, h):
        self.raster_settings["image_height"] = int(h)
        self.raster_settings["image_width"] = int(w)

    def update_camera_pose(self, camera, use_file=False, pose=None):
        if use_file:
            view_mat = camera.get_view_matrix(True, pose["camera_front"], pose["camera_position"],
                                              pose["camera_up"], pose["camera_view"])
            camera.position = pose["camera_position"]
        else:
            view_mat = camera.get_view_matrix(True)
        view_mat = np.array(view_mat, dtype=np.float32)
        self._view_gl = view_mat.copy()
        self._proj_gl = np.array(camera.get_project_matrix(), dtype=np.float32)
        view_mat[[0, 2], :] = -view_mat[[0, 2], :]
        proj = camera.get_project_matrix() @ view_mat
        self.raster_settings["viewmatrix"] = self._upload(view_mat.T)
        self.raster_settings["campos"] = self._upload(camera.position)
        self.raster_settings["projmatrix"] = self._upload(proj.T)

    def _upload(self, a) -> torch.Tensor:
        # contiguous float32 on the host first: a transposed (strided) host tensor would make
        # .to() stage it and launch a device-side permute copy for every matrix
        return torch.from_numpy(np.ascontiguousarray(np.asarray(a), dtype=np.float32)).to(self.device)

    def update_camera_intrin(self, camera):
        view_matrix = np.array(camera.get_view_matrix(), dtype=np.float32)
        view_matrix[[0, 2], :] = -view_matrix[[0, 2], :]
        proj = camera.get_project_matrix() @ view_matrix
        self.raster_settings["projmatrix"] = self._upload(proj.T)
        hfovx, hfovy, focal = camera.get_htanfovxy_focal()
        self.raster_settings["tanfovx"] = hfovx
        self.raster_settings["tanfovy"] = hfovy

    def draw(self):
        settings = dict(self.raster_settings)
        g = self.gaussians
        shs, colors = g.sh, None
        if self.render_mod == -1:
            if self._view_gl is None:
                raise RuntimeError("disparity mode needs update_camera_pose first")
            from .stereo import DISPARITY_SCALE, disparity_colors
            colors = disparity_colors(g.xyz, self._view_gl, self._proj_gl)
            shs = None
            settings["scale_modifier"] = settings["scale_modifier"] * DISPARITY_SCALE
        elif self.render_mod >= 0:
            settings["sh_degree"] = min(settings["sh_degree"], self.render_mod)
        rs = GaussianRasterizationSettings(**settings)
        with torch.no_grad():
            if self.tile_rows is None:
                img, radii = GaussianRasterizer(raster_settings=rs)(
                    means3D=g.xyz, means2D=None, shs=shs, colors_precomp=colors,
                    opacities=g.opacity, scales=g.scale, rotations=g.rot, cov3D_precomp=None)
            else:
                res = rasterize_gaussians_native(
                    rs.bg, g.xyz, colors, g.opacity, g.scale, g.rot, rs.scale_modifier, None,
                    rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height,
                    rs.image_width, shs, rs.sh_degree, rs.campos, rs.prefiltered, rs.debug,
                    tile_rows=self.tile_rows)
                img, radii = res.color, res.radii
        self.image, self.radii = img, radii
        return img

    def rgba(self) -> torch.Tensor:
        """renderer_cuda.py:226-228: (3,H,W) -> (H,W,4) with alpha = 1 (one device pack
        kernel, gsr_pack_image)."""
        from .stereo import pack_image
        return pack_image(self.image, "rgba_f32")


# --- sort backend --------------------------------------------------------------------------
_sort_cache = {"id": None, "xyz": None}


def _sort_gaussian_hip(gaus, view_mat, device="cuda"):
    """renderer_ogl.py:10-53 contract on the device: view-space z of every Gaussian, stable
    ascending argsort (a device LSD radix sort), int32 (P, 1) numpy result.  xyz is uploaded
    once per GaussianData object (the torch backend's cache, renderer_ogl.py:43-45, is never
    read -- it re-uploads every call at :47)."""
    dev = torch.device(device)
    if _sort_cache["id"] != id(gaus) or _sort_cache["xyz"] is None or _sort_cache["xyz"].device != dev:
        _sort_cache["xyz"] = torch.as_tensor(np.ascontiguousarray(gaus.xyz, dtype=np.float32)).to(dev)
        _sort_cache["id"] = id(gaus)
    index = depth_argsort(_sort_cache["xyz"], view_mat)
    return index.cpu().numpy().reshape(-1, 1)


def depth_argsort(xyz: torch.Tensor, view_mat, return_depth: bool = False):
    """Device depth argsort: xyz (P,3) device float32, view_mat host 4x4 math layout."""
    if not xyz.is_cuda:
        raise RuntimeError("depth_argsort needs a device tensor")
    xyz = xyz.float().contiguous()
    P = int(xyz.shape[0])
    dev = xyz.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    view = np.ascontiguousarray(np.asarray(view_mat, dtype=np.float32).reshape(16))
    out = torch.empty((P,), dtype=torch.int32, device=dev)
    depth = torch.empty((P,), dtype=torch.float32, device=dev) if return_depth else None
    lib = _lib.load_library()
    with torch.cuda.device(idx):
        _lib.check(lib.gsr_depth_argsort(
            _lib.context(idx), xyz.data_ptr(), P,
            view.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), _lib.ptr(out), _lib.ptr(depth),
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "gsr_depth_argsort")
    return (out, depth) if return_depth else out
