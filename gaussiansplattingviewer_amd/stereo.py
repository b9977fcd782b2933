"""Stereo dataset capture on the device.

The fork's product is a stereo dataset: for every COLMAP pose the viewer renders the left
view, a disparity image and the right view, and saves them as left/{i}.png, depth/{i}.png and
right/{i}.png (main.py:839-923).  Upstream that only works in the GL backend (render mode -1,
FBO readbacks).  Here the same three images come from the HIP rasterizer:

* `disparity_colors` -- the per-Gaussian disparity grey of gau_vert.glsl:182-207 (HIP kernel
  `gsr_disparity_colors`), composited like any colour with the Gaussians scaled by 1.2
  (gau_vert.glsl:152-156) -- see `HIPRenderer.set_render_mod(-1)`;
* `pack_image` -- the device packer (`gsr_pack_image`): RGB8 as glReadPixels(GL_RGB,
  GL_UNSIGNED_BYTE) converts, uint16 = disparity * 65535 truncated (main.py:873-874), or the
  HWC RGBA float of renderer_cuda.py:226-228;
* `StereoCapture` -- the capture sequence of main.py:843-917 (left pose, disparity with the
  left pose still bound, right pose) on a `HIPRenderer`, returning device tensors; `save`
  writes the PNGs (PIL) the way the viewer names them.

Orientation: the viewer's CUDA path negates view rows 0 and 2 (renderer_cuda.py:189-191),
which puts NDC +y (the top of the GL framebuffer) at raster row 0.  The GL capture reads rows
bottom-up and then flips them (main.py:875-879, 911-912), so its PNG row 0 is the top as well:
the rasterizer's rows are saved as they are (flip_rows=False).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from .colmap import BASELINE, load_camera_positions

DISPARITY_SCALE = 1.2  # gau_vert.glsl:152-153: scale * scale_modifier * 1.2 in mode -1

_FORMATS = {
    "rgba_f32": (_lib.GSR_PACK_RGBA_F32, torch.float32, 4),
    "rgb8": (_lib.GSR_PACK_RGB8, torch.uint8, 3),
    "r16": (_lib.GSR_PACK_R16, torch.uint16, 0),
}


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _mat16(m) -> ctypes.Array:
    a = np.ascontiguousarray(np.asarray(m, dtype=np.float32).reshape(16))
    return (ctypes.c_float * 16)(*a.tolist())


def disparity_colors(xyz: torch.Tensor, view_gl, proj_gl, baseline: float = BASELINE,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """(P, 3) float32 device colours (d, d, d), d = |x_l - x_r| of gau_vert.glsl:182-207.
    view_gl / proj_gl: host 4x4 math-layout GL view and projection (util.py:58-105)."""
    if not (isinstance(xyz, torch.Tensor) and xyz.is_cuda):
        raise RuntimeError("disparity_colors needs a device xyz tensor (no CPU path)")
    if xyz.ndim != 2 or xyz.shape[1] != 3:
        raise RuntimeError("xyz must have dimensions (num_points, 3)")
    xyz = xyz.float().contiguous()
    P = int(xyz.shape[0])
    if out is None:
        out = torch.empty((P, 3), dtype=torch.float32, device=xyz.device)
    elif out.shape != (P, 3) or out.dtype != torch.float32 or not out.is_contiguous():
        raise RuntimeError("out must be a contiguous float32 (P, 3) tensor")
    lib = _lib.load_library()
    _lib.check(lib.gsr_disparity_colors(_lib.ptr(xyz), P, _mat16(view_gl), _mat16(proj_gl),
                                        float(baseline), _lib.ptr(out), _stream(xyz.device)),
               "gsr_disparity_colors")
    return out


def pack_image(image: torch.Tensor, fmt: str, flip_rows: bool = False,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Pack a (3, H, W) float32 device image: "rgb8" -> uint8 (H, W, 3), "r16" -> uint16 (H, W)
    from channel 0, "rgba_f32" -> float32 (H, W, 4) with alpha 1."""
    if fmt not in _FORMATS:
        raise ValueError(f"unknown format {fmt!r}; expected one of {sorted(_FORMATS)}")
    if not (isinstance(image, torch.Tensor) and image.is_cuda):
        raise RuntimeError("pack_image needs a device image (no CPU path)")
    if image.ndim != 3 or image.shape[0] != 3 or image.dtype != torch.float32:
        raise RuntimeError("image must be a float32 (3, H, W) tensor")
    image = image.contiguous()
    code, dtype, ch = _FORMATS[fmt]
    H, W = int(image.shape[1]), int(image.shape[2])
    shape = (H, W, ch) if ch else (H, W)
    if out is None:
        out = torch.empty(shape, dtype=dtype, device=image.device)
    elif tuple(out.shape) != shape or out.dtype != dtype or not out.is_contiguous():
        raise RuntimeError(f"out must be a contiguous {dtype} {shape} tensor")
    lib = _lib.load_library()
    _lib.check(lib.gsr_pack_image(_lib.ptr(image), H, W, code, int(bool(flip_rows)),
                                  _lib.ptr(out), _stream(image.device)), "gsr_pack_image")
    return out


class StereoCapture:
    """main.py:839-923 on a HIPRenderer: left RGB, disparity, right RGB for one pose.

    `render_mode` is the viewer's g_render_mode - 3 (default 3: full SH, main.py:99)."""

    def __init__(self, renderer, camera, render_mode: int = 3):
        self.renderer = renderer
        self.camera = camera
        self.render_mode = int(render_mode)

    def render(self, camera_pose) -> dict:
        """One images.txt entry -> {"left": u8 (H,W,3), "depth": u16 (H,W), "right": u8
        (H,W,3)} device tensors, in the viewer's draw order (main.py:845-900)."""
        r, cam = self.renderer, self.camera
        pose_left, pose_right = load_camera_positions(camera_pose)
        r.update_camera_intrin(cam)                       # main.py:826-827
        r.set_render_mod(self.render_mode)                 # main.py:845
        r.sort_and_update(cam, True, pose_left)
        r.update_camera_pose(cam, True, pose_left)
        left = pack_image(r.draw(), "rgb8")
        r.set_render_mod(-1)                               # main.py:867-868: left pose bound
        depth = pack_image(r.draw(), "r16")
        r.set_render_mod(self.render_mode)                 # main.py:885-889
        r.sort_and_update(cam, True, pose_right)
        r.update_camera_pose(cam, True, pose_right)
        right = pack_image(r.draw(), "rgb8")
        return {"left": left, "depth": depth, "right": right}

    @staticmethod
    def save(frames: dict, out_dir: str, scene: str, pose_index: int) -> list[str]:
        """Write left/right RGB PNGs and the 16-bit disparity PNG under
        out_dir/scene/{left,right,depth}/{pose_index}.png (main.py:701-712, 879, 916-917)."""
        from PIL import Image
        paths = []
        for kind in ("left", "depth", "right"):
            d = os.path.join(out_dir, scene, kind)
            os.makedirs(d, exist_ok=True)
            a = frames[kind].cpu().numpy()
            path = os.path.join(d, f"{pose_index}.png")
            Image.fromarray(a).save(path)
            paths.append(path)
        return paths
