"""Host cost of one forward call (Python wrapper + C ABI + HIP launches), measured on a tiny
scene whose GPU work is negligible: frames/s here is the host-side ceiling of the frame loop."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians  # noqa: E402
from gaussiansplattingviewer_amd.pipeline import FramePipeline  # noqa: E402
from gaussiansplattingviewer_amd.rasterizer import rasterize_gaussians_native  # noqa: E402

dev = torch.device("cuda", 0)
P = int(os.environ.get("P", "2000"))
W, H = 1920, 1080
g = synthetic_gaussians(P, 3, 0)
up = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)  # noqa: E731
xyz, rot, scale, opac = up(g.xyz), up(g.rot), up(g.scale), up(g.opacity)
sh = up(g.sh).reshape(P, -1, 3).contiguous()
view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H))
view, proj, campos, bg = up(view), up(proj), up(campos), torch.zeros(3, device=dev)
# GSR_GRAPHS=1: frame graphs on (GSR_OPT_FRAME_GRAPHS) for every slot
from gaussiansplattingviewer_amd import _lib  # noqa: E402
for _slot in (0, 1):
    _lib.check(_lib.load_library().gsr_set_option(_lib.context(0, _slot), _lib.GSR_OPT_FRAME_GRAPHS,
                                                   int(os.environ.get("GSR_GRAPHS", "0"))),
               "gsr_set_option")
for depth in (1, 2):
    pipe = FramePipeline(depth, dev)
    for it in range(2):
        n = 300
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            with pipe.frame() as slot:
                rasterize_gaussians_native(bg, xyz, None, opac, scale, rot, 1.0, None, view, proj,
                                           tx, ty, H, W, sh, 3, campos, False, False, slot=slot)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"P={P} inflight={depth}: {1e6 * (t1 - t0) / n:.1f} us/frame host loop, "
          f"{1e6 * (t2 - t0) / n:.1f} us/frame incl. drain")

# The C ABI alone (structs built once): the HIP launch + K-wait share of the host cost.
import ctypes  # noqa: E402
from gaussiansplattingviewer_amd import _lib  # noqa: E402

lib = _lib.load_library()
ctx = _lib.context(0)
color = torch.empty((3, H, W), device=dev)
radii = torch.empty((P,), dtype=torch.int32, device=dev)
gs = _lib.GsrGaussians(P=P, D=3, M=16, scale_modifier=1.0, means3D=xyz.data_ptr(),
                       scales=scale.data_ptr(), rotations=rot.data_ptr(),
                       opacities=opac.data_ptr(), shs=sh.data_ptr(), colors_precomp=None,
                       cov3D_precomp=None)
st = _lib.GsrRasterSettings(image_width=W, image_height=H, tanfovx=float(tx), tanfovy=float(ty),
                            viewmatrix=view.data_ptr(), projmatrix=proj.data_ptr(),
                            campos=campos.data_ptr(), bg=bg.data_ptr(), tile_row_begin=0,
                            tile_row_end=0, prefiltered=0, debug=0)
out = _lib.GsrOutputs(color=color.data_ptr(), radii=radii.data_ptr())
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
for it in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(300):
        lib.gsr_forward(ctx, ctypes.byref(gs), ctypes.byref(st), ctypes.byref(out), stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
print(f"C ABI only: {1e6 * (t1 - t0) / 300:.1f} us/frame host loop")
