"""Lab: a few frame-graph forwards of a small scene, for HIP runtime logs (AMD_LOG_LEVEL) and for
timing the graph launches against direct launches with different HIP graph settings."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gaussiansplattingviewer_amd import _lib  # noqa: E402
from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians  # noqa: E402
from gaussiansplattingviewer_amd.rasterizer import rasterize_gaussians_native  # noqa: E402

dev = torch.device("cuda", 0)
P, W, H = int(os.environ.get("P", "2000")), 1920, 1080
n = int(os.environ.get("FRAMES", "5"))
g = synthetic_gaussians(P, 3, 0)
up = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)  # noqa: E731
xyz, rot, scale, opac = up(g.xyz), up(g.rot), up(g.scale), up(g.opacity)
sh = up(g.sh).reshape(P, -1, 3).contiguous()
view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H))
view, proj, campos, bg = up(view), up(proj), up(campos), torch.zeros(3, device=dev)
for graphs in (0, 1):
    _lib.check(_lib.load_library().gsr_set_option(_lib.context(0, 0), _lib.GSR_OPT_FRAME_GRAPHS,
                                                   graphs), "gsr_set_option")
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            rasterize_gaussians_native(bg, xyz, None, opac, scale, rot, 1.0, None, view, proj, tx,
                                       ty, H, W, sh, 3, campos, False, False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
    print(f"graphs={graphs}: {1e6 * (t1 - t0) / n:.1f} us/frame host", _lib.frame_graph_stats(0, 0),
          flush=True)
