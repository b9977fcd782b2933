"""The depth sort alone (gsr_depth_argsort, no other stream busy): P keys with depths in [2, 6)
(D = 24, two passes, as at C3).  Run under `rocprofv3 --kernel-trace --stats` to read each
k_ds_* kernel's duration without the colour pass beside it.

Usage: python tools/micro/sort_alone.py [P] [iters]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gaussiansplattingviewer_amd.renderer import depth_argsort  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rng = np.random.default_rng(0)
xyz = rng.uniform(-1, 1, (P, 3)).astype(np.float32)
xyz[:, 2] = rng.uniform(2, 6, P)
dev = torch.device("cuda", 0)
x = torch.as_tensor(xyz).to(dev)
view = np.eye(4, dtype=np.float32)
out = depth_argsort(x, view)
ref = np.argsort(xyz[:, 2], kind="stable")
assert np.array_equal(out.cpu().numpy(), ref), "sort mismatch"
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(iters):
    depth_argsort(x, view)
torch.cuda.synchronize()
print(f"P={P}: {(time.perf_counter() - t) / iters * 1e6:.1f} us per depth_argsort call (host loop)")
