"""Lab check: a hash of the rendered images of a few configs (frames 0 and 7, full and strip),
so two library builds (GSR_LIB) can be compared for bit-identical output on the GPU box."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import Scene  # noqa: E402

dev = torch.device("cuda", 0)
h = hashlib.sha256()
for cfg in ("c1", "c2", "c3", "c3r"):
    sc = Scene(cfg, dev)
    for step in (0, 7):
        for rows in (None, (3, 11)):
            img = sc.render(step, rows).color
            torch.cuda.synchronize()
            h.update(img.contiguous().view(torch.int32).cpu().numpy().tobytes())
print(os.environ.get("GSR_LIB", "in-tree"), h.hexdigest()[:16])
