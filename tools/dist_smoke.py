"""Two ranks on ONE GPU through RCCL: exercises bench.py's multi-GPU frame loop (StripBalancer +
StripGather + tile_row_pairs) end to end on a 1-GPU box and checks the gathered frame against a
full-frame render.  Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr
127.0.0.1 tools/dist_smoke.py  (diagnostic; RCCL may refuse two ranks on one device)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import Scene  # noqa: E402
from gaussiansplattingviewer_amd.rasterizer import tile_row_pairs  # noqa: E402
from gaussiansplattingviewer_amd.strips import StripBalancer, StripGather, strip_pixel_rows  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group(os.environ.get("BACKEND", "nccl"), rank=rank, world_size=world,
                            device_id=dev)
    scene = Scene("c2", dev)
    H, W = scene.H, scene.W
    gy, gx = (H + 15) // 16, (W + 15) // 16
    bal = StripBalancer(gy, gx, world, rank, device=dev, every=2, lag=1)
    gat = StripGather(H, W, world, rank, device=dev, depth=2)
    full = scene.render(0).color.clone() if rank == 0 else None
    frames = []
    for i in range(6):
        if len(gat.pending) == 1:
            f = gat.finish()
            if rank == 0:
                frames.append(f.clone())
        lay = bal.layout(i)
        mine = lay[rank]
        buf = gat.next_buffer(strip_pixel_rows(mine, H)[1])
        scene.render(i, mine, out_color=buf)
        gat.submit(buf, lay)
        bal.observe(i, tile_row_pairs(mine[1] - mine[0]))
    f = gat.finish()
    if rank == 0:
        frames.append(f.clone())
        for k, fr in enumerate(frames):
            assert torch.equal(fr.view(torch.int32), full.view(torch.int32)), f"frame {k} differs"
        print(f"dist smoke ok: {len(frames)} frames, layouts {bal.history}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
