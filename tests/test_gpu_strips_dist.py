"""GPU, two ranks on one device (gloo carries the GPU tensors; RCCL refuses two ranks on one
GPU): bench.py's multi-GPU frame loop end to end -- StripBalancer boundaries from
gsr_tile_row_pairs, strips rendered by the HIP rasterizer straight into StripGather's send
buffers, received into rank 0's frame -- and every gathered frame bit-identical to a
single-GPU render of the whole frame."""
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path, depth):
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    from bench import Scene
    from gaussiansplattingviewer_amd import _lib
    from gaussiansplattingviewer_amd.pipeline import FramePipeline
    from gaussiansplattingviewer_amd.rasterizer import tile_row_pairs
    from gaussiansplattingviewer_amd.strips import StripBalancer, StripGather, strip_pixel_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = Scene("c2", dev)
        H, W = scene.H, scene.W
        gy, gx = (H + 15) // 16, (W + 15) // 16
        bal = StripBalancer(gy, gx, world, rank, device=dev, every=2, lag=1)
        gat = StripGather(H, W, world, rank, device=dev, depth=depth + 1)
        full = scene.render(0).color.clone() if rank == 0 else None
        torch.cuda.synchronize()
        # depth 4: bench.py's strip mode below 4M Gaussians -- four one-stream frames in flight
        # with the deferred-K chains (GSR_OPT_FRAME_GRAPHS 2), no radii
        pipe = FramePipeline(depth, dev)
        for slot in range(depth):
            _lib.set_option(_lib.context(0, slot), _lib.GSR_OPT_FRAME_GRAPHS,
                            2 if depth > 1 else 0)
        frames = []
        for i in range(6):
            with pipe.frame() as slot:
                if len(gat.pending) == len(gat.slots) - 1:
                    f = gat.finish()
                    if rank == 0:
                        frames.append(f.clone())
                lay = bal.layout(i)
                mine = lay[rank]
                buf = gat.next_buffer(strip_pixel_rows(mine, H)[1])
                scene.render(i, mine, slot, out_color=buf, radii=depth == 1)
                gat.submit(buf, lay)
                bal.observe(i, tile_row_pairs(mine[1] - mine[0], 0, slot))
        while gat.pending:
            f = gat.finish()
            if rank == 0:
                frames.append(f.clone())
        torch.cuda.synchronize()
        for slot in range(depth):
            _lib.set_option(_lib.context(0, slot), _lib.GSR_OPT_FRAME_GRAPHS, 0)
        pipe.close()
        if rank == 0:
            ok = [bool(torch.equal(fr.view(torch.int32), full.view(torch.int32))) for fr in frames]
            np.save(out_path, np.array(ok + [len(bal.history)], dtype=np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("depth", [1, 4])
def test_two_rank_strip_frames_equal_full_frame(tmp_path, gpu, depth):
    import numpy as np
    import torch.multiprocessing as mp
    out = str(tmp_path / "ok.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out, depth), nprocs=2, join=True,
                       start_method="spawn")
    res = np.load(out)
    assert res[:-1].all() and len(res) == 7, res
    assert res[-1] >= 2  # the balancer re-split (same layout on both ranks, or the frames differ)
