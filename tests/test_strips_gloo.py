"""CPU, world_size 2 (gloo): the strip partition + gather reassembles a frame bit-exactly.

The strips are rows of one oracle frame, so this checks the distributed plumbing (row split,
padding, gather, placement) independently of the GPU; the GPU tests check that the HIP strip
renders equal the rows of the single-GPU frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gaussiansplattingviewer_amd.strips import gather_strips, render_strips, strip_pixel_rows, strip_rows

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, H, W, frame_path, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frame = torch.from_numpy(np.load(frame_path))

        def render(tile_rows):
            y0, rows = strip_pixel_rows(tile_rows, H)
            return frame[:, y0:y0 + rows].clone()

        out = render_strips(render, H, W, world, rank)
        if rank == 0:
            np.save(result_path, out.numpy())
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W", [(2, 480, 640), (2, 522, 1160), (3, 100, 48)])
def test_gather_strips_reassembles_frame(tmp_path, oracle_mod, world, H, W):
    from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera
    from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians
    g = synthetic_gaussians(2000, 3, seed=7)
    view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H))
    frame = oracle_mod.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, W, H, shs=g.sh,
                               sh_degree=3, scales=g.scale, rotations=g.rot)["color"]
    fp, rp = tmp_path / "frame.npy", tmp_path / "out.npy"
    np.save(fp, frame)
    mp.start_processes(_worker, args=(world, _free_port(), H, W, str(fp), str(rp)), nprocs=world,
                       join=True, start_method="spawn")
    out = np.load(rp)
    assert out.shape == frame.shape
    np.testing.assert_array_equal(out.view(np.uint32), frame.view(np.uint32))


def _layouts(H, world, n):
    """A different split for every frame: the equal one, then boundaries moved around
    (including empty strips when rows run out)."""
    from gaussiansplattingviewer_amd.strips import balanced_layout, strip_layout
    gy = (H + 15) // 16
    rng = np.random.default_rng(world * 100 + H)
    out = [strip_layout(gy, world)]
    for _ in range(n - 1):
        out.append(balanced_layout(rng.integers(0, 1000, gy), world))
    return out


def _stream_worker(rank, world, port, H, W, result_path, in_place=False):
    from gaussiansplattingviewer_amd.strips import StripGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = [torch.arange(3 * H * W, dtype=torch.float32).reshape(3, H, W) * (k + 1)
                  for k in range(5)]
        layouts = _layouts(H, world, len(frames))
        sg = StripGather(H, W, world, rank, depth=2)
        got = []
        for k, f in enumerate(frames):  # pipelined: frame k's gather overlaps frame k+1
            y0, rows = strip_pixel_rows(layouts[k][rank], H)
            if in_place:  # render straight into the send buffer (the bench's path)
                buf = sg.next_buffer(rows)
                buf.copy_(f[:, y0:y0 + rows])
                sg.submit(buf, layouts[k])
            else:
                sg.submit(f[:, y0:y0 + rows].clone(), layouts[k])
            if k >= 1:
                r = sg.finish()
                got.append(None if r is None else r.clone())
        r = sg.finish()
        got.append(None if r is None else r.clone())
        if rank == 0:
            np.save(result_path, torch.stack(got).numpy())
        else:
            assert all(g is None for g in got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,in_place", [(2, 100, 48, False), (3, 100, 48, False),
                                                (3, 100, 48, True), (2, 36, 40, True),
                                                (4, 40, 24, True)])
def test_strip_gather_pipelined_stream(tmp_path, world, H, W, in_place):
    """StripGather (the bench's pipelined gather): 5 frames, two in flight, each with its own
    strip boundaries, received straight into rank 0's frame, in order and bit-exact; strips
    copied in or rendered into the send buffers."""
    rp = tmp_path / "out.npy"
    mp.start_processes(_stream_worker, args=(world, _free_port(), H, W, str(rp), in_place),
                       nprocs=world,
                       join=True, start_method="spawn")
    out = np.load(rp)
    want = np.stack([np.arange(3 * H * W, dtype=np.float32).reshape(3, H, W) * (k + 1)
                     for k in range(5)])
    np.testing.assert_array_equal(out, want)


def _balancer_worker(rank, world, port, gy, gx, result_path):
    from gaussiansplattingviewer_amd.strips import StripBalancer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the scene's pair counts per tile row: crowded at the top of the image
        costs = (np.arange(gy)[::-1] ** 2 * 50).astype(np.int32)
        bal = StripBalancer(gy, gx, world, rank, every=4, lag=2, tile_cost=8)
        seen = []
        for f in range(13):
            lay = bal.layout(f)
            seen.append([list(t) for t in lay])
            b, e = lay[rank]
            bal.observe(f, torch.from_numpy(costs[b:e].copy()))
        np.save(result_path + f".{rank}.npy", np.array(seen, dtype=np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,gy", [(2, 68), (3, 20), (4, 9)])
def test_strip_balancer_consistent_and_weighted(tmp_path, world, gy):
    """StripBalancer: every rank switches to the same cost-weighted split on the same frame
    (observe every 4 frames, applied 2 frames later), and that split is balanced_layout of the
    all-reduced row costs plus the per-tile constant."""
    from gaussiansplattingviewer_amd.strips import balanced_layout, strip_layout
    gx = 30
    rp = str(tmp_path / "lay")
    mp.start_processes(_balancer_worker, args=(world, _free_port(), gy, gx, rp), nprocs=world,
                       join=True, start_method="spawn")
    seen = [np.load(rp + f".{r}.npy") for r in range(world)]
    for r in range(1, world):
        np.testing.assert_array_equal(seen[r], seen[0])
    costs = np.arange(gy)[::-1] ** 2 * 50
    want = np.array(balanced_layout(costs + 8 * gx, world))
    np.testing.assert_array_equal(seen[0][0], np.array(strip_layout(gy, world)))
    np.testing.assert_array_equal(seen[0][1], np.array(strip_layout(gy, world)))
    np.testing.assert_array_equal(seen[0][2], want)  # observed at 0, applied at 2
    np.testing.assert_array_equal(seen[0][-1], want)
    assert not np.array_equal(want, np.array(strip_layout(gy, world)))


@pytest.mark.parametrize("seed", range(20))
def test_balanced_layout_properties(seed):
    """balanced_layout: contiguous cover of all rows, >= 1 row per strip when rows allow,
    and no strip heavier than its ideal share plus the heaviest single row."""
    from gaussiansplattingviewer_amd.strips import balanced_layout
    rng = np.random.default_rng(seed)
    gy = int(rng.integers(1, 140))
    world = int(rng.integers(1, 9))
    c = rng.integers(0, 5000, gy) * (rng.random(gy) < 0.6)
    lay = balanced_layout(c, world)
    assert len(lay) == world and lay[0][0] == 0 and lay[-1][1] == gy
    for (b0, e0), (b1, e1) in zip(lay, lay[1:]):
        assert e0 == b1 and b0 <= e0
    if gy >= world:
        assert all(e > b for b, e in lay)
    loads = [int(c[b:e].sum()) for b, e in lay]
    if c.sum() > 0 and gy >= world:
        assert max(loads) <= c.sum() / world + c.max() * 2


def _stream_count_worker(rank, world, port, gy, gx, H, W, result_path):
    """A strip rank's bench loop without the renderer (gloo): StripBalancer + StripGather over
    13 frames, with torch.cuda.Stream counted -- they must create none."""
    from gaussiansplattingviewer_amd import strips
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    created = []
    real = torch.cuda.Stream

    class Counting:
        def __new__(cls, *a, **k):
            created.append(1)
            return real(*a, **k)

    torch.cuda.Stream = Counting
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bal = strips.StripBalancer(gy, gx, world, rank, every=4, lag=2)
        gat = strips.StripGather(H, W, world, rank, depth=3)
        for f in range(13):
            if len(gat.pending) == len(gat.slots) - 1:
                gat.finish()
            lay = bal.layout(f)
            b, e = lay[rank]
            buf = gat.next_buffer(strips.strip_pixel_rows(lay[rank], H)[1])
            buf.fill_(float(rank))
            gat.submit(buf, lay)
            bal.observe(f, torch.full((e - b,), 10 + rank, dtype=torch.int32))
        while gat.pending:
            gat.finish()
        np.save(result_path + f".{rank}.npy", np.array([len(created)]))
    finally:
        torch.cuda.Stream = real
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strip_rank_stream_budget(tmp_path, world):
    """The queue budget of a strip rank: the balancer and the gather create no
    streams of their own, and the bench's strip plan (two frames in flight, each with its
    second stream) uses exactly GPU_MAX_HW_QUEUES = 4 streams; four one-stream frames too."""
    from gaussiansplattingviewer_amd.strips import rank_stream_plan
    gy, gx, H, W = 20, 12, 320, 192
    rp = str(tmp_path / "streams")
    mp.start_processes(_stream_count_worker, args=(world, _free_port(), gy, gx, H, W, rp),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        assert int(np.load(rp + f".{r}.npy")[0]) == 0
    assert len(rank_stream_plan(2, True)) == 4
    assert len(rank_stream_plan(4, False)) == 4
    assert len(rank_stream_plan(3, True)) > 4  # (the combination the bench avoids)


@pytest.mark.parametrize("world,preset,expect", [("2", None, "8"), ("8", "4", "8"), ("1", None, None),
                                                 ("2", "16", "16")])
def test_bench_rank_hw_queues(world, preset, expect):
    """bench.py gives a rank of N > 1 eight hardware queues before HIP initialises (RCCL's
    streams beside the four frame streams, DESIGN.md §5 "Queue budget"), leaves N = 1 at HIP's
    default and never lowers a larger setting."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    env["WORLD_SIZE"] = world
    if preset is not None:
        env["GPU_MAX_HW_QUEUES"] = preset
    code = ("import os, sys; sys.argv = ['bench.py']; import bench; "
            "print(os.environ.get('GPU_MAX_HW_QUEUES', 'unset'))")
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == (expect or "unset")
