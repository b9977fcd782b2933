"""Image-space strip partition of one frame across the GPUs of a node (one process per GPU).

The reference renders every frame on one device (renderer_cuda.py:205-224).  Here the frame's
16-px tile rows are split into `world` contiguous strips; every rank holds all Gaussians,
runs the full preprocess + depth sort, and bins / sorts / blends only the pairs that fall in
its strip.  Per-tile work depends only on that tile's depth-sorted list, so each strip is
bit-identical to the same rows of a single-GPU frame.  Rank 0 then gathers the strips with
one collective (torch.distributed `gather`, i.e. RCCL send/recv over xGMI on MI355X; gloo on
CPU in the tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def strip_rows(grid_y: int, world: int, rank: int) -> tuple[int, int]:
    """Tile rows [begin, end) of `rank`: the first grid_y % world ranks get one extra row."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    base, rem = divmod(grid_y, world)
    begin = rank * base + min(rank, rem)
    end = begin + base + (1 if rank < rem else 0)
    return begin, end


def strip_pixel_rows(tile_rows: tuple[int, int], H: int) -> tuple[int, int]:
    """(y0, rows) of the strip in the full image."""
    y0 = tile_rows[0] * 16
    return y0, max(0, min(H, tile_rows[1] * 16) - y0)


def gather_strips(strip: torch.Tensor, H: int, W: int, world: int, rank: int,
                  group=None) -> torch.Tensor | None:
    """Gather every rank's (3, rows_r, W) strip into the (3, H, W) frame on rank 0.

    Strips are padded to the tallest strip so one `gather` moves them all; rank 0 copies the
    valid rows into place.  Returns the frame on rank 0 and None elsewhere."""
    gy = (H + 15) // 16
    layout = [strip_pixel_rows(strip_rows(gy, world, r), H) for r in range(world)]
    hmax = max(rows for _, rows in layout)
    rows_me = layout[rank][1]
    if strip.shape != (3, rows_me, W):
        raise ValueError(f"strip shape {tuple(strip.shape)} != (3, {rows_me}, {W})")
    if rows_me == hmax:
        send = strip.contiguous()
    else:
        send = torch.zeros((3, hmax, W), dtype=strip.dtype, device=strip.device)
        send[:, :rows_me].copy_(strip)
    if rank == 0:
        parts = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, parts, dst=0, group=group)
        frame = torch.empty((3, H, W), dtype=strip.dtype, device=strip.device)
        for (y0, rows), part in zip(layout, parts):
            if rows:
                frame[:, y0:y0 + rows].copy_(part[:, :rows])
        return frame
    dist.gather(send, None, dst=0, group=group)
    return None


def render_strips(render_fn, H: int, W: int, world: int, rank: int, group=None):
    """Render this rank's strip with `render_fn(tile_rows) -> (3, rows, W) tensor` and gather
    the frame on rank 0 (None elsewhere)."""
    gy = (H + 15) // 16
    rows = strip_rows(gy, world, rank)
    strip = render_fn(rows)
    if world == 1:
        return strip
    return gather_strips(strip, H, W, world, rank, group)
