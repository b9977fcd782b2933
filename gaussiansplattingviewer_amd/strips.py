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


class StripGather:
    """Pipelined strip gather for a stream of frames: `submit(strip)` starts the asynchronous
    gather of one frame's strips to rank 0 (RCCL runs it on its own stream, after the render
    that produced the strip) and returns at once; `finish()` waits for the oldest submitted
    frame and returns it on rank 0 (None elsewhere).  Submitting frame i+1 before finishing
    frame i overlaps the gather with the next render, as a display swap chain would.

    Buffers are allocated once: a flat send buffer per in-flight frame holding the strip's
    (3, rows_me, W) planes back to back (padded to the tallest strip), and on rank 0 the
    (world, 3 * hmax * W) receive block; the frame is assembled with one `cat`.
    `next_buffer()` hands out the next send buffer as a (3, rows_me, W) view, so a renderer
    can write its strip straight into it (`submit` then moves no bytes on this rank).
    """

    def __init__(self, H: int, W: int, world: int, rank: int, dtype=torch.float32,
                 device=None, group=None, depth: int = 2):
        gy = (H + 15) // 16
        self.H, self.W, self.world, self.rank, self.group = H, W, world, rank, group
        self.layout = [strip_pixel_rows(strip_rows(gy, world, r), H) for r in range(world)]
        self.hmax = max(rows for _, rows in self.layout)
        self.rows_me = self.layout[rank][1]
        n = 3 * self.hmax * W
        self.slots = [{
            "send": torch.zeros((n,), dtype=dtype, device=device),
            "recv": (torch.empty((world, n), dtype=dtype, device=device)
                     if rank == 0 else None),
            "work": None,
        } for _ in range(depth)]
        self.next_slot = 0
        self.pending = []  # (slot, work)

    def _strip_view(self, flat: torch.Tensor, rows: int) -> torch.Tensor:
        return flat[:3 * rows * self.W].view(3, rows, self.W)

    def next_buffer(self) -> torch.Tensor:
        """The (3, rows_me, W) send view the next `submit` uses, ordered on the current
        stream after the gather that last read it."""
        slot = self.slots[self.next_slot]
        if slot["work"] is not None:
            slot["work"].wait()  # the current stream waits for the previous gather of it
            slot["work"] = None
        return self._strip_view(slot["send"], self.rows_me)

    def submit(self, strip: torch.Tensor) -> None:
        if strip.shape != (3, self.rows_me, self.W):
            raise ValueError(f"strip shape {tuple(strip.shape)} != (3, {self.rows_me}, {self.W})")
        if len(self.pending) == len(self.slots):
            raise RuntimeError("StripGather: every slot is in flight; call finish() first")
        buf = self.next_buffer()
        slot = self.slots[self.next_slot]
        self.next_slot = (self.next_slot + 1) % len(self.slots)
        if strip.data_ptr() != buf.data_ptr():
            buf.copy_(strip)
        parts = list(slot["recv"].unbind(0)) if self.rank == 0 else None
        work = dist.gather(slot["send"], parts, dst=0, group=self.group, async_op=True)
        slot["work"] = work
        self.pending.append((slot, work))

    def finish(self) -> torch.Tensor | None:
        slot, work = self.pending.pop(0)
        work.wait()
        if self.rank != 0:
            return None
        recv = slot["recv"]
        return torch.cat([self._strip_view(recv[r], rows)
                          for r, (_, rows) in enumerate(self.layout) if rows], dim=1)


def render_strips(render_fn, H: int, W: int, world: int, rank: int, group=None):
    """Render this rank's strip with `render_fn(tile_rows) -> (3, rows, W) tensor` and gather
    the frame on rank 0 (None elsewhere)."""
    gy = (H + 15) // 16
    rows = strip_rows(gy, world, rank)
    strip = render_fn(rows)
    if world == 1:
        return strip
    return gather_strips(strip, H, W, world, rank, group)
