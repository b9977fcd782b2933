"""Image-space strip partition of one frame across the GPUs of a node (one process per GPU).

The reference renders every frame on one device (renderer_cuda.py:205-224).  Here the frame's
16-px tile rows are split into `world` contiguous strips; every rank holds all Gaussians,
runs the full preprocess + depth sort, and bins / sorts / blends only the pairs that fall in
its strip.  Per-tile work depends only on that tile's depth-sorted list, so each strip is
bit-identical to the same rows of a single-GPU frame, wherever the boundaries fall.

* Boundaries: equal tile-row counts at first (`strip_layout`); `StripBalancer` then moves them
  so every strip carries about the same blend work -- the pair counts of the tile rows in a
  recent frame (`gsr_tile_row_pairs`, summed over the ranks with one small all-reduce) plus a
  per-tile constant -- since a real scene's splats crowd into part of the image.
* Gather: rank 0 receives every strip straight into its (3, H, W) frame, one point-to-point
  message per colour plane (a CHW strip is three contiguous row blocks of the frame), grouped
  into one `batch_isend_irecv` (RCCL send/recv over xGMI on MI355X; gloo on CPU in the tests).
  No padding, no `cat`: the only copy is rank 0's own strip into the frame.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

TILE = 16


def strip_rows(grid_y: int, world: int, rank: int) -> tuple[int, int]:
    """Tile rows [begin, end) of `rank` in the equal split: the first grid_y % world ranks get
    one extra row."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    base, rem = divmod(grid_y, world)
    begin = rank * base + min(rank, rem)
    end = begin + base + (1 if rank < rem else 0)
    return begin, end


def strip_layout(grid_y: int, world: int) -> list[tuple[int, int]]:
    """The equal split of every rank."""
    return [strip_rows(grid_y, world, r) for r in range(world)]


def balanced_layout(row_costs, world: int) -> list[tuple[int, int]]:
    """Contiguous tile-row strips of about equal total cost: boundary k sits at the first row
    where the cost prefix reaches k / world of the total, kept so that every strip has >= 1
    row while rows remain.  Exact integer arithmetic, so every rank computes the same split."""
    c = np.asarray(row_costs, dtype=np.int64)
    gy = len(c)
    if world < 1:
        raise ValueError("world must be >= 1")
    if gy == 0:
        return [(0, 0)] * world
    pre = np.concatenate([[0], np.cumsum(c)]) * world  # pre[i] = world * cost of rows [0, i)
    total = int(pre[-1]) // world
    bounds = [0]
    for k in range(1, world):
        b = int(np.searchsorted(pre, total * k, side="left"))
        lo = min(bounds[-1] + 1, gy)        # strip k-1 keeps at least one row
        hi = max(gy - (world - k), lo)      # and every later strip one, rows permitting
        bounds.append(min(max(b, lo), hi))
    bounds.append(gy)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def strip_pixel_rows(tile_rows: tuple[int, int], H: int) -> tuple[int, int]:
    """(y0, rows) of the strip in the full image."""
    y0 = min(H, tile_rows[0] * TILE)
    return y0, max(0, min(H, tile_rows[1] * TILE) - y0)


class StripBalancer:
    """Strip boundaries for a stream of frames.  `layout(i)` is frame i's split (identical on
    every rank); after rendering frame i a rank calls `observe(i, row_pairs)` with its strip's
    per-tile-row pair counts (a device tensor, `rasterizer.tile_row_pairs`).  Every `every`
    frames those counts are summed over the ranks with one asynchronous all-reduce of grid_y
    integers; the new split -- weights = pairs + tile_cost * grid_x per row -- takes effect
    `lag` frames later (by then the all-reduce and its copy to the host have long finished, so
    the wait is free).  world == 1 keeps the single strip."""

    def __init__(self, grid_y: int, grid_x: int, world: int, rank: int, device=None,
                 group=None, every: int = 8, lag: int = 3, tile_cost: int = 64):
        self.gy, self.gx, self.world, self.rank = grid_y, grid_x, world, rank
        self.group, self.every, self.lag, self.tile_cost = group, every, lag, tile_cost
        self.device = device
        self.current = strip_layout(grid_y, world)
        self.pending = None  # (apply_at, work, vec, host, event)
        self.history = []    # (frame, layout) of every change (diagnostics)

    def layout(self, frame: int) -> list[tuple[int, int]]:
        p = self.pending
        if p is not None and frame >= p[0]:
            _, work, vec, host, event = p
            if event is not None:
                event.synchronize()
            else:
                work.wait()
                host = vec
            costs = host.numpy().astype(np.int64) + self.tile_cost * self.gx
            self.current = balanced_layout(costs, self.world)
            self.history.append((frame, self.current))
            self.pending = None
        return self.current

    def rows(self, frame: int) -> tuple[int, int]:
        return self.layout(frame)[self.rank]

    def observe(self, frame: int, row_pairs: torch.Tensor) -> None:
        """Call on the frame's own stream (as bench.py does, inside the FramePipeline frame):
        the counts' device -> host copy is queued there behind the all-reduce, so the balancer
        takes no stream (and no hardware queue) of its own; that stream waits for the
        all-reduce once every `every` frames."""
        if self.world == 1 or frame % self.every != 0 or self.pending is not None:
            return
        b, e = self.current[self.rank]
        if row_pairs.numel() != e - b:
            raise ValueError(f"row_pairs has {row_pairs.numel()} rows, strip has {e - b}")
        vec = torch.zeros((self.gy,), dtype=torch.int32, device=row_pairs.device)
        vec[b:e].copy_(row_pairs)
        work = dist.all_reduce(vec, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if vec.is_cuda:
            host = torch.empty((self.gy,), dtype=torch.int32, pin_memory=True)
            work.wait()  # the current (frame) stream waits for the all-reduce
            host.copy_(vec, non_blocking=True)
            event = torch.cuda.Event()
            event.record()
            self.pending = (frame + self.lag, work, vec, host, event)
        else:
            self.pending = (frame + self.lag, work, vec, None, None)


def rank_stream_plan(inflight: int, second_stream: bool) -> list[str]:
    """The HIP streams one rank's frame loop uses (bench.py): the caller's stream
    and inflight - 1 FramePipeline streams, plus each in-flight context's second stream when on.
    StripBalancer and StripGather create none (RCCL's collectives run on RCCL's own streams,
    created with the communicator before these).  The plan stays within 4 streams (HIP's default
    GPU_MAX_HW_QUEUES); bench.py gives a rank of N > 1 eight queues, so RCCL's streams get
    queues of their own beside it."""
    plan = ["caller"] + [f"frame{i}" for i in range(1, inflight)]
    if second_stream:
        plan += [f"second{i}" for i in range(inflight)]
    return plan


class StripGather:
    """Pipelined gather of a stream of frames to rank 0.

    `next_buffer(rows)` hands out this rank's (3, rows, W) render target for the next frame
    (write the strip straight into it); `submit(strip, layout)` starts the frame's transfer --
    every other rank sends its three colour planes, rank 0 receives them directly into the
    rows of the slot's (3, H, W) frame and copies its own strip there -- and returns at once
    (RCCL runs it on its own streams, after the render that produced the strip); `finish()`
    waits for the oldest submitted frame and returns it on rank 0 (None elsewhere).  `depth`
    frames can be in flight; buffers are allocated once."""

    def __init__(self, H: int, W: int, world: int, rank: int, dtype=torch.float32,
                 device=None, group=None, depth: int = 2):
        self.H, self.W, self.world, self.rank, self.group = H, W, world, rank, group
        self.slots = [{
            "send": torch.zeros((3 * H * W,), dtype=dtype, device=device),
            "frame": (torch.zeros((3, H, W), dtype=dtype, device=device) if rank == 0 else None),
            "reqs": None,
        } for _ in range(depth)]
        self.next_slot = 0
        self.pending = []  # slots in flight, oldest first
        # gloo moves device tensors from its own host threads, outside stream order: a submit
        # then waits for the current stream (the render of the strip, earlier reads of the
        # frame slot it receives into) before posting the transfers
        dev = self.slots[0]["send"].device
        self.host_transport = dev.type == "cuda" and dist.get_backend(group) != "nccl"

    def next_buffer(self, rows: int) -> torch.Tensor:
        """The (3, rows, W) render target of the next `submit`, ordered on the current stream
        after the transfer that last read it."""
        slot = self.slots[self.next_slot]
        if slot["reqs"] is not None:
            if any(p is slot for p in self.pending):
                raise RuntimeError("StripGather: every slot is in flight; call finish() first")
            slot["reqs"] = None
        return slot["send"][:3 * rows * self.W].view(3, rows, self.W)

    def submit(self, strip: torch.Tensor, layout: list[tuple[int, int]]) -> None:
        if len(layout) != self.world:
            raise ValueError("layout needs one tile-row range per rank")
        y0, rows = strip_pixel_rows(layout[self.rank], self.H)
        if strip.shape != (3, rows, self.W):
            raise ValueError(f"strip shape {tuple(strip.shape)} != (3, {rows}, {self.W})")
        if len(self.pending) == len(self.slots):
            raise RuntimeError("StripGather: every slot is in flight; call finish() first")
        buf = self.next_buffer(rows)
        slot = self.slots[self.next_slot]
        self.next_slot = (self.next_slot + 1) % len(self.slots)
        if rows and strip.data_ptr() != buf.data_ptr():
            buf.copy_(strip)
        ops = []
        if self.rank == 0:
            frame = slot["frame"]
            if rows:
                frame[:, y0:y0 + rows].copy_(buf)
            for r in range(1, self.world):
                ry0, rrows = strip_pixel_rows(layout[r], self.H)
                for c in range(3):
                    if rrows:
                        ops.append(dist.P2POp(dist.irecv, frame[c, ry0:ry0 + rrows], r,
                                              group=self.group))
        else:
            for c in range(3):
                if rows:
                    ops.append(dist.P2POp(dist.isend, buf[c], 0, group=self.group))
        if ops and self.host_transport:
            torch.cuda.current_stream(buf.device).synchronize()
        slot["reqs"] = dist.batch_isend_irecv(ops) if ops else []
        slot["layout"] = list(layout)
        self.pending.append(slot)

    def finish(self) -> torch.Tensor | None:
        """Wait for the oldest submitted frame; on rank 0 return it (None elsewhere).  The
        returned tensor is the slot's own frame buffer: it stays valid until that slot is
        submitted again (`depth` submits later) -- clone it to keep it longer (e.g. in a display
        queue)."""
        slot = self.pending.pop(0)
        for req in slot["reqs"]:
            req.wait()
        return slot["frame"] if self.rank == 0 else None


def gather_strips(strip: torch.Tensor, H: int, W: int, world: int, rank: int, group=None,
                  layout: list[tuple[int, int]] | None = None) -> torch.Tensor | None:
    """Gather every rank's (3, rows_r, W) strip of `layout` (default: the equal split) into
    the (3, H, W) frame on rank 0.  Returns the frame on rank 0 and None elsewhere."""
    if layout is None:
        layout = strip_layout((H + TILE - 1) // TILE, world)
    g = StripGather(H, W, world, rank, dtype=strip.dtype, device=strip.device, group=group,
                    depth=1)
    g.submit(strip, layout)
    return g.finish()


def render_strips(render_fn, H: int, W: int, world: int, rank: int, group=None,
                  layout: list[tuple[int, int]] | None = None):
    """Render this rank's strip with `render_fn(tile_rows) -> (3, rows, W) tensor` and gather
    the frame on rank 0 (None elsewhere)."""
    if layout is None:
        layout = strip_layout((H + TILE - 1) // TILE, world)
    strip = render_fn(layout[rank])
    if world == 1:
        return strip
    return gather_strips(strip, H, W, world, rank, group, layout)
