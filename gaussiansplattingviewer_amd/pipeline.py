"""Frames in flight: overlap the forward of frame i+1 with the end of frame i on one device.

The reference draws one frame at a time on the legacy default stream (renderer_cuda.py:205-258,
`cu.cudaStreamLegacy` at :231), so the GPU idles whenever the frame's critical path is
latency-bound.  On MI355X the two halves of a frame have opposite profiles: the preprocess and
the depth sort are short dependent launches that leave most of the 256 CUs idle, while the
blend saturates the VALUs of every CU.  `FramePipeline` gives each in-flight frame its own
stream and its own `gsr_context` slot (workspace + second stream, `_lib.context(dev, slot)`),
so the next frame's preprocess / sort / binning fill the CUs the current blend leaves free.
At depth >= 3 each frame keeps all its work on its own stream (no second stream), so the frames
in flight never share the process's four hardware queues.
Every frame is still rendered completely and bit-identically to a serial forward (tested):
only the order in which the GPU interleaves independent frames changes, as in a swap chain.
"""
from __future__ import annotations

import torch


class FramePipeline:
    """Round-robin over `depth` (stream, context slot) pairs of one device.

    Usage::

        pipe = FramePipeline(depth=2, device=dev)
        for cam in cameras:
            with pipe.frame() as slot:          # enters the frame's stream
                res = rasterize_gaussians_native(..., slot=slot)
            ...
        pipe.close()                            # waits; restores slot 0's options

    Frame i runs on stream i % depth; slot 0 is the caller's current stream, so depth=1 is the
    serial forward.  A consumer on another stream must order itself after the frame
    (`wait(stream_of_frame)`); `torch.cuda.synchronize()` waits for all of them.
    """

    def __init__(self, depth: int = 2, device=None, graphs: bool = False,
                 second_stream: bool | None = None):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.device = dev
        self.depth = depth
        self.count = 0
        self.graphs = bool(graphs)
        # second_stream (gsr.h GSR_OPT_SECOND_STREAM; default: off at depth >= 3 without graphs):
        # a frame's tile ranges, blend order and colour on its context's second stream, or in
        # order on the frame's own stream.  The process has GPU_MAX_HW_QUEUES = 4 hardware
        # queues: two frames of two streams each fill them, and so do four frames of one stream
        # each -- which keeps more independent work beside every blend (C3 3,955-3,975 ->
        # 4,100-4,130 frames/s; four two-stream frames 3,850-3,900, three 3,910, and more
        # hardware queues do not help: profiles/r05z3_ab_hw_queues.txt, DESIGN.md decision 13).
        self.second_stream = (not (depth >= 3 and not self.graphs) if second_stream is None
                              else bool(second_stream))
        self.streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                            for _ in range(depth - 1)]
        # graphs=True: frame graphs (gsr.h GSR_OPT_FRAME_GRAPHS 1) on the slots' contexts; the
        # host queues a frame in a few graph launches and reads K after the whole frame is
        # queued.  With two frames in flight that pays on strip frames (a C3 3/8 strip 8.5-10.8k
        # frames/s run to run -> a steady 10.5k, the multi-GPU ranks' regime) and on a tiny scene
        # (the P=2000 host loop 86 -> 63 us), but not on full frames (C3 +1.4 %, C5 and c3r
        # -2 %, C4 even; profiles/r05l_ab_frame_graphs.txt, r05o_ab_graphs_configs.txt), and a
        # serial frame pays ~15 us of GPU time for graph dispatch.  Images are bit-identical
        # either way (tests/test_gpu_frame_graphs.py).
        # Slot 0 is the process-wide context the caller's own forwards (GaussianRasterizer, `_C`)
        # render with: its two options are saved here and restored by close(), so serial callers
        # after the pipeline get back the mode they had.
        from . import _lib
        index = dev.index if dev.index is not None else torch.cuda.current_device()
        self._index = index
        opts = (_lib.GSR_OPT_FRAME_GRAPHS, _lib.GSR_OPT_SECOND_STREAM)
        self._slot0_saved = {o: _lib.get_option(_lib.context(index, 0), o) for o in opts}
        for slot in range(depth):
            ctx = _lib.context(index, slot)
            _lib.set_option(ctx, _lib.GSR_OPT_FRAME_GRAPHS, int(self.graphs))
            _lib.set_option(ctx, _lib.GSR_OPT_SECOND_STREAM, int(self.second_stream))

    def frame(self):
        """Context manager for the next frame: enters its stream, yields its context slot."""
        slot = self.count % self.depth
        self.count += 1
        return _FrameScope(self.streams[slot], slot)

    @property
    def last_stream(self) -> torch.cuda.Stream:
        return self.streams[(self.count - 1) % self.depth]

    def wait_last(self, stream: torch.cuda.Stream | None = None) -> None:
        """Order `stream` (default: the current stream) after the most recent frame."""
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.last_stream)

    def synchronize(self) -> None:
        for s in self.streams:
            s.synchronize()

    def close(self) -> None:
        """Waits for the frames in flight and restores slot 0's options (idempotent)."""
        if self._slot0_saved is None:
            return
        from . import _lib
        self.synchronize()
        ctx = _lib.context(self._index, 0)
        for o, v in self._slot0_saved.items():
            _lib.set_option(ctx, o, v)
        self._slot0_saved = None

    def __enter__(self) -> "FramePipeline":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


class _FrameScope:
    def __init__(self, stream, slot):
        self.stream, self.slot = stream, slot
        self._cm = None

    def __enter__(self) -> int:
        self._cm = torch.cuda.stream(self.stream)
        self._cm.__enter__()
        return self.slot

    def __exit__(self, *exc):
        return self._cm.__exit__(*exc)
