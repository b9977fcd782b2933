"""Lab probe: frame rates of one process as the second streams of its context slots are created
and destroyed (GSR_OPT_SECOND_STREAM) around FramePipeline depths 2 and 4, at C3.
argv: scenario -- 'prior' renders on slot 0 before the pipeline exists, 'prior_destroy' also
destroys that second stream before creating the pipeline, 'fresh' renders nothing before it,
'timing' is 'fresh' with the in-flight blend events (gsr_set_timing 2) bench.py records."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from bench import Scene  # noqa: E402
from gaussiansplattingviewer_amd import _lib  # noqa: E402
from gaussiansplattingviewer_amd.pipeline import FramePipeline  # noqa: E402

dev = torch.device("cuda", 0)
scene = Scene("c3", dev)
lib = _lib.load_library()
mode = sys.argv[1]


def serial(n=100):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        scene.render(i)
    torch.cuda.synchronize()
    return round(1e3 * (time.perf_counter() - t) / n, 4)


def inflight(pipe, n=400):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        with pipe.frame() as slot:
            scene.render(i, slot=slot)
    torch.cuda.synchronize()
    return round(n / (time.perf_counter() - t), 1)


def opt(slot, v):
    _lib.check(lib.gsr_set_option(_lib.context(0, slot), _lib.GSR_OPT_SECOND_STREAM, v), "opt")


if mode in ("prior", "prior_destroy"):
    print(mode, "serial ms before the pipeline:", serial(), serial())
if mode == "prior_destroy":  # slot 0's second stream destroyed before the pipeline's streams exist
    opt(0, 0)
p4 = FramePipeline(4, dev)
ctx0 = _lib.context(0, 0)
if mode == "timing":
    _lib.check(lib.gsr_set_timing(ctx0, 2), "timing")
print(mode, "fps depth 4:", inflight(p4), inflight(p4), inflight(p4, 1000))
if mode == "timing":
    _lib.check(lib.gsr_set_timing(ctx0, 0), "timing")
print(mode, "serial ms one stream:", serial())
opt(0, 1)
print(mode, "serial ms two streams:", serial(), serial(), serial())
opt(0, 0)
print(mode, "fps depth 4 again:", inflight(p4, 1000))
