"""GPU: captured-graph frames (GSR_OPT_GRAPH, api.hip forward_graph) are bit-identical to the
stream path -- full frames and strips on a moving camera (the camera is staged per frame, the
graph replayed), strip boundaries that move (new recordings), a pair count that outgrows the
captured capacity (device-side overflow -> the frame is rendered again on the stream), the
binning state gsr_get_binning reports, and frames in flight."""
import numpy as np
import pytest
import torch

from gaussiansplattingviewer_amd import _lib
from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, orbit_eye, static_camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians
from gaussiansplattingviewer_amd.pipeline import FramePipeline
from gaussiansplattingviewer_amd.rasterizer import binning_state, rasterize_gaussians_native

pytestmark = pytest.mark.gpu

GRAPH_SLOT, STREAM_SLOT = 40, 41  # dedicated context slots (fresh contexts)


def _set_graph(dev, slot, on):
    lib = _lib.load_library()
    _lib.check(lib.gsr_set_option(_lib.context(dev.index or 0, slot), _lib.GSR_OPT_GRAPH, int(on)),
               "gsr_set_option")


def _scene(dev, P, W, H, n_frames, seed):
    g = synthetic_gaussians(P, 3, seed)
    up = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    dg = dict(xyz=up(g.xyz), rot=up(g.rot), scale=up(g.scale), opacity=up(g.opacity),
              sh=up(g.sh).reshape(P, -1, 3).contiguous())
    cams = []
    for i in range(n_frames):
        view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H, orbit_eye(i * 53, 1000)))
        cams.append(dict(view=up(view), proj=up(proj), campos=up(campos), tx=tx, ty=ty))
    return dg, cams


def _render(dg, cam, W, H, dev, slot, tile_rows=None, scale_modifier=1.0, out_color=None):
    return rasterize_gaussians_native(
        torch.zeros(3, device=dev), dg["xyz"], None, dg["opacity"], dg["scale"], dg["rot"],
        scale_modifier, None, cam["view"], cam["proj"], cam["tx"], cam["ty"], H, W, dg["sh"], 3,
        cam["campos"], False, False, slot=slot, tile_rows=tile_rows, out_color=out_color)


def _same(a, b, binning=True):
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1])
    assert torch.equal(a[2].view(torch.int32), b[2].view(torch.int32))  # bit-identical
    if binning:
        for x, y in zip(a[3], b[3]):
            assert torch.equal(x, y)


def _frame(dg, cam, W, H, dev, slot, binning=True, **kw):
    r = _render(dg, cam, W, H, dev, slot, **kw)
    st = binning_state(dev.index or 0, slot) if binning else ()
    return (r.num_rendered, r.radii.clone(), r.color.clone(), st)


@pytest.mark.parametrize("strips", [None, [(0, 30), (0, 30), (10, 25), (10, 25), (0, 30), (29, 30)]])
def test_graph_frames_equal_stream(gpu, strips):
    P, W, H, n = 80_000, 640, 480, 6
    dg, cams = _scene(gpu, P, W, H, n, seed=5)
    _set_graph(gpu, GRAPH_SLOT, True)
    _set_graph(gpu, STREAM_SLOT, False)
    # a new camera every frame (staged, the graph replayed); new boundaries re-record
    for i, cam in enumerate(cams):
        rows = strips[i] if strips else None
        a = _frame(dg, cam, W, H, gpu, GRAPH_SLOT, tile_rows=rows)
        b = _frame(dg, cam, W, H, gpu, STREAM_SLOT, tile_rows=rows)
        _same(a, b)


def test_graph_overflow_rerenders(gpu):
    """K grows ~9x (scale_modifier 3): the captured capacity overflows, the device skips the
    binning, the host grows the buffers and renders the frame again; then it shrinks back."""
    P, W, H = 60_000, 640, 480
    dg, cams = _scene(gpu, P, W, H, 1, seed=9)
    _set_graph(gpu, GRAPH_SLOT + 2, True)
    _set_graph(gpu, STREAM_SLOT + 2, False)
    for sm in (1.0, 1.0, 1.0, 3.0, 3.0, 1.0, 3.0):
        a = _frame(dg, cams[0], W, H, gpu, GRAPH_SLOT + 2, scale_modifier=sm)
        b = _frame(dg, cams[0], W, H, gpu, STREAM_SLOT + 2, scale_modifier=sm)
        _same(a, b)


def test_graph_frames_in_flight(gpu):
    """FramePipeline's two slots, graphs on, on two streams, output buffers reused
    round-robin, against serial stream-path frames."""
    P, W, H, n = 60_000, 640, 480, 8
    dg, cams = _scene(gpu, P, W, H, n, seed=13)
    _set_graph(gpu, STREAM_SLOT + 4, False)
    ref = [_frame(dg, cam, W, H, gpu, STREAM_SLOT + 4, binning=False) for cam in cams]
    pipe = FramePipeline(2, gpu)
    bufs = [torch.empty((3, H, W), device=gpu) for _ in range(3)]
    try:
        for slot in (0, 1):
            _set_graph(gpu, slot, True)
        for start in range(0, n, 3):
            got = []
            for i in range(start, min(n, start + 3)):
                with pipe.frame() as slot:
                    r = _render(dg, cams[i], W, H, gpu, slot, out_color=bufs[i % 3])
                    got.append((i, r.num_rendered, r.radii))
            torch.cuda.synchronize()
            for i, k, radii in got:
                _same((k, radii.clone(), bufs[i % 3].clone(), ()), ref[i], binning=False)
    finally:
        torch.cuda.synchronize()
        for slot in (0, 1):
            _set_graph(gpu, slot, False)
