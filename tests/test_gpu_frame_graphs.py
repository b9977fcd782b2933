"""GPU: frame graphs (GSR_OPT_FRAME_GRAPHS, DESIGN.md decision 12) render every frame exactly as
the direct forward does -- image bits, radii, num_rendered and the exported binning -- on moving
cameras, strips, the LSD depth sort, colours from SH of degree < 3 and precomputed colours; a
list that outgrows the capacity is re-rendered the direct way; new input tensors re-record.

Each test renders through two context slots of its own: one with frame graphs (the default) and
one with them off."""
import numpy as np
import pytest
import torch

from gaussiansplattingviewer_amd import _lib
from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, orbit_eye, static_camera
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians
from gaussiansplattingviewer_amd.rasterizer import binning_state, rasterize_gaussians_native

from gpu_helpers import set_option

pytestmark = pytest.mark.gpu

_next_slot = [20]


def _slots(dev, mode=1):
    """A fresh (graphs on, graphs off) pair of context slots; mode 1 replays recorded graphs, 2
    launches the same deferred-K chains directly; "1-one-stream" / "2-one-stream" do that on a
    context without its second stream (the second stream's chain in order on the frame's stream,
    as four frames in flight run; mode 1 records it on a stream made for the recording)."""
    on, off = _next_slot[0], _next_slot[0] + 1
    _next_slot[0] += 2
    one = isinstance(mode, str)
    set_option(dev, _lib.GSR_OPT_FRAME_GRAPHS, int(mode[0]) if one else mode, on)
    set_option(dev, _lib.GSR_OPT_FRAME_GRAPHS, 0, off)
    set_option(dev, _lib.GSR_OPT_SECOND_STREAM, 0 if one else 1, on)
    set_option(dev, _lib.GSR_OPT_SECOND_STREAM, 0 if one else 1, off)
    return on, off


def _up(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dev)


def _scene(dev, g, deg):
    P = len(g.xyz)
    return dict(xyz=_up(g.xyz, dev), rot=_up(g.rot, dev), scale=_up(g.scale, dev),
                opacity=_up(g.opacity, dev), sh=_up(g.sh, dev).reshape(P, -1, 3).contiguous(),
                deg=deg)


def _cams(dev, W, H, n, step=37):
    out = []
    for i in range(n):
        view, proj, campos, tx, ty = cuda_camera_inputs(static_camera(W, H, orbit_eye(i * step, 1000)))
        out.append(dict(view=_up(view, dev), proj=_up(proj, dev), campos=_up(campos, dev), tx=tx,
                        ty=ty))
    return out


def _render(dev, sc, cam, W, H, slot, tile_rows=None, radii=True, colors=None):
    return rasterize_gaussians_native(
        torch.zeros(3, device=dev), sc["xyz"], colors, sc["opacity"], sc["scale"], sc["rot"], 1.0,
        None, cam["view"], cam["proj"], cam["tx"], cam["ty"], H, W,
        None if colors is not None else sc["sh"], sc["deg"], cam["campos"], False, False,
        slot=slot, tile_rows=tile_rows, radii=radii)


def _same(a, b):
    assert a.num_rendered == b.num_rendered
    assert torch.equal(a.color.view(torch.int32), b.color.view(torch.int32))
    if a.radii is not None:
        assert torch.equal(a.radii, b.radii)


CASES = {
    # name: (scene builder, W, H, tile_rows, radii)
    "orbit_full": (lambda: (synthetic_gaussians(60_000, 3, 11), 3), 640, 480, None, True),
    "strip": (lambda: (synthetic_gaussians(60_000, 3, 12), 3), 640, 480, (3, 9), False),
    "clustered_lsd": (lambda: (clustered_scene(80_000, 7), 3), 640, 480, None, True),
    "sh_degree1": (lambda: (synthetic_gaussians(40_000, 3, 13), 1), 480, 320, None, True),
}


@pytest.mark.parametrize("mode", [1, 2, "1-one-stream", "2-one-stream"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_graph_frames_equal_direct(gpu, case, mode):
    build, W, H, tile_rows, radii = CASES[case]
    g, deg = build()
    sc = _scene(gpu, g, deg)
    on, off = _slots(gpu, mode)
    n = 8
    for cam in _cams(gpu, W, H, n):
        a = _render(gpu, sc, cam, W, H, on, tile_rows, radii)
        b = _render(gpu, sc, cam, W, H, off, tile_rows, radii)
        torch.cuda.synchronize()
        _same(a, b)
    st_on, st_off = _lib.frame_graph_stats(0, on), _lib.frame_graph_stats(0, off)
    assert st_on["graph_frames"] >= n - 1 and st_on["overflows"] == 0
    assert st_off["graph_frames"] == 0
    # the exported lists of the last frame
    la, lb = binning_state(0, on), binning_state(0, off)
    for x, y in zip(la, lb):
        assert torch.equal(x, y)


def test_graph_frames_precomputed_colours(gpu):
    g = synthetic_gaussians(30_000, 0, 21)
    sc = _scene(gpu, g, 0)
    colors = torch.rand((30_000, 3), device=gpu)
    on, off = _slots(gpu)
    for cam in _cams(gpu, 320, 240, 4):
        a = _render(gpu, sc, cam, 320, 240, on, colors=colors)
        b = _render(gpu, sc, cam, 320, 240, off, colors=colors)
        torch.cuda.synchronize()
        _same(a, b)
    assert _lib.frame_graph_stats(0, on)["graph_frames"] >= 3


@pytest.mark.parametrize("mode", [1, 2, "1-one-stream", "2-one-stream"])
def test_graph_overflow_rerenders(gpu, mode):
    """A small scene sets the capacity; a much larger one on the same context overflows it on
    its first frame (rendered again the direct way, identical), then runs on graphs again."""
    W, H = 640, 480
    small = _scene(gpu, synthetic_gaussians(5_000, 3, 31), 3)
    big = _scene(gpu, synthetic_gaussians(150_000, 3, 32), 3)
    on, off = _slots(gpu, mode)
    cams = _cams(gpu, W, H, 6)
    for cam in cams[:3]:
        _render(gpu, small, cam, W, H, on)
    torch.cuda.synchronize()
    cap0 = _lib.frame_graph_stats(0, on)["list_cap"]
    for cam in cams[3:]:
        a = _render(gpu, big, cam, W, H, on)
        b = _render(gpu, big, cam, W, H, off)
        torch.cuda.synchronize()
        _same(a, b)
    st = _lib.frame_graph_stats(0, on)
    assert st["overflows"] == 1 and st["list_cap"] > cap0
    assert st["graph_frames"] >= 4  # 2 small + the overflowed one's attempt + 2 big


def test_graph_rerecords_on_new_inputs(gpu):
    W, H = 480, 320
    g = synthetic_gaussians(40_000, 3, 41)
    sc = _scene(gpu, g, 3)
    on, off = _slots(gpu)
    cams = _cams(gpu, W, H, 4)
    for cam in cams[:2]:
        _render(gpu, sc, cam, W, H, on)
    rec0 = _lib.frame_graph_stats(0, on)["graphs_recorded"]
    sc2 = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in sc.items()}
    del sc  # the old tensors may be freed and their memory reused
    for cam in cams[2:]:
        a = _render(gpu, sc2, cam, W, H, on)
        b = _render(gpu, sc2, cam, W, H, off)
        torch.cuda.synchronize()
        _same(a, b)
    assert _lib.frame_graph_stats(0, on)["graphs_recorded"] == rec0 + 1


def test_one_stream_deferred_k_overflow_at_c3_size(gpu):
    """Four-frames-in-flight regime (one stream, deferred K, GSR_OPT_FRAME_GRAPHS 2) at the
    headline size: a 100k scene sets the capacity, the C3 scene (1M Gaussians, 1920x1080,
    ~5.8M list entries) overflows it on its first frame and is rendered again the direct way;
    every C3 frame equals the direct forward."""
    W, H = 1920, 1080
    small = _scene(gpu, synthetic_gaussians(100_000, 3, 1), 3)
    c3 = _scene(gpu, synthetic_gaussians(1_000_000, 3, 2), 3)
    on, off = _slots(gpu, "2-one-stream")
    cams = _cams(gpu, W, H, 5, step=3)
    for cam in cams[:2]:
        _render(gpu, small, cam, W, H, on)
    torch.cuda.synchronize()
    cap0 = _lib.frame_graph_stats(0, on)["list_cap"]
    for cam in cams[2:]:
        a = _render(gpu, c3, cam, W, H, on)
        b = _render(gpu, c3, cam, W, H, off)
        torch.cuda.synchronize()
        _same(a, b)
    st = _lib.frame_graph_stats(0, on)
    assert st["overflows"] == 1 and st["list_cap"] > cap0 > 0
    la, lb = binning_state(0, on), binning_state(0, off)
    for x, y in zip(la, lb):
        assert torch.equal(x, y)
