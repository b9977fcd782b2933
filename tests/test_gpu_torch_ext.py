"""GPU: the compiled `_C` extension (_native.so, csrc/torch_ext.cpp) renders what the ctypes
entry renders -- bit-identical, both being gsr_forward on the same slot-0 context -- and what
the oracle renders; it follows torch's current stream; mark_visible is upstream's z > 0.2 test."""
import numpy as np
import pytest
import torch

from gaussiansplattingviewer_amd import _C, _lib
from gaussiansplattingviewer_amd.camera import static_camera
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians
from gaussiansplattingviewer_amd.rasterizer import (GaussianRasterizationSettings,
                                                    GaussianRasterizer, binning_state)

from gpu_helpers import (assert_image_close, run_hip, run_oracle, scene_inputs, tight_binning,
                         to_dev)

pytestmark = pytest.mark.gpu


def _args(s, dev):
    g = s["g"]
    P = len(g.xyz)
    e = torch.empty(0)
    return (to_dev(s["bg"], dev), to_dev(g.xyz, dev), e, to_dev(g.opacity, dev),
            to_dev(g.scale, dev), to_dev(g.rot, dev), s["scale_modifier"], e,
            to_dev(s["view"], dev), to_dev(s["proj"], dev), s["tx"], s["ty"], s["H"], s["W"],
            to_dev(g.sh.reshape(P, -1, 3), dev), s["sh_degree"], to_dev(s["campos"], dev),
            False, False)


@pytest.mark.parametrize("P,W,H", [(20_000, 640, 480), (200_000, 1920, 1080)])
def test_extension_matches_ctypes_entry_and_oracle(gpu, oracle_mod, P, W, H):
    s = scene_inputs(synthetic_gaussians(P, 3, seed=7), static_camera(W, H), 3)
    # the viewer's call (tight binning, the default), then upstream's full lists for the export
    tight_color = _C.rasterize_gaussians(*_args(s, gpu))[1].cpu().numpy()
    with tight_binning(gpu, 0):
        num_rendered, color, radii, geom, binning, img = _C.rasterize_gaussians(*_args(s, gpu))
        pl, _, rg = binning_state(gpu.index or 0)  # the shared slot-0 context's binning
    assert color.device == gpu and tuple(color.shape) == (3, H, W)
    assert radii.dtype == torch.int32 and tuple(radii.shape) == (P,)
    for b in (geom, binning, img):
        assert b.dtype == torch.uint8 and b.numel() == 0
    pl = pl.cpu().numpy().view(np.uint32)
    rg = rg.cpu().numpy().view(np.uint32)
    color, radii = color.cpu().numpy(), radii.cpu().numpy()
    np.testing.assert_array_equal(tight_color, color)  # the same splats in the same order
    ref = run_hip(s, gpu, extras=(), binning=False)
    assert num_rendered == ref["num_rendered"]
    np.testing.assert_array_equal(radii, ref["radii"])
    np.testing.assert_array_equal(color, ref["color"])
    orc = run_oracle(oracle_mod, s)
    assert num_rendered == orc["num_rendered"]
    np.testing.assert_array_equal(radii, orc["radii"])
    if _lib._native_shares_library():  # not under a GSR_LIB A/B build: its own context
        np.testing.assert_array_equal(pl, orc["point_list"])
        np.testing.assert_array_equal(rg, orc["ranges"])
    assert_image_close(color, orc["color"])


def test_extension_follows_current_stream(gpu):
    s = scene_inputs(synthetic_gaussians(50_000, 3, seed=3), static_camera(800, 600), 3)
    args = _args(s, gpu)
    want = _C.rasterize_gaussians(*args)[1].clone()
    side = torch.cuda.Stream(gpu)
    side.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(side):
        got = _C.rasterize_gaussians(*args)[1]
        got = got * 1.0  # consumed on the same stream, no host sync in between
    torch.cuda.current_stream(gpu).wait_stream(side)
    torch.testing.assert_close(got, want, rtol=0, atol=0)


def test_rasterizer_module_and_mark_visible(gpu, oracle_mod):
    s = scene_inputs(synthetic_gaussians(30_000, 3, seed=11), static_camera(640, 360), 3)
    g = s["g"]
    P = len(g.xyz)
    rs = GaussianRasterizationSettings(s["H"], s["W"], s["tx"], s["ty"], to_dev(s["bg"], gpu),
                                       1.0, to_dev(s["view"], gpu), to_dev(s["proj"], gpu), 3,
                                       to_dev(s["campos"], gpu), False, False)
    r = GaussianRasterizer(rs)
    xyz = to_dev(g.xyz, gpu)
    with torch.no_grad():
        color, radii = r(means3D=xyz, means2D=None, opacities=to_dev(g.opacity, gpu),
                         shs=to_dev(g.sh.reshape(P, -1, 3), gpu), colors_precomp=None,
                         scales=to_dev(g.scale, gpu), rotations=to_dev(g.rot, gpu),
                         cov3D_precomp=None)
    orc = run_oracle(oracle_mod, s)
    np.testing.assert_array_equal(radii.cpu().numpy(), orc["radii"])
    assert_image_close(color.cpu().numpy(), orc["color"])

    # points on both sides of the camera (eye at z = 4)
    p = np.random.default_rng(5).uniform(-10, 10, (100_000, 3)).astype(np.float32)
    vis = r.markVisible(to_dev(p, gpu))
    assert vis.dtype == torch.bool and vis.device == gpu and tuple(vis.shape) == (len(p),)
    # upstream in_frustum: view-space z of (x, y, z, 1) under the column-major viewmatrix > 0.2
    view = np.asarray(s["view"], np.float32).reshape(4, 4)
    z = p[:, 0] * view[0, 2] + p[:, 1] * view[1, 2] + p[:, 2] * view[2, 2] + view[3, 2]
    want = z > 0.2
    got = vis.cpu().numpy()
    near = np.abs(z - 0.2) < 1e-5  # float rounding of the test itself
    np.testing.assert_array_equal(got[~near], want[~near])
    assert want.sum() > 0 and (~want).sum() > 0
    assert _C.mark_visible(torch.empty((0, 3), device=gpu), rs.viewmatrix,
                           rs.projmatrix).numel() == 0


def test_debug_snapshot_replays(gpu, tmp_path):
    """A debug snapshot (the 19 `_C.rasterize_gaussians` arguments on the host, as the debug
    forward writes it when a forward raises) re-runs bit-identically through replay_snapshot."""
    from gaussiansplattingviewer_amd import rasterizer
    s = scene_inputs(synthetic_gaussians(30_000, 3, seed=5), static_camera(640, 480), 3)
    args = _args(s, gpu)
    want = _C.rasterize_gaussians(*args)
    path = tmp_path / rasterizer.SNAPSHOT_FILE
    torch.save(rasterizer._cpu_copy(args), path)
    got = rasterizer.replay_snapshot(str(path), gpu)
    assert got[0] == want[0]
    torch.testing.assert_close(got[1], want[1], rtol=0, atol=0)
    torch.testing.assert_close(got[2], want[2], rtol=0, atol=0)
