"""Generate tests/golden/*.npz from the REFERENCE itself (run in the build container only).

The reference viewer (/root/reference, read-only) is imported as Python to capture the outputs
of the functions the hot path must reproduce.  Its GUI / IO imports that are absent here
(OpenGL, glm, plyfile, open3d) are replaced by empty modules: none of the captured functions
execute them (the glm calls in util.Camera.__init__ / get_project_matrix only build values that
the captured methods never read).  The reference itself never ships to the GPU box; only these
fixtures do.

Captured:
  sort_backend.npz  -- renderer_ogl._sort_gaussian_cpu (renderer_ogl.py:10-19): the float32
                       depth array the reference sorts (recorded inside its call) and the
                       int32 index it returns, for several (xyz, view) cases incl. ties.
  camera.npz        -- util.Camera.get_project_matrix / get_htanfovxy_focal (util.py:82-113)
                       at the four benchmark resolutions.
  naive_gaussian.npz-- util_gau.naive_gaussian() (util_gau.py:25-60).
  camera_data.npz   -- the 18 viewer poses of the reference's camera_data.csv (front, up,
                       position per row; written by main.py:418-434, read by main.py:529-562),
                       as float32 rows: data the reference ships, parsed with numpy.
  ply_ref.npz       -- util_gau.load_ply (util_gau.py:63-125) itself: its activations (:114-124),
                       f_rest reorder (:87-100), bounding box and center, on raw vertex arrays
                       stored in the same file.  plyfile is absent, so `PlyData.read` is a shim
                       that only hands the reference the vertex arrays and property names
                       (oracle/ply_oracle.read_vertex, numpy's parse of the PLY written from
                       the raw arrays); every line of load_ply after the parse is the
                       reference's own.
  glsl_twins.npz    -- the numeric literals of the reference's GLSL twins of upstream's
                       formulas (gau_vert.glsl:3-18 SH constants, the 1.3 clamp and 0.3
                       low-pass of computeCov2D; gau_frag.glsl:21-27 alpha), parsed from the
                       shader text (make_glsl_twins; --only glsl).
Also writes oracle_c1.npz: the oracle's integer outputs for config C1 (a regression pin of the
restatement, NOT a reference output -- the upstream CUDA forward is not available).

Usage:  python tests/golden/make_golden.py [--only ply|camera_data|glsl]
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def _stub_modules():
    gl = types.ModuleType("OpenGL")
    gl_GL = types.ModuleType("OpenGL.GL")
    gl_shaders = types.ModuleType("OpenGL.GL.shaders")
    gl.GL = gl_GL
    gl_GL.shaders = gl_shaders
    glm = types.ModuleType("glm")
    glm.radians = math.radians
    glm.vec3 = lambda *a: np.array(a, dtype=np.float32)
    glm.angleAxis = lambda *a: None
    glm.perspective = lambda *a: None
    ply = types.ModuleType("plyfile")
    ply.PlyData = None
    o3d = types.ModuleType("open3d")
    for name, mod in [("OpenGL", gl), ("OpenGL.GL", gl_GL), ("OpenGL.GL.shaders", gl_shaders),
                      ("glm", glm), ("plyfile", ply), ("open3d", o3d)]:
        sys.modules[name] = mod


def _views():
    sys.path.insert(0, REPO)
    from gaussiansplattingviewer_amd.camera import look_at
    return {
        "front": look_at((0.0, 0.0, 4.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0)),
        "oblique": look_at((2.5, 1.5, -3.0), (0.1, -0.2, 0.3), (0.0, -1.0, 0.0)),
        "viewer_default": look_at((-3.0, 0.0, 1.5), (-3.0, 0.0, 0.5), (0.0, -1.0, 0.0)),
    }


def make_ply_ref(util_gau, tmpdir):
    """Run the reference's load_ply on a PLY written from seeded raw arrays (float32 fields,
    properties in a shuffled order, extreme values included) and store inputs + outputs."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import ply_oracle  # noqa: E402  (the numpy PLY parse only; the shim below feeds it)
    rng = np.random.default_rng(77)
    P = 1500
    raw = {n: rng.normal(0, 1, P).astype(np.float32) for n in ("x", "y", "z", "nx", "ny", "nz")}
    raw["x"] *= 5
    for i in range(3):
        raw[f"f_dc_{i}"] = rng.normal(0, 0.6, P).astype(np.float32)
    for i in range(45):
        raw[f"f_rest_{i}"] = rng.normal(0, 0.05, P).astype(np.float32)
    raw["opacity"] = rng.normal(0, 4.0, P).astype(np.float32)
    raw["opacity"][:4] = np.float32([-90.0, 90.0, 0.0, -1e-8])
    for i in range(3):
        raw[f"scale_{i}"] = rng.uniform(-9, 1, P).astype(np.float32)
    for i in range(4):
        raw[f"rot_{i}"] = rng.normal(0, 1, P).astype(np.float32)
    raw["rot_0"][5] = np.float32(1e-20)  # tiny components
    order = list(raw)
    rng.shuffle(order)
    path = os.path.join(tmpdir, "ref_input.ply")
    ply_oracle.write_ply(path, raw, order=order)

    class _Prop:
        def __init__(self, name):
            self.name = name

    class _Element(dict):
        pass

    class _PlyData:
        @staticmethod
        def read(p):
            el = _Element(ply_oracle.read_vertex(p))
            el.properties = [_Prop(n) for n in el]
            return types.SimpleNamespace(elements=[el])

    util_gau.PlyData = _PlyData
    g, bbox, center = util_gau.load_ply(path)
    out = {f"raw__{n}": raw[n] for n in order}
    out["order"] = np.array(order)
    out.update(xyz=g.xyz, rot=g.rot, scale=g.scale, opacity=g.opacity, sh=g.sh,
               bbox=np.asarray(bbox), center=np.asarray(center))
    np.savez_compressed(os.path.join(HERE, "ply_ref.npz"), **out)


def make_camera_data():
    rows = np.loadtxt(os.path.join(REF, "camera_data.csv"), delimiter=",", dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "camera_data.npz"), rows=rows.astype(np.float32))
    print(f"wrote camera_data.npz ({len(rows)} poses)")


def make_glsl_twins():
    """The numeric literals of the reference's GLSL twins of the upstream formulas, parsed from
    the shader text (numbers only, no source): gau_vert.glsl:3-18 (the SH basis constants, as
    written with their `f` suffix), :101-102 (the 1.3 tan-fov clamp of computeCov2D), :117-118
    (the 0.3 low-pass), and gau_frag.glsl:21-27 (the -0.5 of the exponent, the 0.99 alpha cap,
    the 1/255 alpha floor).  tests/test_oracle_glsl_twins.py evaluates the GLSL formulas with
    them and compares the oracle."""
    import re
    vert = open(os.path.join(REF, "shaders", "gau_vert.glsl")).read()
    frag = open(os.path.join(REF, "shaders", "gau_frag.glsl")).read()
    out = {}
    for name, val in re.findall(r"#define\s+(SH_C\w+)\s+(-?[0-9.]+)f", vert):
        out[name] = np.array(float(val), dtype=np.float64)
    assert len(out) == 14, sorted(out)

    def one(pattern, text, what):
        m = re.findall(pattern, text)
        assert len(set(m)) == 1, (what, m)
        return np.array(float(m[0]), dtype=np.float64)

    out["COV2D_CLAMP"] = one(r"lim[xy]\s*=\s*([0-9.]+)f\s*\*\s*tan_fov[xy]", vert, "clamp")
    out["COV2D_LOWPASS"] = one(r"cov\[[01]\]\[[01]\]\s*\+=\s*([0-9.]+)f", vert, "low-pass")
    out["ALPHA_EXP_COEF"] = one(r"power\s*=\s*(-[0-9.]+)f\s*\*", frag, "exponent")
    out["ALPHA_CAP"] = one(r"min\(([0-9.]+)f,\s*alpha", frag, "alpha cap")
    num, den = re.findall(r"opacity\s*<\s*([0-9.]+)f\s*/\s*([0-9.]+)f", frag)[0]
    out["ALPHA_MIN"] = np.array(float(num) / float(den), dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "glsl_twins.npz"), **out)
    print("wrote glsl_twins.npz:", {k: float(v) for k, v in out.items()})


def main(only=None):
    if only == "camera_data":
        make_camera_data()
        return
    if only == "glsl":
        make_glsl_twins()
        return
    _stub_modules()
    sys.path.insert(0, REF)
    import renderer_ogl  # noqa: E402  (the reference module)
    import util  # noqa: E402
    import util_gau  # noqa: E402

    if only == "ply":
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            make_ply_ref(util_gau, d)
        print("wrote ply_ref.npz")
        return

    assert renderer_ogl._sort_gaussian is renderer_ogl._sort_gaussian_cpu

    # --- sort backend ---------------------------------------------------------------
    # The depth array is captured from inside the reference call: np.argsort is wrapped for
    # the duration of the call so it records the exact array the reference sorted.
    rng = np.random.default_rng(1234)
    views = _views()
    xyz10k = rng.standard_normal((10_000, 3)).astype(np.float32)
    xyz100k = rng.standard_normal((100_000, 3)).astype(np.float32)
    xyz_ties = (np.round(rng.standard_normal((20_000, 3)) * 4) / 4).astype(np.float32)
    cases = {f"10k_{v}": (xyz10k, views[v]) for v in views}
    cases["100k_front"] = (xyz100k, views["front"])
    cases["ties_front"] = (xyz_ties, views["front"])  # many exactly equal depths
    out = {"xyz_10k": xyz10k, "xyz_100k": xyz100k, "xyz_ties": xyz_ties}
    real_argsort = np.argsort
    for name, (xyz, view) in cases.items():
        seen = []

        def recording_argsort(a, *args, **kw):
            seen.append(np.array(a, copy=True))
            return real_argsort(a, *args, **kw)

        np.argsort = recording_argsort
        try:
            index = renderer_ogl._sort_gaussian_cpu(types.SimpleNamespace(xyz=xyz), view)
        finally:
            np.argsort = real_argsort
        assert len(seen) == 1 and seen[0].dtype == np.float32
        out[f"{name}__view"] = view.astype(np.float32)
        out[f"{name}__depth"] = seen[0]
        out[f"{name}__index"] = index
    np.savez_compressed(os.path.join(HERE, "sort_backend.npz"), **out)

    # --- camera ---------------------------------------------------------------------
    cam_out = {}
    for (w, h) in [(640, 480), (1920, 1080), (3840, 2160), (1160, 522)]:
        cam = util.Camera(h, w)
        cam_out[f"{w}x{h}__proj"] = cam.get_project_matrix()
        cam_out[f"{w}x{h}__htanfovxy_focal"] = np.array(cam.get_htanfovxy_focal(), dtype=np.float64)
        cam_out[f"{w}x{h}__fovy"] = np.array(cam.fovy, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "camera.npz"), **cam_out)

    # --- naive gaussian ---------------------------------------------------------------
    g, _, _ = util_gau.naive_gaussian()
    np.savez_compressed(os.path.join(HERE, "naive_gaussian.npz"), xyz=g.xyz, rot=g.rot,
                        scale=g.scale, opacity=g.opacity, sh=g.sh, flat=g.flat())

    # --- oracle regression pin for config C1 (NOT a reference output) -------------------
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: E402
    from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, static_camera
    from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians
    gs = synthetic_gaussians(10_000, 3, seed=0)
    cam = static_camera(640, 480)
    view, proj, campos, tx, ty = cuda_camera_inputs(cam)
    r = oracle.forward(gs.xyz, gs.opacity, view, proj, campos, tx, ty, 640, 480, shs=gs.sh,
                       sh_degree=3, scales=gs.scale, rotations=gs.rot)
    np.savez_compressed(os.path.join(HERE, "oracle_c1.npz"), radii=r["radii"],
                        tiles_touched=r["tiles_touched"], point_list=r["point_list"],
                        point_keys=r["point_keys"], ranges=r["ranges"],
                        num_rendered=np.array(r["num_rendered"]),
                        color_sum=np.array(r["color"].astype(np.float64).sum()),
                        n_contrib=r["n_contrib"])
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        make_ply_ref(util_gau, d)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main(sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None)
