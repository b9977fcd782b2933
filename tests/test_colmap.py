"""COLMAP pose ingestion and pose -> view math (gaussiansplattingviewer_amd/colmap.py; SURVEY.md
§8(f) row 1) on CPU.

Parsing follows main.py:602-630 and is checked exactly on hand-written COLMAP text files.  The
view matrices are checked three ways: a hand-derived pose (identity rotation) exactly; random
poses against the float64 restatement of the reference chain (oracle/stereo_oracle.py:
create_look_at_from_colmap + the reference's numpy look_at + T(-0.5)) to float32 rounding
(tolerance 2e-6 * (1 + |t|)); and structural properties (orthonormal rotation, camera centre
maps to the origin, right = left shifted by the baseline).  PyGLM, which the reference
calls, is absent: its exact float32 rounding is unpinned."""
import numpy as np
import pytest

import stereo_oracle
from gaussiansplattingviewer_amd import colmap
from gaussiansplattingviewer_amd.camera import Camera

IMAGES_TXT = """# Image list with two lines of data per image:
#   IMAGE_ID, QW, QX, QY, QZ, TX, TY, TZ, CAMERA_ID, NAME
#   POINTS2D[] as (X, Y, POINT3D_ID)
# Number of images: 3, mean observations per image: 1
1 1 0 0 0 1 2 3 1 a.png
10.5 20.5 -1 30.0 40.0 7
2 0.7071068 0.7071068 0 0 0.5 -0.25 4 1 b.png

3 0.9 0.1 -0.3 0.2 -1.5 0.75 2.25 1 c.png
1.0 2.0 3
"""

CAMERAS_TXT = """# Camera list with one line of data per camera:
#   CAMERA_ID, MODEL, WIDTH, HEIGHT, PARAMS[]
# Number of cameras: 1
1 PINHOLE 4640 2088 3443.915946 3437.474033 2320 1044
"""


@pytest.fixture()
def model_dir(tmp_path):
    (tmp_path / "images.txt").write_text(IMAGES_TXT)
    (tmp_path / "cameras.txt").write_text(CAMERAS_TXT)
    return tmp_path


def test_read_images_txt(model_dir):
    poses = colmap.read_images_txt(str(model_dir))
    assert [p[0] for p in poses] == ["1", "2", "3"]
    assert poses[1] == ["2", "0.7071068", "0.7071068", "0", "0", "0.5", "-0.25", "4", "1", "b.png"]
    assert colmap.read_images_txt(str(model_dir / "images.txt")) == poses


def test_read_images_txt_misaligned_raises(tmp_path):
    # A missing POINTS2D line shifts the parity: the reference's 10-way unpack fails.
    (tmp_path / "images.txt").write_text("1 1 0 0 0 1 2 3 1 a.png\n"
                                         "2 1 0 0 0 1 2 3 1 b.png\n1.0 2.0 3\n")
    with pytest.raises(ValueError):
        colmap.read_images_txt(str(tmp_path))


def test_read_cameras_and_viewer_resolution(model_dir):
    cams = colmap.read_cameras_txt(str(model_dir))
    assert cams == [colmap.ColmapCamera(1, "PINHOLE", 4640, 2088, 3443.915946, 3437.474033,
                                        2320.0, 1044.0)]
    poses, cams2, res = colmap.load_colmap_poses(str(model_dir))
    assert len(poses) == 3 and cams2 == cams and res == (1160, 522)


def test_identity_pose_hand_derived():
    # q = identity, t = (1, 2, 3): eye = (-1,-2,-3), forward (0,0,1), up (0,-1,0) ->
    # rows s = (1,0,0), u = (0,-1,0), -f = (0,0,-1); translation (1, -2, -3).
    left, right = colmap.load_camera_positions(["1", "1", "0", "0", "0", "1", "2", "3", "1", "a"])
    want = np.array([[1, 0, 0, 1], [0, -1, 0, -2], [0, 0, -1, -3], [0, 0, 0, 1]], np.float32)
    np.testing.assert_array_equal(left["camera_view"], want)
    want[0, 3] = 0.5
    np.testing.assert_array_equal(right["camera_view"], want)
    np.testing.assert_array_equal(left["camera_position"], [-1, -2, -3])
    np.testing.assert_array_equal(right["camera_position"], [-0.5, -2, -3, 1])
    np.testing.assert_array_equal(left["camera_up"], [0, -1, 0])
    np.testing.assert_array_equal(left["camera_front"], [0, 0, 1])
    assert left["camera_view"].dtype == np.float32 and right["camera_position"].dtype == np.float32


def _random_pose(rng, i):
    q = rng.normal(size=4)
    t = rng.uniform(-5, 5, size=3)
    return [str(i)] + [repr(float(v)) for v in q] + [repr(float(v)) for v in t] + ["1", f"{i}.png"]


def test_random_poses_vs_f64_restatement():
    rng = np.random.default_rng(7)
    for i in range(200):
        pose = _random_pose(rng, i)
        left, right = colmap.load_camera_positions(pose)
        vl, vr, cl, cr = stereo_oracle.colmap_view_f64(pose)
        tol = 2e-6 * (1.0 + np.abs(np.array(pose[5:8], float)).max())
        np.testing.assert_allclose(left["camera_view"], vl, rtol=0, atol=tol)
        np.testing.assert_allclose(right["camera_view"], vr, rtol=0, atol=tol)
        np.testing.assert_allclose(left["camera_position"], cl, rtol=0, atol=0)
        np.testing.assert_allclose(right["camera_position"], cr, rtol=0, atol=tol)
        R = left["camera_view"][:3, :3].astype(np.float64)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-6)
        # the camera centre maps to the view origin; the right view is the left one moved by
        # the baseline along view x (main.py:376-380)
        eye = np.append(left["camera_position"], 1.0)
        np.testing.assert_allclose(left["camera_view"].astype(np.float64) @ eye, [0, 0, 0, 1],
                                   atol=tol * 4)
        d = right["camera_view"] - left["camera_view"]
        assert d[0, 3] == np.float32(-0.5) or abs(d[0, 3] + 0.5) < 1e-6
        d[0, 3] = 0
        assert not d.any()


def test_zero_quaternion_raises():
    with pytest.raises(ValueError):
        colmap.load_camera_positions(["1", "0", "0", "0", "0", "1", "2", "3", "1", "a"])


def test_pose_dict_drives_camera():
    # update_camera_pose's view source (util.py:58-63): the pose's camera_view verbatim.
    left, _ = colmap.load_camera_positions(["1", "0.9", "0.1", "-0.3", "0.2", "1", "2", "3", "1", "a"])
    cam = Camera(522, 1160)
    v = cam.get_view_matrix(True, left["camera_front"], left["camera_position"],
                            left["camera_up"], left["camera_view"])
    np.testing.assert_array_equal(v, left["camera_view"])


def test_csv_poses(tmp_path):
    p = tmp_path / "camera_data.csv"
    p.write_text("0.5,0.25,0.8,0.0,-1.0,0.0,-1.25,0.5,-0.05\n1,2\nx,1,1,1,1,1,1,1,1\n"
                 "0,0,-1,0,1,0,0,0,4\n")
    poses = colmap.read_camera_poses_from_csv(str(p))
    assert len(poses) == 2
    np.testing.assert_array_equal(poses[1]["camera_position"], [0, 0, 4])
    cam = Camera(480, 640)
    pose = poses[1]
    v = cam.get_view_matrix(True, pose["camera_front"], pose["camera_position"],
                            pose["camera_up"], pose["camera_view"])
    # lookAt((0,0,4), (0,0,3), +y): identity rotation, translation -4 in z
    np.testing.assert_array_equal(v, np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, -4],
                                               [0, 0, 0, 1]], np.float32))


def test_camera_markers():
    poses = [["1", "1", "0", "0", "0", "1", "2", "3", "1", "a"],
             ["2", "1", "0", "0", "0", "-1", "0.5", "0", "1", "b"]]
    xyz, rot, scale, op, sh = colmap.camera_marker_gaussians(poses)
    np.testing.assert_array_equal(xyz, [[1, 2, 3], [-1, 0.5, 0]])
    assert rot.shape == (2, 4) and scale.shape == (2, 3) and sh.shape == (2, 48)
    assert not op.any() and (scale == np.float32(0.03)).all()


def test_reference_camera_data_csv_through_the_renderer(tmp_path, golden):
    """The reference's own camera_data.csv (18 viewer poses, tests/golden/camera_data.npz): the
    CSV reader returns every row, and HIPRenderer.update_camera_intrin / update_camera_pose
    (renderer_cuda.py:181-203 on CPU tensors here) upload exactly the upstream settings of the
    lookAt(pos, pos + front, up) view in the viewer's 1160x522 window."""
    from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, look_at
    from gaussiansplattingviewer_amd.renderer import HIPRenderer
    rows = golden("camera_data.npz")["rows"]
    p = tmp_path / "camera_data.csv"
    p.write_text("".join(",".join(repr(float(v)) for v in r) + "\n" for r in rows))
    poses = colmap.read_camera_poses_from_csv(str(p))
    assert len(poses) == len(rows) == 18
    r = HIPRenderer(1160, 522, device="cpu")
    for pose, row in zip(poses, rows):
        np.testing.assert_array_equal(pose["camera_front"], row[0:3])
        np.testing.assert_array_equal(pose["camera_position"], row[6:9])
        cam = Camera(522, 1160)
        r.update_camera_intrin(cam)
        r.update_camera_pose(cam, True, pose)
        view = look_at(row[6:9], row[6:9] + row[0:3], row[3:6])
        cam_ref = Camera(522, 1160)
        cam_ref.position = row[6:9]
        want_view, want_proj, want_campos, tx, ty = cuda_camera_inputs(cam_ref, view)
        rs = r.raster_settings
        np.testing.assert_array_equal(rs["viewmatrix"].numpy(), want_view)
        np.testing.assert_array_equal(rs["projmatrix"].numpy(), want_proj)
        np.testing.assert_array_equal(rs["campos"].numpy(), want_campos)
        assert (rs["tanfovx"], rs["tanfovy"]) == (tx, ty)
        # the camera sits inside the synthetic cloud's cube for all but one pose
        assert np.linalg.norm(row[6:9]) < 7.0
