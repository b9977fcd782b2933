"""Stereo dataset capture benchmark on one MI355X.

The workload the fork exists for (main.py:839-923): for every COLMAP pose render the left view,
the disparity image (left pose, render mode -1) and the right view at the viewer's 1160 x 522
window, and pack them as RGB8 / uint16 frames.  Scene: the synthetic C3 cloud (1M Gaussians,
SH degree 3, seed 2); poses: N synthetic COLMAP image entries on an orbit
around the cloud, written as an images.txt and read back through colmap.read_images_txt.

Reports (one JSON line): poses/s with the three frames resident on the device (`device`),
poses/s including the D2H of the packed frames (`to_host`), and the PNG encode rate of the
host side (PIL, `--png` only, thread pool), plus the live HIP-event time of the disparity and
pack kernels against HBM peak (algorithmic bytes: disparity 24 B per Gaussian, RGB8 pack 15 B
per pixel, uint16 pack 6 B per pixel).

Usage: python tools/stereo_bench.py [--P 1000000] [--poses 60] [--warmup 5] [--png]
"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from gaussiansplattingviewer_amd import colmap  # noqa: E402
from gaussiansplattingviewer_amd.camera import Camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians  # noqa: E402
from gaussiansplattingviewer_amd.renderer import HIPRenderer  # noqa: E402
from gaussiansplattingviewer_amd.stereo import (StereoCapture, disparity_colors,  # noqa: E402
                                                pack_image)

HBM_PEAK_GBS = 8000.0


def rot_to_quat(R):
    """Rotation matrix -> (qw, qx, qy, qz) (Shepperd; any valid branch, sign-normalised)."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = [0.0] * 4
        q[0] = (R[k, j] - R[j, k]) / s
        q[1 + i] = 0.25 * s
        q[1 + j] = (R[j, i] + R[i, j]) / s
        q[1 + k] = (R[k, i] + R[i, k]) / s
    q = np.array(q)
    return q if q[0] >= 0 else -q


def orbit_images_txt(path, n, radius=4.0, height=0.5):
    """COLMAP images.txt with n poses on an orbit looking at the origin, in the viewer's
    convention (camera position = -t, view direction = third row of R, main.py:196-215)."""
    lines = ["# IMAGE_ID, QW, QX, QY, QZ, TX, TY, TZ, CAMERA_ID, NAME",
             "#   POINTS2D[] as (X, Y, POINT3D_ID)"]
    for i in range(n):
        th = 2 * math.pi * i / n
        c = np.array([radius * math.sin(th), height, radius * math.cos(th)])
        fwd = -c / np.linalg.norm(c)
        right = np.cross(fwd, [0.0, 1.0, 0.0])
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        R = np.stack([right, down, fwd])
        q = rot_to_quat(R)
        t = -c
        lines.append(" ".join([str(i + 1)] + [repr(float(v)) for v in (*q, *t)] +
                              ["1", f"{i:05d}.png"]))
        lines.append("")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--poses", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--png", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    W, H = colmap.VIEWER_RESOLUTION
    with tempfile.TemporaryDirectory() as d:
        orbit_images_txt(os.path.join(d, "images.txt"), a.poses)
        poses = colmap.read_images_txt(d)
    g = synthetic_gaussians(a.P, 3, 2)
    cam = Camera(H, W)
    r = HIPRenderer(W, H, device=dev)
    r.update_gaussian_data(g)
    cap = StereoCapture(r, cam)
    for i in range(a.warmup):
        cap.render(poses[i % len(poses)])
    torch.cuda.synchronize()

    t = time.perf_counter()
    for p in poses:
        frames = cap.render(p)
    torch.cuda.synchronize()
    dev_s = time.perf_counter() - t

    host_frames = []
    t = time.perf_counter()
    for p in poses:
        frames = cap.render(p)
        host_frames.append({k: v.cpu() for k, v in frames.items()})
    torch.cuda.synchronize()
    host_s = time.perf_counter() - t

    out = {"workload": f"stereo capture, {a.P} Gaussians SH3 (synthetic C3), {W}x{H}, "
                       f"{len(poses)} COLMAP orbit poses, left+disparity+right per pose",
           "poses": len(poses), "device_poses_per_s": round(len(poses) / dev_s, 1),
           "device_ms_per_pose": round(1e3 * dev_s / len(poses), 3),
           "to_host_poses_per_s": round(len(poses) / host_s, 1)}

    # live kernel timings (HIP events on the stream the kernels run on)
    s = torch.cuda.current_stream(dev)
    left, _ = colmap.load_camera_positions(poses[0])
    xyz = r.gaussians.xyz
    img = r.draw()
    reps = 50
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    kern = {}
    for name, fn, nbytes in (
            ("disparity", lambda: disparity_colors(xyz, left["camera_view"], cam.get_project_matrix()),
             24 * a.P),
            ("pack_rgb8", lambda: pack_image(img, "rgb8"), 15 * W * H),
            ("pack_r16", lambda: pack_image(img, "r16"), 6 * W * H)):
        fn()
        ev[0].record(s)
        for _ in range(reps):
            fn()
        ev[1].record(s)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        gbs = nbytes / (ms * 1e-3) / 1e9
        kern[name] = {"ms": round(ms, 5), "bytes": nbytes, "GB/s": round(gbs, 1),
                      "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}
    out["kernels"] = kern
    out["kernels_note"] = ("ms = back-to-back launches incl. Python/ctypes issue time; the "
                           "rocprof kernel durations are in profiles/")

    if a.png:
        from concurrent.futures import ThreadPoolExecutor
        with tempfile.TemporaryDirectory() as d:
            t = time.perf_counter()
            with ThreadPoolExecutor(max_workers=8) as ex:
                list(ex.map(lambda it: StereoCapture.save(it[1], d, "scene", it[0]),
                            enumerate(host_frames)))
            png_s = time.perf_counter() - t
        out["png_poses_per_s_8_threads"] = round(len(poses) / png_s, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
