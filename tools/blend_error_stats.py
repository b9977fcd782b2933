"""Image error of the HIP forward against the CPU oracle at the BASELINE configs, in both blend
arithmetic modes (GSR_OPT_BLEND_FAST 0 = upstream's operation order, 1 = the default fused
form).  One JSON line per (config, frame, mode): max / mean abs error, the fraction within 1e-5,
PSNR (peak 1), final_T max error, the n_contrib mismatch rate, and whether the frame rendered
WITHOUT the per-pixel extras (the viewer's call: no n_contrib, so the blend runs its paired-slot
variant) is bit-identical to the one rendered with them.  Run on the GPU box:

    python tools/blend_error_stats.py [--configs c2,c3,c4,c5] > profiles/<tag>_blend_error_vs_oracle.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import oracle  # noqa: E402
from gaussiansplattingviewer_amd import _lib  # noqa: E402
from gaussiansplattingviewer_amd.camera import orbit_eye, static_camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians  # noqa: E402
from gpu_helpers import psnr_db, run_hip, run_oracle, scene_inputs  # noqa: E402

# name: (P, W, H, sh_degree, seed, frames of the 1000-frame orbit or None for the static camera)
CONFIGS = {"c1": (10_000, 640, 480, 3, 0, None), "c2": (100_000, 1920, 1080, 0, 1, None),
           "c3": (1_000_000, 1920, 1080, 3, 2, None), "c4": (6_000_000, 3840, 2160, 3, 3, None),
           "c5": (1_000_000, 1920, 1080, 3, 2, (0, 250, 500, 750)),
           "c3r": (1_000_000, 1920, 1080, 3, 7, None)}  # gaussian_data.clustered_scene


def stats(hip, orc):
    d = np.abs(hip["color"].astype(np.float64) - orc["color"])
    dT = np.abs(hip["final_T"].astype(np.float64) - orc["final_T"])
    return {"max_abs": float(d.max()), "mean_abs": float(d.mean()),
            "frac_le_1e-5": float((d <= 1e-5).mean()), "psnr_db": round(psnr_db(hip["color"], orc["color"]), 2),
            "frac_bit_equal": float((hip["color"].view(np.uint32) == orc["color"].view(np.uint32)).mean()),
            "final_T_max_abs": float(dT.max()),
            "n_contrib_mismatch": float((hip["n_contrib"] != orc["n_contrib"]).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.load_library()
    ctx = _lib.context(0)
    for name in a.configs.split(","):
        P, W, H, deg, seed, frames = CONFIGS[name]
        g = clustered_scene(P, seed) if name == "c3r" else synthetic_gaussians(P, deg, seed)
        for f in (frames or (None,)):
            eye = orbit_eye(f, 1000) if f is not None else (0.0, 0.0, 4.0)
            s = scene_inputs(g, static_camera(W, H, eye), deg)
            t0 = time.time()
            orc = run_oracle(oracle, s)
            t_orc = time.time() - t0
            for fast in (0, 1):
                _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_BLEND_FAST, fast), "opt")
                hip = run_hip(s, dev, binning=False)
                plain = run_hip(s, dev, binning=False, extras=())
                torch.cuda.empty_cache()
                line = {"config": name, "frame": f, "P": P, "W": W, "H": H, "sh_degree": deg,
                        "mode": ["exact", "fast"][fast], "K": int(orc["num_rendered"]),
                        "K_equal": int(hip["num_rendered"]) == int(orc["num_rendered"])}
                line.update(stats(hip, orc))
                line["no_extras_bit_identical"] = bool(
                    np.array_equal(plain["color"].view(np.uint32), hip["color"].view(np.uint32)))
                line["oracle_s"] = round(t_orc, 1)
                print(json.dumps(line), flush=True)
            del orc
    _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_BLEND_FAST, 1), "opt")


if __name__ == "__main__":
    main()
