"""Image error of the HIP blend (exact and fast arithmetic) against the CPU oracle on the
benchmark scenes; prints one JSON line per (scene, mode).  Run on the GPU box."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import oracle  # noqa: E402
from gaussiansplattingviewer_amd import _lib  # noqa: E402
from gaussiansplattingviewer_amd.camera import static_camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import synthetic_gaussians  # noqa: E402
from gpu_helpers import run_hip, run_oracle, scene_inputs  # noqa: E402

SCENES = {"C1": (10_000, 640, 480, 3, 0), "C2": (100_000, 1920, 1080, 0, 1),
          "C3": (1_000_000, 1920, 1080, 3, 2)}


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load_library()
    ctx = _lib.context(0)
    for name, (P, W, H, deg, seed) in SCENES.items():
        s = scene_inputs(synthetic_gaussians(P, deg, seed), static_camera(W, H), deg)
        orc = run_oracle(oracle, s)
        for fast in (0, 1):
            _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_BLEND_FAST, fast), "opt")
            hip = run_hip(s, dev, binning=False)
            d = np.abs(hip["color"].astype(np.float64) - orc["color"])
            dT = np.abs(hip["final_T"].astype(np.float64) - orc["final_T"])
            print(json.dumps({
                "scene": name, "mode": ["exact", "fast"][fast], "max_abs": float(d.max()),
                "mean_abs": float(d.mean()), "frac_le_1e-5": float((d <= 1e-5).mean()),
                "frac_le_1e-6": float((d <= 1e-6).mean()), "frac_bit_equal":
                float((hip["color"].view(np.uint32) == orc["color"].view(np.uint32)).mean()),
                "final_T_max_abs": float(dT.max()),
                "n_contrib_mismatch": float((hip["n_contrib"] != orc["n_contrib"]).mean())}),
                flush=True)
    _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_BLEND_FAST, 1), "opt")


if __name__ == "__main__":
    main()
