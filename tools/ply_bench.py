"""Load-time benchmark of the native PLY reader against the restated
reference loader (oracle/ply_oracle.load_ply_reference: util_gau.load_ply's numpy code on a
numpy PLY parse; the reference's plyfile is absent, so its own parse time is not included).

Writes a synthetic 3DGS PLY of P Gaussians (default 1M; --P 6000000 for the C4 scale), then
times: native -> host arrays, native -> device tensors (when a GPU is present), reference
restatement.  One JSON line.  Usage: python tools/ply_bench.py [--P N] [--dir /tmp]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import ply_oracle  # noqa: E402
from gaussiansplattingviewer_amd import ply  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    P = a.P
    vals = {n: rng.standard_normal(P).astype(np.float32) for n in ply_oracle.GS_PROPS}
    with tempfile.TemporaryDirectory(dir=a.dir) as d:
        path = os.path.join(d, "bench.ply")
        ply_oracle.write_ply(path, vals)
        size = os.path.getsize(path)
        out = {"P": P, "file_MB": round(size / 1e6, 1), "threads": min(16, os.cpu_count() or 1)}  # ply_loader.hip caps its pool at 16
        ply.load_ply(path)  # page cache warm
        t = time.perf_counter()
        ply.load_ply(path)
        out["native_host_s"] = round(time.perf_counter() - t, 4)
        try:
            import torch
            if torch.cuda.is_available():
                ply.load_ply(path, device="cuda:0")
                torch.cuda.synchronize()
                t = time.perf_counter()
                ply.load_ply(path, device="cuda:0")
                torch.cuda.synchronize()
                out["native_device_s"] = round(time.perf_counter() - t, 4)
        except ImportError:
            pass
        if not a.no_reference:
            t = time.perf_counter()
            ply_oracle.load_ply_reference(path)
            out["reference_numpy_s"] = round(time.perf_counter() - t, 4)
            out["speedup_host"] = round(out["reference_numpy_s"] / out["native_host_s"], 2)
        out["native_host_GBps"] = round(size / out["native_host_s"] / 1e9, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
