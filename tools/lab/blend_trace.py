"""Lab: per-wave timeline of the blend (not the product).

  python tools/lab/blend_trace.py make            # writes build/lab_trace_src/blend.hip from
                                                   # csrc/blend.hip with per-wave tracing, then
                                                   # tools/lab/build.sh trace blend.hip <it>
  GSR_LIB=.../libgsr_lab_trace.so python tools/lab/blend_trace.py run [--config c3]

Each quadrant wave records {start, end} (s_memrealtime, 100 MHz), its hardware slot (HW_ID,
XCC_ID) and its chunk / composite counts; `run` renders one serial frame and prints the
kernel span, the active-wave curve and the tail (how long the last waves run with the chip
mostly idle), plus the work distribution.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make():
    src = open(os.path.join(REPO, "gaussiansplattingviewer_amd/csrc/blend.hip")).read()
    patches = [
        ("namespace {\n", "namespace {\n__device__ uint4 g_trace[1 << 16];\n", 1),
        ("    StagedSplat *const s_spl = s_spl_q[quad];\n",
         "    StagedSplat *const s_spl = s_spl_q[quad];\n"
         "    const uint32_t work = tile * 4u + quad;  // (trace slot: one per quadrant wave)\n"
         "    const uint32_t t_start = (uint32_t)__builtin_amdgcn_s_memrealtime();\n"
         "    uint32_t n_chunks = 0, n_comp = 0;\n", 1),
        ("    for (uint32_t start = range.x; start < range.y; start += 64) {\n",
         "    for (uint32_t start = range.x; start < range.y; start += 64) {\n        ++n_chunks;\n", 1),
        ("            ++count;\n        }\n", "            ++count;\n        }\n        n_comp += count;\n", 1),
        ("    if (inside) {\n        const int row = py - a.y0;",
         "    if (lane == 0 && work < (1u << 16)) {\n"
         "        const uint32_t t_end = (uint32_t)__builtin_amdgcn_s_memrealtime();\n"
         "        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);\n"
         "        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);\n"
         "        g_trace[work] = make_uint4(t_start, t_end, (hw & 0xFFFFu) | (xcc << 16),\n"
         "                                   (n_chunks << 16) | (n_comp & 0xFFFFu));\n"
         "    }\n"
         "    if (inside) {\n        const int row = py - a.y0;", 1),
    ]
    for old, new, n in patches:
        assert src.count(old) >= n, old
        src = src.replace(old, new, n)
    src += ('\nextern "C" int gsr_lab_blend_trace(void *dst, int n, int clear) {\n'
            '    void *p = nullptr;\n'
            '    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace)) != hipSuccess) return -1;\n'
            '    if (clear) return hipMemset(p, 0, sizeof(uint4) << 16) == hipSuccess ? 0 : -1;\n'
            '    return hipMemcpy(dst, p, (size_t)n * 16, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;\n'
            '}\n')
    out_dir = os.path.join(REPO, "build", "lab_trace_src")
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "blend.hip")
    open(path, "w").write(src)
    subprocess.run(["bash", os.path.join(REPO, "tools/lab/build.sh"), "trace", "blend.hip", path],
                   check=True, env=dict(os.environ, LAB_FLAGS="-I" + os.path.join(REPO, "gaussiansplattingviewer_amd/csrc")))


def run(cfg):
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    import bench
    from gaussiansplattingviewer_amd import _lib
    lib = _lib.load_library()
    fn = lib.gsr_lab_blend_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    scene = bench.Scene(cfg, dev)
    for i in range(5):
        scene.render(0)
    torch.cuda.synchronize()
    n_work = 4 * ((scene.W + 15) // 16) * ((scene.H + 15) // 16)
    buf = np.zeros((1 << 16, 4), np.uint32)
    results = []
    for rep in range(3):
        assert fn(None, 0, 1) == 0
        torch.cuda.synchronize()
        scene.render(0)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, 1 << 16, 0) == 0
        results.append(buf[:n_work].copy())
    for tr in results:
        ok = tr[:, 1] != 0
        t = tr[ok]
        s = t[:, 0].astype(np.int64)
        e = t[:, 1].astype(np.int64)
        t0 = s.min()
        s, e = s - t0, e - t0
        span = e.max() / 100.0  # us (100 MHz)
        dur = (e - s) / 100.0
        chunks = t[:, 3] >> 16
        comp = t[:, 3] & 0xFFFF
        xcc = t[:, 2] >> 16
        hw = t[:, 2] & 0xFFFF
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 7
        slot = ((xcc * 8 + se) * 16 + cu) * 4 + simd
        n_slots = len(np.unique(slot))
        # active waves over time (1 us bins)
        nb = int(np.ceil(span)) + 1
        act = np.zeros(nb)
        for a, b in zip(s // 100, e // 100):
            act[a:b + 1] += 1
        peak = act.max()
        half = np.nonzero(act >= 0.5 * peak)[0]
        tail = span - (half.max() if len(half) else 0)
        # per-SIMD busy sum
        busy = np.zeros(slot.max() + 1)
        np.add.at(busy, slot, dur)
        print(f"waves {ok.sum()} / {n_work}  span {span:.1f} us  SIMD slots {n_slots}  "
              f"peak active {peak:.0f}  tail(<50% of peak) {tail:.1f} us")
        print(f"  wave dur us: mean {dur.mean():.1f} p50 {np.median(dur):.1f} p90 "
              f"{np.percentile(dur, 90):.1f} p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}")
        print(f"  chunks/wave mean {chunks.mean():.2f} max {chunks.max()}  composites/wave mean "
              f"{comp.mean():.1f} max {comp.max()}")
        print(f"  active-wave curve (every 10 us): "
              f"{[int(x) for x in act[::10]]}")
        used = busy[busy > 0]
        print(f"  per-SIMD busy (wave-us): mean {used.mean():.0f} min {used.min():.0f} max "
              f"{used.max():.0f}  => mean occupancy {used.mean() / span:.2f} waves")
        # correlation of start order with duration: late heavy waves
        late = s > np.percentile(s, 90)
        print(f"  waves starting in the last 10% of start times: mean dur {dur[late].mean():.1f} us,"
              f" their ends {e[late].max() / 100:.1f} us")
        # xcd balance
        for x in range(8):
            m = xcc == x
            if m.any():
                print(f"   xcc {x}: waves {m.sum()} wave-us {dur[m].sum():.0f} last end {e[m].max() / 100:.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make()
    else:
        cfg = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c3"
        run(cfg)
