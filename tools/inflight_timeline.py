"""Frames in flight from a rocprofv3 kernel trace (bench.py --inflight 2): per frame, the main
chain's span (preprocess start -> blend start), the blend's span, the period between blend ends,
and the kernels of the chain with their duration and their overlap with the other frame's blend.

Usage: python tools/inflight_timeline.py gpurun_out/prof_<tag>/trace [--last N] [--show F]
"""
import argparse
import csv
import os
import re
import statistics as st


def short(name):
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:40]


ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--last", type=int, default=50)
ap.add_argument("--show", type=int, default=2, help="frames printed in full")
a = ap.parse_args()
path = os.path.join(a.dir, "trace_kernel_trace.csv")
rows = list(csv.DictReader(open(path)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
             r["Queue_Id"]) for r in rows)
# frames: a preprocess opens a frame on its queue; later kernels on that queue belong to it
# until the blend; second-stream kernels are matched by start time to the latest frame whose
# preprocess ended before them on the paired queue (the one that runs k_publish_ next)
frames = []
open_by_q = {}
for s, e, n, q in ev:
    if n.startswith("k_preprocess"):
        fr = {"q": q, "pre": (s, e), "kern": [(s, e, n, q)]}
        frames.append(fr)
        open_by_q[q] = fr
    elif q in open_by_q:
        fr = open_by_q[q]
        fr["kern"].append((s, e, n, q))
        if n.startswith("k_blend_q"):
            fr["blend"] = (s, e)
            del open_by_q[q]
frames = [f for f in frames if "blend" in f][-a.last:]
blends = [f["blend"] for f in frames]
period = [(blends[i][1] - blends[i - 1][1]) / 1e3 for i in range(1, len(blends))]
chain = [(f["blend"][0] - f["pre"][0]) / 1e3 for f in frames]
blend = [(f["blend"][1] - f["blend"][0]) / 1e3 for f in frames]
print(f"frames {len(frames)}: period median {st.median(period):.1f} us, chain (preprocess start "
      f"-> blend start) median {st.median(chain):.1f}, blend median {st.median(blend):.1f}")
# per kernel name: median duration and median fraction overlapped by some blend of another frame
agg = {}
for i, f in enumerate(frames):
    others = [g["blend"] for j, g in enumerate(frames) if j != i]
    for s, e, n, q in f["kern"]:
        ov = sum(max(0, min(e, b1) - max(s, b0)) for b0, b1 in others)
        agg.setdefault(n, []).append(((e - s) / 1e3, ov / max(1, e - s)))
print(f"{'kernel':32s} {'median us':>9s} {'blend overlap':>13s}")
for n, v in agg.items():
    print(f"{n:32s} {st.median(x for x, _ in v):9.1f} {st.median(y for _, y in v):13.2f}")
for f in frames[-a.show:]:
    t0 = f["pre"][0]
    print(f"--- frame on q{f['q']}: chain {(f['blend'][0] - t0) / 1e3:.1f} us")
    for s, e, n, q in f["kern"]:
        print(f"  {(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f}  {n}")
