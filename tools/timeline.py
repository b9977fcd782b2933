"""One frame of a rocprofv3 kernel trace as a timeline: each kernel's start, duration and the
idle gap before it on its queue, plus per-frame totals.  Frames are delimited by k_preprocess.

Usage: python tools/timeline.py gpurun_out/prof_<tag> [--frame N]
"""
import argparse
import csv
import os
import re


def short(name):
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:40]


ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--frame", type=int, default=-3)
a = ap.parse_args()
rows = list(csv.DictReader(open(os.path.join(a.dir, "trace", "trace_kernel_trace.csv"))))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
              r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
starts = [i for i, e in enumerate(ev) if e[2].startswith("k_preprocess")]
f = a.frame if a.frame >= 0 else len(starts) + a.frame
i0, i1 = starts[f], starts[f + 1]
t0 = ev[i0][0]
last_end = {}
busy = 0
print(f"frame {f}: {(ev[i1][0] - t0) / 1e3:.1f} us")
for s, e, n, q in ev[i0:i1]:
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e
    print(f"  q{q:>3} {(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {n}")
