"""Summarise a tools/profile.sh run: per-kernel average duration (rocprofv3 kernel trace) and
HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts exactly half of the bytes of
a wide coalesced streaming read (MI355X_MICROARCH.md §HBM), so the table shows the raw read
bytes and the x2-corrected read bytes; WRITE_SIZE is exact for 16-B streaming stores.

Usage: python tools/prof_summary.py gpurun_out/prof_<tag>_<config> [--out profiles/<name>.md]
                                    [--json profiles/<tag>_<config>_kernels.json]
"""
from __future__ import annotations

import argparse
import csv
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"::(k_[a-z0-9_]+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][:60]


def load_stats(d):
    path = os.path.join(d, "trace", "trace_kernel_stats.csv")
    out = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Name"])
        c, t = int(r["Calls"]), float(r["TotalDurationNs"])
        if k in out:
            c0, _, t0 = out[k]
            c, t = c + c0, t + t0
        out[k] = (c, t / c, t)
    return out


def load_trace(d):
    path = os.path.join(d, "trace", "trace_kernel_trace.csv")
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per


def load_pmc(d, counter):
    path = os.path.join(d, f"pmc_{counter}", "pmc_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--title", default="")
    ap.add_argument("--json", help="also write per-kernel {avg_us, read_bytes_x2, write_bytes}")
    a = ap.parse_args()
    stats = load_stats(a.dir)
    fetch = load_pmc(a.dir, "FETCH_SIZE")
    write = load_pmc(a.dir, "WRITE_SIZE")
    total = sum(v[2] for v in stats.values())
    lines = [f"# rocprofv3 summary {a.title}".rstrip(), "",
             f"Source: `{a.dir}` (kernel trace + stats; FETCH_SIZE and WRITE_SIZE in separate "
             "passes).", "",
             "| kernel | calls | avg us | share | FETCH MB/launch (raw) | read MB x2-corr | "
             "WRITE MB/launch |", "|---|---|---|---|---|---|---|"]
    for k, (calls, avg, tot) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        f = fetch.get(k)
        w = write.get(k)
        fmb = sum(f) / len(f) * 1024 / 1e6 if f else float("nan")
        wmb = sum(w) / len(w) * 1024 / 1e6 if w else float("nan")
        lines.append(f"| {k} | {calls} | {avg / 1e3:.2f} | {100 * tot / total:.1f}% | {fmb:.2f} | "
                     f"{2 * fmb:.2f} | {wmb:.2f} |")
    lines += ["", "FETCH/WRITE are per launch, averaged over the launches of the PMC passes; "
              "`read MB x2-corr` doubles FETCH_SIZE per the gfx950 calibration (wide coalesced "
              "reads); other access widths are uncalibrated."]
    text = "\n".join(lines) + "\n"
    if a.json:
        import json
        out = {}
        for k, (calls, avg, tot) in stats.items():
            f, w = fetch.get(k), write.get(k)
            out[k] = {"calls": calls, "avg_us": avg / 1e3,
                      "read_bytes_x2": 2 * sum(f) / len(f) * 1024 if f else None,
                      "write_bytes": sum(w) / len(w) * 1024 if w else None}
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        sha = os.path.join(a.dir, "lib.sha")
        json.dump({"source": a.dir, "lib_sha16": open(sha).read().strip() if os.path.exists(sha) else None,
                   "kernels": out}, open(a.json, "w"), indent=1, sort_keys=True)
    print(text)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        open(a.out, "w").write(text)


if __name__ == "__main__":
    main()
