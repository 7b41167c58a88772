"""Timeline of a rocprofv3 kernel trace: busy time per kernel and the idle gaps between launches.

    python tools/gaps.py gpurun_out/<tag>/st8   [--top 12]

Reads the *_kernel_trace.csv under the directory; the timed region is taken as the whole trace after the
first ``skip`` fraction (warmup).  Prints per-kernel totals, the GPU-idle total (time with no kernel
running), and the largest gaps with the kernels either side -- where host work or syncs starve the GPU.
"""

from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"\b(k_\w+)(<[^>(]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:40]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--skip", type=float, default=0.4, help="fraction of the trace (warmup) to drop")
    ap.add_argument("--last", type=float, default=0.0, help="only the last MS milliseconds of the trace")
    ap.add_argument("--window", type=float, nargs=2, default=None, help="only [A, B] ms after the trace start")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    cut = t1 - a.last * 1e6 if a.last else (t0 if a.window else t0 + (t1 - t0) * a.skip)
    rows = [r for r in rows if r[0] >= cut]
    if a.window:
        rows = [r for r in rows if t0 + a.window[0] * 1e6 <= r[0] < t0 + a.window[1] * 1e6]
    busy = defaultdict(float)
    cnt = defaultdict(int)
    gaps = []
    idle = 0.0
    end = rows[0][0]
    prev = None
    for s, e, k in rows:
        busy[k] += (e - s) / 1e6
        cnt[k] += 1
        if s > end:
            g = (s - end) / 1e6
            idle += g
            gaps.append((g, prev, k))
        end = max(end, e)
        prev = k
    span = (end - rows[0][0]) / 1e6
    print(f"span {span:.2f} ms, kernels busy {sum(busy.values()):.2f} ms, idle {idle:.2f} ms ({100 * idle / span:.1f}%)"
          f", launches {len(rows)}")
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"  {k:28s} {v:9.3f} ms  {cnt[k]:6d} launches  {1000 * v / cnt[k]:8.1f} us avg")
    gaps.sort(reverse=True)
    print("largest gaps:")
    for g, p, k in gaps[: a.top]:
        print(f"  {1000 * g:9.1f} us  after {p}  before {k}")
    hist = defaultdict(lambda: [0, 0.0])
    for g, p, k in gaps:
        hist[(p, k)][0] += 1
        hist[(p, k)][1] += g
    print("gap totals by (before -> after):")
    for (p, k), (n, g) in sorted(hist.items(), key=lambda x: -x[1][1])[: a.top]:
        print(f"  {g:8.3f} ms  {n:6d}x  {p} -> {k}")


if __name__ == "__main__":
    main()
