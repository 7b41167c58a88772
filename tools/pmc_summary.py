"""Summarise a tools/profile.sh run into profiles/ (kernel stats + HBM traffic per launch).

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are
collected in separate passes, are in KiB, and on gfx950 FETCH_SIZE reports half
the bytes of wide (16 B/lane) coalesced streaming reads, so reads are doubled:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
k_exchange's reads are dominated by 16 B/lane streaming loads (pass 1); its
gathers (pass 3) are a few percent of the bytes, so the x2 may overstate them.

Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> "<workload string>"
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    for k in ("k_exchange", "k_liveness", "k_begin_round", "k_owner_writes", "k_reset_sched", "k_warm",
              "k_boot_self", "k_phi_row"):
        if k in name:
            return k
    return name[:60]


def kernel_stats(root: str) -> dict:
    out = {}
    for path in glob.glob(os.path.join(root, "kt", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            out[short(row["Name"])] = {
                "calls": int(row["Calls"]),
                "avg_ms": float(row["AverageNs"]) / 1e6,
                "total_ms": float(row["TotalDurationNs"]) / 1e6,
                "pct": float(row["Percentage"]),
            }
    return out


def timed_launches(root: str, sub: str = "kt") -> int | None:
    """k_exchange launches inside bench.py's timed region (its JSON line's roofline.launches): the
    trace's LAST that many k_exchange launches, so settle/warmup rounds are not averaged in."""
    path = os.path.join(root, f"bench_{sub}.log")
    if not os.path.exists(path):
        return None
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)["roofline"]["launches"]
    return None


def trace_avg(root: str, last: int | None) -> dict:
    """Average k_exchange duration (ms) over the last `last` launches of the kernel trace."""
    d = []
    for path in glob.glob(os.path.join(root, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if "k_exchange" in row["Kernel_Name"]:
                d.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
    d.sort()
    tail = d[-last:] if last else d
    return {"launches": len(tail), "avg_ms": sum(x for _, x in tail) / max(1, len(tail))} if tail else {}


def counters(root: str, sub: str, name: str, last: int | None = None) -> tuple[dict, dict]:
    """Average counter value per launch, and per work-item-group unit (k_exchange: per exchange); with
    `last`, over each kernel's last `last` dispatches only (the timed region)."""
    rows = defaultdict(list)
    for path in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row.get("Counter_Name") == name:
                k = short(row["Kernel_Name"])
                wg = float(row.get("Grid_Size", 0) or 0) / max(1.0, float(row.get("Workgroup_Size", 1) or 1))
                rows[k].append((int(row.get("Dispatch_Id", 0) or 0), float(row["Counter_Value"]), wg))
    avg, per_unit = {}, {}
    for k, v in rows.items():
        v.sort()
        if last and k == "k_exchange":
            v = v[-last:]
        avg[k] = sum(x[1] for x in v) / len(v)
        u = sum(x[2] for x in v)
        if u > 0:
            per_unit[k] = sum(x[1] for x in v) / u
    return avg, per_unit


def main(root: str, tag: str, workload: str):
    ks = kernel_stats(root)
    lastn = timed_launches(root)
    timed = trace_avg(root, lastn)
    fetch, fetch_u = counters(root, "fetch", "FETCH_SIZE", timed_launches(root, "fetch"))
    write, write_u = counters(root, "write", "WRITE_SIZE", timed_launches(root, "write"))
    traffic = {}
    for k in set(fetch) | set(write):
        f, w = fetch.get(k), write.get(k)
        if f is not None and w is not None:
            traffic[k] = {"fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": (2 * f + w) * 1024,
                          "hbm_bytes_per_workgroup": (2 * fetch_u[k] + write_u[k]) * 1024}
    summary = {"tag": tag, "workload": workload, "kernel_stats": ks, "k_exchange_timed_region": timed,
               "traffic": traffic}
    sq = {}
    for name in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                 "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"):
        avg, _ = counters(root, "sq", name)
        for k, v in avg.items():
            sq.setdefault(k, {})[name] = v
    if sq:
        summary["sq_per_launch"] = sq
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # the file bench.py reads for roofline.traffic
    agg_path = os.path.join(REPO, "profiles", "pmc_summary.json")
    agg = json.load(open(agg_path)) if os.path.exists(agg_path) else {}
    if "k_exchange" in traffic:
        agg[workload] = {"tag": tag, "k_exchange_bytes_per_launch": traffic["k_exchange"]["hbm_bytes_per_launch"],
                         "k_exchange_bytes_per_exchange": traffic["k_exchange"]["hbm_bytes_per_workgroup"],
                         "k_exchange_avg_ms": timed.get("avg_ms", ks.get("k_exchange", {}).get("avg_ms"))}
        with open(agg_path, "w") as f:
            json.dump(agg, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
