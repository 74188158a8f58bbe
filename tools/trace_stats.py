#!/usr/bin/env python3
"""Per-kernel launch statistics from a rocprofv3 --kernel-trace CSV, restricted to the launches of one
batch size (grid size filter), so they compare with bench.py's per-stage HIP-event times of the
configs[1] batch (the --stats summary averages every launch, incl. the 1-update latency calls).

    python tools/trace_stats.py gpurun_out/prof/run_kernel_trace.csv [--n 10000] > kernel_stats_10k.csv
"""
import argparse
import csv
import collections
import re
import sys

# items per launch -> grid threads: one lane per item (k_items), TEAM lanes per item in 64-lane waves of
# 64 // TEAM items (k_sop), 64 lanes per committee (k_team)
SOP_TEAM = {"F_sop_lines": 10, "F_sop_acc": 12, "F_sop_fexp": 12, "F_sop_h2c": 8}


def grid_for(name: str, n: int):
    m = re.match(r"void (k_\w+)<(\w+)>", name)
    if not m:
        return None
    kind, f = m.groups()
    if kind == "k_sop":
        team = SOP_TEAM.get(f)
        return {-(-n // (64 // team)) * 64} if team else None
    if kind == "k_team" and f == "F_agg_team":  # 4 lanes per update, 16 updates per wave
        return {-(-n // 16) * 64}
    if kind == "k_items":
        items = 2 * n if f == "F_h2c_map" else n
        return {-(-items // 64) * 64}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--n", type=int, default=10000)
    a = ap.parse_args()
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        g = grid_for(r["Kernel_Name"], a.n)
        if g and int(r["Grid_Size_X"]) in g:
            d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "AverageMs", "MinMs", "MaxMs", "Items"])
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([k, len(v), round(sum(v) / len(v), 4), round(min(v), 4), round(max(v), 4), a.n])


if __name__ == "__main__":
    main()
