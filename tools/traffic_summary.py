#!/usr/bin/env python3
"""Summarise the two rocprofv3 PMC passes of tools/pmc_traffic.sh (FETCH_SIZE, WRITE_SIZE; KB per
dispatch) into profiles/traffic_pmc.json: per kernel, the average KB per launch of each counter.
bench.py doubles FETCH_SIZE for gfx950 (MI355X_MICROARCH.md) when it reads this file.

    python tools/traffic_summary.py gpurun_out/traffic profiles/traffic_pmc.json
"""
import csv
import json
import os
import re
import sys


def short(name: str) -> str:
    m = re.match(r"void (k_\w+<\w+>)", name)
    return m.group(1) if m else name.split("(")[0]


def main(src: str, dst: str) -> None:
    out = {}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        path = os.path.join(src, sub, f"{sub}_counter_collection.csv")
        acc = {}
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            s, n = acc.get(k, (0.0, 0))
            acc[k] = (s + float(row["Counter_Value"]), n + 1)
        for k, (s, n) in acc.items():
            e = out.setdefault(k, {})
            e[f"{counter}_KB_per_launch"] = round(s / n, 1)
            e["launches"] = n
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k.startswith("k_sop")}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
