#!/usr/bin/env python3
"""Summarise the rocprofv3 counter passes of tools/pmc_collect.sh into one JSON per kernel (average per
launch over the profiled launches), with the derived quantities bench.py's roofline block carries:

  hbm_bytes_per_launch   = 2 * FETCH_SIZE + WRITE_SIZE (KB -> B; FETCH_SIZE doubled on gfx950, see
                           MI355X_MICROARCH.md "FETCH_SIZE reports exactly 1/2 ...")
  valu_busy              = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  (fraction of a resident wave's cycles
                           spent issuing VALU)
  issue_busy             = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  mean_waves_per_simd    = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)  (SQ_WAVE_CYCLES counts
                           quad-cycles per resident wave, summed; GRBM_GUI_ACTIVE is summed over the 8 XCDs,
                           so / 8 is the kernel's cycles; 1024 SIMDs) — the time-averaged occupancy
  lds_bank_conflict_rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (extra cycles per LDS-array cycle)
  valu_insts_per_wave    = SQ_INSTS_VALU / SQ_WAVES
  valu_pipe              = (SOP kernels) the SIMD cycles the launch's VALU stream needs over the launch's
                           SIMD cycles (tools/valu_model.py: exact mad counts from the programs, measured
                           cycles per instruction class); valu_busy above is an issue count, not this

    python tools/pmc_summary.py gpurun_out/pmc profiles/r02_vN/pmc.json [profiles/pmc_latest.json]
"""
import csv
import json
import os
import re
import sys


def short(name: str) -> str:
    m = re.match(r"void (k_\w+<\w+>)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def load(src: str):
    acc = {}
    for sub in sorted(os.listdir(src)):
        d = os.path.join(src, sub)
        if not os.path.isdir(d):
            continue
        for root, _, files in os.walk(d):
            for f in files:
                if not f.endswith("counter_collection.csv"):
                    continue
                for row in csv.DictReader(open(os.path.join(root, f))):
                    k = short(row["Kernel_Name"])
                    c = row["Counter_Name"]
                    key = (row.get("Dispatch_Id") or row.get("Correlation_Id") or "")
                    e = acc.setdefault(k, {}).setdefault(c, {})
                    e[(sub, key)] = e.get((sub, key), 0.0) + float(row["Counter_Value"])
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    return out


def derive(c: dict) -> dict:
    d = {"raw": {k: round(v, 1) for k, v in sorted(c.items())}}
    g = c.get
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        d["hbm_bytes_per_launch"] = round((2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024)
    if g("SQ_WAVE_CYCLES"):
        if g("SQ_ACTIVE_INST_VALU") is not None:
            d["valu_busy"] = round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 4)
        if g("SQ_ACTIVE_INST_ANY") is not None:
            d["issue_busy"] = round(g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES"), 4)
        if g("GRBM_GUI_ACTIVE"):
            d["mean_waves_per_simd"] = round(4 * g("SQ_WAVE_CYCLES") / (g("GRBM_GUI_ACTIVE") / 8 * 1024), 3)
    if g("SQ_LDS_IDX_ACTIVE") and g("SQ_LDS_BANK_CONFLICT") is not None:
        d["lds_bank_conflict_rate"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 4)
    if g("SQ_WAVES") and g("SQ_INSTS_VALU") is not None:
        d["valu_insts_per_wave"] = round(g("SQ_INSTS_VALU") / g("SQ_WAVES"), 1)
    return d


def main(src, dst, latest=None):
    ks = {k: derive(c) for k, c in load(src).items()}
    # the SOP kernels' VALU-pipe occupancy (tools/valu_model.py): instruction counts x measured cycles
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import valu_model
    counts = valu_model.sop_wave_counts()
    for k, d in ks.items():
        p = valu_model.pipe(k, d["raw"], counts)
        if p is not None:
            d["valu_pipe"] = p
    doc = {"source": src, "tool": "tools/pmc_collect.sh (rocprofv3 --kernel-trace --pmc, one pass per group)",
           "kernels": ks}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(doc, open(dst, "w"), indent=1)
    if latest:
        json.dump(doc, open(latest, "w"), indent=1)
    for k, d in ks.items():
        if k.startswith("k_sop") or k in ("k_items<F_h2c_map>", "k_items<F_sig>"):
            print(k, {x: d.get(x) for x in ("hbm_bytes_per_launch", "valu_busy", "issue_busy",
                                              "mean_waves_per_simd", "lds_bank_conflict_rate", "valu_insts_per_wave")},
                  (d.get("valu_pipe") or {}).get("issue_fraction"), (d.get("valu_pipe") or {}).get("mad_share_of_pipe_cycles"))


if __name__ == "__main__":
    main(*sys.argv[1:])
