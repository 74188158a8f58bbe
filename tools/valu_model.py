#!/usr/bin/env python3
"""VALU-pipe model of the SOP kernels: how many SIMD cycles a launch's vector instruction stream needs,
and what fraction of the kernel's SIMD cycles that is — the hardware statement beside the INT32-op
roofline (bench.py "valu_pipe").

Cycle costs: ONE source, tools/microbench/peakbench.hip (profiles/r05_cal/peakbench.txt; inline asm, 128
independent instructions of one kind per loop iteration, wall time over all 1,024 SIMDs at 2.4 GHz), at
the SOP kernels' residency of 3 waves per SIMD — the same measurement bench.py's roofline peak is:
  * v_mad_u64_u32 / v_mad_i64_i32: 4.80 / 4.73 SIMD cycles per wave64 instruction (C_MAD);
  * 64-bit adds (v_lshl_add_u64), v_mul_lo_u32, v_fma_f64: 4.3-4.4 (C_64);
  * a full-rate 32-bit instruction (v_add_u32): 2.3-3.0 over W = 2..8 (C_32, the median 2.5);
  * a stream alternating mads and adds (mix) costs the SUM of its parts (4.15 per instruction at W = 3:
    the adds do not hide in the mads' extra cycles).
So for a launch with N_valu VALU, N_int64 64-bit (SQ_INSTS_VALU_INT64: mads included) and N_mad
multiply-add wave-instructions (N_mad exact from the SOP programs, below):
    issue fraction   = (C_MAD N_mad + C_64 (N_int64 - N_mad) + C_32 (N_valu - N_int64)) / S
    (without an INT64 count: C_MAD N_mad + C_32 (N_valu - N_mad), a lower bound)
with S = GRBM_GUI_ACTIVE / 8 * 1024 the launch's SIMD cycles (GRBM summed over 8 XCDs; DVFS-true).

N_mad per wave-round with K products: K * (147 + 12 mflag) + 196 [K > 0] + 12 nadd — a Karatsuba product
is 3 x 49 mads, the 32-bit m * X scaling 12, the 14-digit Montgomery reduction 14 x 14, an add-in term's
c * v 12 (csrc/lcv_sop.hpp, lcv_col28.hpp; `--isa` counts them in the compiled kernel).

SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES ("valu_busy", 0.46-0.49 for these kernels) equals SQ_INSTS_VALU /
SQ_WAVE_CYCLES here (one quad-cycle per instruction): the share of a resident wave's quad-cycles in which
IT issued a VALU instruction — an issue count per wave, not the pipe's occupancy.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

PEAK_FILE = os.path.join(ROOT, "profiles", "r05_cal", "peakbench.txt")
SIMDS = 1024   # 256 CUs x 4 SIMDs


def _costs(path: str = PEAK_FILE, w: int = 3) -> tuple:
    """(C_MAD, C_64, C_32): SIMD cycles per wave64 instruction from the committed peakbench output."""
    rows = {}
    for line in open(path):
        if line.startswith("#") or "|" not in line:
            continue
        head, *cols = [c.strip() for c in line.split("|")]
        name, ww = head.rsplit(None, 1)
        rows[(name.split()[0], int(ww))] = float(cols[3])  # cycles per instruction at 2.4 GHz (wall)
    c64 = sum(rows[(k, w)] for k in ("add64", "mullo", "fma64")) / 3
    adds = sorted(rows[("add", ww)] for ww in (2, 3, 4, 8))
    return rows[("mad", w)], c64, (adds[1] + adds[2]) / 2


C_MAD, C_64, C_32 = _costs()
C_VALU = C_32  # (name kept for callers: the full-rate class)

# per-construct mad counts of the interpreter (checked against the ISA by --isa)
MADS_PER_PRODUCT = 147      # one subtractive Karatsuba level: P0, P2 (49 unsigned each) + D (49 signed)
MADS_MSCALE = 12            # X *= m on 12 32-bit words (rounds with mflag)
MADS_REDC = 196             # 14 quotient digits x (1 + 13) multiply-adds
MADS_ADDIN = 12             # add-in term c * v on 12 words

# kernel name -> (gen_sop program name, items per wave)
SOP_KERNELS = {"k_sop<F_sop_lines>": "lines", "k_sop<F_sop_acc>": "miller_acc", "k_sop<F_sop_fexp>": "fexp",
               "k_sop<F_sop_h2c>": "h2c"}


_COUNTS = None


def sop_wave_counts() -> dict:
    """(cached: building the programs takes seconds)"""
    global _COUNTS
    if _COUNTS is None:
        _COUNTS = _sop_wave_counts()
    return _COUNTS


def _sop_wave_counts() -> dict:
    """program name -> {"mads_per_wave", "rounds", "team", "items_per_wave"} from the generator's tables."""
    import gen_sop as G
    out = {}
    for p in G.build():
        hdr, _ = p.encode()
        mads = 0
        for r in range(len(hdr) // 4):
            w0 = hdr[4 * r]
            K, nadd, mflag = w0 & 15, (w0 >> 4) & 3, (w0 >> 6) & 1
            mads += K * (MADS_PER_PRODUCT + MADS_MSCALE * mflag) + (MADS_REDC if K else 0) + MADS_ADDIN * nadd
        out[p.name] = {"mads_per_wave": mads, "rounds": len(hdr) // 4, "team": p.team,
                       "items_per_wave": 64 // p.team}
    return out


def pipe(kernel: str, raw: dict, counts: dict | None = None, c_mad: float = C_MAD, c_valu: float = C_VALU):
    """The VALU-pipe block of one kernel from its PMC averages per launch (raw counter dict)."""
    if not raw.get("SQ_INSTS_VALU") or not raw.get("GRBM_GUI_ACTIVE") or not kernel.startswith("k_"):
        return None
    waves = raw["SQ_WAVES"]
    n_valu = raw["SQ_INSTS_VALU"]
    if kernel in SOP_KERNELS:
        counts = counts or sop_wave_counts()
        n_mad = counts[SOP_KERNELS[kernel]]["mads_per_wave"] * waves
        mad_source = "exact: the SOP program tables"
    elif raw.get("SQ_INSTS_VALU_INT64") is not None:
        n_mad = raw["SQ_INSTS_VALU_INT64"]  # v_mad_u64_u32 are INT64 instructions (valubench)
        mad_source = "SQ_INSTS_VALU_INT64 (includes the 64-bit shifts / adds: an upper bound)"
    else:
        return None
    n64 = raw.get("SQ_INSTS_VALU_INT64")
    if n64 is not None and n64 >= n_mad:
        need = c_mad * n_mad + C_64 * (n64 - n_mad) + c_valu * (n_valu - n64)
        model = "mads x C_MAD + other INT64 x C_64 + the rest x C_32 (peakbench costs)"
    else:
        need = c_mad * n_mad + c_valu * (n_valu - n_mad)
        model = "mads x C_MAD + the rest x C_32 (no INT64 count: a lower bound)"
    avail = raw["GRBM_GUI_ACTIVE"] / 8 * SIMDS
    out = {"valu_insts_per_launch": round(n_valu), "mad_insts_per_launch": round(n_mad),
           "mad_fraction_of_valu_insts": round(n_mad / n_valu, 4),
           "mad_share_of_pipe_cycles": round(c_mad * n_mad / need, 4),
           "simd_cycles_per_launch": round(avail),
           "issue_fraction": round(need / avail, 4),
           "pipe_cycles_per_launch": round(need), "model": model,
           "c_mad": round(c_mad, 3), "c_64": round(C_64, 3), "c_32": round(c_valu, 3),
           "waves_per_launch": round(waves), "mad_count_source": mad_source}
    if raw.get("SQ_INSTS_VALU_INT64") is not None:
        out["int64_valu_insts_per_launch"] = round(raw["SQ_INSTS_VALU_INT64"])
    return out


def check_isa(asm_path: str) -> dict:
    """Count v_mad_u64_u32 / v_mad_i64_i32 in the SOP kernels' product loop and round tail of a
    `hipcc --cuda-device-only -S` listing of csrc/lcv_k_sop.hip; returns the counts per kernel."""
    import re
    text = open(asm_path).read().split("\n")
    out, cur = {}, None
    for line in text:
        m = re.match(r"^(_Z5k_sopI\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = {"v_mad_u64_u32": 0, "v_mad_i64_i32": 0}
        elif cur and line.strip().startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
            out[cur][line.split()[0]] += 1
        elif cur and "s_endpgm" in line:
            cur = None
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--isa":
        print(json.dumps(check_isa(sys.argv[2]), indent=1))
    elif len(sys.argv) > 1:
        doc = json.load(open(sys.argv[1]))
        cnt = sop_wave_counts()
        for k, d in doc["kernels"].items():
            p = pipe(k, d["raw"], cnt)
            if p:
                print(k, json.dumps(p))
    else:
        print(json.dumps(sop_wave_counts(), indent=1))
