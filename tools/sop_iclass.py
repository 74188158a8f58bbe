#!/usr/bin/env python3
"""Instruction-class breakdown of the SOP kernels: where every VALU instruction of
a k_sop<...> launch goes, per program, in instructions and in SIMD cycles.

Method
  1. Compile csrc/lcv_k_sop.hip with -DLCV_SOP_MARKERS: the engine (lcv_sop.hpp, lcv_col28.hpp) puts an
     assembler comment at the start of each region of a round, so every basic block of the compiled
     round loop can be tied to a region (product operands, two-term adds, conversion, Karatsuba MACs,
     join, Montgomery reduction, add-ins, quotient estimate, conditional steps, store ...).  The marker
     build's instruction stream is within ~2 % of the product build's (checked below, per kernel).
  2. Execution count of each block per wave: from the program tables of tools/gen_sop.py (wave-uniform
     header of every round: K, the two-term masks, add-ins, m-scaling, reduction steps, flags; per-lane
     add-in signs and destinations).
  3. Every instruction is classed by opcode within its region (mad, conversion, difference, add/carry,
     LDS, address, 64-bit, move, FP64, other) and priced with the peakbench costs (tools/valu_model.py:
     C_MAD, C_64, C_32; profiles/r05_cal/peakbench.txt).
  4. The per-wave VALU total is compared with rocprofv3's SQ_INSTS_VALU / SQ_WAVES of the same kernel
     (a committed pmc.json), which validates the block counts.

The Bernstein-Yang inversion (one team op in a handful of rounds) runs data-dependent loops: its blocks
are counted at the typical 12 outer batches (fp_inv, lcv_field.hpp) and reported as their own class.

    python tools/sop_iclass.py [--pmc profiles/r04_v7/pmc.json] [--json out.json] [--md out.md]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-client-consensus-specs_amd")
sys.path.insert(0, os.path.join(ROOT, "tools"))

KERNELS = {"lines": "_Z5k_sopI11F_sop_linesEvT_jj", "miller_acc": "_Z5k_sopI9F_sop_accEvT_jj",
           "fexp": "_Z5k_sopI10F_sop_fexpEvT_jj", "h2c": "_Z5k_sopI9F_sop_h2cEvT_jj"}
PMC_NAMES = {"lines": "k_sop<F_sop_lines>", "miller_acc": "k_sop<F_sop_acc>", "fexp": "k_sop<F_sop_fexp>",
             "h2c": "k_sop<F_sop_h2c>"}
INV_BATCHES = 12  # typical outer divstep batches of fp_inv on random inputs


def compile_asm(markers: bool) -> str:
    out = os.path.join(tempfile.gettempdir(), f"lcv_k_sop_{'mark' if markers else 'prod'}.s")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-pass-failed",
           "-Ibuild", "--cuda-device-only", "-S", "csrc/lcv_k_sop.hip", "-o", out]
    if markers:
        cmd.insert(1, "-DLCV_SOP_MARKERS")
    subprocess.run(cmd, cwd=PKG, check=True, capture_output=True)
    return open(out).read()


def kernel_text(asm: str, sym: str) -> list:
    lines = asm.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


def blocks(text: list) -> list:
    """[{name, comment, marks, insts: [(opcode, operands)]}] in layout order."""
    out, cur = [], None
    for l in text:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l) or re.match(r"^; (%bb\.\d+):(.*)", l)
        if m:
            cur = {"name": m.group(1), "comment": m.group(2), "marks": [], "insts": []}
            out.append(cur)
            continue
        if cur is None:
            cur = {"name": "entry", "comment": "", "marks": [], "insts": []}
            out.append(cur)
        if "sopmark" in l:
            cur["marks"].append(l.split("sopmark")[1].strip())
            continue
        if "Loop Header" in l:
            cur["comment"] += l
        t = l.strip()
        if re.match(r"^(v_|ds_|s_|global_|buffer_|flat_)", t):
            op = t.split()[0]
            cur["insts"].append((op, t[len(op):].strip()))
    return out


# ------------------------------------------------------------------------------------------ opcode classes
def iclass(op: str, args: str, region: str) -> str:
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "scalar"
    if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
        return "mad"
    if op.startswith(("v_readfirstlane", "v_mov_b", "v_cndmask")) and region not in ("cond_step",):
        return "move"
    if "f64" in op or op.startswith("v_fma") or op.startswith("v_cvt"):
        return "fp64"
    if op.startswith(("v_lshl_add_u64", "v_lshrrev_b64", "v_ashrrev_i64", "v_lshlrev_b64", "v_mul_lo_u32",
                      "v_mul_hi_u32", "v_add_co_u32_e64")) or "u64" in op:
        return "int64"
    return "int32"


def cost(cls: str, c: dict) -> float:
    return {"mad": c["mad"], "int64": c["c64"], "fp64": c["c64"], "int32": c["c32"], "move": c["c32"]}.get(cls, 0.0)


VALU = ("mad", "int64", "fp64", "int32", "move")


# ------------------------------------------------------------------------------------------ block kinds
def classify(bbs: list) -> list:
    """Attach (kind, variant) to every block.  Regions come from the markers; unmarked blocks take the
    region of the block before them in layout (the compiler keeps a region's blocks together), with the
    loop structure deciding per-product vs per-round counts."""
    in_round = False
    last = "prologue"
    variant = None      # "mf" / "plain" product loop
    last_operand = None
    for b in bbs:
        mk = b["marks"]
        c = b["comment"]
        if "Loop Header" in c and "Depth=1" in c and not mk:
            in_round = True
        # the round loop's blocks carry "Loop" in their comment (in Loop / Parent Loop / Loop Header); the
        # kernel's epilogue follows the loop's last block
        if not in_round or "Loop" not in c:
            b["kind"] = "prologue"
            continue
        if "product" in mk:
            last, last_operand = "product", "x"
            # which product loop: decided when its convert block shows whether it scales
        if "two_term" in mk:
            kind = "two_term_" + (last_operand or "x")
            b["kind"] = kind
            continue
        if mk == ["operand"] or (mk and mk[0] == "operand" and "product" not in mk):
            last, last_operand = "operand_y", "y"
        if "convert" in mk or "mscale" in mk:
            last = "convert"
        if "kara" in mk:
            zero_addend = sum(1 for op, a in b["insts"] if op.startswith("v_mad") and a.endswith(", 0"))
            last = "kara_first" if zero_addend > 20 else "kara_acc"
        if "join" in mk:
            last = "join"
        if "redc" in mk:
            last = "redc"
        if "tail" in mk:
            last = "tail"
        if "addin" in mk:
            last = "addin"
        if "addin_neg" in mk:
            last = "addin_neg"
        if "addin_mac" in mk:
            last = "addin_mac"
        if "reduce" in mk:
            last = "reduce"
        if "estimate" in mk:
            last = "estimate"
        if "qp_mads" in mk:
            last = "qp_mads"
        if "qp_table" in mk:
            last = "qp_table"
        if "cond_step" in mk:
            last = "cond_step"
        if "flags" in mk:
            last = "flags"
        if "inv" in mk:
            last = "inv"
        if "store" in mk:
            last = "store"
        b["kind"] = last
        # after the product loop's last block and before the join: per-round glue of the product phase
        if last in ("kara_first", "kara_acc") and not mk:
            b["kind"] = "product_loop"
        if last == "product" and not mk:
            b["kind"] = "product"
    # mark the product loops' variant: a loop whose convert block carries "mscale" is the m-scaled one
    var = None
    for b in bbs:
        if "product" in b["marks"]:
            var = None
            # look ahead to this loop's convert block
        if b["kind"] == "convert":
            var = "mf" if "mscale" in b["marks"] else "plain"
    # assign variants by scanning back from each convert block to the preceding product block
    cur = None
    for i, b in enumerate(bbs):
        if "product" in b["marks"]:
            j = i
            while j < len(bbs) and bbs[j]["kind"] != "convert":
                j += 1
            cur = "mf" if j < len(bbs) and "mscale" in bbs[j]["marks"] else "plain"
        if b["kind"] in ("product", "two_term_x", "two_term_y", "operand_y", "convert", "kara_first", "kara_acc",
                         "product_loop"):
            b["variant"] = cur
        elif b["kind"] == "join":
            b["variant"] = cur
        else:
            b["variant"] = None
    # unmarked blocks between a product loop and its join (phi copies) belong to that join
    for i, b in enumerate(bbs):
        if b["kind"] == "product_loop" and "Depth=1" in b["comment"] and "Depth=2" not in b["comment"]:
            b["kind"] = "join_glue"
    return bbs


# ------------------------------------------------------------------------------------------ execution counts
def round_info(p) -> list:
    """Per round of the encoded program: the header fields and the per-lane facts the device branches on."""
    import gen_sop as G
    hdr, rec = p.encode()
    out = []
    for r in range(len(hdr) // 4):
        w0, off, words, w3 = hdr[4 * r:4 * r + 4]
        K, nadd, mflag = w0 & 15, (w0 >> 4) & 3, (w0 >> 6) & 1
        inv, shadow, red, used = (w0 >> 10) & 1, (w0 >> 13) & 1, (w0 >> 16) & 31, w0 >> 24
        lanes = [rec[off + l * words:off + (l + 1) * words] for l in range(p.team)]
        neg = [any(((ln[2 + j] >> 16) & 0xFFFF) >= 0x8000 for ln in lanes[:used]) for j in range(nadd)]
        store = any((ln[0] & G.SLOT_MASK) != G.SLOT_MASK for ln in lanes[:used])
        shw = shadow and any(((ln[1] >> 12) & G.SHADOW_NONE) != G.SHADOW_NONE for ln in lanes[:used])
        xm = bin(w3 & ((1 << K) - 1)).count("1")
        ym = bin((w3 >> 16) & ((1 << K) - 1)).count("1")
        out.append(dict(K=K, nadd=nadd, mflag=mflag, inv=inv, red=red, neg=neg, store=store, shadow=shw, xm=xm, ym=ym))
    return out


def block_count(b, rounds, n_inv_rounds) -> float:
    k, v = b["kind"], b.get("variant")
    R = rounds

    def rs(pred):
        return [r for r in R if pred(r)]
    loop = (lambda r: r["mflag"]) if v == "mf" else (lambda r: not r["mflag"])
    if k == "prologue":
        return 1.0
    if k in ("product", "operand_y", "convert", "product_loop"):
        return float(sum(r["K"] for r in rs(loop)))
    if k == "two_term_x":
        return float(sum(r["xm"] for r in rs(loop)))
    if k == "two_term_y":
        return float(sum(r["ym"] for r in rs(loop)))
    if k == "kara_first":
        return float(len(rs(lambda r: loop(r) and r["K"] > 0)))
    if k == "kara_acc":
        return float(sum(r["K"] - 1 for r in rs(lambda r: loop(r) and r["K"] > 0)))
    if k in ("join", "join_glue"):
        return float(len(rs(lambda r: loop(r) and r["K"] > 0)))
    if k == "redc":
        return float(len(rs(lambda r: r["K"] > 0)))
    if k in ("tail", "reduce", "flags"):
        return float(len(R))
    if k in ("addin", "addin_mac"):
        return float(sum(r["nadd"] for r in R))
    if k == "addin_neg":
        return float(sum(sum(r["neg"]) for r in R))
    if k in ("estimate",):
        return float(len(rs(lambda r: r["red"] >= 2)))
    if k == "qp_table":
        return float(len(rs(lambda r: 2 <= r["red"] <= 3)))
    if k == "qp_mads":
        return float(len(rs(lambda r: r["red"] >= 4)))
    if k == "cond_step":
        return float(len(rs(lambda r: r["red"] == 1)))
    if k == "inv":
        return float(n_inv_rounds * INV_BATCHES)
    if k == "store":
        return float(len(rs(lambda r: r["store"])))
    return float(len(R))


def analyse(asm: str, prog, name: str, costs: dict) -> dict:
    bbs = classify(blocks(kernel_text(asm, KERNELS[name])))
    rounds = round_info(prog)
    n_inv = sum(r["inv"] for r in rounds)
    regions = {}
    for b in bbs:
        n = block_count(b, rounds, n_inv)
        key = b["kind"] + (f"[{b['variant']}]" if b.get("variant") else "")
        reg = regions.setdefault(key, {})
        for op, a in b["insts"]:
            c = iclass(op, a, b["kind"])
            reg[c] = reg.get(c, 0.0) + n
    # fold regions into the report's rows
    tot = {}
    rows = {}
    for key, cl in regions.items():
        base = key.split("[")[0]
        row = {"prologue": "prologue / epilogue", "product": "product: operand addressing + X term",
               "operand_y": "product: Y term", "two_term_x": "product: two-term X add",
               "two_term_y": "product: two-term Y add", "convert": "product: 28-bit conversion + Karatsuba diffs",
               "kara_first": "product: MACs", "kara_acc": "product: MACs", "product_loop": "product: loop",
               "join": "join (Karatsuba columns)", "join_glue": "join (Karatsuba columns)",
               "redc": "reduction: 14 digits + normalise + pack", "tail": "round: tail dispatch",
               "addin": "add-ins", "addin_neg": "add-ins", "addin_mac": "add-ins", "reduce": "final reduction",
               "estimate": "final reduction", "qp_table": "final reduction", "qp_mads": "final reduction",
               "cond_step": "final reduction", "flags": "round: flags / io", "inv": "inversion (fp_inv)",
               "store": "store + shadow"}.get(base, "round: other")
        if key.endswith("[mf]") and base in ("convert",):
            row = "product: m-scaling + conversion + diffs"
        r = rows.setdefault(row, {})
        for c, v in cl.items():
            r[c] = r.get(c, 0.0) + v
            tot[c] = tot.get(c, 0.0) + v
    valu = sum(tot.get(c, 0.0) for c in VALU)
    cyc = sum(tot.get(c, 0.0) * cost(c, costs) for c in VALU)
    table = []
    for row, cl in sorted(rows.items(), key=lambda kv: -sum(kv[1].get(c, 0) * cost(c, costs) for c in VALU)):
        v = sum(cl.get(c, 0.0) for c in VALU)
        y = sum(cl.get(c, 0.0) * cost(c, costs) for c in VALU)
        table.append({"region": row, "valu_per_wave": round(v), "cycles_per_wave": round(y),
                      "share_of_valu": round(v / valu, 4), "share_of_cycles": round(y / cyc, 4),
                      "by_class": {c: round(cl.get(c, 0.0)) for c in ("mad", "int32", "int64", "fp64", "move", "lds",
                                                                        "vmem") if cl.get(c)}})
    by_class = {c: {"insts_per_wave": round(tot.get(c, 0.0)),
                    "cycles_per_wave": round(tot.get(c, 0.0) * cost(c, costs))} for c in VALU + ("lds", "vmem", "scalar")}
    return {"program": name, "rounds": len(rounds), "team": prog.team, "valu_per_wave": round(valu),
            "mad_per_wave": round(tot.get("mad", 0.0)), "mad_fraction_of_valu": round(tot.get("mad", 0.0) / valu, 4),
            "cycles_per_wave": round(cyc), "mad_share_of_cycles": round(tot.get("mad", 0.0) * costs["mad"] / cyc, 4),
            "by_class": by_class, "regions": table}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r04_v7", "pmc.json"))
    ap.add_argument("--json")
    ap.add_argument("--md")
    a = ap.parse_args(argv)
    import gen_sop as G
    import valu_model as V
    costs = {"mad": V.C_MAD, "c64": V.C_64, "c32": V.C_32}
    asm = compile_asm(True)
    prod = compile_asm(False)
    progs = {p.name: p for p in G.build()}
    pmc = json.load(open(a.pmc))["kernels"] if a.pmc and os.path.exists(a.pmc) else {}
    res = {"costs_cycles_per_wave_instruction": costs, "programs": {}}
    for name in KERNELS:
        r = analyse(asm, progs[name], name, costs)
        # marker build vs product build: static VALU counts of the kernel
        st = lambda txt: sum(1 for op, _ in (i for b in blocks(kernel_text(txt, KERNELS[name])) for i in b["insts"])  # noqa
                             if op.startswith("v_"))
        r["static_valu_marker_build"], r["static_valu_product_build"] = st(asm), st(prod)
        raw = (pmc.get(PMC_NAMES[name]) or {}).get("raw", {})
        if raw.get("SQ_INSTS_VALU") and raw.get("SQ_WAVES"):
            meas = raw["SQ_INSTS_VALU"] / raw["SQ_WAVES"]
            r["pmc_valu_per_wave"] = round(meas)
            r["model_over_pmc"] = round(r["valu_per_wave"] / meas, 4)
        res["programs"][name] = r
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)
    lines = []
    for name, r in res["programs"].items():
        lines.append(f"### {name} (team {r['team']}, {r['rounds']} rounds): {r['valu_per_wave']:,} VALU / wave "
                     f"(PMC {r.get('pmc_valu_per_wave', 0):,}, model/PMC {r.get('model_over_pmc')}), "
                     f"mad fraction {r['mad_fraction_of_valu']}, mads {100 * r['mad_share_of_cycles']:.1f} % of "
                     f"{r['cycles_per_wave']:,} pipe cycles")
        lines.append("")
        lines.append("| region | VALU / wave | share | pipe cycles / wave | share | mad | int32 | int64 | fp64 | move | LDS |")
        lines.append("|---|---|---|---|---|---|---|---|---|---|---|")
        for t in r["regions"]:
            bc = t["by_class"]
            lines.append(f"| {t['region']} | {t['valu_per_wave']:,} | {100 * t['share_of_valu']:.1f} % | "
                         f"{t['cycles_per_wave']:,} | {100 * t['share_of_cycles']:.1f} % | {bc.get('mad', 0):,} | "
                         f"{bc.get('int32', 0):,} | {bc.get('int64', 0):,} | {bc.get('fp64', 0):,} | {bc.get('move', 0):,} | "
                         f"{bc.get('lds', 0):,} |")
        lines.append("")
    md = "\n".join(lines)
    if a.md:
        open(a.md, "w").write(md)
    print(md)


if __name__ == "__main__":
    main()
