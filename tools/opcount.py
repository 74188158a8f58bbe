#!/usr/bin/env python3
"""Count the algorithmic work per verified update, per kernel stage, by running the host-simulation
build of the SAME per-item kernel code with operation counters (build/liblcv_hostsim_ops.so,
-DLCV_OPCOUNT): Fp multiplications (incl. squarings), Fp additions/subtractions/halvings and SHA-256
compressions.  Writes profiles/opcounts.json, the roofline numerator bench.py uses.

    python tools/opcount.py [--n 8] [--participation full|random]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-client-consensus-specs_amd")
sys.path.insert(0, PKG)

from lcv import synth  # noqa: E402
from lcv._native import Lib  # noqa: E402
from lcv.device import Verifier  # noqa: E402


def count(n: int = 8, participation: str = "full", npool: int = 1) -> dict:
    """Per-stage algorithmic operation counts per update (one mark per kernel, so every operation
    lands in exactly one stage).  Team programs count one Fp multiplication per MUL op of the
    program (not per lane of a round) and (terms - 1) additions per combination."""
    lib = Lib(os.path.join(PKG, "build", "liblcv_hostsim_ops.so"))
    lib.dll.lcv_debug_opcounts.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
    v = Verifier(lib=lib)
    # the batch engine's pipeline (each stage its own program), as the bench's batches of 10^4 run it; a
    # few-row batch would otherwise take latency mode's fused Miller program (no separate line stages)
    v.set_latency_mode(0)
    sb = synth.generate(v, n, seed=2, participation=participation, npool=npool)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ok, _ = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert ok.all()
    names = list(v.last_timings().keys())
    buf = (C.c_ulonglong * (4 * len(names)))()
    lib.dll.lcv_debug_opcounts(v.ctx, buf, len(names))
    per, per_comm = {}, {}
    for s, name in enumerate(names):
        # an SOP half-multiplication (a 12x12-limb product or a Montgomery reduction) is half of a
        # reduced Fp multiplication's 288 multiply-accumulates
        fm, fa, sh = buf[4 * s] + buf[4 * s + 3] / 2, buf[4 * s + 1], buf[4 * s + 2]
        if not (fm or fa or sh):
            continue
        # HTR(next_sync_committee) runs once per DISTINCT committee of the batch's pool, not per update
        units, dst = (npool, per_comm) if name == "nsc_htr" else (n, per)
        dst[name] = {"fp_mul": fm / units, "fp_add": fa / units, "sha": sh / units,
                     "int32_ops": (600 * fm + 24 * fa + 2100 * sh) / units}
    tot = {k: sum(d[k] for d in per.values()) for k in ("fp_mul", "fp_add", "sha")}
    return {"config": f"{n} synthetic Deneb updates, {participation} participation, all branches, {npool} distinct "
                      f"next_sync_committee value(s)",
            "counted": "executed: the device's own operations (host-simulation build of the kernel code); an SOP "
                       "op of K products + one reduction counts (K + 1) / 2 Fp multiplications",
            "op_model": "INT32 ops = 600*fp_mul + 24*fp_add + 2100*sha (SURVEY.md 8(d))",
            "per_update": per, "per_committee": per_comm, "total_per_update": tot,
            "int32_ops_per_update": 600 * tot["fp_mul"] + 24 * tot["fp_add"] + 2100 * tot["sha"],
            "note": "total_per_update excludes per_committee stages: a batch of n updates with npool distinct "
                    "committees costs n * per_update + npool * per_committee"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--participation", default="full")
    args = ap.parse_args()
    out = count(args.n, args.participation)
    path = os.path.join(ROOT, "profiles", "opcounts.json")
    if os.path.exists(path):  # keep the sections other tools own (tools/canonical_count.py: "canonical")
        prev = json.load(open(path))
        out = {**{k: v for k, v in prev.items() if k not in out}, **out}
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
