#!/usr/bin/env python3
"""Canonical-algorithm op counts per update ("N_* comes from the oracle's op counter on
the canonical algorithm"), per device stage, written into profiles/opcounts.json["canonical"] beside the
device's executed counts (tools/opcount.py).  The counter and the textbook algorithms it runs are in
oracle/canonical.py; every value they compute is checked against the definitional oracle on the way.

    python tools/canonical_count.py [--n 2] [--participation full|random]

The update rows are configs[1]-shaped synthetic Deneb updates (lcv.synth on the host simulation),
converted to the oracle's containers (tests/helpers.py)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-client-consensus-specs_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import helpers as H  # noqa: E402
from oracle import bls12_381 as B  # noqa: E402
from oracle import canonical as K  # noqa: E402


def count(n: int = 2, participation: str = "full", tower: str = "karatsuba", seed: int = 2) -> dict:
    from lcv import synth
    v = H.hostsim_verifier()
    sb = synth.generate(v, n, seed=seed, participation=participation)
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    pts = [B.g1_decompress(bytes(pk)) for pk in store.current_sync_committee.pubkeys]
    per, comm = {}, {}
    for i in range(n):
        u = H.update_from(sb.updates, i)
        p1, c1, ok = K.count_update(u, store, sb.genesis_validators_root, committee_points=pts, tower=tower)
        assert ok, "the canonical pairing check must accept a valid update"
        for dst, src in ((per, p1), (comm, c1)):
            for k, d in src.items():
                acc = dst.setdefault(k, {"M": 0, "S": 0, "A": 0, "sha": 0})
                for f in acc:
                    acc[f] += d[f]
    per = {k: K.as_opmodel({f: x / n for f, x in d.items()}) for k, d in per.items()}
    comm = {k: K.as_opmodel({f: x / n for f, x in d.items()}) for k, d in comm.items()}
    tot = {f: sum(d[f] for d in per.values()) for f in ("fp_mul", "fp_add", "sha")}
    return {"tower": tower, "per_update": per, "per_committee": comm, "total_per_update": tot,
            "int32_ops_per_update": 600 * tot["fp_mul"] + 24 * tot["fp_add"] + 2100 * tot["sha"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--participation", default="full")
    args = ap.parse_args()
    kara = count(args.n, args.participation, "karatsuba")
    school = count(args.n, args.participation, "schoolbook")
    path = os.path.join(ROOT, "profiles", "opcounts.json")
    oc = json.load(open(path))
    kara["config"] = (f"{args.n} synthetic Deneb updates, {args.participation} participation, all branches; "
                      "oracle/canonical.py (textbook algorithms, Karatsuba tower: the lower, conservative count)")
    kara["algorithms"] = K.__doc__.split("The canonical algorithms", 1)[1].strip()
    kara["schoolbook"] = {k: school[k] for k in ("per_update", "per_committee", "total_per_update",
                                                  "int32_ops_per_update")}
    kara["schoolbook"]["note"] = "the same algorithms over a Karatsuba-free (schoolbook) tower"
    oc["canonical"] = kara
    json.dump(oc, open(path, "w"), indent=1)
    print(json.dumps({k: {s: d["int32_ops"] for s, d in v["per_update"].items()} | {"total": v["int32_ops_per_update"]}
                      for k, v in (("karatsuba", kara), ("schoolbook", school))}, indent=1))


if __name__ == "__main__":
    main()
