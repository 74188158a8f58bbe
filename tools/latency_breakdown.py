#!/usr/bin/env python3
"""Per-stage kernel times (HIP events) of ONE update (and of 16) validated through the C ABI, on the fan engine
(lcv_set_latency_mode(64), the default for batches of <= 64 rows) and on the batch engine (mode 0) — where the
single-call latency of the reference-shaped drop-in (sync-protocol.md:512 -> :464) goes.  GPU only.
LCV_LAT_MODES="64" / LCV_LAT_NS="1" restrict the runs (A/B scripts)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))

from lcv import synth  # noqa: E402
from lcv.device import Verifier  # noqa: E402

v = Verifier(0)
out = {}
modes = [int(x) for x in os.environ.get("LCV_LAT_MODES", "64 0").split()]
ns = [int(x) for x in os.environ.get("LCV_LAT_NS", "1 16").split()]
for mode in modes:
    v.set_latency_mode(mode)
    for n in ns:
        sb = synth.generate(v, n, seed=2)
        v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
        rb = v.upload(sb.updates)
        for _ in range(3):
            v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
        ts, st = [], {}
        for _ in range(int(os.environ.get("LCV_LAT_REPS", "10"))):
            t0 = time.perf_counter()
            ok, _ = v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
            ts.append(1000 * (time.perf_counter() - t0))
            for k, ms in v.last_timings().items():
                st[k] = st.get(k, 0.0) + ms / int(os.environ.get("LCV_LAT_REPS", "10"))
        out[f"{'latency' if mode else 'batch'}_engine_n{n}"] = {
            "wall_ms_median": round(sorted(ts)[len(ts) // 2], 3), "all_valid": bool(ok.all()),
            "stage_ms": {k: round(x, 3) for k, x in st.items() if x > 0}}
print(json.dumps(out, indent=1))
