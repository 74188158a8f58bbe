#!/usr/bin/env python3
"""Wall time of the reference-shaped calls through the C ABI (sync-protocol.md:512 -> :464): one update from
host buffers (lcv_validate_updates) and bls.FastAggregateVerify over 512 keys, median of REPS calls after warm-up.
GPU only; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))

from lcv import synth  # noqa: E402
from lcv.device import Verifier  # noqa: E402

REPS = int(os.environ.get("LCV_CALL_REPS", "30"))
v = Verifier(0)
sb = synth.generate(v, 4, seed=2)
v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
one = sb.updates.slice(0, 1)
gvr = sb.genesis_validators_root


def med(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        ts.append(1000 * (time.perf_counter() - t0))
    return round(sorted(ts)[len(ts) // 2], 3)


out = {"validate_one_update_ms": med(lambda: v.validate(one, sb.current_slot, gvr))}
print(json.dumps(out))
