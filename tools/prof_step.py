#!/usr/bin/env python3
"""One serial validate step of BASELINE configs[1] (10,000 synthetic Deneb updates, resident batch)
after one warm-up step: a short, fixed target for rocprofv3 counter passes (tools/pmc_collect.sh).

    python tools/prof_step.py [N]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))
from lcv import synth  # noqa: E402
from lcv.device import Verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
v = Verifier(0)
sb = synth.generate(v, n, seed=2)
v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
rb = v.upload(sb.updates)
v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
t = time.perf_counter()
ok, _ = v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
print(f"validate {n}: {1e3 * (time.perf_counter() - t):.2f} ms, all valid {bool(ok.all())}")
print({k: round(ms, 3) for k, ms in v.last_timings().items() if ms > 0})
