#!/usr/bin/env python3
"""Wall time of lcv_debug_fp_pow (two square-root-candidate exponentiations per value) for ONE value on the
latency twins' chains (lcv_set_latency_mode(64): one value per wave, lcv_wave.hpp) and on the batch kernels'
one-lane chains (mode 0); median of LCV_POW_REPS calls.  GPU only."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))

from lcv.device import Verifier  # noqa: E402

v = Verifier(0)
a = np.frombuffer((123456789).to_bytes(48, "big"), np.uint8).copy()
out = {}
for mode in (64, 0):
    v.set_latency_mode(mode)
    for _ in range(3):
        v.debug_fp_pow(a)
    ts = []
    for _ in range(int(os.environ.get("LCV_POW_REPS", "30"))):
        t0 = time.perf_counter()
        v.debug_fp_pow(a)
        ts.append(1000 * (time.perf_counter() - t0))
    out[f"mode{mode}_ms_median"] = round(sorted(ts)[len(ts) // 2], 4)
print(json.dumps(out))
