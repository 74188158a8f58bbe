#!/usr/bin/env python3
"""Pairing programs (Miller + final exponentiation team kernels, lcv_debug_pairing) timed at growing
batch sizes: per-round latency of one wave vs a loaded chip (is the engine latency- or
throughput-bound?)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))
from lcv.device import Verifier  # noqa: E402

v = Verifier(0)
rng = np.random.default_rng(0)
N = 32768
p = rng.integers(0, 256, (N, 96), dtype=np.uint8)
q = rng.integers(0, 256, (N, 192), dtype=np.uint8)
for a in (p, q):
    a[:, 0::48] &= 0x0f
v.debug_pairing(p[:64], q[:64])
for n in (4, 64, 256, 1024, 2048, 4096, 7168, 8192, 10000, 16384, 32768):
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        v.debug_pairing(p[:n], q[:n])
        best = min(best, time.perf_counter() - t)
    tm = v.last_timings()
    print(f"n={n:6d}: {1e3 * best:8.2f} ms total, miller {tm.get('miller_accumulate', 0):7.2f} ms, "
          f"fexp {tm.get('final_exp', 0):7.2f} ms", flush=True)
