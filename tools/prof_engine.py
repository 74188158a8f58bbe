#!/usr/bin/env python3
"""Run only the pairing programs (lcv_debug_pairing: Miller + final exponentiation team kernels) on
N random (P, Q) pairs — a small target for rocprofv3 counter passes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))
from lcv.device import Verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
v = Verifier(0)
# valid inputs: k*G1, G2 generator multiples via the device signer's keys is overkill; the programs
# are straight-line, so any field values exercise the same instruction stream
rng = np.random.default_rng(0)
p = rng.integers(0, 256, (n, 96), dtype=np.uint8)
q = rng.integers(0, 256, (n, 192), dtype=np.uint8)
for a in (p, q):
    a[:, 0::48] &= 0x0f  # keep each 48-byte big-endian value below p
v.debug_pairing(p[:64], q[:64])
t = time.perf_counter()
v.debug_pairing(p, q)
print(f"pairing programs: {n} items in {1e3 * (time.perf_counter() - t):.2f} ms")
