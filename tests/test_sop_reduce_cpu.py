"""The SOP engine's final reduction (csrc/lcv_sop.hpp sop_reduce: r < 2^red p -> r mod p), compiled for
the CPU with g++ and checked against Python integers.  For red >= 2 it estimates q = floor(r / p) in
FP64 from r's top words, subtracts q p (from the q p table for red <= 3, else by multiply-adds) and
finishes with one conditional subtraction, skipped when the estimate's fractional part proves it exact —
correct only if the estimate is never above q, at most one below, and the skip test is sound; these cases
sit on and around every multiple of p up to 2^red p and around the skip threshold, where that matters."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

import helpers as H

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
CSRC = os.path.join(H.ROOT, "light-client-consensus-specs_amd", "csrc")

SRC = r"""
#define LCV_HOSTSIM 1
#include "lcv_sop.hpp"
static uint32_t table[lcv::SOP_QP_WORDS];
extern "C" void t_reduce(uint32_t* r, uint32_t red, int use_table) {
  for (uint32_t q = 0; q < lcv::SOP_QP_N; ++q) lcv::sop_qp_entry(table + 16 * q, q);
  lcv::sop_reduce(r, red, use_table ? table : nullptr);
}
"""


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp(prefix="lcv_reduce_")
    src, so = os.path.join(d, "t.cpp"), os.path.join(d, "t.so")
    open(src, "w").write(SRC)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + CSRC, src, "-o", so], check=True)
    return ctypes.CDLL(so)


def _w(v, n=13):
    return (ctypes.c_uint32 * n)(*[(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)])


def _v(w, n=12):
    return sum(int(w[i]) << (32 * i) for i in range(n))


@pytest.mark.parametrize("red", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
def test_sop_reduce_exact(lib, red):
    """Every multiple k p (and its neighbourhood) for red <= 5; for red 6..10 (tools/gen_sop.py allows
    red <= 10, the error analysis needs q < 2^15) sampled multiples: the smallest and the largest 24, and
    100 random k."""
    rng = random.Random(100 + red)
    top = (1 << red) * P
    vals = [0, 1, P - 1, top - 1, top - P]
    ks = range(1, 1 << red)
    if red > 5:
        ks = sorted(set(list(range(1, 25)) + list(range((1 << red) - 24, 1 << red)) +
                        [rng.randrange(1, 1 << red) for _ in range(100)]))
    for k in ks:
        vals += [k * P - 1, k * P, k * P + 1, k * P + (1 << 320) - 1, k * P - (1 << 320),
                 k * P + rng.randrange(1 << 64), k * P - rng.randrange(1, 1 << 64)]
        # around the device's skip threshold (fractional part of the estimate within ~2^-29 of 1)
        for f in (27, 28, 29, 30, 31, 32, 36):
            vals += [(k + 1) * P - (P >> f), k * P + (P >> f), (k + 1) * P - (P >> f) - 1]
    vals += [rng.randrange(top) for _ in range(300)]
    for use_table in ((0, 1) if red <= 3 else (0,)):
        for v in vals:
            if not 0 <= v < top:
                continue
            r = _w(v)
            lib.t_reduce(r, red, use_table)
            assert _v(r) == v % P and int(r[12]) == 0, (red, use_table, hex(v))
