"""CPU: the C-ABI libraries load and export every entry point include/lcv.h declares, and the ctypes
binding (lcv/_native.py) names exactly those (no compute call: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import helpers as H

HEADER = os.path.join(H.ROOT, "include", "lcv.h")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(lcv_[a-z0-9_]+)\s*\(", text)))


def exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_binding_matches_header():
    from lcv._native import SIGNATURES
    assert sorted(SIGNATURES) == declared()


def test_hostsim_exports_every_symbol():
    syms = exported(H.ensure_hostsim())
    missing = [s for s in declared() if s not in syms]
    assert not missing


@pytest.mark.skipif(not os.path.exists(H.PRODUCT), reason="liblcv.so not built (run __graft_entry__.build())")
def test_product_library_exports_every_symbol():
    syms = exported(H.PRODUCT)
    missing = [s for s in declared() if s not in syms]
    assert not missing


@pytest.mark.skipif(not os.path.exists(H.PRODUCT), reason="liblcv.so not built")
def test_product_library_loads_and_binds():
    from lcv._native import Lib
    lib = Lib(H.PRODUCT)  # binds restype/argtypes of every symbol
    n = ctypes.c_int(-1)
    assert lib.lcv_device_count(ctypes.byref(n)) == 0  # no compute: device enumeration only
    assert lib.lcv_stage_name(0) == b"nsc_htr"


def test_no_gpu_fails_loudly():
    """Without a GPU the product path raises (no silent CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lcv._native import LcvError, LcvUnavailable
    from lcv.device import Verifier
    with pytest.raises((LcvError, LcvUnavailable)):
        Verifier(0)
