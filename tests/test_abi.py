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


def test_build_id_matches_sources():
    """lcv_build_id: the libraries carry the hash of the sources they were built from (tools/build_id.py),
    the check __graft_entry__.smoke() runs on the GPU box against the pushed tree."""
    sys_path = os.path.join(H.ROOT, "tools")
    import sys
    if sys_path not in sys.path:
        sys.path.insert(0, sys_path)
    from build_id import build_id
    from lcv._native import Lib
    assert Lib(H.ensure_hostsim()).build_id() == build_id()
    if os.path.exists(H.PRODUCT):
        assert Lib(H.PRODUCT).build_id() == build_id()


def test_work_views_alias_nothing():
    """Work-space aliasing: for every Work field, item j of each slice's work view is
    item base + j of the slot's work space, element for element, as the kernels address them
    (lcv_items.hpp soa_index / f12_index, lcv_functors_sop.hpp lines_index), and no two fields of any of
    the eight slots overlap.  db0f6f9's work_view (W.f, item-major, advanced by `base` instead of
    base * 144) fails check (1) at the first slice with base > 0: field "f"."""
    v = H.hostsim_verifier()
    for cap, slice_, slots in ((4096, 64, 8), (1000, 128, 3), (65536, 4096, 2), (64, 64, 1)):
        rc = v.lib.lcv_debug_work_check(v.ctx, cap, slice_, slots)
        assert rc == 0, v.lib.lcv_last_error(v.ctx)
