"""CPU oracle for the light-client verification hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()`, `bench.py`'s `cpu_baseline` leg and the
golden-vector generator (`tests/golden/make_golden.py`) may import this package.
The product path (`lcv`, `liblcv.so`) never imports, links or executes anything here.
"""
