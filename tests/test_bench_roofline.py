"""bench.py's roofline block recomputed by hand from the committed op counts and a committed bench line's
stage times: every per-kernel frac is executed ops x units / launch time / the MEASURED multiply-add peak
(profiles/r05_cal/peakbench.txt: 2 ops x the v_mad_u64_u32 rate of an all-mad inline-asm stream at 3
waves/SIMD), none exceeds 1, the canonical numerator appears only for the stages
whose device algorithm is of the same class, and the headline is the longest launch."""
import json
import os

import pytest

import helpers as H


@pytest.fixture(scope="module")
def bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(H.ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_recomputes(bench):
    line = json.load(open(os.path.join(H.ROOT, "profiles", "r04_v7", "bench.json")))
    stage_ms = line["stage_kernel_ms_per_step"]
    n = line["config"]["updates_per_gpu"]
    roof = bench.roofline(stage_ms, n, 1)
    oc = json.load(open(os.path.join(H.ROOT, "profiles", "opcounts.json")))
    ops = lambda c: 600 * c["fp_mul"] + 24 * c["fp_add"] + 2100 * c["sha"]  # noqa: E731
    for stage, d in roof["per_kernel"].items():
        assert d["frac"] <= 1.0, (stage, d["frac"])
        if stage in oc["per_update"]:
            work = ops(oc["per_update"][stage]) * n
        else:
            work = ops(oc["per_committee"][stage]) * 1
        peak = bench.PEAK_MAC_TOPS
        assert d["frac"] == pytest.approx(work / (stage_ms[stage] * 1e-3) / (peak * 1e12), abs=1e-4)
        assert d["frac_vs_int32_valu_peak"] == pytest.approx(d["frac"] * peak / 78.6, abs=1e-4)
        if stage not in bench.CANONICAL_MATCHED:
            assert d["frac_canonical"] is None, stage
    assert roof["stage"] == max(roof["per_kernel"], key=lambda k: roof["per_kernel"][k]["ms_per_launch"])
    assert roof["peak"] == bench.PEAK_MAC_TOPS and roof["frac"] == roof["per_kernel"][roof["stage"]]["frac"]
    # the committed line itself: no fraction above 1 anywhere, the pipeline's canonical figure is a rate
    r = line["roofline"]
    assert r["pipeline_frac"] == r["pipeline_frac_executed"] <= 1.0
    assert "pipeline_frac_canonical" not in r and r["pipeline_canonical_equivalent_T_ops_per_s"] > 0
    assert all(v["frac"] <= 1.0 for v in r["per_kernel"].values())


def test_peak_is_the_measured_mad_stream(bench):
    """The denominator is what the chip does: the peakbench all-mad stream scores 0.9..1.0 against it at
    every residency >= 2 waves/SIMD (the SOP kernels run at 1.3-3), the canonical pipeline rate of the
    round-4 bench line (a textbook work-equivalent, 40.7 T) is below it, and the full-rate INT32 figure
    (78.6 T) is above it."""
    rows = bench.measured_peaks()
    peak = bench.PEAK_MAC_TOPS
    assert peak == rows[("mad", 3)]["op_T"]
    for w in (2, 3, 4, 8):
        mads = 128 * 4096 * 64 * 1024 * w  # per launch: instructions per wave x lanes x waves
        frac = 2 * mads / (rows[("mad", w)]["ms"] * 1e-3) / (peak * 1e12)
        assert 0.9 <= frac <= 1.06, (w, frac)
    line = json.load(open(os.path.join(H.ROOT, "profiles", "r04_v7", "bench.json")))
    assert line["roofline"]["pipeline_canonical_equivalent_T_ops_per_s"] < peak < bench.PEAK_INT32_VALU_TOPS
