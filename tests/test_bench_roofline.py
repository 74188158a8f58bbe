"""bench.py's roofline block recomputed by hand from the committed op counts and a
committed bench line's stage times: every per-kernel frac is executed ops x units / launch time / 39.3 T,
none exceeds 1, the canonical numerator appears only for the stages whose device algorithm is of the same
class, and the headline is the longest launch."""
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
        assert d["frac"] == pytest.approx(work / (stage_ms[stage] * 1e-3) / 39.3e12, abs=1e-4)
        assert d["frac_vs_int32_valu_peak"] == pytest.approx(d["frac"] * 39.3 / 78.6, abs=1e-4)
        if stage not in bench.CANONICAL_MATCHED:
            assert d["frac_canonical"] is None, stage
    assert roof["stage"] == max(roof["per_kernel"], key=lambda k: roof["per_kernel"][k]["ms_per_launch"])
    assert roof["peak"] == 39.3 and roof["frac"] == roof["per_kernel"][roof["stage"]]["frac"]
    # the committed line itself: no fraction above 1 anywhere, the pipeline's canonical figure is a rate
    r = line["roofline"]
    assert r["pipeline_frac"] == r["pipeline_frac_executed"] <= 1.0
    assert "pipeline_frac_canonical" not in r and r["pipeline_canonical_equivalent_T_ops_per_s"] > 0
    assert all(v["frac"] <= 1.0 for v in r["per_kernel"].values())
