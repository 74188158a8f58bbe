#!/bin/bash
# Round 6 GPU call (final build): GPU tests, smoke, the one-update latency breakdown, the bench line, rocprofv3 kernel
# traces of the 10^4-row launches and of the one-update path, and the PMC passes (tools/pmc_collect.sh).  Each GPU
# step has its own time limit, chained with && (the first failure ends the call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" && tail -1 $OUT/pytest_gpu.log &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/latency.json 2> $OUT/latency.err &&
echo "latency ok" &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --depth 1 --steps 3 --warmup 1 --quick > $OUT/bench_prof.json 2> $OUT/bench_prof.err &&
echo "rocprof ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lat -o run --output-format csv -- python3 tools/latency_breakdown.py > $OUT/latency_under_rocprof.json 2> $OUT/latency_prof.err &&
echo "rocprof latency ok" &&
OUT=$OUT/pmc bash tools/pmc_collect.sh
