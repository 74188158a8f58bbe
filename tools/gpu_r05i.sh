#!/bin/bash
# Round 5 GPU call (final build, r05_v6): GPU tests, smoke, the bench line, the rocprofv3 kernel trace of the 10^4-row launches,
# and the PMC passes (tools/pmc_collect.sh).  Each GPU step has its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05i}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/latency.json 2> $OUT/latency.err &&
echo "latency ok" &&
timeout -k 10 120 python -u tools/pow_timing.py > $OUT/pow_timing.json 2> $OUT/pow_timing.err &&
echo "pow ok" &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --depth 1 --steps 3 --warmup 1 --quick > $OUT/bench_prof.json 2> $OUT/bench_prof.err &&
echo "rocprof ok" &&
OUT=$OUT/pmc bash tools/pmc_collect.sh
