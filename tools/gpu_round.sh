#!/bin/bash
# One GPU round: parity tests, smoke, bench, rocprofv3 kernel-trace stats.  Every GPU step has its own
# time limit and the steps are chained with && (the first failure ends the call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-5}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --depth 1 --steps 3 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err &&
echo "rocprof ok"
