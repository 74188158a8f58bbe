#!/bin/bash
# Round 6 GPU call: GPU tests (golden fixtures on both engines, engine log), smoke, the bench line.
# Each GPU step has its own time limit, chained with && (the first failure ends the call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench ok"
