#!/bin/bash
# Round 5, first GPU call: the peak microbenchmark, the GPU tests (incl. the held-stream collective
# test), smoke (build provenance), one bench line.  Each GPU step has its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 120 ./tools/microbench/peakbench > $OUT/peakbench.txt 2>&1 &&
echo "peakbench ok" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench ok"
