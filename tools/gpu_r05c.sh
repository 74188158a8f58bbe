#!/bin/bash
# Fan engine (latency mode): its parity tests, then the single-update latency breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_latency_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_latency.log 2>&1 &&
echo "latency tests ok" &&
timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/latency.json 2> $OUT/latency.err &&
echo "latency ok"
