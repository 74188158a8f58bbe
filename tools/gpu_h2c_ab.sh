#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_h2c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_latency_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_latency.txt 2>&1 &&
VAR=LCV_SOP_ITEMS_H2C VALUES="- 6 4" ROUNDS="1 2" tools/env_ab.sh > $OUT/ab_summary.txt 2>&1
