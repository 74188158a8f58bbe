#!/bin/bash
# The pairing SOP kernels at fewer items per wave (LCV_SOP_ITEMS_FEXP / _ACC): parity tests, then a
# same-box A/B of the configs[1] bench over the item counts.   OUT=gpurun_out/<tag> tools/gpu_items_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/items}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_latency_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_latency.txt 2>&1 &&
VAR=LCV_SOP_ITEMS_FEXP VALUES="- 4 3" ROUNDS="1 2" tools/env_ab.sh > $OUT/ab_fexp.txt 2>&1 &&
VAR=LCV_SOP_ITEMS_ACC VALUES="- 4" ROUNDS="1" tools/env_ab.sh > $OUT/ab_acc.txt 2>&1
