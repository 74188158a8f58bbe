#!/bin/bash
# GPU call: the RCCL one-rank test, then the PMC passes of tools/pmc_collect.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1 &&
echo "multi ok" &&
bash tools/pmc_collect.sh
