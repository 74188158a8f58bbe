#!/bin/bash
# Same-box A/B of ab/liblcv_A.so vs ab/liblcv_B.so (B = the in-tree build): the GPU parity tests on B
# first, then tools/ab_bench.sh, then the PMC passes on B.   OUT=gpurun_out/<tag> tools/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
ROUNDS="${ROUNDS:-1 2}" tools/ab_bench.sh > $OUT/ab_summary.txt 2>&1 &&
echo "ab ok" &&
cat $OUT/ab_summary.txt &&
if [ -n "$PMC" ]; then OUT=$OUT/pmc tools/pmc_collect.sh; fi
