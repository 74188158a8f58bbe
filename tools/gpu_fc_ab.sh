set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/fc; mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.orig.so && cp abp/liblcv_${NEW:-F}.so $LIB &&
timeout -k 10 300 python -u -m pytest tests/test_row_tail_gpu.py tests/test_latency_gpu.py tests/test_golden_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_${NEW:-F}.log 2>&1; rc=$?
cp $OUT/.orig.so $LIB
tail -1 $OUT/pytest_${NEW:-F}.log
[ $rc -eq 0 ] || exit $rc
OUT=$OUT VARIANTS="${OLD:-E} ${NEW:-F}" ROUNDS="1 2 3" bash tools/gpu_lat_ab.sh
