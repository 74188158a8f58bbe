#!/bin/bash
# Round 6 latency call: GPU tests of the fan engine on the tree's library (latency tests + the reference-pinned
# fixtures on both engines), a same-box latency A/B (tools/gpu_lat_ab.sh) and, optionally, the tail sub-phase
# timing build $TIMING (abp/liblcv_$TIMING.so, LCV_FAN_X_TIMING=2).  Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_lat}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_row_tail_gpu.py tests/test_latency_gpu.py tests/test_golden_gpu.py tests/test_gpu_parity.py tests/test_wire.py tests/test_producer.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
OUT=$OUT bash tools/gpu_lat_ab.sh || exit 1
if [ -n "${TIMING:-}" ]; then
  LIB=light-client-consensus-specs_amd/lcv/liblcv.so
  cp $LIB $OUT/.orig.so && cp abp/liblcv_$TIMING.so $LIB &&
  LCV_LAT_MODES=64 LCV_LAT_NS=1 LCV_LAT_REPS=1 timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/tail_timing.txt 2>&1; rc=$?
  cp $OUT/.orig.so $LIB
  grep "fan T" $OUT/tail_timing.txt | grep "wave=0" | sort | uniq
  exit $rc
fi
