#!/bin/bash
# Fan-engine experiment: latency A/B over $VARIANTS, then one timing-build run ($TIMING, printing per-phase
# clock sums of the fan kernels) if given.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_lat_ab.sh || exit 1
if [ -n "$TIMING" ]; then
  L=light-client-consensus-specs_amd/lcv/liblcv.so
  cp $L gpurun_out/lat_ab/.orig2.so
  cp abp/liblcv_$TIMING.so $L &&
  LCV_LAT_MODES=64 LCV_LAT_NS=1 LCV_LAT_REPS=1 timeout -k 10 120 python -u tools/latency_breakdown.py > gpurun_out/lat_ab/timing.log 2>&1
  rc=$?
  cp gpurun_out/lat_ab/.orig2.so $L
  grep -h "^fan" gpurun_out/lat_ab/timing.log | tail -8
  exit $rc
fi
