#!/bin/bash
# Fan-engine phase clocks of timing builds abp/liblcv_<V>.so (LCV_FAN_X_TIMING=2) for V in $TIMINGS, one
# latency_breakdown pass each on one box (experiments; the tree's library is restored after each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06_timing}
mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.orig.so || exit 1
for v in $TIMINGS; do
  cp abp/liblcv_$v.so $LIB &&
  LCV_LAT_MODES=64 LCV_LAT_NS=1 LCV_LAT_REPS=1 timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/timing_$v.txt 2>&1; rc=$?
  cp $OUT/.orig.so $LIB
  [ $rc -eq 0 ] || { tail -5 $OUT/timing_$v.txt; exit $rc; }
  echo "== $v"; grep "fan T" $OUT/timing_$v.txt | grep "wave=0" | sort | uniq | awk 'NR % 4 == 1'
done
