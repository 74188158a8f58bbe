set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_tail
mkdir -p $OUT
timeout -k 10 120 ./tools/microbench/fp64bench > $OUT/fp64bench.txt 2>&1 &&
echo fp64 ok && cat $OUT/fp64bench.txt &&
LIB=light-client-consensus-specs_amd/lcv/liblcv.so && cp $LIB $OUT/.orig.so && cp abp/liblcv_T.so $LIB &&
LCV_LAT_MODES=64 LCV_LAT_NS=1 LCV_LAT_REPS=1 timeout -k 10 200 python -u tools/latency_breakdown.py > $OUT/tail_timing.txt 2>&1; rc=$?; cp $OUT/.orig.so $LIB; grep "fan T" $OUT/tail_timing.txt | sort | uniq | head -20; exit $rc
