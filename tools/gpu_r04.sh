#!/bin/bash
# Round-4 GPU pass: parity tests, smoke, the full bench line, the rocprofv3 kernel trace of a
# one-batch-at-a-time bench, the PMC passes (tools/pmc_collect.sh) and the valubench calibration under
# the same VALU counters.  Every GPU step has its own time limit; steps are chained with && (the first
# failure ends the call).   OUT=gpurun_out/<tag> tools/gpu_r04.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 &&
echo "smoke ok" &&
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --depth 1 --steps 3 --warmup 1 --quick > $OUT/bench_prof.json 2> $OUT/bench_prof.err &&
echo "rocprof ok" &&
OUT=$OUT/pmc tools/pmc_collect.sh &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_CYCLES SQ_WAVE_CYCLES -d $OUT/vbpmc -o vb --output-format csv -- tools/microbench/valubench > $OUT/valubench_pmc.log 2>&1 &&
echo "valubench pmc ok"
