#!/bin/bash
# rocprofv3 counter passes over tools/prof_step.py (two configs[1] validate steps), one pass per
# counter group as MI355X_MICROARCH.md prescribes (FETCH_SIZE and WRITE_SIZE in passes of their own,
# <= 8 SQ counters per pass, no trace domains beside --pmc).  Summarise with tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o $name --output-format csv -- \
    python3 tools/prof_step.py > $OUT/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT &&
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS &&
run grbm GRBM_GUI_ACTIVE GRBM_COUNT &&
run valu SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_CYCLES SQ_BUSY_CU_CYCLES &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
echo "pmc ok"
