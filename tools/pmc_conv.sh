#!/bin/bash
# SQ counters of the conv kernels on the serial schedule (one launch per class and forward, no
# recurrence beside them).  Usage (GPU box): tools/pmc_conv.sh <tag> <kernel regex>
set -e
TAG=${1:-c}; RX=${2:-conv01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/$1.log" 2>&1
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
run SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CU_CYCLES
echo done
