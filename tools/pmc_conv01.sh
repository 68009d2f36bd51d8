#!/bin/bash
# SQ counters of the conv01 launch on the serial schedule (one conv01 launch per forward, no LSTM beside it).
# Usage (GPU box): tools/pmc_conv01.sh <tag>
set -e
TAG=${1:-c}; RX=${2:-conv01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export VAP_TIME_CHUNKS=1 VAP_MICROBATCHES=1 VAP_PERSISTENT_LSTM=0
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/$1.log" 2>&1
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo done
