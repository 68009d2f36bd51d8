#!/bin/bash
# PMC passes (separate rocprofv3 runs) over tools/mb_kernels.py (GPU box).
# Usage: tools/pmc_mb.sh <tag> <which>
set -e
TAG=${1:-a}; WHICH=${2:-attn}; CASE=${3:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$ROOT/tools/mb_kernels.py" --which "$WHICH" --case "$CASE" --iters 3 > "$OUT/$1.log" 2>&1
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
run SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_WAIT_INST_ANY
echo done
