#!/bin/bash
# PMC passes over one GEMM case of tools/mb_kernels.py (GPU box).  Usage: tools/pmc_gemm.sh <tag> <case>
set -e
TAG=${1:-g}; CASE=${2:-conv2_plain}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmcg_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/tools/mb_kernels.py" --which gemm --case "$CASE" --iters 3 > "$OUT/$name.log" 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum
run p3 FETCH_SIZE
run p4 WRITE_SIZE
echo done
