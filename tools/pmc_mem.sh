#!/bin/bash
# Memory-path PMC passes over tools/mb_kernels.py (GPU box).  Usage: tools/pmc_mem.sh <tag> <which> [case]
set -e
TAG=${1:-m}; WHICH=${2:-gemm}; CASE=${3:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$ROOT/tools/mb_kernels.py" --which "$WHICH" --case "$CASE" --iters 3 > "$OUT/$1.log" 2>&1
}
run TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE
run TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCC_HIT TCC_MISS TCC_BUSY TCC_REQ
echo done
