#!/bin/bash
# PMC passes over a short bench run (GPU box).  Usage: tools/pmc_bench.sh <tag> [bench args]
set -e
TAG=${1:-a}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$1" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 1 $BENCH_ARGS > "$OUT/$1.log" 2>&1
}
BENCH_ARGS="$*"
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
run SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM
echo done
