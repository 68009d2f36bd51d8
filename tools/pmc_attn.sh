#!/bin/bash
# PMC passes over the attention microbenchmark (GPU box).  Usage: tools/pmc_attn.sh <tag>
set -e
TAG=${1:-a}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/mb_kernels.py" --which attn --iters 3 > "$OUT/p1.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/mb_kernels.py" --which attn --iters 3 > "$OUT/p2.log" 2>&1
echo done
