#!/bin/bash
# PMC passes over the attention microbenchmark (GPU box), default kernel and with $AB_ENV.
# Usage: AB_ENV="VAP_ATTN3=1" tools/pmc_attn.sh <tag>
set -e
TAG=${1:-a}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for V in A B; do
  OUT=$ROOT/gpurun_out/pmc_${TAG}$V
  mkdir -p "$OUT"
  if [ $V = B ]; then E="${AB_ENV:-VAP_AB_DEFAULT=1}"; else E="VAP_AB_DEFAULT=1"; fi
  export $E
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/mb_kernels.py" --which attn --iters 3 > "$OUT/p1.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/mb_kernels.py" --which attn --iters 3 > "$OUT/p2.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE \
    --output-format csv -d "$OUT/p3" -o run -- python3 "$ROOT/tools/mb_kernels.py" --which attn --iters 3 > "$OUT/p3.log" 2>&1
  unset ${E%%=*}
done
echo done
