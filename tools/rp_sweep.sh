#!/bin/bash
# Row-panel variants: parity tests, row sweep (v1 = LDS-staged W, v2 = direct W; plain / packed W) (GPU box).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/rp_${1:-a}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python3 -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "rowpanel" > "$OUT/tests.log" 2>&1
for R in 8000 32000; do
  for P in "" "--packed"; do
    timeout -k 10 120 python3 tools/mb_kernels.py --which rowpanel --rows $R --iters 50 $P > "$OUT/v2_$R$P.log" 2>&1
    VAP_RP_V1=1 timeout -k 10 120 python3 tools/mb_kernels.py --which rowpanel --rows $R --iters 50 $P > "$OUT/v1_$R$P.log" 2>&1
  done
done
echo done
