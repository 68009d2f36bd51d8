#!/bin/bash
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/rps_${1:-a}
mkdir -p "$OUT"
cd "$ROOT"
for R in 8000 32000; do for E in 0 1; do
  timeout -k 10 120 python3 tools/stamps_rowpanel.py --rows $R --epi $E > "$OUT/v2_${R}_$E.log" 2>&1
  VAP_RP_V1=1 timeout -k 10 120 python3 tools/stamps_rowpanel.py --rows $R --epi $E > "$OUT/v1_${R}_$E.log" 2>&1
done; done
echo done
