#!/bin/bash
# HBM traffic per dispatch (FETCH_SIZE, WRITE_SIZE; separate rocprofv3 passes) over a short bench run.
# Usage (GPU box): tools/pmc_traffic.sh <tag>
set -e
TAG=${1:-t}; shift || true; BENCH_ARGS="$*"
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/traffic_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 1 --warmup 1 $BENCH_ARGS > "$OUT/$C.log" 2>&1
done
echo done
