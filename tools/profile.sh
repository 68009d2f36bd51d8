#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (GPU box).  Usage: tools/profile.sh <tag> [bench args]
set -e
TAG=${1:-r1}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/stderr.log"
find "$OUT" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
echo "profile written to $OUT"
