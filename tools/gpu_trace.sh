# rocprofv3 kernel trace of a short bench run + the last forward's timeline (GPU box).
# Usage: bash tools/gpu_trace.sh <tag>   (env passes through to the bench)
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${1:-t}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/stderr.log || exit 1
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 $ROOT/tools/trace_timeline.py $f > $ROOT/gpurun_out/timeline_$TAG.txt
head -2 $ROOT/gpurun_out/timeline_$TAG.txt
