# rocprofv3 kernel traces of short bench runs under two env settings (GPU box): TRACE_ENV_B="VAR=..."
set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for run in A B; do
  OUT=$ROOT/gpurun_out/trace_$run
  mkdir -p $OUT
  ( if [ $run = B ]; then export $TRACE_ENV_B; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/stderr.log ) || exit 1
  f=$(find $OUT -name "*kernel_trace.csv" | head -1)
  python3 $ROOT/tools/trace_timeline.py $f > $ROOT/gpurun_out/timeline_$run.txt
  head -3 $ROOT/gpurun_out/timeline_$run.txt
done
