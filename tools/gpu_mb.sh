# GPU tests, then kernel microbenchmarks (row kernels + attention) and the bench line.  Usage: tools/gpu_mb.sh <tag>
set -o pipefail
TAG=${1:-mb}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_kernels.py --which ${MB_WHICH:-rows,attn} --iters 30 > gpurun_out/${TAG}_mb.log 2>&1 && cat gpurun_out/${TAG}_mb.log &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'], d['ms_per_step'], d['breakdown_ms_per_step'])"
