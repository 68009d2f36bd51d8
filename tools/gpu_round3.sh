# Round check: GPU tests, default bench (with the CPU baseline), C4 / fp32 lines, rocprofv3 kernel stats.
# Usage: tools/gpu_round3.sh <tag>
set -o pipefail
TAG=${1:-r3}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pt.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --seconds 60 --batch 32 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --precision fp32 --steps 5 --warmup 2 > gpurun_out/${TAG}_fp32.json 2> gpurun_out/${TAG}_fp32.err || exit 1
python3 -c "import json;[print(f, json.load(open(f))['value'], json.load(open(f))['ms_per_step']) for f in ['gpurun_out/${TAG}_c4.json','gpurun_out/${TAG}_fp32.json']]"
bash tools/profile.sh $TAG --steps 5 --warmup 2 && echo PROF_OK
