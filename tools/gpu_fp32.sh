# GPU check of the fp32 (parity) mode: the GPU tests, then the fp32 bench line and its kernel stats.
# Usage: tools/gpu_fp32.sh <tag>
set -o pipefail
TAG=${1:-fp32}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pt.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --precision fp32 --steps 5 --warmup 2 > gpurun_out/${TAG}_fp32.json 2> gpurun_out/${TAG}_fp32.err || exit 1
cut -c1-260 gpurun_out/${TAG}_fp32.json
bash tools/profile.sh ${TAG}p --precision fp32 --steps 3 --warmup 1 && echo PROF_OK
