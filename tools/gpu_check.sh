# GPU check of a change: the GPU tests, then the rocprofv3 kernel stats of a short bench.
# Usage: tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-chk}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pt.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh $TAG --steps 10 --warmup 3 && echo PROF_OK && cut -c1-200 gpurun_out/prof_$TAG/bench.json
