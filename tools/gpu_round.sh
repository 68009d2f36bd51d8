# GPU round check: gpu tests, bench line, rocprofv3 kernel stats.  Usage: tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
bash tools/profile.sh $TAG --steps 5 --warmup 2 && echo PROF_OK
