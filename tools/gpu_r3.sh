# Round-3 GPU check: full GPU test suite (printing measured errors), per-fixture bf16/fp32 errors vs
# the reference, then the default bench line.  Usage: tools/gpu_r3.sh <tag>
set -o pipefail
TAG=${1:-r3}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pt.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bf16_errors.py bf16 > gpurun_out/${TAG}_err_bf16.json 2> gpurun_out/${TAG}_err_bf16.log &&
timeout -k 10 300 python -u tools/bf16_errors.py fp32 > gpurun_out/${TAG}_err_fp32.json 2> gpurun_out/${TAG}_err_fp32.log &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
cat gpurun_out/${TAG}_bench.json
