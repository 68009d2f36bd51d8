set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -${TAILN:-8}; tail -3 gpurun_out/pytest_gpu.log; exit $rc
