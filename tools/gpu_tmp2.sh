cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
ENVS="-;VAP_BE_SPLIT=3;VAP_TC_BE=0.704;VAP_TC_BE=0.576;VAP_TC_BE=0.512,0.768;VAP_TC_FE=0.1,0.25,0.45,0.7;VAP_TC_FE=0.12,0.3,0.52,0.76;-;VAP_BE_SPLIT=3" STEPS=20 bash tools/gpu_env_ab.sh
