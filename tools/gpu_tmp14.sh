cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "split or first_forward or stream_bench" > gpurun_out/pt14.log 2>&1; rc=$?; tail -1 gpurun_out/pt14.log; [ $rc -eq 0 ] || exit 1
ENVS="-;VAP_BE_LOWPRIO=1;VAP_BE_LOWPRIO=1 VAP_BE_FRAC=0.53;-;VAP_BE_LOWPRIO=1;VAP_BE_LOWPRIO=1 VAP_BE_FRAC=0.53" STEPS=20 bash tools/gpu_env_ab.sh
