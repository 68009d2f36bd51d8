cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "long_clip_schedule" > gpurun_out/pt19.log 2>&1; rc=$?; tail -1 gpurun_out/pt19.log; [ $rc -eq 0 ] || exit 1
ENVS="-;VAP_TC_BE=0.6;VAP_TC_BE=0.68;VAP_TC_BE=0.704;-;VAP_TC_BE=0.6;VAP_TC_BE=0.68;VAP_TC_BE=0.704" STEPS=20 bash tools/gpu_env_ab.sh
