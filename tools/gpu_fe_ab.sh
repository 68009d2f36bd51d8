cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ENVS="${ENVS:--;VAP_FE_STREAMS=1}" STEPS=20 bash tools/gpu_env_ab.sh && bash tools/gpu_trace.sh ${TAG:-fe}
