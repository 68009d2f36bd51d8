cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ENVS="-;VAP_TC_FE=0.1,0.27,0.48,0.72,0.86;VAP_TC_FE=0.1,0.27,0.48,0.66,0.82;VAP_TC_FE=0.1,0.25,0.42,0.6,0.78,0.9;VAP_TC_FE=0.12,0.3,0.5,0.7,0.85;-" STEPS=20 bash tools/gpu_env_ab.sh
