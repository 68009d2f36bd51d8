cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A="VAP_TC_FE=0.12,0.3,0.5,0.7,0.85"; B="VAP_TC_FE=0.12,0.3,0.52,0.74,0.88"; C="VAP_TC_FE=0.14,0.32,0.52,0.72,0.86"
ENVS="-;$A;$B;$C;-;$A;$B;$C" STEPS=20 bash tools/gpu_env_ab.sh
