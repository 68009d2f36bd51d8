cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS="-;ck4v.so;c01v.so;accv.so" KTESTS="conv or bench or first_forward or vs_reference" bash tools/gpu_var.sh v6
