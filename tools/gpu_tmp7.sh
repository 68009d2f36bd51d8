cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS="-;ck4old.so" KTESTS="convk4 or bench or first_forward or vs_reference" bash tools/gpu_var.sh v4 || exit 1
timeout -k 10 120 python tools/stamps_convk4.py > gpurun_out/stamps_convk4_new.log 2>&1; tail -12 gpurun_out/stamps_convk4_new.log
