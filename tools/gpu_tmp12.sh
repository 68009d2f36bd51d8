cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS="-;attn6ng.so;attn6.so" KTESTS="attention or bench or stream_bench or vs_reference" MB_WHICH=attn bash tools/gpu_var.sh v5
