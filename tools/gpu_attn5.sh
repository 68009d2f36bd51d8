set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attn or attention" > gpurun_out/a5_ptk.log 2>&1; rc=$?
tail -2 gpurun_out/a5_ptk.log; [ $rc -eq 0 ] || exit $rc
ENVS="-;VAP_ATTN_VER=4" MB_WHICH=attn bash tools/gpu_abn.sh a5 && bash tools/gpu_trace.sh r3a
