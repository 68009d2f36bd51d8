cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_first.py > gpurun_out/diag_first.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/diag_first.log | head -8
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
VARS="-;attn5.so;attn5o3.so;rh2.so" KTESTS="attention or bench or stream_bench or block or lnproj or heads" MB_WHICH=attn bash tools/gpu_var.sh v1 || exit 1
ENVS="VAP_BE_SPLIT=1;VAP_BE_SPLIT=2" STEPS=20 bash tools/gpu_env_ab.sh
