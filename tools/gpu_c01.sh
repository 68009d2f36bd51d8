# conv01 A/B: W1 two units ahead (VAP_C01_W3 build, c01w3.so) against the default; kernel tests on both builds
set -o pipefail
cd $GRAFT_REPO_ROOT
VAP_LIB_AB=c01w3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv01 or conv0" > gpurun_out/c01_k.log 2>&1; rc=$?
tail -2 gpurun_out/c01_k.log; [ $rc -eq 0 ] || exit $rc
ENVS="-;VAP_LIB_AB=c01w3.so" NOFULL=1 bash tools/gpu_abn.sh c01ab
