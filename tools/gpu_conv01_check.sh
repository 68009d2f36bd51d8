set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bf16 or stream" > gpurun_out/conv01_pytest.log 2>&1 ; echo "pytest rc=$?"; tail -5 gpurun_out/conv01_pytest.log
timeout -k 10 120 python tools/stamps_conv01.py > gpurun_out/conv01_stamps.log 2>&1 && head -4 gpurun_out/conv01_stamps.log &&
for d in; do echo "== DIAG $d"; VAP_CONV01_DIAG=$d timeout -k 10 120 python tools/stamps_conv01.py > gpurun_out/conv01_d$d.log 2>&1 && head -3 gpurun_out/conv01_d$d.log | tail -2 || exit 1; done &&
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/conv01_bench.json 2> gpurun_out/conv01_bench.err && cut -c 1-900 gpurun_out/conv01_bench.json
