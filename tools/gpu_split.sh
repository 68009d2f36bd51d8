# fp32 parity mode on split-bf16 operands: kernel tests, every fp32 parity test, fp32 errors vs the reference
# fixtures, short fp32 benches (split default, + quad recurrence, exact fp32-MFMA kernels).
# Usage: tools/gpu_split.sh <tag> [quad]   (quad: run the parity tests / errors with VAP_FP32_QUAD=1)
set -o pipefail
TAG=${1:-split}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
[ "$2" = quad ] && export VAP_FP32_QUAD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "test_gemm or test_lstm or test_attention or test_conv0" > gpurun_out/${TAG}_k.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -rP --timeout 300 --timeout-method thread -m gpu -k "fp32 or m32 or oracle or mono or attention_maps_fp32" > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bf16_errors.py fp32 > gpurun_out/${TAG}_err_fp32.json 2> gpurun_out/${TAG}_err_fp32.log || exit 1
cat gpurun_out/${TAG}_err_fp32.json
timeout -k 10 300 python -u bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_fp32.json 2> gpurun_out/${TAG}_fp32.err || exit 1
VAP_FP32_QUAD=1 timeout -k 10 300 python -u bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_fp32q.json 2> gpurun_out/${TAG}_fp32q.err || exit 1
VAP_FP32_EXACT=1 timeout -k 10 300 python -u bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_fp32x.json 2> gpurun_out/${TAG}_fp32x.err || exit 1
python3 -c "
import json
for f in ['gpurun_out/${TAG}_fp32.json','gpurun_out/${TAG}_fp32q.json','gpurun_out/${TAG}_fp32x.json']:
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], json.dumps(d.get('breakdown_ms_per_step')), json.dumps(d.get('parity',{}).get('max_abs_err')))"
