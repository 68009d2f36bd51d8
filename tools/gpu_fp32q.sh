# quick fp32 parity-mode check: split GEMM / attention / LSTM kernel tests, then the fp32 bench line.
set -o pipefail
TAG=${1:-f}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "test_gemm or split or test_lstm or test_conv0" > gpurun_out/${TAG}_k.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_fp32.json 2> gpurun_out/${TAG}_fp32.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/${TAG}_fp32.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('breakdown_ms_per_step')), json.dumps(d.get('parity',{}).get('max_abs_err')))"
if [ "$2" = prof ]; then
  bash tools/profile.sh ${TAG}_prof --precision fp32 --steps 3 --warmup 1 --no-extras > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_${TAG}_prof/kernel_stats.csv')))
for x in r[:14]: print('  %-58s %6s calls %9.1f us avg %6.2f%%'%(x['Name'][:58],x['Calls'],float(x['AverageNs'])/1e3,float(x['Percentage'])))"
fi
