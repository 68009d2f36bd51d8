# Round-4 GPU check: the GPU test suite (printing measured errors), then the default bench line (with its
# extras: C4, fp32 parity mode, fixture errors, CPU baseline).  Usage: tools/gpu_r4.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r4}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu $K > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pt.log | tail -3
grep -E "max abs err" gpurun_out/${TAG}_pt.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json'))
print(d['value'], d['ms_per_step'], json.dumps(d.get('parity')), json.dumps(d.get('extras')), json.dumps(d.get('cpu_baseline')))"
