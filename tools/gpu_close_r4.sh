# Round-4 closing GPU run: full GPU suite + default bench line (tools/gpu_r4.sh), rocprofv3 kernel stats of the
# bench, then per-dispatch HBM traffic of the bench workload alone (serial schedule, no extras).
set -o pipefail
TAG=${1:-close}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_r4.sh $TAG || exit 1
bash tools/profile.sh ${TAG}_prof --steps 10 --warmup 3 --no-extras > /dev/null 2>&1 || exit 1
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_${TAG}_prof/kernel_stats.csv')))
for x in r[:12]: print('  %-58s %6s calls %9.1f us avg %6.2f%%'%(x['Name'][:58],x['Calls'],float(x['AverageNs'])/1e3,float(x['Percentage'])))"
VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 timeout -k 10 400 bash tools/pmc_traffic.sh ${TAG} --no-extras > /dev/null || exit 1
python3 tools/traffic_json.py ${TAG} gpurun_out/${TAG}_traffic_pmc.json > /dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_traffic_pmc.json'))['per_kernel_KiB']
for k,v in d.items():
    if v['FETCH_SIZE_KiB_per_dispatch'] > 10000: print('  %-70s F %9.1f MB  W %9.1f MB  x%d' % (k[:70], v['FETCH_SIZE_KiB_per_dispatch']*1.024/1000, v['WRITE_SIZE_KiB_per_dispatch']*1.024/1000, v['dispatches']))"
