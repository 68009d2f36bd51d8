cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS="-;gxnt.so" KTESTS="bench or first_forward or exchange_tags" bash tools/gpu_var.sh v2 || exit 1
VAP_LIB_AB=gxnt.so VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 bash tools/pmc_traffic.sh gxnt || exit 1
python3 tools/traffic_json.py gxnt gpurun_out/gxnt_traffic.json > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/gxnt_traffic.json'))
for k,v in d['per_kernel_KiB'].items():
    if 'gemm2' in k: print(k[:50], v)"
TAILN=9 bash tools/gpu_handoff.sh
