# gemm2 spill fix: kernel tests + 3-way bench A/B (tools/gpu_abn.sh), then per-dispatch HBM traffic (serial schedule)
set -o pipefail
cd $GRAFT_REPO_ROOT
ENVS="-;VAP_LIB_AB=g2old.so;VAP_LIB_AB=dsmall.so;VAP_LIB_AB=blknt.so;VAP_LIB_AB=attold.so" KTESTS="gemm or block or lnproj or attention" NOFULL=1 bash tools/gpu_abn.sh g2ab || exit 1
VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 timeout -k 10 400 bash tools/pmc_traffic.sh r4 || exit 1
python3 tools/traffic_json.py r4 gpurun_out/r4_traffic_pmc.json && python3 -c "
import json; d=json.load(open('gpurun_out/r4_traffic_pmc.json'))
for k,v in (d.items() if isinstance(d,dict) else []):
    if 'gemm2' in k or 'down' in k: print(k[:70], v)"
