# full GPU round + conv01 stamps + HBM traffic capture (serial schedule) for the roofline (GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh ${TAG:-r2e} && \
timeout -k 10 120 python tools/stamps_conv01.py && \
VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 bash tools/pmc_traffic.sh r2 && echo TRAFFIC_OK
