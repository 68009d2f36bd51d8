set -o pipefail
cd $GRAFT_REPO_ROOT
VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 bash tools/pmc_traffic.sh v9 && echo TRAFFIC_OK
