# attention PMC A/B and block-kernel phase stamps at the bench's chunk size (GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_ENV="VAP_ATTN3=1" bash tools/pmc_attn.sh at && python3 tools/pmc_read.py atA attn && python3 tools/pmc_read.py atB attn &&
timeout -k 10 120 python3 tools/stamps_block.py --rows 81920 --cus 0 > gpurun_out/stamps_block.log 2>&1 && cat gpurun_out/stamps_block.log
