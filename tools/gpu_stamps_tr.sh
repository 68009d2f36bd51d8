set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/stamps_ffn.py --rows 32000 > gpurun_out/st_ffn.log 2>&1; tail -25 gpurun_out/st_ffn.log
timeout -k 10 120 python tools/mb_kernels.py --rows 32000 --which rowpanel,ffn,attn --packed > gpurun_out/mb_tr.log 2>&1; tail -12 gpurun_out/mb_tr.log
