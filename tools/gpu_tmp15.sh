cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/handoff.py --batch 32 --seconds 60 --iters 6 | tail -14
