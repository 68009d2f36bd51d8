# measurement round: kernel stats + timeline of the default bench, PMC HBM traffic (serial schedule), attention PMC
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/profile.sh r3s6 --steps 5 --warmup 2 && cat gpurun_out/prof_r3s6/bench.json | cut -c1-300 || exit 1
bash tools/gpu_trace.sh r3s6 || exit 1
VAP_TIME_CHUNKS=0 VAP_MICROBATCHES=1 bash tools/pmc_traffic.sh r3s6 || exit 1
python3 tools/traffic_json.py r3s6 gpurun_out/r3_traffic_pmc.json || exit 1
bash tools/pmc_attn.sh r3s6 || exit 1
echo ALLDONE
