cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/pmc_mb.sh rows rows || exit 1
python3 tools/pmc_read.py rows block > gpurun_out/pmc_rows_block.txt; python3 tools/pmc_read.py rows lnproj > gpurun_out/pmc_rows_lnproj.txt
cat gpurun_out/pmc_rows_block.txt | head -40
timeout -k 10 300 python tools/bench_stream.py --streams 128 > gpurun_out/c5.json 2> gpurun_out/c5.err; cut -c1-300 gpurun_out/c5.json
