cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/pmc_conv.sh c01 conv01m && python3 tools/pmc_read.py c01 conv01m > gpurun_out/pmc_c01.txt && cat gpurun_out/pmc_c01.txt
bash tools/pmc_conv.sh ck4 convk4 && python3 tools/pmc_read.py ck4 convk4 > gpurun_out/pmc_ck4.txt && cat gpurun_out/pmc_ck4.txt
