# in-kernel clock (s_memtime / s_memrealtime) of convk4 alone and conv01 inside bench forwards
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
REPS=3 timeout -k 10 120 python tools/stamps_convk4.py > gpurun_out/clk_ck4_cold.txt 2>&1 || exit 1
grep wg gpurun_out/clk_ck4_cold.txt | head -3
REPS=3000 timeout -k 10 120 python tools/stamps_convk4.py > gpurun_out/clk_ck4_hot.txt 2>&1 || exit 1
grep wg gpurun_out/clk_ck4_hot.txt
REPS=300 timeout -k 10 200 python tools/stamps_conv01.py > gpurun_out/clk_c01_bench.txt 2>&1 || exit 1
grep wg gpurun_out/clk_c01_bench.txt
