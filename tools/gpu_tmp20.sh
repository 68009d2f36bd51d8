cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in - ${VARS}; do
  for m in 0 1 3 5; do
    if [ "$v" = "-" ]; then e=VAP_AB_DEFAULT=1; else e=VAP_LIB_AB=$v; fi
    env $e VAP_CONVK4_DBG=$m timeout -k 10 120 python tools/mb_convk4.py 128 16000 30 2>&1 | grep convk4 || exit 1
  done
done
timeout -k 10 120 python tools/stamps_convk4.py > gpurun_out/stamps_ck4.txt 2>&1 || exit 1
cat gpurun_out/stamps_ck4.txt | grep wg
