# Session-6 A/B: attention row sums by VALU adds (attvs.so: parity + attention kernel tests), x stores plain / nt
# (blkx1.so / blkx2.so: bit identity), then the bench per library, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VAP_LIB_AB=attvs.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bf16 or attention" > gpurun_out/s6_attvs_pt.log 2>&1; rc=$?
echo "attvs tests: $(tail -1 gpurun_out/s6_attvs_pt.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/s6_attvs_pt.log | head -20; exit $rc; }
LIBS="blkx1.so blkx2.so attvs.so" KTESTS="block or lnproj" bash tools/gpu_abv.sh s6
