# A/B of the 128-row two-workgroups-per-CU convk4 (ck4h.so): convk4 kernel tests and the bf16 parity
# tests on the variant, the bit-identity dump, then the bench per library, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VAP_LIB_AB=ck4h.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "convk4 or bf16" > gpurun_out/ck4h_pt.log 2>&1; rc=$?
echo "ck4h tests: $(tail -1 gpurun_out/ck4h_pt.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/ck4h_pt.log | head -20; exit $rc; }
LIBS="ck4h.so" bash tools/gpu_abv.sh ck4h && python3 -c "import json;[print(f, json.load(open(f))[\"extras\"][\"c4\"][\"value\"]) for f in [\"gpurun_out/ck4h_default_1.json\",\"gpurun_out/ck4h_ck4h.so_1.json\",\"gpurun_out/ck4h_default_2.json\",\"gpurun_out/ck4h_ck4h.so_2.json\"]]"
