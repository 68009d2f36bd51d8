# A/B of the 128-row two-workgroups-per-CU conv01 (c01h.so): bf16 parity / encoder tests on the
# variant, the bit-identity dump, then the bench per library, two rounds (+ C4 from the extras legs)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VAP_LIB_AB=c01h.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bf16" > gpurun_out/c01h_pt.log 2>&1; rc=$?
echo "c01h tests: $(tail -1 gpurun_out/c01h_pt.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/c01h_pt.log | head -20; exit $rc; }
LIBS="c01h.so" bash tools/gpu_abv.sh c01h && python3 -c "import json;[print(f, json.load(open(f))['extras']['c4']['value']) for f in ['gpurun_out/c01h_default_1.json','gpurun_out/c01h_c01h.so_1.json','gpurun_out/c01h_default_2.json','gpurun_out/c01h_c01h.so_2.json']]"
