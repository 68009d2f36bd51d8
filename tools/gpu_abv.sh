# A/B of variant libraries on one GPU box: for each library in LIBS (space-separated _lib names),
# the kernel tests selected by KTESTS and a bit-identity check of a bench-shaped forward against the
# default library; then the bench for the default and every variant, two rounds in alternating order.
# Usage: LIBS="a.so b.so" KTESTS="convk4" tools/gpu_abv.sh <tag>
set -o pipefail
TAG=${1:-abv}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_dump.py --out gpurun_out/${TAG}_ref.npz > gpurun_out/${TAG}_dump0.log 2>&1 || { tail -20 gpurun_out/${TAG}_dump0.log; exit 1; }
for lib in $LIBS; do
  if [ -n "$KTESTS" ]; then
    VAP_LIB_AB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$KTESTS" > gpurun_out/${TAG}_${lib}_pt.log 2>&1; rc=$?
    echo "== $lib kernel tests: $(tail -1 gpurun_out/${TAG}_${lib}_pt.log)"
    [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_${lib}_pt.log; exit $rc; }
  fi
  VAP_LIB_AB=$lib timeout -k 10 200 python -u tools/ab_dump.py --out gpurun_out/${TAG}_${lib}.npz > gpurun_out/${TAG}_${lib}_dump.log 2>&1 || { tail -20 gpurun_out/${TAG}_${lib}_dump.log; exit 1; }
  python tools/ab_dump.py --compare gpurun_out/${TAG}_ref.npz gpurun_out/${TAG}_${lib}.npz | tr '\n' ' '; echo " <- $lib vs default"
done
for r in 1 2; do
  for lib in default $LIBS; do
    if [ $lib = default ]; then e="VAP_AB_DEFAULT=1"; else e="VAP_LIB_AB=$lib"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG}_${lib}_$r.json 2>gpurun_out/${TAG}_${lib}_$r.err || { tail -20 gpurun_out/${TAG}_${lib}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_${lib}_$r.json'));b=d['breakdown_ms_per_step'];print(sys.argv[1], d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in b.items() if v})" "$lib"
  done
done
