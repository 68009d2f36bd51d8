# N-way A/B on one GPU box: quick kernel tests (pytest -k $KTESTS), every GPU test, then per env
# setting in ENVS (';'-separated, '-' = defaults) the microbenchmarks (MB_WHICH) and the bench,
# two rounds in alternating order.  Usage: ENVS="-;VAP_LIB_AB=x.so" KTESTS="block" tools/gpu_abn.sh <tag>
set -o pipefail
TAG=${1:-abn}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$KTESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$KTESTS" > gpurun_out/${TAG}_ptk.log 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_ptk.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOFULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_pt.log
  [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra SETS <<< "${ENVS:--}"
i=0
for e in "${SETS[@]}"; do
  i=$((i+1)); [ "$e" = "-" ] && e="VAP_AB_DEFAULT=1"
  if [ -n "$MB_WHICH" ]; then
    env $e timeout -k 10 300 python -u tools/mb_kernels.py --which $MB_WHICH --iters 30 > gpurun_out/${TAG}_mb$i.log 2>&1 || exit 1
    echo "== $e"; grep -v "^{\|amdgpu.ids" gpurun_out/${TAG}_mb$i.log
  fi
done
for r in 1 2; do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1)); [ "$e" = "-" ] && e="VAP_AB_DEFAULT=1"
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG}_b${i}_$r.json 2>gpurun_out/${TAG}_b${i}_$r.err || exit 1
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_b${i}_$r.json'));b=d['breakdown_ms_per_step'];print(sys.argv[1], d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in b.items() if v})" "$e"
  done
done
