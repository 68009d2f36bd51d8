# attention A/B (GPU box): GPU tests, attention + row-kernel microbenchmarks, bench with the default
# and with $AB_ENV.  Usage: AB_ENV="VAP_ATTN3=1" tools/gpu_attn_ab.sh <tag>
set -o pipefail
TAG=${1:-ab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_pt.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_kernels.py --which ${MB_WHICH:-attn,rows} --iters 30 > gpurun_out/${TAG}_mbA.log 2>&1 && grep -v "^{" gpurun_out/${TAG}_mbA.log &&
env $AB_ENV timeout -k 10 300 python -u tools/mb_kernels.py --which attn --iters 30 > gpurun_out/${TAG}_mbB.log 2>&1 && grep -v "^{" gpurun_out/${TAG}_mbB.log || exit 1
for run in A B A B; do
  if [ $run = B ]; then E="$AB_ENV"; else E="VAP_AB_DEFAULT=1"; fi
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG}_$run.json 2>gpurun_out/${TAG}_$run.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$run.json'));b=d['breakdown_ms_per_step'];print('$run', d['value'], d['ms_per_step'], 'attn', b['attn'], 'tr', b['tr_gemm'])"
done
