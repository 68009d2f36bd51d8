# Variant libraries on one GPU box: per VARS entry (';'-separated, '-' = the default library) the
# kernel / parity tests selected by KTESTS under VAP_LIB_AB, the microbenchmarks MB_WHICH, then
# the bench in two alternating rounds.  Usage: VARS="-;attn5.so" KTESTS="attention" MB_WHICH=attn tools/gpu_var.sh <tag>
set -o pipefail
TAG=${1:-var}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${VARS:--}"
env_of() { [ "$1" = "-" ] && echo "VAP_AB_DEFAULT=1" || echo "VAP_LIB_AB=$1"; }
i=0
for v in "${SETS[@]}"; do
  i=$((i+1)); e=$(env_of "$v")
  if [ -n "$KTESTS" ]; then
    env $e timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$KTESTS" > gpurun_out/${TAG}_pt$i.log 2>&1; rc=$?
    echo "== $v tests: $(tail -1 gpurun_out/${TAG}_pt$i.log)"
    [ $rc -eq 0 ] || exit $rc
  fi
  if [ -n "$MB_WHICH" ]; then
    env $e timeout -k 10 300 python -u tools/mb_kernels.py --which $MB_WHICH --iters 30 > gpurun_out/${TAG}_mb$i.log 2>&1 || exit 1
    grep -v "^{\|amdgpu.ids" gpurun_out/${TAG}_mb$i.log
  fi
done
for r in 1 2; do
  i=0
  for v in "${SETS[@]}"; do
    i=$((i+1)); e=$(env_of "$v")
    env $e ${BENV} timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG}_b${i}_$r.json 2>gpurun_out/${TAG}_b${i}_$r.err || exit 1
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_b${i}_$r.json'));b=d['breakdown_ms_per_step'];print(sys.argv[1], d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in b.items() if v})" "$v"
  done
done
