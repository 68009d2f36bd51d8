# schedule sweep on one box (bench 20 s, B = 64): each configuration twice, interleaved with the default
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/sw_$n.json 2> gpurun_out/sw_$n.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$n.json')); print('%-10s %9.1f %7.3f' % ('$n', d['value'], d['ms_per_step']), flush=True)"
}
for r in 1 2; do
  run def$r VAP_X=0 || exit 1
  run fe6$r VAP_TC_FE=0.1,0.25,0.42,0.6,0.76,0.89 || exit 1
  run fea$r VAP_TC_FE=0.1,0.27,0.46,0.66,0.84 || exit 1
  run feb$r VAP_TC_FE=0.14,0.33,0.53,0.72,0.87 || exit 1
  run be60$r VAP_TC_BE=0.6 || exit 1
  run be68$r VAP_TC_BE=0.68 || exit 1
  run bf47$r VAP_BE_FRAC=0.47 || exit 1
  run bf53$r VAP_BE_FRAC=0.53 || exit 1
done
