# schedule sweep after convk4h (faster conv2..4 on the front-end stream): each configuration three
# times, interleaved with the default
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/sw6_$n.json 2> gpurun_out/sw6_$n.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/sw6_$n.json')); print('%-10s %9.1f %7.3f' % ('$n', d['value'], d['ms_per_step']), flush=True)"
}
for r in 1 2 3; do
  run def$r VAP_X=0 || exit 1
  run fe10$r VAP_TC_FE=0.1,0.3,0.5,0.7,0.85 || exit 1
  run fe08$r VAP_TC_FE=0.08,0.26,0.46,0.66,0.84 || exit 1
  run fe4p$r VAP_TC_FE=0.12,0.34,0.58,0.8 || exit 1
  run be62$r VAP_TC_BE=0.62 || exit 1
  run be66$r VAP_TC_BE=0.66 || exit 1
done
