# C4 (32 x 60 s) back-end chunk sweep on one box: VAP_TC_BE boundary sets (fractions of T = 3000) vs the rule
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --batch 32 --seconds 60 --steps 6 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/c4s_$n.json 2> gpurun_out/c4s_$n.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/c4s_$n.json')); print('%-8s %9.1f %7.3f' % ('$n', d['value'], d['ms_per_step']), flush=True)"
}
for r in 1 2; do
  run def$r VAP_X=0 || exit 1
  run a$r VAP_TC_BE=0.4267,0.6827,0.8533,0.9387 || exit 1
  run b$r VAP_TC_BE=0.512,0.768,0.896,0.9387 || exit 1
  run c$r VAP_TC_BE=0.3413,0.5973,0.768,0.896,0.9387 || exit 1
  run d$r VAP_TC_BE=0.4267,0.6827,0.8107,0.896,0.9387 || exit 1
done
