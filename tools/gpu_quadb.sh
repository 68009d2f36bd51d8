# bf16 quad-split recurrence (lstm_quadb_kernel): kernel tests, then standalone step time against the pair kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "test_lstm" > gpurun_out/qb_k.log 2>&1; rc=$?
tail -3 gpurun_out/qb_k.log; [ $rc -eq 0 ] || exit $rc
for v in 3 5; do
  for S in 128 64; do
    timeout -k 10 60 python tools/mb_lstm.py --variant $v --S $S --T 2000 --iters 5 || exit 1
  done
done
VAP_LSTM_STAMPS=1 timeout -k 10 60 python tools/mb_lstm.py --variant 5 --S 128 --T 2000 --iters 2 || exit 1
# bench A/B: pair (default) vs quad, 20 s bench shape and C4 (32 x 60 s); then the GPU tests that run the model
if [ "$1" = bench ]; then
  for q in 0 1 0 1; do
    VAP_LSTM_QUAD=$q timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/qb_b$q.json 2> gpurun_out/qb_b$q.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/qb_b$q.json')); print('quad=$q 20s', d['value'], d['ms_per_step'], d.get('parity',{}).get('within_tolerance'), d['breakdown_ms_per_step'].get('lstm_rec'))"
    VAP_LSTM_QUAD=$q timeout -k 10 120 python -u bench.py --steps 6 --warmup 2 --batch 32 --seconds 60 --no-cpu-baseline --no-extras > gpurun_out/qb_c$q.json 2> gpurun_out/qb_c$q.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/qb_c$q.json')); print('quad=$q C4', d['value'], d['ms_per_step'])"
  done
fi
