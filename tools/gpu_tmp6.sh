cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS="-;dssmall.so" KTESTS="bench or first_forward or downsample or batch_invariance" bash tools/gpu_var.sh v3 || exit 1
for r in 1 2; do for ev in -1 1 0; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --roofline-events $ev > gpurun_out/ev_${ev}_$r.json 2>gpurun_out/ev_${ev}_$r.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ev_${ev}_$r.json'));print('events', sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['launches'])" $ev
done; done
timeout -k 10 120 python tools/stamps_convk4.py > gpurun_out/stamps_convk4.log 2>&1; tail -15 gpurun_out/stamps_convk4.log
