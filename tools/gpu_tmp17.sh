cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "60 or long or c4 or C4 or stream or first_forward" > gpurun_out/pt17.log 2>&1; rc=$?; tail -1 gpurun_out/pt17.log; [ $rc -eq 0 ] || exit 1
for e in "VAP_AB_DEFAULT=1" "VAP_TC_BE=0.4,0.7,0.88" "VAP_AB_DEFAULT=1" "VAP_TC_BE=0.4,0.7,0.88"; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --seconds 60 --batch 32 --steps 6 --warmup 2 > gpurun_out/c4ab.json 2>gpurun_out/c4ab.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/c4ab.json'));print(sys.argv[1], d['value'], d['ms_per_step'])" "$e"
done
