cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for e in "VAP_AB_DEFAULT=1" "VAP_TC_FE=0.04,0.12,0.3,0.5,0.7,0.85" "VAP_TC_FE=0.04,0.3,0.5,0.7,0.85" "VAP_TC_FE=0.06,0.2,0.4,0.6,0.8" "VAP_AB_DEFAULT=1" "VAP_TC_FE=0.04,0.12,0.3,0.5,0.7,0.85"; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --seconds 60 --batch 32 --steps 6 --warmup 2 > gpurun_out/c4ab.json 2>gpurun_out/c4ab.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/c4ab.json'));print(sys.argv[1], d['value'], d['ms_per_step'])" "$e"
done
