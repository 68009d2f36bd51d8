# Diagnostic builds (outputs not meaningful): the bench per library in LIBS, printing the dominant
# kernel's isolated / shared ms per launch and the breakdown.  Usage: LIBS="a.so b.so" tools/gpu_diag.sh <tag>
set -o pipefail
TAG=${1:-diag}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in default $LIBS; do
    if [ $lib = default ]; then e="VAP_AB_DEFAULT=1"; else e="VAP_LIB_AB=$lib"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --steps 10 > gpurun_out/${TAG}_${lib}_$r.json 2>gpurun_out/${TAG}_${lib}_$r.err || { tail -20 gpurun_out/${TAG}_${lib}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_${lib}_$r.json'));b=d['breakdown_ms_per_step'];r=d['roofline'];print(sys.argv[1], d['value'], d['ms_per_step'], 'iso', r.get('isolated',{}).get('ms_per_launch'), 'shared', r['ms_per_launch'], {k: round(v, 3) for k, v in b.items() if v})" "$lib"
  done
done
