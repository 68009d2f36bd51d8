# Bench sweep over env settings (GPU box): SWEEP="A=1 B=x,y;A=3" -- configs separated by ';', vars by spaces
set -o pipefail
cd $GRAFT_REPO_ROOT
i=0
IFS=';' read -ra CFGS <<< "$SWEEP"
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  ( for kv in $cfg; do export "$kv"; done
    timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sw_$i.json 2>gpurun_out/sw_$i.err ) || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sw_$i.json'));print('$cfg', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['breakdown_ms_per_step'].items() if v})"
done
