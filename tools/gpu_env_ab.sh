# Bench under several env settings in one GPU call: ENVS="A=1 B=2;C=3" (';' separates settings,
# '-' = defaults); prints value / ms per step / LSTM time per setting.  GPU box.
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra SETS <<< "${ENVS:--}"
i=0
for e in "${SETS[@]}"; do
  i=$((i+1))
  if [ "$e" = "-" ]; then e="VAP_AB_DEFAULT=1"; fi
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-20} > gpurun_out/ab_$i.json 2>gpurun_out/ab_$i.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$i.json'));b=d['breakdown_ms_per_step'];print(sys.argv[1], d['value'], d['ms_per_step'], 'lstm', b['lstm_rec'], 'tr', b['tr_gemm'], 'attn', b['attn'])" "$e"
done
