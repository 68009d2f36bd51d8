# Recurrence hand-off timelines under several env settings (GPU box): ENVS="A=1;B=2" ('-' = defaults)
cd $GRAFT_REPO_ROOT
IFS=';' read -ra SETS <<< "${ENVS:--}"
for e in "${SETS[@]}"; do
  if [ "$e" = "-" ]; then e="VAP_AB_DEFAULT=1"; fi
  echo "== $e"
  env $e timeout -k 10 120 python tools/handoff.py --iters 12 | tail -${TAILN:-7} || exit 1
done
