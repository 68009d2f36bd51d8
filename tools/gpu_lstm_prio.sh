cd $GRAFT_REPO_ROOT
for e in "VAP_X=0" "VAP_LSTM_PRIO=1" "VAP_LSTM_PRIO=3" "VAP_X=0"; do
  echo "== $e"
  env $e timeout -k 10 60 python tools/mb_lstm.py --variant 3 --iters 5 || exit 1
done
