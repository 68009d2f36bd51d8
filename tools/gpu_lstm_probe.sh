# Pair-LSTM step decomposition (GPU box): default, plain-store exchange, no exchange wait, stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
for e in "VAP_X=0" "VAP_LSTM_XPLAIN=1" "VAP_LSTM_XNOWAIT=1" "VAP_LSTM_STAMPS=1"; do
  echo "== $e"
  env $e timeout -k 10 60 python tools/mb_lstm.py --variant 3 --iters 5 || exit 1
done
