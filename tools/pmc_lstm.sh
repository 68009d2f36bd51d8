# SQ counters of the standalone resident LSTM (GPU box): where the ~6.4k cycles per step go
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_lstm
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU --output-format csv -d "$OUT" -o run -- python3 "$ROOT/tools/mb_lstm.py" --iters 1 > "$OUT/log.txt" 2>&1
f=$(find "$OUT" -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "lstm_resident" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(f"{k:32s} {v:16.0f}")
PY
