set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 4 5 6 8; do
  VAP_TIME_CHUNKS=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/tc_$c.json 2>gpurun_out/tc_$c.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/tc_$c.json'));print($c, d['value'], d['ms_per_step'], d['breakdown_ms_per_step'])"
done
