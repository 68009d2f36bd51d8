# A/B bench: GPU tests, then bench with env A (default) and env B ($AB_ENV)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
for run in A B; do
  if [ $run = B ]; then export $AB_ENV; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_$run.json 2>gpurun_out/ab_$run.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$run.json'));print('$run', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['breakdown_ms_per_step'])"
done
