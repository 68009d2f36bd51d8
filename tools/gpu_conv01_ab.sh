# conv01 variants (GPU box): GPU tests, bench A/B and SQ counters of the serial-schedule launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
ENVS="${ENVS:--;VAP_CONV01_V10=1;-}" STEPS=20 bash tools/gpu_env_ab.sh || exit 1
for i in 1 2 3; do python3 -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('conv1', d['breakdown_ms_per_step']['conv1'])"; done
bash tools/pmc_conv01.sh m && python3 tools/pmc_read.py m conv01
