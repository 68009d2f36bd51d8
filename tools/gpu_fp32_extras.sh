set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/x1.json 2> gpurun_out/x1.err || { tail -20 gpurun_out/x1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/x1.json'));print(d['value'], {k:(v['value'],v['ms_per_step']) for k,v in d['extras'].items()})"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --precision fp32 --steps 5 --warmup 3 > gpurun_out/x2.json 2> gpurun_out/x2.err || { tail -20 gpurun_out/x2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/x2.json'));print('fp32 alone', d['value'], d['ms_per_step'])"
