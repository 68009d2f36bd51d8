# Other BASELINE configs on one GPU: C4 (32 x 60 s bf16), the fp32 parity mode at the bench config,
# C5 streaming (128 streams, 10 s window, 1 s hop).  Usage: tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-r3}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --seconds 60 --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err &&
timeout -k 10 300 python -u bench.py --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_fp32.json 2> gpurun_out/${TAG}_fp32.err &&
timeout -k 10 300 python -u tools/bench_stream.py --streams 128 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err &&
timeout -k 10 300 python -u tools/bench_stream.py --streams 128 --check-each > gpurun_out/${TAG}_c5_checked.json 2> gpurun_out/${TAG}_c5c.err &&
tail -c 400 gpurun_out/${TAG}_c4.json gpurun_out/${TAG}_fp32.json gpurun_out/${TAG}_c5.json gpurun_out/${TAG}_c5_checked.json
