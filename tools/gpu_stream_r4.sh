# C5 streaming bench on one GPU (16 and 128 streams per GPU, the exact per-rank check included), plus the
# tightened bf16 tolerance tests.  Usage: tools/gpu_stream_r4.sh <tag>
set -o pipefail
TAG=${1:-r4}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "encoder_bf16 or attention_maps_bf16" > gpurun_out/${TAG}_pt.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_pt.log
timeout -k 10 200 python -u tools/bench_stream.py --streams-per-gpu 16 > gpurun_out/${TAG}_c5_16.json 2> gpurun_out/${TAG}_c5_16.err || exit 1
timeout -k 10 200 python -u tools/bench_stream.py --streams-per-gpu 128 > gpurun_out/${TAG}_c5_128.json 2> gpurun_out/${TAG}_c5_128.err || exit 1
cut -c1-600 gpurun_out/${TAG}_c5_16.json gpurun_out/${TAG}_c5_128.json
