set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_stream.py > gpurun_out/stream_graph.json 2>gpurun_out/stream_graph.err && cat gpurun_out/stream_graph.json &&
VAP_STREAM_GRAPH=0 timeout -k 10 300 python tools/bench_stream.py > gpurun_out/stream_eager.json 2>gpurun_out/stream_eager.err && cat gpurun_out/stream_eager.json
