# conv01h A/B, then (only if it passed) the closing run on the default library
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_ab_c01h.sh > gpurun_out/combo_c01h.txt 2>&1; rc=$?
tail -12 gpurun_out/combo_c01h.txt
[ $rc -eq 0 ] || { echo "c01h failed rc=$rc"; exit $rc; }
bash tools/gpu_close_r4.sh r4s6b
