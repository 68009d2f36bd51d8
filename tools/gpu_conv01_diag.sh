set -o pipefail
cd $GRAFT_REPO_ROOT
for d in ${DIAGS:-1 2 3 4 8}; do
  echo "== DIAG $d"
  VAP_CONV01_DIAG=$d timeout -k 10 120 python tools/stamps_conv01.py > gpurun_out/diag_$d.log 2>&1 && head -3 gpurun_out/diag_$d.log | tail -2 || exit 1
done
