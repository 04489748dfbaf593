#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in nofence fence; do
  timeout -k 10 150 python -u scripts/diag_pipeline3.py 20000 $m > gpurun_out/diag4_$m.log 2>&1 || { echo "FAIL $m"; tail -5 gpurun_out/diag4_$m.log; exit 1; }
  tail -1 gpurun_out/diag4_$m.log | cut -c1-3000
done
