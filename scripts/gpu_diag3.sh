#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in plain eager sync_rollout sync_opt barrier; do
  timeout -k 10 120 python -u scripts/diag_pipeline2.py 5000 $m > gpurun_out/diag3_$m.log 2>&1 || { echo "FAIL $m"; tail -5 gpurun_out/diag3_$m.log; exit 1; }
  tail -1 gpurun_out/diag3_$m.log | cut -c1-300
done
