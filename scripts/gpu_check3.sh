#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -x -q -s -k "lstm" > gpurun_out/pytest_lstm.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert|^\{" gpurun_out/pytest_lstm.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python scripts/solve.py --preset pong --minutes 1.5 --lr 0.003 --env-reduction sum --debug --report-every 20 --curve gpurun_out/anom.jsonl > gpurun_out/anom.log 2>&1 || { tail -5 gpurun_out/anom.log; exit 3; }
grep anomaly gpurun_out/anom.log | head -4
SWEEP_FILE=scripts/sweep_configs2.txt SWEEP_MIN=3 bash scripts/gpu_sweep.sh
