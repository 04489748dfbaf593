#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -15
exit $rc
