#!/bin/bash
# GPU tests + rocprofv3 kernel stats of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
exit $rc
