#!/bin/bash
# tests + timing profile + one PMC pass (counters in their own run, no sys/runtime trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/prof.log
if [ $rc -ne 0 ]; then exit $rc; fi
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph > gpurun_out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 gpurun_out/pmc.log
exit $rc
