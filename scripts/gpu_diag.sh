#!/bin/bash
# Engine-vs-oracle gradient test + learning diagnostic (HIP vs torch backend).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -q -x -s -k "gradient_matches_oracle" > gpurun_out/grad_test.log 2>&1
rc=$?
tail -15 gpurun_out/grad_test.log
# 0 = pass, 1 = assertion failure (keep going); anything else (abort/segv/timeout) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/diag_learning.py --seconds ${DIAG_SEC:-150} $DIAG_ARGS > gpurun_out/diag.log 2>&1
rc=$?
tail -40 gpurun_out/diag.log
exit $rc
