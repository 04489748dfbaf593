#!/bin/bash
# per-sample LDS-tile conv2/conv3 forward + 8-column slot sum: x3 tests, windows for the default and the row kernels.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_v14.log 2>&1
tail -1 gpurun_out/r3/x3_tests_v14.log; grep -E "FAIL|Error|^layer" gpurun_out/r3/x3_tests_v14.log | head -16
grep -q " passed" gpurun_out/r3/x3_tests_v14.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_v14.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv_fwd\|fc_slot\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v14
prof x3_v14_rows --kernel-opt fast_conv_set_x3_fwd_tile=0
prof x3_v14_rep
