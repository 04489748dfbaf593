#!/bin/bash
# module-major LDS-tiled fc forward with 3 k-steps of loads in flight: x3 tests, then windows for the default
# (fc1 module-major, fc2 path-major), fc2 module-major too, and path-major for both.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_mm2b.log 2>&1
tail -1 gpurun_out/r3/x3_tests_mm2b.log; grep -E "FAIL|Error" gpurun_out/r3/x3_tests_mm2b.log | head -12
grep -q " passed" gpurun_out/r3/x3_tests_mm2b.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_mm2b.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "fc_fwd\|fc_slot\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v12
PATHNET_X3_FC_MM_MIN_K=0 prof x3_v12_mmall
PATHNET_X3_FC_MM=0 prof x3_v12_pm
prof x3_v12_rep
