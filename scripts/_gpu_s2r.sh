#!/bin/bash
# XCD-major unit walks for the module-major fc forward and the fc dgrad GEMM: x3 tests, then the window (vs v16b:
# fc_fwd_mm2 44.1 us, fc_dgrad_gemm 2 x 249.7 us), repeated.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_v17.log 2>&1
tail -1 gpurun_out/r3/x3_tests_v17.log; grep -E "FAIL|Error" gpurun_out/r3/x3_tests_v17.log | head -8
grep -q " passed" gpurun_out/r3/x3_tests_v17.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_v17.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "fc_fwd_mm2\|fc_dgrad_gemm\|fc_wgrad_gm" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v17
prof x3_v17_rep
