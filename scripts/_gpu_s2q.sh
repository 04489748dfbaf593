#!/bin/bash
# conv1 forward with the input band in LDS (conv1_fwd_band_x2): x3 tests, windows for the default and conv1_fwd_x2.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_v16b.log 2>&1
tail -1 gpurun_out/r3/x3_tests_v16b.log; grep -E "FAIL|Error|^layer 0|fp32x" gpurun_out/r3/x3_tests_v16b.log | head -16
grep -q " passed" gpurun_out/r3/x3_tests_v16b.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_v16b.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd\|pong_step\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v16b
prof x3_v16b_noband --kernel-opt fast_conv_set_x3_c1_band=0
prof x3_v16b_rep
