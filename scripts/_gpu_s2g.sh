#!/bin/bash
# fp32x kernel A/B: x3 tests, then steady-state windows for the defaults (swapped conv1 epilogue, tile conv3 wgrad,
# module-major LDS-tiled fc forward), path-major fc forward, the swapped epilogue alone off, tile wgrad alone off,
# everything off; default repeated last.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_mm2.log 2>&1
tail -1 gpurun_out/r3/x3_tests_mm2.log; grep -E "fp32x|wgrad tile|FAIL|Error" gpurun_out/r3/x3_tests_mm2.log | head -12
grep -q " passed" gpurun_out/r3/x3_tests_mm2.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_mm2.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "fc_fwd\|fc_slot\|conv_dgrad_x3<x3::CG<39\|conv1_fwd\|CG<18, 13, 8, 3, 3, 1, false> >" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v11
PATHNET_X3_FC_MM=0 prof x3_v11_pm
PATHNET_X3_FC_MM=0 prof x3_v11_pm_nosw --kernel-opt fast_conv_set_x3_fwd_sw=0
PATHNET_X3_FC_MM=0 prof x3_v11_pm_notile --kernel-opt fast_conv_set_x3_wg3_tile=0
PATHNET_X3_FC_MM=0 prof x3_v11_off --kernel-opt fast_conv_set_x3_fwd_sw=0 --kernel-opt fast_conv_set_x3_wg3_tile=0
prof x3_v11_rep
