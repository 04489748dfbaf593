#!/bin/bash
# module-major fc forward with the k range split over two workgroups (fc_fwd_mm2_x3 KS=2 + fc_slot_sum2_x3): x3 tests,
# then windows for the default (fc1 module-major KS=2), KS=1, and fc2 module-major too.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_mm3.log 2>&1
tail -1 gpurun_out/r3/x3_tests_mm3.log; grep -E "FAIL|Error" gpurun_out/r3/x3_tests_mm3.log | head -12
grep -q " passed" gpurun_out/r3/x3_tests_mm3.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_mm3.log && exit 1
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "fc_fwd\|fc_slot\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v13
prof x3_v13_ks1 --kernel-opt fast_conv_set_x3_fc_mmv=2
PATHNET_X3_FC_MM_MIN_K=0 prof x3_v13_mmall
prof x3_v13_dgold --kernel-opt fast_conv_set_x3_fc_dg_gemm=0
prof x3_v13_rep
PROF_BY_GRID=1 DT=fp32x TAG=x3_v13_grid bash scripts/gpu_r3_prof.sh > /dev/null && grep "dgrad\|wgrad" gpurun_out/r3/kwin_x3_v13_grid.md | cut -c1-120
