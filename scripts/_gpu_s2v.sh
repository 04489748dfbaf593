#!/bin/bash
# conv1 slab weight gradient with fewer VALU ops (byte -> bf16 as one v_cvt_f32_ubyte + one v_perm per pair, ReLU
# masks as v_bfe_i32 + v_and, packed-fp32 bias sums and split subtraction): tests, then ring windows x2.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 500 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py tests/test_hip_kernels.py \
    -k "x3_engine_gradient or two_percent or frame_ring or dgrad or wgrad_tile" -s \
    > gpurun_out/r3/x3_tests_v22.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v22.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v22.log
grep "oracle, per layer" gpurun_out/r3/x3_tests_v22.log | cut -c1-250
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd_band\|CG<160, 120, 4, 8, 8, 4, true>, 2\|CG<39, 29, 8, 4, 4, 2, false>, 7\|conv_dgrad\|conv_wgrad_tile" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v22
prof x3_v22_rep
