#!/bin/bash
# default conv2 paired forward tiles (X3_FWD_TILE=3) vs single tiles (1): tests, interleaved windows.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "conv_forward or x3_engine_gradient or frame_ring" -s \
    > gpurun_out/r3/x3_tests_v25.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v25.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v25.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv_fwd_tile\|band\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v25
prof x3_v25_single --kernel-opt fast_conv_set_x3_fwd_tile=1
prof x3_v25_rep
prof x3_v25_single_rep --kernel-opt fast_conv_set_x3_fwd_tile=1
