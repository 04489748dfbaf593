#!/bin/bash
# fp32x first layer on the frame ring: ring tests (x3 + bf16), then steady-state windows packed vs ring (x2 each).
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py tests/test_hip_kernels.py \
    -k "ring or x3_engine_gradient or two_percent" -s > gpurun_out/r3/x3_tests_v20.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v20.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v20.log
grep "oracle, per layer" gpurun_out/r3/x3_tests_v20.log | cut -c1-250
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd_band\|CG<160, 120, 4, 8, 8, 4, true>, 2\|pong_step\|conv_fwd_tile_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v20_ring --ring
prof x3_v20
prof x3_v20_ring_rep --ring
