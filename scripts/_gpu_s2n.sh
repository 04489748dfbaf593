#!/bin/bash
# launch-shape A/B: fc1 weight-gradient workgroup count (768 vs 512 target), conv1 forward tiles per wave (9 vs 8);
# Pong env kernel with two old-stack loads in flight (env tests first).
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_hip_kernels.py \
    -k "pong_env or frame_ring" > gpurun_out/r3/env_tests_v15.log 2>&1 || { tail -20 gpurun_out/r3/env_tests_v15.log; exit 1; }
tail -1 gpurun_out/r3/env_tests_v15.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd\|fc_wgrad_gm\|conv_dgrad_x3<x3::CG<39\|pong_step" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v15
PATHNET_X3_FC_WGRAD_WGS=512 prof x3_v15_wgs512
prof x3_v15_nt9 --kernel-opt fast_conv_set_x3_fwd_nt=9
prof x3_v15_rep
