#!/bin/bash
# launch-shape A/B: fc1 weight-gradient workgroup count (768 vs 512 target), conv1 forward tiles per wave (9 vs 8).
set -o pipefail
mkdir -p gpurun_out/r3
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd\|fc_wgrad_gm\|conv_dgrad_x3<x3::CG<39" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v15
PATHNET_X3_FC_WGRAD_WGS=512 prof x3_v15_wgs512
prof x3_v15_nt9 --kernel-opt fast_conv_set_x3_fwd_nt=9
prof x3_v15_rep
