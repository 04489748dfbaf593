#!/bin/bash
# fc1 forward k split in 4 vs 2, heads forward 16 vs 64 samples per workgroup: fc/heads tests, windows; then the
# 4-task from-scratch controls, seed 2.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py tests/test_hip_kernels.py \
    -k "fc_forward or heads" > gpurun_out/r3/x3_tests_v18.log 2>&1 || { tail -20 gpurun_out/r3/x3_tests_v18.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v18.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "fc_fwd_mm2\|fc_slot\|heads_fwd" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v18
prof x3_v18_ks4 --kernel-opt fast_conv_set_x3_fc_mmv=4
prof x3_v18_h64 --kernel-opt heads_set_s16=0
prof x3_v18_rep
SEED=2 bash scripts/_gpu_s2j.sh
