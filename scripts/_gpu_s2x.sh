#!/bin/bash
# conv2/3 forward tiles two per weight read (X3_FWD_TILE=2) + the int64 ring tail copy: test, interleaved windows.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "conv_forward" -s \
    > gpurun_out/r3/x3_tests_v24.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v24.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v24.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv_fwd_tile\|copy\|elementwise" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v24
prof x3_v24_pair --kernel-opt fast_conv_set_x3_fwd_tile=2
prof x3_v24_rep
prof x3_v24_pair_rep --kernel-opt fast_conv_set_x3_fwd_tile=2
