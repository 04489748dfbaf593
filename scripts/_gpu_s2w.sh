#!/bin/bash
# conv1 band forward with the next k-step's LDS fragments in flight (X3_C1_PIPE): bit-equality test, then
# interleaved windows base / pipe / base / pipe.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_x3_engine.py -k "conv_forward" -s \
    > gpurun_out/r3/x3_tests_v23.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v23.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v23.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "conv1_fwd_band\|CG<160, 120, 4, 8, 8, 4, true>, 2" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v23
prof x3_v23_pipe --kernel-opt fast_conv_set_x3_c1_pipe=1
prof x3_v23_rep
prof x3_v23_pipe_rep --kernel-opt fast_conv_set_x3_c1_pipe=1
