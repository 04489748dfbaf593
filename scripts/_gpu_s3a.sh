#!/bin/bash
# heads backward in 32-row chunks (atomic mode, heads_set_bwd_rows=32) vs the default 128: heads tests, windows.
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_hip_kernels.py tests/test_x3_engine.py \
    -k "heads or x3_engine_gradient" > gpurun_out/r3/x3_tests_v26.log 2>&1 || { tail -30 gpurun_out/r3/x3_tests_v26.log; exit 1; }
tail -1 gpurun_out/r3/x3_tests_v26.log
prof() {
  tag=$1; shift
  DT=fp32x TAG=$tag EXTRA="$*" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
  echo "== $tag $(sed -n 3p gpurun_out/r3/kwin_$tag.md | grep -o 'wall between.*')"
  grep "heads_bwd" gpurun_out/r3/kwin_$tag.md | cut -c1-110
}
prof x3_v26 --kernel-opt heads_set_bwd_rows=32
prof x3_v26_r128
