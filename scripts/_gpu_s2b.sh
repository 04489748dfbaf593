#!/bin/bash
# conv forward swapped epilogue (conv_epi_sw) + per-sample tile conv3 weight gradient: x3 tests, then steady-state
# kernel windows for the defaults (SW = 1, tile wgrad), SW = 3 (all conv layers) and the old kernels (SW = 0, rows).
set -o pipefail
mkdir -p gpurun_out/r3
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_x3_engine.py > gpurun_out/r3/x3_tests_sw.log 2>&1
tail -1 gpurun_out/r3/x3_tests_sw.log; grep -E "^layer|fp32x|wgrad tile" gpurun_out/r3/x3_tests_sw.log | head -14
grep -q " passed" gpurun_out/r3/x3_tests_sw.log || exit 1
grep -q "failed" gpurun_out/r3/x3_tests_sw.log && exit 1
DT=fp32x TAG=x3_v10 bash scripts/gpu_r3_prof.sh > /dev/null && \
DT=fp32x TAG=x3_v10_sw3 EXTRA="--kernel-opt fast_conv_set_x3_fwd_sw=3" bash scripts/gpu_r3_prof.sh > /dev/null && \
DT=fp32x TAG=x3_v10_base EXTRA="--kernel-opt fast_conv_set_x3_fwd_sw=0 --kernel-opt fast_conv_set_x3_wg3_tile=0" bash scripts/gpu_r3_prof.sh > /dev/null || exit 1
for t in x3_v10 x3_v10_sw3 x3_v10_base; do echo "== $t"; sed -n 3p gpurun_out/r3/kwin_$t.md | cut -c100-; grep "conv1_fwd\|conv_fwd_x3\|CG<18, 13, 8, 3, 3, 1, false> >" gpurun_out/r3/kwin_$t.md; done
