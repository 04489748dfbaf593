#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py -q -k "image_staged or slab or dgrad_mfma" > gpurun_out/pytest_ab.log 2>&1
rc=$?; grep -E "passed|failed|assert" gpurun_out/pytest_ab.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for opts in "" "--kernel-opt img_fwd=0" "--kernel-opt wgrad_ob=3"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $opts > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 4; }
  echo "[$opts] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
