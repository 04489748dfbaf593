#!/bin/bash
# Typed-module trunk (K19) tests, then MNIST -> SVHN transfer runs (fc and conv_module PathNets) with controls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/supervised
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py \
    -k "typed or supervised" > gpurun_out/supervised/test.log 2>&1 || { echo "TEST FAIL"; tail -30 gpurun_out/supervised/test.log; exit 1; }
tail -1 gpurun_out/supervised/test.log
for spec in "fc64:--arch fc --width 64" "fc160:--arch fc --width 160" "conv64:--arch conv --width 64"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 ${SUP_TIMEOUT:-280} python -u -m pathnet_gym_amd.cli supervised $args --control ${SUP_ARGS:-} \
      > gpurun_out/supervised/$tag.json 2> >(tee gpurun_out/supervised/$tag.err | grep -E "generation (0|9|19|29|39|49) " >&2) || { echo "RUN FAIL $tag"; tail -5 gpurun_out/supervised/$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t=d['per_task']; c=d.get('control',{})
print(sys.argv[2], 'task1 test', round(t[0]['test_accuracy'],3), 'task2 train', round(t[-1]['best_accuracy'],3), 'test', round(t[-1]['test_accuracy'],3),
      '| control train', round(c.get('best_accuracy',0),3), 'test', round(c.get('test_accuracy',0),3), '| gens-to-acc', d.get('generations_to_accuracy'), round(d['seconds']),'s')
" gpurun_out/supervised/$tag.json $tag
done
