#!/bin/bash
# MNIST -> SVHN small-data transfer with frozen modules AVAILABLE to task-2 paths (not forced): conv and fc, 3 seeds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/supervised2
run() {
  tag=$1; shift
  timeout -k 10 330 python -u -m pathnet_gym_amd.cli supervised "$@" --control --train_sizes 4096,256 --frozen_mode available \
      > gpurun_out/supervised2/$tag.json 2> gpurun_out/supervised2/$tag.err || { echo "RUN FAIL $tag"; tail -5 gpurun_out/supervised2/$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t=d['per_task']; c=d.get('control',{})
print(sys.argv[2], 'task2 test', round(t[-1]['test_accuracy'],3), '| scratch test', round(c.get('test_accuracy',0),3), '| gens-to-0.9 (train)', d['generations_to_accuracy']['transfer'], d['generations_to_accuracy']['from_scratch'], round(d['seconds']),'s', flush=True)
" gpurun_out/supervised2/$tag.json $tag
}
for seed in 1 2 3; do
  run conv64_avail_s$seed --arch conv --width 64 --seed $seed || exit 1
done
for seed in 1 2 3; do
  run fc64_avail_s$seed --arch fc --width 64 --seed $seed || exit 1
done
