#!/bin/bash
# conv_module MNIST -> SVHN small-data transfer, frozen modules available: seeds 4-7
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/supervised2
for seed in 4 5 6 7; do
  tag=conv64_avail_s$seed
  timeout -k 10 330 python -u -m pathnet_gym_amd.cli supervised --arch conv --width 64 --seed $seed --control \
      --train_sizes 4096,256 --frozen_mode available > gpurun_out/supervised2/$tag.json 2> gpurun_out/supervised2/$tag.err \
    || { echo "RUN FAIL $tag"; tail -5 gpurun_out/supervised2/$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t=d['per_task']; c=d.get('control',{})
print(sys.argv[2], 'task2 test', round(t[-1]['test_accuracy'],3), '| scratch test', round(c.get('test_accuracy',0),3), flush=True)
" gpurun_out/supervised2/$tag.json $tag
done
