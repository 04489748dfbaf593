#!/bin/bash
# conv_module PathNet MNIST -> SVHN small-data transfer: seeds 2 and 3 (seed 1 in gpu_supervised2.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/supervised2
for seed in 2 3; do
  tag=conv64_s$seed
  timeout -k 10 400 python -u -m pathnet_gym_amd.cli supervised --arch conv --width 64 --seed $seed --control \
      --train_sizes 4096,256 > gpurun_out/supervised2/$tag.json 2> gpurun_out/supervised2/$tag.err \
    || { echo "RUN FAIL $tag"; tail -5 gpurun_out/supervised2/$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t=d['per_task']; c=d.get('control',{})
print(sys.argv[2], 'task2 test', round(t[-1]['test_accuracy'],3), '| scratch test', round(c.get('test_accuracy',0),3), '| gens-to-0.9 (train)', d['generations_to_accuracy']['transfer'], d['generations_to_accuracy']['from_scratch'], round(d['seconds']),'s')
" gpurun_out/supervised2/$tag.json $tag
done
