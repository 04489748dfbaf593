#!/bin/bash
# Supervised MNIST -> SVHN (synthetic digit sets, 4096 / 256 training images), conv trunk, frozen_mode available,
# paired from-scratch control; one run per seed argument.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/supervised3
for seed in "$@"; do
  tag=conv64_avail_paired_s$seed
  timeout -k 10 400 python -u -m pathnet_gym_amd.cli supervised --tasks mnist,svhn --arch conv --width 64 \
      --frozen_mode available --control --paired_control 1 --train_sizes 4096,256 --seed $seed \
      > gpurun_out/supervised3/$tag.json 2> gpurun_out/supervised3/$tag.err \
      || { echo "RUN FAIL $tag"; tail -5 gpurun_out/supervised3/$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t=d['per_task']; c=d.get('control',{})
print(sys.argv[2], 'task2 test', round(t[-1]['test_accuracy'],3), '| paired scratch test', round(c.get('test_accuracy',0),3), round(d['seconds']),'s')
" gpurun_out/supervised3/$tag.json $tag
done
