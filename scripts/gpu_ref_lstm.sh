#!/bin/bash
# The reference's own network (L=4 + BasicLSTMCell(256), T=20, 18-way head) on its own experiment: synthetic
# Alien -> Centipede continual (task 1 -> freeze -> re-init -> task 2) + a from-scratch Centipede control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/continual
for seed in ${SEEDS:-1 2}; do
  timeout -k 10 ${CAP:-560} python -u scripts/continual.py --preset reference --tasks Alien,Centipede \
      --frames ${FRAMES:-300000000} --control --seed $seed --report-every 20 \
      --out gpurun_out/continual/ref_lstm_alien_centipede_s$seed.json > gpurun_out/continual/ref_lstm_s$seed.log 2>&1 \
      || { echo "RUN FAIL seed $seed"; tail -20 gpurun_out/continual/ref_lstm_s$seed.log; exit 1; }
  tail -4 gpurun_out/continual/ref_lstm_s$seed.log | cut -c1-400
done
