#!/bin/bash
# The reference's own network (L=4 + LSTM 256, 18-way head, 64 x 16, T=20) on synthetic Alien -> Centipede with a
# from-scratch Centipede control, seeds 1 and 2 (after-task evaluations on the task-end parameters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
SEEDS="1 2" FRAMES=200e6,200e6 CAP=575 bash scripts/gpu_ref_lstm.sh
