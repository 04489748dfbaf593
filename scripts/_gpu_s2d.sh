#!/bin/bash
# Long evidence runs, part 2: reference network on Alien -> Centipede seed 2; supervised MNIST -> SVHN transfer with
# the paired from-scratch control (common random numbers), conv trunk, frozen modules available, seeds 1 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
SEEDS=2 FRAMES=300e6,200e6 CAP=520 bash scripts/gpu_ref_lstm.sh || exit 1
bash scripts/_gpu_sup.sh 1 2
