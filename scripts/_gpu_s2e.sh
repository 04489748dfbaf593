#!/bin/bash
# Supervised MNIST -> SVHN transfer, conv trunk, frozen modules available, paired from-scratch control, seeds 1-3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/_gpu_sup.sh 1 2 3
