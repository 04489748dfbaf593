#!/bin/bash
# 2 ranks sharing the single GPU over gloo: exercises the distributed trainer + HIP engine +
# fused all-reduce + replicated GA exactly as the 8-GPU run does (RCCL swapped for gloo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
export PATHNET_DIST_BACKEND=gloo
if [ "$1" != "consistency" ]; then
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --paths 16 > gpurun_out/dist_bench.log 2>&1
rc=$?; echo "dist bench rc=$rc"; grep -E "metric|Error|error" gpurun_out/dist_bench.log | head -5
if [ $rc -ne 0 ]; then tail -30 gpurun_out/dist_bench.log; exit $rc; fi
fi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  scripts/dist_consistency.py > gpurun_out/dist_consistency.log 2>&1
rc=$?; echo "dist consistency rc=$rc"; tail -5 gpurun_out/dist_consistency.log
exit $rc
