#!/bin/bash
# Session check after a container rebuild: full GPU suite, smoke, a short bench (no in-run solve) and a short
# reference-preset (L=4 + LSTM 256) continual run to confirm the shape runs before the long runs.
set -o pipefail
mkdir -p gpurun_out/s2
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s2/pytest_gpu.log 2>&1 \
    || { tail -30 gpurun_out/s2/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s2/pytest_gpu.log
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || { tail -20 gpurun_out/s2/smoke.log; exit 1; }
tail -1 gpurun_out/s2/smoke.log | cut -c1-200
$T 300 python -u bench.py --steps 20 --warmup 5 --solve-seconds 0 > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err \
    || { tail -20 gpurun_out/s2/bench.err; exit 1; }
cat gpurun_out/s2/bench.json
$T 240 python -u scripts/continual.py --preset reference --tasks Alien,Centipede --frames 3000000 --control --seed 1 \
    --report-every 10 --out gpurun_out/s2/ref_lstm_short.json > gpurun_out/s2/ref_lstm_short.log 2>&1 \
    || { tail -20 gpurun_out/s2/ref_lstm_short.log; exit 1; }
tail -5 gpurun_out/s2/ref_lstm_short.log | cut -c1-300
