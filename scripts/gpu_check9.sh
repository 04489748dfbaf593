#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|assert" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --preset atari4 --steps 5 --warmup 2 > gpurun_out/bench_atari4.log 2>&1 || { tail -20 gpurun_out/bench_atari4.log; exit 4; }
echo "atari4(Pong task): $(tail -1 gpurun_out/bench_atari4.log | cut -c1-200)"
timeout -k 10 400 python bench.py --preset reference --paths 64 --envs 32 --steps 10 --warmup 3 > gpurun_out/bench_ref.log 2>&1 || { tail -20 gpurun_out/bench_ref.log; exit 5; }
echo "reference LSTM: $(tail -1 gpurun_out/bench_ref.log | cut -c1-200)"
timeout -k 10 600 python - > gpurun_out/breakout_speed.log 2>&1 <<'PY'
import time, torch
from pathnet_gym_amd import _build; _build.build()
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.algo.trainer import PathNetTrainer
cfg = preset("atari4"); cfg.tasks = ["Breakout"]; cfg.ga.backend = "device"
tr = PathNetTrainer(cfg, device="cuda")
for _ in range(2): tr.update()
tr.flush(); torch.cuda.synchronize(); t0 = time.time()
for _ in range(5): tr.update()
tr.flush(); torch.cuda.synchronize(); dt = time.time() - t0
print("breakout frames/s", 5 * cfg.a2c.t_max * cfg.paths * cfg.envs_per_path / dt, "ms/update", dt / 5 * 1e3)
PY
tail -2 gpurun_out/breakout_speed.log
exit $rc
