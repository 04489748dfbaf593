set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_x3_engine.py tests/test_split_rollout.py tests/test_games_hip.py -k "pong or ring or folded or digits" -x -q --timeout 300 --timeout-method thread > gpurun_out/envq_tests.log 2>&1 || { tail -30 gpurun_out/envq_tests.log; exit 1; }
tail -2 gpurun_out/envq_tests.log
: > gpurun_out/probe_env.txt
bash scripts/diag/cmd_probe_env.sh || exit 1
bash scripts/diag/kwin.sh p8_envq 8 || exit 1
bash scripts/diag/kwin.sh p64_envq 64 || exit 1
