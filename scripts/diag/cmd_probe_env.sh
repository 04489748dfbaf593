# per-phase stamps of the frame-ring Pong step at 256 envs (8 paths) and 2048 envs (64 paths)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc -w scripts/probe_env.hip -o /tmp/probe_env || exit 1
for b in 256 2048; do
  timeout -k 10 60 /tmp/probe_env $b >> gpurun_out/probe_env.txt 2>&1 || exit 1
done
