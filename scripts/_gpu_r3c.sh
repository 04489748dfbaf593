set -o pipefail
mkdir -p gpurun_out/r3 gpurun_out/solve
T="timeout -k 10"
PYT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
SEL="oracle or forward or backward or lstm or conv_gradients"
$T 400 $PYT tests/test_hip_kernels.py tests/test_f32_engine.py -k "$SEL" > gpurun_out/r3/numerics_check.log 2>&1
$T 400 $PYT tests/test_dist_hip.py tests/test_games_hip.py -k "resume or games or invaders or Invaders" > gpurun_out/r3/dist_resume.log 2>&1
tail -1 gpurun_out/r3/numerics_check.log; tail -1 gpurun_out/r3/dist_resume.log
NOTEST=1 DT=fp32x SEEDS="${SEEDS:-1}" SECS=${SECS:-840} bash scripts/gpu_solve_seeds.sh
