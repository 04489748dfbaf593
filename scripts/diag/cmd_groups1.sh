set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_split_rollout.py -k "x3_ring" > gpurun_out/t_groups.log 2>&1
echo "tests rc=$?" >> gpurun_out/t_groups.log
for g in 1 0; do
  for p in 8 16; do
    timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --steps 20 --warmup 5 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build --rollout-groups $g > gpurun_out/b_g${g}_p${p}.json 2> gpurun_out/b_g${g}_p${p}.err || exit 1
  done
done
