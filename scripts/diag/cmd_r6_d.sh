set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
for arm in gc det gc det; do
  extra=""; [ $arm = det ] && extra="--deterministic"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build $extra > $OUT/d_$arm.log 2>&1 || { echo "bench $arm failed"; tail -20 $OUT/d_$arm.log; exit 1; }
  grep '^{' $OUT/d_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['ms_per_step'], d['windows_ms_per_step'], d['config']['deterministic'], [t.get('sclk_mhz') for t in d['windows_telemetry']])"
done
