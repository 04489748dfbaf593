set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "deterministic or heldout" > $OUT/pytest_det.log 2>&1; echo "det tests rc=$?"
grep -E "PASS|FAIL|Error|per layer" $OUT/pytest_det.log | head -30
for arm in nodet det nodet det; do
  extra=""; [ $arm = det ] && extra="--deterministic"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build $extra > $OUT/ab_$arm.log 2>&1 || { echo "bench $arm failed"; tail -20 $OUT/ab_$arm.log; exit 1; }
  grep '^{' $OUT/ab_$arm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['ms_per_step'], d['windows_ms_per_step'], d['config']['deterministic'])"
done
