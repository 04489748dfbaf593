set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_f.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|^E " $OUT/pytest_f.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build > $OUT/f_drift.log 2>&1 || { echo "bench failed"; tail -20 $OUT/f_drift.log; exit 1; }
grep '^{' $OUT/f_drift.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('drift6', d['ms_per_step'], d['windows_ms_per_step'], [t.get('sclk_mhz') for t in d['windows_telemetry']])"
