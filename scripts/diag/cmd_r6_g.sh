set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build > $OUT/g_drift.log 2>&1 || { echo "bench failed"; tail -20 $OUT/g_drift.log; exit 1; }
grep '^{' $OUT/g_drift.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('drift6', d['ms_per_step'], d['windows_ms_per_step']); [print(t['ms'], t.get('host_ms_per_update')) for t in d['windows_telemetry']]"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "pipeline or device_lr or x3_shipped or deterministic_200 or split_rollout or smoke" > $OUT/pytest_g.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|^E " $OUT/pytest_g.log | tail -15
