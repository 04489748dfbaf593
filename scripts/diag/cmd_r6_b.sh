set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 200 python -u scripts/diag/fx_leftover.py > $OUT/fx_leftover.log 2>&1; echo "fx rc=$?"; tail -30 $OUT/fx_leftover.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build > $OUT/drift6.log 2>&1 || { echo "drift bench failed"; tail -20 $OUT/drift6.log; exit 1; }
grep '^{' $OUT/drift6.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['windows_ms_per_step'], d['generations_in_timed_windows']); [print(t) for t in d['windows_telemetry']]"
OUT=$OUT bash scripts/gpu.sh "kwin ref --preset reference --per-rank-shapes '' --reference-preset 0 --no-verify-build"
