# window drift with the deterministic engine (one state sequence): six unprofiled windows, then kernel traces of
# window 0 and window 3 of the same sequence
set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --deterministic --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build > $OUT/drift_det6.log 2>&1 || { echo "bench failed"; tail -20 $OUT/drift_det6.log; exit 1; }
grep '^{' $OUT/drift_det6.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('det6', d['windows_ms_per_step']); [print(t['ms'], t['sclk_mhz'], t['power'], t['host_ms_per_update']['collect']) for t in d['windows_telemetry']]"
KSTEPS=20 OUT=$OUT bash scripts/gpu.sh "kwin det_w0 --windows 6 --warmup 5 --deterministic --prof-window-index 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin det_w3 --windows 6 --warmup 5 --deterministic --prof-window-index 3 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
