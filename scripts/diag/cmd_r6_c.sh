set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag/rects_bench.py > $OUT/rects_bench.log 2>&1 || { echo "rects bench failed"; tail -20 $OUT/rects_bench.log; exit 1; }
tail -1 $OUT/rects_bench.log
timeout -k 10 300 python -u scripts/diag/ab_kernel.py --kernel layer_bwd --layer 3 --part w --opt x3_fcw_kt=128 --opt x3_fcw_kt=256 > $OUT/ab_fcw_kt.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_fcw_kt.log; exit 1; }
tail -3 $OUT/ab_fcw_kt.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "deterministic or rasteriser or fc_wgrad or x3_engine_gradient or frame_ring_gradient or shipped_graph" > $OUT/pytest_c.log 2>&1; echo "tests rc=$?"
grep -E "PASS|FAIL|Error" $OUT/pytest_c.log | head -30
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --windows 6 --no-stagger --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build > $OUT/drift6_nostag.log 2>&1 || { echo "drift bench failed"; tail -20 $OUT/drift6_nostag.log; exit 1; }
grep '^{' $OUT/drift6_nostag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nostagger', d['windows_ms_per_step'], d['generations_in_timed_windows'])"
OUT=$OUT bash scripts/gpu.sh "kwin ref --preset reference --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin p64w0 --windows 6 --prof-window-index 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin p64w5 --windows 6 --prof-window-index 5 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
