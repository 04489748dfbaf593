# end-of-round validation, part 2: forced one-rank RCCL vs no group (medians of 5 windows, interleaved), the task-2
# exchange on the forced group, kernel windows at 64 / 8 paths, the preset kernel A/B, PMC of the 64-path update
set -o pipefail
OUT=gpurun_out/r6_final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread -k "typed_fc" > $OUT/pytest_typed.log 2>&1; echo "typed tests rc=$?"
grep -E "FAILED|passed|failed" $OUT/pytest_typed.log | tail -4
for arm in nogroup forced nogroup forced; do
  for p in 8 64; do
    if [ $arm = forced ]; then export PATHNET_DIST_FORCE=1; else unset PATHNET_DIST_FORCE; fi
    timeout -k 10 300 python -u bench.py --paths $p --paths-total $p --steps 20 --warmup 5 --windows 5 --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build --no-strong > $OUT/rccl_${arm}_p$p.log 2>&1 || { echo "rccl bench $arm $p failed"; tail -20 $OUT/rccl_${arm}_p$p.log; exit 1; }
    grep '^{' $OUT/rccl_${arm}_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm p$p', d['ms_per_step'], d['windows_ms_per_step'])"
  done
done
unset PATHNET_DIST_FORCE
PATHNET_DIST_FORCE=1 timeout -k 10 300 python -u scripts/diag/task2_exchange.py --paths 8 > $OUT/task2_exchange_p8.log 2>&1 || { echo "task2 failed"; tail -20 $OUT/task2_exchange_p8.log; exit 1; }
tail -1 $OUT/task2_exchange_p8.log
KSTEPS=20 OUT=$OUT bash scripts/gpu.sh "kwin p64_final --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin p8_final --paths 8 --paths-total 8 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
timeout -k 10 400 python -u scripts/diag/preset_kernel_ab.py > $OUT/preset_kernel_ab.log 2>&1 || { echo "preset ab failed"; tail -20 $OUT/preset_kernel_ab.log; exit 1; }
tail -30 $OUT/preset_kernel_ab.log | head -40
OUT=$OUT bash scripts/gpu.sh "pmc p64 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
