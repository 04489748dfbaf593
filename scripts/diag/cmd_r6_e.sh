set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "x3 or ring or split_rollout or games or checkpoint or deterministic" > $OUT/pytest_e.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAIL|Error|passed|failed" $OUT/pytest_e.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
OUT=$OUT bash scripts/gpu.sh "smoke"
KSTEPS=20 OUT=$OUT bash scripts/gpu.sh "kwin d0 --windows 6 --prof-window-index 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build" "kwin d5 --windows 6 --prof-window-index 5 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
