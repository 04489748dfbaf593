set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_h.log 2>&1; rc=$?; echo "tests rc=$rc"
grep -E "FAILED|passed|failed|^E " $OUT/pytest_h.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
OUT=$OUT bash scripts/gpu.sh "smoke"
