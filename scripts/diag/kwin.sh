# kernel-trace window of the 1-GPU bench: kwin.sh LABEL PATHS [bench args...] -> gpurun_out/kwin_LABEL.md
set -o pipefail
L=$1; P=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/kw_$L
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kw_$L -o k -- python3 $R/bench.py --paths $P --paths-total $P --steps 10 --warmup 5 --windows 1 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build --prof-window "$@" > $R/gpurun_out/kw_$L.log 2>&1 || exit 1
f=$(find /tmp/kw_$L -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/prof_window.py $f 10 "bench --paths $P $*, steady-state window ($L)" > $R/gpurun_out/kwin_$L.md
