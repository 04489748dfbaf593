# kernel traces of the 8-path update, one and two rollout groups
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for g in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kp8g$g -o k -- python3 $R/bench.py --paths 8 --paths-total 8 --steps 10 --warmup 5 --windows 1 --no-strong --per-rank-shapes "" --solve-seconds 0 --no-verify-build --prof-window --rollout-groups $g > $R/gpurun_out/kp8g$g.log 2>&1 || exit 1
  f=$(find /tmp/kp8g$g -name "*kernel_trace.csv" | head -1)
  python3 $R/scripts/prof_window.py $f 10 "bench --paths 8, rollout groups $g" > $R/gpurun_out/kwin_p8_groups$g.md || exit 1
  cp $f $R/gpurun_out/kp8g${g}_trace.csv
done
