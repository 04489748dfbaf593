#!/bin/bash
# The one GPU-box runner (replaces the per-experiment scripts of rounds 1-3).  Every argument is one STEP: its
# first word names the step, the rest are that step's arguments.  Steps run in order; each has its own time limit;
# the chain stops at the first failure (no GPU work after a fault, an abort or a time limit).
#
#   scripts/gpu.sh "tests" "smoke" "bench --steps 20"
#   scripts/gpu.sh "tests x3_lstm,two_tile"                  pytest -m gpu [-k "x3_lstm or two_tile"]
#   scripts/gpu.sh "smoke"                                   __graft_entry__.smoke()
#   scripts/gpu.sh "bench <bench.py args>"                   -> gpurun_out/r4/bench_<n>.json
#   scripts/gpu.sh "kwin TAG <bench.py args>"                rocprofv3 kernel trace, steady-state window summary
#                                                            (scripts/prof_window.py) -> gpurun_out/r4/kwin_TAG.md
#   scripts/gpu.sh "pmc TAG <bench.py args>"                 PMC passes (VALU / MFMA / LDS / waits, L2, MFMA busy,
#                                                            HBM bytes), graph off -> gpurun_out/r4/pmc_TAG_*.md
#   scripts/gpu.sh "solve NAME SECONDS <solve.py args>"      scripts/solve.py -> gpurun_out/r4/solve/NAME.json(l)
#   scripts/gpu.sh "continual NAME SECONDS <continual.py args>"
#   scripts/gpu.sh "supervised NAME SECONDS <cli supervised args>"
#   scripts/gpu.sh "py SECONDS <python args>"                any python entry point (e.g. a diag script)
#   scripts/gpu.sh "seeds A B MINUTES"                       two generations-to-solve seeds of the bench config at
#                                                            once (deterministic fp32x, v2 criterion; "1r" = a repeat
#                                                            of seed 1 under its own name) -> OUT/solve/v2_seed*.json
#   scripts/gpu.sh "rccl P [WINDOWS]"                        forced one-rank RCCL vs no group at P paths, interleaved
#                                                            (nogroup forced nogroup forced), median windows
#   scripts/gpu.sh "windows N <bench.py args>"               N back-to-back windows with per-window telemetry
#   scripts/gpu.sh "driver"                                  the driver's one-GPU bench command (bench.py --gpus 1)
#
# Env: OUT (default gpurun_out/r4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
OUT=${OUT:-gpurun_out/r4}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="timeout -k 10"
nb=0

fail() { echo "STEP FAIL ($1) rc=$2"; [ -n "$3" ] && tail -25 "$3"; exit 1; }

step_tests() {
  local k=()
  [ -n "$1" ] && k=(-k "${1//,/ or }")
  local rc=0
  $T 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread "${k[@]}" \
      > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
  # a failed assertion (rc 1) is a result, not a fault: report it and go on with the next steps; a time limit, an
  # abort or a crash (rc 124 / 137 / 134 / 139 / >128) ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then fail tests $rc "$OUT/pytest_gpu.log"; fi
  [ $rc -ne 0 ] && grep -E "^E |^FAILED|per layer" "$OUT/pytest_gpu.log" | head -12
  tail -2 "$OUT/pytest_gpu.log"
}

step_smoke() {
  $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke $? "$OUT/smoke.log"
  tail -1 "$OUT/smoke.log" | cut -c1-300
}

step_bench() {
  nb=$((nb + 1))
  $T 700 python -u bench.py "$@" > "$OUT/bench_$nb.log" 2>&1 || fail bench $? "$OUT/bench_$nb.log"
  grep '^{' "$OUT/bench_$nb.log" > "$OUT/bench_$nb.json"
  python3 - "$OUT/bench_$nb.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("strong_scaling") or {}
print("bench", d["dtype"], d["value"], "frames/s", d["ms_per_step"], "ms", d.get("windows_ms_per_step"),
      "| bf16", d.get("value_bf16"), d.get("ms_per_step_bf16"), "| strong", s.get("ms_per_update"),
      s.get("predicted_seconds_to_solve"), "| solve", (d.get("generations_to_solve_in_run") or {}).get("solved"))
EOF
}

step_kwin() {
  local tag=$1; shift
  rm -rf /tmp/kprof_$tag
  (cd /tmp && $T 300 rocprofv3 --kernel-trace -d /tmp/kprof_$tag -o k --output-format csv \
      -- python3 "$ROOT/bench.py" --steps ${KSTEPS:-10} --warmup 3 --windows 1 --prof-window --solve-seconds 0 \
      --compare-bf16 0 "$@" > "$ROOT/$OUT/prof_$tag.log" 2>&1) || fail "kwin $tag" $? "$OUT/prof_$tag.log"
  local f
  f=$(find /tmp/kprof_$tag -name "*kernel_trace.csv" | head -1)
  python3 scripts/prof_window.py "$f" ${KSTEPS:-10} "bench $*, steady-state window ($tag)" > "$OUT/kwin_$tag.md"
  sed -n 3p "$OUT/kwin_$tag.md"
  sed -n 5,14p "$OUT/kwin_$tag.md" | cut -c1-120
}

pmc_pass() {
  local tag=$1 pass=$2; shift 2
  local counters=$1; shift
  rm -rf /tmp/pmc_${tag}_$pass
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $counters -d /tmp/pmc_${tag}_$pass -o pmc --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --windows 1 --no-graph --solve-seconds 0 --compare-bf16 0 "$@" \
     > "$ROOT/$OUT/pmc_${tag}_$pass.log" 2>&1) || fail "pmc $tag $pass" $? "$OUT/pmc_${tag}_$pass.log"
  cp "$(find /tmp/pmc_${tag}_$pass -name '*counter_collection.csv' | head -1)" "$OUT/pmc_${tag}_$pass.csv"
}

step_pmc() {
  local tag=$1; shift
  pmc_pass "$tag" a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "$@"
  pmc_pass "$tag" b "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum" "$@"
  pmc_pass "$tag" c "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES FETCH_SIZE" "$@"
  pmc_pass "$tag" d "WRITE_SIZE SQ_WAVES" "$@"
  python3 scripts/pmc_summary.py "$OUT/pmc_${tag}_a.csv" "$OUT/pmc_${tag}_b.csv" > "$OUT/pmc_${tag}_summary.md"
  python3 scripts/pmc_summary.py --mem "$OUT/pmc_${tag}_c.csv" "$OUT/pmc_${tag}_d.csv" > "$OUT/pmc_${tag}_mem.md"
  head -20 "$OUT/pmc_${tag}_summary.md" | cut -c1-140
}

step_solve() {
  local name=$1 secs=$2; shift 2
  mkdir -p "$OUT/solve"
  $T $((secs + 120)) python -u scripts/solve.py --minutes "$(python3 -c "print($secs/60)")" --report-every 30 \
      --curve "$OUT/solve/$name.jsonl" --out "$OUT/solve/$name.json" "$@" > "$OUT/solve/$name.log" 2>&1 \
      || fail "solve $name" $? "$OUT/solve/$name.log"
  tail -1 "$OUT/solve/$name.json" | cut -c1-420
}

step_continual() {
  local name=$1 secs=$2; shift 2
  mkdir -p "$OUT/continual"
  $T $((secs + 60)) python -u scripts/continual.py --out "$OUT/continual/$name.json" "$@" \
      > "$OUT/continual/$name.log" 2>&1 || fail "continual $name" $? "$OUT/continual/$name.log"
  grep -v '"run"' "$OUT/continual/$name.log" | tail -8 | cut -c1-300
}

step_supervised() {
  local name=$1 secs=$2; shift 2
  mkdir -p "$OUT/supervised"
  $T "$secs" python -u -m pathnet_gym_amd.cli supervised "$@" > "$OUT/supervised/$name.json" \
      2> "$OUT/supervised/$name.err" || fail "supervised $name" $? "$OUT/supervised/$name.err"
  tail -1 "$OUT/supervised/$name.json" | cut -c1-300
}

step_py() {
  local secs=$1; shift
  nb=$((nb + 1))
  $T "$secs" python -u "$@" > "$OUT/py_$nb.log" 2>&1 || fail "py $*" $? "$OUT/py_$nb.log"
  tail -5 "$OUT/py_$nb.log" | cut -c1-300
}

step_seeds() {
  local a=$1 b=$2 min=${3:-17.5}
  mkdir -p "$OUT/solve"
  local S="--preset pong --paths 64 --envs 32 --ring --dtype fp32x --ga-backend device --deterministic --report-every 30"
  local pids=() seed rc=0
  for seed in $a $b; do
    $T "$(python3 -c "print(int($min*60+90))")" python -u scripts/solve.py --minutes "$min" $S --seed "${seed%r}" \
        --curve "$OUT/solve/v2_seed$seed.jsonl" --out "$OUT/solve/v2_seed$seed.json" > "$OUT/solve/v2_seed$seed.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || rc=$?; done
  for seed in $a $b; do
    tail -1 "$OUT/solve/v2_seed$seed.json" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seed $seed', d['stopped'], d['generations_to_solve'], d['updates_to_solve'], d.get('heldout_mean'), d['wall_s'])" \
      || echo "seed $seed: no record"
  done
  [ $rc -eq 0 ] || fail "seeds $a $b" $rc "$OUT/solve/v2_seed$a.log"
}

step_rccl() {
  local p=$1 w=${2:-5} arm
  for arm in nogroup forced nogroup forced; do
    nb=$((nb + 1))
    if [ $arm = forced ]; then export PATHNET_DIST_FORCE=1; else unset PATHNET_DIST_FORCE; fi
    $T 300 python -u bench.py --paths "$p" --paths-total "$p" --steps 20 --warmup 5 --windows "$w" --solve-seconds 0 \
        --compare-bf16 0 --per-rank-shapes '' --reference-preset 0 --no-verify-build --no-strong \
        > "$OUT/rccl_${arm}_p${p}_$nb.log" 2>&1 || fail "rccl $arm $p" $? "$OUT/rccl_${arm}_p${p}_$nb.log"
    grep '^{' "$OUT/rccl_${arm}_p${p}_$nb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm p$p median', d['ms_per_step'], d['windows_ms_per_step'])"
  done
  unset PATHNET_DIST_FORCE
}

step_windows() {
  local n=$1; shift
  nb=$((nb + 1))
  $T 400 python -u bench.py --steps 20 --warmup 5 --windows "$n" --solve-seconds 0 --compare-bf16 0 --per-rank-shapes '' \
      --reference-preset 0 --no-verify-build "$@" > "$OUT/windows_$nb.log" 2>&1 || fail windows $? "$OUT/windows_$nb.log"
  grep '^{' "$OUT/windows_$nb.log" > "$OUT/windows_$nb.json"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print('windows', d['ms_per_step'], d['windows_ms_per_step']); [print(' ', t.get('ms'), t.get('sclk_mhz'), t.get('power'), t.get('active_modules_max_per_layer'), (t.get('host_ms_per_update') or {}).get('collect')) for t in d['windows_telemetry']]" "$OUT/windows_$nb.json"
}

step_driver() {
  $T 800 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || fail driver $? "$OUT/bench_driver.log"
  grep '^{' "$OUT/bench_driver.log" > "$OUT/bench_driver.json"
  python3 scripts/bench_digest.py "$OUT/bench_driver.json"
}

for s in "$@"; do
  read -r -a words <<< "$s"
  kind=${words[0]}
  echo "== $s"
  case $kind in
    tests|smoke|bench|kwin|pmc|solve|continual|supervised|py|seeds|rccl|windows|driver) "step_$kind" "${words[@]:1}" ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "== all steps ok"
