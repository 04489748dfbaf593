#!/bin/bash
# env kernel: size scaling + one PMC pass (SQ counters only, own run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/env_microbench.py --envs 256 --iters 100 || exit 1
timeout -k 10 120 python -u scripts/env_microbench.py --envs 8192 --iters 50 || exit 1
rm -rf /tmp/epmc
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
   -d /tmp/epmc -o pmc --output-format csv -- python3 "$ROOT/scripts/env_microbench.py" --iters 20 > "$ROOT/gpurun_out/env_pmc.log" 2>&1) || { echo PMC FAIL; tail -5 gpurun_out/env_pmc.log; exit 1; }
f=$(find /tmp/epmc -name "*counter_collection.csv" | head -1)
cp "$f" gpurun_out/env_pmc.csv
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/env_pmc.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "pong" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    c = {m: v / n[(k, m)] for m, v in d.items()}
    print(k[:40], {m: round(v) for m, v in sorted(c.items())})
PY
