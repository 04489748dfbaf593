set -o pipefail
OUT=gpurun_out/r6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/diag/preset_kernel_ab.py > $OUT/preset_kernel_ab.log 2>&1 || { echo "preset ab failed"; tail -20 $OUT/preset_kernel_ab.log; exit 1; }
python3 -c "
import json,sys
t=open('$OUT/preset_kernel_ab.log').read(); i=t.index('{'); d=json.loads(t[i:])
for k,v in d.items(): print(k, {a:b for a,b in v.items() if a!='stats'}); print('   ', v['stats'])
"
OUT=$OUT bash scripts/gpu.sh "pmc p64 --per-rank-shapes '' --reference-preset 0 --no-verify-build"
