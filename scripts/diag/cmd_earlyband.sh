# conv1 band forward: first band loads before (1) / after (0) the weight staging, two libraries alternated
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_earlyband.json
for r in 1 2; do
  for v in 0 1; do
    cp alt_lib/lib_early$v.so pathnet_gym_amd/_hip/libpathnet_hip.so || exit 1
    for p in 8 64; do
      echo "{\"early\": $v, \"round\": $r}" >> gpurun_out/ab_earlyband.json
      timeout -k 10 200 python -u scripts/diag/ab_kernel.py --paths $p --kernel ring_fwd --reps 20 >> gpurun_out/ab_earlyband.json 2>> gpurun_out/ab_earlyband.err || exit 1
    done
  done
done
cp alt_lib/lib_early1.so pathnet_gym_amd/_hip/libpathnet_hip.so
