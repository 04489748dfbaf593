# alternate two prebuilt libraries (alt_lib/lib_<A>.so, lib_<B>.so) under one ab_kernel command line:
#   cmd_ab_libs.sh A B OUT ab_kernel-args...   (restores lib_<B> at the end)
set -o pipefail
A=$1; B=$2; OUT=$3; shift 3
mkdir -p gpurun_out
: > gpurun_out/$OUT
for r in 1 2; do
  for v in $A $B; do
    cp alt_lib/lib_$v.so pathnet_gym_amd/_hip/libpathnet_hip.so || exit 1
    echo "{\"lib\": \"$v\", \"round\": $r}" >> gpurun_out/$OUT
    timeout -k 10 200 python -u scripts/diag/ab_kernel.py "$@" >> gpurun_out/$OUT 2>> gpurun_out/$OUT.err || exit 1
  done
done
cp alt_lib/lib_$B.so pathnet_gym_amd/_hip/libpathnet_hip.so
