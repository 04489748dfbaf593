// Active-path gradient packing for the fused per-update all-reduce (parallel/comm.py).
//
// The reference applies RMSProp only to the variables of unfrozen modules
// (rmsprop_applier.py:92-106 via get_vars_idx, a3c_training_thread.py:190-216);
// inactive modules carry zero gradient because their mask is 0.  Here a rank
// all-reduces only the modules that some path of the WHOLE population
// expresses and that are not frozen, plus the heads/LSTM tail:
//
//  active_union : union[l*M+m] = (OR_p geno[p][l][m]) AND NOT frozen[l][m]  over P_total paths.
//                 Runs inside the optimizer hipGraph right after the device GA, so it describes the
//                 genotypes of the NEXT rollout; the host reads the L*M bytes back and turns them
//                 into a range table (one contiguous chunk per module, module-major layout).
//  pack_ranges  : dst[dst_off[r] + i] = src[src_off[r] + i]  (or the reverse for unpack), one thread
//                 per packed element, range found by binary search over the (<= L*M+1) dst offsets.
#include "common.h"

__global__ __launch_bounds__(256) void active_union_kernel(const uint8_t* __restrict__ geno,
                                                           const uint8_t* __restrict__ frozen, int P, int LM,
                                                           uint8_t* __restrict__ out) {
  const int lm = blockIdx.x;
  int any = 0;
  for (int p = threadIdx.x; p < P && !any; p += blockDim.x) any = geno[(long)p * LM + lm] != 0;
  any = __syncthreads_or(any);
  if (threadIdx.x == 0) out[lm] = (any && !frozen[lm]) ? 1 : 0;
}

// table: int64 [nr][3] = (src_off, len, dst_off), dst offsets ascending and contiguous
__global__ __launch_bounds__(256) void pack_ranges_kernel(float* __restrict__ flat, float* __restrict__ packed,
                                                          const long long* __restrict__ table, int nr, long n,
                                                          int unpack) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int lo = 0, hi = nr - 1;
    while (lo < hi) {                       // last range whose dst_off <= i
      const int mid = (lo + hi + 1) >> 1;
      if (table[3 * mid + 2] <= i) lo = mid;
      else hi = mid - 1;
    }
    const long src = table[3 * lo] + (i - table[3 * lo + 2]);
    if (unpack) flat[src] = packed[i];
    else packed[i] = flat[src];
  }
}

// Profiling window marker (bench.py --prof-window): an empty kernel whose name brackets the timed updates in a
// rocprofv3 kernel trace, so the per-kernel summary (scripts/prof_window.py) counts steady-state work only.
__global__ void prof_window_marker_kernel(int id) { (void)id; }

extern "C" {
int launch_prof_marker(int id, hipStream_t stream) {
  if (id < 0) return -22;
  prof_window_marker_kernel<<<1, 64, 0, stream>>>(id);
  return (int)hipGetLastError();
}

int launch_active_union(const void* geno, const void* frozen, int P, int L, int M, void* out, hipStream_t stream) {
  if (P <= 0 || L <= 0 || M <= 0) return -22;
  if ((long)L * M > 65535) return -1;            // one workgroup per (layer, module)
  active_union_kernel<<<L * M, 256, 0, stream>>>((const uint8_t*)geno, (const uint8_t*)frozen, P, L * M,
                                                 (uint8_t*)out);
  return (int)hipGetLastError();
}

int launch_pack_ranges(float* flat, float* packed, const long long* table, int nr, long n, int unpack,
                       hipStream_t stream) {
  if (nr < 0 || n < 0 || unpack < 0) return -22;
  if (nr <= 0 || n < 0) return -1;
  if (n == 0) return 0;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  pack_ranges_kernel<<<(int)blocks, 256, 0, stream>>>(flat, packed, table, nr, n, unpack);
  return (int)hipGetLastError();
}
}
