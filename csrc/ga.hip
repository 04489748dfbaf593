// Counter-based tournament GA on device (SURVEY.md K17/K18 + "genotype -> index compaction").
// Bit-exact mirror: pathnet_gym_amd/algo/ga_device.py (CounterPopulation).
//
//  ga_step     : one workgroup.  For every tournament slot whose B candidates all have a
//                fitness (!= -1000): winner = first argmax; each loser := counter-hash
//                mutation of the winner's genotype (reference operator, pathnet.py:50-63);
//                all candidates -> pending; freed slots redraw B disjoint non-busy paths.
//                Runs inside the optimizer hipGraph right after the fitness all-reduce.
//  ga_compact  : expressed = genotype | frozen for the rank's local paths -> the kernels'
//                mask / act_idx / act_cnt and the module-major inverse lists (in place).
#include "common.h"

#define GA_MAXC 64
#define GA_MAXB 8
#define GA_MAXL 16
#define GA_MAXM 16
#define GA_PENDING (-1000.0f)

DEVI uint32_t ga_rand(uint32_t seed, uint32_t gen, uint32_t x, uint32_t y, uint32_t z) {
  uint32_t h = wang_hash(wang_hash(seed) ^ gen);
  h = wang_hash(h ^ x);
  return wang_hash(h ^ (((y & 0xFFFFu) << 16) + (z & 0xFFFFu)));
}

__global__ __launch_bounds__(256) void ga_step_kernel(uint8_t* __restrict__ geno, float* __restrict__ fitness,
                                                      int* __restrict__ slots, long long* __restrict__ gen_ctr,
                                                      int* __restrict__ events, int P, int L, int M, int N, int B,
                                                      int C, uint32_t seed, uint8_t* __restrict__ reset) {
  __shared__ int ready[GA_MAXC], winner[GA_MAXC], gen_of[GA_MAXC];
  __shared__ int nfired;
  const int tid = threadIdx.x;
  // reset[i] = 1 for the candidates of tournaments that fire now (their episode windows restart)
  if (reset)
    for (int i = tid; i < P; i += 256) reset[i] = 0;
  if (tid < C) {
    int r = slots[tid * B] >= 0;
    int w = -1;
    float best = 0.f;
    for (int b = 0; r && b < B; ++b) {
      const int i = slots[tid * B + b];
      const float f = fitness[i];
      if (f == GA_PENDING) r = 0;
      else if (w < 0 || f > best) { best = f; w = i; }
    }
    ready[tid] = r;
    winner[tid] = r ? w : -1;
  }
  __syncthreads();
  if (tid == 0) {
    long long g = gen_ctr[0];
    int n = 0;
    for (int c = 0; c < C; ++c) {
      gen_of[c] = ready[c] ? (int)(g++) : -1;
      n += ready[c];
    }
    gen_ctr[0] = g;
    nfired = n;
  }
  __syncthreads();
  if (nfired == 0) {
    if (tid < C) events[tid * 3] = 0;
    return;
  }
  // mutation: one thread per (slot, candidate, layer); the layer's modules in order (the operator is sequential)
  const long ka = (long)L * N, ki = (long)L * (M - N) * M;
  for (int item = tid; item < C * B * L; item += 256) {
    const int c = item / (B * L), rem = item - c * B * L, b = rem / L, l = rem - b * L;
    if (!ready[c]) continue;
    const int i = slots[c * B + b], w = winner[c];
    if (i == w) continue;
    uint8_t g[GA_MAXM];
    for (int m = 0; m < M; ++m) g[m] = geno[((long)w * L + l) * M + m];
    const uint32_t gen = (uint32_t)gen_of[c];
    for (int m = 0; m < M; ++m) {
      const uint32_t h0 = ga_rand(seed, gen, (uint32_t)i, (uint32_t)l, (uint32_t)(2 * m));
      const uint32_t h1 = ga_rand(seed, gen, (uint32_t)i, (uint32_t)l, (uint32_t)(2 * m + 1));
      const long long u24 = (long long)(h0 >> 8);
      if (g[m]) {
        if (u24 * ka < (1ll << 25)) { g[m] = 0; g[h1 % (uint32_t)M] = 1; }
      } else if (u24 * ki < (1ll << 25)) {
        g[h1 % (uint32_t)M] = 1;
      }
    }
    for (int m = 0; m < M; ++m) geno[((long)i * L + l) * M + m] = g[m];
  }
  __syncthreads();
  if (tid < C) {
    events[tid * 3 + 0] = ready[tid];
    events[tid * 3 + 1] = winner[tid];
    events[tid * 3 + 2] = gen_of[tid];
  }
  // every fired slot's candidates -> pending (read by nothing else in this kernel from here on)
  for (int item = tid; item < C * B; item += 256) {
    const int c = item / B;
    if (ready[c]) {
      fitness[slots[item]] = GA_PENDING;
      if (reset) reset[slots[item]] = 1;
    }
  }
  __syncthreads();
  // redraw the freed slots (serial, as the mirror): busy = candidates of slots still pending
  if (tid == 0) {
    extern __shared__ uint8_t busy[];     // [P]
    for (int i = 0; i < P; ++i) busy[i] = 0;
    for (int c = 0; c < C; ++c)
      if (!ready[c] && slots[c * B] >= 0)
        for (int b = 0; b < B; ++b) busy[slots[c * B + b]] = 1;
    int nfree = 0;
    for (int i = 0; i < P; ++i) nfree += !busy[i];
    for (int c = 0; c < C; ++c) {
      if (!ready[c]) continue;
      if (nfree < B) {
        for (int b = 0; b < B; ++b) slots[c * B + b] = -1;
        continue;
      }
      int got = 0, attempt = 0;
      while (got < B && attempt < 64 * B) {
        const int i = (int)(ga_rand(seed, (uint32_t)gen_of[c], 0xFFFFu, (uint32_t)c, (uint32_t)attempt) % (uint32_t)P);
        ++attempt;
        if (!busy[i]) { busy[i] = 1; slots[c * B + got++] = i; }
      }
      for (int i = 0; got < B; ++i)
        if (!busy[i]) { busy[i] = 1; slots[c * B + got++] = i; }
      nfree -= B;
    }
  }
}

// expressed masks + compacted lists for paths [p_off, p_off + P_local)
__global__ void ga_compact_paths_kernel(const uint8_t* __restrict__ geno, const uint8_t* __restrict__ frozen,
                                        int p_off, int P_local, int L, int M, float* __restrict__ mask,
                                        int* __restrict__ act_idx, int* __restrict__ act_cnt) {
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= P_local * L) return;
  const int p = item / L, l = item - p * L;
  const uint8_t* g = geno + ((long)(p_off + p) * L + l) * M;
  int n = 0;
  for (int m = 0; m < M; ++m) {
    const int e = (g[m] | frozen[l * M + m]) ? 1 : 0;
    mask[((long)p * L + l) * M + m] = (float)e;
    if (e) act_idx[((long)p * L + l) * M + n++] = m;
  }
  for (int m = n; m < M; ++m) act_idx[((long)p * L + l) * M + m] = -1;
  act_cnt[p * L + l] = n;
}

// module-major inverse lists (paths in ascending order, slot = rank of the module in the path's list).
// One wave per (layer, module): lane i tests paths i, i+64, ...; a ballot + popcount gives each user its
// position in path order (the serial per-module scan over P paths took 55 us per update at P = 64).
__global__ __launch_bounds__(64) void ga_compact_inverse_kernel(const float* __restrict__ mask, int P_local, int L,
                                                                int M, int* __restrict__ inv_path,
                                                                int* __restrict__ inv_slot,
                                                                int* __restrict__ inv_cnt) {
  const int item = blockIdx.x;
  if (item >= L * M) return;
  const int l = item / M, j = item - l * M;
  const int lane = threadIdx.x;
  const long base = ((long)l * M + j) * P_local;
  int n = 0;
  for (int p0 = 0; p0 < P_local; p0 += 64) {
    const int p = p0 + lane;
    bool use = false;
    int slot = 0;
    if (p < P_local) {
      const float* row = mask + ((long)p * L + l) * M;
      use = row[j] > 0.5f;
      for (int m = 0; m < j; ++m) slot += row[m] > 0.5f;
    }
    const uint64_t bal = __ballot(use);
    const int rank = n + __popcll(bal & ((1ull << lane) - 1ull));
    if (use) {
      inv_path[base + rank] = p;
      inv_slot[base + rank] = slot;
    }
    n += __popcll(bal);
  }
  for (int k = n + lane; k < P_local; k += 64) {
    inv_path[base + k] = 0;
    inv_slot[base + k] = 0;
  }
  if (lane == 0) inv_cnt[l * M + j] = n;
}

// inverse lists of one path group [p0, p0 + np) of the split rollout (runtime/engine.py): every module's path-ordered
// list is cut to the group's paths and re-based to group-local path indices, so the module-major fc forward of the
// group sees a population of np paths (its X / Y / bits / act tables passed at the group's base).  One wave per
// (layer, module).  Layout [L][M][np].
__global__ __launch_bounds__(64) void inv_group_kernel(const int* __restrict__ inv_path, const int* __restrict__ inv_slot,
                                                       const int* __restrict__ inv_cnt, int P, int L, int M, int p0,
                                                       int np, int* __restrict__ gpath, int* __restrict__ gslot,
                                                       int* __restrict__ gcnt) {
  const int item = blockIdx.x;
  if (item >= L * M) return;
  const int lane = threadIdx.x;
  const long base = (long)item * P, gbase = (long)item * np;
  const int n = inv_cnt[item];
  int k = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const int p = i < n ? inv_path[base + i] : -1;
    const bool in = p >= p0 && p < p0 + np;
    const uint64_t bal = __ballot(in);
    const int rank = k + __popcll(bal & ((1ull << lane) - 1ull));
    if (in) {
      gpath[gbase + rank] = p - p0;
      gslot[gbase + rank] = inv_slot[base + i];
    }
    k += __popcll(bal);
  }
  for (int kk = k + lane; kk < np; kk += 64) {
    gpath[gbase + kk] = 0;
    gslot[gbase + kk] = 0;
  }
  if (lane == 0) gcnt[item] = k;
}

// The optimizer graph's small tail in one launch (runtime/engine.py _optimizer_body): the local fitness <- the device
// GA's view, the episode windows of the candidates of tournaments that just fired restarted (fit_window > 0), the
// frame ring's first-valid-channel row carried (fc_dst = fc_src, n_fc bytes) and the update counter advanced --
// four to six small torch launches before
__global__ __launch_bounds__(256) void opt_tail_kernel(const float* __restrict__ fit, const uint8_t* __restrict__ reset,
                                                       int p_off, int P, int fit_window, float* __restrict__ fitness,
                                                       float* __restrict__ fit_cnt, float* __restrict__ fit_sum,
                                                       const uint8_t* __restrict__ fc_src, uint8_t* __restrict__ fc_dst,
                                                       int n_fc, long long* __restrict__ ctr,
                                                       double* __restrict__ lr_sched, float* __restrict__ lr_next) {
  const int i = (int)(blockIdx.x * 256 + threadIdx.x);
  // the NEXT update's learning rate, on device (no host fill per update): lr_sched = {lr0, max_t, mode, frames per
  // update, frames done}; frames done += frames per update; lr = lr0 (mode 0, "none") or max(lr0 * (max_t - t) / max_t,
  // 0) with t = frames done (algo/optim.py anneal_lr: the same double operations, rounded to fp32 once)
  if (i == 0 && lr_sched) {
    const double t = lr_sched[4] + lr_sched[3];
    lr_sched[4] = t;
    double lr = lr_sched[0];
    if (lr_sched[2] != 0.0) {
      lr = lr_sched[0] * (lr_sched[1] - t) / lr_sched[1];
      lr = lr > 0.0 ? lr : 0.0;
    }
    lr_next[0] = (float)lr;
  }
  if (i < P) {
    fitness[i] = fit[p_off + i];
    if (fit_window > 0 && reset[p_off + i]) {
      fit_cnt[i] = 0.f;
      fit_sum[i] = 0.f;
    }
  }
  if (i < n_fc) fc_dst[i] = fc_src[i];
  if (i == 0 && ctr) ctr[0] += 1;
}

extern "C" {
int launch_opt_tail(const float* fit, const void* reset, int p_off, int P, int fit_window, float* fitness,
                    float* fit_cnt, float* fit_sum, const void* fc_src, void* fc_dst, int n_fc, long long* ctr,
                    double* lr_sched, float* lr_next, hipStream_t stream) {
  if ((lr_sched != nullptr) != (lr_next != nullptr)) return -22;
  if (P < 0 || p_off < 0 || n_fc < 0 || (P > 0 && (!fit || !reset || !fitness || !fit_cnt || !fit_sum)) ||
      (n_fc > 0 && (!fc_src || !fc_dst))) return -22;
  const int n = P > n_fc ? P : n_fc;
  opt_tail_kernel<<<(n > 0 ? n + 255 : 256) / 256, 256, 0, stream>>>(fit, (const uint8_t*)reset, p_off, P, fit_window,
                                                                    fitness, fit_cnt, fit_sum,
                                                                    (const uint8_t*)fc_src, (uint8_t*)fc_dst, n_fc,
                                                                    ctr, lr_sched, lr_next);
  return (int)hipGetLastError();
}

int launch_inv_group(const int* inv_path, const int* inv_slot, const int* inv_cnt, int P, int L, int M, int p0, int np,
                     int* gpath, int* gslot, int* gcnt, hipStream_t stream) {
  if (P <= 0 || L <= 0 || M <= 0 || p0 < 0 || np <= 0 || p0 + np > P || !gpath || !gslot || !gcnt) return -22;
  inv_group_kernel<<<L * M, 64, 0, stream>>>(inv_path, inv_slot, inv_cnt, P, L, M, p0, np, gpath, gslot, gcnt);
  return (int)hipGetLastError();
}

int launch_ga_step(void* geno, float* fitness, int* slots, long long* gen_ctr, int* events, int P, int L, int M,
                   int N, int B, int C, unsigned seed, void* reset, hipStream_t stream) {
  if (P <= 0 || L <= 0 || M <= 0 || N <= 0 || B <= 0 || C <= 0) return -22;
  if (C > GA_MAXC || B > GA_MAXB || L > GA_MAXL || M > GA_MAXM || C < 1) return -1;
  ga_step_kernel<<<1, 256, (size_t)P, stream>>>((uint8_t*)geno, fitness, slots, gen_ctr, events, P, L, M, N, B, C,
                                                seed, (uint8_t*)reset);
  return (int)hipGetLastError();
}

int launch_ga_compact(const void* geno, const void* frozen, int p_off, int P_local, int L, int M, float* mask,
                      int* act_idx, int* act_cnt, int* inv_path, int* inv_slot, int* inv_cnt, hipStream_t stream) {
  if (P_local <= 0 || L <= 0 || M <= 0 || p_off < 0) return -22;
  if (M > GA_MAXM) return -1;
  const int n1 = P_local * L;
  ga_compact_paths_kernel<<<(n1 + 255) / 256, 256, 0, stream>>>((const uint8_t*)geno, (const uint8_t*)frozen, p_off,
                                                                P_local, L, M, mask, act_idx, act_cnt);
  if (inv_path) {
    ga_compact_inverse_kernel<<<L * M, 64, 0, stream>>>(mask, P_local, L, M, inv_path, inv_slot, inv_cnt);
  }
  return (int)hipGetLastError();
}
}
