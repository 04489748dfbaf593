// Typed fully-connected PathNet layers: the supervised builders' module
// variants (reference pathnet.py:122-196): per module j a type from a table --
//   0 skip      out_j = x                      (no weights used)
//   1 fc        out_j = relu(x W_j + b_j)
//   2 residual  out_j = relu(x W_j + b_j) + x
// layer output = sum over the ACTIVE modules of the row's path (mask [P][M]).
//
// fp32 in and out: this is the supervised MNIST/SVHN path, where width-20 modules and
// 3072-wide inputs make MFMA tiles mostly padding, and the torch oracle is fp32.
// Rows are grouped by path (row r belongs to path r / rows_per_path), so a workgroup's
// active-module list is uniform. Weights are read in place from the flat module-major
// parameter buffer (module j of the layer: W at off + j*chunk as [K][C], b right after),
// and the gradients are written into a flat gradient buffer of the same layout.
//
//  typed_fc_fwd   : grid (P, ceil(rpp/16)). 16 rows staged through LDS in 256-wide K chunks.
//                   Each thread keeps (row, c) accumulators for every active weighted module.
//                   It writes out[R][C] and the relu mask [R][M][C] (uint8) for backward.
//  typed_fc_dgrad : grid (P, ceil(rpp/16)). g_m = dY * relu' is staged in LDS for all active modules.
//                   dX[r][k] = sum_m g_m[r] . W_m[k] + n_ident * dY[r][k].
//  typed_fc_wgrad : grid (M, ceil(K/16)). Each (m, k, c) has one owner (no atomics); loops over the rows of
//                   the paths where m is active.  Inactive and skip modules get zero gradient.
#include "common.h"

#define TF_RT 16
#define TF_KC 256
#define TF_MAXM 16
#define TF_MAXC 64
#define TF_PPT 4        // (row, c) pairs per thread: TF_RT * C <= 256 * TF_PPT

__global__ __launch_bounds__(256) void typed_fc_fwd_kernel(const float* __restrict__ x, int K,
                                                          const float* __restrict__ flat, long off, long chunk,
                                                          int C, int M, const float* __restrict__ mask,
                                                          const int* __restrict__ types, int rpp,
                                                          float* __restrict__ out, uint8_t* __restrict__ relu) {
  __shared__ float xs[TF_RT][TF_KC + 1];
  __shared__ int act[TF_MAXM];
  __shared__ int nact_s, nid_s;
  const int p = blockIdx.x, r0 = blockIdx.y * TF_RT, tid = threadIdx.x;
  const int nrows = min(TF_RT, rpp - r0);
  if (tid == 0) {
    int n = 0, ni = 0;
    for (int j = 0; j < M; ++j) {
      if (mask[(long)p * M + j] > 0.5f) {
        if (types[j] != 0) act[n++] = j;
        if (types[j] != 1) ++ni;
      }
    }
    nact_s = n;
    nid_s = ni;
  }
  __syncthreads();
  const int nact = nact_s;
  const long row_base = (long)p * rpp + r0;
  float acc[TF_PPT][TF_MAXM];
#pragma unroll
  for (int q = 0; q < TF_PPT; ++q)
#pragma unroll
    for (int a = 0; a < TF_MAXM; ++a) acc[q][a] = 0.f;
  for (int k0 = 0; k0 < K; k0 += TF_KC) {
    const int kc = min(TF_KC, K - k0);
    for (int i = tid; i < TF_RT * TF_KC; i += 256) {
      const int r = i / TF_KC, k = i - r * TF_KC;
      xs[r][k] = (r < nrows && k < kc) ? x[(row_base + r) * K + k0 + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TF_PPT; ++q) {
      const int o = tid + 256 * q;
      if (o >= TF_RT * C) continue;
      const int r = o / C, c = o - r * C;
#pragma unroll
      for (int a = 0; a < TF_MAXM; ++a) {
        if (a < nact) {
          const float* W = flat + off + (long)act[a] * chunk + (long)k0 * C + c;
          float s = 0.f;
          for (int k = 0; k < kc; ++k) s = fmaf(xs[r][k], W[(long)k * C], s);
          acc[q][a] += s;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < TF_PPT; ++q) {
    const int o = tid + 256 * q;
    if (o >= TF_RT * C) continue;
    const int r = o / C, c = o - r * C;
    if (r >= nrows) continue;
    const long row = row_base + r;
    float y = nid_s ? (float)nid_s * x[row * K + c] : 0.f;      // skip / residual identity terms (K == C)
    for (int j = 0; j < M; ++j) relu[(row * M + j) * C + c] = 0;
#pragma unroll
    for (int a = 0; a < TF_MAXM; ++a) {
      if (a < nact) {
        const int j = act[a];
        const float pre = acc[q][a] + flat[off + (long)j * chunk + (long)K * C + c];
        const bool on = pre > 0.f;
        y += on ? pre : 0.f;
        relu[(row * M + j) * C + c] = on;
      }
    }
    out[row * C + c] = y;
  }
}

__global__ __launch_bounds__(256) void typed_fc_dgrad_kernel(const float* __restrict__ dy, int K,
                                                            const float* __restrict__ flat, long off, long chunk,
                                                            int C, int M, const float* __restrict__ mask,
                                                            const int* __restrict__ types, int rpp,
                                                            const uint8_t* __restrict__ relu,
                                                            float* __restrict__ dx) {
  extern __shared__ float gs[];          // [nact][TF_RT][C]
  __shared__ int act[TF_MAXM];
  __shared__ int nact_s, nid_s;
  const int p = blockIdx.x, r0 = blockIdx.y * TF_RT, tid = threadIdx.x;
  const int nrows = min(TF_RT, rpp - r0);
  if (tid == 0) {
    int n = 0, ni = 0;
    for (int j = 0; j < M; ++j) {
      if (mask[(long)p * M + j] > 0.5f) {
        if (types[j] != 0) act[n++] = j;
        if (types[j] != 1) ++ni;
      }
    }
    nact_s = n;
    nid_s = ni;
  }
  __syncthreads();
  const int nact = nact_s;
  const long row_base = (long)p * rpp + r0;
  for (int i = tid; i < nact * TF_RT * C; i += 256) {
    const int a = i / (TF_RT * C), rem = i - a * TF_RT * C, r = rem / C, c = rem - r * C;
    float g = 0.f;
    if (r < nrows) {
      const long row = row_base + r;
      g = relu[(row * M + act[a]) * C + c] ? dy[row * C + c] : 0.f;
    }
    gs[i] = g;
  }
  __syncthreads();
  const float nid = (float)nid_s;
  for (int i = tid; i < nrows * K; i += 256) {
    const int r = i / K, k = i - r * K;
    const long row = row_base + r;
    float s = (nid != 0.f && k < C) ? nid * dy[row * C + k] : 0.f;
    for (int a = 0; a < nact; ++a) {
      const float* W = flat + off + (long)act[a] * chunk + (long)k * C;
      const float* g = gs + (a * TF_RT + r) * C;
      for (int c = 0; c < C; ++c) s = fmaf(g[c], W[c], s);
    }
    dx[row * K + k] = s;
  }
}

__global__ __launch_bounds__(256) void typed_fc_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                            int K, long off, long chunk, int C, int M, int P,
                                                            const float* __restrict__ mask,
                                                            const int* __restrict__ types, int rpp,
                                                            const uint8_t* __restrict__ relu,
                                                            float* __restrict__ gflat) {
  constexpr int KT = 16, RC = 64;
  __shared__ float xs[RC][KT + 1];
  __shared__ float gs[RC][TF_MAXC + 1];
  const int m = blockIdx.x, k0 = blockIdx.y * KT, tid = threadIdx.x;
  const int kt = min(KT, K - k0);
  const bool bias_blk = blockIdx.y == 0;
  float acc[TF_PPT], bacc = 0.f;
#pragma unroll
  for (int q = 0; q < TF_PPT; ++q) acc[q] = 0.f;
  if (types[m] != 0) {
    for (int p = 0; p < P; ++p) {
      if (!(mask[(long)p * M + m] > 0.5f)) continue;          // uniform
      for (int rr = 0; rr < rpp; rr += RC) {
        const int nr = min(RC, rpp - rr);
        const long row_base = (long)p * rpp + rr;
        for (int i = tid; i < RC * KT; i += 256) {
          const int r = i / KT, k = i - r * KT;
          xs[r][k] = (r < nr && k < kt) ? x[(row_base + r) * K + k0 + k] : 0.f;
        }
        for (int i = tid; i < RC * C; i += 256) {
          const int r = i / C, c = i - r * C;
          float g = 0.f;
          if (r < nr) {
            const long row = row_base + r;
            g = relu[(row * M + m) * C + c] ? dy[row * C + c] : 0.f;
          }
          gs[r][c] = g;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TF_PPT; ++q) {
          const int o = tid + 256 * q;
          if (o >= KT * C) continue;
          const int k = o / C, c = o - k * C;
          float s = acc[q];
          for (int r = 0; r < nr; ++r) s = fmaf(xs[r][k], gs[r][c], s);
          acc[q] = s;
        }
        if (bias_blk && tid < C)
          for (int r = 0; r < nr; ++r) bacc += gs[r][tid];
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int q = 0; q < TF_PPT; ++q) {
    const int o = tid + 256 * q;
    if (o >= KT * C) continue;
    const int k = o / C, c = o - k * C;
    if (k < kt) gflat[off + (long)m * chunk + (long)(k0 + k) * C + c] = acc[q];
  }
  if (bias_blk && tid < C) gflat[off + (long)m * chunk + (long)K * C + tid] = bacc;
}

extern "C" {
int launch_typed_fc_fwd(const float* x, int K, const float* flat, long off, long chunk, int C, int M,
                        const float* mask, const int* types, int P, int rpp, float* out, void* relu,
                        hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (C > TF_MAXC || M > TF_MAXM || TF_RT * C > 256 * TF_PPT || P < 1 || rpp < 1) return -1;
  dim3 grid(P, (rpp + TF_RT - 1) / TF_RT);
  typed_fc_fwd_kernel<<<grid, 256, 0, stream>>>(x, K, flat, off, chunk, C, M, mask, types, rpp, out,
                                                (uint8_t*)relu);
  return (int)hipGetLastError();
}

int launch_typed_fc_dgrad(const float* dy, int K, const float* flat, long off, long chunk, int C, int M,
                          const float* mask, const int* types, int P, int rpp, const void* relu, float* dx,
                          hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (C > TF_MAXC || M > TF_MAXM || P < 1 || rpp < 1) return -1;
  dim3 grid(P, (rpp + TF_RT - 1) / TF_RT);
  const size_t lds = (size_t)M * TF_RT * C * sizeof(float);
  typed_fc_dgrad_kernel<<<grid, 256, lds, stream>>>(dy, K, flat, off, chunk, C, M, mask, types, rpp,
                                                    (const uint8_t*)relu, dx);
  return (int)hipGetLastError();
}

int launch_typed_fc_wgrad(const float* x, const float* dy, int K, long off, long chunk, int C, int M, int P,
                          const float* mask, const int* types, int rpp, const void* relu, float* gflat,
                          hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (C > TF_MAXC || M > TF_MAXM || 16 * C > 256 * TF_PPT || P < 1 || rpp < 1) return -1;
  dim3 grid(M, (K + 15) / 16);
  typed_fc_wgrad_kernel<<<grid, 256, 0, stream>>>(x, dy, K, off, chunk, C, M, P, mask, types, rpp,
                                                  (const uint8_t*)relu, gflat);
  return (int)hipGetLastError();
}
}

// ===========================================================================
// MFMA variants (any width; the VALU kernels above cap C at 64): LDS-tiled fp32 GEMMs on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation -- the supervised oracle is fp32).
// Same semantics, relu-mask layout [R][M][C] and deterministic ownership as the VALU kernels:
//   fwd   grid (P, ceil(rpp/64), ceil(C/64))   out tile 64 x 64, the path's active modules in order
//   dgrad grid (P, ceil(rpp/64), ceil(K/64))   dX tile = sum_m (dY . relu'_m) W_m^T  (+ n_ident dY)
//   wgrad grid (M, ceil(K/64), ceil(C/64))     dW_m tile = sum over the rows of the paths using m of X^T G_m;
//                                              the k-tile-0 workgroups also own db_m
// Fragments (16x16x4 f32): lane l holds A[row l&15][k l>>4] and B[k l>>4][col l&15]; the result
// C[4(l>>4)+i][l&15] lands in lane l, register i.
// ===========================================================================
#define TM_T 64         // output tile edge
#define TM_KC 32        // reduction chunk staged per barrier pair

DEVI f4v mfma_f32_4(float a, float b, const f4v& c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// tile product: acc[ct] += As[16w + (l&15)][k] * Bs[k][16ct + (l&15)] over the staged chunk
DEVI void tm_chunk(const float (*As)[TM_KC + 1], const float (*Bs)[TM_T + 1], int w, int l, f4v (&acc)[4]) {
#pragma unroll
  for (int kk = 0; kk < TM_KC / 4; ++kk) {
    const float a = As[16 * w + (l & 15)][4 * kk + (l >> 4)];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = mfma_f32_4(a, Bs[4 * kk + (l >> 4)][16 * ct + (l & 15)], acc[ct]);
  }
}

DEVI void tm_active(const float* mask, const int* types, int p, int M, int* act, int* isact, int& nact, int& nid) {
  int n = 0, ni = 0;
  for (int j = 0; j < M; ++j) {
    isact[j] = 0;
    if (mask[(long)p * M + j] > 0.5f) {
      if (types[j] != 0) {
        act[n++] = j;
        isact[j] = 1;
      }
      if (types[j] != 1) ++ni;
    }
  }
  nact = n;
  nid = ni;
}

__global__ __launch_bounds__(256) void typed_fc_fwd_mfma_kernel(const float* __restrict__ x, int K,
                                                               const float* __restrict__ flat, long off, long chunk,
                                                               int C, int M, const float* __restrict__ mask,
                                                               const int* __restrict__ types, int rpp,
                                                               float* __restrict__ out, uint8_t* __restrict__ relu) {
  __shared__ float As[TM_T][TM_KC + 1];
  __shared__ float Bs[TM_KC][TM_T + 1];
  __shared__ int act[TF_MAXM], isact[TF_MAXM];
  __shared__ int nact_s, nid_s;
  const int p = blockIdx.x, r0 = blockIdx.y * TM_T, c0 = blockIdx.z * TM_T;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  if (tid == 0) tm_active(mask, types, p, M, act, isact, nact_s, nid_s);
  __syncthreads();
  const long row_base = (long)p * rpp;
  float y[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int i = 0; i < 4; ++i) y[ct][i] = 0.f;
  for (int a = 0; a < nact_s; ++a) {
    const int m = act[a];
    const float* W = flat + off + (long)m * chunk;
    f4v acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K; k0 += TM_KC) {
      __syncthreads();
      for (int i = tid; i < TM_T * TM_KC; i += 256) {
        const int r = i / TM_KC, k = i - r * TM_KC;
        As[r][k] = (r0 + r < rpp && k0 + k < K) ? x[(row_base + r0 + r) * K + k0 + k] : 0.f;
      }
      for (int i = tid; i < TM_KC * TM_T; i += 256) {
        const int k = i / TM_T, c = i - k * TM_T;
        Bs[k][c] = (k0 + k < K && c0 + c < C) ? W[(long)(k0 + k) * C + c0 + c] : 0.f;
      }
      __syncthreads();
      tm_chunk(As, Bs, w, l, acc);
    }
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int col = c0 + 16 * ct + (l & 15);
      const float bb = col < C ? W[(long)K * C + col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + 16 * w + 4 * (l >> 4) + i;
        const float pre = acc[ct][i] + bb;
        const bool on = pre > 0.f;
        y[ct][i] += on ? pre : 0.f;
        if (r < rpp && col < C) relu[((row_base + r) * M + m) * C + col] = on;
      }
    }
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int col = c0 + 16 * ct + (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + 16 * w + 4 * (l >> 4) + i;
      if (r >= rpp || col >= C) continue;
      const long row = row_base + r;
      const float id = nid_s ? (float)nid_s * x[row * K + col] : 0.f;      // skip / residual identity (K == C)
      out[row * C + col] = y[ct][i] + id;
      for (int j = 0; j < M; ++j)
        if (!isact[j]) relu[(row * M + j) * C + col] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void typed_fc_dgrad_mfma_kernel(const float* __restrict__ dy, int K,
                                                                 const float* __restrict__ flat, long off, long chunk,
                                                                 int C, int M, const float* __restrict__ mask,
                                                                 const int* __restrict__ types, int rpp,
                                                                 const uint8_t* __restrict__ relu,
                                                                 float* __restrict__ dx) {
  __shared__ float As[TM_T][TM_KC + 1];     // G_m rows x c-chunk
  __shared__ float Bs[TM_KC][TM_T + 1];     // W_m^T: c-chunk x k-cols
  __shared__ int act[TF_MAXM], isact[TF_MAXM];
  __shared__ int nact_s, nid_s;
  const int p = blockIdx.x, r0 = blockIdx.y * TM_T, kc0 = blockIdx.z * TM_T;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  if (tid == 0) tm_active(mask, types, p, M, act, isact, nact_s, nid_s);
  __syncthreads();
  const long row_base = (long)p * rpp;
  f4v acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = {0.f, 0.f, 0.f, 0.f};
  for (int a = 0; a < nact_s; ++a) {
    const int m = act[a];
    const float* W = flat + off + (long)m * chunk;
    for (int cc = 0; cc < C; cc += TM_KC) {
      __syncthreads();
      for (int i = tid; i < TM_T * TM_KC; i += 256) {
        const int r = i / TM_KC, c = i - r * TM_KC;
        float g = 0.f;
        if (r0 + r < rpp && cc + c < C) {
          const long row = row_base + r0 + r;
          g = relu[(row * M + m) * C + cc + c] ? dy[row * C + cc + c] : 0.f;
        }
        As[r][c] = g;
      }
      for (int i = tid; i < TM_KC * TM_T; i += 256) {
        const int k = i / TM_KC, c = i - k * TM_KC;       // c fastest: contiguous W_m[k][cc..]
        Bs[c][k] = (cc + c < C && kc0 + k < K) ? W[(long)(kc0 + k) * C + cc + c] : 0.f;
      }
      __syncthreads();
      tm_chunk(As, Bs, w, l, acc);
    }
  }
  const float nid = (float)nid_s;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int k = kc0 + 16 * ct + (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + 16 * w + 4 * (l >> 4) + i;
      if (r >= rpp || k >= K) continue;
      const long row = row_base + r;
      dx[row * K + k] = acc[ct][i] + ((nid != 0.f && k < C) ? nid * dy[row * C + k] : 0.f);
    }
  }
}

__global__ __launch_bounds__(256) void typed_fc_wgrad_mfma_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ dy, int K, long off,
                                                                 long chunk, int C, int M, int P,
                                                                 const float* __restrict__ mask,
                                                                 const int* __restrict__ types, int rpp,
                                                                 const uint8_t* __restrict__ relu,
                                                                 float* __restrict__ gflat) {
  __shared__ float As[TM_T][TM_KC + 1];     // X^T: k x row-chunk
  __shared__ float Bs[TM_KC][TM_T + 1];     // G_m: row-chunk x c
  const int m = blockIdx.x, k0 = blockIdx.y * TM_T, c0 = blockIdx.z * TM_T;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const bool bias_blk = blockIdx.y == 0;
  f4v acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = {0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  if (types[m] != 0) {
    for (int p = 0; p < P; ++p) {
      if (!(mask[(long)p * M + m] > 0.5f)) continue;      // uniform over the workgroup
      const long row_base = (long)p * rpp;
      for (int rr = 0; rr < rpp; rr += TM_KC) {
        __syncthreads();
        for (int i = tid; i < TM_KC * TM_T; i += 256) {
          const int r = i / TM_T, k = i - r * TM_T;        // k fastest: contiguous x[row][k0..]
          As[k][r] = (rr + r < rpp && k0 + k < K) ? x[(row_base + rr + r) * K + k0 + k] : 0.f;
        }
        for (int i = tid; i < TM_KC * TM_T; i += 256) {
          const int r = i / TM_T, c = i - r * TM_T;
          float g = 0.f;
          if (rr + r < rpp && c0 + c < C) {
            const long row = row_base + rr + r;
            g = relu[(row * M + m) * C + c0 + c] ? dy[row * C + c0 + c] : 0.f;
          }
          Bs[r][c] = g;
        }
        __syncthreads();
        tm_chunk(As, Bs, w, l, acc);
        if (bias_blk && tid < TM_T)
          for (int r = 0; r < TM_KC; ++r) bacc += Bs[r][tid];
      }
    }
  }
  float* G = gflat + off + (long)m * chunk;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int c = c0 + 16 * ct + (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + 16 * w + 4 * (l >> 4) + i;
      if (k < K && c < C) G[(long)k * C + c] = acc[ct][i];
    }
  }
  if (bias_blk && tid < TM_T && c0 + tid < C) G[(long)K * C + c0 + tid] = bacc;
}

extern "C" {
int launch_typed_fc_fwd_mfma(const float* x, int K, const float* flat, long off, long chunk, int C, int M,
                             const float* mask, const int* types, int P, int rpp, float* out, void* relu,
                             hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (M > TF_MAXM || P < 1 || rpp < 1 || K < 1 || C < 1) return -1;
  dim3 grid(P, (rpp + TM_T - 1) / TM_T, (C + TM_T - 1) / TM_T);
  typed_fc_fwd_mfma_kernel<<<grid, 256, 0, stream>>>(x, K, flat, off, chunk, C, M, mask, types, rpp, out,
                                                     (uint8_t*)relu);
  return (int)hipGetLastError();
}

int launch_typed_fc_dgrad_mfma(const float* dy, int K, const float* flat, long off, long chunk, int C, int M,
                               const float* mask, const int* types, int P, int rpp, const void* relu, float* dx,
                               hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (M > TF_MAXM || P < 1 || rpp < 1 || K < 1 || C < 1) return -1;
  dim3 grid(P, (rpp + TM_T - 1) / TM_T, (K + TM_T - 1) / TM_T);
  typed_fc_dgrad_mfma_kernel<<<grid, 256, 0, stream>>>(dy, K, flat, off, chunk, C, M, mask, types, rpp,
                                                       (const uint8_t*)relu, dx);
  return (int)hipGetLastError();
}

int launch_typed_fc_wgrad_mfma(const float* x, const float* dy, int K, long off, long chunk, int C, int M, int P,
                               const float* mask, const int* types, int rpp, const void* relu, float* gflat,
                               hipStream_t stream) {
  if (K <= 0 || chunk <= 0 || C <= 0 || M <= 0 || P <= 0 || rpp <= 0 || off < 0) return -22;
  if (M > TF_MAXM || P < 1 || rpp < 1 || K < 1 || C < 1) return -1;
  dim3 grid(M, (K + TM_T - 1) / TM_T, (C + TM_T - 1) / TM_T);
  typed_fc_wgrad_mfma_kernel<<<grid, 256, 0, stream>>>(x, dy, K, off, chunk, C, M, P, mask, types, rpp,
                                                       (const uint8_t*)relu, gflat);
  return (int)hipGetLastError();
}
}
