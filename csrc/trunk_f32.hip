// PathNet trunk in fp32 (TrainConfig.compute_dtype = "fp32").
//
// The reference computes in fp32 throughout (TF default dtype; game_ac_network.py:89-110 builds every
// conv/fc variable as float32).  This file is the engine's fp32-operand mode: activations, weight copies,
// masked gradients and MFMA operands are all fp32, on v_mfma_f32_16x16x4_f32 (exact fp32 products and
// accumulation, 64 FLOP/clk/SIMD -- 1/16 of the bf16 rate, so this mode is the precision reference, not
// the throughput mode).
//
// The epilogues (bias, ReLU, ReLU bits by ballot, per-layer module sum) have the form of the bf16 kernels'
// (trunk_fwd.hip / trunk_bwd.hip).  A 32-wide k chunk per lane group keeps the bf16 kernels' load shape:
// lane group g = l>>4 holds k = kk+8g .. kk+8g+7 and the chunk is eight 16x16x4 MFMAs, sub-step j feeding
// k-slot g with element kk+8g+j (A and B use the same permutation of k, so the sum is unchanged).
//   conv fwd   : B fragments straight from the L1-resident weight copy (no LDS staging), RT = 2 row tiles
//                per wave, raw (uint8) A fragments of the next k-step prefetched during this step's MFMAs.
//   conv dgrad : one thread per input pixel, weights in LDS as [slot][tap][c][ci] (two ds_read_b128 per 8 FMAs).
//   fc fwd     : register pipeline (next k-step's A and B loaded during this step's MFMAs).
//
// Every reduction is in a FIXED order -- no float atomics anywhere in this file:
//   conv wgrad : each (path, row chunk) workgroup writes its partial dW/db of every active slot to a
//                scratch slab; conv_wgrad_reduce_f32 sums the slabs of the (path, slot) users of each
//                module in (path, chunk) order (inv_path lists are path-ordered, csrc/ga.hip).
//   fc wgrad   : module-major, one workgroup owns a 64x64 dW tile and walks every user in path order.
//   biases     : per-thread partials over fixed rows, then an ordered LDS reduction.
// so one seed gives a bit-identical gradient run to run.
#include "common.h"

#define F32_MAXM 16
#define F32_MAX_CT 8
#define F32_BM 64

struct ConvGeomF {
  int Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP;
};

// eight k-sub-steps of one 32-wide chunk (see header)
DEVI f4v mfma_f32x8(const float* a, const float* b, f4v c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
  return c;
}

DEVI void ld8f(const float* p, float* r) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
  r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
}

DEVI void st8f(float* p, const float* r) {
  *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(r[4], r[5], r[6], r[7]);
}

// Input element kinds: uint8 frames (exact in fp32), bf16 activations (the bf16 engine's deterministic
// weight-gradient mode reads them here), fp32 activations.
enum XKind { XU8 = 0, XBF16 = 1, XF32 = 2 };

// 8 consecutive input values of one im2col / fc row
template <int XK>
DEVI void load_a8f(const void* X, long off, float* r) {
  if constexpr (XK == XU8) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + off);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = (float)((v.x >> (8 * j)) & 0xFFu);
      r[j + 4] = (float)((v.y >> (8 * j)) & 0xFFu);
    }
  } else if constexpr (XK == XBF16) {
    const s8v v = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = bf2f((bf16_t)v[j]);
  } else {
    ld8f(reinterpret_cast<const float*>(X) + off, r);
  }
}

// raw (unconverted) prefetch registers of 8 input values: 2 / 4 / 8 VGPRs for uint8 / bf16 / fp32
template <int XK> struct XRaw { float4 a, b; };
template <> struct XRaw<XU8> { uint2 a; };
template <> struct XRaw<XBF16> { uint4 a; };

template <int XK>
DEVI XRaw<XK> load_raw8(const void* X, long off) {
  XRaw<XK> r;
  if constexpr (XK == XU8) r.a = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + off);
  else if constexpr (XK == XBF16) r.a = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(X) + off);
  else {
    r.a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + off);
    r.b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + off + 4);
  }
  return r;
}

template <int XK>
DEVI XRaw<XK> zero_raw8() {
  XRaw<XK> r;
  if constexpr (XK == XU8) r.a = make_uint2(0, 0);
  else if constexpr (XK == XBF16) r.a = make_uint4(0, 0, 0, 0);
  else { r.a = make_float4(0.f, 0.f, 0.f, 0.f); r.b = r.a; }
  return r;
}

template <int XK>
DEVI void raw8_to_f(const XRaw<XK>& r, float* o) {
  if constexpr (XK == XU8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (float)((r.a.x >> (8 * j)) & 0xFFu);
      o[j + 4] = (float)((r.a.y >> (8 * j)) & 0xFFu);
    }
  } else if constexpr (XK == XBF16) {
    const uint32_t u[4] = {r.a.x, r.a.y, r.a.z, r.a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = __uint_as_float(u[j] << 16);
      o[2 * j + 1] = __uint_as_float(u[j] & 0xFFFF0000u);
    }
  } else {
    o[0] = r.a.x; o[1] = r.a.y; o[2] = r.a.z; o[3] = r.a.w;
    o[4] = r.b.x; o[5] = r.b.y; o[6] = r.b.z; o[7] = r.b.w;
  }
}

template <int XK>
DEVI float load_a1f(const void* X, long off) {
  if constexpr (XK == XU8) return (float)reinterpret_cast<const uint8_t*>(X)[off];
  else if constexpr (XK == XBF16) return bf2f(reinterpret_cast<const bf16_t*>(X)[off]);
  else return reinterpret_cast<const float*>(X)[off];
}

// ---------------------------------------------------------------------------
// conv forward.  grid = (ceil(T*E*Ho*Wo / (64*RT)), P), block 256; wave w owns RT row tiles of 16 rows.
// X : [T'][P*E][Hin*Win*Cin] (uint8 or fp32), Y: [T'][P*E][Ho*Wo*8] fp32
// bits: [M][bits_rows] uint8;  Wc: [M][8][KP] fp32 (k contiguous, zero padded)
// B fragments are read straight from the L1/L2-resident fp32 weight copy and each feeds RT MFMAs.  (v1
// staged the active columns in LDS per 64-row workgroup: 1.2 GB of L2->LDS traffic per rollout step and
// 83 KB of LDS, i.e. one workgroup per CU -- 1.40 ms per conv1 step.)
// ---------------------------------------------------------------------------
template <bool U8IN, int RT, int MCT>
__global__ __launch_bounds__(256) void conv_fwd_f32_kernel(
    const void* __restrict__ X, float* __restrict__ Y, uint8_t* __restrict__ bits, const float* __restrict__ Wc,
    const float* __restrict__ flat, long bias_off, int chunk, const int* __restrict__ act_idx,
    const int* __restrict__ act_cnt, int layer, int L, int M, ConvGeomF g, int P, int E, int T, int t0,
    long bits_rows, float in_scale, float out_scale) {
  __shared__ int koff[64];
  __shared__ int mods[F32_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < F32_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  for (int kc = tid; kc < g.KP / 8; kc += 256) {
    const int k0 = kc * 8;
    int off = -1;
    if (k0 < g.K) {
      const int tap = k0 / g.Cin;
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
      off = (kh * g.Win + kw) * g.Cin + (k0 - tap * g.Cin);
    }
    koff[kc] = off;
  }
  __syncthreads();
  const int HoWo = g.Ho * g.Wo;
  const int Rtot = T * E * HoWo;                  // rows of this path (< 2^31, checked by the launcher)
  const int PE = P * E;
  const int w = tid >> 6, l = tid & 63, grp = l >> 4, c16 = l & 15;
  const int rw = blockIdx.x * 64 * RT + w * 16 * RT;
  if (rw >= Rtot) return;
  long xbase[RT];
  bool va[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const int ra = rw + i * 16 + c16;
    va[i] = ra < Rtot;
    const int rr = va[i] ? ra : rw;
    const int s = rr / HoWo;
    const int pos = rr - s * HoWo;
    const int oh = pos / g.Wo, ow = pos - oh * g.Wo;
    xbase[i] = sample_global(p, s, E, PE, t0) * (long)(g.Hin * g.Win * g.Cin) +
               (long)(oh * g.S * g.Win + ow * g.S) * g.Cin;
  }
  // B column c16 of tile ct = (slot ct*2 + c16/8, map c16%8); slots >= cnt read module mods[0] (masked below)
  const float* wrow[MCT];
#pragma unroll
  for (int ct = 0; ct < MCT; ++ct) {
    const int slot = ct * 2 + (c16 >> 3);
    wrow[ct] = Wc + ((long)((slot < cnt ? mods[slot] : mods[0]) * 8 + (c16 & 7))) * g.KP;
  }
  f4v acc[RT][MCT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
  // the next k-step's A fragments (raw: 2 VGPRs per row tile for uint8) are loaded before this step's MFMAs
  constexpr int XK = U8IN ? XU8 : XF32;
  XRaw<XK> an[RT];
  auto aload = [&](int kk) {
    const int off = koff[(kk + 8 * grp) >> 3];
#pragma unroll
    for (int i = 0; i < RT; ++i) an[i] = (va[i] && off >= 0) ? load_raw8<XK>(X, xbase[i] + off) : zero_raw8<XK>();
  };
  aload(0);
  for (int kk = 0; kk < g.KP; kk += 32) {
    const int k0 = kk + 8 * grp;
    float a[RT][8];
#pragma unroll
    for (int i = 0; i < RT; ++i) raw8_to_f<XK>(an[i], a[i]);
    if (kk + 32 < g.KP) aload(kk + 32);
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct) {
      if (ct < nct) {
        float b[8];
        ld8f(wrow[ct] + k0, b);
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i][ct] = mfma_f32x8(a[i], b, acc[i][ct]);
      }
    }
  }
  // epilogue per row tile: bias, ReLU, ReLU bits, module sum (layout of conv_fwd_kernel, trunk_fwd.hip)
  const int h = c16 >> 3, ch = l & 7;
  float bb[MCT];
#pragma unroll
  for (int ct = 0; ct < MCT; ++ct) {
    const int slot = ct * 2 + h;
    bb[ct] = (ct < nct && slot < cnt) ? flat[bias_off + (long)mods[slot] * chunk + ch] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const int rbase = rw + i * 16;
    if (rbase >= Rtot) break;
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
    long grow4;
    {
      const int r4 = rbase + 4 * grp;
      const int s = r4 / HoWo;
      grow4 = sample_global(p, s, E, PE, t0) * HoWo + (r4 - s * HoWo);
    }
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct) {
      if (ct < nct) {
        const int slot = ct * 2 + h;
        const bool sv = slot < cnt;
        uint32_t word = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][ct][r] * in_scale + bb[ct];
          const bool pos = sv && v > 0.f;
          sum[r] += pos ? v : 0.f;
          const uint64_t bal = __ballot(pos);
          word |= (uint32_t)((bal >> (16 * grp + 8 * h)) & 0xFFull) << (8 * r);
        }
        if (ch == 0 && sv) *reinterpret_cast<uint32_t*>(bits + (long)slot * bits_rows + grow4) = word;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
    if (h == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + 4 * grp + r;
        if (row < Rtot) {
          const int s = row / HoWo;
          const int pos = row - s * HoWo;
          Y[(sample_global(p, s, E, PE, t0) * HoWo + pos) * 8 + ch] = sum[r] * out_scale;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fc forward (indexed grouped GEMM).  grid = (ceil(T*E/BM), ceil(Cout/64), P).
// X: [T'][P*E][ldx] fp32;  Y: [T'][P*E][Cout] fp32;  bits16: [M][bits_rows][Cout/16]
// Wc: [M][Cout][KP] fp32.  4 waves as 2 (rows) x 2 (cols); wave tile (BM/2) x 32.
// Rows shorter than 8 k values (vector observations, ldx = K < 8) load element-wise.
// ---------------------------------------------------------------------------
template <int BM>
__global__ __launch_bounds__(256) void fc_fwd_f32_kernel(
    const float* __restrict__ X, int ldx, float* __restrict__ Y, uint16_t* __restrict__ bits,
    const float* __restrict__ Wc, const float* __restrict__ flat, long bias_off, int chunk,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M, int K, int KP,
    int Cout, int P, int E, int T, int t0, long bits_rows, float out_scale) {
  constexpr int RT = BM / 32;
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * BM + wr * (BM / 2);
  const int col0 = blockIdx.y * 64 + wc * 32;
  if (row0 >= Rtot || col0 >= Cout) return;
  const int grp = l >> 4, c16 = l & 15;
  long xrow[RT];
  bool xv[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const long r = row0 + i * 16 + c16;
    xv[i] = r < Rtot;
    xrow[i] = sample_global(p, (int)(xv[i] ? r : row0), E, PE, t0) * ldx;
  }
  const bool vec8 = (ldx % 4 == 0) && (K % 8 == 0);
  float sum[RT][2][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[i][j][r] = 0.f;

  for (int a = 0; a < cnt; ++a) {
    const int mod = act_idx[(p * L + layer) * M + a];
    const float* Wm = Wc + (long)mod * Cout * KP;
    f4v acc[RT][2];
#pragma unroll
    for (int i = 0; i < RT; ++i) { acc[i][0] = {0.f, 0.f, 0.f, 0.f}; acc[i][1] = {0.f, 0.f, 0.f, 0.f}; }
    if (vec8) {
      // register pipeline: the next k-step's A and B fragments load during this step's MFMAs
      float an[RT][8], bn[2][8];
      auto fload = [&](int kk) {
        const int k0 = kk + 8 * grp;
#pragma unroll
        for (int i = 0; i < RT; ++i) {
          if (xv[i] && k0 < K) ld8f(X + xrow[i] + k0, an[i]);
          else {
#pragma unroll
            for (int j = 0; j < 8; ++j) an[i][j] = 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) ld8f(Wm + (long)(col0 + j * 16 + c16) * KP + k0, bn[j]);
      };
      fload(0);
      for (int kk = 0; kk < KP; kk += 32) {
        float av[RT][8], bv[2][8];
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) av[i][j] = an[i][j];
#pragma unroll
        for (int jn = 0; jn < 2; ++jn)
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[jn][j] = bn[jn][j];
        if (kk + 32 < KP) fload(kk + 32);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < RT; ++i) acc[i][j] = mfma_f32x8(av[i], bv[j], acc[i][j]);
      }
    } else {
      for (int kk = 0; kk < KP; kk += 32) {
        const int k0 = kk + 8 * grp;
        float av[RT][8];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
#pragma unroll
          for (int j = 0; j < 8; ++j) av[i][j] = (xv[i] && k0 + j < K) ? X[xrow[i] + k0 + j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float b[8];
          ld8f(Wm + (long)(col0 + j * 16 + c16) * KP + k0, b);
#pragma unroll
          for (int i = 0; i < RT; ++i) acc[i][j] = mfma_f32x8(av[i], b, acc[i][j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + j * 16 + c16;
      const float bb = flat[bias_off + (long)mod * chunk + col];
#pragma unroll
      for (int i = 0; i < RT; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r] + bb;
          const bool pos = v > 0.f;
          sum[i][j][r] += pos ? v : 0.f;
          const uint64_t bal = __ballot(pos);
          const long row = row0 + i * 16 + 4 * grp + r;
          if (c16 == 0 && row < Rtot) {
            const long sg = sample_global(p, (int)row, E, PE, t0);
            bits[((long)a * bits_rows + sg) * (Cout / 16) + (col0 + j * 16) / 16] =
                (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + i * 16 + 4 * grp + r;
      if (row < Rtot) {
        const long sg = sample_global(p, (int)row, E, PE, t0);
#pragma unroll
        for (int j = 0; j < 2; ++j) Y[sg * Cout + col0 + j * 16 + c16] = sum[i][j][r] * out_scale;
      }
    }
}

// ---------------------------------------------------------------------------
// conv wgrad partials.  grid = (nch, P), block 256; chunk c of path p covers the path-local im2col rows
// [c*rpc, (c+1)*rpc).  Writes, for every active slot a,
//   part[((p*nch + c)*M + a)*(K*8 + 8) + e]  (e < K*8: dW[k][ch] at k*8+ch; e = K*8+ch: db[ch]).
// Active slots are processed in passes of 4 (two 16-wide column tiles; one pass when cnt <= 4): the
// accumulators are acc[4 k-tiles][2 col tiles] = 32 registers, not sized for 16 modules (v1: 128 AGPRs +
// 150 VGPRs = one wave per SIMD, 51 ms for conv1).  Per 32-row stage: Xs [32][XS] fp32 im2col rows and
// Gs [32][F32_WG_GS] masked G of the pass's 4 slots; the next stage's global loads are issued into
// registers before this stage's MFMAs.  D[k][col] += sum_rows Xs[row][k] Gs[row][col], 4 rows per MFMA.
// ---------------------------------------------------------------------------
#define F32_WG_GS (32 + 16)
#define F32_WG_NX 4            // X items (8 values) per thread per stage: 32 rows * KP/8 <= 1024 for KP <= 256
template <int XK>
__global__ __launch_bounds__(256) void conv_wgrad_f32_kernel(
    const void* __restrict__ X, const float* __restrict__ G, const uint8_t* __restrict__ bits,
    float* __restrict__ part, const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L,
    int M, ConvGeomF g, int P, int E, int T, long bits_rows, int rows_per_chunk, float in_scale, float g_scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.y, nch = gridDim.x;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int XS = g.KP + 16;                 // row stride = 16 banks: the 4 k-slot rows of an MFMA hit 64 banks
  constexpr int GS = F32_WG_GS;
  float* Xs = reinterpret_cast<float*>(smem);                     // [32][XS]
  float* Gs = Xs + 32 * XS;                                        // [32][GS]
  float* bred = Gs + 32 * GS;                                      // [32 rows][4 slots][8]
  int* koff = reinterpret_cast<int*>(bred + 32 * 4 * 8);           // [KP/8]
  const int tid = threadIdx.x;
  for (int kc = tid; kc < g.KP / 8; kc += 256) {
    const int k0 = kc * 8;
    int off = -1;
    if (k0 < g.K) {
      const int tap = k0 / g.Cin;
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
      off = (kh * g.Win + kw) * g.Cin + (k0 - tap * g.Cin);
    }
    koff[kc] = off;
  }
  __syncthreads();

  const int HoWo = g.Ho * g.Wo;
  const int Rtot = T * E * HoWo;
  const int PE = P * E;
  const int HWC = g.Hin * g.Win * g.Cin;
  const int r_begin = blockIdx.x * rows_per_chunk;
  const int r_end = min(Rtot, r_begin + rows_per_chunk);
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15;
  const int nmt = g.KP / 16;
  const int kvec = g.KP / 8;
  const int nx = 32 * kvec;
  const int K8 = g.K * 8;
  const long pstride = (long)K8 + 8;
  float* pbase = part + ((long)(p * nch + blockIdx.x) * M) * pstride;
  // G staging: thread tid < 128 -> row gr = tid >> 2, slot (of the pass) gs = tid & 3
  const int gr = tid >> 2, gs = tid & 3;
  // this thread's X items (stage-invariant): im2col row within the stage, input offset of the k chunk
  // (-1: padding chunk or no item) and LDS offset (-1: no item)
  int xrow[F32_WG_NX], xoff[F32_WG_NX], xsoff[F32_WG_NX];
#pragma unroll
  for (int q = 0; q < F32_WG_NX; ++q) {
    const int it = tid + 256 * q;
    xrow[q] = 0;
    xoff[q] = -1;
    xsoff[q] = -1;
    if (it < nx) {
      const int row = it / kvec, kc = it - row * kvec;
      xrow[q] = row;
      xoff[q] = koff[kc];
      xsoff[q] = row * XS + kc * 8;
    }
  }

  for (int s0 = 0; s0 < cnt; s0 += 4) {
    const int ns = min(4, cnt - s0);
    const int nct = (ns + 1) >> 1;
    const bool gact = tid < 128 && gs < ns;
    float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    f4v acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
    XRaw<XK> xr[F32_WG_NX];
    float gvr[8];
    uint32_t gbits = 0;
    auto gload = [&](int rb) {
#pragma unroll
      for (int q = 0; q < F32_WG_NX; ++q) {
        xr[q] = zero_raw8<XK>();
        if (xoff[q] >= 0) {
          const int r = rb + xrow[q];
          if (r < r_end) {
            const int s = r / HoWo;
            const int pos = r - s * HoWo;
            const int oh = pos / g.Wo, ow = pos - oh * g.Wo;
            const long xb = sample_global(p, s, E, PE, 0) * (long)HWC + (long)(oh * g.S * g.Win + ow * g.S) * g.Cin +
                            xoff[q];
            xr[q] = load_raw8<XK>(X, xb);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) gvr[c] = 0.f;
      gbits = 0;
      if (gact) {
        const int r = rb + gr;
        if (r < r_end) {
          const int s = r / HoWo;
          const long gi = sample_global(p, s, E, PE, 0) * HoWo + (r - s * HoWo);
          ld8f(G + gi * 8, gvr);
          gbits = bits[(long)(s0 + gs) * bits_rows + gi];
        }
      }
    };
    gload(r_begin);
    for (int rb = r_begin; rb < r_end; rb += 32) {
      // registers -> LDS (masked G; bias partials accumulate per (row, slot) thread in stage order)
#pragma unroll
      for (int q = 0; q < F32_WG_NX; ++q) {
        if (xsoff[q] >= 0) {
          float v[8];
          raw8_to_f<XK>(xr[q], v);
          st8f(Xs + xsoff[q], v);
        }
      }
      if (tid < 128) {
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = ((gbits >> c) & 1u) ? gvr[c] * g_scale : 0.f;
          bpart[c] += v[c];
        }
        st8f(Gs + gr * GS + gs * 8, v);
      }
      __syncthreads();
      if (rb + 32 < r_end) gload(rb + 32);          // in flight during the MFMAs below
      float bv[8][2];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) bv[j][nt] = Gs[(4 * j + grp) * GS + nt * 16 + i16];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int mt = w + 4 * mi;
        if (mt < nmt) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float av = Xs[(4 * j + grp) * XS + mt * 16 + i16];
            acc[mi][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j][0], acc[mi][0], 0, 0, 0);
            if (nct > 1) acc[mi][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j][1], acc[mi][1], 0, 0, 0);
          }
        }
      }
      __syncthreads();
    }
    // ---- weight partials of this pass's slots (plain stores: this workgroup owns its slab) ----
    const int h = i16 >> 3, ch = l & 7;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mt = w + 4 * mi;
      if (mt < nmt) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int sl = nt * 2 + h;
          if (sl < ns) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = mt * 16 + 4 * grp + r;
              if (k < g.K) pbase[(long)(s0 + sl) * pstride + k * 8 + ch] = acc[mi][nt][r] * in_scale;
            }
          }
        }
      }
    }
    // ---- bias partials: ordered reduction over the 32 row threads of each slot ----
    if (tid < 128) {
#pragma unroll
      for (int c = 0; c < 8; ++c) bred[(gr * 4 + gs) * 8 + c] = bpart[c];
    }
    __syncthreads();
    if (tid < ns * 8) {
      const int a = tid >> 3, c = tid & 7;
      float sacc = 0.f;
      for (int rr = 0; rr < 32; ++rr) sacc += bred[(rr * 4 + a) * 8 + c];
      pbase[(long)(s0 + a) * pstride + K8 + c] = sacc;
    }
    __syncthreads();
  }
}

// grad[w_off + j*chunk + e] (e < K*8) and grad[b_off + j*chunk + c] = sum over module j's (path, slot)
// users in path order, then over row chunks in order.  grid = (ceil((K*8+8)/256), M).
__global__ __launch_bounds__(256) void conv_wgrad_reduce_f32_kernel(
    const float* __restrict__ part, float* __restrict__ grad, long w_off, long b_off, int chunk,
    const int* __restrict__ inv_path, const int* __restrict__ inv_slot, const int* __restrict__ inv_cnt, int layer,
    int M, int Pmax, int K8, int nch) {
  const int j = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= K8 + 8) return;
  const long pstride = (long)K8 + 8;
  const int n = inv_cnt[layer * M + j];
  float s = 0.f;
  for (int u = 0; u < n; ++u) {
    const int p = inv_path[(layer * M + j) * Pmax + u];
    const int a = inv_slot[(layer * M + j) * Pmax + u];
    for (int c = 0; c < nch; ++c) s += part[(((long)p * nch + c) * M + a) * pstride + e];
  }
  if (e < K8) grad[w_off + (long)j * chunk + e] = s;
  else grad[b_off + (long)j * chunk + (e - K8)] = s;
}

// ---------------------------------------------------------------------------
// conv dgrad, fp32 (Cin = Cout = 8).  grid = (ceil(T*E*Hin*Win/256), P), one thread per input pixel.
// dX[sample][ih][iw][ci] = sum_{valid taps} sum_slots sum_c Gm[out][slot][c] W[slot][kh][kw][ci][c].
// Weights sit in LDS as [cnt][tap][c][ci] so each (tap, slot, c) is two broadcast ds_read_b128 for 8 FMAs
// (the generic trunk_bwd.hip kernel reads one float per FMA); valid taps are enumerated directly
// (kh = ih mod S, ih mod S + S, ...), no per-tap divisibility tests; plain stores, fixed order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_dgrad_f32_kernel(
    const float* __restrict__ G, const uint8_t* __restrict__ bits, const float* __restrict__ flat, long w_off,
    int chunk, const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
    ConvGeomF g, int P, int E, int T, long bits_rows, float g_scale, float* __restrict__ dX) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Wl = reinterpret_cast<float*>(smem);   // [cnt][KH*KW][8 c][8 ci]
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x;
  const int ntap = g.KH * g.KW;
  const int per = ntap * 64;
  for (int i = tid; i < cnt * per; i += 256) {
    const int a = i / per, e = i - a * per;
    const int tap = e >> 6, c = (e >> 3) & 7, ci = e & 7;
    const int mod = act_idx[(p * L + layer) * M + a];
    Wl[i] = flat[w_off + (long)mod * chunk + tap * 64 + ci * 8 + c];      // TF layout [kh][kw][ci][c]
  }
  __syncthreads();
  const int HinWin = g.Hin * g.Win, HoWo = g.Ho * g.Wo;
  const int npix = T * E * HinWin;
  const int pix = blockIdx.x * 256 + tid;
  if (pix >= npix) return;
  const int s = pix / HinWin;
  const int ipos = pix - s * HinWin;
  const int ih = ipos / g.Win, iw = ipos - ih * g.Win;
  const long sg = sample_global(p, s, E, P * E, 0);
  float dx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int kh = ih % g.S; kh < g.KH && kh <= ih; kh += g.S) {
    const int oh = (ih - kh) / g.S;
    if (oh >= g.Ho) continue;
    for (int kw = iw % g.S; kw < g.KW && kw <= iw; kw += g.S) {
      const int ow = (iw - kw) / g.S;
      if (ow >= g.Wo) continue;
      const long gi = sg * HoWo + oh * g.Wo + ow;
      float gv[8];
      ld8f(G + gi * 8, gv);
      const int tap = kh * g.KW + kw;
      for (int a = 0; a < cnt; ++a) {
        const uint32_t b = bits[(long)a * bits_rows + gi];
        if (!b) continue;
        const float4* wt = reinterpret_cast<const float4*>(Wl + (a * ntap + tap) * 64);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float gm = ((b >> c) & 1u) ? gv[c] * g_scale : 0.f;
          const float4 w0 = wt[2 * c], w1 = wt[2 * c + 1];
          dx[0] += gm * w0.x; dx[1] += gm * w0.y; dx[2] += gm * w0.z; dx[3] += gm * w0.w;
          dx[4] += gm * w1.x; dx[5] += gm * w1.y; dx[6] += gm * w1.z; dx[7] += gm * w1.w;
        }
      }
    }
  }
  st8f(dX + (sg * HinWin + ipos) * 8, dx);
}

// ---------------------------------------------------------------------------
// fc dgrad.  grid = (ceil(T*E/64), ceil(K/64), P).  dX [T*P*E][K] fp32 (plain stores).
// WcT: [M][KP][Cout] fp32 (n contiguous).  A = ReLU-masked G (fp32, not rounded).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fc_dgrad_f32_kernel(
    const float* __restrict__ G, const uint16_t* __restrict__ bits, const float* __restrict__ WcT,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M, int K, int KP,
    int Cout, int P, int E, int T, long bits_rows, float g_scale, float* __restrict__ dX) {
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * 64 + wr * 32;
  const int col0 = blockIdx.y * 64 + wc * 32;
  if (row0 >= Rtot || col0 >= K) return;
  const int grp = l >> 4, c16 = l & 15;
  long sgr[2];
  bool rv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long r = row0 + i * 16 + c16;
    rv[i] = r < Rtot;
    sgr[i] = sample_global(p, (int)(rv[i] ? r : row0), E, PE, 0);
  }
  f4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { acc[i][0] = {0.f, 0.f, 0.f, 0.f}; acc[i][1] = {0.f, 0.f, 0.f, 0.f}; }
  const int nwords = Cout / 16;
  for (int a = 0; a < cnt; ++a) {
    const int mod = act_idx[(p * L + layer) * M + a];
    const float* Wm = WcT + (long)mod * KP * Cout;
    for (int n0 = 0; n0 < Cout; n0 += 32) {
      const int nb = n0 + 8 * grp;
      float af[2][8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) af[i][c] = 0.f;
        if (rv[i]) {
          float gv[8];
          ld8f(G + sgr[i] * Cout + nb, gv);
          const uint32_t bw = bits[((long)a * bits_rows + sgr[i]) * nwords + (nb >> 4)] >> (nb & 15);
#pragma unroll
          for (int c = 0; c < 8; ++c) af[i][c] = ((bw >> c) & 1u) ? gv[c] * g_scale : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = col0 + j * 16 + c16;
        float bf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (k < KP) ld8f(Wm + (long)k * Cout + nb, bf);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma_f32x8(af[i], bf, acc[i][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + i * 16 + 4 * grp + r;
      if (row < Rtot) {
        const long sg = sample_global(p, (int)row, E, PE, 0);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int k = col0 + j * 16 + c16;
          if (k < K) dX[sg * K + k] = acc[i][j][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------
// fc wgrad, module-major, deterministic.  grid = (ceil(K/64), ceil(Cout/64), M).
// One workgroup owns dW_j[k0b:k0b+64][n0b:n0b+64] and walks the users of module j in path order,
// 32 rows per stage.  Xs/Gs rows of 64 fp32 (+16 pad); D[k][n] += sum_rows X[row][k] Gm[row][n].
// The k-tile-0 workgroups also write db_j from fixed per-thread partials + an ordered LDS sum.
// ---------------------------------------------------------------------------
template <int XK>
__global__ __launch_bounds__(256) void fc_wgrad_f32_kernel(
    const void* __restrict__ X, int ldx, const float* __restrict__ G, const uint16_t* __restrict__ bits,
    float* __restrict__ grad, long w_off, long b_off, int chunk, const int* __restrict__ inv_path,
    const int* __restrict__ inv_slot, const int* __restrict__ inv_cnt, int layer, int M, int Pmax, int K, int Cout,
    int P, int E, int T, long bits_rows, float g_scale) {
  constexpr int S = 64 + 16;
  __shared__ __attribute__((aligned(16))) float Xs[32 * S];
  __shared__ __attribute__((aligned(16))) float Gs[32 * S];
  __shared__ float bred[32 * 64];
  const int j = blockIdx.z;
  const int n_all = inv_cnt[layer * M + j];
  const int k0b = blockIdx.x * 64, n0b = blockIdx.y * 64;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const int nwords = Cout / 16;
  f4v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int srow = tid >> 3, sc = (tid & 7) * 8;
  const int mt0 = 2 * (w >> 1), nt0 = 2 * (w & 1);
  const bool xvec = (ldx % (XK == XBF16 ? 8 : 4) == 0) && (K % 8 == 0);
  for (int u = 0; u < n_all; ++u) {
    const int p = inv_path[(layer * M + j) * Pmax + u];
    const int a = inv_slot[(layer * M + j) * Pmax + u];
    for (long rb = 0; rb < Rtot; rb += 32) {
      const long r = rb + srow;
      float xv[8] = {0, 0, 0, 0, 0, 0, 0, 0}, gv8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < Rtot) {
        const long sg = sample_global(p, (int)r, E, PE, 0);
        const int kx = k0b + sc;
        if (xvec) {
          if (kx < K) load_a8f<XK>(X, sg * ldx + kx, xv);
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (kx + c < K) xv[c] = load_a1f<XK>(X, sg * ldx + kx + c);
        }
        const int n = n0b + sc;
        if (n < Cout) {
          float gg[8];
          ld8f(G + sg * Cout + n, gg);
          const uint32_t bw = bits[((long)a * bits_rows + sg) * nwords + (n >> 4)] >> (n & 15);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            gv8[c] = ((bw >> c) & 1u) ? gg[c] * g_scale : 0.f;
            bpart[c] += gv8[c];
          }
        }
      }
      st8f(Xs + srow * S + sc, xv);
      st8f(Gs + srow * S + sc, gv8);
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int rr = 4 * jj + grp;
        float af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          af[i] = Xs[rr * S + (mt0 + i) * 16 + i16];
          bf[i] = Gs[rr * S + (nt0 + i) * 16 + i16];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jn = 0; jn < 2; ++jn)
            acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[jn], acc[i][jn], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  const long base = w_off + (long)j * chunk;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0b + (mt0 + i) * 16 + 4 * grp + r;
        const int n = n0b + (nt0 + jn) * 16 + i16;
        if (k < K && n < Cout) grad[base + (long)k * Cout + n] = acc[i][jn][r];
      }
  if (blockIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) bred[srow * 64 + sc + c] = bpart[c];
    __syncthreads();
    if (tid < 64 && n0b + tid < Cout) {
      float s = 0.f;
      for (int rr = 0; rr < 32; ++rr) s += bred[rr * 64 + tid];
      grad[b_off + (long)j * chunk + n0b + tid] = s;
    }
  }
}

// fp32 operand copies: Wc[j][c][k] (k contiguous, zero padded to KP) and optionally WcT[j][k][c]
__global__ __launch_bounds__(256) void refresh_weights_f32_kernel(const float* __restrict__ flat, long w_off,
                                                                  int chunk, int K, int KP, int Cout, int M,
                                                                  float* __restrict__ Wc, float* __restrict__ WcT) {
  const long n = (long)M * KP * Cout;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int j = (int)(i / ((long)KP * Cout));
    const int rem = (int)(i - (long)j * KP * Cout);
    const int k = rem / Cout, c = rem - k * Cout;
    const float v = k < K ? flat[w_off + (long)j * chunk + (long)k * Cout + c] : 0.f;
    if (WcT) WcT[i] = v;
    Wc[((long)j * Cout + c) * KP + k] = v;
  }
}

extern "C" {

size_t conv_wgrad_f32_smem(int KP) {
  if (KP <= 0) return 0;
  return (size_t)32 * (KP + 16) * 4 + 32 * F32_WG_GS * 4 + 32 * 4 * 8 * 4 + (KP / 8) * 4;
}

int launch_conv_fwd_f32(const void* X, int u8in, void* Y, void* bits, const void* Wc, const float* flat,
                        long bias_off, int chunk, const int* act_idx, const int* act_cnt, int layer, int L, int M,
                        int Hin, int Win, int Cin, int KH, int KW, int S, int Ho, int Wo, int K, int KP, int P, int E,
                        int T, int t0, long bits_rows, float in_scale, float out_scale, hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      Ho <= 0 || Wo <= 0 || K <= 0 || KP <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 || u8in < 0 ||
      bias_off < 0 || layer < 0 || t0 < 0) return -22;
  if (M > F32_MAXM || KP % 32 != 0 || KP > 512 || (E * Ho * Wo) % 16 != 0 || (KW * Cin) % 8 != 0) return -1;
  ConvGeomF g{Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP};
  constexpr int RT = 2;
  const long rows = (long)T * E * Ho * Wo;
  if (rows >= (1L << 31)) return -1;
  dim3 grid((unsigned)((rows + 64 * RT - 1) / (64 * RT)), P);
#define CF32(U8_, MCT_)                                                                                          \
  conv_fwd_f32_kernel<U8_, RT, MCT_><<<grid, 256, 0, stream>>>(X, (float*)Y, (uint8_t*)bits, (const float*)Wc, flat, \
                                                               bias_off, chunk, act_idx, act_cnt, layer, L, M, g, P, \
                                                               E, T, t0, bits_rows, in_scale, out_scale)
  if (M <= 10) {
    if (u8in) CF32(true, 5); else CF32(false, 5);
  } else {
    if (u8in) CF32(true, 8); else CF32(false, 8);
  }
#undef CF32
  return (int)hipGetLastError();
}

int launch_fc_fwd_f32(const void* X, int ldx, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                      int chunk, const int* act_idx, const int* act_cnt, int layer, int L, int M, int K, int KP,
                      int Cout, int P, int E, int T, int t0, long bits_rows, float out_scale, hipStream_t stream) {
  if (ldx <= 0 || chunk <= 0 || L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      bits_rows <= 0 || bias_off < 0 || layer < 0 || t0 < 0) return -22;
  if (M > F32_MAXM || KP % 32 != 0 || Cout % 32 != 0 || ldx < K) return -1;
  const long rows = (long)T * E;
  if (rows <= 32) {
    dim3 grid((unsigned)((rows + 31) / 32), (Cout + 63) / 64, P);
    fc_fwd_f32_kernel<32><<<grid, 256, 0, stream>>>((const float*)X, ldx, (float*)Y, (uint16_t*)bits,
                                                    (const float*)Wc, flat, bias_off, chunk, act_idx, act_cnt, layer,
                                                    L, M, K, KP, Cout, P, E, T, t0, bits_rows, out_scale);
  } else {
    dim3 grid((unsigned)((rows + 63) / 64), (Cout + 63) / 64, P);
    fc_fwd_f32_kernel<64><<<grid, 256, 0, stream>>>((const float*)X, ldx, (float*)Y, (uint16_t*)bits,
                                                    (const float*)Wc, flat, bias_off, chunk, act_idx, act_cnt, layer,
                                                    L, M, K, KP, Cout, P, E, T, t0, bits_rows, out_scale);
  }
  return (int)hipGetLastError();
}

// part: scratch of P * nch * M * (K*8 + 8) floats (conv_wgrad_f32_part_numel); the reduce writes every
// weight and bias element of the layer (modules without users get 0).
long conv_wgrad_f32_part_numel(int P, int nch, int M, int K) { return (long)P * nch * M * ((long)K * 8 + 8); }

// xkind: 0 uint8 frames, 1 bf16 activations (bf16 engine, deterministic mode), 2 fp32 activations
int launch_conv_wgrad_f32(const void* X, int xkind, const float* G, const void* bits, float* grad, float* part,
                          long w_off, long b_off, int chunk, const int* act_idx, const int* act_cnt,
                          const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int L, int M,
                          int Pmax, int Hin, int Win, int Cin, int KH, int KW, int S, int Ho, int Wo, int K, int KP,
                          int P, int E, int T, long bits_rows, int nch, float in_scale, float g_scale,
                          hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Pmax <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 ||
      S <= 0 || Ho <= 0 || Wo <= 0 || K <= 0 || KP <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 ||
      nch <= 0 || xkind < 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (M > F32_MAXM || KP % 32 != 0 || KP > 256 || nch < 1 || (KW * Cin) % 8 != 0) return -1;
  if ((long)T * E * Ho * Wo >= (1L << 31)) return -1;
  ConvGeomF g{Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP};
  const long rows = (long)T * E * Ho * Wo;
  int rpc = (int)((rows + nch - 1) / nch);
  rpc = (rpc + 31) / 32 * 32;
  const int nch_eff = (int)((rows + rpc - 1) / rpc);
  if (nch_eff != nch) return -3;      // the host sizes part / the reduce for exactly nch chunks
  dim3 grid((unsigned)nch, P);
  const size_t sm = conv_wgrad_f32_smem(KP);
#define CW32(XK_)                                                                                             \
  conv_wgrad_f32_kernel<XK_><<<grid, 256, sm, stream>>>(X, G, (const uint8_t*)bits, part, act_idx, act_cnt, layer, L, \
                                                        M, g, P, E, T, bits_rows, rpc, in_scale, g_scale)
  if (xkind == XU8) CW32(XU8);
  else if (xkind == XBF16) CW32(XBF16);
  else if (xkind == XF32) CW32(XF32);
  else return -1;
#undef CW32
  const int K8 = K * 8;
  dim3 rgrid((unsigned)((K8 + 8 + 255) / 256), M);
  conv_wgrad_reduce_f32_kernel<<<rgrid, 256, 0, stream>>>(part, grad, w_off, b_off, chunk, inv_path, inv_slot,
                                                          inv_cnt, layer, M, Pmax, K8, nch);
  return (int)hipGetLastError();
}

int launch_conv_dgrad_f32(const float* G, const void* bits, const float* flat, long w_off, int chunk,
                          const int* act_idx, const int* act_cnt, int layer, int L, int M, int Hin, int Win, int Cin,
                          int KH, int KW, int S, int Ho, int Wo, int P, int E, int T, long bits_rows, float g_scale,
                          float* dX, hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      Ho <= 0 || Wo <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 || w_off < 0 || layer < 0) return -22;
  if (Cin != 8 || M > F32_MAXM) return -1;
  const long npix = (long)T * E * Hin * Win;
  if (npix >= (1L << 31)) return -1;
  ConvGeomF g{Hin, Win, Cin, KH, KW, S, Ho, Wo, KH * KW * Cin, 0};
  dim3 grid((unsigned)((npix + 255) / 256), P);
  const size_t sm = (size_t)M * KH * KW * 64 * 4;
  if (sm > 160 * 1024) return -2;
  conv_dgrad_f32_kernel<<<grid, 256, sm, stream>>>(G, (const uint8_t*)bits, flat, w_off, chunk, act_idx, act_cnt,
                                                   layer, L, M, g, P, E, T, bits_rows, g_scale, dX);
  return (int)hipGetLastError();
}

int launch_fc_dgrad_f32(const float* G, const void* bits, const void* WcT, const int* act_idx, const int* act_cnt,
                        int layer, int L, int M, int K, int KP, int Cout, int P, int E, int T, long bits_rows,
                        float g_scale, float* dX, hipStream_t stream) {
  if (L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 ||
      layer < 0) return -22;
  if (M > F32_MAXM || Cout % 32 != 0) return -1;
  dim3 grid((unsigned)(((long)T * E + 63) / 64), (K + 63) / 64, P);
  fc_dgrad_f32_kernel<<<grid, 256, 0, stream>>>(G, (const uint16_t*)bits, (const float*)WcT, act_idx, act_cnt, layer,
                                                L, M, K, KP, Cout, P, E, T, bits_rows, g_scale, dX);
  return (int)hipGetLastError();
}

int launch_fc_wgrad_f32(const void* X, int xkind, int ldx, const float* G, const void* bits, float* grad, long w_off, long b_off,
                        int chunk, const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int M,
                        int Pmax, int K, int Cout, int P, int E, int T, long bits_rows, float g_scale,
                        hipStream_t stream) {
  if (ldx <= 0 || chunk <= 0 || M <= 0 || Pmax <= 0 || K <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      bits_rows <= 0 || xkind < 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (Cout % 16 != 0 || ldx < K || (xkind != XBF16 && xkind != XF32)) return -1;
  dim3 grid((K + 63) / 64, (Cout + 63) / 64, M);
  if (xkind == XBF16)
    fc_wgrad_f32_kernel<XBF16><<<grid, 256, 0, stream>>>(X, ldx, G, (const uint16_t*)bits, grad, w_off, b_off, chunk,
                                                         inv_path, inv_slot, inv_cnt, layer, M, Pmax, K, Cout, P, E,
                                                         T, bits_rows, g_scale);
  else
    fc_wgrad_f32_kernel<XF32><<<grid, 256, 0, stream>>>(X, ldx, G, (const uint16_t*)bits, grad, w_off, b_off, chunk,
                                                        inv_path, inv_slot, inv_cnt, layer, M, Pmax, K, Cout, P, E, T,
                                                        bits_rows, g_scale);
  return (int)hipGetLastError();
}

int launch_refresh_weights_f32(const float* flat, long w_off, int chunk, int K, int KP, int Cout, int M, void* Wc,
                               void* WcT, hipStream_t stream) {
  if (chunk <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || M <= 0 || w_off < 0) return -22;
  const long n = (long)M * KP * Cout;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  refresh_weights_f32_kernel<<<blocks, 256, 0, stream>>>(flat, w_off, chunk, K, KP, Cout, M, (float*)Wc,
                                                         (float*)WcT);
  return (int)hipGetLastError();
}
}
