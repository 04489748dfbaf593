// Compile-time-geometry conv kernels for the standard PathNet pixel trunk
// (160x120x4 input, kernels 8/4/3, strides 4/2/1: game_ac_network.py:376,
// doom_pathnet.py:356-358).  Same math and buffer layouts as the generic
// kernels in trunk_fwd.hip / trunk_bwd.hip (those remain the fallback for
// other shapes); these add:
//   fwd  : LDS weights staged ONCE per 256-row workgroup, 32-row wave tiles
//          sharing each B fragment (half the LDS traffic), fully unrolled k.
//   wgrad: 64-row stages (2 MFMA k-steps per barrier pair), per-row address
//          table in LDS, bias grads in registers, ~4K workgroups.
//   dgrad: one workgroup = one stride-parity class of input pixels, so the
//          tap set and every weight index are wave-uniform -> weights come
//          through the scalar cache (s_load) and feed v_fma as SGPR operands.
#include "common.h"

#define NCT 5            // column-tile capacity: 10 modules x 8 maps (M <= 10)
#define MAXM_F 16

template <int HIN_, int WIN_, int CIN_, int KH_, int KW_, int S_, bool U8_>
struct CG {
  static constexpr int HIN = HIN_, WIN = WIN_, CIN = CIN_, KH = KH_, KW = KW_, S = S_;
  static constexpr bool U8 = U8_;
  static constexpr int HO = (HIN - KH) / S + 1, WO = (WIN - KW) / S + 1, HOWO = HO * WO;
  static constexpr int K = KH * KW * CIN, KP = (K + 31) / 32 * 32, KC = KP / 8;
  static constexpr int IN_ELEMS = HIN * WIN * CIN;
  static constexpr __host__ __device__ int koff(int kc) {
    return kc * 8 >= K ? -1
                       : ((kc * 8 / CIN) / KW * WIN + (kc * 8 / CIN) % KW) * CIN + (kc * 8) % CIN;
  }
};
using C1 = CG<160, 120, 4, 8, 8, 4, true>;
using C2 = CG<39, 29, 8, 4, 4, 2, false>;
using C3 = CG<18, 13, 8, 3, 3, 1, false>;

template <bool U8IN>
DEVI s8v ld8(const void* X, long off) {
  s8v r;
  if constexpr (U8IN) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + off);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j] = (short)(__float_as_uint((float)((v.x >> (8 * j)) & 0xFFu)) >> 16);
      r[j + 4] = (short)(__float_as_uint((float)((v.y >> (8 * j)) & 0xFFu)) >> 16);
    }
  } else {
    r = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + off);
  }
  return r;
}

// ===========================================================================
// forward: grid = (ceil(T*E*HOWO / 256), P); each wave loops over 32-row tiles
// ===========================================================================
#define FF_ROWS 256
template <class G>
__global__ __launch_bounds__(256) void conv_fwd_fast(const void* __restrict__ X, bf16_t* __restrict__ Y,
                                                     uint8_t* __restrict__ bits, const bf16_t* __restrict__ Wc,
                                                     const float* __restrict__ flat, long bias_off, int chunk,
                                                     const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                     int layer, int L, int M, int P, int E, int T, int t0,
                                                     long bits_rows, float in_scale, float out_scale) {
  constexpr int KPs = G::KP + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Ws[NCT * 16 * KPs];
  __shared__ float bias_s[NCT * 16];
  __shared__ int mods[MAXM_F];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  __syncthreads();
  for (int i = tid; i < nct * 16 * G::KC; i += 256) {
    const int col = i / G::KC, kc = i - col * G::KC;
    const int slot = col >> 3;
    s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (slot < cnt) v = *reinterpret_cast<const s8v*>(Wc + ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8);
    *reinterpret_cast<s8v*>(Ws + col * KPs + kc * 8) = v;
  }
  if (tid < NCT * 16) bias_s[tid] = (tid >> 3) < cnt ? flat[bias_off + (long)mods[tid >> 3] * chunk + (tid & 7)] : 0.f;
  __syncthreads();

  const long Rtot = (long)T * E * G::HOWO;
  const int PE = P * E;
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
  for (int tile = 0; tile < FF_ROWS / 128; ++tile) {
    const long rbase = (long)blockIdx.x * FF_ROWS + tile * 128 + w * 32;
    if (rbase >= Rtot) break;
    long xb[2];
    bool va[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long ra = rbase + i * 16 + c16;
      va[i] = ra < Rtot;
      const long rr = va[i] ? ra : rbase;
      const int s = (int)(rr / G::HOWO);
      const int pos = (int)(rr - (long)s * G::HOWO);
      const int oh = pos / G::WO, ow = pos - oh * G::WO;
      xb[i] = sample_global(p, s, E, PE, t0) * (long)G::IN_ELEMS + (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN;
    }
    f4v acc[2][NCT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < G::KP / 32; ++kk) {
      const int kc = kk * 4 + grp;
      const int off = G::koff(kc);     // grp-dependent: computed per lane from a constexpr table
      s8v a[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
        if (va[i] && off >= 0) a[i] = ld8<G::U8>(X, xb[i] + off);
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        if (ct < nct) {
          const s8v b = *reinterpret_cast<const s8v*>(Ws + (ct * 16 + c16) * KPs + kc * 8);
          acc[0][ct] = mfma16(a[0], b, acc[0][ct]);
          acc[1][ct] = mfma16(a[1], b, acc[1][ct]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long r16 = rbase + i * 16;
      if (r16 >= Rtot) break;
      float sum[4] = {0.f, 0.f, 0.f, 0.f};
      long grow4;
      {
        const long r4 = r16 + 4 * q;
        const int s = (int)(r4 / G::HOWO);
        const int pos = (int)(r4 - (long)s * G::HOWO);
        grow4 = sample_global(p, s, E, PE, t0) * G::HOWO + pos;
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        if (ct < nct) {
          const int slot = ct * 2 + h;
          const bool sv = slot < cnt;
          const float bb = bias_s[ct * 16 + c16];
          uint32_t word = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[i][ct][r] * in_scale + bb;
            const bool pos = sv && v > 0.f;
            sum[r] += pos ? v : 0.f;
            const uint64_t bal = __ballot(pos);
            word |= (uint32_t)((bal >> (16 * q + 8 * h)) & 0xFFull) << (8 * r);
          }
          if (ch == 0 && sv) *reinterpret_cast<uint32_t*>(bits + (long)slot * bits_rows + grow4) = word;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
      // pack: lanes c16 0..7 hold maps 0..7 of rows 4q+r -> gather 8 bf16 into lane c16==0 per row
      if (h == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = r16 + 4 * q + r;
          const int s = (int)(row / G::HOWO);
          const int pos = (int)(row - (long)s * G::HOWO);
          Y[(sample_global(p, s, E, PE, t0) * G::HOWO + pos) * 8 + ch] = f2bf(sum[r] * out_scale);
        }
      }
    }
  }
}

// ===========================================================================
// wgrad: grid = (nchunks, P); 64-row stages
// ===========================================================================
#define WG_RB 64
template <class G>
__global__ __launch_bounds__(256) void conv_wgrad_fast(const void* __restrict__ X, const float* __restrict__ Gr,
                                                       const uint8_t* __restrict__ bits, float* __restrict__ grad,
                                                       long w_off, long b_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M,
                                                       int P, int E, int T, long bits_rows, int rows_per_chunk,
                                                       float in_scale, float g_scale) {
  constexpr int XS = G::KP + 8;
  constexpr int GS = NCT * 16 + 8;
  constexpr int NMT = G::KP / 16;
  constexpr int MPW = (NMT + 3) / 4;   // m tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t Xs[WG_RB * XS];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[WG_RB * GS];
  __shared__ long rowx[WG_RB];
  __shared__ long rowg[WG_RB];
  __shared__ float dbias[NCT * 16];
  __shared__ int mods[MAXM_F];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < NCT * 16) dbias[tid] = 0.f;
  for (int i = tid; i < WG_RB * GS; i += 256) Gs[i] = 0;
  const long Rtot = (long)T * E * G::HOWO;
  const int PE = P * E;
  const long r_begin = (long)blockIdx.x * rows_per_chunk;
  const long r_end = min(Rtot, r_begin + rows_per_chunk);
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  // G staging role: fixed slot per thread
  const int gslot = tid & 15, grow0 = tid >> 4;          // rows grow0 + 16*i
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  f4v acc[MPW][NCT];
#pragma unroll
  for (int a = 0; a < MPW; ++a)
#pragma unroll
    for (int b = 0; b < NCT; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (long rb = r_begin; rb < r_end; rb += WG_RB) {
    if (tid < WG_RB) {
      const long r = rb + tid;
      long xo = -1, go = -1;
      if (r < r_end) {
        const int s = (int)(r / G::HOWO);
        const int pos = (int)(r - (long)s * G::HOWO);
        const int oh = pos / G::WO, ow = pos - oh * G::WO;
        const long sg = sample_global(p, s, E, PE, 0);
        xo = sg * (long)G::IN_ELEMS + (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN;
        go = sg * G::HOWO + pos;
      }
      rowx[tid] = xo;
      rowg[tid] = go;
    }
    __syncthreads();
    // X tile
#pragma unroll
    for (int it0 = 0; it0 < WG_RB * G::KC; it0 += 256) {
      const int it = it0 + tid;
      if (it < WG_RB * G::KC) {
        const int row = it / G::KC, kc = it - row * G::KC;
        const long xo = rowx[row];
        const int off = G::koff(kc);
        s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (xo >= 0 && off >= 0) v = ld8<G::U8>(X, xo + off);
        *reinterpret_cast<s8v*>(Xs + row * XS + kc * 8) = v;
      }
    }
    // masked G tile: thread = (slot gslot, rows grow0 + 16 i)
    if (gslot < cnt) {
#pragma unroll
      for (int i = 0; i < WG_RB / 16; ++i) {
        const int row = grow0 + 16 * i;
        const long go = rowg[row];
        s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (go >= 0) {
          const float4 g0 = *reinterpret_cast<const float4*>(Gr + go * 8);
          const float4 g1 = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
          const uint32_t b = bits[(long)gslot * bits_rows + go];
          const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float x = ((b >> c) & 1u) ? gv[c] * g_scale : 0.f;
            bpart[c] += x;
            v[c] = (short)f2bf(x);
          }
        }
        *reinterpret_cast<s8v*>(Gs + row * GS + gslot * 8) = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < WG_RB / 32; ++ks) {
      s8v bfr[NCT];
#pragma unroll
      for (int nt = 0; nt < NCT; ++nt) {
        if (nt < nct) {
          const s4v v0 = lds_tr16(Gs + (32 * ks + 8 * grp + q) * GS + nt * 16 + 4 * pp);
          const s4v v1 = lds_tr16(Gs + (32 * ks + 8 * grp + 4 + q) * GS + nt * 16 + 4 * pp);
          bfr[nt] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        }
      }
#pragma unroll
      for (int mi = 0; mi < MPW; ++mi) {
        const int mt = w + 4 * mi;
        if (mt < NMT) {
          const s4v v0 = lds_tr16(Xs + (32 * ks + 8 * grp + q) * XS + mt * 16 + 4 * pp);
          const s4v v1 = lds_tr16(Xs + (32 * ks + 8 * grp + 4 + q) * XS + mt * 16 + 4 * pp);
          const s8v afr = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
          for (int nt = 0; nt < NCT; ++nt)
            if (nt < nct) acc[mi][nt] = mfma16(afr, bfr[nt], acc[mi][nt]);
        }
      }
    }
    __syncthreads();
  }
  const int h = i16 >> 3, ch = l & 7;
#pragma unroll
  for (int mi = 0; mi < MPW; ++mi) {
    const int mt = w + 4 * mi;
    if (mt < NMT) {
#pragma unroll
      for (int nt = 0; nt < NCT; ++nt) {
        if (nt < nct) {
          const int slot = nt * 2 + h;
          if (slot < cnt) {
            const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = mt * 16 + 4 * grp + r;
              if (k < G::K) atomicAdd(&grad[base + (long)k * 8 + ch], acc[mi][nt][r] * in_scale);
            }
          }
        }
      }
    }
  }
  if (gslot < cnt) {
#pragma unroll
    for (int c = 0; c < 8; ++c) atomicAdd(&dbias[gslot * 8 + c], bpart[c]);
  }
  __syncthreads();
  if (tid < cnt * 8) atomicAdd(&grad[b_off + (long)mods[tid >> 3] * chunk + (tid & 7)], dbias[tid]);
}

// ===========================================================================
// dgrad (Cin = Cout = 8): grid = (ceil(T*E*NI*NJ/256), S*S, P), class (ph,pw) = blockIdx.y
// ===========================================================================
template <class G>
__global__ __launch_bounds__(256) void conv_dgrad_fast(const float* __restrict__ Gr, const uint8_t* __restrict__ bits,
                                                       const float* __restrict__ flat, long w_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M,
                                                       int P, int E, int T, long bits_rows, float g_scale,
                                                       float* __restrict__ dX) {
  constexpr int S = G::S;
  const int cls = blockIdx.y;
  const int ph = cls / S, pw = cls - ph * S;
  const int NI = (G::HIN - ph + S - 1) / S, NJ = (G::WIN - pw + S - 1) / S;
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const long npix = (long)T * E * NI * NJ;
  const long pix = (long)blockIdx.x * 256 + threadIdx.x;
  if ((long)blockIdx.x * 256 >= npix) return;
  const bool valid = pix < npix;
  const long pixc = valid ? pix : 0;
  const int s = (int)(pixc / (NI * NJ));
  const int rem = (int)(pixc - (long)s * NI * NJ);
  const int i = rem / NJ, j = rem - i * NJ;
  const int ih = ph + S * i, iw = pw + S * j;
  const long sg = sample_global(p, s, E, P * E, 0);
  float dx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int NA = (G::KH + S - 1) / S, NB = (G::KW + S - 1) / S;
#pragma unroll
  for (int ta = 0; ta < NA; ++ta) {
    const int kh = ph + S * ta;            // wave-uniform
    if (kh >= G::KH) continue;
    const int oh = i - ta;
#pragma unroll
    for (int tb = 0; tb < NB; ++tb) {
      const int kw = pw + S * tb;
      if (kw >= G::KW) continue;
      const int ow = j - tb;
      const bool ok = valid && oh >= 0 && oh < G::HO && ow >= 0 && ow < G::WO;
      const long gi = sg * G::HOWO + (ok ? oh * G::WO + ow : 0);
      float gv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) {
        const float4 g0 = *reinterpret_cast<const float4*>(Gr + gi * 8);
        const float4 g1 = *reinterpret_cast<const float4*>(Gr + gi * 8 + 4);
        gv[0] = g0.x * g_scale; gv[1] = g0.y * g_scale; gv[2] = g0.z * g_scale; gv[3] = g0.w * g_scale;
        gv[4] = g1.x * g_scale; gv[5] = g1.y * g_scale; gv[6] = g1.z * g_scale; gv[7] = g1.w * g_scale;
      }
      const int tap = kh * G::KW + kw;
      for (int a = 0; a < cnt; ++a) {
        const int mod = act_idx[(p * L + layer) * M + a];        // uniform -> scalar load
        const uint32_t b = ok ? bits[(long)a * bits_rows + gi] : 0u;
        const float* wt = flat + w_off + (long)mod * chunk + tap * 64;   // uniform address
        float gm[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) gm[c] = ((b >> c) & 1u) ? gv[c] : 0.f;
#pragma unroll
        for (int ci = 0; ci < 8; ++ci)
#pragma unroll
          for (int c = 0; c < 8; ++c) dx[ci] += gm[c] * wt[ci * 8 + c];
      }
    }
  }
  if (valid) {
    float4* o = reinterpret_cast<float4*>(dX + (sg * (G::HIN * G::WIN) + ih * G::WIN + iw) * 8);
    o[0] = make_float4(dx[0], dx[1], dx[2], dx[3]);
    o[1] = make_float4(dx[4], dx[5], dx[6], dx[7]);
  }
}

// ---------------------------------------------------------------------------
template <class G>
static int fwd_t(const void* X, void* Y, void* bits, const void* Wc, const float* flat, long bias_off, int chunk,
                 const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, int t0, long br,
                 float is, float os, hipStream_t st) {
  const long rows = (long)T * E * G::HOWO;
  dim3 grid((unsigned)((rows + FF_ROWS - 1) / FF_ROWS), P);
  conv_fwd_fast<G><<<grid, 256, 0, st>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat, bias_off, chunk, ai,
                                         ac, layer, L, M, P, E, T, t0, br, is, os);
  return (int)hipGetLastError();
}

template <class G>
static int wgrad_t(const void* X, const float* Gr, const void* bits, float* grad, long w_off, long b_off, int chunk,
                   const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, long br, float is,
                   float gs, hipStream_t st) {
  const long rows = (long)T * E * G::HOWO;
  // ~64 chunks per path (>= 16 workgroups per CU at P=64) in whole 64-row stages
  long rpc = (rows + 63) / 64;
  rpc = (rpc + WG_RB - 1) / WG_RB * WG_RB;
  if (rpc < WG_RB * 4) rpc = WG_RB * 4;
  dim3 grid((unsigned)((rows + rpc - 1) / rpc), P);
  conv_wgrad_fast<G><<<grid, 256, 0, st>>>(X, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai, ac, layer, L,
                                           M, P, E, T, br, (int)rpc, is, gs);
  return (int)hipGetLastError();
}

template <class G>
static int dgrad_t(const float* Gr, const void* bits, const float* flat, long w_off, int chunk, const int* ai,
                   const int* ac, int layer, int L, int M, int P, int E, int T, long br, float gs, float* dX,
                   hipStream_t st) {
  constexpr int S = G::S;
  const int NI = (G::HIN + S - 1) / S, NJ = (G::WIN + S - 1) / S;    // largest class
  const long npix = (long)T * E * NI * NJ;
  dim3 grid((unsigned)((npix + 255) / 256), S * S, P);
  conv_dgrad_fast<G><<<grid, 256, 0, st>>>(Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E,
                                           T, br, gs, dX);
  return (int)hipGetLastError();
}

template <class G>
static bool is_shape(int Hin, int Win, int Cin, int KH, int KW, int S, int u8) {
  return Hin == G::HIN && Win == G::WIN && Cin == G::CIN && KH == G::KH && KW == G::KW && S == G::S &&
         (u8 != 0) == G::U8;
}

extern "C" {
// return 1 if handled by a fast kernel, 0 if the shape is not specialised, <0 on error
int fast_conv_fwd(const void* X, int u8in, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                  int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH,
                  int KW, int S, int P, int E, int T, int t0, long br, float is, float os, hipStream_t st) {
  if (M > 2 * NCT) return 0;
#define FWD(Gx)                                                                                              \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, u8in)) {                                                        \
    if ((E * Gx::HOWO) % 16) return -2;                                                                      \
    const int rc = fwd_t<Gx>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st); \
    return rc ? -rc : 1;                                                                                     \
  }
  FWD(C1) FWD(C2) FWD(C3)
#undef FWD
  return 0;
}

int fast_conv_wgrad(const void* X, int u8in, const float* Gr, const void* bits, float* grad, long w_off, long b_off,
                    int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win, int Cin,
                    int KH, int KW, int S, int P, int E, int T, long br, float is, float gs, hipStream_t st) {
  if (M > 2 * NCT) return 0;
#define WG(Gx)                                                                                                 \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, u8in)) {                                                          \
    const int rc = wgrad_t<Gx>(X, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is, gs, st); \
    return rc ? -rc : 1;                                                                                       \
  }
  WG(C1) WG(C2) WG(C3)
#undef WG
  return 0;
}

int fast_conv_dgrad(const float* Gr, const void* bits, const float* flat, long w_off, int chunk, const int* ai,
                    const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH, int KW, int S, int P,
                    int E, int T, long br, float gs, float* dX, hipStream_t st) {
#define DG(Gx)                                                                                          \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, 0)) {                                                      \
    const int rc = dgrad_t<Gx>(Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, st); \
    return rc ? -rc : 1;                                                                                \
  }
  DG(C2) DG(C3)
#undef DG
  return 0;
}
}
