// PathNet trunk backward on CDNA4.
//
// Gradient flows ONLY through active modules (the reference gets the same
// effect from mask=0 multiplications, game_ac_network.py:188,386): a module
// slot's local gradient is Gm = G (grad of the layer-sum output) masked by the
// ReLU bits saved in the forward epilogue.
//
//   conv_wgrad : path-major; LDS-staged im2col rows + masked G, both read with
//                ds_read_b64_tr_b16 so the reduction (row) index lands in the
//                MFMA k-slot; fp32 atomics combine paths sharing a module.
//   conv_dgrad : transposed conv as a per-input-pixel gather (VALU, LDS weights).
//   fc_wgrad   : MODULE-major (no atomics): one workgroup owns a 64x64 tile of
//                dW_j and walks every (path, slot) that uses module j.
//   fc_dgrad   : grouped GEMM dX = sum_a Gm_a W_a^T over active slots (MFMA).
#include "common.h"

#define MAXM 16

struct ConvGeomB {
  int Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP;
};

// ---------------------------------------------------------------------------
// conv wgrad.  grid = (nchunks, P), block 256, chunk = rows_per_chunk (mult of 32)
// ---------------------------------------------------------------------------
template <bool U8IN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(
    const void* __restrict__ X, const float* __restrict__ G, const uint8_t* __restrict__ bits,
    float* __restrict__ grad, long w_off, long b_off, int chunk, const int* __restrict__ act_idx,
    const int* __restrict__ act_cnt, int layer, int L, int M, ConvGeomB g, int P, int E, int T,
    long bits_rows, int rows_per_chunk, float in_scale, float g_scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int ncol = nct * 16;
  const int XS = g.KP + 8;            // Xs row stride (elements)
  const int GS = 16 * 8 + 8;          // Gs row stride: capacity 8 col tiles (16 modules)
  bf16_t* Xs = reinterpret_cast<bf16_t*>(smem);                  // [32][XS]
  bf16_t* Gs = Xs + 32 * XS;                                      // [32][GS]
  float* dbias = reinterpret_cast<float*>(Gs + 32 * GS);          // [128]
  int* koff = reinterpret_cast<int*>(dbias + 128);                // [KP/8]
  int* mods = koff + g.KP / 8;                                    // [MAXM]
  const int tid = threadIdx.x;
  if (tid < MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < 128) dbias[tid] = 0.f;
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
  // zero the padded G columns once
  for (int i = tid; i < 32 * GS; i += 256) Gs[i] = 0;
  __syncthreads();

  const int HoWo = g.Ho * g.Wo;
  const long Rtot = (long)T * E * HoWo;
  const int PE = P * E;
  const long r_begin = (long)blockIdx.x * rows_per_chunk;
  const long r_end = min(Rtot, r_begin + rows_per_chunk);
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int nmt = g.KP / 16;         // m tiles over k
  const int kvec = g.KP / 8;

  f4v acc[4][MAXM / 2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < MAXM / 2; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};

  for (long rb = r_begin; rb < r_end; rb += 32) {
    // ---- stage X (im2col rows) ----
    for (int it = tid; it < 32 * kvec; it += 256) {
      const int row = it / kvec, kc = it - row * kvec;
      const long r = rb + row;
      s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
      const int off = koff[kc];
      if (r < r_end && off >= 0) {
        const int s = (int)(r / HoWo);
        const int pos = (int)(r - (long)s * HoWo);
        const int oh = pos / g.Wo, ow = pos - oh * g.Wo;
        const long sg = sample_global(p, s, E, PE, 0);
        const long xb = sg * (long)(g.Hin * g.Win * g.Cin) + (long)(oh * g.S * g.Win + ow * g.S) * g.Cin + off;
        if constexpr (U8IN) {
          const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xb);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = (short)(__float_as_uint((float)((u.x >> (8 * j)) & 0xFFu)) >> 16);
            v[j + 4] = (short)(__float_as_uint((float)((u.y >> (8 * j)) & 0xFFu)) >> 16);
          }
        } else {
          v = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xb);
        }
      }
      *reinterpret_cast<s8v*>(Xs + row * XS + kc * 8) = v;
    }
    // ---- stage masked G: item = (row, slot) ----
    for (int it = tid; it < 32 * cnt; it += 256) {
      const int row = it / cnt, a = it - row * cnt;
      const long r = rb + row;
      s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < r_end) {
        const int s = (int)(r / HoWo);
        const int pos = (int)(r - (long)s * HoWo);
        const long sg = sample_global(p, s, E, PE, 0);
        const long gi = (sg * HoWo + pos);
        const float4 g0 = *reinterpret_cast<const float4*>(G + gi * 8);
        const float4 g1 = *reinterpret_cast<const float4*>(G + gi * 8 + 4);
        const uint32_t b = bits[(long)a * bits_rows + gi];
        float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float x = ((b >> c) & 1u) ? gv[c] * g_scale : 0.f;
          v[c] = (short)f2bf(x);
          if (x != 0.f) atomicAdd(&dbias[a * 8 + c], x);
        }
      }
      *reinterpret_cast<s8v*>(Gs + row * GS + a * 8) = v;
    }
    __syncthreads();
    // ---- MFMA: acc[m-tile][n-tile] += Xs^T(m) * Gs(n) over the 32 rows ----
    s8v bfr[MAXM / 2];
#pragma unroll
    for (int nt = 0; nt < MAXM / 2; ++nt) {
      if (nt < nct) {
        const s4v v0 = lds_tr16(Gs + (8 * grp + q) * GS + nt * 16 + 4 * pp);
        const s4v v1 = lds_tr16(Gs + (8 * grp + 4 + q) * GS + nt * 16 + 4 * pp);
        bfr[nt] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mt = w + 4 * mi;
      if (mt < nmt) {
        const s4v v0 = lds_tr16(Xs + (8 * grp + q) * XS + mt * 16 + 4 * pp);
        const s4v v1 = lds_tr16(Xs + (8 * grp + 4 + q) * XS + mt * 16 + 4 * pp);
        const s8v afr = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int nt = 0; nt < MAXM / 2; ++nt)
          if (nt < nct) acc[mi][nt] = mfma16(afr, bfr[nt], acc[mi][nt]);
      }
    }
    __syncthreads();
  }
  // ---- epilogue: atomics into the flat gradient ----
  const int h = i16 >> 3, ch = l & 7;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int mt = w + 4 * mi;
    if (mt < nmt) {
#pragma unroll
      for (int nt = 0; nt < MAXM / 2; ++nt) {
        if (nt < nct) {
          const int slot = nt * 2 + h;
          if (slot < cnt) {
            const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = mt * 16 + 4 * grp + r;
              if (k < g.K) atomicAdd(&grad[base + (long)k * 8 + ch], acc[mi][nt][r] * in_scale);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (tid < cnt * 8) atomicAdd(&grad[b_off + (long)mods[tid >> 3] * chunk + (tid & 7)], dbias[tid]);
}

// ---------------------------------------------------------------------------
// conv dgrad (Cin = Cout = 8).  grid = (ceil(T*E*Hin*Win/256), P)
// dX[sample][ih][iw][ci] = sum_{valid taps} sum_slots sum_c Gm[out][slot][c] W[slot][kh][kw][ci][c]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_dgrad_kernel(
    const float* __restrict__ G, const uint8_t* __restrict__ bits, const float* __restrict__ flat, long w_off,
    int chunk, const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
    ConvGeomB g, int P, int E, int T, long bits_rows, float g_scale, float* __restrict__ dX) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Wl = reinterpret_cast<float*>(smem);   // [cnt][KH*KW][8 ci][8 c]
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x;
  const int per = g.KH * g.KW * 64;
  for (int i = tid; i < cnt * per; i += 256) {
    const int a = i / per, e = i - a * per;
    const int mod = act_idx[(p * L + layer) * M + a];
    Wl[i] = flat[w_off + (long)mod * chunk + e];      // TF layout [kh][kw][ci][c] == e
  }
  __syncthreads();
  const int HinWin = g.Hin * g.Win, HoWo = g.Ho * g.Wo;
  const long npix = (long)T * E * HinWin;
  const long pix = (long)blockIdx.x * 256 + tid;
  if (pix >= npix) return;
  const int s = (int)(pix / HinWin);
  const int ipos = (int)(pix - (long)s * HinWin);
  const int ih = ipos / g.Win, iw = ipos - ih * g.Win;
  const long sg = sample_global(p, s, E, P * E, 0);
  float dx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int kh = 0; kh < g.KH; ++kh) {
    const int th = ih - kh;
    if (th < 0 || th % g.S) continue;
    const int oh = th / g.S;
    if (oh >= g.Ho) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int tw = iw - kw;
      if (tw < 0 || tw % g.S) continue;
      const int ow = tw / g.S;
      if (ow >= g.Wo) continue;
      const long gi = sg * HoWo + oh * g.Wo + ow;
      const float4 g0 = *reinterpret_cast<const float4*>(G + gi * 8);
      const float4 g1 = *reinterpret_cast<const float4*>(G + gi * 8 + 4);
      const float gv[8] = {g0.x * g_scale, g0.y * g_scale, g0.z * g_scale, g0.w * g_scale,
                           g1.x * g_scale, g1.y * g_scale, g1.z * g_scale, g1.w * g_scale};
      const int tap = kh * g.KW + kw;
      for (int a = 0; a < cnt; ++a) {
        const uint32_t b = bits[(long)a * bits_rows + gi];
        if (!b) continue;
        const float* wt = Wl + (a * g.KH * g.KW + tap) * 64;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float gm = ((b >> c) & 1u) ? gv[c] : 0.f;
#pragma unroll
          for (int ci = 0; ci < 8; ++ci) dx[ci] += gm * wt[ci * 8 + c];
        }
      }
    }
  }
  float4* o = reinterpret_cast<float4*>(dX + (sg * HinWin + ipos) * 8);
  o[0] = make_float4(dx[0], dx[1], dx[2], dx[3]);
  o[1] = make_float4(dx[4], dx[5], dx[6], dx[7]);
}

// ---------------------------------------------------------------------------
// fc dgrad.  grid = (ceil(T*E/64), ceil(K/64), P).  dX [T*P*E][K] fp32.
// WcT: [M][KP][Cout] bf16 (n contiguous).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fc_dgrad_kernel(
    const float* __restrict__ G, const uint16_t* __restrict__ bits, const bf16_t* __restrict__ WcT,
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
    const bf16_t* Wm = WcT + (long)mod * KP * Cout;
    for (int n0 = 0; n0 < Cout; n0 += 32) {
      const int nb = n0 + 8 * grp;
      s8v af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
        if (rv[i]) {
          const float4 g0 = *reinterpret_cast<const float4*>(G + sgr[i] * Cout + nb);
          const float4 g1 = *reinterpret_cast<const float4*>(G + sgr[i] * Cout + nb + 4);
          const uint32_t bw = bits[((long)a * bits_rows + sgr[i]) * nwords + (nb >> 4)] >> (nb & 15);
          const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int c = 0; c < 8; ++c) af[i][c] = (short)f2bf(((bw >> c) & 1u) ? gv[c] * g_scale : 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = col0 + j * 16 + c16;
        s8v bf = {0, 0, 0, 0, 0, 0, 0, 0};
        if (k < KP) bf = *reinterpret_cast<const s8v*>(Wm + (long)k * Cout + nb);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma16(af[i], bf, acc[i][j]);
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
// fc dgrad, LDS-staged: 1-D grid over (KSPLIT, P, ceil(T*E/64)), 512 threads (8 waves).
// The masked bf16 gradient of up to 4 active modules for the workgroup's 64 rows
// is built ONCE in LDS (G read once per row, ReLU bits applied per module), then
// every 128-column chunk of dX is swept: wave w owns 16 columns x 64 rows, so each
// weight fragment (global, WcT [M][KP][Cout]) feeds 4 MFMAs and each LDS A
// fragment is a plain ds_read_b128.  >4 active modules: further groups of 4
// accumulate into dX (the workgroup owns those outputs: no atomics).
// ---------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(512) void fc_dgrad_lds_kernel(
    const float* __restrict__ G, const uint16_t* __restrict__ bits, const bf16_t* __restrict__ WcT,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M, int K, int KP, int P,
    int E, int T, long bits_rows, float g_scale, float* __restrict__ dX, int chunks_per_split, int nrowb,
    int nsplit, bf16_t* __restrict__ Gm) {
  constexpr int CS = COUT + 8;
  constexpr int NW = COUT / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Gs[4 * 64 * CS];   // 132 KiB at COUT=256 (1 WG/CU)
  // XCD-aware order (workgroup b runs on XCD b % 8): split-major, so each XCD's L2 holds the
  // weight columns of one chunk range instead of every XCD cycling through all of them
  const int seq = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (seq >= nrowb * P * nsplit) return;
  const int bz = seq / (nrowb * P), sr_ = seq - bz * (nrowb * P);
  const int p = sr_ / nrowb, bx = sr_ - p * nrowb;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const long R = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)bx * 64;
  const int nchunks = (K + 127) / 128;
  const int ch_beg = bz * chunks_per_split;
  const int ch_end = min(nchunks, ch_beg + chunks_per_split);
  if (ch_beg >= ch_end) return;
  // epilogue rows of this lane
  long sg_out[4][4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + rb * 16 + 4 * grp + r;
      sg_out[rb][r] = row < R ? sample_global(p, (int)row, E, PE, 0) : -1;
    }
  const int ngroups = cnt > 0 ? (cnt + 3) / 4 : 1;
  for (int gi = 0; gi < ngroups; ++gi) {
    const int g0 = gi * 4;
    const int ng = min(4, cnt - g0);
    __syncthreads();
    {   // stage: thread -> (row sr, column segment); G read once, masked per module
      constexpr int SEG = COUT / 8;                 // 8 threads per row
      const int sr = tid >> 3, c0 = (tid & 7) * SEG;
      const long r = row0 + sr;
      const bool v = r < R;
      const long sg = v ? sample_global(p, (int)r, E, PE, 0) : 0;
#pragma unroll
      for (int cc = 0; cc < SEG; cc += 8) {
        const int c = c0 + cc;
        float gv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (v) {
          const float4 a0 = *reinterpret_cast<const float4*>(G + sg * COUT + c);
          const float4 a1 = *reinterpret_cast<const float4*>(G + sg * COUT + c + 4);
          gv[0] = a0.x * g_scale; gv[1] = a0.y * g_scale; gv[2] = a0.z * g_scale; gv[3] = a0.w * g_scale;
          gv[4] = a1.x * g_scale; gv[5] = a1.y * g_scale; gv[6] = a1.z * g_scale; gv[7] = a1.w * g_scale;
        }
        for (int a = 0; a < ng; ++a) {
          const uint32_t bw = v ? ((uint32_t)bits[((long)(g0 + a) * bits_rows + sg) * NW + (c >> 4)] >> (c & 15)) : 0u;
          float m[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = ((bw >> j) & 1u) ? gv[j] : 0.f;
          const s8v mb = f32x8_to_bf16(m);
          *reinterpret_cast<s8v*>(Gs + (a * 64 + sr) * CS + c) = mb;
          // side output for fc_wgrad_gm_kernel: the masked bf16 gradient of slot g0+a, row sg
          // (every K split stages the same rows: each writes its share of the column segments)
          if (Gm != nullptr && v && (tid & 7) % nsplit == bz)
            *reinterpret_cast<s8v*>(Gm + ((long)(g0 + a) * bits_rows + sg) * COUT + c) = mb;
        }
      }
    }
    __syncthreads();
    // (chunk, module) iterations flattened and software-pipelined: the 8 weight fragments of
    // iteration it+1 are loaded into registers before the 32 MFMAs of iteration it
    if (ng <= 0) {   // no active module in this layer: dX = 0
      for (int ch = ch_beg; ch < ch_end; ++ch) {
        const int kcol = ch * 128 + w * 16 + c16;
        if (kcol < K)
          for (int rb = 0; rb < 4; ++rb)
            for (int r = 0; r < 4; ++r)
              if (sg_out[rb][r] >= 0) dX[sg_out[rb][r] * K + kcol] = 0.f;
      }
      continue;
    }
    const int n_it = (ch_end - ch_beg) * ng;
    const int* aidx = act_idx + (p * L + layer) * M + g0;
    // two weight-fragment register sets used alternately (no bcur = bnxt copy), and the in-loop prefetch is
    // unconditional (the last 1-2 iterations are peeled): a conditional prefetch is a loop-carried phi that
    // made the compiler copy register sets every iteration
    s8v b0[COUT / 32], b1[COUT / 32];
    auto wload = [&](s8v* b, int it) {
      const int ch = ch_beg + it / ng, a = it - (it / ng) * ng;
      const int kc = ch * 128 + w * 16 + c16;
      const bf16_t* Wm = WcT + (long)aidx[a] * KP * COUT + (long)kc * COUT + 8 * grp;
#pragma unroll
      for (int c = 0; c < COUT / 32; ++c)
        b[c] = kc < KP ? *reinterpret_cast<const s8v*>(Wm + 32 * c) : (s8v){0, 0, 0, 0, 0, 0, 0, 0};
    };
    f4v acc[4];
    auto body = [&](const s8v* bc, int it) {
      const int ch = ch_beg + it / ng, a = it - (it / ng) * ng;
      if (a == 0) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = {0.f, 0.f, 0.f, 0.f};
      }
      const bf16_t* As = Gs + (a * 64 + c16) * CS + 8 * grp;
#pragma unroll
      for (int c = 0; c < COUT / 32; ++c)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const s8v af = *reinterpret_cast<const s8v*>(As + rb * 16 * CS + 32 * c);
          acc[rb] = mfma16(af, bc[c], acc[rb]);
        }
      const int kcol = ch * 128 + w * 16 + c16;
      if (a == ng - 1 && kcol < K) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const long sg = sg_out[rb][r];
            if (sg >= 0) {
              float* o = dX + sg * K + kcol;
              *o = gi == 0 ? acc[rb][r] : *o + acc[rb][r];
            }
          }
      }
    };
    wload(b0, 0);
    int it = 0;
    for (; it + 2 < n_it; it += 2) {
      wload(b1, it + 1);
      body(b0, it);
      wload(b0, it + 2);
      body(b1, it + 1);
    }
    if (it + 1 < n_it) {
      wload(b1, it + 1);
      body(b0, it);
      body(b1, it + 1);
    } else {
      body(b0, it);
    }
  }
}

// ---------------------------------------------------------------------------
// fc wgrad, module-major.  grid = (ceil(K/64), ceil(Cout/64), M).
// inv_path/inv_slot: [L][M][Pmax] the (path, slot) pairs using module j; inv_cnt [L][M]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fc_wgrad_kernel(
    const bf16_t* __restrict__ X, int ldx, const float* __restrict__ G, const uint16_t* __restrict__ bits,
    float* __restrict__ grad, long w_off, long b_off, int chunk, const int* __restrict__ inv_path,
    const int* __restrict__ inv_slot, const int* __restrict__ inv_cnt, int layer, int M, int Pmax, int K, int Cout,
    int P, int E, int T, long bits_rows, float g_scale, int nsplit) {
  constexpr int S = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[32 * S];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[32 * S];
  __shared__ float dbias[64];
  // blockIdx.z = module * nsplit + split: the (path, slot) users of a module are split across
  // nsplit workgroups that accumulate with fp32 atomics (grad is zeroed before the backward)
  const int j = blockIdx.z / nsplit, split = blockIdx.z - j * nsplit;
  const int n_all = inv_cnt[layer * M + j];
  const int u_beg = (int)((long)n_all * split / nsplit), u_end = (int)((long)n_all * (split + 1) / nsplit);
  if (u_beg >= u_end) return;
  const int k0b = blockIdx.x * 64, n0b = blockIdx.y * 64;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const bool do_bias = blockIdx.x == 0;
  if (tid < 64) dbias[tid] = 0.f;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const int nwords = Cout / 16;
  f4v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int srow = tid >> 3, sc = (tid & 7) * 8;
  const int mt0 = 2 * (w >> 1), nt0 = 2 * (w & 1);
  for (int u = u_beg; u < u_end; ++u) {
    const int p = inv_path[(layer * M + j) * Pmax + u];
    const int a = inv_slot[(layer * M + j) * Pmax + u];
    for (long rb = 0; rb < Rtot; rb += 32) {
      const long r = rb + srow;
      s8v xv = {0, 0, 0, 0, 0, 0, 0, 0}, gv8 = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < Rtot) {
        const long sg = sample_global(p, (int)r, E, PE, 0);
        if (k0b + sc < K) xv = *reinterpret_cast<const s8v*>(X + sg * ldx + k0b + sc);
        const int n = n0b + sc;
        if (n < Cout) {
          const float4 g0 = *reinterpret_cast<const float4*>(G + sg * Cout + n);
          const float4 g1 = *reinterpret_cast<const float4*>(G + sg * Cout + n + 4);
          const uint32_t bw = bits[((long)a * bits_rows + sg) * nwords + (n >> 4)] >> (n & 15);
          const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float x = ((bw >> c) & 1u) ? gg[c] * g_scale : 0.f;
            bpart[c] += x;
            gv8[c] = (short)f2bf(x);
          }
        }
      }
      *reinterpret_cast<s8v*>(Xs + srow * S + sc) = xv;
      *reinterpret_cast<s8v*>(Gs + srow * S + sc) = gv8;
      __syncthreads();
      s8v af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const s4v v0 = lds_tr16(Xs + (8 * grp + q) * S + (mt0 + i) * 16 + 4 * pp);
        const s4v v1 = lds_tr16(Xs + (8 * grp + 4 + q) * S + (mt0 + i) * 16 + 4 * pp);
        af[i] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        const s4v u0 = lds_tr16(Gs + (8 * grp + q) * S + (nt0 + i) * 16 + 4 * pp);
        const s4v u1 = lds_tr16(Gs + (8 * grp + 4 + q) * S + (nt0 + i) * 16 + 4 * pp);
        bf[i] = (s8v){u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma16(af[i], bf[jj], acc[i][jj]);
      __syncthreads();
    }
  }
  // dW[k][n] (TF layout [K][Cout]) -- owned by this workgroup: plain stores
  const long base = w_off + (long)j * chunk;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0b + (mt0 + i) * 16 + 4 * grp + r;
        const int n = n0b + (nt0 + jj) * 16 + i16;
        if (k < K && n < Cout) {
          if (nsplit == 1) grad[base + (long)k * Cout + n] = acc[i][jj][r];
          else atomicAdd(&grad[base + (long)k * Cout + n], acc[i][jj][r]);
        }
      }
  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 8; ++c) atomicAdd(&dbias[sc + c], bpart[c]);
    __syncthreads();
    if (tid < 64 && n0b + tid < Cout) {
      if (nsplit == 1) grad[b_off + (long)j * chunk + n0b + tid] = dbias[tid];
      else atomicAdd(&grad[b_off + (long)j * chunk + n0b + tid], dbias[tid]);
    }
  }
}

// ---------------------------------------------------------------------------
// fc wgrad from the masked bf16 gradient Gm [slot][bits_rows][COUT] that fc_dgrad_lds_kernel
// writes while staging (wide layers, K >= 1024).  The old kernel re-read fp32 G + ReLU bits for
// each of its K/64 x COUT/64 tiles (3.7 GB of G traffic for fc1 per update); a 128 x COUT tile
// reads each X row once per module user and each Gm row K/128 times at half the bytes.
// 1-D grid: (module, split) major, then k-tile.  512 threads: wave w owns k rows
// 32*(w>>1).. and n columns (COUT/2)*(w&1).., i.e. 2 x COUT/32 MFMA tiles; the row stages are
// double-buffered in LDS with the next stage's global loads issued before the MFMAs.
// The k-tile-0 workgroups also reduce the bias gradient from the same B fragments.
// ---------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(512) void fc_wgrad_gm_kernel(
    const bf16_t* __restrict__ X, int ldx, const bf16_t* __restrict__ Gm, float* __restrict__ grad, long w_off,
    long b_off, int chunk, const int* __restrict__ inv_path, const int* __restrict__ inv_slot,
    const int* __restrict__ inv_cnt, int layer, int M, int Pmax, int K, int P, int E, int T, long bits_rows,
    int nsplit) {
  constexpr int XS = 128 + 8;
  constexpr int GS = COUT + 8;
  constexpr int NT = COUT / 32;                               // n tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][32 * XS];
  __shared__ __attribute__((aligned(16))) bf16_t Gsh[2][32 * GS];
  const int kt = (K + 127) / 128;
  const int zt = blockIdx.x / kt, tile_k = blockIdx.x - zt * kt;
  const int j = zt / nsplit, split = zt - j * nsplit;
  const int n_all = inv_cnt[layer * M + j];
  const int u_beg = (int)((long)n_all * split / nsplit), u_end = (int)((long)n_all * (split + 1) / nsplit);
  if (u_beg >= u_end) return;
  const int k0 = tile_k * 128;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int wk = w >> 1, wn = w & 1;
  const int Rtot = T * E, PE = P * E;
  const int nrb = (Rtot + 31) / 32;
  const int n_it = (u_end - u_beg) * nrb;
  const int* ip = inv_path + (layer * M + j) * Pmax;
  const int* is = inv_slot + (layer * M + j) * Pmax;
  // loader: thread -> row lr of the 32-row stage, 8 k values of X and COUT/16 n values of Gm
  constexpr int GSEG = COUT / 16;
  const int lr = tid >> 4, lxs = (tid & 15) * 8, lgs = (tid & 15) * GSEG;
  const bool xin = k0 + lxs < K;
  s8v xr, gr[GSEG / 8];
  auto gload = [&](int it) {
    const int ui = it / nrb;
    const int r = (it - ui * nrb) * 32 + lr;
    const int p = ip[u_beg + ui], a = is[u_beg + ui];
    xr = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int h = 0; h < GSEG / 8; ++h) gr[h] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
    if (r < Rtot) {
      const long sg = sample_global(p, r, E, PE, 0);
      if (xin) xr = *reinterpret_cast<const s8v*>(X + sg * ldx + k0 + lxs);
      const bf16_t* gp = Gm + ((long)a * bits_rows + sg) * COUT + lgs;
#pragma unroll
      for (int h = 0; h < GSEG / 8; ++h) gr[h] = *reinterpret_cast<const s8v*>(gp + 8 * h);
    }
  };
  f4v acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) acc[i][jj] = {0.f, 0.f, 0.f, 0.f};
  float bsum[NT];
#pragma unroll
  for (int jj = 0; jj < NT; ++jj) bsum[jj] = 0.f;
  const bool do_bias = tile_k == 0 && wk == 0;
  gload(0);
  for (int it = 0; it < n_it; ++it) {
    const int buf = it & 1;
    bf16_t* xs = Xs[buf];
    bf16_t* gs = Gsh[buf];
    *reinterpret_cast<s8v*>(xs + lr * XS + lxs) = xr;
#pragma unroll
    for (int h = 0; h < GSEG / 8; ++h) *reinterpret_cast<s8v*>(gs + lr * GS + lgs + 8 * h) = gr[h];
    __syncthreads();
    if (it + 1 < n_it) gload(it + 1);
    s8v af[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const s4v v0 = lds_tr16(xs + (8 * grp + q) * XS + 32 * wk + 16 * i + 4 * pp);
      const s4v v1 = lds_tr16(xs + (8 * grp + 4 + q) * XS + 32 * wk + 16 * i + 4 * pp);
      af[i] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) {
      const int nb = (COUT / 2) * wn + 16 * jj;
      const s4v u0 = lds_tr16(gs + (8 * grp + q) * GS + nb + 4 * pp);
      const s4v u1 = lds_tr16(gs + (8 * grp + 4 + q) * GS + nb + 4 * pp);
      const s8v bf = (s8v){u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      acc[0][jj] = mfma16(af[0], bf, acc[0][jj]);
      acc[1][jj] = mfma16(af[1], bf, acc[1][jj]);
      if (do_bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[jj] += bf2f((uint16_t)bf[e]);
      }
    }
  }
  const long base = w_off + (long)j * chunk;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + 32 * wk + 16 * i + 4 * grp + r;
        const int n = (COUT / 2) * wn + 16 * jj + i16;
        if (k < K) {
          if (nsplit == 1) grad[base + (long)k * COUT + n] = acc[i][jj][r];
          else atomicAdd(&grad[base + (long)k * COUT + n], acc[i][jj][r]);
        }
      }
  if (do_bias) {
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) {
      float v = bsum[jj];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (grp == 0) {
        const long o = b_off + (long)j * chunk + (COUT / 2) * wn + 16 * jj + i16;
        if (nsplit == 1) grad[o] = v;
        else atomicAdd(&grad[o], v);
      }
    }
  }
}

extern "C" {

size_t conv_wgrad_smem(int KP) {
  if (KP <= 0) return 0;
  return (size_t)32 * (KP + 8) * 2 + 32 * (16 * 8 + 8) * 2 + 128 * 4 + (KP / 8) * 4 + MAXM * 4;
}

int launch_conv_wgrad(const void* X, int u8in, const float* G, const void* bits, float* grad, long w_off,
                      long b_off, int chunk, const int* act_idx, const int* act_cnt, int layer, int L, int M,
                      int Hin, int Win, int Cin, int KH, int KW, int S, int Ho, int Wo, int K, int KP, int P, int E,
                      int T, long bits_rows, int rows_per_chunk, float in_scale, float g_scale, hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      Ho <= 0 || Wo <= 0 || K <= 0 || KP <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 ||
      rows_per_chunk <= 0 || u8in < 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (M > MAXM || KP % 32 != 0 || KP > 512 || rows_per_chunk % 32 != 0) return -1;
  ConvGeomB g{Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP};
  const long rows = (long)T * E * Ho * Wo;
  dim3 grid((unsigned)((rows + rows_per_chunk - 1) / rows_per_chunk), P);
  const size_t sm = conv_wgrad_smem(KP);
  if (u8in)
    conv_wgrad_kernel<true><<<grid, 256, sm, stream>>>(X, G, (const uint8_t*)bits, grad, w_off, b_off, chunk,
                                                        act_idx, act_cnt, layer, L, M, g, P, E, T, bits_rows,
                                                        rows_per_chunk, in_scale, g_scale);
  else
    conv_wgrad_kernel<false><<<grid, 256, sm, stream>>>(X, G, (const uint8_t*)bits, grad, w_off, b_off, chunk,
                                                         act_idx, act_cnt, layer, L, M, g, P, E, T, bits_rows,
                                                         rows_per_chunk, in_scale, g_scale);
  return (int)hipGetLastError();
}

int launch_conv_dgrad(const float* G, const void* bits, const float* flat, long w_off, int chunk,
                      const int* act_idx, const int* act_cnt, int layer, int L, int M, int Hin, int Win, int Cin,
                      int KH, int KW, int S, int Ho, int Wo, int P, int E, int T, long bits_rows, float g_scale,
                      float* dX, hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      Ho <= 0 || Wo <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 || w_off < 0 || layer < 0) return -22;
  if (Cin != 8 || M > MAXM) return -1;
  ConvGeomB g{Hin, Win, Cin, KH, KW, S, Ho, Wo, KH * KW * Cin, 0};
  const long npix = (long)T * E * Hin * Win;
  dim3 grid((unsigned)((npix + 255) / 256), P);
  const size_t sm = (size_t)M * KH * KW * 64 * 4;
  conv_dgrad_kernel<<<grid, 256, sm, stream>>>(G, (const uint8_t*)bits, flat, w_off, chunk, act_idx, act_cnt, layer,
                                               L, M, g, P, E, T, bits_rows, g_scale, dX);
  return (int)hipGetLastError();
}

int launch_fc_dgrad(const float* G, const void* bits, const void* WcT, const int* act_idx, const int* act_cnt,
                    int layer, int L, int M, int K, int KP, int Cout, int P, int E, int T, long bits_rows,
                    float g_scale, float* dX, void* Gm, hipStream_t stream) {
  if (L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 ||
      layer < 0) return -22;
  if (M > MAXM || Cout % 32 != 0) return -1;
  if (Cout == 256) {
    const int nchunks = (K + 127) / 128;
    const int split = nchunks >= 8 ? 2 : 1;
    const int per = (nchunks + split - 1) / split;
    const int nrowb = (int)(((long)T * E + 63) / 64);
    const int nwg = (nrowb * P * split + 7) / 8 * 8;
    fc_dgrad_lds_kernel<256><<<nwg, 512, 0, stream>>>(G, (const uint16_t*)bits, (const bf16_t*)WcT, act_idx,
                                                       act_cnt, layer, L, M, K, KP, P, E, T, bits_rows, g_scale, dX,
                                                       per, nrowb, split, (bf16_t*)Gm);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)(((long)T * E + 63) / 64), (K + 63) / 64, P);
  fc_dgrad_kernel<<<grid, 256, 0, stream>>>(G, (const uint16_t*)bits, (const bf16_t*)WcT, act_idx, act_cnt, layer, L,
                                            M, K, KP, Cout, P, E, T, bits_rows, g_scale, dX);
  return (int)hipGetLastError();
}

int launch_fc_wgrad_gm(const void* X, int ldx, const void* Gm, float* grad, long w_off, long b_off, int chunk,
                       const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int M, int Pmax,
                       int K, int Cout, int P, int E, int T, long bits_rows, int nsplit, hipStream_t stream) {
  if (ldx <= 0 || chunk <= 0 || M <= 0 || Pmax <= 0 || K <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      bits_rows <= 0 || nsplit <= 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (Cout != 256 || ldx % 8 != 0 || K % 8 != 0 || nsplit < 1) return -1;
  const int kt = (K + 127) / 128;
  fc_wgrad_gm_kernel<256><<<kt * M * nsplit, 512, 0, stream>>>((const bf16_t*)X, ldx, (const bf16_t*)Gm, grad, w_off,
                                                               b_off, chunk, inv_path, inv_slot, inv_cnt, layer, M,
                                                               Pmax, K, P, E, T, bits_rows, nsplit);
  return (int)hipGetLastError();
}

int launch_fc_wgrad(const void* X, int ldx, const float* G, const void* bits, float* grad, long w_off, long b_off,
                    int chunk, const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int M,
                    int Pmax, int K, int Cout, int P, int E, int T, long bits_rows, float g_scale,
                    hipStream_t stream) {
  if (ldx <= 0 || chunk <= 0 || M <= 0 || Pmax <= 0 || K <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      bits_rows <= 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (Cout % 16 != 0 || ldx % 8 != 0) return -1;
  // split the users of each module so the grid covers >= ~2K workgroups
  const int tiles = ((K + 63) / 64) * ((Cout + 63) / 64) * M;
  int nsplit = (2048 + tiles - 1) / tiles;
  nsplit = nsplit < 1 ? 1 : (nsplit > Pmax ? Pmax : nsplit);
  dim3 grid((K + 63) / 64, (Cout + 63) / 64, M * nsplit);
  fc_wgrad_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)X, ldx, G, (const uint16_t*)bits, grad, w_off, b_off,
                                            chunk, inv_path, inv_slot, inv_cnt, layer, M, Pmax, K, Cout, P, E, T,
                                            bits_rows, g_scale, nsplit);
  return (int)hipGetLastError();
}
}
