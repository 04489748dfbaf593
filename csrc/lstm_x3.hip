// Fused LSTM cell in the fp32-accurate split-operand mode (TrainConfig.compute_dtype = "fp32x"): the reference's
// default network, BasicLSTMCell(256) unrolled over the rollout (game_ac_network.py:397-416, constants.py:30 USE_LSTM),
// at the reference's precision.
//
// Same cell, batching and launch structure as csrc/lstm.hip (TF gate order i, j, f, o; forget_bias = 1; state reset
// by the previous step's done flag); what changes is the operand precision, as in csrc/trunk_x3.hip:
//   forward  z = [x | h] K + b : fp16 pairs, x = hi + lo (22 significant bits) against the fp16 pair of K * 2^8,
//                                three MFMAs per product (hi*hi + hi*lo + lo*hi), fp32 accumulation; x (the fp32
//                                trunk output) and h / c / the saved gates stay fp32
//   backward dz K^T, dK = [x|h]^T dz : scaled fp16 pairs (csrc/trunk_x3.hip G16): dz_t * 2^e_t (e_t from the amax of
//                                      step t's dz, written by the pointwise kernel), [x|h] * 2^e_x (amax written by the
//                                      forward), K * 2^8; three f16 MFMAs, so 22 significant bits on both operands
// Per-layer error against a plain fp32 oracle: tests/test_x3_engine.py (<= 2e-5, like the trunk).
// Range: an input of the forward GEMM at or beyond fp16's 65504, or a kernel weight whose 2^8 multiple reaches
// 32768, sets the engine's fp32x status word (value 2: an fp16-pair state overflow; value 1: a scaled LSTM kernel weight
// overflow -- the same bit as a trunk weight; X3RangeError on the host).
#include "common.h"

namespace lstmx3 {

#define LX3_SHIFT 8

DEVI float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
DEVI float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}
DEVI uint16_t f2h(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
DEVI float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }

// 8 fp32 -> fp16 pair (hi = rnd(v), lo = rnd(v - hi))
DEVI void split8h(const float (&v)[8], s8v& hi, s8v& lo) {
  _Float16 h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (_Float16)v[j];
    l[j] = (_Float16)(v[j] - (float)h[j]);
  }
  __builtin_memcpy(&hi, h, 16);
  __builtin_memcpy(&lo, l, 16);
}
// 8 fp32 -> bf16 pair
DEVI void split8b(const float (&v)[8], s8v& hi, s8v& lo) {
  bf16_t h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = f2bf(v[j]);
    l[j] = f2bf(v[j] - bf2f(h[j]));
  }
  __builtin_memcpy(&hi, h, 16);
  __builtin_memcpy(&lo, l, 16);
}
DEVI void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
DEVI void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
// G16 (csrc/trunk_x3.hip): power-of-two scale putting amax into [2^13, 2^14); one atomicMax per wave
DEVI float g16_scale_of(float m) {
  const uint32_t b = __float_as_uint(m);
  const int e = (int)((b >> 23) & 0xFFu) - 127;
  if ((b & 0x7FFFFFFFu) == 0u || e < -110 || e >= 128) return 1.0f;
  const int se = min(13 - e, 126);
  return __uint_as_float((uint32_t)(se + 127) << 23);
}
DEVI void g16_flush_amax(float m, float* __restrict__ amax) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m > 0.f && amax) atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
}
// the same for a whole 256-thread workgroup: one atomic per workgroup (every thread must call it).  A per-wave
// flush of an elementwise kernel put ~8 K atomics on one address per launch (lstm_bwd_point_x3: 98 us per step)
DEVI void g16_flush_amax_wg(float m, float* __restrict__ amax) {
  __shared__ float wm[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    if (v > 0.f && amax) atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(v));
  }
}
DEVI void split8hs(const float (&v)[8], float s, s8v& hi, s8v& lo) {
  float t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = v[j] * s;
  split8h(t, hi, lo);
}

// products from hi / lo pairs, the two small cross terms first (csrc/trunk_x3.hip mma3 / mma3h)
DEVI f4v mma3h(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16_f16(al, bh, c);
  c = mfma16_f16(ah, bl, c);
  return mfma16_f16(ah, bh, c);
}
DEVI f4v mma3(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16(al, bh, c);
  c = mfma16(ah, bl, c);
  return mfma16(ah, bh, c);
}

// ---------------------------------------------------------------------------
// forward: grid (ceil(B/64), H/16), 256 threads.  The workgroup owns 64 rows (wave w: rows 16w..16w+15) and the 4
// gate blocks of 16 units (KpT2 columns permuted tile-major like csrc/lstm.hip: p = (u/16)*64 + g*16 + u%16).  The
// 64 weight columns of each 32-wide k-step are staged once per workgroup in LDS (double-buffered, the next step's
// loads in flight during this step's MFMAs): every 16-row block reading the whole weight copy from L2 made the
// kernel L2-bandwidth-bound (256 MB per call at B = 2048: 50 us).
// X: fp32 [B][ldx] (features), hprev / cprev fp32 [B][H]; KpT2: fp16 [2][4H][KK] (hi, lo of K^T * 2^8).
// ---------------------------------------------------------------------------
#define LX3_BSTR 40                               // LDS halves per staged column (32 + 8 pad)
__global__ __launch_bounds__(256) void lstm_fwd_x3_kernel(
    const float* __restrict__ X, int ldx, const float* __restrict__ hprev, const float* __restrict__ cprev,
    const uint8_t* __restrict__ prev_done, const uint16_t* __restrict__ KpT2, const float* __restrict__ flat,
    long b_off, float* __restrict__ hout, float* __restrict__ cout, float* __restrict__ gates,
    float* __restrict__ xh, uint32_t* __restrict__ status, float* __restrict__ amax_xh, int F, int H, int B) {
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][2][64 * LX3_BSTR];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int row0 = blockIdx.x * 64 + w * 16;
  const int ut = blockIdx.y;
  const int KK = F + H;
  const long plane = (long)4 * H * KK;
  const int arow = row0 + c16;
  const bool av = arow < B;
  const bool keep = av && !(prev_done && prev_done[arow]);
  const bool wr_xh = xh != nullptr && blockIdx.y == 0;
  // staging role: column sc (0..63) of the tile, 8 halves at k-offset 8 * sp, both planes
  const int sc = tid >> 2, sp = tid & 3;
  const uint16_t* Bg = KpT2 + (long)(ut * 64 + sc) * KK + 8 * sp;
  uint4 rh = *reinterpret_cast<const uint4*>(Bg), rl = *reinterpret_cast<const uint4*>(Bg + plane);
  f4v acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = {0.f, 0.f, 0.f, 0.f};
  bool bad = false;
  float am = 0.f;                                 // amax of the saved [x | h] rows (G16 scale of the weight gradient)
  const int nsteps = KK / 32;
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1, k0 = st * 32;
    *reinterpret_cast<uint4*>(&Bs[buf][0][sc * LX3_BSTR + 8 * sp]) = rh;
    *reinterpret_cast<uint4*>(&Bs[buf][1][sc * LX3_BSTR + 8 * sp]) = rl;
    __syncthreads();                              // this step's tile in LDS; the step before last is read out
    if (st + 1 < nsteps) {
      rh = *reinterpret_cast<const uint4*>(Bg + k0 + 32);
      rl = *reinterpret_cast<const uint4*>(Bg + plane + k0 + 32);
    }
    const int k = k0 + 8 * grp;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (av) {
      if (k < F) ld8(X + (long)arow * ldx + k, v);
      else if (keep) ld8(hprev + (long)arow * H + (k - F), v);
    }
    if (wr_xh && av) st8(xh + (long)arow * KK + k, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bad |= !(fabsf(v[j]) < 65504.f);
      am = fmaxf(am, fabsf(v[j]));
    }
    s8v ah, al;
    split8h(v, ah, al);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int o = (g * 16 + c16) * LX3_BSTR + 8 * grp;
      const s8v bh = *reinterpret_cast<const s8v*>(&Bs[buf][0][o]);
      const s8v bl = *reinterpret_cast<const s8v*>(&Bs[buf][1][o]);
      acc[g] = mma3h(ah, al, bh, bl, acc[g]);
    }
  }
  if (bad && status) atomicOr(status, 2u);
  if (wr_xh) g16_flush_amax(am, amax_xh);        // (whole waves: blockIdx.y is uniform)
  if (row0 >= B) return;
  const float sc_ = 1.0f / (float)(1 << LX3_SHIFT);
  const int u = ut * 16 + c16;
  const float bi = flat[b_off + u], bj = flat[b_off + H + u], bff = flat[b_off + 2 * H + u],
              bo = flat[b_off + 3 * H + u];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + 4 * grp + r;
    if (row >= B) continue;
    const bool kp = !(prev_done && prev_done[row]);
    const float c0 = kp ? cprev[(long)row * H + u] : 0.f;
    const float si = sigm(acc[0][r] * sc_ + bi);
    const float tj = tanh_f(acc[1][r] * sc_ + bj);
    const float sf = sigm(acc[2][r] * sc_ + bff + 1.0f);
    const float so = sigm(acc[3][r] * sc_ + bo);
    const float c = c0 * sf + si * tj;
    const float h = tanh_f(c) * so;
    cout[(long)row * H + u] = c;
    hout[(long)row * H + u] = h;
    if (gates) {
      float* gr = gates + (long)row * 4 * H;
      gr[u] = si;
      gr[H + u] = tj;
      gr[2 * H + u] = sf;
      gr[3 * H + u] = so;
    }
  }
}

// ---------------------------------------------------------------------------
// backward GEMM: out[b][n] = sum_p dz[b][p] K[n][p]; n < F -> dx, n >= F -> dh_prev.  Kb2: fp16 [2][KK][4H]
// (hi, lo of K * 2^8).  grid (ceil(B/64), KK/64): a workgroup owns 64 rows (16 per wave) x 64 columns (4 blocks
// of 16); each 32-wide k-step's weight tile is staged once per workgroup in LDS, as in the forward
// ---------------------------------------------------------------------------
// pointwise backward of one step (csrc/lstm.hip lstm_bwd_point_kernel) + the amax of the step's dz (G16)
__global__ __launch_bounds__(256) void lstm_bwd_point_x3_kernel(
    const float* __restrict__ dh_heads, const float* __restrict__ dh_rec, const float* __restrict__ dc_rec,
    const uint8_t* __restrict__ done_t, const float* __restrict__ gates, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, const uint8_t* __restrict__ prev_done, float* __restrict__ dz,
    float* __restrict__ dc_out, float* __restrict__ amax_dz, int H, int B) {
  float am = 0.f;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < (long)B * H; idx += (long)gridDim.x * 256) {
    const int row = (int)(idx / H), u = (int)(idx - (long)row * H);
    const float kt = (done_t && done_t[row]) ? 0.f : 1.f;
    float dh = dh_heads[idx];
    float dc = 0.f;
    if (dh_rec) dh += kt * dh_rec[idx];
    if (dc_rec) dc = kt * dc_rec[idx];
    const float* gr = gates + (long)row * 4 * H;
    const float si = gr[u], tj = gr[H + u], sf = gr[2 * H + u], so = gr[3 * H + u];
    const float c = c_t[idx];
    const float tc = tanh_f(c);
    const float c0 = (prev_done && prev_done[row]) ? 0.f : c_prev[idx];
    dc += dh * so * (1.f - tc * tc);
    float* dzr = dz + (long)row * 4 * H;
    const float z0 = dc * tj * si * (1.f - si), z1 = dc * si * (1.f - tj * tj), z2 = dc * c0 * sf * (1.f - sf),
                z3 = dh * tc * so * (1.f - so);
    dzr[u] = z0;
    dzr[H + u] = z1;
    dzr[2 * H + u] = z2;
    dzr[3 * H + u] = z3;
    dc_out[idx] = dc * sf;
    am = fmaxf(am, fmaxf(fmaxf(fabsf(z0), fabsf(z1)), fmaxf(fabsf(z2), fabsf(z3))));
  }
  g16_flush_amax_wg(am, amax_dz);
}

__global__ __launch_bounds__(256) void lstm_bwd_gemm_x3_kernel(
    const float* __restrict__ dz, const uint16_t* __restrict__ Kb2, float* __restrict__ dx, int lddx,
    float* __restrict__ dh_prev, const float* __restrict__ amax_dz, int F, int H, int B) {
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][2][64 * LX3_BSTR];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int row0 = blockIdx.x * 64 + w * 16;     // the workgroup's 64 rows share each staged weight tile
  const int n0 = blockIdx.y * 64;
  const int G4 = 4 * H;
  const long plane = (long)(F + H) * G4;
  const int arow = row0 + c16;
  const bool av = arow < B;
  const int sc = tid >> 2, sp = tid & 3;
  const uint16_t* Bg = Kb2 + (long)(n0 + sc) * G4 + 8 * sp;
  uint4 rh = *reinterpret_cast<const uint4*>(Bg), rl = *reinterpret_cast<const uint4*>(Bg + plane);
  f4v acc[4], accn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = accn[j] = (f4v){0.f, 0.f, 0.f, 0.f};
  const float gs = g16_scale_of(*amax_dz);
  const int nsteps = G4 / 32;
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1, p0 = st * 32;
    *reinterpret_cast<uint4*>(&Bs[buf][0][sc * LX3_BSTR + 8 * sp]) = rh;
    *reinterpret_cast<uint4*>(&Bs[buf][1][sc * LX3_BSTR + 8 * sp]) = rl;
    __syncthreads();
    if (st + 1 < nsteps) {
      rh = *reinterpret_cast<const uint4*>(Bg + p0 + 32);
      rl = *reinterpret_cast<const uint4*>(Bg + plane + p0 + 32);
    }
    const int p = p0 + 8 * grp;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (av) ld8(dz + (long)arow * G4 + p, v);
    // odd k-steps on the negated pieces into a second chain, subtracted at the end: the f16 MFMA's -inf rounding
    // bias enters with alternating signs instead of accumulating (csrc/trunk_x3.hip fc_dgrad_gemm_x3 FOLD 2)
    const bool odd = st & 1;
    s8v ah, al;
    split8hs(v, odd ? -gs : gs, ah, al);          // fp16 pair of dz * 2^e against the fp16 pair of K * 2^8
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = (j * 16 + c16) * LX3_BSTR + 8 * grp;
      const s8v bh = *reinterpret_cast<const s8v*>(&Bs[buf][0][o]);
      const s8v bl = *reinterpret_cast<const s8v*>(&Bs[buf][1][o]);
      if (odd) accn[j] = mma3h(ah, al, bh, bl, accn[j]);
      else acc[j] = mma3h(ah, al, bh, bl, acc[j]);
    }
  }
  if (row0 >= B) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] -= accn[j];
  const float inv = 1.0f / (gs * (float)(1 << LX3_SHIFT));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + c16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * grp + r;
      if (row >= B) continue;
      if (n < F) dx[(long)row * lddx + n] = acc[j][r] * inv;
      else dh_prev[(long)row * H + (n - F)] = acc[j][r] * inv;
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient: dK[n][p] += sum_r xh[r][n] dz[r][p] over a chunk of rows (xh, dz fp32, split into scaled fp16
// pairs while staging in LDS: xh * 2^ex, dz * 2^ez from their amaxes); db[p] += sum_r dz[r][p] (blockIdx.x == 0 tiles).  grid (KK/64, 4H/64, nchunks)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_wgrad_x3_kernel(
    const float* __restrict__ xh, const float* __restrict__ dz, float* __restrict__ grad, long k_off, long b_off,
    int F, int H, long R, int rows_per_chunk, const float* __restrict__ amax_dz, int T,
    const float* __restrict__ amax_xh, long long* __restrict__ fx) {
  constexpr int S = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][32 * S];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][32 * S];
  __shared__ unsigned long long dbq[64];         // det: int64 fixed point (common.h gacc); else the float view
  float* const dbias = reinterpret_cast<float*>(dbq);
  const int KK = F + H, G4 = 4 * H;
  const int n0b = blockIdx.x * 64, p0b = blockIdx.y * 64;
  const long r_beg = (long)blockIdx.z * rows_per_chunk;
  const long r_end = min(R, r_beg + rows_per_chunk);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const bool do_bias = blockIdx.x == 0;
  if (tid < 64) dbq[tid] = 0ull;
  f4v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int srow = tid >> 3, sc = (tid & 7) * 8;
  const int mt0 = 2 * (w >> 1), nt0 = 2 * (w & 1);
  float mdz = 0.f;                                 // dz amax over the T steps (one slot per step)
  for (int t = 0; t < T; ++t) mdz = fmaxf(mdz, amax_dz[t]);
  const float sg = g16_scale_of(mdz), sx = g16_scale_of(*amax_xh);
  for (long rb = r_beg; rb < r_end; rb += 32) {
    const long r = rb + srow;
    float xv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (r < r_end) {
      ld8(xh + r * KK + n0b + sc, xv);
      ld8(dz + r * G4 + p0b + sc, gv);
#pragma unroll
      for (int c = 0; c < 8; ++c) bpart[c] += gv[c];
    }
    s8v xhi, xlo, ghi, glo;
    split8hs(xv, sx, xhi, xlo);
    split8hs(gv, sg, ghi, glo);
    *reinterpret_cast<s8v*>(Xs[0] + srow * S + sc) = xhi;
    *reinterpret_cast<s8v*>(Xs[1] + srow * S + sc) = xlo;
    *reinterpret_cast<s8v*>(Gs[0] + srow * S + sc) = ghi;
    *reinterpret_cast<s8v*>(Gs[1] + srow * S + sc) = glo;
    __syncthreads();
    s8v af[2][2], bf[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const s4v v0 = lds_tr16(Xs[h] + (8 * grp + q) * S + (mt0 + i) * 16 + 4 * pp);
        const s4v v1 = lds_tr16(Xs[h] + (8 * grp + 4 + q) * S + (mt0 + i) * 16 + 4 * pp);
        af[h][i] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        const s4v u0 = lds_tr16(Gs[h] + (8 * grp + q) * S + (nt0 + i) * 16 + 4 * pp);
        const s4v u1 = lds_tr16(Gs[h] + (8 * grp + 4 + q) * S + (nt0 + i) * 16 + 4 * pp);
        bf[h][i] = (s8v){u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mma3h(af[0][i], af[1][i], bf[0][jj], bf[1][jj], acc[i][jj]);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0b + (mt0 + i) * 16 + 4 * grp + r;
        const int p = p0b + (nt0 + jj) * 16 + i16;
        gacc(grad, fx, k_off + (long)n * G4 + p, acc[i][jj][r] * (1.0f / (sx * sg)));
      }
  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 8; ++c) lds_acc(dbias, dbq, sc + c, bpart[c], fx != nullptr);
    __syncthreads();
    if (tid < 64) {
      if (fx) gacc_q(fx, b_off + p0b + tid, dbq[tid]);
      else atomicAdd(&grad[b_off + p0b + tid], dbias[tid]);
    }
  }
}

// operand copies of the fp32 master kernel: KpT2 = fp16 pair of K^T * 2^8 (permuted, forward), Kb2 = fp16 pair of
// K * 2^8 (TF layout, backward); status |= 1 when a scaled weight leaves the fp16 range
__global__ void lstm_refresh_x3_kernel(const float* __restrict__ flat, long k_off, int F, int H,
                                       uint16_t* __restrict__ KpT2, uint16_t* __restrict__ Kb2,
                                       uint32_t* __restrict__ status) {
  const int KK = F + H, G4 = 4 * H;
  const long n_el = (long)KK * G4;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n_el) return;
  const int n = (int)(idx / G4), col = (int)(idx - (long)n * G4);   // TF [n][col], col = g*H + u
  const float v = flat[k_off + idx];
  const float x = v * (float)(1 << LX3_SHIFT);
  const uint16_t hh = f2h(x);
  Kb2[idx] = hh;                                   // backward copy: the same fp16 pair of K * 2^8, TF layout
  Kb2[n_el + idx] = f2h(x - h2f(hh));
  const int g = col / H, u = col - g * H;
  const int p = (u >> 4) * 64 + g * 16 + (u & 15);
  KpT2[(long)p * KK + n] = hh;
  KpT2[n_el + (long)p * KK + n] = f2h(x - h2f(hh));
  if (!(fabsf(x) < 32768.f) && status) atomicOr(status, 1u);
}

// fp32 state carried into the next rollout: slot0 = slotT * (1 - done_last)
__global__ void lstm_carry_f32_kernel(const float* __restrict__ hT, const float* __restrict__ cT,
                                      const uint8_t* __restrict__ done_last, float* __restrict__ h0,
                                      float* __restrict__ c0, int H, int B) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H) return;
  const bool kp = !done_last[idx / H];
  h0[idx] = kp ? hT[idx] : 0.f;
  c0[idx] = kp ? cT[idx] : 0.f;
}

}  // namespace lstmx3
using namespace lstmx3;

extern "C" {

int launch_lstm_fwd_x3(const float* X, int ldx, const float* hprev, const float* cprev, const uint8_t* prev_done,
                       const void* KpT2, const float* flat, long b_off, float* hout, float* cout, float* gates,
                       float* xh, void* status, float* amax_xh, int F, int H, int B, hipStream_t stream) {
  if (ldx <= 0 || F <= 0 || H <= 0 || B <= 0 || b_off < 0) return -22;
  if (F % 64 != 0 || H % 64 != 0 || ldx % 8 != 0 || ldx < F) return -1;
  dim3 grid((B + 63) / 64, H / 16);
  lstm_fwd_x3_kernel<<<grid, 256, 0, stream>>>(X, ldx, hprev, cprev, prev_done, (const uint16_t*)KpT2, flat, b_off,
                                               hout, cout, gates, xh, (uint32_t*)status, amax_xh, F, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_bwd_point_x3(const float* dh_heads, const float* dh_rec, const float* dc_rec, const uint8_t* done_t,
                             const float* gates, const float* c_t, const float* c_prev, const uint8_t* prev_done,
                             float* dz, float* dc_out, float* amax_dz, int H, int B, hipStream_t stream) {
  if (H <= 0 || B <= 0 || !amax_dz) return -22;
  const long n = (long)B * H;
  lstm_bwd_point_x3_kernel<<<(unsigned)min((n + 255) / 256, 512L), 256, 0, stream>>>(dh_heads, dh_rec, dc_rec, done_t, gates,
                                                                            c_t, c_prev, prev_done, dz, dc_out,
                                                                            amax_dz, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_bwd_gemm_x3(const float* dz, const void* Kb2, float* dx, int lddx, float* dh_prev,
                            const float* amax_dz, int F, int H, int B, hipStream_t stream) {
  if (lddx <= 0 || F <= 0 || H <= 0 || B <= 0 || !amax_dz) return -22;
  if (F % 64 != 0 || H % 64 != 0 || lddx < F) return -1;
  dim3 grid((B + 63) / 64, (F + H) / 64);
  lstm_bwd_gemm_x3_kernel<<<grid, 256, 0, stream>>>(dz, (const uint16_t*)Kb2, dx, lddx, dh_prev, amax_dz, F, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_wgrad_x3(const float* xh, const float* dz, float* grad, long k_off, long b_off, int F, int H, long R,
                         int rows_per_chunk, const float* amax_dz, int T, const float* amax_xh, hipStream_t stream) {
  if (F <= 0 || H <= 0 || R <= 0 || rows_per_chunk <= 0 || k_off < 0 || b_off < 0 || T <= 0 || !amax_dz || !amax_xh)
    return -22;
  if (F % 64 != 0 || H % 64 != 0 || rows_per_chunk % 32 != 0) return -1;
  dim3 grid((F + H) / 64, (4 * H) / 64, (unsigned)((R + rows_per_chunk - 1) / rows_per_chunk));
  lstm_wgrad_x3_kernel<<<grid, 256, 0, stream>>>(xh, dz, grad, k_off, b_off, F, H, R, rows_per_chunk, amax_dz, T,
                                                 amax_xh, g_fx_accum);
  return (int)hipGetLastError();
}

int launch_lstm_refresh_x3(const float* flat, long k_off, int F, int H, void* KpT2, void* Kb2, void* status,
                           hipStream_t stream) {
  if (F <= 0 || H <= 0 || k_off < 0) return -22;
  const long n = (long)(F + H) * 4 * H;
  lstm_refresh_x3_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(flat, k_off, F, H, (uint16_t*)KpT2,
                                                                          (uint16_t*)Kb2, (uint32_t*)status);
  return (int)hipGetLastError();
}

int launch_lstm_carry_f32(const float* hT, const float* cT, const uint8_t* done_last, float* h0, float* c0, int H,
                          int B, hipStream_t stream) {
  if (H <= 0 || B <= 0) return -22;
  const long n = (long)B * H;
  lstm_carry_f32_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(hT, cT, done_last, h0, c0, H, B);
  return (int)hipGetLastError();
}
}
