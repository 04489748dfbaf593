// Fused LSTM cell (TF BasicLSTMCell, gate order i, j, f, o, forget_bias = 1) for the
// PathNet-LSTM network (reference game_ac_network.py:397-416, SURVEY.md kernel K6).
//
// The recurrent state is batched over all P*E agents of the rank:
//   z = [x_t | h_{t-1}*keep] @ K + b       K: [F+H][4H] (TF layout, fp32 master in the flat buffer)
//   c_t = c_{t-1}*keep*sig(f+1) + sig(i)*tanh(j);  h_t = tanh(c_t)*sig(o)
// keep = 1 - done of the previous env step (state reset at episode end).
//
// Forward (one launch per env step): MFMA GEMM whose 64-column tile covers 16 hidden
// units x 4 gates (KpT is a bf16 copy of K^T with columns permuted tile-major:
// p = (u/16)*64 + g*16 + u%16), so every lane finds the 4 gates of its unit in its own
// 4 accumulators and the whole cell update is the GEMM epilogue -- no gate tensor
// round-trips HBM except the activations saved for the backward pass.
// Backward per step: pointwise gate gradients (fp32) + MFMA GEMM dz @ K^T (Kb = bf16 K in
// TF layout) producing dx (into the trunk's feature gradient) and dh_{t-1}.  Weight
// gradient: one split-R MFMA GEMM over all T*B rows after the reverse scan (LDS
// transposed reads, fp32 atomics into the flat gradient), bias gradient fused.
#include "common.h"

namespace lstmk {

DEVI float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
DEVI float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}

// ---------------------------------------------------------------------------
// forward: grid (ceil(B/64), H/16), 256 threads; wave w owns rows 16w..16w+15 of the
// 64-row tile and all 4 gate blocks of 16 units.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_fwd_kernel(
    const bf16_t* __restrict__ X, int ldx, const bf16_t* __restrict__ hprev, const float* __restrict__ cprev,
    const uint8_t* __restrict__ prev_done, const bf16_t* __restrict__ KpT, const float* __restrict__ flat,
    long b_off, bf16_t* __restrict__ hout, float* __restrict__ cout, float* __restrict__ gates,
    bf16_t* __restrict__ xh, int F, int H, int B) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int row0 = blockIdx.x * 64 + w * 16;
  if (row0 >= B) return;
  const int ut = blockIdx.y;                 // unit tile (16 units)
  const int KK = F + H;
  const int arow = row0 + c16;
  const bool av = arow < B;
  const bool keep = av && !(prev_done && prev_done[arow]);
  const bool wr_xh = xh != nullptr && blockIdx.y == 0;
  f4v acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = {0.f, 0.f, 0.f, 0.f};
  const bf16_t* Bp = KpT + (long)(ut * 64 + c16) * KK + 8 * grp;
  for (int k0 = 0; k0 < KK; k0 += 32) {
    const int k = k0 + 8 * grp;
    s8v a = {0, 0, 0, 0, 0, 0, 0, 0};
    if (av) {
      if (k < F) a = *reinterpret_cast<const s8v*>(X + (long)arow * ldx + k);
      else if (keep) a = *reinterpret_cast<const s8v*>(hprev + (long)arow * H + (k - F));
    }
    if (wr_xh && av) *reinterpret_cast<s8v*>(xh + (long)arow * KK + k) = a;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const s8v b = *reinterpret_cast<const s8v*>(Bp + (long)g * 16 * KK + k0);
      acc[g] = mfma16(a, b, acc[g]);
    }
  }
  const int u = ut * 16 + c16;
  const float bi = flat[b_off + u], bj = flat[b_off + H + u], bff = flat[b_off + 2 * H + u],
              bo = flat[b_off + 3 * H + u];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + 4 * grp + r;
    if (row >= B) continue;
    const bool kp = !(prev_done && prev_done[row]);
    const float c0 = kp ? cprev[(long)row * H + u] : 0.f;
    const float si = sigm(acc[0][r] + bi);
    const float tj = tanh_f(acc[1][r] + bj);
    const float sf = sigm(acc[2][r] + bff + 1.0f);
    const float so = sigm(acc[3][r] + bo);
    const float c = c0 * sf + si * tj;
    const float h = tanh_f(c) * so;
    cout[(long)row * H + u] = c;
    hout[(long)row * H + u] = f2bf(h);
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
// backward pointwise: one thread per (row, unit)
//   dh = dh_heads + keep_t*dh_rec ; dc = keep_t*dc_rec + dh*so*(1-tanh(c)^2)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_bwd_point_kernel(
    const float* __restrict__ dh_heads, const float* __restrict__ dh_rec, const float* __restrict__ dc_rec,
    const uint8_t* __restrict__ done_t, const float* __restrict__ gates, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, const uint8_t* __restrict__ prev_done, float* __restrict__ dz,
    float* __restrict__ dc_out, int H, int B) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H) return;
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
  dzr[u] = dc * tj * si * (1.f - si);
  dzr[H + u] = dc * si * (1.f - tj * tj);
  dzr[2 * H + u] = dc * c0 * sf * (1.f - sf);
  dzr[3 * H + u] = dh * tc * so * (1.f - so);
  dc_out[idx] = dc * sf;
}

// ---------------------------------------------------------------------------
// backward GEMM: out[b][n] = sum_p dz[b][p] K[n][p];  n < F -> dx, n >= F -> dh_prev
// grid (ceil(B/64), (F+H)/64); wave w: 16 rows x 64 cols (4 blocks of 16)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_bwd_gemm_kernel(
    const float* __restrict__ dz, const bf16_t* __restrict__ Kb, float* __restrict__ dx, int lddx,
    float* __restrict__ dh_prev, int F, int H, int B) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int row0 = blockIdx.x * 64 + w * 16;
  if (row0 >= B) return;
  const int n0 = blockIdx.y * 64;
  const int G4 = 4 * H;
  const int arow = row0 + c16;
  const bool av = arow < B;
  f4v acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = {0.f, 0.f, 0.f, 0.f};
  for (int p0 = 0; p0 < G4; p0 += 32) {
    const int p = p0 + 8 * grp;
    s8v a = {0, 0, 0, 0, 0, 0, 0, 0};
    if (av) {
      const float4 v0 = *reinterpret_cast<const float4*>(dz + (long)arow * G4 + p);
      const float4 v1 = *reinterpret_cast<const float4*>(dz + (long)arow * G4 + p + 4);
      const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      a = f32x8_to_bf16(f);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s8v b = *reinterpret_cast<const s8v*>(Kb + (long)(n0 + j * 16 + c16) * G4 + p);
      acc[j] = mfma16(a, b, acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + c16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * grp + r;
      if (row >= B) continue;
      if (n < F) dx[(long)row * lddx + n] = acc[j][r];
      else dh_prev[(long)row * H + (n - F)] = acc[j][r];
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient: dK[n][p] += sum_r xh[r][n] dz[r][p] over a chunk of rows;
// db[p] += sum_r dz[r][p] (blockIdx.x == 0 tiles).  grid ((F+H)/64, 4H/64, nchunks)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_wgrad_kernel(
    const bf16_t* __restrict__ xh, const float* __restrict__ dz, float* __restrict__ grad, long k_off, long b_off,
    int F, int H, long R, int rows_per_chunk) {
  constexpr int S = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[32 * S];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[32 * S];
  __shared__ float dbias[64];
  const int KK = F + H, G4 = 4 * H;
  const int n0b = blockIdx.x * 64, p0b = blockIdx.y * 64;
  const long r_beg = (long)blockIdx.z * rows_per_chunk;
  const long r_end = min(R, r_beg + rows_per_chunk);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const bool do_bias = blockIdx.x == 0;
  if (tid < 64) dbias[tid] = 0.f;
  f4v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int srow = tid >> 3, sc = (tid & 7) * 8;
  const int mt0 = 2 * (w >> 1), nt0 = 2 * (w & 1);
  for (long rb = r_beg; rb < r_end; rb += 32) {
    const long r = rb + srow;
    s8v xv = {0, 0, 0, 0, 0, 0, 0, 0}, gv8 = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < r_end) {
      xv = *reinterpret_cast<const s8v*>(xh + r * KK + n0b + sc);
      const float4 g0 = *reinterpret_cast<const float4*>(dz + r * G4 + p0b + sc);
      const float4 g1 = *reinterpret_cast<const float4*>(dz + r * G4 + p0b + sc + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
      for (int c = 0; c < 8; ++c) bpart[c] += gg[c];
      gv8 = f32x8_to_bf16(gg);
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
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0b + (mt0 + i) * 16 + 4 * grp + r;
        const int p = p0b + (nt0 + jj) * 16 + i16;
        atomicAdd(&grad[k_off + (long)n * G4 + p], acc[i][jj][r]);
      }
  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 8; ++c) atomicAdd(&dbias[sc + c], bpart[c]);
    __syncthreads();
    if (tid < 64) atomicAdd(&grad[b_off + p0b + tid], dbias[tid]);
  }
}

// bf16 compute copies of the fp32 master kernel: KpT (permuted K^T, forward) and Kb (TF layout, backward)
__global__ void lstm_refresh_kernel(const float* __restrict__ flat, long k_off, int F, int H,
                                    bf16_t* __restrict__ KpT, bf16_t* __restrict__ Kb) {
  const int KK = F + H, G4 = 4 * H;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)KK * G4) return;
  const int n = (int)(idx / G4), col = (int)(idx - (long)n * G4);   // TF [n][col], col = g*H + u
  const bf16_t v = f2bf(flat[k_off + idx]);
  Kb[idx] = v;
  const int g = col / H, u = col - g * H;
  const int p = (u >> 4) * 64 + g * 16 + (u & 15);
  KpT[(long)p * KK + n] = v;
}

// state carried into the next rollout: slot0 = slotT * (1 - done_last)
__global__ void lstm_carry_kernel(const bf16_t* __restrict__ hT, const float* __restrict__ cT,
                                  const uint8_t* __restrict__ done_last, bf16_t* __restrict__ h0,
                                  float* __restrict__ c0, int H, int B) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H) return;
  const bool kp = !done_last[idx / H];
  h0[idx] = kp ? hT[idx] : (bf16_t)0;
  c0[idx] = kp ? cT[idx] : 0.f;
}

}  // namespace lstmk
using namespace lstmk;

extern "C" {

int launch_lstm_fwd(const void* X, int ldx, const void* hprev, const float* cprev, const uint8_t* prev_done,
                    const void* KpT, const float* flat, long b_off, void* hout, float* cout, float* gates, void* xh,
                    int F, int H, int B, hipStream_t stream) {
  if (ldx <= 0 || F <= 0 || H <= 0 || B <= 0 || b_off < 0) return -22;
  if (F % 64 != 0 || H % 64 != 0 || ldx % 8 != 0) return -1;
  dim3 grid((B + 63) / 64, H / 16);
  lstm_fwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)X, ldx, (const bf16_t*)hprev, cprev, prev_done,
                                            (const bf16_t*)KpT, flat, b_off, (bf16_t*)hout, cout, gates,
                                            (bf16_t*)xh, F, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_bwd_point(const float* dh_heads, const float* dh_rec, const float* dc_rec, const uint8_t* done_t,
                          const float* gates, const float* c_t, const float* c_prev, const uint8_t* prev_done,
                          float* dz, float* dc_out, int H, int B, hipStream_t stream) {
  if (H <= 0 || B <= 0) return -22;
  const long n = (long)B * H;
  lstm_bwd_point_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(dh_heads, dh_rec, dc_rec, done_t, gates,
                                                                         c_t, c_prev, prev_done, dz, dc_out, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_bwd_gemm(const float* dz, const void* Kb, float* dx, int lddx, float* dh_prev, int F, int H, int B,
                         hipStream_t stream) {
  if (lddx <= 0 || F <= 0 || H <= 0 || B <= 0) return -22;
  if (F % 64 != 0 || H % 64 != 0) return -1;
  dim3 grid((B + 63) / 64, (F + H) / 64);
  lstm_bwd_gemm_kernel<<<grid, 256, 0, stream>>>(dz, (const bf16_t*)Kb, dx, lddx, dh_prev, F, H, B);
  return (int)hipGetLastError();
}

int launch_lstm_wgrad(const void* xh, const float* dz, float* grad, long k_off, long b_off, int F, int H, long R,
                      int rows_per_chunk, hipStream_t stream) {
  if (F <= 0 || H <= 0 || R <= 0 || rows_per_chunk <= 0 || k_off < 0 || b_off < 0) return -22;
  if (F % 64 != 0 || H % 64 != 0 || rows_per_chunk % 32 != 0) return -1;
  dim3 grid((F + H) / 64, (4 * H) / 64, (unsigned)((R + rows_per_chunk - 1) / rows_per_chunk));
  lstm_wgrad_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)xh, dz, grad, k_off, b_off, F, H, R, rows_per_chunk);
  return (int)hipGetLastError();
}

int launch_lstm_refresh(const float* flat, long k_off, int F, int H, void* KpT, void* Kb, hipStream_t stream) {
  if (F <= 0 || H <= 0 || k_off < 0) return -22;
  const long n = (long)(F + H) * 4 * H;
  lstm_refresh_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(flat, k_off, F, H, (bf16_t*)KpT,
                                                                       (bf16_t*)Kb);
  return (int)hipGetLastError();
}

int launch_lstm_carry(const void* hT, const float* cT, const uint8_t* done_last, void* h0, float* c0, int H, int B,
                      hipStream_t stream) {
  if (H <= 0 || B <= 0) return -22;
  const long n = (long)B * H;
  lstm_carry_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>((const bf16_t*)hT, cT, done_last,
                                                                     (bf16_t*)h0, c0, H, B);
  return (int)hipGetLastError();
}
}
