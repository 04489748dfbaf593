// Actor-critic heads, sampling and the A2C loss gradient (CDNA4).
//
//  heads_fwd_sample : logits = feat Wp + bp, v = feat Wv + bv, action ~ softmax
//                     by Gumbel-max on a counter-based hash RNG (replaces
//                     np.random.choice on the host, a3c_training_thread.py:89-90).
//                     One wave per sample.
//  a2c_grad         : reverse scan over T (n-step return / GAE, reward clip,
//                     a3c_training_thread.py:155-180) fused with the analytic
//                     gradient of the reference loss (game_ac_network.py:38-59)
//                     w.r.t. logits and value.  One thread per env.
//  heads_bwd        : dfeat = dz Wp^T + dv Wv^T and dWp/dbp/dWv/dbv.
#include "common.h"

#define AMAX 32

// key for the sampling RNG: depends on (seed, update counter, step, sample, action) (common.h sample_u01)
DEVI float u01(uint32_t seed, uint32_t stepkey, uint32_t b, uint32_t j) { return sample_u01(seed, stepkey, b, j); }

// trunk features are bf16 (bf16 engine) or fp32 (compute_dtype = "fp32", csrc/trunk_f32.hip)
DEVI float ldfeat(const bf16_t* p) { return bf2f(*p); }
DEVI float ldfeat(const float* p) { return *p; }

template <typename FT>
__global__ __launch_bounds__(256) void heads_fwd_sample_kernel(
    const FT* __restrict__ feat, int F, const float* __restrict__ flat, long pw, long pb, long vw, long vb, int A,
    int B, float* __restrict__ logits, float* __restrict__ value, int* __restrict__ actions, uint32_t seed,
    const long long* __restrict__ ctr, int t, int T, int greedy, int b0, uint32_t rb) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int b = b0 + blockIdx.x * 4 + w;
  if (b >= B) return;
  float part[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j) part[j] = 0.f;
  float pv = 0.f;
  for (int f = l; f < F; f += 64) {
    const float x = ldfeat(feat + (long)b * F + f);
#pragma unroll
    for (int j = 0; j < AMAX; ++j)
      if (j < A) part[j] += x * flat[pw + (long)f * A + j];
    pv += x * flat[vw + f];
  }
  float lg[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) lg[j] = wave_sum(part[j]) + flat[pb + j];
  pv = wave_sum(pv) + flat[vb];
  if (l == 0) {
    const uint32_t stepkey = (uint32_t)(ctr[0] * T + t);
    int best = 0;
    float bv = -3.0e38f;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
      if (j < A) {
        logits[(long)b * A + j] = lg[j];
        float s = lg[j];
        if (!greedy) s += -__logf(-__logf(u01(seed, stepkey, rb + (uint32_t)b, (uint32_t)j)));
        if (s > bv) { bv = s; best = j; }
      }
    }
    value[b] = pv;
    actions[b] = best;
  }
}

// Lane-per-sample variant (F % 32 == 0): a workgroup owns 64 samples, lane = sample; the policy and value
// weights are staged once per workgroup in LDS as [F][AM+1] (broadcast reads), wave w sums the features
// [w*F/4, (w+1)*F/4) of its lane's sample from 16-byte loads, the 4 partials meet in LDS in wave order
// and wave 0 adds the biases and samples one action per lane.  (The wave-per-sample kernel spends most of
// its time in A+1 cross-lane reductions per sample.)
DEVI void ldfeat8(const bf16_t* p, float* x) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x[2 * i] = __uint_as_float(u[i] << 16);
    x[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
  }
}
DEVI void ldfeat8(const float* p, float* x) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}

template <int AM, typename FT>
__global__ __launch_bounds__(256) void heads_fwd_lanes_kernel(
    const FT* __restrict__ feat, int F, const float* __restrict__ flat, long pw, long pb, long vw, long vb, int A,
    int B, float* __restrict__ logits, float* __restrict__ value, int* __restrict__ actions, uint32_t seed,
    const long long* __restrict__ ctr, int t, int T, int greedy, int b0, uint32_t rb) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  constexpr int AW = AM + 1;
  float* Wl = hsm;                       // [F][AW]: policy weights (zero padded to AM) + value weight
  float* red = hsm + F * AW;             // [3][AW][64]
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < F * AW; i += 256) {
    const int f = i / AW, j = i - f * AW;
    Wl[i] = j == AM ? flat[vw + f] : (j < A ? flat[pw + (long)f * A + j] : 0.f);
  }
  __syncthreads();
  const int b = b0 + blockIdx.x * 64 + l;
  const bool valid = b < B;
  const int fq = F >> 2;
  const int f0 = w * fq;
  float acc[AW];
#pragma unroll
  for (int j = 0; j < AW; ++j) acc[j] = 0.f;
  const FT* fr = feat + (long)(valid ? b : 0) * F;
  for (int f = f0; f < f0 + fq; f += 8) {
    float x[8];
    ldfeat8(fr + f, x);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const float* wr = Wl + (f + jj) * AW;
#pragma unroll
      for (int j = 0; j < AW; ++j) acc[j] += x[jj] * wr[j];
    }
  }
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < AW; ++j) red[((w - 1) * AW + j) * 64 + l] = acc[j];
  }
  __syncthreads();
  if (w != 0 || !valid) return;
#pragma unroll
  for (int j = 0; j < AW; ++j) acc[j] = ((acc[j] + red[j * 64 + l]) + red[(AW + j) * 64 + l]) + red[(2 * AW + j) * 64 + l];
  const uint32_t stepkey = (uint32_t)(ctr[0] * T + t);
  int best = 0;
  float bv = -3.0e38f;
#pragma unroll
  for (int j = 0; j < AM; ++j) {
    if (j < A) {
      const float lg = acc[j] + flat[pb + j];
      logits[(long)b * A + j] = lg;
      float sc = lg;
      if (!greedy) sc += -__logf(-__logf(u01(seed, stepkey, rb + (uint32_t)b, (uint32_t)j)));
      if (sc > bv) { bv = sc; best = j; }
    }
  }
  value[b] = acc[AM] + flat[vb];
  actions[b] = best;
}

// 16 samples per workgroup (128 workgroups at the bench shape instead of 32): thread (slice fs = tid >> 4,
// sample s = tid & 15) sums features [fs*F/16, (fs+1)*F/16) of its sample against LDS-staged weights; the 16
// partials meet in LDS in slice order and threads 0..15 add biases and sample.  (The 64-sample kernel above left
// 7/8 of the CUs idle and ran ~10.6 us per step on one GPU.)
template <int AM, typename FT>
__global__ __launch_bounds__(256) void heads_fwd_s16_kernel(
    const FT* __restrict__ feat, int F, const float* __restrict__ flat, long pw, long pb, long vw, long vb, int A,
    int B, float* __restrict__ logits, float* __restrict__ value, int* __restrict__ actions, uint32_t seed,
    const long long* __restrict__ ctr, int t, int T, int greedy, int b0, uint32_t rb) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  constexpr int AW = AM + 1;
  float* Wl = hsm;                       // [F][AW]
  float* red = hsm + F * AW;             // [16 slices][AW][16 samples]
  const int fs = threadIdx.x >> 4, sl = threadIdx.x & 15;
  for (int i = threadIdx.x; i < F * AW; i += 256) {
    const int f = i / AW, j = i - f * AW;
    Wl[i] = j == AM ? flat[vw + f] : (j < A ? flat[pw + (long)f * A + j] : 0.f);
  }
  __syncthreads();
  const int b = b0 + blockIdx.x * 16 + sl;
  const bool valid = b < B;
  const int fq = F >> 4;
  const int f0 = fs * fq;
  float acc[AW];
#pragma unroll
  for (int j = 0; j < AW; ++j) acc[j] = 0.f;
  const FT* fr = feat + (long)(valid ? b : 0) * F;
  for (int f = f0; f < f0 + fq; f += 8) {
    float x[8];
    ldfeat8(fr + f, x);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      // explicit fused multiply-adds (common.h heads_fma): trunk_x3.hip fc_heads_fwd_x3 repeats this sum bit for bit
      heads_fma<AW>(acc, x[jj], Wl + (f + jj) * AW);
    }
  }
#pragma unroll
  for (int j = 0; j < AW; ++j) red[(fs * AW + j) * 16 + sl] = acc[j];
  __syncthreads();
  if (fs != 0 || !valid) return;
#pragma unroll
  for (int j = 0; j < AW; ++j) {
    float v = 0.f;
    for (int k = 0; k < 16; ++k) v += red[(k * AW + j) * 16 + sl];
    acc[j] = v;
  }
  const uint32_t stepkey = (uint32_t)(ctr[0] * T + t);
  int best = 0;
  float bv = -3.0e38f;
#pragma unroll
  for (int j = 0; j < AM; ++j) {
    if (j < A) {
      const float lg = acc[j] + flat[pb + j];
      logits[(long)b * A + j] = lg;
      float sc = lg;
      if (!greedy) sc += -__logf(-__logf(u01(seed, stepkey, rb + (uint32_t)b, (uint32_t)j)));
      if (sc > bv) { bv = sc; best = j; }
    }
  }
  value[b] = acc[AM] + flat[vb];
  actions[b] = best;
}

static int HEADS_S16 = 1;
extern "C" void heads_set_s16(int v) { HEADS_S16 = v; }

template <typename FT>
static bool heads_fwd_lanes_launch(const void* feat, int F, const float* flat, long pw, long pb, long vw, long vb,
                                   int A, int B, float* logits, float* value, int* actions, unsigned seed,
                                   const long long* ctr, int t, int T, int greedy, int b0, unsigned rb,
                                   hipStream_t stream) {
  if (F % 32 != 0 || A > 18) return false;
  if (HEADS_S16 && F % 128 == 0 && A <= 8) {
    const size_t sm = (size_t)(F * 9 + 16 * 9 * 16) * 4;
    if (sm <= 64 * 1024) {
      heads_fwd_s16_kernel<8, FT><<<(unsigned)((B - b0 + 15) / 16), 256, sm, stream>>>(
          (const FT*)feat, F, flat, pw, pb, vw, vb, A, B, logits, value, actions, seed, ctr, t, T, greedy, b0, rb);
      return true;
    }
  }
  // the 18-way head (the reference's ACTION_SIZEZ, the LSTM preset): 16 samples per workgroup as well (the 64-sample
  // kernel below ran 25 us per step at 2048 samples, 32 workgroups)
  if (HEADS_S16 && F % 128 == 0 && A <= 18) {
    const size_t sm = (size_t)(F * 19 + 16 * 19 * 16) * 4;
    if (sm <= 64 * 1024) {
      heads_fwd_s16_kernel<18, FT><<<(unsigned)((B - b0 + 15) / 16), 256, sm, stream>>>(
          (const FT*)feat, F, flat, pw, pb, vw, vb, A, B, logits, value, actions, seed, ctr, t, T, greedy, b0, rb);
      return true;
    }
  }
  const unsigned g = (unsigned)((B - b0 + 63) / 64);
  if (A <= 8) {
    const size_t sm = (size_t)(F * 9 + 3 * 9 * 64) * 4;
    if (sm > 64 * 1024) return false;
    heads_fwd_lanes_kernel<8, FT><<<g, 256, sm, stream>>>((const FT*)feat, F, flat, pw, pb, vw, vb, A, B, logits,
                                                          value, actions, seed, ctr, t, T, greedy, b0, rb);
  } else {
    const size_t sm = (size_t)(F * 19 + 3 * 19 * 64) * 4;
    if (sm > 64 * 1024) return false;
    heads_fwd_lanes_kernel<18, FT><<<g, 256, sm, stream>>>((const FT*)feat, F, flat, pw, pb, vw, vb, A, B, logits,
                                                           value, actions, seed, ctr, t, T, greedy, b0, rb);
  }
  return true;
}

// logits/values/actions/rewards/dones: [T][B](...); vboot [B]
__global__ __launch_bounds__(256) void a2c_grad_kernel(
    const float* __restrict__ logits, const float* __restrict__ values, const int* __restrict__ actions,
    const float* __restrict__ rewards, const uint8_t* __restrict__ dones, const float* __restrict__ vboot, int T,
    int B, int A, float gamma, float lam, float rclip, float beta, float vcoef, float weight,
    float* __restrict__ dlogits, float* __restrict__ dvalue, float* __restrict__ stats) {
  // one thread per (t, b): the n-step / GAE recurrence from T-1 down to t is recomputed per
  // thread (O(T) independent loads, same arithmetic order as a serial scan, so bit-identical),
  // which spreads the T*B softmax gradients over the whole GPU instead of B threads.
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  float spol = 0.f, sval = 0.f, sent = 0.f;
  if (idx < (long)T * B) {
    const int t = (int)(idx / B), b = (int)(idx - (long)t * B);
    float R = vboot[b];
    float gae = 0.f;
    float next_v = vboot[b];
    float adv = 0.f, v = 0.f;
    for (int tt = T - 1; tt >= t; --tt) {
      const long i = (long)tt * B + b;
      float r = rewards[i];
      if (rclip > 0.f) r = fminf(fmaxf(r, -rclip), rclip);
      const float nd = dones[i] ? 0.f : 1.f;
      v = values[i];
      if (lam == 1.0f) {
        R = r + gamma * R * nd;
        adv = R - v;
      } else {
        const float delta = r + gamma * next_v * nd - v;
        gae = delta + gamma * lam * nd * gae;
        adv = gae;
        R = gae + v;
        next_v = v;
      }
    }
    const long i = idx;
    {
      // softmax + clipped log (game_ac_network.py:38)
      float z[AMAX];
      float m = -3.0e38f;
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) { z[j] = logits[i * A + j]; m = fmaxf(m, z[j]); }
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) { z[j] = __expf(z[j] - m); se += z[j]; }
      const float inv = 1.f / se;
      float H = 0.f;
      float lp[AMAX];
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) {
          z[j] *= inv;                                   // pi
          lp[j] = __logf(fmaxf(z[j], 1e-20f));
          H -= z[j] * lp[j];
        }
      const int a = actions[i];
      float lpa = 0.f;
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A && j == a) lpa = lp[j];
      spol += -(lpa * adv + beta * H) * weight;
      sval += vcoef * 0.5f * (R - v) * (R - v) * weight;
      sent += H;
      // d/dz_j [-(log pi_a * adv) - beta*H] = -adv*(1[j==a] - pi_j) + beta*pi_j*(log pi_j + H)
      // (clip(pi, 1e-20) has zero gradient below 1e-20; negligible, ignored)
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) {
          const float oh = (j == a) ? 1.f : 0.f;
          dlogits[i * A + j] = weight * (-adv * (oh - z[j]) + beta * z[j] * (lp[j] + H));
        }
      dvalue[i] = weight * vcoef * (v - R);
    }
  }
  // block reduce stats
  __shared__ float red[3][4];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  spol = wave_sum(spol);
  sval = wave_sum(sval);
  sent = wave_sum(sent);
  if (l == 0) { red[0][w] = spol; red[1][w] = sval; red[2][w] = sent; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float s = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    atomicAdd(&stats[threadIdx.x], s);
  }
}

// grid = ceil(N / ROWS), block 256 (thread = feature f, looping f += 256)
// part == nullptr: the row-chunk partials meet in grad with fp32 atomics.  Deterministic mode: chunk c writes
// its partials to part[c][F*A + F + A + 1] (dWp, dWv, dbp, dbv) and heads_reduce_kernel sums the chunks in order.
#define HB_ROWS 128
// non-deterministic mode (launch_heads_bwd_split, default heads_set_bwd_rows(32)): 32-row chunks (1 280 workgroups at
// T*B = 40 960 instead of 320: each thread's serial row loop of dependent loads is 4x shorter and ~5 workgroups share
// a CU) writing partials that heads_reduce_wide_kernel sums: 32 + 20 vs 113 us for the 128-row kernel with fp32
// atomics (heads_set_bwd_rows(128)).  32-row chunks with atomics instead of partials ran 257 us (2.3 M atomics on the
// 1 799 weight / bias gradient addresses).
static int HB_ROWS_ATOMIC = 32;
template <int AM, typename FT, int ROWS = HB_ROWS>
__global__ __launch_bounds__(256) void heads_bwd_kernel(
    const FT* __restrict__ feat, int F, const float* __restrict__ dlogits, const float* __restrict__ dvalue,
    int N, int A, const float* __restrict__ flat, long pw, long pb, long vw, long vb, float* __restrict__ grad,
    float* __restrict__ dfeat, float* __restrict__ part) {
  const long PS = (long)F * A + F + A + 1;
  float* pc = part ? part + blockIdx.x * PS : nullptr;
  const long r0 = (long)blockIdx.x * ROWS;
  const long r1 = min((long)N, r0 + ROWS);
  // the chunk's dlogits / dvalue rows, staged once (coalesced) and read as LDS broadcasts: per-row uniform
  // global loads put one memory latency on every row of the serial row loop (138 us per update at T*B = 40960)
  __shared__ float dzs[ROWS][AM + 1];
  const int nr = (int)(r1 - r0);
  for (int i = threadIdx.x; i < nr * (AM + 1); i += 256) {
    const int rr = i / (AM + 1), j = i - rr * (AM + 1);
    dzs[rr][j] = j == AM ? dvalue[r0 + rr] : (j < A ? dlogits[(r0 + rr) * A + j] : 0.f);
  }
  __syncthreads();
  for (int f = threadIdx.x; f < F; f += 256) {
    float w[AM], gw[AM];
#pragma unroll
    for (int j = 0; j < AM; ++j) {
      w[j] = j < A ? flat[pw + (long)f * A + j] : 0.f;
      gw[j] = 0.f;
    }
    const float wv = flat[vw + f];
    float gv = 0.f;
#pragma unroll 8
    for (int rr = 0; rr < nr; ++rr) {
      const long r = r0 + rr;
      const float x = ldfeat(feat + r * F + f);
      const float dv = dzs[rr][AM];
      float d = dv * wv;
#pragma unroll
      for (int j = 0; j < AM; ++j) {
        const float dz = dzs[rr][j];      // zero for j >= A
        d += dz * w[j];
        gw[j] += x * dz;
      }
      gv += x * dv;
      dfeat[r * F + f] = d;
    }
    if (pc) {
#pragma unroll
      for (int j = 0; j < AM; ++j)
        if (j < A) pc[(long)f * A + j] = gw[j];
      pc[(long)F * A + f] = gv;
    } else {
#pragma unroll
      for (int j = 0; j < AM; ++j)
        if (j < A) atomicAdd(&grad[pw + (long)f * A + j], gw[j]);
      atomicAdd(&grad[vw + f], gv);
    }
  }
  if (threadIdx.x < 64) {
    // bias grads: wave 0 reduces dz / dv over the chunk
    const int l = threadIdx.x;
    float bz[AM];
#pragma unroll
    for (int j = 0; j < AM; ++j) bz[j] = 0.f;
    float bvv = 0.f;
    for (long r = r0 + l; r < r1; r += 64) {
#pragma unroll
      for (int j = 0; j < AM; ++j)
        if (j < A) bz[j] += dlogits[r * A + j];
      bvv += dvalue[r];
    }
#pragma unroll
    for (int j = 0; j < AM; ++j)
      if (j < A) {
        const float s = wave_sum(bz[j]);
        if (l == 0) {
          if (pc) pc[(long)F * A + F + j] = s;
          else atomicAdd(&grad[pb + j], s);
        }
      }
    bvv = wave_sum(bvv);
    if (l == 0) {
      if (pc) pc[PS - 1] = bvv;
      else atomicAdd(&grad[vb], bvv);
    }
  }
}

// deterministic mode: grad[head param e] += sum over the row chunks of part[c][e], in chunk order
__global__ __launch_bounds__(256) void heads_reduce_kernel(const float* __restrict__ part, int nchunk, int F, int A,
                                                           long pw, long pb, long vw, long vb,
                                                           float* __restrict__ grad) {
  const long PS = (long)F * A + F + A + 1;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= PS) return;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += part[c * PS + e];
  long dst;
  if (e < (long)F * A) dst = pw + e;
  else if (e < (long)F * A + F) dst = vw + (e - (long)F * A);
  else if (e < PS - 1) dst = pb + (e - (long)F * A - F);
  else dst = vb;
  grad[dst] += s;
}

extern "C" {

// samples [b0, B) (a path group of the split rollout, runtime/engine.py); RNG keys use the global sample index
// row_base + b (row_base = this rank's first sample: the same draws whatever the population's sharding)
int launch_heads_fwd_sample(const void* feat, int F, const float* flat, long pw, long pb, long vw, long vb, int A,
                            int B, float* logits, float* value, int* actions, unsigned seed, const long long* ctr,
                            int t, int T, int greedy, int b0, unsigned row_base, hipStream_t stream) {
  if (F <= 0 || A <= 0 || B <= 0 || T <= 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0 || t < 0 || greedy < 0 ||
      b0 < 0) return -22;
  if (A > AMAX || A < 1 || b0 < 0 || b0 >= B) return -1;
  if (!heads_fwd_lanes_launch<bf16_t>(feat, F, flat, pw, pb, vw, vb, A, B, logits, value, actions, seed, ctr, t, T,
                                      greedy, b0, row_base, stream))
    heads_fwd_sample_kernel<bf16_t><<<(B - b0 + 3) / 4, 256, 0, stream>>>((const bf16_t*)feat, F, flat, pw, pb, vw,
                                                                           vb, A, B, logits, value, actions, seed, ctr,
                                                                           t, T, greedy, b0, row_base);
  return (int)hipGetLastError();
}

int launch_heads_fwd_sample_f32(const void* feat, int F, const float* flat, long pw, long pb, long vw, long vb,
                                int A, int B, float* logits, float* value, int* actions, unsigned seed,
                                const long long* ctr, int t, int T, int greedy, int b0, unsigned row_base,
                                hipStream_t stream) {
  if (F <= 0 || A <= 0 || B <= 0 || T <= 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0 || t < 0 || greedy < 0 ||
      b0 < 0) return -22;
  if (A > AMAX || A < 1 || b0 < 0 || b0 >= B) return -1;
  if (!heads_fwd_lanes_launch<float>(feat, F, flat, pw, pb, vw, vb, A, B, logits, value, actions, seed, ctr, t, T,
                                     greedy, b0, row_base, stream))
    heads_fwd_sample_kernel<float><<<(B - b0 + 3) / 4, 256, 0, stream>>>((const float*)feat, F, flat, pw, pb, vw, vb,
                                                                          A, B, logits, value, actions, seed, ctr, t,
                                                                          T, greedy, b0, row_base);
  return (int)hipGetLastError();
}

int launch_a2c_grad(const float* logits, const float* values, const int* actions, const float* rewards,
                    const void* dones, const float* vboot, int T, int B, int A, float gamma, float lam, float rclip,
                    float beta, float vcoef, float weight, float* dlogits, float* dvalue, float* stats,
                    hipStream_t stream) {
  if (T <= 0 || B <= 0 || A <= 0) return -22;
  if (A > AMAX) return -1;
  a2c_grad_kernel<<<(unsigned)(((long)T * B + 255) / 256), 256, 0, stream>>>(logits, values, actions, rewards, (const uint8_t*)dones,
                                                        vboot, T, B, A, gamma, lam, rclip, beta, vcoef, weight,
                                                        dlogits, dvalue, stats);
  return (int)hipGetLastError();
}

}  // extern "C"

// the split path's chunk reduction: 64 elements per workgroup, the 4 waves each sum a quarter of the chunks (8
// independent partial sums per lane), combined in LDS; one writer per element.  (heads_reduce_kernel's one thread
// per element over all 1 280 chunks was a 1 280-long dependent load chain: 307 us.)
__global__ __launch_bounds__(256) void heads_reduce_wide_kernel(const float* __restrict__ part, int nchunk, int F,
                                                                int A, long pw, long pb, long vw, long vb,
                                                                float* __restrict__ grad) {
  __shared__ float red[4][64];
  const long PS = (long)F * A + F + A + 1;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const long e = (long)blockIdx.x * 64 + l;
  const int c0 = (int)((long)nchunk * w / 4), c1 = (int)((long)nchunk * (w + 1) / 4);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < PS) {
    int c = c0;
    for (; c + 8 <= c1; c += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += part[(long)(c + j) * PS + e];
    }
    for (; c < c1; ++c) a[0] += part[(long)c * PS + e];
  }
  red[w][l] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (w > 0 || e >= PS) return;
  const float s = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
  long dst;
  if (e < (long)F * A) dst = pw + e;
  else if (e < (long)F * A + F) dst = vw + (e - (long)F * A);
  else if (e < PS - 1) dst = pb + (e - (long)F * A - F);
  else dst = vb;
  grad[dst] += s;
}

template <typename FT>
static int heads_bwd_split32(const void* feat, int F, const float* dlogits, const float* dvalue, int N, int A,
                             const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                             float* part, hipStream_t stream) {
  const int nc = (N + 31) / 32;
  if (A <= 8)
    heads_bwd_kernel<8, FT, 32><<<nc, 256, 0, stream>>>((const FT*)feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw,
                                                        vb, grad, dfeat, part);
  else
    heads_bwd_kernel<AMAX, FT, 32><<<nc, 256, 0, stream>>>((const FT*)feat, F, dlogits, dvalue, N, A, flat, pw, pb,
                                                           vw, vb, grad, dfeat, part);
  const long PS = (long)F * A + F + A + 1;
  heads_reduce_wide_kernel<<<(unsigned)((PS + 63) / 64), 256, 0, stream>>>(part, nc, F, A, pw, pb, vw, vb, grad);
  return (int)hipGetLastError();
}

template <typename FT>
static int heads_bwd_launch(const void* feat, int F, const float* dlogits, const float* dvalue, int N, int A,
                            const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                            float* part, hipStream_t stream) {
  if (A > AMAX) return -1;
  const int nchunk = (N + HB_ROWS - 1) / HB_ROWS;
  if (A <= 8)
    heads_bwd_kernel<8, FT><<<nchunk, 256, 0, stream>>>((const FT*)feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw,
                                                        vb, grad, dfeat, part);
  else
    heads_bwd_kernel<AMAX, FT><<<nchunk, 256, 0, stream>>>((const FT*)feat, F, dlogits, dvalue, N, A, flat, pw, pb,
                                                           vw, vb, grad, dfeat, part);
  if (part) {
    const long PS = (long)F * A + F + A + 1;
    heads_reduce_kernel<<<(unsigned)((PS + 255) / 256), 256, 0, stream>>>(part, nchunk, F, A, pw, pb, vw, vb, grad);
  }
  return (int)hipGetLastError();
}

extern "C" {
int launch_heads_bwd(const void* feat, int F, const float* dlogits, const float* dvalue, int N, int A,
                     const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                     hipStream_t stream) {
  if (F <= 0 || N <= 0 || A <= 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0) return -22;
  return heads_bwd_launch<bf16_t>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, nullptr,
                                  stream);
}

int launch_heads_bwd_f32(const void* feat, int F, const float* dlogits, const float* dvalue, int N, int A,
                         const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                         hipStream_t stream) {
  if (F <= 0 || N <= 0 || A <= 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0) return -22;
  return heads_bwd_launch<float>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, nullptr,
                                 stream);
}

extern "C" void heads_set_bwd_rows(int r) { HB_ROWS_ATOMIC = r == 32 ? 32 : HB_ROWS; }

// non-deterministic heads backward with a partials buffer of heads_bwd_split_numel floats: 32-row chunks + ordered
// chunk reduction when heads_set_bwd_rows(32), else the 128-row atomic kernel (part unused)
long heads_bwd_split_numel(int N, int F, int A) {
  if (N <= 0 || F <= 0 || A <= 0) return -1;
  return (long)((N + 31) / 32) * ((long)F * A + F + A + 1);
}

int launch_heads_bwd_split(const void* feat, int f32, int F, const float* dlogits, const float* dvalue, int N, int A,
                           const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                           float* part, hipStream_t stream) {
  if (F <= 0 || N <= 0 || A <= 0 || f32 < 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0 || !part) return -22;
  if (A > AMAX) return -1;
  if (HB_ROWS_ATOMIC != 32)
    return f32 ? heads_bwd_launch<float>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, nullptr,
                                         stream)
               : heads_bwd_launch<bf16_t>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, nullptr,
                                          stream);
  return f32 ? heads_bwd_split32<float>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, part, stream)
             : heads_bwd_split32<bf16_t>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, part,
                                         stream);
}

// deterministic heads backward (fixed-order chunk reduction); part: ceil(N/128) * (F*A + F + A + 1) floats
long heads_bwd_part_numel(int N, int F, int A) {
  if (N <= 0 || F <= 0 || A <= 0) return -1;
  return (long)((N + HB_ROWS - 1) / HB_ROWS) * ((long)F * A + F + A + 1);
}

int launch_heads_bwd_det(const void* feat, int f32, int F, const float* dlogits, const float* dvalue, int N, int A,
                         const float* flat, long pw, long pb, long vw, long vb, float* grad, float* dfeat,
                         float* part, hipStream_t stream) {
  if (F <= 0 || N <= 0 || A <= 0 || f32 < 0 || pw < 0 || pb < 0 || vw < 0 || vb < 0) return -22;
  if (!part) return -1;
  if (f32) return heads_bwd_launch<float>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, part,
                                          stream);
  return heads_bwd_launch<bf16_t>(feat, F, dlogits, dvalue, N, A, flat, pw, pb, vw, vb, grad, dfeat, part, stream);
}
}

// ---------------------------------------------------------------------------
// fitness bookkeeping after a rollout: per path, the return of the most
// recently finished episode(s) (a3c_training_thread.py:145-147; mean over
// envs finishing at the same step), plus episode counters.
// counters: [0] agent steps, [1] episodes finished, [2] sum of their returns, [3] 0.
// Deterministic and memset-free: every sum runs in a fixed order (thread t sums step t over the envs in
// order; path partials are combined by one thread in path order), so non-integer returns (Doom) give
// bit-identical fitness run to run, and nothing in the captured graph depends on a hipMemsetAsync node.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fitness_update_kernel(const uint8_t* __restrict__ dones,
                                                             const float* __restrict__ epret, int T, int P, int E,
                                                             float* __restrict__ fitness,
                                                             float* __restrict__ fit_cnt, float* __restrict__ fit_sum,
                                                             float* __restrict__ path_part, int window) {
  // window == 0: fitness = return of the most recently finished episode(s) (a3c_training_thread.py:145-147);
  // window >= 1: fitness = mean return of the episodes finished since the path's last tournament,
  //              pending (-1000) until at least `window` of them have finished.
  extern __shared__ float ts[];                  // [T][2]: finished episodes, sum of their returns
  const int p = blockIdx.x, tid = threadIdx.x;
  const long PE = (long)P * E;
  for (int t = tid; t < T; t += blockDim.x) {
    float c = 0.f, s = 0.f;
    const long base = t * PE + (long)p * E;
    for (int e = 0; e < E; ++e)
      if (dones[base + e]) {
        c += 1.f;
        s += epret[base + e];
      }
    ts[2 * t] = c;
    ts[2 * t + 1] = s;
  }
  __syncthreads();
  if (tid != 0) return;
  float fit = fitness[p];
  float nep = 0.f, sret = 0.f;
  for (int t = 0; t < T; ++t) {
    const float c = ts[2 * t], s = ts[2 * t + 1];
    if (c > 0.f) fit = s / c;
    nep += c;
    sret += s;
  }
  if (window > 0) {
    const float cnt = fit_cnt[p] + nep, sum = fit_sum[p] + sret;
    fit_cnt[p] = cnt;
    fit_sum[p] = sum;
    fit = cnt >= (float)window ? sum / cnt : -1000.f;
  }
  fitness[p] = fit;
  path_part[2 * p] = nep;
  path_part[2 * p + 1] = sret;
}

__global__ void fitness_counters_kernel(const float* __restrict__ path_part, int T, int P, int E,
                                        float* __restrict__ counters) {
  if (threadIdx.x != 0) return;
  float n = 0.f, s = 0.f;
  for (int p = 0; p < P; ++p) {
    n += path_part[2 * p];
    s += path_part[2 * p + 1];
  }
  counters[0] = (float)T * P * E;
  counters[1] = n;
  counters[2] = s;
  counters[3] = 0.f;
}

extern "C" int launch_fitness_update(const void* dones, const float* epret, int T, int P, int E, float* fitness,
                                     float* counters, float* fit_cnt, float* fit_sum, int window, float* path_part,
                                     hipStream_t stream) {
  if (T <= 0 || P <= 0 || E <= 0) return -1;
  fitness_update_kernel<<<P, 64, sizeof(float) * 2 * T, stream>>>((const uint8_t*)dones, epret, T, P, E, fitness,
                                                                   fit_cnt, fit_sum, path_part, window);
  fitness_counters_kernel<<<1, 64, 0, stream>>>(path_part, T, P, E, counters);
  return (int)hipGetLastError();
}
