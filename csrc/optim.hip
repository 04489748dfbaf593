// Multi-tensor TF-RMSProp with per-tensor clip_by_norm, over the flat buffer.
//
// Reference: rmsprop_applier.py:79-106 -> per variable: g = clip_by_norm(g, 40);
// ApplyRMSProp: ms = rho*ms + (1-rho)*g^2; mom = mu*mom + lr*g/sqrt(ms+eps);
// var -= mom.  A "variable" is a segment of the flat buffer; frozen segments
// are skipped (no apply op in the reference, a3c_training_thread.py:190-216).
//
// Three launches, no atomics and no memset (deterministic and safe inside a hipGraph replayed
// back-to-back -- see profiles/r2_graph_fence.md for what a captured hipMemsetAsync did):
//  (1) seg_sqnorm: every <= 8192-element block of a segment writes its partial sum of squares, or NaN when
//      one of its gradient entries is not finite (a finite gradient whose square sum overflows writes +inf:
//      clip_by_norm then scales it to 0, as tf.clip_by_norm does -- it is not skipped);
//  (2) nonfinite_flag (one workgroup): partial[nblk] = 1 if a TRAINABLE block's partial is NaN -- the update
//      is then skipped on every rank alike (the partials come from the all-reduced gradient); status[0] too;
//  (3) rmsprop_apply: reads that flag, sums its segment's partials in a fixed order (identical in every block
//      of the segment, bit-reproducible) for clip_by_norm, and applies.
// ``partial`` holds nblk + 1 floats.
// A third kernel refreshes the bf16 MFMA operand copies of the trunk weights (Wc [M][Cout][KP],
// WcT [M][KP][Cout]).
#include "common.h"

__global__ __launch_bounds__(256) void seg_sqnorm_kernel(const float* __restrict__ g,
                                                         const long long* __restrict__ blk_beg,
                                                         const long long* __restrict__ blk_end,
                                                         float* __restrict__ partial) {
  const int blk = blockIdx.x;
  const long b0 = blk_beg[blk], b1 = blk_end[blk];
  float s = 0.f;
  int nf = 0;
  for (long i = b0 + threadIdx.x; i < b1; i += 256) {
    const float v = g[i];
    nf |= !isfinite(v);
    s += v * v;
  }
  __shared__ float red[4];
  nf = __syncthreads_or(nf);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blk] = nf ? __builtin_nanf("") : (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void nonfinite_flag_kernel(float* __restrict__ partial, const int* __restrict__ blk_seg,
                                                             int nblk, const uint8_t* __restrict__ trainable,
                                                             float* __restrict__ status) {
  int bad = 0;
  for (int i = threadIdx.x; i < nblk; i += 256)
    if (trainable[blk_seg[i]] && isnan(partial[i])) bad = 1;
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    partial[nblk] = bad ? 1.f : 0.f;
    if (status) status[0] = bad ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void rmsprop_apply_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                            float* __restrict__ ms, float* __restrict__ mom,
                                                            const int* __restrict__ blk_seg,
                                                            const long long* __restrict__ blk_beg,
                                                            const long long* __restrict__ blk_end,
                                                            const float* __restrict__ partial,
                                                            const int* __restrict__ seg_blk0, int nblk,
                                                            const uint8_t* __restrict__ trainable,
                                                            const float* __restrict__ lr_ptr,
                                                            float decay, float momentum, float eps, float clip) {
  const int blk = blockIdx.x, tid = threadIdx.x;
  const int seg = blk_seg[blk];
  // partial[nblk]: non-finite flag of nonfinite_flag_kernel; lr_ptr = {lr, skip}: skip = host-decided skip
  if (partial[nblk] != 0.f || !trainable[seg] || lr_ptr[1] != 0.f) return;
  __shared__ float segsq;
  if (tid == 0) {
    float s = 0.f;
    for (int i = seg_blk0[seg]; i < seg_blk0[seg + 1]; ++i) s += partial[i];
    segsq = s;
  }
  __syncthreads();
  const long b0 = blk_beg[blk], b1 = blk_end[blk];
  const float norm = sqrtf(segsq);
  const float scale = clip / fmaxf(norm, clip);          // tf.clip_by_norm
  const float lr = lr_ptr[0];
  for (long i = b0 + tid; i < b1; i += 256) {
    const float gi = g[i] * scale;
    const float m = decay * ms[i] + (1.f - decay) * gi * gi;
    const float mo = momentum * mom[i] + lr * gi / sqrtf(m + eps);
    ms[i] = m;
    mom[i] = mo;
    w[i] -= mo;
  }
}

// one thread per (module, k, c) of a layer: Wc[j][c][k], WcT[j][k][c]; k in [0, KP)
__global__ __launch_bounds__(256) void refresh_weights_kernel(const float* __restrict__ flat, long w_off, int chunk,
                                                              int K, int KP, int Cout, int M, bf16_t* __restrict__ Wc,
                                                              bf16_t* __restrict__ WcT) {
  const long n = (long)M * KP * Cout;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int j = (int)(i / ((long)KP * Cout));
    const int rem = (int)(i - (long)j * KP * Cout);
    const int k = rem / Cout, c = rem - k * Cout;
    const float v = k < K ? flat[w_off + (long)j * chunk + (long)k * Cout + c] : 0.f;
    const bf16_t hv = f2bf(v);
    if (WcT) WcT[i] = hv;                                      // [j][k][c] == i
    Wc[((long)j * Cout + c) * KP + k] = hv;
  }
}

// fp16 operand copy of a uint8-input conv layer (conv_fwd_fast F16 path): Wh[j][c][k] = fp16(w) for k < K
// (zero to KP), and hcorr[j*Cout + c] = sum_k float(fp16(w_k)) -- the (1024 + pixel) offset's share of the
// accumulator, removed through the bias.  One workgroup per (module, map); fixed-order reduction.
__global__ __launch_bounds__(256) void refresh_f16_kernel(const float* __restrict__ flat, long w_off, int chunk, int K,
                                                          int KP, int Cout, uint16_t* __restrict__ Wh,
                                                          float* __restrict__ hcorr) {
  const int jc = blockIdx.x, j = jc / Cout, c = jc - j * Cout, tid = threadIdx.x;
  float s = 0.f;
  for (int k = tid; k < KP; k += 256) {
    const float v = k < K ? flat[w_off + (long)j * chunk + (long)k * Cout + c] : 0.f;
    const _Float16 h = (_Float16)v;
    Wh[(long)jc * KP + k] = __builtin_bit_cast(uint16_t, h);
    s += (float)h;
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) hcorr[jc] = (red[0] + red[1]) + (red[2] + red[3]);
}

// first conv layer on the frame ring: Wc[j][c][k'] with channel-major k' = (ci*KH + kh)*KW + kw,
// read from the flat (kh, kw, ci)-ordered module weights.  K == KP (K % 32 == 0).
__global__ __launch_bounds__(256) void refresh_cmajor_kernel(const float* __restrict__ flat, long w_off, int chunk,
                                                             int KH, int KW, int CIN, int Cout, int M,
                                                             bf16_t* __restrict__ Wc, int f16) {
  const int K = KH * KW * CIN;
  const long n = (long)M * K * Cout;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int j = (int)(i / ((long)K * Cout));
    const int rem = (int)(i - (long)j * K * Cout);
    const int c = rem / K, kd = rem - c * K;
    const int ci = kd / (KH * KW), kh = (kd / KW) % KH, kw = kd % KW;
    const int ks = (kh * KW + kw) * CIN + ci;
    const float v = flat[w_off + (long)j * chunk + (long)ks * Cout + c];
    Wc[i] = f16 ? __builtin_bit_cast(uint16_t, (_Float16)v) : f2bf(v);
  }
}

extern "C" {

int launch_refresh_weights_cmajor(const float* flat, long w_off, int chunk, int KH, int KW, int CIN, int Cout, int M,
                                  void* Wc, int f16, hipStream_t stream) {
  if (chunk <= 0 || KH <= 0 || KW <= 0 || CIN <= 0 || Cout <= 0 || M <= 0 || w_off < 0 || f16 < 0) return -22;
  if (((long)KH * KW * CIN) % 32) return -22;
  const long n = (long)M * KH * KW * CIN * Cout;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  refresh_cmajor_kernel<<<blocks, 256, 0, stream>>>(flat, w_off, chunk, KH, KW, CIN, Cout, M, (bf16_t*)Wc, f16);
  return (int)hipGetLastError();
}

// partial: float [nblk + 1] scratch; seg_blk0: int [nseg + 1] first block of every segment (blocks are
// segment-ordered); status: float [1] <- 1 if the (reduced) gradient held a non-finite value (update skipped)
int launch_rmsprop(float* w, const float* g, float* ms, float* mom, const int* blk_seg, const long long* blk_beg,
                   const long long* blk_end, int nblk, float* partial, const int* seg_blk0, const void* trainable,
                   const float* lr_ptr, float* status, float decay, float momentum, float eps, float clip,
                   hipStream_t stream) {
  if (nblk < 0) return -22;
  if (nblk <= 0) return -1;
  seg_sqnorm_kernel<<<nblk, 256, 0, stream>>>(g, blk_beg, blk_end, partial);
  nonfinite_flag_kernel<<<1, 256, 0, stream>>>(partial, blk_seg, nblk, (const uint8_t*)trainable, status);
  rmsprop_apply_kernel<<<nblk, 256, 0, stream>>>(w, g, ms, mom, blk_seg, blk_beg, blk_end, partial, seg_blk0, nblk,
                                                 (const uint8_t*)trainable, lr_ptr, decay, momentum, eps, clip);
  return (int)hipGetLastError();
}

int launch_refresh_weights_f16(const float* flat, long w_off, int chunk, int K, int KP, int Cout, int M, void* Wh,
                               float* hcorr, hipStream_t stream) {
  if (chunk <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || M <= 0 || w_off < 0) return -22;
  if (M <= 0 || Cout <= 0 || KP < K) return -1;
  refresh_f16_kernel<<<M * Cout, 256, 0, stream>>>(flat, w_off, chunk, K, KP, Cout, (uint16_t*)Wh, hcorr);
  return (int)hipGetLastError();
}

int launch_refresh_weights(const float* flat, long w_off, int chunk, int K, int KP, int Cout, int M, void* Wc,
                           void* WcT, hipStream_t stream) {
  if (chunk <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || M <= 0 || w_off < 0) return -22;
  const long n = (long)M * KP * Cout;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  refresh_weights_kernel<<<blocks, 256, 0, stream>>>(flat, w_off, chunk, K, KP, Cout, M, (bf16_t*)Wc, (bf16_t*)WcT);
  return (int)hipGetLastError();
}
}
