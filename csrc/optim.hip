// Multi-tensor TF-RMSProp with per-tensor clip_by_norm, over the flat buffer.
//
// Reference: rmsprop_applier.py:79-106 -> per variable: g = clip_by_norm(g, 40);
// ApplyRMSProp: ms = rho*ms + (1-rho)*g^2; mom = mu*mom + lr*g/sqrt(ms+eps);
// var -= mom.  A "variable" is a segment of the flat buffer; frozen segments
// are skipped (no apply op in the reference, a3c_training_thread.py:190-216).
//
// Two launches: (1) per-segment squared norms (block partials + one atomic per
// block), (2) fused clip + apply.  A third kernel refreshes the bf16 MFMA
// operand copies of the trunk weights (Wc [M][Cout][KP], WcT [M][KP][Cout]).
#include "common.h"

__global__ __launch_bounds__(256) void seg_sqnorm_kernel(const float* __restrict__ g, const int* __restrict__ blk_seg,
                                                         const long long* __restrict__ blk_beg,
                                                         const long long* __restrict__ blk_end,
                                                         float* __restrict__ sq) {
  const int blk = blockIdx.x;
  const long b0 = blk_beg[blk], b1 = blk_end[blk];
  float s = 0.f;
  for (long i = b0 + threadIdx.x; i < b1; i += 256) {
    const float v = g[i];
    s += v * v;
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&sq[blk_seg[blk]], red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void rmsprop_apply_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                            float* __restrict__ ms, float* __restrict__ mom,
                                                            const int* __restrict__ blk_seg,
                                                            const long long* __restrict__ blk_beg,
                                                            const long long* __restrict__ blk_end,
                                                            const float* __restrict__ sq,
                                                            const uint8_t* __restrict__ trainable,
                                                            const float* __restrict__ lr_ptr, float decay,
                                                            float momentum, float eps, float clip) {
  const int blk = blockIdx.x;
  const int seg = blk_seg[blk];
  if (!trainable[seg] || lr_ptr[1] != 0.f) return;      // lr_ptr = {lr, skip}: skip = non-finite update
  const long b0 = blk_beg[blk], b1 = blk_end[blk];
  const float norm = sqrtf(sq[seg]);
  const float scale = clip / fmaxf(norm, clip);          // tf.clip_by_norm
  const float lr = lr_ptr[0];
  for (long i = b0 + threadIdx.x; i < b1; i += 256) {
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

// first conv layer on the frame ring: Wc[j][c][k'] with channel-major k' = (ci*KH + kh)*KW + kw,
// read from the flat (kh, kw, ci)-ordered module weights.  K == KP (K % 32 == 0).
__global__ __launch_bounds__(256) void refresh_cmajor_kernel(const float* __restrict__ flat, long w_off, int chunk,
                                                             int KH, int KW, int CIN, int Cout, int M,
                                                             bf16_t* __restrict__ Wc) {
  const int K = KH * KW * CIN;
  const long n = (long)M * K * Cout;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int j = (int)(i / ((long)K * Cout));
    const int rem = (int)(i - (long)j * K * Cout);
    const int c = rem / K, kd = rem - c * K;
    const int ci = kd / (KH * KW), kh = (kd / KW) % KH, kw = kd % KW;
    const int ks = (kh * KW + kw) * CIN + ci;
    Wc[i] = f2bf(flat[w_off + (long)j * chunk + (long)ks * Cout + c]);
  }
}

extern "C" {

int launch_refresh_weights_cmajor(const float* flat, long w_off, int chunk, int KH, int KW, int CIN, int Cout, int M,
                                  void* Wc, hipStream_t stream) {
  if ((KH * KW * CIN) % 32) return -22;
  const long n = (long)M * KH * KW * CIN * Cout;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  refresh_cmajor_kernel<<<blocks, 256, 0, stream>>>(flat, w_off, chunk, KH, KW, CIN, Cout, M, (bf16_t*)Wc);
  return (int)hipGetLastError();
}

int launch_rmsprop(float* w, const float* g, float* ms, float* mom, const int* blk_seg, const long long* blk_beg,
                   const long long* blk_end, int nblk, float* sq, int nseg, const void* trainable, const float* lr_ptr,
                   float decay, float momentum, float eps, float clip, hipStream_t stream) {
  hipMemsetAsync(sq, 0, sizeof(float) * nseg, stream);
  seg_sqnorm_kernel<<<nblk, 256, 0, stream>>>(g, blk_seg, blk_beg, blk_end, sq);
  rmsprop_apply_kernel<<<nblk, 256, 0, stream>>>(w, g, ms, mom, blk_seg, blk_beg, blk_end, sq,
                                                 (const uint8_t*)trainable, lr_ptr, decay, momentum, eps, clip);
  return (int)hipGetLastError();
}

int launch_refresh_weights(const float* flat, long w_off, int chunk, int K, int KP, int Cout, int M, void* Wc,
                           void* WcT, hipStream_t stream) {
  const long n = (long)M * KP * Cout;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  refresh_weights_kernel<<<blocks, 256, 0, stream>>>(flat, w_off, chunk, K, KP, Cout, M, (bf16_t*)Wc, (bf16_t*)WcT);
  return (int)hipGetLastError();
}
}
