// Shared helpers for the pathnet_gym_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; workgroups are 256 threads (4 waves) unless noted.
//  * MFMA: v_mfma_f32_16x16x32_bf16.  Lane l holds A[row=l&15][k=8*(l>>4)+j],
//    B[k=8*(l>>4)+j][col=l&15] (j=0..7) and C/D[row=4*(l>>4)+r][col=l&15].
//  * bf16 is carried as uint16 bits; fp32 accumulation everywhere.
//  * Batch layout of activations: [T][P*E][features] (step-major, path-major
//    inside a step).  A kernel working on path p sees rows
//    R = (s, pos) with s in [0, T*E), sample_global = (t0 + s/E)*P*E + p*E + s%E.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned short bf16_t;

#define DEVI __device__ __forceinline__

DEVI float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// RNE conversion through the compiler's __bf16 type: lowers to v_cvt_pk_bf16_f32 on gfx950
DEVI bf16_t f2bf(float f) {
  const __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

// 8 x uint8 (0..255, exact in bf16) -> 8 x bf16: v_cvt_f32_ubyteN + v_cvt_pk_bf16_f32
// float(v) of a byte has zero low 16 mantissa bits, so its upper half IS bf16(v): one v_cvt_f32_ubyte per value
// and one v_perm_b32 per pair (the (__bf16) conversion compiled to a v_cvt_pk_bf16_f32 per value plus merges)
DEVI s8v u8x8_to_bf16(uint2 v) {
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float a = (float)(v.x >> (16 * j) & 0xFFu), b = (float)(v.x >> (16 * j + 8) & 0xFFu);
    const float c = (float)(v.y >> (16 * j) & 0xFFu), d = (float)(v.y >> (16 * j + 8) & 0xFFu);
    w[j] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a), 0x07060302u);
    w[j + 2] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, d), __builtin_bit_cast(uint32_t, c), 0x07060302u);
  }
  s8v r;
  __builtin_memcpy(&r, w, 16);
  return r;
}

// 8 x uint8 -> 8 x fp16 holding (1024 + v): fp16(1024 + v) has the bit pattern 0x6400 | v for v < 1024,
// so one v_perm_b32 per 2 pixels builds it (vs 12 VALU for u8 -> f32 -> bf16).  The +1024 offset is
// removed in the epilogue through a per-column bias correction (1024 * sum_k w_k, csrc/optim.hip).
DEVI s8v u8x8_to_f16off(uint2 v) {
  const uint32_t o = 0x64646464u;
  uint32_t d[4];
  d[0] = __builtin_amdgcn_perm(o, v.x, 0x04010400u);
  d[1] = __builtin_amdgcn_perm(o, v.x, 0x04030402u);
  d[2] = __builtin_amdgcn_perm(o, v.y, 0x04010400u);
  d[3] = __builtin_amdgcn_perm(o, v.y, 0x04030402u);
  s8v r;
  __builtin_memcpy(&r, d, 16);
  return r;
}

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
DEVI f4v mfma16_f16(const s8v& a, const s8v& b, const f4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}

DEVI s8v f32x8_to_bf16(const float* f) {
  __bf16 h[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (__bf16)f[j];
  s8v r;
  __builtin_memcpy(&r, h, 16);
  return r;
}

DEVI uint32_t pack2bf(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

DEVI f4v mfma16(const s8v& a, const s8v& b, const f4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS transposed read: within each 16-lane group, lane 4q+p passes the address of
// row q, columns 4p..4p+3 of a 4x16 block of 16-bit values; lane i receives
// column i of the 4 rows (row q in element q).
DEVI s4v lds_tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}

DEVI int lane_id() { return threadIdx.x & 63; }

// sample index (in the [T][P*E] batch) of path-local sample s
// Every exported launcher starts with a guard that returns -22 (EINVAL; 0 for the *_smem sizes) when a size
// argument is <= 0 or an offset / index argument is negative, so invalid arguments never reach the host-side
// grid and shared-memory arithmetic (checked by the host ASan/UBSan harness, pathnet_gym_amd/_sanitize.py).
DEVI long sample_global(int p, int s, int E, int PE, int t0) {
  int t = s / E;
  int e = s - t * E;
  return (long)(t0 + t) * PE + (long)p * E + e;
}

// wave-wide sum
DEVI float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DEVI float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 32-bit Wang hash: bit-identical to envs/base.py:wang_hash
DEVI uint32_t wang_hash(uint32_t x) {
  x = (x ^ 61u) ^ (x >> 16);
  x = x * 9u;
  x = x ^ (x >> 4);
  x = x * 0x27D4EB2Du;
  x = x ^ (x >> 15);
  return x;
}

// heads accumulation acc[j] += x * w[j] (j < AW) as fused multiply-adds, pairs of j on v_pk_fma_f32, the odd one on
// v_fma_f32: the same instructions in every kernel that repeats the heads sum (heads.hip, trunk_x3.hip fused heads)
template <int AW>
DEVI void heads_fma(float (&acc)[AW], float x, const float* w) {
  typedef float hf2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j + 1 < AW; j += 2) {
    const hf2 r = __builtin_elementwise_fma((hf2){x, x}, (hf2){w[j], w[j + 1]}, (hf2){acc[j], acc[j + 1]});
    acc[j] = r[0];
    acc[j + 1] = r[1];
  }
  if constexpr (AW % 2) acc[AW - 1] = __builtin_fmaf(x, w[AW - 1], acc[AW - 1]);
}

// action-sampling RNG (heads.hip Gumbel-max, trunk_x3.hip fused heads): a uniform in (0, 1) keyed by
// (seed, update counter x step, sample, action)
DEVI float sample_u01(uint32_t seed, uint32_t stepkey, uint32_t b, uint32_t j) {
  uint32_t h = wang_hash(stepkey * 64u + j);
  h = wang_hash(h ^ b);
  h = wang_hash(h ^ seed);
  return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

DEVI uint32_t env_rand_u32(uint32_t seed, uint32_t env_id, uint32_t counter, uint32_t stream) {
  uint32_t h = wang_hash(counter * 4u + stream);
  h = wang_hash(h ^ env_id);
  h = wang_hash(h ^ seed);
  return h;
}

#define HIP_LAUNCH_CHECK() (hipGetLastError())

// ---------------------------------------------------------------------------------------------------------------
// Order-independent (bit-reproducible) weight-gradient accumulation: TrainConfig.deterministic with fp32x.
// Every contribution that would meet others in an fp32 atomic is added as an int64 fixed-point number in units of
// 2^-FX_SHIFT instead (global_atomic_add_x2 / ds_add_u64).  Integer addition is associative, so the sum does not
// depend on the order in which workgroups or waves arrive; x3_fx_flush converts it back and adds it to the fp32
// gradient.  fx == nullptr selects the fp32 atomics (the default, non-deterministic mode).
// Resolution 2^-34 ~ 5.8e-11 absolute per contribution; range guard: a contribution of magnitude >= FX_LIMIT (or a
// NaN) sets fx[-1], which the flush turns into the fp32x range flag (runtime.guard.X3RangeError) -- with at most 2^13
// contributions per entry (every kernel here stays below it) the int64 sum cannot wrap.
// ---------------------------------------------------------------------------------------------------------------
#define FX_SHIFT 34
extern long long* g_fx_accum;      // host side: the accumulator of the backward being launched (csrc/trunk_x3.hip)
#define FX_LIMIT 65536.f
DEVI unsigned long long fx_q(float v) { return (unsigned long long)__float2ll_rn(v * 0x1p34f); }
DEVI void fx_guard(long long* fx, float v) {
  if (!(fabsf(v) < FX_LIMIT)) atomicOr(reinterpret_cast<unsigned long long*>(fx - 1), 1ull);
}
// grad[i] += v, many writers
DEVI void gacc(float* grad, long long* fx, long i, float v) {
  if (fx) {
    fx_guard(fx, v);
    atomicAdd(reinterpret_cast<unsigned long long*>(fx + i), fx_q(v));
  } else {
    atomicAdd(grad + i, v);
  }
}
// LDS partial (a workgroup's bias sums): float atomics, or int64 fixed point in the same (8-byte) slots
DEVI void lds_acc(float* f, unsigned long long* q, int i, float v, bool det) {
  if (det) atomicAdd(q + i, fx_q(v));
  else atomicAdd(f + i, v);
}
// fx[i] += q (an LDS fixed-point partial, already quantised), with the same range guard
DEVI void gacc_q(long long* fx, long i, unsigned long long q) {
  const long long s = (long long)q;
  if (s >= (1ll << 50) || s <= -(1ll << 50)) atomicOr(reinterpret_cast<unsigned long long*>(fx - 1), 1ull);
  atomicAdd(reinterpret_cast<unsigned long long*>(fx + i), q);
}
DEVI float fx_f(unsigned long long q) { return (float)((double)(long long)q * 0x1p-34); }
