// PathNet trunk in the fp32-accurate split-operand mode (TrainConfig.compute_dtype = "fp32x").
//
// The reference computes in fp32 (TF default dtype, game_ac_network.py:89-110).  gfx950 has no xf32 MFMA and its
// fp32-input MFMA runs at 1/16 of the bf16 rate, so this mode keeps every value the bf16 engine keeps in 16 bits as
// a PAIR: x = hi + lo, hi = rnd(x), lo = rnd(x - hi), fp16 halves (22 significant bits).  Activations are ReLU sums
// and weights enter as W * 2^8, both far inside fp16's range; output gradients enter as G * 2^e, one power of two per
// layer from the gradient's amax (G16, below).  A product is three MFMAs into one fp32 accumulator,
//     a*b ~ a_hi*b_hi + a_hi*b_lo + a_lo*b_hi          (the dropped a_lo*b_lo term is <= 2^-22 |a*b|)
// so each MFMA k-step costs 3x the bf16 engine's, against 16x for v_mfma_f32_16x16x4_f32 (csrc/trunk_f32.hip).
// Inputs that are exact in 16 bits need two: the uint8 frame stack (exact in fp16) against the fp16 hi/lo pair of
// the first layer's weights, and the same stack against the output gradient's pair in that layer's weight gradient.
// The input gradients accumulate odd k-steps on negated operands in a second chain (X3_DG_FOLD = 2): the f16 MFMA's
// sum is biased toward -inf, which the weight gradients below would otherwise sum coherently
// (profiles/r4/x3_precision.md).
//
// Storage (pathnet_gym_amd/ops/pathnet_ops.py allocates it):
//   activations between layers : the fp16 pair (hi | lo planes of the bf16 engine's layout; kernels take the hi
//                                base and the element offset of the lo plane, xlo / ylo); the forward reads it as
//                                is, the weight gradients convert it to the bf16 pair while staging.  The last
//                                layer writes fp32 (its only consumers are the fp32 heads kernels).
//   activation gradients       : fp32 (masked and split into hi/lo while staging into LDS).
//   weight operand copies      : [2][M][Cout][KP] (hi plane, lo plane), WcT likewise; conv1 [2][M][8][KP] fp16.
// Kernel structure follows the bf16 engine (conv_fast.hip, trunk_fwd.hip, trunk_bwd.hip): the same row tilings,
// LDS layouts and epilogues (bias + ReLU + ReLU bits + module sum), with the B operand and the masked-G staging
// doubled.  LDS holds X3_NCX column tiles (6 modules) per pass; a path with more active modules in a layer runs
// further passes over the same rows (forward: the epilogue adds into the output; weight gradients: separate
// accumulation passes; conv dgrad: 4 slots per pass), so occupancy is sized for the common N = 4 genotypes.
#include "common.h"
#include <type_traits>

namespace x3 {

#define X3_NCX 3          // column tiles (16 = 2 modules x 8 maps) of B / masked G in LDS per pass
#define X3_MAXM 16
#define X3_NCT 5          // column tiles of a full layer (M <= 10)
#define X3_RING_FCS 1024  // frame-ring weight gradient: first-valid-channel bytes staged per workgroup
#define X3_C1_FWD_FCS 128  // frame-ring band forward: first-valid-channel bytes staged per workgroup
#define X3_W0_SHIFT 8     // first-layer weights enter the fp16 MFMA as W * 2^8 (hi/lo pair)

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

struct RowIt {
  int r, t, e, pos;
};
DEVI void rowit_init(RowIt& it, int r, int E, int howo) {
  it.r = r;
  const int s = r / howo;
  it.pos = r - s * howo;
  it.t = s / E;
  it.e = s - it.t * E;
}
DEVI void rowit_adv(RowIt& it, int n, int E, int howo) {
  it.r += n;
  it.pos += n;
  while (it.pos >= howo) {
    it.pos -= howo;
    if (++it.e == E) { it.e = 0; ++it.t; }
  }
}
DEVI long rowit_sample(const RowIt& it, int p, int E, int PE, int t0) {
  return (long)(t0 + it.t) * PE + (long)p * E + it.e;
}

DEVI uint32_t relu_bits_word(const uint64_t (&bal)[4], uint32_t k) {
  uint32_t w = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    w |= __builtin_amdgcn_perm((uint32_t)(bal[r] >> 32), (uint32_t)bal[r],
                               (k << (8 * r)) | (0x0C0C0C0Cu & ~(0xFFu << (8 * r))));
  return w;
}

// ---- split-bf16 helpers ----
typedef __bf16 b2v __attribute__((ext_vector_type(2)));
typedef float f2v_ __attribute__((ext_vector_type(2)));
// hi = RNE bf16(v), lo = RNE bf16(v - hi): one v_cvt_pk_bf16_f32 per PAIR for hi (the scalar form converted each
// value twice: once alone for the residual, once paired for the store), the residual's operand rebuilt from the
// packed word by a shift / mask
// bit C of v sign-extended (0 or ~0): one v_bfe_i32 (written out: the compiler turns the shift form back into a
// compare + select per use)
template <int C>
DEVI uint32_t sbfe1(uint32_t v) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(v), "n"(C));
  return r;
}
// m[c] = bit c of b ? g[c] : 0, as v_bfe_i32 + v_and per value
DEVI void mask8(const float (&g)[8], uint32_t b, float (&m)[8]) {
  const uint32_t mk[8] = {sbfe1<0>(b), sbfe1<1>(b), sbfe1<2>(b), sbfe1<3>(b),
                          sbfe1<4>(b), sbfe1<5>(b), sbfe1<6>(b), sbfe1<7>(b)};
#pragma unroll
  for (int c = 0; c < 8; ++c) m[c] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, g[c]) & mk[c]);
}
// an fp16 pair (hi, lo) of 8 values masked by the ReLU bits b (bit c: channel c): the pair of the masked values, since
// the split of 0 is (0, 0).  Per dword j (channels 2j, 2j+1): the two sign-extended bits joined by one v_perm.
DEVI void mask_pair8(const s8v& hi, const s8v& lo, uint32_t b, s8v& mh, s8v& ml) {
  const uint32_t m[4] = {__builtin_amdgcn_perm(sbfe1<1>(b), sbfe1<0>(b), 0x07060100u),
                         __builtin_amdgcn_perm(sbfe1<3>(b), sbfe1<2>(b), 0x07060100u),
                         __builtin_amdgcn_perm(sbfe1<5>(b), sbfe1<4>(b), 0x07060100u),
                         __builtin_amdgcn_perm(sbfe1<7>(b), sbfe1<6>(b), 0x07060100u)};
  uint32_t h[4], l[4];
  __builtin_memcpy(h, &hi, 16);
  __builtin_memcpy(l, &lo, 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] &= m[j];
    l[j] &= m[j];
  }
  __builtin_memcpy(&mh, h, 16);
  __builtin_memcpy(&ml, l, 16);
}
DEVI void split8(const float (&v)[8], s8v& hi, s8v& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2v_ vv = {v[2 * j], v[2 * j + 1]};
    h[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(vv, b2v));
    const f2v_ bb = {__builtin_bit_cast(float, h[j] << 16), __builtin_bit_cast(float, h[j] & 0xFFFF0000u)};
    l[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(vv - bb, b2v));      // one v_pk_add_f32
  }
  __builtin_memcpy(&hi, h, 16);
  __builtin_memcpy(&lo, l, 16);
}
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
DEVI uint16_t f2h(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
DEVI float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }

// fp16-pair range guard.  An activation stored as an fp16 pair must stay below fp16's largest finite value (65504):
// beyond it the hi half is inf and the pair is garbage.  Every epilogue that writes a pair ORs X3_RANGE_ACT into
// this flag when one of its values is out of range (a branch around one vector atomic, taken only on overflow); the
// weight refresh of the next optimizer step folds it into the status word the host reads
// (HipPathNet.check_x3_status raises X3RangeError).
#define X3_RANGE_W 1u        // a weight * 2^X3_W0_SHIFT left the fp16 range (refresh_x3_kernel)
#define X3_RANGE_ACT 2u      // an activation written as an fp16 pair left the fp16 range (forward epilogues)
#define X3_RANGE_FX 4u       // deterministic mode: a weight-gradient contribution left the fixed-point range (x3_fx_flush)
__device__ uint32_t g_x3_range;
DEVI bool x3_oor(float v) { return !(fabsf(v) < 65504.f); }     // NaN counts as out of range
DEVI void x3_flag_range(bool bad) {
  if (bad) atomicOr(&g_x3_range, X3_RANGE_ACT);
}
// An activation between layers is stored as its fp16 pair in two 16-bit planes, ylo elements apart (22 significant
// bits; the next layer's forward reads it as is).  The weight gradients meet it with the output gradient, which needs
// bf16's exponent range, so they convert it to the bf16 pair while staging (x16pair_to_bf16pair).
DEVI void st_x4(uint16_t* Y, long ylo, long i, float v) {
  x3_flag_range(x3_oor(v));
  const uint16_t h = f2h(v);
  Y[i] = h;
  Y[i + ylo] = f2h(v - h2f(h));
}
DEVI float ld_x4(const uint16_t* Y, long ylo, long i) { return h2f(Y[i]) + h2f(Y[i + ylo]); }
DEVI void st8_x4(uint16_t* Y, long ylo, const float (&o)[8]) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) bad |= x3_oor(o[j]);
  x3_flag_range(bad);
  s8v a, b;
  split8h(o, a, b);
  *reinterpret_cast<s8v*>(Y) = a;
  *reinterpret_cast<s8v*>(Y + ylo) = b;
}
// 8 values as an fp16 pair (hi, lo) -> the bf16 pair of their fp32 sum
DEVI void x16pair_to_bf16pair(const s8v& h, const s8v& l, s8v& bh, s8v& bl) {
  const h8v hh = __builtin_bit_cast(h8v, h), ll = __builtin_bit_cast(h8v, l);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)hh[j] + (float)ll[j];
  split8(v, bh, bl);
}
// a*b over one 32-wide k-step from hi/lo operands: the two small cross terms first
DEVI f4v mma3(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16(al, bh, c);
  c = mfma16(ah, bl, c);
  return mfma16(ah, bh, c);
}
// the same on fp16 pairs (forward: activations x weights * 2^8)
DEVI f4v mma3h(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16_f16(al, bh, c);
  c = mfma16_f16(ah, bl, c);
  return mfma16_f16(ah, bh, c);
}
// the same products with the weights as the A operand (D = [columns][rows], conv_epi_sw), in mma3h's order
DEVI f4v mma3h_t(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16_f16(bh, al, c);
  c = mfma16_f16(bl, ah, c);
  return mfma16_f16(bh, ah, c);
}
// exact operand a (uint8 pixels in bf16) against a hi/lo pair b
DEVI f4v mma2(const s8v& a, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16(a, bl, c);
  return mfma16(a, bh, c);
}
// exact operand a (uint8 pixels in fp16) against an fp16 pair b
DEVI f4v mma2h(const s8v& a, const s8v& bh, const s8v& bl, f4v c) {
  c = mfma16_f16(a, bl, c);
  return mfma16_f16(a, bh, c);
}

// ---- scaled fp16-pair gradients ("G16") ----
// Every output gradient G of a trunk layer enters the backward GEMMs as the fp16 pair of G * 2^e, one power of two per
// layer and update chosen from the tensor's largest magnitude (amax) so that amax * 2^e lies in [2^13, 2^14): 22
// significant bits down to amax * 2^-27 (the bf16 pair kept 16), on the f16 MFMA at the bf16 rate, and the
// activation operands (already fp16 pairs) need no conversion.  The producer of G writes its amax: x3_amax for the
// last layer's input gradient (heads / LSTM), the input-gradient epilogues (conv_dgrad_x3, fc_dgrad_gemm_x3,
// fc_dgrad_x3) for the layer below; float bits of non-negative values order like unsigned ints, so one
// atomicMax per wave (per workgroup for elementwise producers).  scripts/x3_numerics.py: per-layer weight-gradient
// error 1.1-1.8e-5 with bf16 pairs -> 2-3e-7 in float64 emulation.
DEVI float g16_scale(const float* amax) {
  const uint32_t b = __float_as_uint(*amax);
  const int e = (int)((b >> 23) & 0xFFu) - 127;           // floor(log2 amax) (normal amax)
  if ((b & 0x7FFFFFFFu) == 0u || e < -110 || e >= 128) return 1.0f;   // zero / tiny / non-finite: unscaled
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
// 8 values * s -> fp16 pair
DEVI void split8hs(const float (&v)[8], float s, s8v& hi, s8v& lo) {
  float t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = v[j] * s;
  split8h(t, hi, lo);
}

// 8 x uint8 -> 8 x fp16 holding the exact pixel value: fp16(1024 + v) built by v_perm, minus 1024 (exact)
DEVI s8v u8x8_to_f16(uint2 v) {
  h8v x = __builtin_bit_cast(h8v, u8x8_to_f16off(v));
  x = x - (h8v){(_Float16)1024.f, (_Float16)1024.f, (_Float16)1024.f, (_Float16)1024.f,
                (_Float16)1024.f, (_Float16)1024.f, (_Float16)1024.f, (_Float16)1024.f};
  return __builtin_bit_cast(s8v, x);
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

// ---- conv forward epilogue, swapped MFMA orientation (weights as the A operand, im2col rows as B) ----
// acc[ct] = D[16 output columns][16 rows]: lane (q, c16) holds columns 4q..4q+3 of column tile ct -- slot
// 2*(ct0+ct) + (q>>1), channels 4*(q&1) + r -- for row c16, i.e. four consecutive channels of one row.  Compared with
// rows-as-A (lane = one channel of four rows) the module-pair sum is one xor-32 exchange, the ReLU-bit byte of a
// (slot, row) is two lanes' nibbles (no ballot transposes), and each lane writes its four channels of one plane as
// one 8-byte store (hi plane: q < 2, lo plane: q >= 2) instead of 16 two-byte stores.  Same arithmetic and summation
// order as the rows-as-A epilogue: bit-identical outputs.
template <int NC>
DEVI void conv_epi_sw(const f4v (&acc)[NC], const float* bias_s, int ct0, int cnt, int q, float in_scale,
                      float out_scale, long grow, uint8_t* __restrict__ bits, long bits_rows,
                      uint16_t* __restrict__ Y, long ylo, bool accumulate, bool valid = true) {
  float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ct = 0; ct < NC; ++ct) {
    const float4 bb = *reinterpret_cast<const float4*>(bias_s + ct * 16 + 4 * q);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
    uint32_t nib = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = acc[ct][r] * in_scale + bv[r];
      const bool pos = v > 0.f;
      sum[r] += pos ? v : 0.f;
      nib |= pos ? (1u << r) : 0u;
    }
    // channels 4..7 of the same slot and row: lane l ^ 16.  v_permlane16_swap (x, x) leaves row 2k+1's values in the
    // SECOND result's row 2k, which is what the lanes that store the byte (rows 0 and 2: q even) need -- one VALU op
    // instead of a ds_bpermute round trip
    const uint32_t hi4 = __builtin_amdgcn_permlane16_swap(nib, nib, false, false)[1];
    const int slot = (ct0 + ct) * 2 + (q >> 1);
    if ((q & 1) == 0 && slot < cnt && valid) bits[(long)slot * bits_rows + grow] = (uint8_t)(nib | (hi4 << 4));
  }
  // + the other slot of each pair (lane l ^ 32): v_permlane32_swap (x, x) gives {lanes 0-31's half, lanes 32-63's
  // half} on every lane; their sum is the same float addition as the shuffle's in either order (bit-identical)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_uint(sum[r]), __float_as_uint(sum[r]), false, false);
    sum[r] = __uint_as_float(pr[0]) + __uint_as_float(pr[1]);
  }
  float y[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) y[r] = sum[r] * out_scale;
  if (!valid) return;                            // (after the exchanges: every lane took part in them)
  const long o = grow * 8 + 4 * (q & 1);
  if (accumulate) {
    const uint2 ph = *reinterpret_cast<const uint2*>(Y + o), pl = *reinterpret_cast<const uint2*>(Y + ylo + o);
    const uint32_t hw[4] = {ph.x & 0xFFFFu, ph.x >> 16, ph.y & 0xFFFFu, ph.y >> 16};
    const uint32_t lw[4] = {pl.x & 0xFFFFu, pl.x >> 16, pl.y & 0xFFFFu, pl.y >> 16};
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] += h2f((uint16_t)hw[r]) + h2f((uint16_t)lw[r]);
  }
  x3_flag_range(x3_oor(y[0]) || x3_oor(y[1]) || x3_oor(y[2]) || x3_oor(y[3]));
  const h2v h01 = __builtin_convertvector((f2v){y[0], y[1]}, h2v);
  const h2v h23 = __builtin_convertvector((f2v){y[2], y[3]}, h2v);
  uint2 out;
  if (q < 2) {
    out = make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
  } else {
    const h2v l01 = __builtin_convertvector((f2v){y[0] - (float)h01[0], y[1] - (float)h01[1]}, h2v);
    const h2v l23 = __builtin_convertvector((f2v){y[2] - (float)h23[0], y[3] - (float)h23[1]}, h2v);
    out = make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
  }
  *reinterpret_cast<uint2*>(Y + (q < 2 ? 0 : ylo) + o) = out;
}

// ===========================================================================
// first layer forward (uint8 frame stack, 8x8/s4, 160x120x4): fp16 MFMA, exact pixels x (W*2^8) hi/lo pair.
// grid = (ceil(T*E*HOWO / (NT*128)), P), 256 threads; each wave owns 32-row tiles (2 MFMA row tiles) and walks
// NT of them with the bf16 engine's one-register-set reload pipeline (conv_fast.hip conv_fwd_fast AFF8 path):
// a k-step's raw bytes are converted, the same registers are reloaded with the next tile's k-step, then the MFMAs.
// Wh: [2][M][8][KP] fp16 (hi plane, lo plane at +wlo).  Y: two bf16 planes (lo at +ylo).
// ===========================================================================
template <class G, int NT, int LB, bool SW>
__global__ __launch_bounds__(256, LB) void conv1_fwd_x2(const uint8_t* __restrict__ X, uint16_t* __restrict__ Y,
                                                      long ylo, uint8_t* __restrict__ bits,
                                                      const uint16_t* __restrict__ Wh, long wlo,
                                                      const float* __restrict__ flat, long bias_off, int chunk,
                                                      const int* __restrict__ act_idx,
                                                      const int* __restrict__ act_cnt, int layer, int L, int M, int P,
                                                      int E, int T, int t0, long bits_rows, float in_scale,
                                                      float out_scale) {
  static_assert(G::U8 && G::KW * G::CIN == 32 && G::K == G::KP, "affine uint8 first-layer geometry");
  constexpr int KPs = G::KP + 8;
  constexpr int NK = G::KP / 32;
  constexpr int FF_ROWS = NT * 128;
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2][X3_NCX * 16 * KPs];
  __shared__ __attribute__((aligned(16))) float bias_s[X3_NCX * 16];
  __shared__ float wsum_s[X3_NCX * 16];
  __shared__ int mods[X3_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  const int Rtot = T * E * G::HOWO;
  const int PE = P * E;
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
  const uint32_t bkey = (uint32_t)(2 * q + h);
  const bool lin = T == 1;
  // SW: pixels enter the MFMA as fp16(1024 + v) straight from v_perm (no per-element subtraction); the offset's
  // contribution 1024 * sum_k W[col][k] is taken out of the bias (wsum_s: the fp32 sum of the staged fp16 pair)
  static_assert(!SW || G::KC == 32, "SW weight-sum reduction: one column per 32 lanes");
  const long rowbase = ((long)t0 * PE + (long)p * E) * G::HOWO;
  const int rfirst = blockIdx.x * FF_ROWS + w * 32;
  const int npass = nct > X3_NCX ? (nct + X3_NCX - 1) / X3_NCX : 1;
  RowIt ait[2], eit[2];
  uint2 araw[2][NK];
  const uint8_t* asrc[2];
  // rows past the end read row 0 of the path's first sample: their 16-row halves are never stored
  auto aff_addr = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool va = ait[i].r < Rtot;
      const int oh = ait[i].pos / G::WO, ow = ait[i].pos - oh * G::WO;
      const long xb = va ? rowit_sample(ait[i], p, E, PE, t0) * (long)G::IN_ELEMS +
                               (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN
                         : rowit_sample(RowIt{0, 0, 0, 0}, p, E, PE, t0) * (long)G::IN_ELEMS;
      asrc[i] = X + xb + G::koff(grp);
      rowit_adv(ait[i], 128, E, G::HOWO);
    }
  };
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * X3_NCX;
    const int ncg = nct == 0 ? 1 : min(X3_NCX, nct - ct0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rowit_init(ait[i], rfirst + i * 16 + c16, E, G::HOWO);
      rowit_init(eit[i], rfirst + i * 16 + (SW ? c16 : 4 * q), E, G::HOWO);
    }
    // the first tile's A loads do not depend on LDS: issued before the staging barriers
    aff_addr();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) araw[i][kk] = *reinterpret_cast<const uint2*>(asrc[i] + kk * G::WIN * G::CIN);
    __syncthreads();       // mods visible / the previous pass's LDS reads done
    for (int i = tid; i < ncg * 16 * G::KC; i += 256) {
      const int col = i / G::KC, kc = i - col * G::KC;
      const int slot = ct0 * 2 + (col >> 3);
      s8v vh = {0, 0, 0, 0, 0, 0, 0, 0}, vl = vh;
      if (slot < cnt) {
        const long o = ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8;
        vh = *reinterpret_cast<const s8v*>(Wh + o);
        vl = *reinterpret_cast<const s8v*>(Wh + wlo + o);
      }
      *reinterpret_cast<s8v*>(Ws[0] + col * KPs + kc * 8) = vh;
      *reinterpret_cast<s8v*>(Ws[1] + col * KPs + kc * 8) = vl;
      if constexpr (SW) {
        const h8v hh = __builtin_bit_cast(h8v, vh), ll = __builtin_bit_cast(h8v, vl);
        float ws = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ws += (float)hh[j] + (float)ll[j];
#pragma unroll
        for (int m = 16; m >= 1; m >>= 1) ws += __shfl_xor(ws, m, 64);
        if (kc == 0) wsum_s[col] = ws;
      }
    }
    __syncthreads();
    if (tid < ncg * 16) {
      const int slot = ct0 * 2 + (tid >> 3);
      const float b = slot < cnt ? flat[bias_off + (long)mods[slot] * chunk + (tid & 7)] : 0.f;
      bias_s[tid] = SW ? b - in_scale * 1024.f * wsum_s[tid] : b;
    }
    __syncthreads();
    auto run = [&](auto ncc) {
      constexpr int NC = decltype(ncc)::value;
      auto do_tile = [&](const int rbase, auto reload_c) {
        constexpr bool RELOAD = decltype(reload_c)::value;
        f4v acc[2][NC];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (RELOAD) aff_addr();
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const s8v a0 = SW ? u8x8_to_f16off(araw[0][kk]) : u8x8_to_f16(araw[0][kk]);
          const s8v a1 = SW ? u8x8_to_f16off(araw[1][kk]) : u8x8_to_f16(araw[1][kk]);
          if constexpr (RELOAD) {
            araw[0][kk] = *reinterpret_cast<const uint2*>(asrc[0] + kk * G::WIN * G::CIN);
            araw[1][kk] = *reinterpret_cast<const uint2*>(asrc[1] + kk * G::WIN * G::CIN);
          }
          const int kc = kk * 4 + grp;
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const s8v bh = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
            const s8v bl = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
            if constexpr (SW) {
              acc[0][ct] = mfma16_f16(bl, a0, acc[0][ct]);
              acc[0][ct] = mfma16_f16(bh, a0, acc[0][ct]);
              acc[1][ct] = mfma16_f16(bl, a1, acc[1][ct]);
              acc[1][ct] = mfma16_f16(bh, a1, acc[1][ct]);
            } else {
              acc[0][ct] = mfma16_f16(a0, bl, acc[0][ct]);
              acc[0][ct] = mfma16_f16(a0, bh, acc[0][ct]);
              acc[1][ct] = mfma16_f16(a1, bl, acc[1][ct]);
              acc[1][ct] = mfma16_f16(a1, bh, acc[1][ct]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r16 = rbase + i * 16;
          long grow4;
          if (lin) {
            grow4 = rowbase + r16 + (SW ? c16 : 4 * q);
          } else {
            const RowIt e0 = eit[i];
            rowit_adv(eit[i], 128, E, G::HOWO);
            grow4 = rowit_sample(e0, p, E, PE, t0) * G::HOWO + e0.pos;
          }
          if (r16 >= Rtot) continue;
          if constexpr (SW) {
            conv_epi_sw<NC>(acc[i], bias_s, ct0, cnt, q, in_scale, out_scale, grow4, bits, bits_rows, Y, ylo, pass > 0);
            continue;
          }
          float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const int slot = (ct0 + ct) * 2 + h;
            const float bb = bias_s[ct * 16 + c16];
            uint64_t bal[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = acc[i][ct][r] * in_scale + bb;
              const bool pos = v > 0.f;
              sum[r] += pos ? v : 0.f;
              bal[r] = __ballot(pos);
            }
            const uint32_t word = relu_bits_word(bal, bkey);
            if (ch == 0 && slot < cnt) *reinterpret_cast<uint32_t*>(bits + (long)slot * bits_rows + grow4) = word;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
          if (h == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const long o = (grow4 + r) * 8 + ch;
              float y = sum[r] * out_scale;
              if (pass > 0) y += ld_x4(Y, ylo, o);
              st_x4(Y, ylo, o, y);
            }
          }
        }
      };
      int tile = 0;
#pragma unroll
      for (; tile + 1 < NT; ++tile) {
        const int rbase = rfirst + tile * 128;
        if (rbase + 128 >= Rtot) break;
        do_tile(rbase, std::true_type{});
      }
      const int rbase = rfirst + tile * 128;
      if (rbase < Rtot) do_tile(rbase, std::false_type{});
    };
    switch (ncg) {
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      default: run(std::integral_constant<int, 3>{}); break;
    }
  }
}

// ===========================================================================
// first layer forward with the input BAND in LDS: a stage = 8 output rows of one sample (232 positions), whose 36
// input rows (17 KB of uint8) are copied into LDS with coalesced 16-byte loads while the previous band computes;
// every pixel fragment is then one conflict-free ds_read_b64 (2 pixels x 4 channels) instead of conv1_fwd_x2's
// 8-byte global loads (each input byte fetched 4 times through L2, the kernel waiting on them at 2 waves/SIMD).
// Pixels enter as fp16(1024 + v) (v_perm) with the offset folded into the bias, weights (W * 2^8 hi/lo pair) as
// the MFMA A operand, conv_epi_sw epilogue.  Passes of <= 2 column tiles (4 modules) keep LDS at 2 x 17.3 KB +
// 33.8 KB so two workgroups share a CU.  grid = (chunks of bands, P).
// ===========================================================================
template <class G>
struct BD1 {
  static constexpr int OBR = 8;                                  // output rows per band
  static constexpr int NB = (G::HO + OBR - 1) / OBR;             // bands per sample (5; the last has 7 rows)
  static constexpr int IR = (OBR - 1) * G::S + G::KH;            // input rows per band (36)
  static constexpr int RB = G::WIN * G::CIN;                     // bytes per input row (480)
  static constexpr int BYTES = IR * RB;                          // 17 280
  static constexpr int NCH = BYTES / 16;                         // 16-byte chunks (1 080)
  static constexpr int CIT = (NCH + 255) / 256;
  static constexpr int NPOS = OBR * G::WO;                       // 232
  static constexpr int NRT = (NPOS + 15) / 16;                   // 15 position tiles
  static_assert(BYTES % 16 == 0 && G::U8 && G::KW * G::CIN == 32 && G::K == G::KP, "uint8 first-layer geometry");
};

// channel planes -> packed pixels: v.x .. v.w are 4 pixels of channel planes 0..3; returns the 4 pixels as
// (c0, c1, c2, c3) byte words, the packed-stack layout (a 4x4 byte transpose, 8 v_perm_b32)
DEVI uint4 planes_to_px4(uint4 v) {
  const uint32_t t0 = __builtin_amdgcn_perm(v.y, v.x, 0x05010400u);   // A0 B0 A1 B1
  const uint32_t t1 = __builtin_amdgcn_perm(v.y, v.x, 0x07030602u);   // A2 B2 A3 B3
  const uint32_t t2 = __builtin_amdgcn_perm(v.w, v.z, 0x05010400u);   // C0 D0 C1 D1
  const uint32_t t3 = __builtin_amdgcn_perm(v.w, v.z, 0x07030602u);   // C2 D2 C3 D3
  return make_uint4(__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
                    __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u));
}

// RING: X is the frame ring [P*E][nslots][HIN*WIN] uint8 (runtime/engine.py frame_ring); channel c of sample (t, b)
// is frame slot t + max(c, fcv[t][b]) of env b.  A staging chunk is then 4 pixels of each of the 4 planes (four
// coalesced 4-byte loads) transposed into the packed (pixel, channel) layout at LDS-write time, so the band in LDS
// and every MFMA operand read are those of the packed-stack kernel.
// PIPE: the next k-step's pixel and weight fragments are read from LDS while this k-step's MFMAs run (one k-step of
// fragments ahead instead of a wait on every k-step's reads)
// F16B: the band is converted to fp16 (1024 + v) ONCE while it is staged (single LDS buffer of 2 x 17.3 KB, one more
// barrier per band) instead of per MFMA operand read: every pixel of an 8x8/s4 band feeds 4 positions x 2 kernel
// rows, so the per-read conversion (v_perm per 2 pixels) ran ~4x per pixel
// SB1: ONE uint8 band buffer (17.3 KB; one more barrier per band, like F16B) so that the workgroup's 51 KB of LDS
// lets three workgroups share a CU (3 waves / SIMD, <= 168 VGPRs) instead of two
#ifndef X3_C1_EARLY_BAND
#define X3_C1_EARLY_BAND 1
#endif
// Cost-balanced 1-D schedule over the (path, item) units of P paths x n items, a unit of path p costing
// cost(act_cnt[p]) (>= 1): called by ONE wave (all 64 lanes), it writes to sched the range of workgroup blockIdx.x of
// gridDim.x -- from (sched[0], sched[1]) up to, not including, (sched[2], sched[3]) -- the blockIdx.x-th equal share of
// the population's total cost, rounded down to unit boundaries (consecutive workgroups' ranges tile the units).
// mods_out (optional): the first segment's path's active-module list is loaded into it and its count written to
// sched[4] (-1: not prefetched), so the kernel's first segment skips two dependent global loads.
template <class CostF>
DEVI void bal_schedule(const int* __restrict__ act_cnt, int L, int layer, int P, int n, CostF cost, int* sched,
                       const int* __restrict__ act_idx = nullptr, int M = 0, int* mods_out = nullptr) {
  const int l = threadIdx.x & 63;
  if (mods_out && l == 0) sched[4] = -1;
  if (P <= 64) {
    // one chunk (every population of <= 64 paths per GPU): one act_cnt load per lane, one scan, 32-bit arithmetic
    // while the cost bound fits (the schedule is a serial prologue: at 8 paths a launch lasts ~20 us)
    const int craw = l < P ? act_cnt[l * L + layer] : 0;
    const int np = l < P ? cost(craw) : 0;
    int x = np * n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (l >= d) x += y;
    }
    const int U = __shfl(x, 63, 64), excl = x - np * n;
    int ca, cb;
    if ((long)U * gridDim.x < (1L << 31)) {
      ca = (int)((unsigned)U * blockIdx.x / gridDim.x);
      cb = (int)((unsigned)U * (blockIdx.x + 1) / gridDim.x);
    } else {
      ca = (int)((long)U * blockIdx.x / gridDim.x);
      cb = (int)((long)U * (blockIdx.x + 1) / gridDim.x);
    }
    if (np > 0 && ca >= excl && ca < x) {
      sched[0] = l;
      sched[1] = (ca - excl) / np;
    }
    if (np > 0 && cb >= excl && cb < x) {
      sched[2] = l;
      sched[3] = (cb - excl) / np;
    }
    if (l == 0 && cb >= U) {
      sched[2] = P - 1;
      sched[3] = n;
    }
    if (mods_out) {
      const unsigned long long hit = __ballot(np > 0 && ca >= excl && ca < x);
      if (hit) {
        const int src = __ffsll((long long)hit) - 1;
        const int p0 = __shfl(l, src, 64), c0 = __shfl(craw, src, 64);
        if (l < X3_MAXM) mods_out[l] = l < c0 ? act_idx[(p0 * L + layer) * M + l] : 0;
        if (l == 0) sched[4] = c0;
      }
    }
    return;
  }
  int tot = 0;
  for (int pb = 0; pb < P; pb += 64) {
    int c = pb + l < P ? cost(act_cnt[(pb + l) * L + layer]) : 0;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
    tot += c;
  }
  const long U = (long)tot * n;
  const long ca = U * blockIdx.x / gridDim.x, cb = U * (blockIdx.x + 1) / gridDim.x;
  long base = 0;
  for (int pb = 0; pb < P; pb += 64) {
    const int pp = pb + l;
    const int np = pp < P ? cost(act_cnt[pp * L + layer]) : 0;
    int x = np * n;                                    // inclusive scan of the paths' costs in this chunk
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (l >= d) x += y;
    }
    const long incl = base + x, excl = incl - (long)np * n;
    if (np > 0 && ca >= excl && ca < incl) {
      sched[0] = pp;
      sched[1] = (int)((ca - excl) / np);
    }
    if (np > 0 && cb >= excl && cb < incl) {
      sched[2] = pp;
      sched[3] = (int)((cb - excl) / np);
    }
    base += __shfl(x, 63, 64);
  }
  if (l == 0 && cb >= U) {
    sched[2] = P - 1;
    sched[3] = n;
  }
}

// BAL: cost-balanced schedule.  A path of 5-6 active modules runs two passes over its bands (NCXT = 2 column tiles per
// pass), so with one fixed band range per (workgroup, path) its workgroups took twice as long as the others and the
// launch waited on them (reference preset: 95 -> 162 us per step once the GA grew one path to 5 modules).  With BAL
// the grid is 1-D and workgroup w takes the w-th equal share of the population's total cost (a band of path p costs
// its pass count), i.e. a contiguous run of (path, band) units that may span paths; all passes of a band stay in one
// workgroup, in order (pass > 0 adds into Y), so the output is bit-identical to the per-path grid.
DEVI int c1_npass(int cnt) {
  const int nct = (cnt + 1) >> 1;
  return nct > 2 ? (nct + 1) / 2 : 1;
}

template <class G, bool RING = false, bool PIPE = false, bool F16B = false, bool SB1 = false, bool BAL = false>
__global__ __launch_bounds__(256, SB1 ? 3 : 2) void conv1_fwd_band_x2(const uint8_t* __restrict__ X, uint16_t* __restrict__ Y,
                                                           long ylo, uint8_t* __restrict__ bits,
                                                           const uint16_t* __restrict__ Wh, long wlo,
                                                           const float* __restrict__ flat, long bias_off, int chunk,
                                                           const int* __restrict__ act_idx,
                                                           const int* __restrict__ act_cnt, int layer, int L, int M,
                                                           int P, int E, int T, int t0, long bits_rows,
                                                           int bands_per_wg, float in_scale, float out_scale,
                                                           const uint8_t* __restrict__ fcv = nullptr, int nslots = 0,
                                                           int rbase = 0) {
  using B = BD1<G>;
  constexpr int KPs = G::KP + 8;
  constexpr int NK = G::KP / 32;
  constexpr int NCXT = 2;
  static_assert(!(F16B && PIPE) && !(SB1 && (F16B || PIPE)), "F16B / SB1: plain k loop, one band buffer");
  constexpr bool ONEBUF = F16B || SB1;
  __shared__ __attribute__((aligned(16))) uint8_t Xb[ONEBUF ? 1 : 2][F16B ? 2 * B::BYTES : B::BYTES];
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2][NCXT * 16 * KPs];
  __shared__ __attribute__((aligned(16))) float bias_s[NCXT * 16];
  __shared__ float wsum_s[NCXT * 16];
  __shared__ int mods[X3_MAXM];
  // RING: the first-valid channel of every sample of the workgroup's bands, staged once.  Read per band from global
  // memory it put a dependent byte load (and a full vmcnt wait) in front of every band's frame loads.
  __shared__ uint8_t fcs[RING ? X3_C1_FWD_FCS : 1];
  __shared__ int sched[5];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp;
  const int PE = P * E;
  const int nbands = T * E * B::NB;
  // this workgroup's units: (path, band) from (seg_p0, seg_b0) up to, not including, (seg_p1, seg_b1)
  int seg_p0, seg_b0, seg_p1, seg_b1, pre_cnt = -1;
  if constexpr (BAL) {
    if (w == 0) bal_schedule(act_cnt, L, layer, P, nbands, [](int c) { return c1_npass(c); }, sched, act_idx, M, mods);
    __syncthreads();
    seg_p0 = __builtin_amdgcn_readfirstlane(sched[0]);     // uniform: SGPRs, scalar address math
    seg_b0 = __builtin_amdgcn_readfirstlane(sched[1]);
    seg_p1 = __builtin_amdgcn_readfirstlane(sched[2]);
    seg_b1 = __builtin_amdgcn_readfirstlane(sched[3]);
    pre_cnt = __builtin_amdgcn_readfirstlane(sched[4]);
    if (seg_p0 == seg_p1 && seg_b0 >= seg_b1) return;
  } else {
    seg_p0 = seg_p1 = blockIdx.y;
    seg_b0 = blockIdx.x * bands_per_wg;
    seg_b1 = min(nbands, seg_b0 + bands_per_wg);
    if (seg_b0 >= seg_b1) return;
  }
  int p = seg_p0, cnt = 0, nct = 0, b_beg = 0, b_end = 0, s_first = 0;
  static_assert(B::CIT == 5, "five named staging registers");
  uint4 rg0, rg1, rg2, rg3, rg4;                       // (an indexed array captured by the lambdas went to scratch)
  // band u -> (sample s = u / NB, first output row oh0 = (u % NB) * OBR); the last band's rows past HO read the
  // sample's own last input rows (clamped) and are never stored.  Chunks past NCH reload chunk NCH - 1 (harmless).
  auto band_src = [&](int u, int j) {
    const int s = u / B::NB, oh0 = (u - s * B::NB) * B::OBR;
    const int c = min(tid + 256 * j, B::NCH - 1);
    const int r = c / (B::RB / 16), cc = c - r * (B::RB / 16);
    const int ir = min(oh0 * G::S + r, G::HIN - 1);
    return reinterpret_cast<const uint4*>(X + sample_global(p, s, E, PE, t0) * (long)G::IN_ELEMS + (long)ir * B::RB +
                                          cc * 16);
  };
  // RING: the 4 plane words of chunk j of band u (rg = {c0, c1, c2, c3} words of 4 pixels).  Measured: 8 pixels
  // per plane and chunk (3 chunks per thread, two 16-byte LDS stores 32 bytes apart) ran 98.8-100.2 vs 97.4 us
  auto ring_src = [&](int u, int j) {
    const int s = u / B::NB, oh0 = (u - s * B::NB) * B::OBR;
    const int st = s / E, e = s - st * E;
    const int fc = (int)fcs[s - s_first];
    const int c = min(tid + 256 * j, B::NCH - 1);
    const int r = c / (G::WIN / 4), cc = c - r * (G::WIN / 4);
    const int ir = min(oh0 * G::S + r, G::HIN - 1);
    constexpr long HW = (long)G::HIN * G::WIN;
    // modular ring: channel k of step t lives in slot (rbase + t + max(k, fc)) mod nslots (runtime/engine.py)
    const uint8_t* src = X + (long)(p * E + e) * nslots * HW + (long)ir * G::WIN + cc * 4;
    const int s0 = rbase + t0 + st;
    auto pl = [&](int k) {
      int sl = s0 + max(k, fc);
      sl -= sl >= nslots ? nslots : 0;
      return *reinterpret_cast<const uint32_t*>(src + sl * HW);
    };
    return make_uint4(pl(0), pl(1), pl(2), pl(3));
  };
  auto load_band = [&](int u) {
    if constexpr (RING) {
      rg0 = ring_src(u, 0);
      rg1 = ring_src(u, 1);
      rg2 = ring_src(u, 2);
      rg3 = ring_src(u, 3);
      rg4 = ring_src(u, 4);
    } else {
      rg0 = *band_src(u, 0);
      rg1 = *band_src(u, 1);
      rg2 = *band_src(u, 2);
      rg3 = *band_src(u, 3);
      rg4 = *band_src(u, 4);
    }
  };
  auto px = [&](const uint4& v) {
    if constexpr (RING) return planes_to_px4(v);
    else return v;
  };
  auto put = [&](int buf, int c, const uint4& v) {
    if constexpr (F16B) {                           // 16 pixel bytes -> 16 fp16 (1024 + v), 32 bytes
      const uint4 q = px(v);
      *reinterpret_cast<s8v*>(&Xb[0][c * 32]) = u8x8_to_f16off(make_uint2(q.x, q.y));
      *reinterpret_cast<s8v*>(&Xb[0][c * 32 + 16]) = u8x8_to_f16off(make_uint2(q.z, q.w));
    } else {
      *reinterpret_cast<uint4*>(&Xb[buf][c * 16]) = px(v);
    }
  };
  auto store_band = [&](int buf) {
    put(buf, tid, rg0);
    put(buf, tid + 256, rg1);
    put(buf, tid + 512, rg2);
    put(buf, tid + 768, rg3);
    if (tid + 1024 < B::NCH) put(buf, tid + 1024, rg4);
  };


  // segments: one path's run of bands, at most X3_C1_FWD_FCS - 2 samples (the staged fc bytes) at a time
  constexpr int MAXB = (X3_C1_FWD_FCS - 2) * B::NB;
  for (int sp = seg_p0; sp <= seg_p1; ++sp)
  for (int cb = sp == seg_p0 ? seg_b0 : 0, ce = sp == seg_p1 ? seg_b1 : nbands; cb < ce; cb += MAXB) {
  p = sp;
  b_beg = cb;
  b_end = min(ce, cb + MAXB);
  if (sp != seg_p0 || cb != seg_b0) __syncthreads();  // the previous segment's LDS reads (mods, fcs, Ws, Xb) done
  if (BAL && pre_cnt >= 0 && sp == seg_p0 && cb == seg_b0) {
    cnt = pre_cnt;                                     // mods prefetched by the schedule wave
  } else {
    cnt = act_cnt[p * L + layer];
    if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  }
  nct = (cnt + 1) >> 1;
  s_first = b_beg / B::NB;
  if constexpr (RING) {
    const int ns = (b_end - 1) / B::NB - s_first + 1;     // <= X3_C1_FWD_FCS (launcher caps bands_per_wg)
    for (int i = tid; i < ns; i += 256) {
      const int s = s_first + i, st = s / E, e = s - st * E;
      fcs[i] = fcv[(long)(t0 + st) * PE + (long)p * E + e];
    }
  }
  const int npass = nct > NCXT ? (nct + NCXT - 1) / NCXT : 1;
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * NCXT;
    const int ncg = nct == 0 ? 1 : min(NCXT, nct - ct0);
    __syncthreads();                                   // mods (and fcs) visible; the previous pass's LDS reads done
    // the first band's loads go out before the weight staging's, so the two global latencies overlap (the staging
    // loop's waits then cover both)
    if (X3_C1_EARLY_BAND) load_band(b_beg);
    static_assert(G::KC == 32, "weight-sum reduction: one column per 32 lanes");
    for (int i = tid; i < ncg * 16 * G::KC; i += 256) {
      const int col = i / G::KC, kc = i - col * G::KC;
      const int slot = ct0 * 2 + (col >> 3);
      s8v vh = {0, 0, 0, 0, 0, 0, 0, 0}, vl = vh;
      if (slot < cnt) {
        const long o = ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8;
        vh = *reinterpret_cast<const s8v*>(Wh + o);
        vl = *reinterpret_cast<const s8v*>(Wh + wlo + o);
      }
      *reinterpret_cast<s8v*>(Ws[0] + col * KPs + kc * 8) = vh;
      *reinterpret_cast<s8v*>(Ws[1] + col * KPs + kc * 8) = vl;
      const h8v hh = __builtin_bit_cast(h8v, vh), ll = __builtin_bit_cast(h8v, vl);
      float ws = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ws += (float)hh[j] + (float)ll[j];
#pragma unroll
      for (int m = 16; m >= 1; m >>= 1) ws += __shfl_xor(ws, m, 64);
      if (kc == 0) wsum_s[col] = ws;
    }
    if (!X3_C1_EARLY_BAND) load_band(b_beg);
    __syncthreads();
    if (tid < ncg * 16) {
      const int slot = ct0 * 2 + (tid >> 3);
      const float b = slot < cnt ? flat[bias_off + (long)mods[slot] * chunk + (tid & 7)] : 0.f;
      bias_s[tid] = b - in_scale * 1024.f * wsum_s[tid];
    }
    store_band(0);
    auto run = [&](auto ncc) {
      constexpr int NC = decltype(ncc)::value;
      int buf = 0;
      for (int u = b_beg; u < b_end; ++u, buf ^= (ONEBUF ? 0 : 1)) {
        __syncthreads();                               // band u in LDS (and bias_s); buf ^ 1 free
        if (u + 1 < b_end) load_band(u + 1);
        const int s = u / B::NB, oh0 = (u - s * B::NB) * B::OBR;
        const long growb = sample_global(p, s, E, PE, t0) * G::HOWO + (long)oh0 * G::WO;
        const uint8_t* xb = Xb[buf];
        // wave w: position tiles 4w .. 4w+3 (64 positions); every weight fragment read from LDS feeds 4 tiles x 2
        // MFMAs (one tile per read made the kernel bound by LDS bandwidth: 124 vs 108 us)
        static_assert(B::NRT <= 16, "4 waves x 4 position tiles");
        int abase[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pos = (4 * w + i) * 16 + c16;      // band-local position of this lane's column
          const int po = pos < B::NPOS ? pos : 0;
          const int orow = po / G::WO, ocol = po - orow * G::WO;
          abase[i] = orow * G::S * B::RB + ocol * G::S * G::CIN + grp * 8;
        }
        f4v acc[4][NC];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[i][ct] = (f4v){0.f, 0.f, 0.f, 0.f};
        if constexpr (PIPE) {
          uint2 ra[4];
          s8v rbh[NC], rbl[NC];
#pragma unroll
          for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const uint2*>(xb + abase[i]);
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            rbh[ct] = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + grp * 8);
            rbl[ct] = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + grp * 8);
          }
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            s8v a[4], bh[NC], bl[NC];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = u8x8_to_f16off(ra[i]);
#pragma unroll
            for (int ct = 0; ct < NC; ++ct) {
              bh[ct] = rbh[ct];
              bl[ct] = rbl[ct];
            }
            if (kk + 1 < NK) {                           // (compile-time after unrolling)
              const int kc = (kk + 1) * 4 + grp;
#pragma unroll
              for (int i = 0; i < 4; ++i) ra[i] = *reinterpret_cast<const uint2*>(xb + abase[i] + (kk + 1) * B::RB);
#pragma unroll
              for (int ct = 0; ct < NC; ++ct) {
                rbh[ct] = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
                rbl[ct] = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
              }
            }
#pragma unroll
            for (int ct = 0; ct < NC; ++ct)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                acc[i][ct] = mfma16_f16(bl[ct], a[i], acc[i][ct]);
                acc[i][ct] = mfma16_f16(bh[ct], a[i], acc[i][ct]);
              }
            __builtin_amdgcn_sched_barrier(0);         // this k-step's MFMAs + the next one's reads in flight
          }
        } else {
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {                // k-step kk = kernel row kh
          s8v a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if constexpr (F16B) a[i] = *reinterpret_cast<const s8v*>(xb + 2 * (abase[i] + kk * B::RB));
            else a[i] = u8x8_to_f16off(*reinterpret_cast<const uint2*>(xb + abase[i] + kk * B::RB));
          }
          const int kc = kk * 4 + grp;
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const s8v bh = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
            const s8v bl = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              acc[i][ct] = mfma16_f16(bl, a[i], acc[i][ct]);
              acc[i][ct] = mfma16_f16(bh, a[i], acc[i][ct]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);           // one k-step of LDS fragments live at a time
        }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pos = (4 * w + i) * 16 + c16;
          const bool valid = pos < B::NPOS && oh0 + pos / G::WO < G::HO;
          conv_epi_sw<NC>(acc[i], bias_s, ct0, cnt, q, in_scale, out_scale, growb + pos, bits, bits_rows, Y, ylo,
                          pass > 0, valid);
        }
        if constexpr (ONEBUF) {
          if (u + 1 < b_end) {
            __syncthreads();                           // every wave done with band u (one buffer)
            store_band(0);
          }
        } else {
          if (u + 1 < b_end) store_band(buf ^ 1);      // buf ^ 1 was read in band u - 1, before this band's barrier
        }
      }
    };
    if (ncg == 1) run(std::integral_constant<int, 1>{});
    else run(std::integral_constant<int, 2>{});
  }
  }
}

// ===========================================================================
// forward of the bf16-activation conv layers (39x29x8 4x4/s2, 18x13x8 3x3/s1): A hi/lo planes, B hi/lo in LDS,
// three MFMAs per (row tile, column tile, k-step).  grid = (ceil(T*E*HOWO / (NT*128)), P).  The next 32-row
// tile's A fragments (both planes) are loaded while this tile's MFMAs run.
// ===========================================================================
template <class G, int NT, int LB, bool DB, bool SW>
__global__ __launch_bounds__(256, LB) void conv_fwd_x3(const uint16_t* __restrict__ X, long xlo,
                                                     uint16_t* __restrict__ Y, long ylo, uint8_t* __restrict__ bits,
                                                     const uint16_t* __restrict__ Wc, long wlo,
                                                     const float* __restrict__ flat, long bias_off, int chunk,
                                                     const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                     int layer, int L, int M, int P, int E, int T, int t0,
                                                     long bits_rows, float in_scale, float out_scale) {
  static_assert(!G::U8, "bf16-activation layers");
  constexpr int KPs = G::KP + 8;
  constexpr int NK = G::KP / 32;
  constexpr int FF_ROWS = NT * 128;
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2][X3_NCX * 16 * KPs];
  __shared__ __attribute__((aligned(16))) float bias_s[X3_NCX * 16];
  __shared__ int mods[X3_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  const int Rtot = T * E * G::HOWO;
  const int PE = P * E;
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
  const uint32_t bkey = (uint32_t)(2 * q + h);
  const int rfirst = blockIdx.x * FF_ROWS + w * 32;
  const int npass = nct > X3_NCX ? (nct + X3_NCX - 1) / X3_NCX : 1;
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * X3_NCX;
    const int ncg = nct == 0 ? 1 : min(X3_NCX, nct - ct0);
    __syncthreads();
    for (int i = tid; i < ncg * 16 * G::KC; i += 256) {
      const int col = i / G::KC, kc = i - col * G::KC;
      const int slot = ct0 * 2 + (col >> 3);
      s8v vh = {0, 0, 0, 0, 0, 0, 0, 0}, vl = vh;
      if (slot < cnt) {
        const long o = ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8;
        vh = *reinterpret_cast<const s8v*>(Wc + o);
        vl = *reinterpret_cast<const s8v*>(Wc + wlo + o);
      }
      *reinterpret_cast<s8v*>(Ws[0] + col * KPs + kc * 8) = vh;
      *reinterpret_cast<s8v*>(Ws[1] + col * KPs + kc * 8) = vl;
    }
    if (tid < ncg * 16) {
      const int slot = ct0 * 2 + (tid >> 3);
      bias_s[tid] = slot < cnt ? flat[bias_off + (long)mods[slot] * chunk + (tid & 7)] : 0.f;
    }
    __syncthreads();
    auto run = [&](auto ncc) {
      constexpr int NC = decltype(ncc)::value;
      RowIt ait[2], eit[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        rowit_init(ait[i], rfirst + i * 16 + c16, E, G::HOWO);
        rowit_init(eit[i], rfirst + i * 16 + (SW ? c16 : 4 * q), E, G::HOWO);
      }
      s8v ah[2][NK], al[2][NK];
      auto load_tile = [&](int rbase) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bool va = rbase < Rtot && ait[i].r < Rtot;
          const int oh = ait[i].pos / G::WO, ow = ait[i].pos - oh * G::WO;
          const long xb = rowit_sample(ait[i], p, E, PE, t0) * (long)G::IN_ELEMS +
                          (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN;
          rowit_adv(ait[i], 128, E, G::HOWO);
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            const int off = G::koff(kk * 4 + grp);
            ah[i][kk] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
            al[i][kk] = ah[i][kk];
            if (va && off >= 0) {
              ah[i][kk] = *reinterpret_cast<const s8v*>(X + xb + off);
              al[i][kk] = *reinterpret_cast<const s8v*>(X + xlo + xb + off);
            }
          }
        }
      };
      // DB: the next tile's A fragments load into a second register set during this tile's MFMAs (2 waves/SIMD);
      // otherwise one set, loaded at the top of each tile, and latency is hidden by occupancy (3 waves/SIMD)
      if constexpr (DB) load_tile(rfirst);
      for (int tile = 0; tile < NT; ++tile) {
        const int rbase = rfirst + tile * 128;
        if (rbase >= Rtot) break;
        s8v ch_[2][NK], cl_[2][NK];
        if constexpr (DB) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) { ch_[i][kk] = ah[i][kk]; cl_[i][kk] = al[i][kk]; }
          if (tile + 1 < NT) load_tile(rbase + 128);
        } else {
          load_tile(rbase);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) { ch_[i][kk] = ah[i][kk]; cl_[i][kk] = al[i][kk]; }
        }
        f4v acc[2][NC];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int kc = kk * 4 + grp;
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const s8v bh = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
            const s8v bl = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
            if constexpr (SW) {
              acc[0][ct] = mma3h_t(ch_[0][kk], cl_[0][kk], bh, bl, acc[0][ct]);
              acc[1][ct] = mma3h_t(ch_[1][kk], cl_[1][kk], bh, bl, acc[1][ct]);
            } else {
              acc[0][ct] = mma3h(ch_[0][kk], cl_[0][kk], bh, bl, acc[0][ct]);
              acc[1][ct] = mma3h(ch_[1][kk], cl_[1][kk], bh, bl, acc[1][ct]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r16 = rbase + i * 16;
          const RowIt e0 = eit[i];
          rowit_adv(eit[i], 128, E, G::HOWO);
          if (r16 >= Rtot) continue;
          const long grow4 = rowit_sample(e0, p, E, PE, t0) * G::HOWO + e0.pos;
          if constexpr (SW) {
            conv_epi_sw<NC>(acc[i], bias_s, ct0, cnt, q, in_scale, out_scale, grow4, bits, bits_rows, Y, ylo, pass > 0);
            continue;
          }
          float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const int slot = (ct0 + ct) * 2 + h;
            const float bb = bias_s[ct * 16 + c16];
            uint64_t bal[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = acc[i][ct][r] * in_scale + bb;
              const bool pos = v > 0.f;
              sum[r] += pos ? v : 0.f;
              bal[r] = __ballot(pos);
            }
            const uint32_t word = relu_bits_word(bal, bkey);
            if (ch == 0 && slot < cnt) *reinterpret_cast<uint32_t*>(bits + (long)slot * bits_rows + grow4) = word;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
          if (h == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const long o = (grow4 + r) * 8 + ch;
              float y = sum[r] * out_scale;
              if (pass > 0) y += ld_x4(Y, ylo, o);
              st_x4(Y, ylo, o, y);
            }
          }
        }
      }
    };
    switch (ncg) {
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      default: run(std::integral_constant<int, 3>{}); break;
    }
  }
}

// ===========================================================================
// forward of the bf16-activation conv layers, one SAMPLE per stage: the sample's fp16-pair input (39x29x8 or
// 18x13x8, 36 / 7.5 KB) is staged in LDS once and every im2col fragment is a ds_read_b128 of one pixel's 8 channels
// at (position offset) + (tap offset), instead of conv_fwd_x3's 16-byte global fragment loads that read each input
// element KH*KW/S^2 times through L2.  Weights as the MFMA A operand (conv_epi_sw epilogue, rows past the
// sample's positions masked).  Next sample's tile in registers while this one computes.  grid = (chunks, P).
// ===========================================================================
template <class G>
struct FT3 {
  static constexpr int NRT = (G::HOWO + 15) / 16;              // 16-row position tiles per sample
  static constexpr int NK = G::KP / 32;
  static constexpr int NXC = G::IN_ELEMS / 8;                  // 8-channel pixel chunks per plane
  static constexpr int XIT = (NXC + 255) / 256;
  static constexpr int TILEP = G::IN_ELEMS + 8;                // + a zero chunk for padded taps
  static_assert(G::CIN == 8 && !G::U8 && G::IN_ELEMS % 8 == 0, "8-channel fp16-pair input");
};

// PAIR: a wave computes two position tiles (rt, rt + 4) per weight-fragment read (one tile per read left the
// kernel bound by LDS reads, as the first conv1 band kernel was)
// LDS of one layer's tile forward: the sample's input planes and the staged weight pairs (conv_fwd_tile_body)
template <class G>
struct TileLds {
  static constexpr int KPs = G::KP + 8;
  static constexpr int XT = FT3<G>::TILEP;           // u16 per input plane
  static constexpr int WS = 2 * 16 * KPs;            // u16 per weight plane
  static constexpr int BYTES = (2 * XT + 2 * WS) * 2;
};

template <class G, bool PAIR>
DEVI void conv_fwd_tile_body(const uint16_t* __restrict__ X, long xlo, uint16_t* __restrict__ Y, long ylo,
                             uint8_t* __restrict__ bits, const uint16_t* __restrict__ Wc, long wlo,
                             const float* __restrict__ flat, long bias_off, int chunk,
                             const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
                             int P, int E, int T, int t0, long bits_rows, int samples_per_wg, float in_scale,
                             float out_scale, uint16_t* __restrict__ lds, float* __restrict__ bias_s,
                             int* __restrict__ mods) {
  using F = FT3<G>;
  using TL = TileLds<G>;
  constexpr int KPs = G::KP + 8;
  uint16_t* const Xt[2] = {lds, lds + TL::XT};
  uint16_t* const Ws[2] = {lds + 2 * TL::XT, lds + 2 * TL::XT + TL::WS};
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp;
  const int PE = P * E, nsamp = T * E;
  const int s_beg = blockIdx.x * samples_per_wg;
  const int s_end = min(nsamp, s_beg + samples_per_wg);
  if (s_beg >= s_end) return;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < 16) Xt[tid >> 3][G::IN_ELEMS + (tid & 7)] = 0;
  // B (pixel) fragment addresses: lane c16 = position in the tile, grp = 8-element k chunk of the k-step
  int koffs[F::NK];
#pragma unroll
  for (int kk = 0; kk < F::NK; ++kk) {
    const int kc = kk * 4 + grp;                                   // pixel chunk = tap (kh, kw)
    koffs[kk] = kc * 8 < G::K ? ((kc / G::KW) * G::WIN + kc % G::KW) * 8 : -1;
  }
  constexpr int NCXT = 2;                          // column tiles per pass (a third set of accumulators spilled)
  const int npass = nct > NCXT ? (nct + NCXT - 1) / NCXT : 1;
  s8v xh[F::XIT], xl[F::XIT];
  auto load_sample = [&](int s) {
    const long xb = sample_global(p, s, E, PE, t0) * (long)G::IN_ELEMS;
#pragma unroll
    for (int j = 0; j < F::XIT; ++j) {
      const int c = tid + 256 * j;
      if (c < F::NXC) {
        xh[j] = *reinterpret_cast<const s8v*>(X + xb + c * 8);
        xl[j] = *reinterpret_cast<const s8v*>(X + xlo + xb + c * 8);
      }
    }
  };
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * NCXT;
    const int ncg = nct == 0 ? 1 : min(NCXT, nct - ct0);
    __syncthreads();
    for (int i = tid; i < ncg * 16 * G::KC; i += 256) {
      const int col = i / G::KC, kc = i - col * G::KC;
      const int slot = ct0 * 2 + (col >> 3);
      s8v vh = {0, 0, 0, 0, 0, 0, 0, 0}, vl = vh;
      if (slot < cnt) {
        const long o = ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8;
        vh = *reinterpret_cast<const s8v*>(Wc + o);
        vl = *reinterpret_cast<const s8v*>(Wc + wlo + o);
      }
      *reinterpret_cast<s8v*>(Ws[0] + col * KPs + kc * 8) = vh;
      *reinterpret_cast<s8v*>(Ws[1] + col * KPs + kc * 8) = vl;
    }
    if (tid < ncg * 16) {
      const int slot = ct0 * 2 + (tid >> 3);
      bias_s[tid] = slot < cnt ? flat[bias_off + (long)mods[slot] * chunk + (tid & 7)] : 0.f;
    }
    load_sample(s_beg);
    auto run = [&](auto ncc) {
      constexpr int NC = decltype(ncc)::value;
      for (int s = s_beg; s < s_end; ++s) {
        __syncthreads();                           // previous sample's tile reads (and the staging above) done
#pragma unroll
        for (int j = 0; j < F::XIT; ++j) {
          const int c = tid + 256 * j;
          if (c < F::NXC) {
            *reinterpret_cast<s8v*>(&Xt[0][c * 8]) = xh[j];
            *reinterpret_cast<s8v*>(&Xt[1][c * 8]) = xl[j];
          }
        }
        __syncthreads();
        if (s + 1 < s_end) load_sample(s + 1);
        const long growb = sample_global(p, s, E, PE, t0) * G::HOWO;
        if constexpr (PAIR) {
#pragma unroll 1
          for (int rt = w; rt < F::NRT; rt += 8) {                  // tiles rt and rt + 4 (wave-uniform)
            int poff[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int pos = (rt + 4 * h) * 16 + c16;
              const int oh = pos / G::WO, ow = pos - (pos / G::WO) * G::WO;
              poff[h] = pos < G::HOWO ? (oh * G::S * G::WIN + ow * G::S) * 8 : -1;
            }
            f4v acc[2][NC];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int ct = 0; ct < NC; ++ct) acc[h][ct] = (f4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < F::NK; ++kk) {
              s8v ph[2], pl[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int a = (poff[h] < 0 || koffs[kk] < 0) ? G::IN_ELEMS : poff[h] + koffs[kk];
                ph[h] = *reinterpret_cast<const s8v*>(&Xt[0][a]);
                pl[h] = *reinterpret_cast<const s8v*>(&Xt[1][a]);
              }
              const int kc = kk * 4 + grp;
#pragma unroll
              for (int ct = 0; ct < NC; ++ct) {
                const s8v bh = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
                const s8v bl = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
#pragma unroll
                for (int h = 0; h < 2; ++h) acc[h][ct] = mma3h_t(ph[h], pl[h], bh, bl, acc[h][ct]);
              }
              __builtin_amdgcn_sched_barrier(0);       // one k-step of fragments live at a time
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int pos = (rt + 4 * h) * 16 + c16;
              conv_epi_sw<NC>(acc[h], bias_s, ct0, cnt, q, in_scale, out_scale, growb + pos, bits, bits_rows, Y, ylo,
                              pass > 0, pos < G::HOWO);
            }
          }
          continue;
        }
#pragma unroll 1
        for (int rt = w; rt < F::NRT; rt += 4) {                    // wave-uniform
          int poff;
          {
            const int pos = rt * 16 + c16;
            const int oh = pos / G::WO, ow = pos - (pos / G::WO) * G::WO;
            poff = pos < G::HOWO ? (oh * G::S * G::WIN + ow * G::S) * 8 : -1;
          }
          f4v acc[NC];
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[ct] = (f4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < F::NK; ++kk) {
            const int a = (poff < 0 || koffs[kk] < 0) ? G::IN_ELEMS : poff + koffs[kk];
            const s8v ph = *reinterpret_cast<const s8v*>(&Xt[0][a]);
            const s8v pl = *reinterpret_cast<const s8v*>(&Xt[1][a]);
            const int kc = kk * 4 + grp;
#pragma unroll
            for (int ct = 0; ct < NC; ++ct) {
              const s8v bh = *reinterpret_cast<const s8v*>(Ws[0] + (ct * 16 + c16) * KPs + kc * 8);
              const s8v bl = *reinterpret_cast<const s8v*>(Ws[1] + (ct * 16 + c16) * KPs + kc * 8);
              acc[ct] = mma3h_t(ph, pl, bh, bl, acc[ct]);
            }
          }
          const int pos = rt * 16 + c16;
          conv_epi_sw<NC>(acc, bias_s, ct0, cnt, q, in_scale, out_scale, growb + pos, bits, bits_rows, Y, ylo,
                          pass > 0, pos < G::HOWO);
        }
      }
    };
    if (ncg == 1) run(std::integral_constant<int, 1>{});
    else run(std::integral_constant<int, 2>{});
  }
}

template <class G, bool PAIR = false>
__global__ __launch_bounds__(256, 2) void conv_fwd_tile_x3(const uint16_t* __restrict__ X, long xlo,
                                                          uint16_t* __restrict__ Y, long ylo,
                                                          uint8_t* __restrict__ bits, const uint16_t* __restrict__ Wc,
                                                          long wlo, const float* __restrict__ flat, long bias_off,
                                                          int chunk, const int* __restrict__ act_idx,
                                                          const int* __restrict__ act_cnt, int layer, int L, int M,
                                                          int P, int E, int T, int t0, long bits_rows,
                                                          int samples_per_wg, float in_scale, float out_scale) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[TileLds<G>::BYTES / 2];
  __shared__ __attribute__((aligned(16))) float bias_s[2 * 16];
  __shared__ int mods[X3_MAXM];
  conv_fwd_tile_body<G, PAIR>(X, xlo, Y, ylo, bits, Wc, wlo, flat, bias_off, chunk, act_idx, act_cnt, layer, L, M, P,
                              E, T, t0, bits_rows, samples_per_wg, in_scale, out_scale, lds, bias_s, mods);
}

// The 4x4/s2 and 3x3/s1 layers' forwards in ONE launch: a workgroup runs conv_fwd_tile_body for layer `layer` over
// its samples (writing Y1 and its ReLU bits as the conv2 kernel does), then -- the same samples, so no other workgroup
// is involved -- layer + 1 reading those Y1 rows back (L2-hot), into Y2; the barrier between the phases orders the
// workgroup's own global stores and loads.  Same arithmetic as the two launches (bit-identical).
template <class G1, class G2, bool PAIR1>
__global__ __launch_bounds__(256, 2) void conv23_fwd_tile_x3(const uint16_t* __restrict__ X, long xlo,
                                                            uint16_t* __restrict__ Y1, long y1lo,
                                                            uint8_t* __restrict__ bits1, long bits_rows1,
                                                            const uint16_t* __restrict__ Wc1, long w1lo,
                                                            long bias1_off, int chunk1,
                                                            uint16_t* __restrict__ Y2, long y2lo,
                                                            uint8_t* __restrict__ bits2, long bits_rows2,
                                                            const uint16_t* __restrict__ Wc2, long w2lo,
                                                            long bias2_off, int chunk2, const float* __restrict__ flat,
                                                            const int* __restrict__ act_idx,
                                                            const int* __restrict__ act_cnt, int layer, int L, int M,
                                                            int P, int E, int T, int t0, int samples_per_wg,
                                                            float in_scale, float out_scale1, float out_scale2) {
  constexpr int B1 = TileLds<G1>::BYTES, B2 = TileLds<G2>::BYTES;
  __shared__ __attribute__((aligned(16))) uint16_t lds[(B1 > B2 ? B1 : B2) / 2];
  __shared__ __attribute__((aligned(16))) float bias_s[2 * 16];
  __shared__ int mods[X3_MAXM];
  conv_fwd_tile_body<G1, PAIR1>(X, xlo, Y1, y1lo, bits1, Wc1, w1lo, flat, bias1_off, chunk1, act_idx, act_cnt, layer, L,
                                M, P, E, T, t0, bits_rows1, samples_per_wg, in_scale, out_scale1, lds, bias_s, mods);
  __syncthreads();     // the workgroup's Y1 stores are visible to its own waves (workgroup-scope fences; a device-scope
                       // __threadfence here wrote back L2 per workgroup: 85 vs 43 us per step at 64 paths)
  conv_fwd_tile_body<G2, false>(Y1, y1lo, Y2, y2lo, bits2, Wc2, w2lo, flat, bias2_off, chunk2, act_idx, act_cnt,
                                layer + 1, L, M, P, E, T, t0, bits_rows2, samples_per_wg, in_scale, out_scale2, lds,
                                bias_s, mods);
}

// ===========================================================================
// weight gradient, LDS-slab implicit im2col (KW*CIN == 32, S*CIN == 16: the 160x120x4 8x8/s4 and 39x29x8 4x4/s2
// layers; conv_fast.hip conv_wgrad_slab describes the slab).  A stage is a band of OB output rows of one sample:
// its input rows are copied once into LDS (uint8 -> bf16 exact, or the hi and lo planes), the MFMA A operand
// (im2col^T) is read from the slab with ds_read_b64_tr_b16; the fp32 output gradient is masked by the ReLU bits and
// split into hi/lo rows of Gs.  uint8 input: 2 MFMAs (X exact), bf16 input: 3.  Register prefetch of the next stage
// + double-buffered LDS; passes of X3_NCX column tiles.  grid = (chunks, P).
// ===========================================================================
template <class G, int OB>
struct Slab {
  static constexpr int RL = G::WIN * G::CIN;
  static constexpr int PS = G::S * G::CIN;
  static constexpr int SEG = G::KW * G::CIN;
  static constexpr int NB = (G::HO + OB - 1) / OB;
  static constexpr int NPOS = OB * G::WO;
  static constexpr int KS = (NPOS + 31) / 32;
  static constexpr int SR = (OB - 1) * G::S + G::KH;
  static constexpr int SLAB = SR * RL;
  static constexpr int SLABP = SLAB + 64;
  static constexpr int NG8 = SLAB / 8;
  static constexpr int XIT = (NG8 + 255) / 256;
  static_assert(SEG == 32 && PS == 16, "slab wgrad needs KW*CIN == 32 and S*CIN == 16");
  static_assert(SLAB % 8 == 0, "slab must be a whole number of 8-element groups");
};

DEVI s8v tr8(const bf16_t* p0, const bf16_t* p1) {
  const s4v v0 = lds_tr16(p0);
  const s4v v1 = lds_tr16(p1);
  return (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
}

// RING (uint8 first layer): X is the frame ring (conv1_fwd_band_x2); a stage loads 4 pixels of each of the 4 channel
// planes per thread and transposes them into the packed slab at LDS-write time (planes_to_px4).  The first-valid
// channels of the workgroup's samples are staged in LDS once (a per-stage global byte load would sit in front of
// the stage's X loads).
// NCXP: column tiles per pass (X3_NCX = 3: paths of <= 6 active modules in one pass at 2 waves / SIMD; 2: <= 4
// modules per pass -- the common N = 4 genotype -- with 16 fewer accumulator VGPRs, which fits 3 waves / SIMD)
template <class G, int OB, int PFM, bool RING = false, int NCXP = X3_NCX>
__global__ __launch_bounds__(256, NCXP <= 2 ? 3 : 2) void conv_wgrad_slab_x3(const void* __restrict__ X, long xlo,
                                                            const float* __restrict__ Gr,
                                                            const uint8_t* __restrict__ bits, float* __restrict__ grad,
                                                            long w_off, long b_off, int chunk,
                                                            const int* __restrict__ act_idx,
                                                            const int* __restrict__ act_cnt, int layer, int L, int M,
                                                            int P, int E, int T, long bits_rows, int units_per_wg,
                                                            float in_scale, float g_scale,
                                                            const uint8_t* __restrict__ fcv, int nslots,
                                                            const float* __restrict__ gamax, int pmap,
                                                            long long* __restrict__ fx, int rbase) {
  using SB = Slab<G, OB>;
  static_assert(!RING || (G::U8 && G::CIN == 4 && G::WIN % 4 == 0), "ring input: uint8 4-channel first layer");
  // ring: 4-pixel groups per slab (one 16-byte LDS store each; 8-pixel groups, one round of loads but four stores
  // 64 bytes apart, measured 2565 vs 2477 us)
  constexpr int NG4 = SB::SR * G::WIN / 4;
  constexpr int XIT4 = (NG4 + 255) / 256;
  constexpr int FCS = RING ? X3_RING_FCS : 1;
  __shared__ uint8_t fcs[FCS];
  constexpr bool XL = !G::U8;                       // bf16 input: lo plane too
  constexpr int NXP = XL ? 2 : 1;
  // G rows: 48 elements (24 dwords) apart, so the 8 rows one lane group of a transposed B read touches land on 8
  // disjoint 8-bank windows (40 put rows q and q + 3 on shared banks)
  constexpr int GS = 48;
  static_assert(NCXP * 16 <= GS, "column tiles of a pass fit a G row");
  constexpr int NMT = G::KP / 16;
  constexpr int MPW = NMT / 4;
  constexpr int GROWS = SB::KS * 32;
  constexpr int GIT = (GROWS * 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][NXP][SB::SLABP];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][2][GROWS * GS];
  __shared__ unsigned long long dbq[X3_NCT * 16];       // det: int64 fixed point; else the float view
  float* const dbias = reinterpret_cast<float*>(dbq);
  __shared__ int mods[X3_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < X3_NCT * 16) dbq[tid] = 0ull;
  for (int i = tid; i < 2 * NXP * 64; i += 256) Xs[i / (NXP * 64)][(i / 64) % NXP][SB::SLAB + (i & 63)] = 0;
  const int PE = P * E;
  const int nunits = T * E * SB::NB;
  const int u_beg = blockIdx.x * units_per_wg;
  const int u_end = min(nunits, u_beg + units_per_wg);
  const int s_first = u_beg / SB::NB;
  // pmap bit 1 (ring, atomic mode): units in env-major order -- sample index e * T + t instead of t * E + e -- so a
  // workgroup walks one env's consecutive steps and re-reads the 3 frame planes each step shares with the previous
  // one from L2 (t-major: the next step of an env was another workgroup's, 32 samples on)
  const bool emaj = RING && (pmap & 2);
  pmap &= 1;
  if constexpr (RING) {
    const int s_last = min(T * E, (u_end + SB::NB - 1) / SB::NB);
    for (int i = tid; i < s_last - s_first && i < FCS; i += 256) {
      const int si = s_first + i;
      fcs[i] = fcv[sample_global(p, emaj ? (si % T) * E + si / T : si, E, PE, 0)];
    }
  }
  int aoff[SB::KS][2];
#pragma unroll
  for (int ks = 0; ks < SB::KS; ++ks)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // position of k-slot (grp, hf, q) of k-step ks.  pmap 1: lanes 0-31 of one transposed read take 8 consecutive
      // positions (64 consecutive dwords of the slab: every bank once); pmap 0 (round 4): positions p and p + 8,
      // 64 dwords apart, two lanes per bank on every read.  The B reads below use the same map, so the MFMA sums
      // the same 32 products per k-step in another slot order.
      int rho = ks * 32 + (pmap ? 16 * hf + 4 * grp : 8 * grp + 4 * hf) + q;
      if (rho >= SB::NPOS) rho = 0;                     // padded position: its G row is zero
      const int ob = rho / G::WO, ow = rho - ob * G::WO;
      aoff[ks][hf] = ob * G::S * SB::RL + ow * SB::PS + 4 * pp;
    }
  const int r0 = pmap ? 4 * grp : 8 * grp, r1 = pmap ? 16 + 4 * grp : 8 * grp + 4;   // B rows of k-slots hf = 0, 1
  const int npass = (nct + NCXP - 1) / NCXP;
  const float gs = g16_scale(gamax), ginv = 1.0f / gs;   // G16: the staged gradient is the fp16 pair of G * 2^e
  using XRaw = typename std::conditional<G::U8, uint2, s8v>::type;
  auto run = [&](auto ncc, const int ct0) {
    constexpr int NC = decltype(ncc)::value;
    f2v_ acc_b[2][4];                                // channel pairs: v_pk_add_f32
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc_b[k][c] = (f2v_){0.f, 0.f};
    f4v acc[MPW][NC];
#pragma unroll
    for (int a = 0; a < MPW; ++a)
#pragma unroll
      for (int b = 0; b < NC; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};
    // PF register sets of stage loads in flight (PFM = 2 for paths of <= 2 column tiles: a second set beside the
    // 3-tile accumulators would cap occupancy); stages load strictly in unit order
    constexpr int PF = (PFM >= 2 && NC <= 2) ? 2 : 1;
    struct Regs {
      XRaw xr[RING ? 1 : SB::XIT];
      uint4 xq[RING ? XIT4 : 1];                     // ring: {c0, c1, c2, c3} words of 4 pixels
      s8v xl[XL ? SB::XIT : 1];
      float4 g0r[GIT], g1r[GIT];
      uint32_t gbr[GIT][2];
      bool gvr[GIT];
      int navail;
    };
    Regs R[PF];
    int it_band, it_e, it_t;
    {
      const int s0 = u_beg / SB::NB;
      it_band = u_beg - s0 * SB::NB;
      it_t = emaj ? s0 % T : s0 / E;
      it_e = emaj ? s0 / T : s0 - it_t * E;
    }
    auto load_stage = [&](Regs& Rg) {
      const int band = it_band, ut = it_t, ue = it_e;
      const long sg = (long)ut * PE + (long)p * E + ue;
      if (++it_band == SB::NB) {
        it_band = 0;
        if (emaj) {
          if (++it_t == T) { it_t = 0; ++it_e; }
        } else {
          if (++it_e == E) { it_e = 0; ++it_t; }
        }
      }
      const int ih0 = band * OB * G::S;
      const int navail = min(SB::SR, G::HIN - ih0) * SB::RL;
      Rg.navail = navail;
      if constexpr (RING) {
        constexpr long HW = (long)G::HIN * G::WIN;
        const int fc = (int)fcs[(emaj ? ue * T + ut : ut * E + ue) - s_first];
        const uint8_t* src = reinterpret_cast<const uint8_t*>(X) + (long)(p * E + ue) * nslots * HW +
                             (long)ih0 * G::WIN;
        const int s0 = rbase + ut;               // modular ring (conv1_fwd_band_x2 ring_src)
        const int npx = min(SB::SR, G::HIN - ih0) * G::WIN;
        Rg.navail = npx;
        long po[4];                               // the 4 channel planes' slot offsets
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          int sl = s0 + max(k, fc);
          sl -= sl >= nslots ? nslots : 0;
          po[k] = (long)sl * HW;
        }
#pragma unroll
        for (int j = 0; j < XIT4; ++j) {
          const int gi = tid + 256 * j;
          const int e0 = (gi < NG4 && gi * 4 < npx) ? gi * 4 : 0;        // clamped, zeroed at write time
          Rg.xq[j] = make_uint4(*reinterpret_cast<const uint32_t*>(src + po[0] + e0),
                                *reinterpret_cast<const uint32_t*>(src + po[1] + e0),
                                *reinterpret_cast<const uint32_t*>(src + po[2] + e0),
                                *reinterpret_cast<const uint32_t*>(src + po[3] + e0));
        }
      }
      const long xbase = sg * (long)G::IN_ELEMS + (long)ih0 * SB::RL;
#pragma unroll
      for (int j = 0; j < (RING ? 0 : SB::XIT); ++j) {
        const int gi = tid + 256 * j;
        const int e0 = (gi < SB::NG8 && gi * 8 < navail) ? gi * 8 : 0;   // clamped, zeroed at write time
        if constexpr (G::U8) {
          Rg.xr[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xbase + e0);
        } else {
          Rg.xr[j] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xbase + e0);
          Rg.xl[j] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xlo + xbase + e0);
        }
      }
      const int oh0 = band * OB;
#pragma unroll
      for (int j = 0; j < GIT; ++j) {
        const int it = tid + 256 * j;
        const int rho = it >> 2, sub = it & 3;
        const int ob = rho / G::WO, ow = rho - ob * G::WO;
        Rg.gvr[j] = it < GROWS * 4 && rho < SB::NPOS && oh0 + ob < G::HO;
        if (Rg.gvr[j]) {
          const long go = sg * G::HOWO + (oh0 + ob) * G::WO + ow;
          Rg.g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
          Rg.g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int slot = 2 * ct0 + sub + 4 * k;
            Rg.gbr[j][k] = (sub + 4 * k < 2 * NC && slot < cnt) ? bits[(long)slot * bits_rows + go] : 0u;
          }
        }
      }
    };
    auto write_stage = [&](const Regs& Rg, int buf) {
      if constexpr (RING) {
#pragma unroll
        for (int j = 0; j < XIT4; ++j) {
          const int gi = tid + 256 * j;
          if (gi < NG4) {
            s8v v0 = {0, 0, 0, 0, 0, 0, 0, 0}, v1 = v0;
            if (gi * 4 < Rg.navail) {
              const uint4 px = planes_to_px4(Rg.xq[j]);
              v0 = u8x8_to_f16(make_uint2(px.x, px.y));      // pixels exact in fp16
              v1 = u8x8_to_f16(make_uint2(px.z, px.w));
            }
            *reinterpret_cast<s8v*>(&Xs[buf][0][gi * 16]) = v0;
            *reinterpret_cast<s8v*>(&Xs[buf][0][gi * 16 + 8]) = v1;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < (RING ? 0 : SB::XIT); ++j) {
        const int gi = tid + 256 * j;
        if (gi < SB::NG8) {
          const bool ok = gi * 8 < Rg.navail;
          s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
          if constexpr (G::U8) {
            if (ok) v = u8x8_to_f16(Rg.xr[j]);                            // pixels exact in fp16
          } else {
            s8v vl = v;
            if (ok) {                                                     // the activation's fp16 pair as is
              v = Rg.xr[j];
              vl = Rg.xl[j];
            }
            *reinterpret_cast<s8v*>(&Xs[buf][XL ? 1 : 0][gi * 8]) = vl;
          }
          *reinterpret_cast<s8v*>(&Xs[buf][0][gi * 8]) = v;
        }
      }
#pragma unroll
      for (int j = 0; j < GIT; ++j) {
        const int it = tid + 256 * j;
        if (it >= GROWS * 4) continue;
        const int rho = it >> 2, sub = it & 3;
        const float gg[8] = {Rg.g0r[j].x, Rg.g0r[j].y, Rg.g0r[j].z, Rg.g0r[j].w,
                             Rg.g1r[j].x, Rg.g1r[j].y, Rg.g1r[j].z, Rg.g1r[j].w};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int rel = sub + 4 * k;
          if (rel < 2 * NC) {
            // ReLU mask as a sign-extended bit field AND the value's bits (v_bfe_i32 + v_and instead of a compare,
            // a select and a scalar mask merge per value)
            const uint32_t bm = Rg.gvr[j] ? (uint32_t)Rg.gbr[j][k] : 0u;
            const uint32_t mk[8] = {sbfe1<0>(bm), sbfe1<1>(bm), sbfe1<2>(bm), sbfe1<3>(bm),
                                    sbfe1<4>(bm), sbfe1<5>(bm), sbfe1<6>(bm), sbfe1<7>(bm)};
            float m[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) m[c] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, gg[c]) & mk[c]);
#pragma unroll
            for (int c = 0; c < 4; ++c) acc_b[k][c] += (f2v_){m[2 * c], m[2 * c + 1]};
            s8v hi, lo;
            split8hs(m, gs, hi, lo);
            *reinterpret_cast<s8v*>(&Gs[buf][0][rho * GS + rel * 8]) = hi;
            *reinterpret_cast<s8v*>(&Gs[buf][1][rho * GS + rel * 8]) = lo;
          }
        }
      }
    };
    auto compute_stage = [&](int buf) {
      const bf16_t* xh = Xs[buf][0];
      const bf16_t* xlp = Xs[buf][XL ? 1 : 0];
#pragma unroll
      for (int ks = 0; ks < SB::KS; ++ks) {
        s8v bh[NC], bl[NC];
#pragma unroll
        for (int nt = 0; nt < NC; ++nt) {
          const int o0 = (ks * 32 + r0 + q) * GS + nt * 16 + 4 * pp;
          const int o1 = (ks * 32 + r1 + q) * GS + nt * 16 + 4 * pp;
          bh[nt] = tr8(Gs[buf][0] + o0, Gs[buf][0] + o1);
          bl[nt] = tr8(Gs[buf][1] + o0, Gs[buf][1] + o1);
        }
#pragma unroll
        for (int mi = 0; mi < MPW; ++mi) {
          const int mt = w * MPW + mi;
          const int kb = (mt * 16 / SB::SEG) * SB::RL + (mt * 16) % SB::SEG;
          const s8v ah = tr8(xh + kb + aoff[ks][0], xh + kb + aoff[ks][1]);
          if constexpr (XL) {
            const s8v al = tr8(xlp + kb + aoff[ks][0], xlp + kb + aoff[ks][1]);
#pragma unroll
            for (int nt = 0; nt < NC; ++nt) acc[mi][nt] = mma3h(ah, al, bh[nt], bl[nt], acc[mi][nt]);
          } else {
#pragma unroll
            for (int nt = 0; nt < NC; ++nt) acc[mi][nt] = mma2h(ah, bh[nt], bl[nt], acc[mi][nt]);
          }
        }
      }
    };
    __syncthreads();     // the previous pass's LDS reads are done (and the init above is visible)
    // the last stage(s) are peeled so every in-loop reload is unconditional (a conditional reload is a loop-carried
    // phi: the compiler copied the register set to merge it, conv_fast.hip conv_wgrad_slab)
    if constexpr (PF == 1) {
      if (u_beg < u_end) load_stage(R[0]);
      int u = u_beg, buf = 0;
      for (; u + 1 < u_end; ++u, buf ^= 1) {
        write_stage(R[0], buf);
        __syncthreads();
        load_stage(R[0]);
        compute_stage(buf);
      }
      if (u < u_end) {
        write_stage(R[0], buf);
        __syncthreads();
        compute_stage(buf);
      }
    } else {
      // stage u lives in register set and LDS buffer (u - u_beg) & 1: stage u+2's loads fly during stage u
      if (u_beg < u_end) load_stage(R[0]);
      if (u_beg + 1 < u_end) load_stage(R[PF - 1]);
      int u = u_beg;
      for (; u + 3 < u_end; u += 2) {
        write_stage(R[0], 0);
        __syncthreads();
        load_stage(R[0]);
        compute_stage(0);
        write_stage(R[PF - 1], 1);
        __syncthreads();
        load_stage(R[PF - 1]);
        compute_stage(1);
      }
      const int rem = u_end - u;
      if (rem >= 1) {
        write_stage(R[0], 0);
        __syncthreads();
        if (rem >= 3) load_stage(R[0]);
        compute_stage(0);
      }
      if (rem >= 2) {
        write_stage(R[PF - 1], 1);
        __syncthreads();
        compute_stage(1);
      }
      if (rem >= 3) {
        write_stage(R[0], 0);
        __syncthreads();
        compute_stage(0);
      }
    }
    const int h = i16 >> 3, ch = l & 7;
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const int mt = w * MPW + mi;
#pragma unroll
      for (int nt = 0; nt < NC; ++nt) {
        const int slot = (ct0 + nt) * 2 + h;
        if (slot < cnt) {
          const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = mt * 16 + 4 * grp + r;
            if (k < G::K) gacc(grad, fx, base + (long)k * 8 + ch, acc[mi][nt][r] * (in_scale * g_scale * ginv));
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int rel = (tid & 3) + 4 * k;
      const int slot = 2 * ct0 + rel;
      if (rel < 2 * NC && slot < cnt) {
#pragma unroll
        for (int c = 0; c < 8; ++c) lds_acc(dbias, dbq, slot * 8 + c, acc_b[k][c >> 1][c & 1] * g_scale, fx != nullptr);
      }
    }
  };
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * NCXP;
    switch (min(NCXP, nct - ct0)) {
      case 1: run(std::integral_constant<int, 1>{}, ct0); break;
      case 2: run(std::integral_constant<int, 2>{}, ct0); break;
      default: run(std::integral_constant<int, (NCXP >= 3 ? 3 : 2)>{}, ct0); break;
    }
  }
  __syncthreads();
  if (tid < cnt * 8) {
    const long bi = b_off + (long)mods[tid >> 3] * chunk + (tid & 7);
    if (fx) gacc_q(fx, bi, dbq[tid]);
    else atomicAdd(&grad[bi], dbias[tid]);
  }
}

// ===========================================================================
// weight gradient of the 18x13x8 3x3/s1 layer (KW*CIN = 24: no slab): 512 threads, 32-row stages of im2col rows
// (hi and lo planes) + masked, split G in double-buffered LDS, one register set of next-stage loads in flight.
// grid = (chunks, P) (conv_fast.hip conv_wgrad_fast is the bf16 form).
// ===========================================================================
#define X3_WG_RB 32
template <class G>
__global__ __launch_bounds__(512, 2) void conv_wgrad_x3(const bf16_t* __restrict__ X, long xlo,
                                                       const float* __restrict__ Gr, const uint8_t* __restrict__ bits,
                                                       float* __restrict__ grad, long w_off, long b_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M, int P,
                                                       int E, int T, long bits_rows, int rows_per_chunk,
                                                       float in_scale, float g_scale, const float* __restrict__ gamax,
                                                       long long* __restrict__ fx) {
  static_assert(!G::U8 && G::HOWO > X3_WG_RB, "bf16 input; one row wrap per stage");
  constexpr int XS = G::KP + 8;
  constexpr int GS = X3_NCX * 16 + 8;
  constexpr int NMT = G::KP / 16;
  constexpr int NW = 8;
  constexpr int MPW = (NMT + NW - 1) / NW;
  constexpr int XIT = (X3_WG_RB * G::KC + 511) / 512;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][2][X3_WG_RB * XS];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][2][X3_WG_RB * GS];
  __shared__ unsigned long long dbq[X3_NCT * 16];       // det: int64 fixed point; else the float view
  float* const dbias = reinterpret_cast<float*>(dbq);
  __shared__ int mods[X3_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < X3_NCT * 16) dbq[tid] = 0ull;
  const int Rtot = T * E * G::HOWO;
  const int PE = P * E;
  const int r_begin = blockIdx.x * rows_per_chunk;
  const int r_end = min(Rtot, r_begin + rows_per_chunk);
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int grow = tid >> 3, gsl = tid & 7;       // G staging role (threads < 256): row, slot of the pass
  const int npass = (nct + X3_NCX - 1) / X3_NCX;
  const float gs = g16_scale(gamax), ginv = 1.0f / gs;   // G16
  int xkoff[XIT];
#pragma unroll
  for (int j = 0; j < XIT; ++j) {
    const int it = tid + 512 * j;
    xkoff[j] = it < X3_WG_RB * G::KC ? G::koff(it % G::KC) : -1;
  }
  auto run = [&](auto ncc, const int ct0) {
    constexpr int NC = decltype(ncc)::value;
    const bool gact = tid < 256 && gsl < 2 * NC && 2 * ct0 + gsl < cnt;
    float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    f4v acc[MPW][NC];
#pragma unroll
    for (int a = 0; a < MPW; ++a)
#pragma unroll
      for (int b = 0; b < NC; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};
    RowIt xit[XIT], git;
#pragma unroll
    for (int j = 0; j < XIT; ++j) rowit_init(xit[j], r_begin + (tid + 512 * j) / G::KC, E, G::HOWO);
    rowit_init(git, r_begin + grow, E, G::HOWO);
    s8v xh[XIT], xlr[XIT];
    bool xv[XIT];
    float4 g0r, g1r;
    uint32_t gbr = 0;
    bool gv = false;
    auto load_stage = [&]() {
#pragma unroll
      for (int j = 0; j < XIT; ++j) {
        xv[j] = xkoff[j] >= 0 && xit[j].r < r_end;
        if (xv[j]) {
          const int oh = xit[j].pos / G::WO, ow = xit[j].pos - oh * G::WO;
          const long xo = rowit_sample(xit[j], p, E, PE, 0) * (long)G::IN_ELEMS +
                          (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN + xkoff[j];
          xh[j] = *reinterpret_cast<const s8v*>(X + xo);
          xlr[j] = *reinterpret_cast<const s8v*>(X + xlo + xo);
        }
        rowit_adv(xit[j], X3_WG_RB, E, G::HOWO);
      }
      gv = gact && git.r < r_end;
      if (gv) {
        const long go = rowit_sample(git, p, E, PE, 0) * G::HOWO + git.pos;
        g0r = *reinterpret_cast<const float4*>(Gr + go * 8);
        g1r = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
        gbr = bits[(long)(2 * ct0 + gsl) * bits_rows + go];
      }
      rowit_adv(git, X3_WG_RB, E, G::HOWO);
    };
    auto write_stage = [&](int buf) {
#pragma unroll
      for (int j = 0; j < XIT; ++j) {
        const int it = tid + 512 * j;
        if (it < X3_WG_RB * G::KC) {
          const int row = it / G::KC, kc = it - row * G::KC;
          s8v bh = {0, 0, 0, 0, 0, 0, 0, 0}, bl = bh;
          if (xv[j]) {                                                // the activation's fp16 pair as is
            bh = xh[j];
            bl = xlr[j];
          }
          *reinterpret_cast<s8v*>(&Xs[buf][0][row * XS + kc * 8]) = bh;
          *reinterpret_cast<s8v*>(&Xs[buf][1][row * XS + kc * 8]) = bl;
        }
      }
      if (tid < 256 && gsl < 2 * NC) {
        float m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (gv) {
          const float gg[8] = {g0r.x, g0r.y, g0r.z, g0r.w, g1r.x, g1r.y, g1r.z, g1r.w};
          mask8(gg, (uint32_t)gbr, m);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) bpart[c] += m[c];
        s8v hi, lo;
        split8hs(m, gs, hi, lo);
        *reinterpret_cast<s8v*>(&Gs[buf][0][grow * GS + gsl * 8]) = hi;
        *reinterpret_cast<s8v*>(&Gs[buf][1][grow * GS + gsl * 8]) = lo;
      }
    };
    auto compute = [&](int buf) {
      s8v bh[NC], bl[NC];
#pragma unroll
      for (int nt = 0; nt < NC; ++nt) {
        const int o0 = (8 * grp + q) * GS + nt * 16 + 4 * pp, o1 = (8 * grp + 4 + q) * GS + nt * 16 + 4 * pp;
        bh[nt] = tr8(Gs[buf][0] + o0, Gs[buf][0] + o1);
        bl[nt] = tr8(Gs[buf][1] + o0, Gs[buf][1] + o1);
      }
#pragma unroll
      for (int mi = 0; mi < MPW; ++mi) {
        const int mt = w + NW * mi;
        if (mt < NMT) {
          const int o0 = (8 * grp + q) * XS + mt * 16 + 4 * pp, o1 = (8 * grp + 4 + q) * XS + mt * 16 + 4 * pp;
          const s8v ah = tr8(Xs[buf][0] + o0, Xs[buf][0] + o1);
          const s8v al = tr8(Xs[buf][1] + o0, Xs[buf][1] + o1);
#pragma unroll
          for (int nt = 0; nt < NC; ++nt) acc[mi][nt] = mma3h(ah, al, bh[nt], bl[nt], acc[mi][nt]);
        }
      }
    };
    __syncthreads();
    if (r_begin < r_end) load_stage();
    int rb = r_begin, buf = 0;
    for (; rb + X3_WG_RB < r_end; rb += X3_WG_RB, buf ^= 1) {
      write_stage(buf);
      __syncthreads();
      load_stage();
      compute(buf);
    }
    if (rb < r_end) {
      write_stage(buf);
      __syncthreads();
      compute(buf);
    }
    const int h = i16 >> 3, ch = l & 7;
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const int mt = w + NW * mi;
      if (mt < NMT) {
#pragma unroll
        for (int nt = 0; nt < NC; ++nt) {
          const int slot = (ct0 + nt) * 2 + h;
          if (slot < cnt) {
            const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = mt * 16 + 4 * grp + r;
              if (k < G::K) gacc(grad, fx, base + (long)k * 8 + ch, acc[mi][nt][r] * (in_scale * g_scale * ginv));
            }
          }
        }
      }
    }
    if (gact) {
#pragma unroll
      for (int c = 0; c < 8; ++c) lds_acc(dbias, dbq, (2 * ct0 + gsl) * 8 + c, bpart[c] * g_scale, fx != nullptr);
    }
  };
  for (int pass = 0; pass < npass; ++pass) {
    const int ct0 = pass * X3_NCX;
    switch (min(X3_NCX, nct - ct0)) {
      case 1: run(std::integral_constant<int, 1>{}, ct0); break;
      case 2: run(std::integral_constant<int, 2>{}, ct0); break;
      default: run(std::integral_constant<int, 3>{}, ct0); break;
    }
  }
  __syncthreads();
  if (tid < cnt * 8) {
    const long bi = b_off + (long)mods[tid >> 3] * chunk + (tid & 7);
    if (fx) gacc_q(fx, bi, dbq[tid]);
    else atomicAdd(&grad[bi], dbias[tid]);
  }
}

// ===========================================================================
// weight gradient of the 18x13x8 3x3/s1 layer, one SAMPLE per stage: the sample's fp16-pair input tile is converted
// to a bf16 pair ONCE into LDS (1872 elements, instead of 9 im2col copies of each element as in conv_wgrad_x3), and
// the MFMA A operand (im2col^T: k = (kh, kw, ci) x 8 positions) is read straight from the tile with
// ds_read_b64_tr_b16 -- a lane's address is (position offset) + (tap/channel-chunk offset), both precomputed, so
// there is no im2col staging at all.  B = the masked, split output gradient of <= 4 slots [192 positions][32].
// 5 waves: wave w owns k rows 16w..16w+15 (the fifth tile is half padding) for every position step and column tile.
// Double-buffered LDS, one register set of next-sample loads in flight.  grid = (chunks, P).
// ===========================================================================
template <class G>
struct WT3 {
  static constexpr int NPOS = G::HOWO;                   // 176 output positions
  static constexpr int NKS = (NPOS + 31) / 32;           // 6 position steps (192 rows, 16 zero)
  static constexpr int NPP = NKS * 32;
  static constexpr int NMT = (G::K + 15) / 16;           // 5 k tiles
  static constexpr int NW = NMT;
  static constexpr int NT = NW * 64;
  static constexpr int TILE = G::IN_ELEMS;               // 1872
  static constexpr int TILEP = (TILE + 8 + 7) / 8 * 8;   // + a zero pad chunk
  static constexpr int NXC = TILE / 8;                   // 234 8-element chunks
  static constexpr int GS = 2 * 16 + 8;                  // 4 slots x 8 maps + pad (bf16)
  static constexpr int NGI = NPOS * 4;                   // (position, slot) staging items
  static constexpr int GIT = (NGI + NT - 1) / NT;
  static_assert(G::S == 1 && G::CIN == 8 && TILE % 8 == 0, "3x3/s1 8-channel layer");
  static_assert(NT % 4 == 0, "a thread's staging items share one slot");
};

template <class G>
__global__ __launch_bounds__(WT3<G>::NT, 2) void conv_wgrad_tile_x3(const uint16_t* __restrict__ X, long xlo,
                                                                   const float* __restrict__ Gr,
                                                                   const uint8_t* __restrict__ bits,
                                                                   float* __restrict__ grad, long w_off, long b_off,
                                                                   int chunk, const int* __restrict__ act_idx,
                                                                   const int* __restrict__ act_cnt, int layer, int L,
                                                                   int M, int P, int E, int T, long bits_rows,
                                                                   int samples_per_wg, float in_scale, float g_scale,
                                                                   const float* __restrict__ gamax,
                                                                   long long* __restrict__ fx) {
  using W = WT3<G>;
  __shared__ __attribute__((aligned(16))) bf16_t Xt[2][2][W::TILEP];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][2][W::NPP * W::GS];
  __shared__ unsigned long long dbq[X3_NCT * 16];       // det: int64 fixed point; else the float view
  float* const dbias = reinterpret_cast<float*>(dbq);
  __shared__ int mods[X3_MAXM];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  // passes of 2 column tiles (4 slots) are spread over blockIdx.z: a path of 5..8 active slots runs its two passes
  // in two workgroups of the usual length instead of one of twice the length (the launch's tail)
  const int nct = (cnt + 1) >> 1;
  const int npass = (nct + 1) / 2;
  if ((int)blockIdx.z >= npass) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int PE = P * E;
  const int nsamp = T * E;
  const int s_beg = blockIdx.x * samples_per_wg;
  const int s_end = min(nsamp, s_beg + samples_per_wg);
  if (s_beg >= s_end) return;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < X3_NCT * 16) dbq[tid] = 0ull;
  // zero rows 176..191 of both G buffers and the tile pad chunk (never rewritten)
  for (int i = tid; i < 2 * 2 * (W::NPP - W::NPOS) * W::GS; i += W::NT) {
    const int per = (W::NPP - W::NPOS) * W::GS;
    Gs[i / (2 * per)][(i / per) & 1][W::NPOS * W::GS + i % per] = 0;
  }
  for (int i = tid; i < 2 * 2 * (W::TILEP - W::TILE); i += W::NT) {
    const int per = W::TILEP - W::TILE;
    Xt[i / (2 * per)][(i / per) & 1][W::TILE + i % per] = 0;
  }
  // A addresses: lane 4q+pp of a 16-lane group supplies (position 8*grp + 4*hf + q of step ks, k chunk 4*pp of the
  // wave's k tile); out-of-range positions / k read the zero pad chunk (their G rows / D rows are zero / dropped)
  int posoff[W::NKS][2];
#pragma unroll
  for (int ks = 0; ks < W::NKS; ++ks)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int pos = ks * 32 + 8 * grp + 4 * hf + q;
      const int oh = pos / G::WO, ow = pos - (pos / G::WO) * G::WO;
      posoff[ks][hf] = pos < W::NPOS ? (oh * G::WIN + ow) * 8 : -1;
    }
  int koff;
  {
    const int k = w * 16 + 4 * pp;
    const int tap = k >> 3, kh = tap / G::KW, kw = tap - (tap / G::KW) * G::KW;
    koff = k < G::K ? (kh * G::WIN + kw) * 8 + (k & 7) : -1;
  }
#pragma unroll
  for (int ks = 0; ks < W::NKS; ++ks)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) posoff[ks][hf] = (posoff[ks][hf] < 0 || koff < 0) ? W::TILE : posoff[ks][hf] + koff;
  const int a_my = tid & 3;                       // the slot (within the pass) of every staging item of this thread
  const float gs = g16_scale(gamax), ginv = 1.0f / gs;   // G16
  for (int pass = blockIdx.z; pass < npass; pass += gridDim.z) {
    const int ct0 = pass * 2;
    const int nc = min(2, nct - ct0);
    const bool slot_ok = a_my < 2 * nc && 2 * ct0 + a_my < cnt;
    float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    f4v acc[2];
    acc[0] = acc[1] = (f4v){0.f, 0.f, 0.f, 0.f};
    float4 g0r[W::GIT], g1r[W::GIT];
    uint32_t gb[W::GIT];
    s8v xh, xl;
    auto load_sample = [&](int s) {
      const long sg = sample_global(p, s, E, PE, 0);
#pragma unroll
      for (int j = 0; j < W::GIT; ++j) {
        const int it = tid + W::NT * j;
        gb[j] = 0;
        if (it < W::NGI) {
          const long go = sg * G::HOWO + (it >> 2);
          g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
          g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
          if (slot_ok) gb[j] = bits[(long)(2 * ct0 + a_my) * bits_rows + go];
        }
      }
      if (tid < W::NXC) {
        const long xo = sg * (long)W::TILE + tid * 8;
        xh = *reinterpret_cast<const s8v*>(X + xo);
        xl = *reinterpret_cast<const s8v*>(X + xlo + xo);
      }
    };
    auto write_sample = [&](int buf) {
      if (tid < W::NXC) {                          // the activation's fp16 pair as is
        *reinterpret_cast<s8v*>(&Xt[buf][0][tid * 8]) = xh;
        *reinterpret_cast<s8v*>(&Xt[buf][1][tid * 8]) = xl;
      }
#pragma unroll
      for (int j = 0; j < W::GIT; ++j) {
        const int it = tid + W::NT * j;
        if (it < W::NGI) {
          const float gg[8] = {g0r[j].x, g0r[j].y, g0r[j].z, g0r[j].w, g1r[j].x, g1r[j].y, g1r[j].z, g1r[j].w};
          float m[8];
          mask8(gg, (uint32_t)gb[j], m);
#pragma unroll
          for (int c = 0; c < 8; ++c) bpart[c] += m[c];
          s8v hi, lo;
          split8hs(m, gs, hi, lo);
          const int o = (it >> 2) * W::GS + a_my * 8;
          *reinterpret_cast<s8v*>(&Gs[buf][0][o]) = hi;
          *reinterpret_cast<s8v*>(&Gs[buf][1][o]) = lo;
        }
      }
    };
    auto compute = [&](int buf, auto ncc) {
      constexpr int NC = decltype(ncc)::value;
#pragma unroll
      for (int ks = 0; ks < W::NKS; ++ks) {
        const s8v ah = tr8(Xt[buf][0] + posoff[ks][0], Xt[buf][0] + posoff[ks][1]);
        const s8v al = tr8(Xt[buf][1] + posoff[ks][0], Xt[buf][1] + posoff[ks][1]);
#pragma unroll
        for (int nt = 0; nt < NC; ++nt) {
          const int o0 = (ks * 32 + 8 * grp + q) * W::GS + nt * 16 + 4 * pp;
          const int o1 = (ks * 32 + 8 * grp + 4 + q) * W::GS + nt * 16 + 4 * pp;
          const s8v bh = tr8(Gs[buf][0] + o0, Gs[buf][0] + o1);
          const s8v bl = tr8(Gs[buf][1] + o0, Gs[buf][1] + o1);
          acc[nt] = mma3h(ah, al, bh, bl, acc[nt]);
        }
      }
    };
    __syncthreads();     // mods / dbias / pads visible; the previous pass's LDS reads done
    load_sample(s_beg);
    int buf = 0;
    for (int s = s_beg; s < s_end; ++s, buf ^= 1) {
      write_sample(buf);
      __syncthreads();
      if (s + 1 < s_end) load_sample(s + 1);
      if (nc == 2) compute(buf, std::integral_constant<int, 2>{});
      else compute(buf, std::integral_constant<int, 1>{});
    }
    const int h = i16 >> 3, ch = l & 7;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int slot = (ct0 + nt) * 2 + h;
      if (nt < nc && slot < cnt) {
        const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = w * 16 + 4 * grp + r;
          if (k < G::K) gacc(grad, fx, base + (long)k * 8 + ch, acc[nt][r] * (in_scale * g_scale * ginv));
        }
      }
    }
    if (slot_ok) {
#pragma unroll
      for (int c = 0; c < 8; ++c) lds_acc(dbias, dbq, (2 * ct0 + a_my) * 8 + c, bpart[c] * g_scale, fx != nullptr);
    }
  }
  __syncthreads();
  if (tid < cnt * 8 && ((tid >> 5) % (int)gridDim.z) == (int)blockIdx.z) {   // the slots of this workgroup's passes
    const long bi = b_off + (long)mods[tid >> 3] * chunk + (tid & 7);
    if (fx) gacc_q(fx, bi, dbq[tid]);
    else atomicAdd(&grad[bi], dbias[tid]);
  }
}

// ===========================================================================
// input gradient of the bf16-activation conv layers on MFMA, "superpixel" implicit GEMM (conv_fast.hip
// conv_dgrad_mfma describes the geometry): one GEMM row = one superpixel (the S x S input pixels that read the
// same output positions through different taps), N = (ph, pw, ci), K = (tap, slot, c).  Per sample the masked
// output gradient of 4 active slots is split into hi/lo planes in LDS (a path with more active slots runs a pass
// per group of 4, adding into dX); B = the hi/lo weights of those slots.  fp32 dX.  grid = (chunks, P).
// ===========================================================================
#define X3_DG_PSTR 32        // one position's 4 slots x 8 maps
#define X3_DG_SPLIT 2        // conv_dgrad_x3 gridDim.z: the sample split of paths of > 4 active slots
DEVI int dg_swz(int i) { return (i >> 1) & 3; }
template <class G>
struct DGM {
  static constexpr int S = G::S;
  static constexpr int NA = (G::KH + S - 1) / S;
  static constexpr int NTAP = NA * NA;
  static constexpr int NI = (G::HIN + S - 1) / S, NJ = (G::WIN + S - 1) / S;
  static constexpr int NSP = NI * NJ;
  static constexpr int NRT = (NSP + 15) / 16;
  static constexpr int NN = 8 * S * S;
  static constexpr int NT = (NN + 15) / 16;
};

// BAL: the cost-balanced 1-D schedule (bal_schedule; a sample of a path costs its slot-group count): a workgroup's
// samples may span paths, each sample's dX is still computed by one workgroup in group order (bit-identical)
DEVI int dg_ngroup(int cnt) { return cnt > 4 ? (cnt + 3) >> 2 : 1; }

template <class G, bool W3 = false, bool ALT = false, bool BAL = false>
__global__ __launch_bounds__(256, 2) void conv_dgrad_x3(const float* __restrict__ Gr, const uint8_t* __restrict__ bits,
                                                       const float* __restrict__ flat, long w_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M, int P,
                                                       int E, int T, long bits_rows, float g_scale,
                                                       float* __restrict__ dX, int samples_per_wg,
                                                       const float* __restrict__ gamax, float* __restrict__ gamax_out,
                                                       int presplit) {
  using D = DGM<G>;
  constexpr int S = D::S;
  constexpr int NTAPP = (D::NTAP + 3) & ~3;
  constexpr int GPL = (G::HOWO + 1) * X3_DG_PSTR;
  constexpr int BPL = D::NTAP * D::NT * 16 * 32;
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][GPL];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[W3 ? 3 : 2][BPL];
  __shared__ int mods[X3_MAXM];
  __shared__ __attribute__((aligned(16))) uint16_t atap[D::NRT * 16 * NTAPP];
  __shared__ __attribute__((aligned(8))) uint16_t etab[D::NRT * 16];
  __shared__ int sched[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int PE = P * E;
  const int nsamp = T * E;
  // this workgroup's units: (path, sample) from (seg_p0, seg_s0) up to, not including, (seg_p1, seg_s1)
  int seg_p0, seg_s0, seg_p1, seg_s1;
  if constexpr (BAL) {
    // wave 0 computes the schedule while the other waves build the position tables below (read after the barrier)
    if (w == 0) bal_schedule(act_cnt, L, layer, P, nsamp, [](int c) { return dg_ngroup(c); }, sched);
    seg_p0 = seg_s0 = seg_p1 = seg_s1 = 0;
  } else {
    // a path of more than 4 active slots runs a pass per group of 4: with gridDim.z = 2 its workgroup's samples are
    // split over blockIdx.z (the z = 1 half dispatched after every z = 0 workgroup, so a path of <= 4 slots leaves no
    // empty workgroups among the first round)
    seg_p0 = seg_p1 = blockIdx.y;
    const int nsplit = dg_ngroup(act_cnt[seg_p0 * L + layer]) > 1 ? (int)gridDim.z : 1;
    if ((int)blockIdx.z >= nsplit) return;
    const int c_beg = blockIdx.x * samples_per_wg;
    const int c_end = min(nsamp, c_beg + samples_per_wg);
    const int spw = (samples_per_wg + nsplit - 1) / nsplit;
    seg_s0 = c_beg + (int)blockIdx.z * spw;
    seg_s1 = min(c_end, seg_s0 + spw);
    if (seg_s0 >= seg_s1) return;
  }
  int p = 0, cnt = 0;
  // B[k][n] of slot group g: k = (tap, slot a4, c), n = (ph*S + pw)*8 + ci  ->  W_a[kh][kw][ci][c], hi/lo
  auto stage_b = [&](int g) {
    for (int it = tid; it < D::NTAP * D::NT * 16 * 4; it += 256) {
      const int a4 = it & 3, rest = it >> 2;
      const int n = rest % (D::NT * 16), tap = rest / (D::NT * 16);
      const int a = 4 * g + a4;
      const int ta = tap / D::NA, tb = tap - ta * D::NA;
      const int cls = n >> 3, ci = n & 7, ph = cls / S, pw = cls - ph * S;
      const int kh = ph + S * ta, kw = pw + S * tb;
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (n < D::NN && a < cnt && kh < G::KH && kw < G::KW) {
        const float* wp = flat + w_off + (long)mods[a] * chunk + ((kh * G::KW + kw) * 8 + ci) * 8;
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = wp[c];
      }
      s8v hi, lo;
      // fp16 pair of W * 2^8 (G16); ALT: odd taps' weights staged negated (the second accumulator chain)
      split8hs(v, (ALT && (tap & 1)) ? -(float)(1 << X3_W0_SHIFT) : (float)(1 << X3_W0_SHIFT), hi, lo);
      const int o = (tap * D::NT * 16 + n) * 32 + (a4 ^ dg_swz(n)) * 8;
      *reinterpret_cast<s8v*>(Bs[0] + o) = hi;
      *reinterpret_cast<s8v*>(Bs[1] + o) = lo;
      if constexpr (W3) {                                   // third piece: W * 2^8 - hi - lo
        const h8v hh = __builtin_bit_cast(h8v, hi), ll = __builtin_bit_cast(h8v, lo);
        _Float16 r[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) r[c] = (_Float16)(v[c] * (float)(1 << X3_W0_SHIFT) - (float)hh[c] - (float)ll[c]);
        *reinterpret_cast<s8v*>(Bs[2] + o) = __builtin_bit_cast(s8v, r);
      }
    }
  };
  constexpr int GIT = (G::HOWO + 255) / 256;
  float4 g0r[GIT], g1r[GIT];
  uint8_t gbr[GIT][4];
  // the output gradient of sample s and the ReLU bits of slot group g
  auto load_sample = [&](int s, int g) {
    const long sg = sample_global(p, s, E, PE, 0);
#pragma unroll
    for (int j = 0; j < GIT; ++j) {
      const int pos = tid + 256 * j;
      if (pos < G::HOWO) {
        const long go = sg * G::HOWO + pos;
        g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
        g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
#pragma unroll
        for (int a4 = 0; a4 < 4; ++a4) {
          const int a = 4 * g + a4;
          gbr[j][a4] = a < cnt ? bits[(long)a * bits_rows + go] : (uint8_t)0;
        }
      }
    }
  };
  static_assert(S <= 2, "dgrad class limits are packed for strides 1 and 2");
  static_assert((G::HOWO + 1) * X3_DG_PSTR < (1 << 16), "atap offset field");
  static_assert((S * (D::NI - 1) * G::WIN + S * (D::NJ - 1)) * 8 < (1 << 14), "etab offset field");
  for (int sp = tid; sp < D::NRT * 16; sp += 256) {
    const int ii = sp / D::NJ, jj = sp - ii * D::NJ;
#pragma unroll
    for (int tap = 0; tap < NTAPP; ++tap) {
      const int ta = tap / D::NA, tb = tap - ta * D::NA;
      const int oh = ii - ta, ow = jj - tb;
      const bool ok = tap < D::NTAP && sp < D::NSP && oh >= 0 && oh < G::HO && ow >= 0 && ow < G::WO;
      const int apos = ok ? oh * G::WO + ow : G::HOWO;
      atap[sp * NTAPP + tap] = (uint16_t)(apos * X3_DG_PSTR + (dg_swz(apos) << 3));
    }
    etab[sp] = sp < D::NSP ? (uint16_t)((S * ii * G::WIN + S * jj) * 8 | ((S * ii + 1 < G::HIN) << 14) |
                                        ((S * jj + 1 < G::WIN) << 15))
                           : (uint16_t)0xFFFF;
  }
  for (int i = tid; i < 2 * X3_DG_PSTR; i += 256) Gs[i / X3_DG_PSTR][G::HOWO * X3_DG_PSTR + (i % X3_DG_PSTR)] = 0;
  int nofs[D::NT], nph[D::NT], npw[D::NT];
#pragma unroll
  for (int nt = 0; nt < D::NT; ++nt) {
    const int n = nt * 16 + c16;
    const int cls = n >> 3, ci = n & 7;
    nph[nt] = n < D::NN ? cls / S : 9;
    npw[nt] = cls - (cls / S) * S;
    nofs[nt] = ((cls / S) * G::WIN + npw[nt]) * 8 + ci;
  }
  const float gs = g16_scale(gamax), inv = 1.0f / (gs * (float)(1 << X3_W0_SHIFT));
  float am = 0.f;
  if constexpr (BAL) {
    __syncthreads();                               // the schedule (and the position tables) visible
    seg_p0 = __builtin_amdgcn_readfirstlane(sched[0]);     // uniform: SGPRs, scalar address math
    seg_s0 = __builtin_amdgcn_readfirstlane(sched[1]);
    seg_p1 = __builtin_amdgcn_readfirstlane(sched[2]);
    seg_s1 = __builtin_amdgcn_readfirstlane(sched[3]);
    if (seg_p0 == seg_p1 && seg_s0 >= seg_s1) return;
  }
  for (int sp = seg_p0; sp <= seg_p1; ++sp) {
  const int s_beg = sp == seg_p0 ? seg_s0 : 0, s_end = sp == seg_p1 ? seg_s1 : nsamp;
  if (s_beg >= s_end) continue;
  p = sp;
  cnt = act_cnt[p * L + layer];
  const int ngroup = dg_ngroup(cnt);
  __syncthreads();                                 // the previous segment's LDS reads (mods, Bs, Gs) done
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  __syncthreads();
  // slot groups outermost: each group's weights are staged ONCE per segment (they were restaged per sample when
  // the group loop ran inside the sample loop); group g > 0 adds into the dX its own threads wrote for group g - 1
  for (int g = 0; g < ngroup; ++g) {
    if (g > 0) __syncthreads();                    // the previous group's LDS reads done
    stage_b(g);
    load_sample(s_beg, g);
    for (int s = s_beg; s < s_end; ++s) {
      const long sg = sample_global(p, s, E, PE, 0);
      float* __restrict__ dXs = dX + sg * (long)(G::HIN * G::WIN * 8);
      __syncthreads();                             // previous LDS reads done; B staged
#pragma unroll
      for (int j = 0; j < GIT; ++j) {
        const int pos = tid + 256 * j;
        if (pos < G::HOWO) {
          const float gg[8] = {g0r[j].x * g_scale, g0r[j].y * g_scale, g0r[j].z * g_scale, g0r[j].w * g_scale,
                               g1r[j].x * g_scale, g1r[j].y * g_scale, g1r[j].z * g_scale, g1r[j].w * g_scale};
          // presplit: the fp16 pair of G * 2^e once per position, masked per slot (bit-identical to masking the fp32
          // values and splitting per slot, at a quarter of the conversions)
          s8v ph, pl;
          if (presplit) split8hs(gg, gs, ph, pl);
#pragma unroll
          for (int a4 = 0; a4 < 4; ++a4) {
            const int b = (int)gbr[j][a4];
            s8v hi, lo;
            if (presplit) {
              mask_pair8(ph, pl, (uint32_t)b, hi, lo);
            } else {
              float m[8];
              mask8(gg, (uint32_t)b, m);
              split8hs(m, gs, hi, lo);
            }
            const int o = pos * X3_DG_PSTR + (a4 ^ dg_swz(pos)) * 8;
            *reinterpret_cast<s8v*>(Gs[0] + o) = hi;
            *reinterpret_cast<s8v*>(Gs[1] + o) = lo;
          }
        }
      }
      __syncthreads();
      if (s + 1 < s_end) load_sample(s + 1, g);
      for (int rt = w; rt < D::NRT; rt += 4) {
        const uint16_t* tp = atap + (rt * 16 + c16) * NTAPP;
        f4v acc[D::NT], accn[ALT ? D::NT : 1];
#pragma unroll
        for (int nt = 0; nt < D::NT; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (ALT) {
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) accn[nt] = {0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int tap = 0; tap < D::NTAP; ++tap) {
          const int ao = (int)tp[tap] ^ (grp << 3);
          const s8v ah = *reinterpret_cast<const s8v*>(Gs[0] + ao);
          const s8v al = *reinterpret_cast<const s8v*>(Gs[1] + ao);
          // ALT: odd taps (negated weights in LDS) into a second chain, subtracted at the end (the f16 MFMA's -inf
          // rounding bias enters with alternating signs; fc_dgrad_gemm_x3 FOLD 2)
          const bool neg = ALT && (tap & 1);
          const int bo = (tap * D::NT * 16 + c16) * 32 + (grp ^ dg_swz(c16)) * 8;
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) {
            const s8v bh = *reinterpret_cast<const s8v*>(Bs[0] + bo + nt * 16 * 32);
            const s8v bl = *reinterpret_cast<const s8v*>(Bs[1] + bo + nt * 16 * 32);
            if (neg) {
              accn[nt] = mma3h(ah, al, bh, bl, accn[nt]);
            } else {
              if constexpr (W3) acc[nt] = mfma16_f16(ah, *reinterpret_cast<const s8v*>(Bs[2] + bo + nt * 16 * 32), acc[nt]);
              acc[nt] = mma3h(ah, al, bh, bl, acc[nt]);
            }
          }
        }
        if constexpr (ALT) {
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) acc[nt] -= accn[nt];
        }
        const uint2 e4 = *reinterpret_cast<const uint2*>(etab + rt * 16 + 4 * grp);
        const uint32_t ev[4] = {e4.x & 0xFFFFu, e4.x >> 16, e4.y & 0xFFFFu, e4.y >> 16};
#pragma unroll
        for (int nt = 0; nt < D::NT; ++nt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t v = ev[r];
            const bool okh = nph[nt] == 0 || (nph[nt] == 1 && ((v >> 14) & 1u));
            const bool okw = npw[nt] == 0 || ((v >> 15) & 1u);
            if (v != 0xFFFFu && okh && okw) {
              float* o = dXs + (int)(v & 0x3FFFu) + nofs[nt];
              const float y = g == 0 ? acc[nt][r] * inv : *o + acc[nt][r] * inv;
              *o = y;
              if (g == ngroup - 1) am = fmaxf(am, fabsf(y));
            }
          }
        }
      }
    }
  }
  }
  g16_flush_amax(am, gamax_out);
}

// the round-6 form of conv_dgrad_x3 (slot groups inside the sample loop, one chunk per workgroup): kept for the
// interleaved A/B of the restructured kernel (X3_DG_V0 = 1)
template <class G, bool W3 = false, bool ALT = false>
__global__ __launch_bounds__(256, 2) void conv_dgrad_x3v0(const float* __restrict__ Gr, const uint8_t* __restrict__ bits,
                                                       const float* __restrict__ flat, long w_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M, int P,
                                                       int E, int T, long bits_rows, float g_scale,
                                                       float* __restrict__ dX, int samples_per_wg,
                                                       const float* __restrict__ gamax, float* __restrict__ gamax_out,
                                                       int presplit) {
  using D = DGM<G>;
  constexpr int S = D::S;
  constexpr int NTAPP = (D::NTAP + 3) & ~3;
  constexpr int GPL = (G::HOWO + 1) * X3_DG_PSTR;
  constexpr int BPL = D::NTAP * D::NT * 16 * 32;
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][GPL];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[W3 ? 3 : 2][BPL];
  __shared__ int mods[X3_MAXM];
  __shared__ __attribute__((aligned(16))) uint16_t atap[D::NRT * 16 * NTAPP];
  __shared__ __attribute__((aligned(8))) uint16_t etab[D::NRT * 16];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int PE = P * E;
  const int nsamp = T * E;
  const int s_beg = blockIdx.x * samples_per_wg;
  const int s_end = min(nsamp, s_beg + samples_per_wg);
  if (s_beg >= s_end) return;
  if (tid < X3_MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  __syncthreads();
  const int ngroup = cnt > 4 ? (cnt + 3) >> 2 : 1;
  // B[k][n] of slot group g: k = (tap, slot a4, c), n = (ph*S + pw)*8 + ci  ->  W_a[kh][kw][ci][c], hi/lo
  auto stage_b = [&](int g) {
    for (int it = tid; it < D::NTAP * D::NT * 16 * 4; it += 256) {
      const int a4 = it & 3, rest = it >> 2;
      const int n = rest % (D::NT * 16), tap = rest / (D::NT * 16);
      const int a = 4 * g + a4;
      const int ta = tap / D::NA, tb = tap - ta * D::NA;
      const int cls = n >> 3, ci = n & 7, ph = cls / S, pw = cls - ph * S;
      const int kh = ph + S * ta, kw = pw + S * tb;
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (n < D::NN && a < cnt && kh < G::KH && kw < G::KW) {
        const float* wp = flat + w_off + (long)mods[a] * chunk + ((kh * G::KW + kw) * 8 + ci) * 8;
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = wp[c];
      }
      s8v hi, lo;
      // fp16 pair of W * 2^8 (G16); ALT: odd taps' weights staged negated (the second accumulator chain)
      split8hs(v, (ALT && (tap & 1)) ? -(float)(1 << X3_W0_SHIFT) : (float)(1 << X3_W0_SHIFT), hi, lo);
      const int o = (tap * D::NT * 16 + n) * 32 + (a4 ^ dg_swz(n)) * 8;
      *reinterpret_cast<s8v*>(Bs[0] + o) = hi;
      *reinterpret_cast<s8v*>(Bs[1] + o) = lo;
      if constexpr (W3) {                                   // third piece: W * 2^8 - hi - lo
        const h8v hh = __builtin_bit_cast(h8v, hi), ll = __builtin_bit_cast(h8v, lo);
        _Float16 r[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) r[c] = (_Float16)(v[c] * (float)(1 << X3_W0_SHIFT) - (float)hh[c] - (float)ll[c]);
        *reinterpret_cast<s8v*>(Bs[2] + o) = __builtin_bit_cast(s8v, r);
      }
    }
  };
  constexpr int GIT = (G::HOWO + 255) / 256;
  float4 g0r[GIT], g1r[GIT];
  uint8_t gbr[GIT][12];
  auto load_sample = [&](int s) {
    const long sg = sample_global(p, s, E, PE, 0);
#pragma unroll
    for (int j = 0; j < GIT; ++j) {
      const int pos = tid + 256 * j;
      if (pos < G::HOWO) {
        const long go = sg * G::HOWO + pos;
        g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
        g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
#pragma unroll
        for (int a = 0; a < 12; ++a) gbr[j][a] = a < cnt ? bits[(long)a * bits_rows + go] : (uint8_t)0;
      }
    }
  };
  static_assert(S <= 2, "dgrad class limits are packed for strides 1 and 2");
  static_assert((G::HOWO + 1) * X3_DG_PSTR < (1 << 16), "atap offset field");
  static_assert((S * (D::NI - 1) * G::WIN + S * (D::NJ - 1)) * 8 < (1 << 14), "etab offset field");
  for (int sp = tid; sp < D::NRT * 16; sp += 256) {
    const int ii = sp / D::NJ, jj = sp - ii * D::NJ;
#pragma unroll
    for (int tap = 0; tap < NTAPP; ++tap) {
      const int ta = tap / D::NA, tb = tap - ta * D::NA;
      const int oh = ii - ta, ow = jj - tb;
      const bool ok = tap < D::NTAP && sp < D::NSP && oh >= 0 && oh < G::HO && ow >= 0 && ow < G::WO;
      const int apos = ok ? oh * G::WO + ow : G::HOWO;
      atap[sp * NTAPP + tap] = (uint16_t)(apos * X3_DG_PSTR + (dg_swz(apos) << 3));
    }
    etab[sp] = sp < D::NSP ? (uint16_t)((S * ii * G::WIN + S * jj) * 8 | ((S * ii + 1 < G::HIN) << 14) |
                                        ((S * jj + 1 < G::WIN) << 15))
                           : (uint16_t)0xFFFF;
  }
  for (int i = tid; i < 2 * X3_DG_PSTR; i += 256) Gs[i / X3_DG_PSTR][G::HOWO * X3_DG_PSTR + (i % X3_DG_PSTR)] = 0;
  int nofs[D::NT], nph[D::NT], npw[D::NT];
#pragma unroll
  for (int nt = 0; nt < D::NT; ++nt) {
    const int n = nt * 16 + c16;
    const int cls = n >> 3, ci = n & 7;
    nph[nt] = n < D::NN ? cls / S : 9;
    npw[nt] = cls - (cls / S) * S;
    nofs[nt] = ((cls / S) * G::WIN + npw[nt]) * 8 + ci;
  }
  if (ngroup == 1) stage_b(0);
  const float gs = g16_scale(gamax), inv = 1.0f / (gs * (float)(1 << X3_W0_SHIFT));
  float am = 0.f;
  load_sample(s_beg);
  for (int s = s_beg; s < s_end; ++s) {
    const long sg = sample_global(p, s, E, PE, 0);
    float* __restrict__ dXs = dX + sg * (long)(G::HIN * G::WIN * 8);
    for (int g = 0; g < ngroup; ++g) {
      __syncthreads();                             // previous LDS reads done
      if (ngroup > 1) stage_b(g);
#pragma unroll
      for (int j = 0; j < GIT; ++j) {
        const int pos = tid + 256 * j;
        if (pos < G::HOWO) {
          const float gg[8] = {g0r[j].x * g_scale, g0r[j].y * g_scale, g0r[j].z * g_scale, g0r[j].w * g_scale,
                               g1r[j].x * g_scale, g1r[j].y * g_scale, g1r[j].z * g_scale, g1r[j].w * g_scale};
          // presplit: the fp16 pair of G * 2^e once per position, masked per slot (bit-identical to masking the fp32
          // values and splitting per slot, at a quarter of the conversions)
          s8v ph, pl;
          if (presplit) split8hs(gg, gs, ph, pl);
#pragma unroll
          for (int a4 = 0; a4 < 4; ++a4) {
            const int b = (int)gbr[j][(4 * g + a4) < 12 ? 4 * g + a4 : 0] * (4 * g + a4 < cnt ? 1 : 0);
            s8v hi, lo;
            if (presplit) {
              mask_pair8(ph, pl, (uint32_t)b, hi, lo);
            } else {
              float m[8];
              mask8(gg, (uint32_t)b, m);
              split8hs(m, gs, hi, lo);
            }
            const int o = pos * X3_DG_PSTR + (a4 ^ dg_swz(pos)) * 8;
            *reinterpret_cast<s8v*>(Gs[0] + o) = hi;
            *reinterpret_cast<s8v*>(Gs[1] + o) = lo;
          }
        }
      }
      __syncthreads();
      if (g == ngroup - 1 && s + 1 < s_end) load_sample(s + 1);
      for (int rt = w; rt < D::NRT; rt += 4) {
        const uint16_t* tp = atap + (rt * 16 + c16) * NTAPP;
        f4v acc[D::NT], accn[ALT ? D::NT : 1];
#pragma unroll
        for (int nt = 0; nt < D::NT; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (ALT) {
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) accn[nt] = {0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int tap = 0; tap < D::NTAP; ++tap) {
          const int ao = (int)tp[tap] ^ (grp << 3);
          const s8v ah = *reinterpret_cast<const s8v*>(Gs[0] + ao);
          const s8v al = *reinterpret_cast<const s8v*>(Gs[1] + ao);
          // ALT: odd taps (negated weights in LDS) into a second chain, subtracted at the end (the f16 MFMA's -inf
          // rounding bias enters with alternating signs; fc_dgrad_gemm_x3 FOLD 2)
          const bool neg = ALT && (tap & 1);
          const int bo = (tap * D::NT * 16 + c16) * 32 + (grp ^ dg_swz(c16)) * 8;
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) {
            const s8v bh = *reinterpret_cast<const s8v*>(Bs[0] + bo + nt * 16 * 32);
            const s8v bl = *reinterpret_cast<const s8v*>(Bs[1] + bo + nt * 16 * 32);
            if (neg) {
              accn[nt] = mma3h(ah, al, bh, bl, accn[nt]);
            } else {
              if constexpr (W3) acc[nt] = mfma16_f16(ah, *reinterpret_cast<const s8v*>(Bs[2] + bo + nt * 16 * 32), acc[nt]);
              acc[nt] = mma3h(ah, al, bh, bl, acc[nt]);
            }
          }
        }
        if constexpr (ALT) {
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) acc[nt] -= accn[nt];
        }
        const uint2 e4 = *reinterpret_cast<const uint2*>(etab + rt * 16 + 4 * grp);
        const uint32_t ev[4] = {e4.x & 0xFFFFu, e4.x >> 16, e4.y & 0xFFFFu, e4.y >> 16};
#pragma unroll
        for (int nt = 0; nt < D::NT; ++nt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t v = ev[r];
            const bool okh = nph[nt] == 0 || (nph[nt] == 1 && ((v >> 14) & 1u));
            const bool okw = npw[nt] == 0 || ((v >> 15) & 1u);
            if (v != 0xFFFFu && okh && okw) {
              float* o = dXs + (int)(v & 0x3FFFu) + nofs[nt];
              const float y = g == 0 ? acc[nt][r] * inv : *o + acc[nt][r] * inv;
              *o = y;
              if (g == ngroup - 1) am = fmaxf(am, fabsf(y));
            }
          }
        }
      }
    }
  }
  g16_flush_amax(am, gamax_out);
}

// ===========================================================================
// fc forward for the rollout (<= 32 rows per path), module per wave (trunk_fwd.hip fc_fwd_mw_kernel): A hi/lo
// planes and B hi/lo from the [2][M][Cout][KP] weight copy, a D-deep register ring, three MFMAs per k-step.
// OF32: the last layer writes fp32 (heads input); otherwise two bf16 planes.  grid = (1, Cout/64, P).
// ===========================================================================
template <int RT, int D, int NKS, bool OF32>
__global__ __launch_bounds__(256) void fc_fwd_x3(const uint16_t* __restrict__ X, long xlo, int ldx,
                                                 void* __restrict__ Yv, long ylo, uint16_t* __restrict__ bits,
                                                 const uint16_t* __restrict__ Wc, long wlo,
                                                 const float* __restrict__ flat, long bias_off, int chunk,
                                                 const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                 int layer, int L, int M, int K, int KP, int Cout, int P, int E, int T,
                                                 int t0, long bits_rows, float in_scale, float out_scale) {
  __shared__ float part[4][32][64 + 1];
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * (16 * RT);
  const int col0 = blockIdx.y * 64;
  long xrow[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const long r = row0 + i * 16 + c16;
    xrow[i] = sample_global(p, (int)(r < Rtot ? r : row0), E, PE, t0) * ldx;
  }
  float sum[RT][4][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[i][j][r] = 0.f;
  const int nwords = Cout / 16;
  long sgb[RT][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + i * 16 + 4 * grp + r;
      sgb[i][r] = sample_global(p, (int)(row < Rtot ? row : row0), E, PE, t0);
    }
  // this wave's first module index goes out beside the count (the list is padded with -1 past it), so the first
  // weight loads wait for one load level instead of two
  const int mod_w = w < M ? act_idx[(p * L + layer) * M + w] : -1;
  for (int a = w; a < cnt; a += 4) {
    const int mod = a == w ? mod_w : act_idx[(p * L + layer) * M + a];
    const uint16_t* Wm = Wc + (long)mod * Cout * KP + (long)(col0 + c16) * KP + 8 * grp;
    f4v acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
    s8v ah[D][RT], al[D][RT], bh[D][4], bl[D][4];
    auto load = [&](int d, int kk) {
      const int k0 = kk + 8 * grp;
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if (K == KP) {
          ah[d][i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
          al[d][i] = *reinterpret_cast<const s8v*>(X + xlo + xrow[i] + k0);
        } else {
          ah[d][i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
          al[d][i] = ah[d][i];
          if (k0 < K) {
            ah[d][i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
            al[d][i] = *reinterpret_cast<const s8v*>(X + xlo + xrow[i] + k0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bh[d][j] = *reinterpret_cast<const s8v*>(Wm + (long)j * 16 * KP + kk);
        bl[d][j] = *reinterpret_cast<const s8v*>(Wm + wlo + (long)j * 16 * KP + kk);
      }
    };
    auto mma = [&](int d) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i][j] = mma3h(ah[d][i], al[d][i], bh[d][j], bl[d][j], acc[i][j]);
    };
    const int nks = NKS > 0 ? NKS : KP / 32;
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d < nks) load(d, d * 32);
    int s = 0;
#pragma unroll
    for (; s + 2 * D <= nks; s += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        mma(d);
        load(d, (s + d + D) * 32);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + d < nks) {
        mma(d);
        if (s + d + D < nks) load(d, (s + d + D) * 32);
      }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + D + d < nks) mma(d);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bb = flat[bias_off + (long)mod * chunk + col0 + j * 16 + c16];
#pragma unroll
      for (int i = 0; i < RT; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r] * in_scale + bb;
          const bool pos = v > 0.f;
          sum[i][j][r] += pos ? v : 0.f;
          const uint64_t bal = __ballot(pos);
          if (c16 == 0 && row0 + i * 16 + 4 * grp + r < Rtot)
            bits[((long)a * bits_rows + sgb[i][r]) * nwords + (col0 + j * 16) / 16] =
                (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[w][i * 16 + 4 * grp + r][j * 16 + c16] = sum[i][j][r];
  __syncthreads();
  const int orow = tid >> 3, oc = (tid & 7) * 8;
  const long row = row0 + orow;
  if (orow < RT * 16 && row < Rtot) {
    const long sg = sample_global(p, (int)row, E, PE, t0);
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      o[c] = (part[0][orow][oc + c] + part[1][orow][oc + c] + part[2][orow][oc + c] + part[3][orow][oc + c]) *
             out_scale;
    if constexpr (OF32) {
      float* Y = reinterpret_cast<float*>(Yv) + sg * Cout + col0 + oc;
      *reinterpret_cast<float4*>(Y) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(Y + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      st8_x4(reinterpret_cast<uint16_t*>(Yv) + sg * Cout + col0 + oc, ylo, o);
    }
  }
}

// ===========================================================================
// the last trunk fc layer (fp32 output) + the actor-critic heads + action sampling in ONE launch, for the rollout's
// one-step forwards: a workgroup = one path x 16 sample rows, wave w = output columns [64w, 64w + 64) of EVERY active
// module in slot order.  Per module the 16 x 64 tile is fc_fwd_x3's (same fragments, same k order, same epilogue and
// ReLU bits) and the wave keeps fc_fwd_x3's four per-wave slot partials (slots k, k + 4, ...) in registers and sums
// them in the same order; the 16 x 256 feature rows go to Y and to LDS, and the heads run heads_fwd_s16_kernel<8, float>'s
// arithmetic on them (16 feature slices x 16 samples, slices summed in order).  Bit-identical to the two launches;
// one launch and no feature round trip instead of two chains of ~8-16 us each.
// grid = (ceil(E / 16), P), T = 1.
// ===========================================================================
template <int NKS, int D>
__global__ __launch_bounds__(256) void fc_heads_fwd_x3(const uint16_t* __restrict__ X, long xlo, int ldx,
                                                       float* __restrict__ Y, uint16_t* __restrict__ bits,
                                                       const uint16_t* __restrict__ Wc, long wlo,
                                                       const float* __restrict__ flat, long bias_off, int chunk,
                                                       const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                       int layer, int L, int M, int P, int E, int t0, long bits_rows,
                                                       float in_scale, float out_scale, long pw, long pb, long vw,
                                                       long vb, int A, float* __restrict__ logits,
                                                       float* __restrict__ value, int* __restrict__ actions,
                                                       uint32_t seed, const long long* __restrict__ ctr, int t,
                                                       int Tsteps, int greedy, uint32_t rb) {
  constexpr int COUT = 256, KP = NKS * 32, F = COUT, AM = 8, AW = AM + 1, NWORDS = COUT / 16;
  __shared__ __attribute__((aligned(16))) float feat_s[16][F + 4];
  __shared__ float Wl[F * AW];
  __shared__ float red[16 * AW * 16];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int PE = P * E;
  const int row0 = (int)blockIdx.x * 16;
  const int col0 = w * 64;
  // heads weights [F][AW] (policy columns zero-padded to AM, then the value weight): independent of the fc work
  for (int i = tid; i < F * AW; i += 256) {
    const int f = i / AW, j = i - f * AW;
    Wl[i] = j == AM ? flat[vw + f] : (j < A ? flat[pw + (long)f * A + j] : 0.f);
  }
  const long xrow = sample_global(p, row0 + c16 < E ? row0 + c16 : row0, E, PE, t0) * ldx;
  long sgb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + 4 * grp + r;
    sgb[r] = sample_global(p, row < E ? row : row0, E, PE, t0);
  }
  // slot partials as fc_fwd_x3's waves keep them (partial k = slots k, k + 4, ... in order), summed in order below
  float tot[4][4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tot[k][j][r] = 0.f;
  for (int a = 0; a < cnt; ++a) {
    const int ka = a & 3;                 // the partial this slot joins (adding 0.f to the others is exact)
    const int mod = act_idx[(p * L + layer) * M + a];
    const uint16_t* Wm = Wc + (long)mod * COUT * KP + (long)(col0 + c16) * KP + 8 * grp;
    f4v acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = {0.f, 0.f, 0.f, 0.f};
    s8v ah[D], al[D], bh[D][4], bl[D][4];
    auto load = [&](int d, int kk) {
      ah[d] = *reinterpret_cast<const s8v*>(X + xrow + kk + 8 * grp);
      al[d] = *reinterpret_cast<const s8v*>(X + xlo + xrow + kk + 8 * grp);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bh[d][j] = *reinterpret_cast<const s8v*>(Wm + (long)j * 16 * KP + kk);
        bl[d][j] = *reinterpret_cast<const s8v*>(Wm + wlo + (long)j * 16 * KP + kk);
      }
    };
    auto mma = [&](int d) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = mma3h(ah[d], al[d], bh[d][j], bl[d][j], acc[j]);
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d < NKS) load(d, d * 32);
    int s = 0;
#pragma unroll
    for (; s + 2 * D <= NKS; s += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        mma(d);
        load(d, (s + d + D) * 32);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + d < NKS) {
        mma(d);
        if (s + d + D < NKS) load(d, (s + d + D) * 32);
      }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + D + d < NKS) mma(d);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bb = flat[bias_off + (long)mod * chunk + col0 + j * 16 + c16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[j][r] * in_scale + bb;
        const bool pos = v > 0.f;
        const float pv = pos ? v : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) tot[k][j][r] += ka == k ? pv : 0.f;
        const uint64_t bal = __ballot(pos);
        if (c16 == 0 && row0 + 4 * grp + r < E)
          bits[((long)a * bits_rows + sgb[r]) * NWORDS + (col0 + j * 16) / 16] =
              (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
      }
    }
  }
  // features: Y (the heads backward and the next update's inputs read it) and the LDS rows of the heads
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = 4 * grp + r;
      const float y = (((tot[0][j][r] + tot[1][j][r]) + tot[2][j][r]) + tot[3][j][r]) * out_scale;
      feat_s[lr][col0 + j * 16 + c16] = row0 + lr < E ? y : 0.f;
      if (row0 + lr < E) Y[sgb[r] * COUT + col0 + j * 16 + c16] = y;
    }
  __syncthreads();
  // heads_fwd_s16_kernel: thread (feature slice fs, sample sl)
  const int fs = tid >> 4, sl = tid & 15;
  const bool valid = row0 + sl < E;
  float hacc[AW];
#pragma unroll
  for (int j = 0; j < AW; ++j) hacc[j] = 0.f;
  constexpr int FQ = F / 16;
  for (int f = fs * FQ; f < fs * FQ + FQ; f += 8) {
    float x[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) x[jj] = feat_s[sl][f + jj];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) heads_fma<AW>(hacc, x[jj], Wl + (f + jj) * AW);
  }
#pragma unroll
  for (int j = 0; j < AW; ++j) red[(fs * AW + j) * 16 + sl] = hacc[j];
  __syncthreads();
  if (fs != 0 || !valid) return;
#pragma unroll
  for (int j = 0; j < AW; ++j) {
    float v = 0.f;
    for (int k = 0; k < 16; ++k) v += red[(k * AW + j) * 16 + sl];
    hacc[j] = v;
  }
  const int b = p * E + row0 + sl;                     // the sample's row of this step's [B] buffers
  const uint32_t stepkey = (uint32_t)(ctr[0] * Tsteps + t);
  int best = 0;
  float bv = -3.0e38f;
#pragma unroll
  for (int j = 0; j < AM; ++j) {
    if (j < A) {
      const float lg = hacc[j] + flat[pb + j];
      logits[(long)b * A + j] = lg;
      float sc = lg;
      if (!greedy) sc += -__logf(-__logf(sample_u01(seed, stepkey, rb + (uint32_t)b, (uint32_t)j)));
      if (sc > bv) { bv = sc; best = j; }
    }
  }
  value[b] = hacc[AM] + flat[vb];
  actions[b] = best;
}

// ===========================================================================
// fc forward, split-K: fc_fwd_x3 with KS waves per module (KS x 256 threads), each summing 1/KS of the k-steps;
// the partial accumulators of a module meet in LDS before its bias + ReLU.  The rollout's fc launches have one
// workgroup per (path, 64 columns) -- 256 workgroups at the bench shape -- so the module-per-wave kernel runs one
// wave per SIMD and waits on its weight loads; KS multiplies the waves in flight on the same traffic.
// ===========================================================================
template <int RT, int D, int NKS, bool OF32, int KS>
__global__ __launch_bounds__(256 * KS) void fc_fwd_ks_x3(const uint16_t* __restrict__ X, long xlo, int ldx,
                                                         void* __restrict__ Yv, long ylo, uint16_t* __restrict__ bits,
                                                         const uint16_t* __restrict__ Wc, long wlo,
                                                         const float* __restrict__ flat, long bias_off, int chunk,
                                                         const int* __restrict__ act_idx,
                                                         const int* __restrict__ act_cnt, int layer, int L, int M,
                                                         int K, int KP, int Cout, int P, int E, int T, int t0,
                                                         long bits_rows, float in_scale, float out_scale) {
  static_assert(KS >= 2 && KS <= 4, "split-K 2..4");
  __shared__ float kpart[KS - 1][4][RT * 16][64 + 4];
  __shared__ float part[4][32][64 + 1];
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int mw = w & 3, kp = w >> 2;
  const int grp = l >> 4, c16 = l & 15;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * 32;
  const int col0 = blockIdx.y * 64;
  long xrow[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const long r = row0 + i * 16 + c16;
    xrow[i] = sample_global(p, (int)(r < Rtot ? r : row0), E, PE, t0) * ldx;
  }
  // per-module-lane ReLU sums live in LDS (part[mw]: only the k-part-0 wave of lane mw writes it), not in VGPRs
  for (int x = tid; x < 4 * 32 * 65; x += 256 * KS) (&part[0][0][0])[x] = 0.f;
  const int nwords = Cout / 16;
  const int nks = NKS > 0 ? NKS : KP / 32;
  const int kb = kp * nks / KS, nk = (kp + 1) * nks / KS - kb;
  const int nit = (cnt + 3) >> 2;
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int a = mw + 4 * it;
    const bool act = a < cnt;
    f4v acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
    const int mod = act ? act_idx[(p * L + layer) * M + a] : 0;
    if (act) {
      const uint16_t* Wm = Wc + (long)mod * Cout * KP + (long)(col0 + c16) * KP + 8 * grp;
      s8v ah[D][RT], al[D][RT], bh[D][4], bl[D][4];
      auto load = [&](int d, int ks) {
        const int kk = (kb + ks) * 32;
        const int k0 = kk + 8 * grp;
#pragma unroll
        for (int i = 0; i < RT; ++i) {
          if (K == KP) {
            ah[d][i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
            al[d][i] = *reinterpret_cast<const s8v*>(X + xlo + xrow[i] + k0);
          } else {
            ah[d][i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
            al[d][i] = ah[d][i];
            if (k0 < K) {
              ah[d][i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
              al[d][i] = *reinterpret_cast<const s8v*>(X + xlo + xrow[i] + k0);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bh[d][j] = *reinterpret_cast<const s8v*>(Wm + (long)j * 16 * KP + kk);
          bl[d][j] = *reinterpret_cast<const s8v*>(Wm + wlo + (long)j * 16 * KP + kk);
        }
      };
      auto mma = [&](int d) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < RT; ++i) acc[i][j] = mma3h(ah[d][i], al[d][i], bh[d][j], bl[d][j], acc[i][j]);
      };
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (d < nk) load(d, d);
      int s = 0;
      for (; s + 2 * D <= nk; s += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          mma(d);
          load(d, s + d + D);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (s + d < nk) {
          mma(d);
          if (s + d + D < nk) load(d, s + d + D);
        }
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (s + D + d < nk) mma(d);
      if (kp > 0) {
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) kpart[kp - 1][mw][i * 16 + 4 * grp + r][j * 16 + c16] = acc[i][j][r];
      }
    }
    __syncthreads();
    if (kp == 0 && act) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float bb = flat[bias_off + (long)mod * chunk + col0 + j * 16 + c16];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j][r];
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) v += kpart[q][mw][i * 16 + 4 * grp + r][j * 16 + c16];
            v = v * in_scale + bb;
            const bool pos = v > 0.f;
            part[mw][i * 16 + 4 * grp + r][j * 16 + c16] += pos ? v : 0.f;
            const uint64_t bal = __ballot(pos);
            const long row = row0 + i * 16 + 4 * grp + r;
            if (c16 == 0 && row < Rtot)
              bits[((long)a * bits_rows + sample_global(p, (int)row, E, PE, t0)) * nwords + (col0 + j * 16) / 16] =
                  (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
          }
        }
      }
    }
    __syncthreads();
  }
  if (tid >= 256) return;
  const int orow = tid >> 3, oc = (tid & 7) * 8;
  const long row = row0 + orow;
  if (orow < RT * 16 && row < Rtot) {
    const long sg = sample_global(p, (int)row, E, PE, t0);
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      o[c] = (part[0][orow][oc + c] + part[1][orow][oc + c] + part[2][orow][oc + c] + part[3][orow][oc + c]) *
             out_scale;
    if constexpr (OF32) {
      float* Y = reinterpret_cast<float*>(Yv) + sg * Cout + col0 + oc;
      *reinterpret_cast<float4*>(Y) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(Y + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      st8_x4(reinterpret_cast<uint16_t*>(Yv) + sg * Cout + col0 + oc, ylo, o);
    }
  }
}

// ===========================================================================
// fc forward, MODULE-MAJOR (share each module's weight slice across the paths that use it).
// The path-major kernel above re-reads a module's [Cout][KP] hi/lo slice once per (path, 64-column tile): 553 MB
// of L2/MALL traffic per fc1 launch at the bench shape.  Here one workgroup = one active module j x 64 rows (4 row
// tiles of 16 taken from the paths on j's inverse list, ga.hip ga_compact_inverse_kernel) x all 256 columns, so
// the slice is read once per 64 rows; 8 waves: wave w owns column quarter w & 3 and k half w >> 2 (split-K, the
// halves meet in LDS).  relu(W_j x + b_j) goes to the path's slot plane Ys[slot][p*R + r][256] (fp32), the relu
// bits straight to `bits`; fc_slot_sum_x3 sums every path's slots in slot order (deterministic) into Y.  The
// (module, chunk) units are walked XCD-major -- XCD x takes the x-th contiguous eighth of the unit list -- so an
// XCD's L2 holds the slices of ~2 modules rather than all of them.
// ===========================================================================
template <int NKS>
__global__ __launch_bounds__(512) void fc_fwd_mm_x3(const uint16_t* __restrict__ X, long xlo, int ldx,
                                                    float* __restrict__ Ys, uint16_t* __restrict__ bits,
                                                    const uint16_t* __restrict__ Wc, long wlo,
                                                    const float* __restrict__ flat, long bias_off, int chunk,
                                                    const int* __restrict__ inv_path, const int* __restrict__ inv_slot,
                                                    const int* __restrict__ inv_cnt, int layer, int M, int KP, int P,
                                                    int E, int T, int t0, long bits_rows, float in_scale) {
  constexpr int COUT = 256, RTW = 4, D = 2, NWORDS = COUT / 16;
  constexpr int CPW = 2;                               // 16-column tiles per wave
  constexpr int NH = COUT / (4 * 16 * CPW);            // column slices per (module, 64 rows): units = chunks x NH
  __shared__ float red[4][64][16 * CPW + 4];           // k-half-1 partials per wave column slice
  const int R = T * E, tpp = (R + 15) / 16;
  int U = 0;
  for (int j = 0; j < M; ++j) U += NH * ((inv_cnt[layer * M + j] * tpp + RTW - 1) / RTW);
  const int per = (U + 7) >> 3;
  const int kx = (int)(blockIdx.x >> 3);
  int u = (int)(blockIdx.x & 7) * per + kx;
  if (kx >= per || u >= U) return;
  int j = 0, ncnt = 0;
  for (; j < M; ++j) {
    ncnt = inv_cnt[layer * M + j];
    const int n = NH * ((ncnt * tpp + RTW - 1) / RTW);
    if (u < n) break;
    u -= n;
  }
  const int hslice = u % NH;
  u /= NH;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int cq = w & 3, kh = w >> 2;
  const int cbase = (hslice * 4 + cq) * 16 * CPW;      // first output column of this wave
  const int PE = P * E;
  const long lbase = ((long)layer * M + j) * P;
  int xrow[RTW];                                       // element offsets (the activation buffer is < 2^31)
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int tile = u * RTW + i;
    const int q = tile / tpp, lt = tile - q * tpp;
    const bool tv = q < ncnt;
    const int r = lt * 16 + c16;
    xrow[i] = (int)sample_global(inv_path[lbase + (tv ? q : 0)], tv && r < R ? r : 0, E, PE, t0) * ldx;
  }
  const uint16_t* Wm = Wc + (long)j * COUT * KP + (long)(cbase + c16) * KP + 8 * grp;
  f4v acc[RTW][CPW];
#pragma unroll
  for (int i = 0; i < RTW; ++i)
#pragma unroll
    for (int jj = 0; jj < CPW; ++jj) acc[i][jj] = {0.f, 0.f, 0.f, 0.f};
  s8v ah[D][RTW], al[D][RTW], bh[D][CPW], bl[D][CPW];
  auto load = [&](int d, int kk) {
    const int k0 = kk + 8 * grp;
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
      ah[d][i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
      al[d][i] = *reinterpret_cast<const s8v*>(X + xlo + xrow[i] + k0);
    }
#pragma unroll
    for (int jj = 0; jj < CPW; ++jj) {
      bh[d][jj] = *reinterpret_cast<const s8v*>(Wm + (long)jj * 16 * KP + kk);
      bl[d][jj] = *reinterpret_cast<const s8v*>(Wm + wlo + (long)jj * 16 * KP + kk);
    }
  };
  auto mma = [&](int d) {
#pragma unroll
    for (int jj = 0; jj < CPW; ++jj)
#pragma unroll
      for (int i = 0; i < RTW; ++i) acc[i][jj] = mma3h(ah[d][i], al[d][i], bh[d][jj], bl[d][jj], acc[i][jj]);
  };
  const int nks = NKS > 0 ? NKS : KP / 32;
  const int ks0 = kh ? nks / 2 : 0, nk = kh ? nks - nks / 2 : nks / 2;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < nk) load(d, (ks0 + d) * 32);
  int s = 0;
#pragma unroll 1
  for (; s + 2 * D <= nk; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      mma(d);
      load(d, (ks0 + s + d + D) * 32);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (s + d < nk) {
      mma(d);
      if (s + d + D < nk) load(d, (ks0 + s + d + D) * 32);
    }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (s + D + d < nk) mma(d);
  if (kh) {
#pragma unroll
    for (int i = 0; i < RTW; ++i)
#pragma unroll
      for (int jj = 0; jj < CPW; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[cq][i * 16 + 4 * grp + r][jj * 16 + c16] = acc[i][jj][r];
  }
  __syncthreads();
  if (kh) return;
  const long PR = (long)P * R;
  int pth[RTW], slot[RTW], rbase[RTW];
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    const int tile = u * RTW + i;
    const int q = tile / tpp;
    const bool tv = q < ncnt;
    pth[i] = tv ? inv_path[lbase + q] : -1;
    slot[i] = tv ? inv_slot[lbase + q] : 0;
    rbase[i] = (tile - q * tpp) * 16;
  }
#pragma unroll
  for (int jj = 0; jj < CPW; ++jj) {
    const int col = cbase + jj * 16;
    const float bb = flat[bias_off + (long)j * chunk + col + c16];
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase[i] + 4 * grp + r;
        const bool ok = pth[i] >= 0 && row < R;
        const float v = (acc[i][jj][r] + red[cq][i * 16 + 4 * grp + r][jj * 16 + c16]) * in_scale + bb;
        const bool pos = v > 0.f;
        const uint64_t bal = __ballot(pos);
        if (ok) {
          Ys[((long)slot[i] * PR + (long)pth[i] * R + row) * COUT + col + c16] = pos ? v : 0.f;
          if (c16 == 0)
            bits[((long)slot[i] * bits_rows + sample_global(pth[i], row, E, PE, t0)) * NWORDS + col / 16] =
                (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
        }
      }
    }
  }
}

// ===========================================================================
// fc forward, module-major with LDS-staged tiles.  fc_fwd_mm_x3 above shares a module's weights across paths but
// keeps the path-major kernel's ratio of global fragment loads to MFMAs (12 16-byte loads per 24 MFMAs per wave),
// and that ratio is what bounds both: the kernel waits on its L1/L2 fragment traffic, not on HBM.  Here a
// workgroup = one active module j x 128 rows (taken from the paths on j's inverse list) x 128 columns; each k-step
// stages the A tile [128 rows][32] and B tile [128 columns][32] (fp16 hi/lo planes, 32 KB) once in LDS with four
// 16-byte loads per thread, and 8 waves (2 x 4, wave tile 64 rows x 32 columns) read them: 12 ds_read_b128 per
// 24 MFMAs, each global byte read once per workgroup.  Double-buffered LDS, next k-step's loads in registers.  LDS
// rows are 64 B with the 16-byte chunk index XORed by (-(row >> 2)) & 3, conflict-free for the ds_read_b128 lane
// groups of the MFMA operand reads.  relu(W_j x + b_j) -> slot plane Ys, bits -> `bits`; fc_slot_sum_x3 sums.
// ===========================================================================
DEVI int mm2_sw(int row, int ch) { return (row << 2) + (ch ^ ((-(row >> 2)) & 3)); }   // 16-byte chunk index

template <int NKS, int PF, int KS>
__global__ __launch_bounds__(512, 2) void fc_fwd_mm2_x3(const uint16_t* __restrict__ X, long xlo, int ldx,
                                                       float* __restrict__ Ys, uint16_t* __restrict__ bits,
                                                       const uint16_t* __restrict__ Wc, long wlo,
                                                       const float* __restrict__ flat, long bias_off, int chunk,
                                                       const int* __restrict__ inv_path,
                                                       const int* __restrict__ inv_slot,
                                                       const int* __restrict__ inv_cnt, int layer, int M, int KP, int P,
                                                       int E, int T, int t0, long bits_rows, float in_scale) {
  constexpr int COUT = 256, BR = 128, BC = 128, NCS = COUT / BC, NWORDS = COUT / 16;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][2][BR * 32];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][2][BC * 32];
  const int R = T * E;
  // unit -> (module j, row block, column half, k part); units of module j = ceil(inv_cnt[j] * R / 128) x NCS x KS.
  // (An XCD-major walk -- a module's workgroups on one XCD -- measured slower: 46.3 vs 44.1 us, kwin_x3_v17.md;
  // consecutive units go round-robin over the XCDs.)
  int u = (int)blockIdx.x, j = 0, ncnt = 0;
  for (; j < M; ++j) {
    ncnt = inv_cnt[layer * M + j];
    const int n = KS * NCS * ((ncnt * R + BR - 1) / BR);
    if (u < n) break;
    u -= n;
  }
  if (j >= M) return;
  const int kpart = u % KS;
  u /= KS;
  const int chalf = u % NCS, rb = u / NCS;
  const int nrows = ncnt * R;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int wr = w >> 2, wc = w & 3;                     // wave tile: rows 64*wr.., columns 32*wc.. of the block
  const int PE = P * E;
  const long lbase = ((long)layer * M + j) * P;
  const int col0 = chalf * BC;
  // staging role: thread -> (row / column srow, 16-byte chunk skc) of the 128 x 32 tiles
  const int srow = tid >> 2, skc = tid & 3;
  long xoff;
  {
    const int gr = rb * BR + srow;
    const int q = gr < nrows ? gr / R : 0, rr = gr < nrows ? gr - q * R : 0;
    xoff = sample_global(inv_path[lbase + q], rr, E, PE, t0) * (long)ldx + skc * 8;
  }
  // KS > 1: this workgroup sums k-steps [ks_beg, ks_beg + nks) only; the pre-activation partials of the parts go
  // to separate planes of Ys and fc_slot_sum2_x3 adds them, then bias, ReLU, bits and the module sum
  const int nks_all = NKS > 0 ? NKS : KP / 32;
  const int ks_beg = kpart * (nks_all / KS) + min(kpart, nks_all % KS);
  const int nks = nks_all / KS + (kpart < nks_all % KS ? 1 : 0);
  xoff += (long)ks_beg * 32;
  const uint16_t* wsrc = Wc + ((long)j * COUT + col0 + srow) * KP + skc * 8 + ks_beg * 32;
  const int sdst = mm2_sw(srow, skc) * 8;
  // PF register sets of k-step loads in flight (a k-step's MFMA work is ~400 cycles per wave, far below the
  // L2/MALL latency of its loads: one step of lookahead left the kernel waiting on every step).  Plain vector
  // registers (a struct array captured by the lambdas went to scratch).
  static_assert(PF == 3, "three named register sets (an indexed array of them went to scratch)");
  uint4 ga0, gx0, gb0, gy0, ga1, gx1, gb1, gy1, ga2, gx2, gb2, gy2;
#define MM2_GLOAD(d, ks)                                                     \
  do {                                                                       \
    const int k0_ = (ks) * 32;                                               \
    ga##d = *reinterpret_cast<const uint4*>(X + xoff + k0_);                 \
    gx##d = *reinterpret_cast<const uint4*>(X + xlo + xoff + k0_);           \
    gb##d = *reinterpret_cast<const uint4*>(wsrc + k0_);                     \
    gy##d = *reinterpret_cast<const uint4*>(wsrc + wlo + k0_);               \
  } while (0)
#define MM2_LSTORE(d, buf)                                                   \
  do {                                                                       \
    *reinterpret_cast<uint4*>(&As[buf][0][sdst]) = ga##d;                    \
    *reinterpret_cast<uint4*>(&As[buf][1][sdst]) = gx##d;                    \
    *reinterpret_cast<uint4*>(&Bs[buf][0][sdst]) = gb##d;                    \
    *reinterpret_cast<uint4*>(&Bs[buf][1][sdst]) = gy##d;                    \
  } while (0)
  f4v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = (f4v){0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    s8v bh[2], bl[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int o = mm2_sw(wc * 32 + jj * 16 + c16, grp) * 8;
      bh[jj] = *reinterpret_cast<const s8v*>(&Bs[buf][0][o]);
      bl[jj] = *reinterpret_cast<const s8v*>(&Bs[buf][1][o]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = mm2_sw(wr * 64 + i * 16 + c16, grp) * 8;
      const s8v ah = *reinterpret_cast<const s8v*>(&As[buf][0][o]);
      const s8v al = *reinterpret_cast<const s8v*>(&As[buf][1][o]);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mma3h(ah, al, bh[jj], bl[jj], acc[i][jj]);
    }
  };
  MM2_GLOAD(0, 0);
  MM2_LSTORE(0, 0);
  if (1 < nks) MM2_GLOAD(0, 1);                    // set d holds k-step d + 1, then d + 1 + PF, ...
  if (2 < nks) MM2_GLOAD(1, 2);
  if (3 < nks) MM2_GLOAD(2, 3);
  __syncthreads();
  // full groups of PF steps: every reload unconditional (clamped to the last k-step; a conditional reload is a
  // loop-carried phi), the remainder peeled.  Buffer (ks + 1) & 1 was last read in step ks - 1, before the
  // barrier that ended it; after the last step the store is dead (nothing reads that buffer again).
#define MM2_STEP(d, ks)                                                      \
  do {                                                                       \
    compute((ks) & 1);                                                       \
    MM2_LSTORE(d, ((ks) + 1) & 1);                                           \
    MM2_GLOAD(d, min((ks) + 1 + PF, nks - 1));                               \
    __syncthreads();                                                         \
  } while (0)
  int k0 = 0;
  for (; k0 + PF <= nks; k0 += PF) {
    MM2_STEP(0, k0);
    MM2_STEP(1, k0 + 1);
    MM2_STEP(2, k0 + 2);
  }
  if (k0 < nks) { compute(k0 & 1); MM2_LSTORE(0, (k0 + 1) & 1); __syncthreads(); }
  if (k0 + 1 < nks) { compute((k0 + 1) & 1); MM2_LSTORE(1, (k0 + 2) & 1); __syncthreads(); }
#undef MM2_STEP
#undef MM2_GLOAD
#undef MM2_LSTORE
  // epilogue: rows-as-A D layout (lane: rows 4*grp + r of each 16-row tile, column c16), bits as 16-bit ballots
  const long PR = (long)P * R;
  if constexpr (KS > 1) {
    float* Yp = Ys + (long)kpart * M * PR * COUT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gr0 = rb * BR + wr * 64 + i * 16 + 4 * grp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = gr0 + r;
        if (gr >= nrows) continue;
        const int q = gr / R;
        const long o = ((long)inv_slot[lbase + q] * PR + (long)inv_path[lbase + q] * R + (gr - q * R)) * COUT;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) Yp[o + col0 + wc * 32 + jj * 16 + c16] = acc[i][jj][r] * in_scale;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gr0 = rb * BR + wr * 64 + i * 16 + 4 * grp;
    int pth[4], slt[4], rr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = gr0 + r;
      const int q = gr < nrows ? gr / R : -1;
      pth[r] = q >= 0 ? inv_path[lbase + q] : -1;
      slt[r] = q >= 0 ? inv_slot[lbase + q] : 0;
      rr[r] = q >= 0 ? gr - q * R : 0;
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int col = col0 + wc * 32 + jj * 16;
      const float bb = flat[bias_off + (long)j * chunk + col + c16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[i][jj][r] * in_scale + bb;
        const bool pos = v > 0.f;
        const uint64_t bal = __ballot(pos);
        if (pth[r] >= 0) {
          Ys[((long)slt[r] * PR + (long)pth[r] * R + rr[r]) * COUT + col + c16] = pos ? v : 0.f;
          if (c16 == 0)
            bits[((long)slt[r] * bits_rows + sample_global(pth[r], rr[r], E, PE, t0)) * NWORDS + col / 16] =
                (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
        }
      }
    }
  }
}

// KS-part partials of the module-major fc forward -> per slot: sum of the parts + bias, ReLU, the 16-bit ReLU word
// of (slot, row, 16 columns); the slots summed in slot order -> Y.  One thread per (row, 8 columns); the two threads
// of a 16-column word (adjacent lanes) join their ReLU bytes with one xor-1 exchange.
template <bool OF32, int KS>
__global__ __launch_bounds__(256) void fc_slot_sum2_x3(const float* __restrict__ Ys, const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, const float* __restrict__ flat,
                                                       long bias_off, int chunk, uint16_t* __restrict__ bits,
                                                       long bits_rows, int layer, int L, int M, int P, int E, int T,
                                                       int t0, void* __restrict__ Yv, long ylo, float out_scale) {
  constexpr int COUT = 256, NWORDS = COUT / 16;
  const int R = T * E;
  const long PR = (long)P * R;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = idx >> 5;                                   // 32 threads per row: whole waves share 2 rows
  const int c0 = (int)(idx & 31) * 8;
  const bool live = row < PR;
  const long rowc = live ? row : 0;
  const int p = (int)(rowc / R), r = (int)(rowc - (long)p * R);
  // act_cnt and the slot's module index are loaded side by side (the index list is padded with -1 past the count,
  // so it does not wait for it), and the first slot's partial planes go out with them: one dependent load level
  // (the bias) instead of three in front of the first sum
  const int cnt = live ? act_cnt[p * L + layer] : 0;
  const int mod0 = act_idx[(p * L + layer) * M];
  float4 x0[KS], y0[KS];
#pragma unroll
  for (int kp = 0; kp < KS; ++kp) {
    const float* src = Ys + (((long)kp * M) * PR + rowc) * COUT + c0;
    x0[kp] = *reinterpret_cast<const float4*>(src);
    y0[kp] = *reinterpret_cast<const float4*>(src + 4);
  }
  const long sg = sample_global(p, r, E, P * E, t0);
  float o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = 0.f;
  // the xor-1 partner is in the same row (32 lanes per row), so it runs the same slot count
  for (int a = 0; a < cnt; ++a) {
    float v[8];
    const int mod = a == 0 ? mod0 : act_idx[(p * L + layer) * M + a];
    const float* bsrc = flat + bias_off + (long)mod * chunk + c0;      // (no alignment assumed)
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = bsrc[c];
#pragma unroll
    for (int kp = 0; kp < KS; ++kp) {
      float4 x, y;
      if (a == 0) {
        x = x0[kp];
        y = y0[kp];
      } else {
        const float* src = Ys + (((long)kp * M + a) * PR + row) * COUT + c0;
        x = *reinterpret_cast<const float4*>(src);
        y = *reinterpret_cast<const float4*>(src + 4);
      }
      v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
      v[4] += y.x; v[5] += y.y; v[6] += y.z; v[7] += y.w;
    }
    uint32_t byte = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bool pos = v[c] > 0.f;
      byte |= pos ? (1u << c) : 0u;
      o[c] += pos ? v[c] : 0.f;
    }
    const uint32_t other = (uint32_t)__shfl_xor((int)byte, 1, 64);
    if ((c0 & 8) == 0) bits[((long)a * bits_rows + sg) * NWORDS + (c0 >> 4)] = (uint16_t)(byte | (other << 8));
  }
  if (!live) return;
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] *= out_scale;
  if constexpr (OF32) {
    float* Y = reinterpret_cast<float*>(Yv) + sg * COUT + c0;
    *reinterpret_cast<float4*>(Y) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(Y + 4) = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    st8_x4(reinterpret_cast<uint16_t*>(Yv) + sg * COUT + c0, ylo, o);
  }
}

// sum every path's module slots in slot order (one thread per row x 8 columns) -> Y (fp32, or an fp16 pair)
template <bool OF32>
__global__ __launch_bounds__(256) void fc_slot_sum_x3(const float* __restrict__ Ys, const int* __restrict__ act_cnt,
                                                      int layer, int L, int P, int E, int T, int t0,
                                                      void* __restrict__ Yv, long ylo, float out_scale) {
  constexpr int COUT = 256;
  const int R = T * E;
  const long PR = (long)P * R;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = idx >> 5;
  const int c8 = (int)(idx & 31) * 8;
  if (row >= PR) return;
  const int p = (int)(row / R), r = (int)(row - (long)p * R);
  const int cnt = act_cnt[p * L + layer];
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int a = 0; a < cnt; ++a) {
    const float4* src = reinterpret_cast<const float4*>(Ys + ((long)a * PR + row) * COUT + c8);
    const float4 x = src[0], y = src[1];
    o[0] += x.x; o[1] += x.y; o[2] += x.z; o[3] += x.w;
    o[4] += y.x; o[5] += y.y; o[6] += y.z; o[7] += y.w;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] *= out_scale;
  const long sg = sample_global(p, r, E, P * E, t0);
  if constexpr (OF32) {
    float* Y = reinterpret_cast<float*>(Yv) + sg * COUT + c8;
    *reinterpret_cast<float4*>(Y) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(Y + 4) = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    st8_x4(reinterpret_cast<uint16_t*>(Yv) + sg * COUT + c8, ylo, o);
  }
}

// ===========================================================================
// fc input gradient (trunk_bwd.hip fc_dgrad_lds_kernel): per workgroup 64 rows; the masked gradient of 2 active
// slots is split into hi/lo planes in LDS (135 KB: 1 workgroup of 512 threads per CU), every 128-column chunk of
// dX is swept with the hi/lo weight fragments of WcT [2][M][KP][COUT] in registers (next iteration's prefetched).
// Slot groups beyond the first add into dX.  Gm (optional): the masked hi/lo gradient per slot for the weight
// gradient, [2][M][bits_rows][COUT] (lo plane at +gmlo).  1-D grid (split, path, row block), XCD-aware order.
// ===========================================================================
template <int COUT>
__global__ __launch_bounds__(512) void fc_dgrad_x3(const float* __restrict__ G, const uint16_t* __restrict__ bits,
                                                   const bf16_t* __restrict__ WcT, long wlo,
                                                   const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                   int layer, int L, int M, int K, int KP, int P, int E, int T,
                                                   long bits_rows, float g_scale, float* __restrict__ dX,
                                                   int chunks_per_split, int nrowb, int nsplit,
                                                   bf16_t* __restrict__ Gm, long gmlo,
                                                   const float* __restrict__ gamax, float* __restrict__ gamax_out) {
  constexpr int CS = COUT + 8;
  constexpr int NW = COUT / 16;
  constexpr int NSL = 2;                               // slots per group
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][NSL * 64 * CS];
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
  long sg_out[4][4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + rb * 16 + 4 * grp + r;
      sg_out[rb][r] = row < R ? sample_global(p, (int)row, E, PE, 0) : -1;
    }
  const int ngroups = cnt > 0 ? (cnt + NSL - 1) / NSL : 1;
  const float gs = g16_scale(gamax), inv = 1.0f / (gs * (float)(1 << X3_W0_SHIFT));
  float am = 0.f;
  for (int gi = 0; gi < ngroups; ++gi) {
    const int g0 = gi * NSL;
    const int ng = min(NSL, cnt - g0);
    __syncthreads();
    {
      constexpr int SEG = COUT / 8;
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
          s8v hi, lo;
          split8hs(m, gs, hi, lo);
          *reinterpret_cast<s8v*>(Gs[0] + (a * 64 + sr) * CS + c) = hi;
          *reinterpret_cast<s8v*>(Gs[1] + (a * 64 + sr) * CS + c) = lo;
          if (Gm != nullptr && v && (tid & 7) % nsplit == bz) {
            bf16_t* gp = Gm + ((long)(g0 + a) * bits_rows + sg) * COUT + c;
            *reinterpret_cast<s8v*>(gp) = hi;
            *reinterpret_cast<s8v*>(gp + gmlo) = lo;
          }
        }
      }
    }
    __syncthreads();
    if (ng <= 0) {
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
    s8v b0h[COUT / 32], b0l[COUT / 32], b1h[COUT / 32], b1l[COUT / 32];
    auto wload = [&](s8v* bh, s8v* bl, int it) {
      const int ch = ch_beg + it / ng, a = it - (it / ng) * ng;
      const int kc = ch * 128 + w * 16 + c16;
      const bf16_t* Wm = WcT + (long)aidx[a] * KP * COUT + (long)kc * COUT + 8 * grp;
#pragma unroll
      for (int c = 0; c < COUT / 32; ++c) {
        bh[c] = kc < KP ? *reinterpret_cast<const s8v*>(Wm + 32 * c) : (s8v){0, 0, 0, 0, 0, 0, 0, 0};
        bl[c] = kc < KP ? *reinterpret_cast<const s8v*>(Wm + wlo + 32 * c) : (s8v){0, 0, 0, 0, 0, 0, 0, 0};
      }
    };
    f4v acc[4];
    auto body = [&](const s8v* bh, const s8v* bl, int it) {
      const int ch = ch_beg + it / ng, a = it - (it / ng) * ng;
      if (a == 0) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = {0.f, 0.f, 0.f, 0.f};
      }
      const int ao = (a * 64 + c16) * CS + 8 * grp;
#pragma unroll
      for (int c = 0; c < COUT / 32; ++c)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const s8v fh = *reinterpret_cast<const s8v*>(Gs[0] + ao + rb * 16 * CS + 32 * c);
          const s8v fl = *reinterpret_cast<const s8v*>(Gs[1] + ao + rb * 16 * CS + 32 * c);
          acc[rb] = mma3h(fh, fl, bh[c], bl[c], acc[rb]);
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
              const float v = gi == 0 ? acc[rb][r] * inv : *o + acc[rb][r] * inv;
              *o = v;
              if (gi == ngroups - 1) am = fmaxf(am, fabsf(v));
            }
          }
      }
    };
    wload(b0h, b0l, 0);
    int it = 0;
    for (; it + 2 < n_it; it += 2) {
      wload(b1h, b1l, it + 1);
      body(b0h, b0l, it);
      wload(b0h, b0l, it + 2);
      body(b1h, b1l, it + 1);
    }
    if (it + 1 < n_it) {
      wload(b1h, b1l, it + 1);
      body(b0h, b0l, it);
      body(b1h, b1l, it + 1);
    } else {
      body(b0h, b0l, it);
    }
  }
  g16_flush_amax(am, gamax_out);
}

// ===========================================================================
// fc input gradient as a per-path GEMM with LDS-staged 128 x 256 tiles.  fc_dgrad_x3 above gives a workgroup 64
// rows and streams the path's whole weight set past them (~2.9 MB per workgroup, ~3.6 GB of L2/MALL traffic per
// fc1 backward).  Here the masked, split gradient of every active slot is written once by fc_gm_x3 (the same Gm the
// weight gradient reads), and dX[rows][K] = sum over (slot a, c) Gm[a][row][c] * W_a[k][c] runs as a GEMM with the
// reduction over (a, c) in steps of 32: a workgroup = path x 128 rows x 256 columns of dX, 8 waves (2 x 4, wave
// tile 64 x 64), A [128][32] and B [256][32] hi/lo tiles staged per step (6 16-byte loads per thread, 48 MFMAs per
// wave), two steps of loads in flight, double-buffered LDS with the XOR-swizzled 64-byte rows of fc_fwd_mm2_x3.
// ===========================================================================
template <int COUT>
__global__ __launch_bounds__(256) void fc_gm_x3(const float* __restrict__ G, const uint16_t* __restrict__ bits,
                                                const int* __restrict__ act_cnt, int layer, int L, int P, int E, int T,
                                                long bits_rows, float g_scale, bf16_t* __restrict__ Gm, long gmlo,
                                                const float* __restrict__ gamax) {
  constexpr int NW = COUT / 16, C8 = COUT / 8;
  const int R = T * E;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = idx / C8;
  const int c = (int)(idx - row * C8) * 8;
  if (row >= (long)P * R) return;
  const int p = (int)(row / R), r = (int)(row - (long)p * R);
  const int cnt = act_cnt[p * L + layer];
  const long sg = sample_global(p, r, E, P * E, 0);
  const float4 a0 = *reinterpret_cast<const float4*>(G + sg * COUT + c);
  const float4 a1 = *reinterpret_cast<const float4*>(G + sg * COUT + c + 4);
  const float gv[8] = {a0.x * g_scale, a0.y * g_scale, a0.z * g_scale, a0.w * g_scale,
                       a1.x * g_scale, a1.y * g_scale, a1.z * g_scale, a1.w * g_scale};
  const float gs = g16_scale(gamax);
  for (int a = 0; a < cnt; ++a) {
    const uint32_t bw = (uint32_t)bits[((long)a * bits_rows + sg) * NW + (c >> 4)] >> (c & 15);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = ((bw >> j) & 1u) ? gv[j] : 0.f;
    s8v hi, lo;
    split8hs(m, gs, hi, lo);                   // Gm: the fp16 pair of the masked gradient * 2^e (G16)
    bf16_t* gp = Gm + ((long)a * bits_rows + sg) * COUT + c;
    *reinterpret_cast<s8v*>(gp) = hi;
    *reinterpret_cast<s8v*>(gp + gmlo) = lo;
  }
}

template <int COUT, bool W3 = false, int FOLD = 0>
__global__ __launch_bounds__(512) void fc_dgrad_gemm_x3(const bf16_t* __restrict__ Gm, long gmlo,
                                                        const bf16_t* __restrict__ WcT, long wlo,
                                                        const int* __restrict__ act_idx,
                                                        const int* __restrict__ act_cnt, int layer, int L, int M, int K,
                                                        int KP, int P, int E, int T, long bits_rows,
                                                        float* __restrict__ dX, int nrb, int ncb,
                                                        const float* __restrict__ gamax, float* __restrict__ gamax_out) {
  constexpr int BM = 128, BN = 256, CS = COUT / 32;                 // reduction steps per slot
  constexpr int NBP = W3 ? 3 : 2;                                    // weight pieces staged (W3: + the third)
  __shared__ __attribute__((aligned(16))) bf16_t As[2][2][BM * 32];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][NBP][BN * 32];
  // XCD-major: XCD x (= blockIdx % 8) takes the x-th contiguous eighth of the (path, row block, column block) list,
  // so one path's weight set is fetched into one XCD's L2 rather than into all eight
  const int ntot = P * nrb * ncb, per = (ntot + 7) >> 3, kx = (int)(blockIdx.x >> 3);
  const int bid = (int)(blockIdx.x & 7) * per + kx;
  if (kx >= per || bid >= ntot) return;
  const int p = bid / (nrb * ncb), rem = bid - p * (nrb * ncb);
  const int rbk = rem / ncb, cb = rem - rbk * ncb;
  const int R = T * E, PE = P * E;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const int wm = w >> 2, wn = w & 3;                                 // wave tile: rows 64*wm.., columns 64*wn..
  const int row0 = rbk * BM, col0 = cb * BN;
  const int nsteps = cnt * CS;
  f4v acc[4][4], accn[FOLD == 2 ? 4 : 1][FOLD == 2 ? 4 : 1];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (f4v){0.f, 0.f, 0.f, 0.f};
  if constexpr (FOLD == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) accn[i][jj] = (f4v){0.f, 0.f, 0.f, 0.f};
  }
  if (nsteps > 0) {
    // staging roles: A: thread -> (row tid >> 2, chunk tid & 3), both planes; B: two columns (tid >> 2, + 128)
    const int sr = tid >> 2, sk = tid & 3;
    const int ra = min(row0 + sr, R - 1);
    const long asg = sample_global(p, ra, E, PE, 0);
    const int kb0 = min(col0 + sr, K - 1), kb1 = min(col0 + 128 + sr, K - 1);
    const int* aidx = act_idx + (p * L + layer) * M;
    const int sdA = mm2_sw(sr, sk) * 8, sdB0 = sdA, sdB1 = mm2_sw(sr + 128, sk) * 8;
    // two sets: A hi/lo, B col hi/lo(/third), B col+128 hi/lo(/third)
    uint4 x0, x1, y0, y1, z0, z1, u0, u1, v0, v1, t0_, t1_, r0, r1, q0, q1;
#define DG_LOAD(S, st)                                                                                      \
    do {                                                                                                    \
      const int a_ = (st) / CS, c_ = ((st) - a_ * CS) * 32 + sk * 8;                                        \
      const bf16_t* ga_ = Gm + ((long)a_ * bits_rows + asg) * COUT + c_;                                    \
      const bf16_t* wb_ = WcT + (long)aidx[a_] * KP * COUT + c_;                                            \
      x##S = *reinterpret_cast<const uint4*>(ga_);                                                          \
      y##S = *reinterpret_cast<const uint4*>(ga_ + gmlo);                                                   \
      z##S = *reinterpret_cast<const uint4*>(wb_ + (long)kb0 * COUT);                                       \
      u##S = *reinterpret_cast<const uint4*>(wb_ + wlo + (long)kb0 * COUT);                                 \
      v##S = *reinterpret_cast<const uint4*>(wb_ + (long)kb1 * COUT);                                       \
      t##S##_ = *reinterpret_cast<const uint4*>(wb_ + wlo + (long)kb1 * COUT);                              \
      if constexpr (W3) {                                                                                   \
        r##S = *reinterpret_cast<const uint4*>(wb_ + 2 * wlo + (long)kb0 * COUT);                           \
        q##S = *reinterpret_cast<const uint4*>(wb_ + 2 * wlo + (long)kb1 * COUT);                           \
      }                                                                                                     \
    } while (0)
#define DG_STORE(S, buf)                                                                                    \
    do {                                                                                                    \
      if (FOLD == 2 && (buf) == 1) {            /* odd k-steps: the gradient pieces negated (sign bits) */  \
        x##S.x ^= 0x80008000u; x##S.y ^= 0x80008000u; x##S.z ^= 0x80008000u; x##S.w ^= 0x80008000u;         \
        y##S.x ^= 0x80008000u; y##S.y ^= 0x80008000u; y##S.z ^= 0x80008000u; y##S.w ^= 0x80008000u;         \
      }                                                                                                     \
      *reinterpret_cast<uint4*>(&As[buf][0][sdA]) = x##S;                                                   \
      *reinterpret_cast<uint4*>(&As[buf][1][sdA]) = y##S;                                                   \
      *reinterpret_cast<uint4*>(&Bs[buf][0][sdB0]) = z##S;                                                  \
      *reinterpret_cast<uint4*>(&Bs[buf][1][sdB0]) = u##S;                                                  \
      *reinterpret_cast<uint4*>(&Bs[buf][0][sdB1]) = v##S;                                                  \
      *reinterpret_cast<uint4*>(&Bs[buf][1][sdB1]) = t##S##_;                                               \
      if constexpr (W3) {                                                                                   \
        *reinterpret_cast<uint4*>(&Bs[buf][NBP - 1][sdB0]) = r##S;                                          \
        *reinterpret_cast<uint4*>(&Bs[buf][NBP - 1][sdB1]) = q##S;                                          \
      }                                                                                                     \
    } while (0)
    auto compute = [&](int buf) {
      s8v bh[4], bl[4], br[W3 ? 4 : 1];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int o = mm2_sw(wn * 64 + jj * 16 + c16, grp) * 8;
        bh[jj] = *reinterpret_cast<const s8v*>(&Bs[buf][0][o]);
        bl[jj] = *reinterpret_cast<const s8v*>(&Bs[buf][1][o]);
        if constexpr (W3) br[jj] = *reinterpret_cast<const s8v*>(&Bs[buf][NBP - 1][o]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = mm2_sw(wm * 64 + i * 16 + c16, grp) * 8;
        const s8v ah = *reinterpret_cast<const s8v*>(&As[buf][0][o]);
        const s8v al = *reinterpret_cast<const s8v*>(&As[buf][1][o]);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          // W3: the weights' third piece first (smallest term).  FOLD 1: each k-step's products into a zeroed
          // accumulator, added to the running sum with one IEEE fp32 add.  FOLD 2: odd k-steps run on negated
          // gradient pieces into a second accumulator chain, subtracted at the end: the f16 MFMA's sum is biased
          // toward -inf (measured: mean error / mean |error| = -0.13 on the fc input gradient,
          // scripts/x3_lstm_diag.py), which the weight gradients below sum coherently; on the negated chain the
          // same bias enters with the opposite sign
          if constexpr (FOLD == 2) {
            if (buf == 1) {
              accn[i][jj] = mma3h(ah, al, bh[jj], bl[jj], accn[i][jj]);
              continue;
            }
          }
          f4v c = FOLD == 1 ? (f4v){0.f, 0.f, 0.f, 0.f} : acc[i][jj];
          if constexpr (W3) c = mfma16_f16(ah, br[jj], c);
          c = mma3h(ah, al, bh[jj], bl[jj], c);
          if constexpr (FOLD == 1) acc[i][jj] += c;
          else acc[i][jj] = c;
        }
      }
    };
    // set 0 holds the even steps' loads, set 1 the odd ones; step s stores step s + 1's set, then reloads it with
    // step s + 3 (clamped: a conditional reload is a loop-carried phi); the remainder step is peeled
    DG_LOAD(0, 0);
    DG_STORE(0, 0);
    DG_LOAD(1, min(1, nsteps - 1));
    DG_LOAD(0, min(2, nsteps - 1));
    __syncthreads();
    int s = 0;
    for (; s + 2 <= nsteps; s += 2) {
      compute(0);
      DG_STORE(1, 1);
      DG_LOAD(1, min(s + 3, nsteps - 1));
      __syncthreads();
      compute(1);
      DG_STORE(0, 0);
      DG_LOAD(0, min(s + 4, nsteps - 1));
      __syncthreads();
    }
    if (s < nsteps) compute(0);
#undef DG_LOAD
#undef DG_STORE
  }
  // epilogue: rows-as-A D layout, fp32 dX (zeros for a path with no active slot); Gm * 2^e against W * 2^8, so
  // scaled back by 2^-(e + 8); the amax of dX for the layer below (G16)
  const float inv = 1.0f / (g16_scale(gamax) * (float)(1 << X3_W0_SHIFT));
  float am = 0.f;
  if constexpr (FOLD == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] -= accn[i][jj];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + wm * 64 + i * 16 + 4 * grp + r;
      if (row >= R) continue;
      float* o = dX + sample_global(p, row, E, PE, 0) * (long)K;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int k = col0 + wn * 64 + jj * 16 + c16;
        if (k < K) {
          const float v = acc[i][jj][r] * inv;
          o[k] = v;
          am = fmaxf(am, fabsf(v));
        }
      }
    }
  }
  g16_flush_amax(am, gamax_out);
}

// ===========================================================================
// fc weight gradient from the masked hi/lo gradient Gm written by fc_dgrad_x3 (trunk_bwd.hip fc_wgrad_gm_kernel):
// 128 x COUT tiles, module-major users, 32-row stages of X (hi/lo) and Gm (hi/lo) double-buffered in LDS.
// ===========================================================================
template <int COUT, int KT = 128>
__global__ __launch_bounds__(512) void fc_wgrad_gm_x3(const bf16_t* __restrict__ X, long xlo, int ldx,
                                                      const bf16_t* __restrict__ Gm, long gmlo,
                                                      float* __restrict__ grad, long w_off, long b_off, int chunk,
                                                      const int* __restrict__ inv_path,
                                                      const int* __restrict__ inv_slot,
                                                      const int* __restrict__ inv_cnt, int layer, int M, int Pmax,
                                                      int K, int P, int E, int T, long bits_rows, int nsplit,
                                                      const float* __restrict__ gamax, long long* __restrict__ fx) {
  constexpr int XS = KT + 8;
  constexpr int MI = KT / 64;              // 16-row m tiles of k per wave (each wave owns KT / 4 k values)
  constexpr int XC = KT / 128;             // 8-element X chunks per thread and plane
  constexpr int GS = COUT + 8;
  constexpr int NT = COUT / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][2][32 * XS];
  __shared__ __attribute__((aligned(16))) bf16_t Gsh[2][2][32 * GS];
  const int kt = (K + KT - 1) / KT;
  const int zt = blockIdx.x / kt, tile_k = blockIdx.x - zt * kt;
  const int j = zt / nsplit, split = zt - j * nsplit;
  const int n_all = inv_cnt[layer * M + j];
  const int u_beg = (int)((long)n_all * split / nsplit), u_end = (int)((long)n_all * (split + 1) / nsplit);
  if (u_beg >= u_end) return;
  const int k0 = tile_k * KT;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int wk = w >> 1, wn = w & 1;
  const int Rtot = T * E, PE = P * E;
  const int nrb = (Rtot + 31) / 32;
  const int n_it = (u_end - u_beg) * nrb;
  const int* ip = inv_path + (layer * M + j) * Pmax;
  const int* is = inv_slot + (layer * M + j) * Pmax;
  constexpr int GSEG = COUT / 16;
  const int lr = tid >> 4, lxs = (tid & 15) * 8, lgs = (tid & 15) * GSEG;
  s8v xrh[XC], xrl[XC], grh[GSEG / 8], grl[GSEG / 8];
  auto gload = [&](int it) {
    const int ui = it / nrb;
    const int r = (it - ui * nrb) * 32 + lr;
    const int p = ip[u_beg + ui], a = is[u_beg + ui];
    const s8v z = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < XC; ++c) { xrh[c] = z; xrl[c] = z; }
#pragma unroll
    for (int h = 0; h < GSEG / 8; ++h) { grh[h] = z; grl[h] = z; }
    if (r < Rtot) {
      const long sg = sample_global(p, r, E, PE, 0);
#pragma unroll
      for (int c = 0; c < XC; ++c) {
        if (k0 + lxs + 128 * c < K) {
          xrh[c] = *reinterpret_cast<const s8v*>(X + sg * ldx + k0 + lxs + 128 * c);
          xrl[c] = *reinterpret_cast<const s8v*>(X + xlo + sg * ldx + k0 + lxs + 128 * c);
        }
      }
      const bf16_t* gp = Gm + ((long)a * bits_rows + sg) * COUT + lgs;
#pragma unroll
      for (int h = 0; h < GSEG / 8; ++h) {
        grh[h] = *reinterpret_cast<const s8v*>(gp + 8 * h);
        grl[h] = *reinterpret_cast<const s8v*>(gp + gmlo + 8 * h);
      }
    }
  };
  f4v acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) acc[i][jj] = {0.f, 0.f, 0.f, 0.f};
  float bsum[NT];
#pragma unroll
  for (int jj = 0; jj < NT; ++jj) bsum[jj] = 0.f;
  const bool do_bias = tile_k == 0 && wk == 0;
  gload(0);
  for (int it = 0; it < n_it; ++it) {
    const int buf = it & 1;
#pragma unroll
    for (int c = 0; c < XC; ++c) {                                  // the activation's fp16 pair as is (G16)
      *reinterpret_cast<s8v*>(Xs[buf][0] + lr * XS + lxs + 128 * c) = xrh[c];
      *reinterpret_cast<s8v*>(Xs[buf][1] + lr * XS + lxs + 128 * c) = xrl[c];
    }
#pragma unroll
    for (int h = 0; h < GSEG / 8; ++h) {
      *reinterpret_cast<s8v*>(Gsh[buf][0] + lr * GS + lgs + 8 * h) = grh[h];
      *reinterpret_cast<s8v*>(Gsh[buf][1] + lr * GS + lgs + 8 * h) = grl[h];
    }
    __syncthreads();
    if (it + 1 < n_it) gload(it + 1);
    s8v afh[MI], afl[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int o0 = (8 * grp + q) * XS + (KT / 4) * wk + 16 * i + 4 * pp;
      const int o1 = (8 * grp + 4 + q) * XS + (KT / 4) * wk + 16 * i + 4 * pp;
      afh[i] = tr8(Xs[buf][0] + o0, Xs[buf][0] + o1);
      afl[i] = tr8(Xs[buf][1] + o0, Xs[buf][1] + o1);
    }
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) {
      const int nb = (COUT / 2) * wn + 16 * jj;
      const int o0 = (8 * grp + q) * GS + nb + 4 * pp, o1 = (8 * grp + 4 + q) * GS + nb + 4 * pp;
      const s8v bh = tr8(Gsh[buf][0] + o0, Gsh[buf][0] + o1);
      const s8v bl = tr8(Gsh[buf][1] + o0, Gsh[buf][1] + o1);
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[i][jj] = mma3h(afh[i], afl[i], bh, bl, acc[i][jj]);
      if (do_bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[jj] += h2f((uint16_t)bh[e]) + h2f((uint16_t)bl[e]);
      }
    }
  }
  const long base = w_off + (long)j * chunk;
  const float ginv = 1.0f / g16_scale(gamax);          // Gm holds the gradient * 2^e
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + (KT / 4) * wk + 16 * i + 4 * grp + r;
        const int n = (COUT / 2) * wn + 16 * jj + i16;
        if (k < K) {
          if (nsplit == 1) grad[base + (long)k * COUT + n] = acc[i][jj][r] * ginv;
          else gacc(grad, fx, base + (long)k * COUT + n, acc[i][jj][r] * ginv);
        }
      }
  if (do_bias) {
#pragma unroll
    for (int jj = 0; jj < NT; ++jj) {
      float v = bsum[jj] * ginv;
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (grp == 0) {
        const long o = b_off + (long)j * chunk + (COUT / 2) * wn + 16 * jj + i16;
        if (nsplit == 1) grad[o] = v;
        else gacc(grad, fx, o, v);
      }
    }
  }
}

// ===========================================================================
// fc weight gradient, 64 x 64 tiles (trunk_bwd.hip fc_wgrad_kernel) for the narrow fc layers: X hi/lo planes,
// fp32 G masked by the ReLU bits and split into hi/lo while staging.  grid = (K/64, Cout/64, M * nsplit).
// ===========================================================================
__global__ __launch_bounds__(256) void fc_wgrad_x3(const bf16_t* __restrict__ X, long xlo, int ldx,
                                                   const float* __restrict__ G, const uint16_t* __restrict__ bits,
                                                   float* __restrict__ grad, long w_off, long b_off, int chunk,
                                                   const int* __restrict__ inv_path, const int* __restrict__ inv_slot,
                                                   const int* __restrict__ inv_cnt, int layer, int M, int Pmax, int K,
                                                   int Cout, int P, int E, int T, long bits_rows, float g_scale,
                                                   int nsplit, const float* __restrict__ gamax,
                                                   long long* __restrict__ fx) {
  constexpr int S = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][32 * S];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][32 * S];
  __shared__ unsigned long long dbq[64];        // det: int64 fixed point; else the float view
  float* const dbias = reinterpret_cast<float*>(dbq);
  const int j = blockIdx.z / nsplit, split = blockIdx.z - j * nsplit;
  const int n_all = inv_cnt[layer * M + j];
  const int u_beg = (int)((long)n_all * split / nsplit), u_end = (int)((long)n_all * (split + 1) / nsplit);
  if (u_beg >= u_end) return;
  const int k0b = blockIdx.x * 64, n0b = blockIdx.y * 64;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const bool do_bias = blockIdx.x == 0;
  if (tid < 64) dbq[tid] = 0ull;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const int nwords = Cout / 16;
  f4v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) { acc[a][0] = {0.f, 0.f, 0.f, 0.f}; acc[a][1] = {0.f, 0.f, 0.f, 0.f}; }
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int srow = tid >> 3, sc = (tid & 7) * 8;
  const int mt0 = 2 * (w >> 1), nt0 = 2 * (w & 1);
  const float gs = g16_scale(gamax), ginv = 1.0f / gs;
  for (int u = u_beg; u < u_end; ++u) {
    const int p = inv_path[(layer * M + j) * Pmax + u];
    const int a = inv_slot[(layer * M + j) * Pmax + u];
    for (long rb = 0; rb < Rtot; rb += 32) {
      const long r = rb + srow;
      s8v xh = {0, 0, 0, 0, 0, 0, 0, 0}, xl = xh;
      float m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < Rtot) {
        const long sg = sample_global(p, (int)r, E, PE, 0);
        if (k0b + sc < K) {
          xh = *reinterpret_cast<const s8v*>(X + sg * ldx + k0b + sc);
          xl = *reinterpret_cast<const s8v*>(X + xlo + sg * ldx + k0b + sc);
        }
        const int n = n0b + sc;
        if (n < Cout) {
          const float4 g0 = *reinterpret_cast<const float4*>(G + sg * Cout + n);
          const float4 g1 = *reinterpret_cast<const float4*>(G + sg * Cout + n + 4);
          const uint32_t bw = bits[((long)a * bits_rows + sg) * nwords + (n >> 4)] >> (n & 15);
          const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            m[c] = ((bw >> c) & 1u) ? gg[c] * g_scale : 0.f;
            bpart[c] += m[c];
          }
        }
      }
      s8v gh, gl;
      split8hs(m, gs, gh, gl);                         // G16: fp16 pair of the masked gradient * 2^e
      *reinterpret_cast<s8v*>(Xs[0] + srow * S + sc) = xh;     // the activation's fp16 pair as is
      *reinterpret_cast<s8v*>(Xs[1] + srow * S + sc) = xl;
      *reinterpret_cast<s8v*>(Gs[0] + srow * S + sc) = gh;
      *reinterpret_cast<s8v*>(Gs[1] + srow * S + sc) = gl;
      __syncthreads();
      s8v afh[2], afl[2], bfh[2], bfl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int xo0 = (8 * grp + q) * S + (mt0 + i) * 16 + 4 * pp, xo1 = (8 * grp + 4 + q) * S + (mt0 + i) * 16 + 4 * pp;
        afh[i] = tr8(Xs[0] + xo0, Xs[0] + xo1);
        afl[i] = tr8(Xs[1] + xo0, Xs[1] + xo1);
        const int go0 = (8 * grp + q) * S + (nt0 + i) * 16 + 4 * pp, go1 = (8 * grp + 4 + q) * S + (nt0 + i) * 16 + 4 * pp;
        bfh[i] = tr8(Gs[0] + go0, Gs[0] + go1);
        bfl[i] = tr8(Gs[1] + go0, Gs[1] + go1);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mma3h(afh[i], afl[i], bfh[jj], bfl[jj], acc[i][jj]);
      __syncthreads();
    }
  }
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
          if (nsplit == 1) grad[base + (long)k * Cout + n] = acc[i][jj][r] * ginv;
          else gacc(grad, fx, base + (long)k * Cout + n, acc[i][jj][r] * ginv);
        }
      }
  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 8; ++c) lds_acc(dbias, dbq, sc + c, bpart[c], fx != nullptr);
    __syncthreads();
    if (tid < 64 && n0b + tid < Cout) {
      const long bi = b_off + (long)j * chunk + n0b + tid;
      if (fx) {
        if (nsplit == 1) grad[bi] = fx_f(dbq[tid]);
        else gacc_q(fx, bi, dbq[tid]);
      } else if (nsplit == 1) {
        grad[bi] = dbias[tid];
      } else {
        atomicAdd(&grad[bi], dbias[tid]);
      }
    }
  }
}

// hi/lo operand copies of one layer's weights: Wc [2][M][Cout][KP] (forward B operand, k contiguous, zero padded):
// the fp16 pair of W * 2^X3_W0_SHIFT (f16 != 0) or the bf16 pair of W; optionally WcT [3][M][KP][Cout] (the fc input
// gradient's B operand): the fp16 hi, lo and third piece of W * 2^X3_W0_SHIFT, as the scaled fp16-pair gradients it
// meets (G16).  *status |= X3_RANGE_W when a scaled
// weight leaves the fp16 range; x3_status_fold (end of the next rollout) moves it and the forward epilogues' flag
// into the update's all-reduced counters, where every rank sees it (algo/trainer.py raises X3RangeError)
DEVI void refresh_x3_tile(const float* __restrict__ flat, long w_off, int chunk, int K, int KP, int Cout, int M,
                          uint16_t* __restrict__ Wc, uint16_t* __restrict__ WcT, int f16, uint32_t* __restrict__ status,
                          int b) {
  // one 32 (k) x 64 (column) tile of one module per workgroup, transposed through LDS: the master weights are read
  // and WcT ([M][KP][Cout], the flat order) written along the columns, Wc ([M][Cout][KP]) written along k -- both
  // coalesced (the flat-order loop wrote Wc with a KP stride: 5 launches x ~16 us per update)
  __shared__ float tile[32][65];
  const int tk = (KP + 31) / 32, tc = (Cout + 63) / 64;
  const int j = b / (tk * tc), rem = b - j * tk * tc;
  const int kt = rem / tc, ct = rem - kt * tc;
  if (j >= M) return;
  const long n = (long)M * KP * Cout;
  const int t = (int)threadIdx.x;
  bool bad = false;
  for (int kk = t >> 6; kk < 32; kk += 4) {
    const int k = kt * 32 + kk, c = ct * 64 + (t & 63);
    const float v = (k < K && c < Cout) ? flat[w_off + (long)j * chunk + (long)k * Cout + c] : 0.f;
    tile[kk][t & 63] = v;
    if (WcT && k < KP && c < Cout) {  // the fc input gradient's B operand: fp16 pieces of W * 2^8 (meets G16 gradients)
      const long i = ((long)j * KP + k) * Cout + c;
      const float x = v * (float)(1 << X3_W0_SHIFT);
      const uint16_t th = f2h(x);
      const float r = x - h2f(th);
      const uint16_t tl = f2h(r);
      WcT[i] = th;
      WcT[n + i] = tl;
      WcT[2 * n + i] = f2h(r - h2f(tl));           // third piece: W exact to 33 bits (X3_DG_W3)
    }
  }
  __syncthreads();
  for (int cc = t >> 5; cc < 64; cc += 8) {
    const int k = kt * 32 + (t & 31), c = ct * 64 + cc;
    if (k >= KP || c >= Cout) continue;
    const float v = tile[t & 31][cc];
    uint16_t hi, lo;
    if (f16) {
      const float x = v * (float)(1 << X3_W0_SHIFT);
      hi = f2h(x);
      lo = f2h(x - h2f(hi));
      bad |= !(fabsf(x) < 32768.f);
    } else {
      const bf16_t bh = f2bf(v);
      hi = bh;
      lo = f2bf(v - bf2f(bh));
    }
    const long wi = ((long)j * Cout + c) * KP + k;
    Wc[wi] = hi;
    Wc[n + wi] = lo;
  }
  if (bad && status) atomicOr(status, X3_RANGE_W);
}

__global__ __launch_bounds__(256) void refresh_x3_kernel(const float* __restrict__ flat, long w_off, int chunk, int K,
                                                         int KP, int Cout, int M, uint16_t* __restrict__ Wc,
                                                         uint16_t* __restrict__ WcT, int f16,
                                                         uint32_t* __restrict__ status) {
  refresh_x3_tile(flat, w_off, chunk, K, KP, Cout, M, Wc, WcT, f16, status, (int)blockIdx.x);
}

// every layer's refresh in ONE launch (x3_refresh_weights_all): layer i owns blocks [b0[i], b0[i + 1])
constexpr int X3_REFRESH_MAXL = 8;
struct RefreshSet {
  long w_off[X3_REFRESH_MAXL];
  uint16_t* Wc[X3_REFRESH_MAXL];
  uint16_t* WcT[X3_REFRESH_MAXL];
  int chunk[X3_REFRESH_MAXL], K[X3_REFRESH_MAXL], KP[X3_REFRESH_MAXL], Cout[X3_REFRESH_MAXL];
  int b0[X3_REFRESH_MAXL + 1];
  int n, M, f16;
};
__global__ __launch_bounds__(256) void refresh_x3_all_kernel(const float* __restrict__ flat, RefreshSet rs,
                                                             uint32_t* __restrict__ status) {
  const int b = (int)blockIdx.x;
  int i = 0;
  while (i + 1 < rs.n && b >= rs.b0[i + 1]) ++i;
  refresh_x3_tile(flat, rs.w_off[i], rs.chunk[i], rs.K[i], rs.KP[i], rs.Cout[i], rs.M, rs.Wc[i], rs.WcT[i], rs.f16,
                  status, b - rs.b0[i]);
}

// deterministic mode: grad[i] += fx[i] * 2^-FX_SHIFT and fx[i] = 0 over [n0, n1) (entries no kernel touched stay 0 and
// are neither read-modified nor written back); fx[-1] (the range guard word) becomes X3_RANGE_FX
__global__ __launch_bounds__(256) void fx_flush_kernel(long long* __restrict__ fx, float* __restrict__ grad, long n0,
                                                      long n1) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && fx[-1] != 0) {
    fx[-1] = 0;
    atomicOr(&g_x3_range, X3_RANGE_FX);
  }
  for (long i = n0 + (long)blockIdx.x * 256 + threadIdx.x; i < n1; i += (long)gridDim.x * 256) {
    const long long q = fx[i];
    if (q != 0) {
      fx[i] = 0;
      grad[i] += fx_f((unsigned long long)q);
    }
  }
}

// one thread: out[0] = (float)(activation flags since the last fold | weight flags of the last refresh), both reset
__global__ void x3_status_fold_kernel(uint32_t* __restrict__ wstatus, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const uint32_t f = atomicExch(&g_x3_range, 0u) | atomicExch(wstatus, 0u);
  out[0] = (float)f;
}

}  // namespace x3

// ---------------------------------------------------------------------------
// C ABI.  Every launcher returns 1 when it handled the call, 0 when the shape is not one of the specialised
// geometries (the caller must not run the fp32x mode for it), <0 on invalid arguments (-22) or launch errors.
// ---------------------------------------------------------------------------
using namespace x3;

template <class G>
struct Tag {
  using type = G;
};

template <class G>
static bool x3_is(int Hin, int Win, int Cin, int KH, int KW, int S, int u8) {
  return Hin == G::HIN && Win == G::WIN && Cin == G::CIN && KH == G::KH && KW == G::KW && S == G::S &&
         (u8 != 0) == G::U8;
}

static int X3_FWD_NT = 8;      // 32-row tiles per wave in the first-layer forward (4 for the bf16-input layers)
static int X3_FWD_LB = 2;      // first-layer forward: min waves/SIMD (2: 194 VGPRs, no spill; 3: 168 with spills)
static int X3_FWD_DB = 0;      // bf16-activation conv forward: 1 = double-buffered A registers (2 waves/SIMD),
                               // 0 = one register set at 3 waves/SIMD (measured: conv3 24.6 -> 16.9 us, conv2 31.1 -> 30.3)
// slab weight gradient: stages of loads in flight for <= 2 column tiles: 1, 2, or 3 = 2 for the bf16-input layers
// and 1 for the uint8 first layer (measured, steady-state window: conv1 2.63 (2) -> 2.32 ms (1), conv2 0.50 (2) vs
// 0.52 ms (1); profiles/r3/kwin_x3_v4*.md)
static int X3_WGRAD_PF = 3;
// first-layer (frame ring) slab weight gradient: column tiles per pass (conv_wgrad_slab_x3 NCXP): 3 (2 waves / SIMD)
// or 2 (3 waves / SIMD, a second pass for paths with > 4 active modules)
// measured (profiles/r4/kwin_c1ncx*.md): 2.28 ms (3 tiles, PF 1) -> 2.02 (2, PF 1) -> 1.94 (2, PF 2; the default: PF 2
// unless X3_WGRAD_PF == 1)
static int X3_C1_WG_NCX = 2;
// conv forward epilogue, bit 0: first layer, bit 1: the bf16-activation layers; set = swapped MFMA orientation
// (conv_epi_sw; first layer also with the 1024-offset pixels folded into the bias), clear = rows-as-A
static int X3_FWD_SW = 1;
static int X3_FC_D = 4;        // fc forward register ring depth (k-steps of hi/lo A and B fragments in flight)
// fc forward split-K waves per module (1 = fc_fwd_x3, 2 = fc_fwd_ks_x3).  Measured: fc1 66.4 (2) vs 65.1 us (1),
// fc2 19.7 vs 17.4 (profiles/r3/kwin_x3_v7*.md): more waves on the same weight traffic do not help -- the launch
// is bound by its L2/MALL traffic, not by load latency
static int X3_FC_KS = 1;
// module-major fc forward kernel (when the Python side selects module-major): 1 = fc_fwd_mm_x3 (register
// fragments), 2 = fc_fwd_mm2_x3 (LDS-staged 128 x 128 tiles), 3 = the same with k split in two workgroups
// (pre-activation planes; bias, ReLU, bits and the slot sum in fc_slot_sum2_x3)
static int X3_FC_MMV = 3;
static int X3_WG3_TILE = 1;
// conv2/3 forward: 1 = one position tile per weight read, 2 = two (PAIR), 3 = two for the 4x4/s2 layer only (234
// output positions; the 3x3 layer's 176 leave paired waves idle).  Measured (kwin_x3_v24*.md, v25*.md): 4x4/s2
// 25.3 us paired vs 26.0-26.2 single (32.5-32.7 in slow runs), 3x3 18.4-18.8 paired vs 15.9-16.2 single
static int X3_FWD_TILE = 3;
static int X3_C1_F16B = 1;     // band forward: 1 = the band converted to fp16 once at staging (conv1_fwd_band_x2 F16B;
                               // interleaved A/B: 64 paths 97.1 -> 95.8 us, 8 paths 20.9 -> 20.4)
static int X3_C1_SB1 = 0;      // band forward (ring): 1 = one band buffer, three workgroups per CU (conv1_fwd_band_x2 SB1)
static int X3_C1_PIPE = 0;     // band forward: 1 = next k-step's LDS fragments read during this k-step's MFMAs
static int X3_C1_EMAJ = 1;     // ring slab weight gradient, atomic mode: env-major unit order
static int X3_C1_BAL = 1;      // ring band forward: cost-balanced 1-D schedule (conv1_fwd_band_x2 BAL)
static int X3_C1_BAND = 1;     // first-layer forward: 1 = input band in LDS (conv1_fwd_band_x2), 0 = conv1_fwd_x2    // bf16-activation conv forward: 1 = per-sample LDS tile (conv_fwd_tile_x3), 0 = rows
// input gradients (conv_dgrad_x3, fc_dgrad_gemm_x3): 1 = the weights as THREE fp16 pieces (a fourth MFMA per k-step),
// exact for fp32 weights: the pair's 2^-23 weight rounding is the same for every row, so it enters a layer's input
// gradient coherently and the weight gradients below sum it without cancellation (scripts/x3_lstm_diag.py)
static int X3_DG_W3 = 0;
// fc input gradient: 1 = every k-step's MFMA products summed from zero and added to the running fp32 sum by a VALU add;
// 2 = the same with odd k-steps on negated operands, subtracted (cancels the f16 MFMA's -inf rounding bias)
static int X3_DG_FOLD = 2;
// grid sizes of the backward kernels.  Measured with interleaved A/Bs (scripts/diag/ab_kernel.py): a grid that is
// ONE whole round of resident workgroups (2 per CU: 512) beats the fixed per-path sizes and the ~2-round targets of
// round 5's first half at every population for the conv2 / conv3 input gradients and the conv2 weight gradient
// (8 paths: conv2 backward 214 -> 167 us, conv3 backward 153 -> 128 us; 64 paths -1.5 to -2 %).  The conv1 ring
// weight gradient (3 per CU) takes 1, 2 or 4 whole rounds by its work (x3_conv1_ring_wgrad, X3_WG_AUTO); with
// X3_WG_AUTO = 0 it takes ~X3_WG_TARGET workgroups.  0 = the fixed per-path sizes (24 / 32 chunks per path).
static int X3_WG_TARGET = 1536;
static int X3_WG_AUTO = 1;
static int X3_WG2_TARGET = 512;    // 4x4/s2 slab weight gradient (units per workgroup = units * P / target, >= 8)
static int X3_DG3_TARGET = 512;    // 3x3 input gradient (samples per workgroup >= 2)
static int X3_FC_RT1 = 2;          // path-major fc forward, 17..32 rows per path: 16-row workgroups (0 off, 1 on, 2 auto)
static int X3_C1F_TARGET = 512;    // ring band forward: workgroups (bands per workgroup >= X3_C1F_MINB)
static int X3_C1F_MINB = 2;
static int X3_C23_TARGET = 512;    // fused conv2 + conv3 forward: workgroups (samples per workgroup >= X3_C23_MINS)
static int X3_C23_MINS = 1;        // (2 before: 16 paths 17.5 -> 16.2 us, 8 paths 16.1 -> 15.9, 64 paths equal)
static int X3_WG3_TARGET = 256;    // 3x3 tile weight gradient, one round at 1 per CU (samples per workgroup >= 4;
                                   // 512 before: conv3 backward 8 paths 128 -> 117 us, 64 paths 682 -> 676)
static int X3_FCW_TARGET = 1024;   // narrow fc weight gradient (fc_wgrad_x3): workgroups, via the path split
                                   // (2048 before: fc2 backward 8 paths 114 -> 109 us, 64 paths 330 -> 323)
// slab weight gradient: k-slot -> position map of the transposed operand reads (conv_wgrad_slab_x3 pmap)
static int X3_SLAB_PMAP = 1;
// staged output gradients: 1 = one fp16-pair split per value, masked per slot (mask_pair8); 0 = mask, then split per slot
static int X3_PRESPLIT = 1;
static int X3_FH_D = 3;        // fused last fc + heads: k-steps of fragments in flight (fc_heads_fwd_x3 D)
static int X3_DG_BAL = 1;         // conv_dgrad_x3: cost-balanced 1-D schedule (BAL)
static int X3_DG_V0 = 0;         // 1 = conv_dgrad_x3v0 (A/B only)
static int X3_DG_GSPLIT = X3_DG_SPLIT;   // conv_dgrad_x3 grid split (1 = one chunk per workgroup, no balancing)
static int X3_DG_CAP = 1;          // conv_dgrad_x3: cap at 2 workgroups per CU (dynamic LDS)
static int X3_DG_TARGET = 512;     // 4x4/s2 input gradient (2048 -> 1536 -> 512: 8 paths 224 -> 214 -> 191 -> 167 us with
                                   // the conv2 weight gradient)
// module-major fc forward k split: 0 = auto by rows (P*T*E <= 768: 4 parts, else 3), else the fixed part count (2 / 3 / 4 /
// 8), capped so every part keeps >= 2 k-steps
static int X3_FC_KS_PARTS = 0;
static int X3_FCW_KT = 256;     // fc weight gradient from Gm: k tile 256 (Gm re-read 6x at K = 1408) or 128 (11x)
static int X3_FC_DG_GEMM = 1;  // fc input gradient: 1 = fc_gm_x3 + per-path GEMM (fc_dgrad_gemm_x3), 0 = fc_dgrad_x3    // 3x3/s1 weight gradient: 1 = per-sample LDS tile (conv_wgrad_tile_x3), 0 = im2col rows

// dynamic LDS that caps kernel KERN at CAP resident workgroups per CU.  The latency-bound backward kernels' grids are
// whole rounds of a given occupancy (X3_DG_TARGET: 512 = 2 per CU); a build whose VGPR count lets a third workgroup
// fit leaves a third of the CUs idle (conv_dgrad_x3 at 168 VGPRs: 580 -> 955 us in the 4x4 layer)
template <auto KERN, int CAP>
static size_t lds_cap_pad() {
  static const size_t pad = [] {
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(KERN)) != hipSuccess) return (size_t)0;
    const long need = 160L * 1024 / (CAP + 1) + 1;
    return need > (long)a.sharedSizeBytes ? (size_t)(need - (long)a.sharedSizeBytes) : (size_t)0;
  }();
  return pad;
}

// the fixed-point weight-gradient accumulator of the backward being launched (deterministic mode), else nullptr:
// set by x3_set_fx around one backward's launches (one host thread, as graph capture is), read by the launchers
long long* g_fx_accum = nullptr;

extern "C" {

// deterministic (bit-reproducible) fp32x backward: fx = an int64 buffer of numel + 1 entries passed as base + 1 (fx[-1]
// is the range guard word), indexed like the fp32 gradient; nullptr restores the fp32 atomics
int x3_set_fx(void* fx) {
  g_fx_accum = reinterpret_cast<long long*>(fx);
  return 0;
}

int x3_fx_flush(void* fx, float* grad, long n0, long n1, hipStream_t st) {
  if (!fx || !grad || n0 < 0 || n1 < n0) return -22;
  if (n1 == n0) return 0;
  long blocks = (n1 - n0 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  fx_flush_kernel<<<(unsigned)blocks, 256, 0, st>>>(reinterpret_cast<long long*>(fx), grad, n0, n1);
  return (int)hipGetLastError();
}

void fast_conv_set_x3_fwd_nt(int nt) { X3_FWD_NT = nt; }
void fast_conv_set_x3_c1_wg_ncx(int v) { X3_C1_WG_NCX = v == 2 ? 2 : 3; }
void fast_conv_set_x3_fwd_lb(int lb) { X3_FWD_LB = lb; }
void fast_conv_set_x3_fwd_db(int db) { X3_FWD_DB = db; }
void fast_conv_set_x3_fwd_sw(int sw) { X3_FWD_SW = sw; }
void fast_conv_set_x3_wg3_tile(int t) { X3_WG3_TILE = t; }
void fast_conv_set_x3_fc_mmv(int v) { X3_FC_MMV = v; }
void fast_conv_set_x3_fc_dg_gemm(int v) { X3_FC_DG_GEMM = v; }
void fast_conv_set_x3_fcw_kt(int v) { X3_FCW_KT = v == 128 ? 128 : 256; }
void fast_conv_set_x3_dg_w3(int v) { X3_DG_W3 = v; }
void fast_conv_set_x3_dg_fold(int v) { X3_DG_FOLD = v; }
void fast_conv_set_x3_dg_v0(int v) { X3_DG_V0 = v; }
void fast_conv_set_x3_dg_bal(int v) { X3_DG_BAL = v; }
void fast_conv_set_x3_dg_gsplit(int v) { X3_DG_GSPLIT = v == 1 ? 1 : X3_DG_SPLIT; }
void fast_conv_set_x3_dg_cap(int v) { X3_DG_CAP = v; }
void fast_conv_set_x3_fwd_tile(int v) { X3_FWD_TILE = v; }
void fast_conv_set_x3_c1_band(int v) { X3_C1_BAND = v; }
void fast_conv_set_x3_c1_bal(int v) { X3_C1_BAL = v; }
void fast_conv_set_x3_c1_emaj(int v) { X3_C1_EMAJ = v; }
void fast_conv_set_x3_c1_sb1(int v) { X3_C1_SB1 = v; }
void fast_conv_set_x3_c1_pipe(int v) { X3_C1_PIPE = v; }
void fast_conv_set_x3_c1_f16b(int v) { X3_C1_F16B = v; }
void fast_conv_set_x3_fc_d(int d) { X3_FC_D = d; }
void fast_conv_set_x3_fc_ks(int ks) { X3_FC_KS = ks; }
void fast_conv_set_x3_wgrad_pf(int pf) { X3_WGRAD_PF = pf; }
void fast_conv_set_x3_fh_d(int v) { X3_FH_D = v; }
void fast_conv_set_x3_presplit(int v) { X3_PRESPLIT = v ? 1 : 0; }
void fast_conv_set_x3_slab_pmap(int v) { X3_SLAB_PMAP = v ? 1 : 0; }
void fast_conv_set_x3_fc_rt1(int v) { X3_FC_RT1 = v; }
void fast_conv_set_x3_c1f_target(int v) { X3_C1F_TARGET = v < 1 ? 1 : v; }
void fast_conv_set_x3_c1f_minb(int v) { X3_C1F_MINB = v < 1 ? 1 : v; }
void fast_conv_set_x3_c23_target(int v) { X3_C23_TARGET = v < 1 ? 1 : v; }
void fast_conv_set_x3_c23_mins(int v) { X3_C23_MINS = v < 1 ? 1 : v; }
void fast_conv_set_x3_wg3_target(int v) { X3_WG3_TARGET = v < 1 ? 1 : v; }
void fast_conv_set_x3_fcw_target(int v) { X3_FCW_TARGET = v < 1 ? 1 : v; }
void fast_conv_set_x3_wg2_target(int v) { X3_WG2_TARGET = v < 0 ? 0 : v; }
void fast_conv_set_x3_dg3_target(int v) { X3_DG3_TARGET = v < 0 ? 0 : v; }
void fast_conv_set_x3_wg_auto(int v) { X3_WG_AUTO = v; }
void fast_conv_set_x3_wg_target(int v) { X3_WG_TARGET = v < 0 ? 0 : v; }
void fast_conv_set_x3_dg_target(int v) { X3_DG_TARGET = v < 0 ? 0 : v; }
void fast_conv_set_x3_fc_ks_parts(int v) { X3_FC_KS_PARTS = (v == 2 || v == 3 || v == 4 || v == 8) ? v : 0; }

int x3_conv_fwd(const void* X, long xlo, int u8in, void* Y, long ylo, void* bits, const void* Wc, long wlo,
                const float* flat, long bias_off, int chunk, const int* ai, const int* ac, int layer, int L, int M,
                int Hin, int Win, int Cin, int KH, int KW, int S, int P, int E, int T, int t0, long br, float is,
                float os, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 || P <= 0 ||
      E <= 0 || T <= 0 || br <= 0 || u8in < 0 || bias_off < 0 || layer < 0 || t0 < 0 || xlo < 0 || ylo <= 0 ||
      wlo <= 0) return -22;
  if (M > 2 * X3_NCT) return 0;
  if (x3_is<C1>(Hin, Win, Cin, KH, KW, S, u8in)) {
    if ((E * C1::HOWO) % 16) return -2;
    const long rows = (long)T * E * C1::HOWO;
    const float isc = is / (float)(1 << X3_W0_SHIFT);
    if (X3_C1_BAND) {
      const long nbands = (long)T * E * BD1<C1>::NB;
      long bpw = (nbands * P + 511) / 512;                 // ~2 workgroups per CU over the launch
      if (bpw < 2) bpw = 2;
      if (X3_C1_F16B)
        conv1_fwd_band_x2<C1, false, false, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
            (const uint8_t*)X, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac,
            layer, L, M, P, E, T, t0, br, (int)bpw, isc, os);
      else if (X3_C1_PIPE)
        conv1_fwd_band_x2<C1, false, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
            (const uint8_t*)X, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac,
            layer, L, M, P, E, T, t0, br, (int)bpw, isc, os);
      else
        conv1_fwd_band_x2<C1><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
            (const uint8_t*)X, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac,
            layer, L, M, P, E, T, t0, br, (int)bpw, isc, os);
      const int rc = (int)hipGetLastError();
      return rc ? -rc : 1;
    }
#define C1L(NT_, LB_)                                                                                           \
  if (X3_FWD_SW & 1) C1LS(NT_, LB_, true); else C1LS(NT_, LB_, false)
#define C1LS(NT_, LB_, SW_)                                                                                     \
  conv1_fwd_x2<C1, NT_, LB_, SW_><<<dim3((unsigned)((rows + NT_ * 128 - 1) / (NT_ * 128)), P), 256, 0, st>>>(             \
      (const uint8_t*)X, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, \
      layer, L, M, P, E, T, t0, br, isc, os)
    if (X3_FWD_LB >= 3) {
      if (X3_FWD_NT >= 8) C1L(8, 3); else C1L(4, 3);
    } else {
      if (X3_FWD_NT >= 9) C1L(9, 2); else if (X3_FWD_NT >= 8) C1L(8, 2); else C1L(4, 2);
    }
#undef C1L
#undef C1LS
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
#define CFX(Gx)                                                                                                   \
  if (x3_is<Gx>(Hin, Win, Cin, KH, KW, S, u8in)) {                                                                \
    if ((E * Gx::HOWO) % 16) return -2;                                                                           \
    const long rows = (long)T * E * Gx::HOWO;                                                                     \
    const dim3 grid((unsigned)((rows + 511) / 512), P);                                                           \
    const float isc = is / (float)(1 << X3_W0_SHIFT);                                                             \
    if (X3_FWD_TILE) {                                                                                            \
      const long nsamp = (long)T * E;                                                                             \
      long spw = (nsamp * P + 511) / 512;                                                                         \
      if (spw < 2) spw = 2;                                                                                       \
      if (X3_FWD_TILE == 2 || (X3_FWD_TILE == 3 && Gx::HOWO > 200))                                              \
        conv_fwd_tile_x3<Gx, true><<<dim3((unsigned)((nsamp + spw - 1) / spw), P), 256, 0, st>>>(                 \
            (const uint16_t*)X, xlo, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off,   \
            chunk, ai, ac, layer, L, M, P, E, T, t0, br, (int)spw, isc, os);                                      \
      else                                                                                                        \
        conv_fwd_tile_x3<Gx><<<dim3((unsigned)((nsamp + spw - 1) / spw), P), 256, 0, st>>>(                       \
            (const uint16_t*)X, xlo, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off,   \
            chunk, ai, ac, layer, L, M, P, E, T, t0, br, (int)spw, isc, os);                                      \
    } else if (X3_FWD_DB)                                                                                         \
      conv_fwd_x3<Gx, 4, 2, true, false><<<grid, 256, 0, st>>>(                                                   \
          (const uint16_t*)X, xlo, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off,     \
          chunk, ai, ac, layer, L, M, P, E, T, t0, br, isc, os);                                                  \
    else if (X3_FWD_SW & 2)                                                                                       \
      conv_fwd_x3<Gx, 4, 3, false, true><<<grid, 256, 0, st>>>(                                                   \
          (const uint16_t*)X, xlo, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off,     \
          chunk, ai, ac, layer, L, M, P, E, T, t0, br, isc, os);                                                  \
    else                                                                                                          \
      conv_fwd_x3<Gx, 4, 3, false, false><<<grid, 256, 0, st>>>(                                                  \
          (const uint16_t*)X, xlo, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off,     \
          chunk, ai, ac, layer, L, M, P, E, T, t0, br, isc, os);                                                  \
    const int rc = (int)hipGetLastError();                                                                        \
    return rc ? -rc : 1;                                                                                          \
  }
  if (xlo <= 0) return -22;
  CFX(C2) CFX(C3)
#undef CFX
  return 0;
}

// first layer on the frame ring (frames [P*E][nslots][160*120] u8, fc [T+1][P*E] u8; runtime/engine.py frame_ring)
int x3_conv1_ring_fwd(const void* frames, const void* fc, void* Y, long ylo, void* bits, const void* Wc, long wlo,
                      const float* flat, long bias_off, int chunk, const int* ai, const int* ac, int L, int M, int P,
                      int E, int T, int t0, int nslots, int rbase, long br, float is, float os, hipStream_t st) {
  // rbase: the modular ring's base slot (step t's channel k in slot (rbase + t + max(k, fc)) mod nslots)
  if (!frames || !fc || chunk <= 0 || L <= 0 || M <= 0 || P <= 0 || E <= 0 || T <= 0 || t0 < 0 || br <= 0 ||
      bias_off < 0 || ylo <= 0 || wlo <= 0 || nslots < t0 + T + 3 || rbase < 0 || rbase >= nslots) return -22;
  if (M > 2 * X3_NCT) return 0;
  if ((E * C1::HOWO) % 16) return -2;
  const float isc = is / (float)(1 << X3_W0_SHIFT);
  const long nbands = (long)T * E * BD1<C1>::NB;
  long bpw = (nbands * P + X3_C1F_TARGET - 1) / X3_C1F_TARGET;
  if (bpw < X3_C1F_MINB) bpw = X3_C1F_MINB;
  if (bpw > (X3_C1_FWD_FCS - 2) * BD1<C1>::NB) bpw = (X3_C1_FWD_FCS - 2) * BD1<C1>::NB;   // staged fc bytes
  if (X3_C1_BAL && X3_C1_F16B && !X3_C1_SB1)         // the same workgroup count, cost-balanced over the population
    conv1_fwd_band_x2<C1, true, false, true, false, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw) * P), 256, 0, st>>>(
        (const uint8_t*)frames, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai,
        ac, 0, L, M, P, E, T, t0, br, (int)bpw, isc, os, (const uint8_t*)fc, nslots, rbase);
  else if (X3_C1_SB1)
    conv1_fwd_band_x2<C1, true, false, false, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
        (const uint8_t*)frames, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai,
        ac, 0, L, M, P, E, T, t0, br, (int)bpw, isc, os, (const uint8_t*)fc, nslots, rbase);
  else if (X3_C1_F16B)
    conv1_fwd_band_x2<C1, true, false, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
        (const uint8_t*)frames, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai,
        ac, 0, L, M, P, E, T, t0, br, (int)bpw, isc, os, (const uint8_t*)fc, nslots, rbase);
  else if (X3_C1_PIPE)
    conv1_fwd_band_x2<C1, true, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
        (const uint8_t*)frames, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai,
        ac, 0, L, M, P, E, T, t0, br, (int)bpw, isc, os, (const uint8_t*)fc, nslots, rbase);
  else
    conv1_fwd_band_x2<C1, true><<<dim3((unsigned)((nbands + bpw - 1) / bpw), P), 256, 0, st>>>(
        (const uint8_t*)frames, (uint16_t*)Y, ylo, (uint8_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai,
        ac, 0, L, M, P, E, T, t0, br, (int)bpw, isc, os, (const uint8_t*)fc, nslots, rbase);
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

// the 4x4/s2 and 3x3/s1 layers' forwards in one launch (conv23_fwd_tile_x3): layer `layer` (C2 geometry) reads X and
// writes Y1 / bits1, layer + 1 (C3) reads Y1 and writes Y2 / bits2, over the same sample partition as the two
// conv_fwd_tile_x3 launches
int x3_conv23_fwd(const void* X, long xlo, void* Y1, long y1lo, void* bits1, long br1, const void* Wc1, long w1lo,
                  long bias1_off, int chunk1, void* Y2, long y2lo, void* bits2, long br2, const void* Wc2, long w2lo,
                  long bias2_off, int chunk2, const float* flat, const int* ai, const int* ac, int layer, int L, int M,
                  int P, int E, int T, int t0, float os1, float os2, hipStream_t st) {
  if (!X || !Y1 || !Y2 || !bits1 || !bits2 || !Wc1 || !Wc2 || !flat || !ai || !ac || xlo <= 0 || y1lo <= 0 ||
      y2lo <= 0 || w1lo <= 0 || w2lo <= 0 || br1 <= 0 || br2 <= 0 || chunk1 <= 0 || chunk2 <= 0 || bias1_off < 0 ||
      bias2_off < 0 || layer < 0 || layer + 1 >= L || M <= 0 || P <= 0 || E <= 0 || T <= 0 || t0 < 0) return -22;
  if (M > 2 * X3_NCT || !X3_FWD_TILE) return 0;
  if ((E * C2::HOWO) % 16 || (E * C3::HOWO) % 16) return -2;
  const long nsamp = (long)T * E;
  long spw = (nsamp * P + X3_C23_TARGET - 1) / X3_C23_TARGET;
  if (spw < X3_C23_MINS) spw = X3_C23_MINS;
  const float isc = 1.f / (float)(1 << X3_W0_SHIFT);
  const dim3 grid((unsigned)((nsamp + spw - 1) / spw), P);
  if (X3_FWD_TILE == 2 || X3_FWD_TILE == 3)
    conv23_fwd_tile_x3<C2, C3, true><<<grid, 256, 0, st>>>(
        (const uint16_t*)X, xlo, (uint16_t*)Y1, y1lo, (uint8_t*)bits1, br1, (const uint16_t*)Wc1, w1lo, bias1_off, chunk1,
        (uint16_t*)Y2, y2lo, (uint8_t*)bits2, br2, (const uint16_t*)Wc2, w2lo, bias2_off, chunk2, flat, ai, ac, layer, L,
        M, P, E, T, t0, (int)spw, isc, os1, os2);
  else
    conv23_fwd_tile_x3<C2, C3, false><<<grid, 256, 0, st>>>(
        (const uint16_t*)X, xlo, (uint16_t*)Y1, y1lo, (uint8_t*)bits1, br1, (const uint16_t*)Wc1, w1lo, bias1_off, chunk1,
        (uint16_t*)Y2, y2lo, (uint8_t*)bits2, br2, (const uint16_t*)Wc2, w2lo, bias2_off, chunk2, flat, ai, ac, layer, L,
        M, P, E, T, t0, (int)spw, isc, os1, os2);
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

int x3_conv1_ring_wgrad(const void* frames, const void* fc, const float* Gr, const void* bits, float* grad, long w_off,
                        long b_off, int chunk, const int* ai, const int* ac, int L, int M, int P, int E, int T,
                        int nslots, int rbase, long br, float is, float gs, const float* gamax, hipStream_t st) {
  if (!frames || !fc || chunk <= 0 || L <= 0 || M <= 0 || P <= 0 || E <= 0 || T <= 0 || br <= 0 || w_off < 0 ||
      b_off < 0 || nslots < T + 3 || rbase < 0 || rbase >= nslots || !gamax) return -22;
  if (M > 2 * X3_NCT) return 0;
  using SB = Slab<C1, 2>;
  const long units = (long)T * E * SB::NB;
  // whole rounds of resident workgroups (3 per CU at 2 column tiles per pass): a partial last round is a tail in
  // which most CUs idle.  Rounds: 1, 2 or 4 by the work in ~133-stage rounds (<= 1.5, <= 5, more; interleaved A/B,
  // scripts/diag/ab_kernel.py: 8 paths 293 (1536) -> 261 us (768); 16 paths 487 (1536) vs 517 (1024) / 636 (800);
  // 32 paths 888 (1536) vs 898 (3072); 64 paths 1766 (1536) -> 1722 (3072)).  X3_WG_AUTO = 0: X3_WG_TARGET as is.
  long wgs = X3_WG_TARGET;
  if (X3_WG_AUTO && wgs > 0) {
    static int ncu = 0;
    if (ncu == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    }
    const long cap = 3L * ncu;
    const long r10 = units * P * 10 / (cap * 133);       // work in tenths of a 133-stage round
    wgs = cap * (r10 <= 15 ? 1 : (r10 <= 50 ? 2 : 4));
  }
  long upw = wgs > 0 ? (units * P + wgs - 1) / wgs : (units + 23) / 24;
  if (upw < 8) upw = 8;
  if (upw / SB::NB + 2 > X3_RING_FCS) return -22;       // the workgroup's first-valid bytes fit the LDS table
  const dim3 grid((unsigned)((units + upw - 1) / upw), P);
  // env-major unit order in the atomic mode (the deterministic mode keeps the committed partition of its fixed-point
  // partial sums, so its runs repeat bit for bit)
  const int pm = X3_SLAB_PMAP | ((X3_C1_EMAJ && !g_fx_accum) ? 2 : 0);
  if (X3_C1_WG_NCX == 2 && X3_WGRAD_PF != 1)       // 2 tiles per pass: two stages in flight fit (162 VGPRs)
    conv_wgrad_slab_x3<C1, 2, 2, true, 2><<<grid, 256, 0, st>>>(frames, 0, Gr, (const uint8_t*)bits, grad, w_off,
                                                                b_off, chunk, ai, ac, 0, L, M, P, E, T, br, (int)upw,
                                                                is, gs, (const uint8_t*)fc, nslots, gamax, pm, g_fx_accum, rbase);
  else if (X3_C1_WG_NCX == 2)
    conv_wgrad_slab_x3<C1, 2, 1, true, 2><<<grid, 256, 0, st>>>(frames, 0, Gr, (const uint8_t*)bits, grad, w_off,
                                                                b_off, chunk, ai, ac, 0, L, M, P, E, T, br, (int)upw,
                                                                is, gs, (const uint8_t*)fc, nslots, gamax, pm, g_fx_accum, rbase);
  else if (X3_WGRAD_PF == 2)
    conv_wgrad_slab_x3<C1, 2, 2, true><<<grid, 256, 0, st>>>(frames, 0, Gr, (const uint8_t*)bits, grad, w_off, b_off,
                                                             chunk, ai, ac, 0, L, M, P, E, T, br, (int)upw, is, gs,
                                                             (const uint8_t*)fc, nslots, gamax, pm, g_fx_accum, rbase);
  else
    conv_wgrad_slab_x3<C1, 2, 1, true><<<grid, 256, 0, st>>>(frames, 0, Gr, (const uint8_t*)bits, grad, w_off, b_off,
                                                             chunk, ai, ac, 0, L, M, P, E, T, br, (int)upw, is, gs,
                                                             (const uint8_t*)fc, nslots, gamax, pm, g_fx_accum, rbase);
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

int x3_conv_wgrad(const void* X, long xlo, int u8in, const float* Gr, const void* bits, float* grad, long w_off,
                  long b_off, int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win,
                  int Cin, int KH, int KW, int S, int P, int E, int T, long br, float is, float gs,
                  const float* gamax, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 || P <= 0 ||
      E <= 0 || T <= 0 || br <= 0 || u8in < 0 || w_off < 0 || b_off < 0 || layer < 0 || xlo < 0 || !gamax) return -22;
  if (M > 2 * X3_NCT) return 0;
  auto slab = [&](auto gc, auto obc) {
    using Gx = typename decltype(gc)::type;
    constexpr int OB = decltype(obc)::value;
    using SB = Slab<Gx, OB>;
    const long units = (long)T * E * SB::NB;
    // the P-scaled grid pays for the uint8 first layer (P = 8: 567 -> 305 us) but not for the 4x4/s2 layer
    // (105 -> 126 us: its per-workgroup setup is a larger share of a shorter unit walk)
    const long tgt = Gx::U8 ? X3_WG_TARGET : X3_WG2_TARGET;
    long upw = tgt > 0 ? (units * P + tgt - 1) / tgt : (units + 23) / 24;
    if (upw < 8) upw = 8;
    const dim3 grid((unsigned)((units + upw - 1) / upw), P);
    const int pf = Gx::U8 ? (X3_WGRAD_PF == 2 ? 2 : 1) : (X3_WGRAD_PF >= 2 ? 2 : 1);
    if (pf == 2)
      conv_wgrad_slab_x3<Gx, OB, 2><<<grid, 256, 0, st>>>(X, xlo, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk,
                                                          ai, ac, layer, L, M, P, E, T, br, (int)upw, is, gs, nullptr,
                                                          0, gamax, X3_SLAB_PMAP, g_fx_accum, 0);
    else
      conv_wgrad_slab_x3<Gx, OB, 1><<<grid, 256, 0, st>>>(X, xlo, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk,
                                                          ai, ac, layer, L, M, P, E, T, br, (int)upw, is, gs, nullptr,
                                                          0, gamax, X3_SLAB_PMAP, g_fx_accum, 0);
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  };
  if (x3_is<C1>(Hin, Win, Cin, KH, KW, S, u8in)) return slab(Tag<C1>{}, std::integral_constant<int, 2>{});
  if (x3_is<C2>(Hin, Win, Cin, KH, KW, S, u8in)) {
    if (xlo <= 0) return -22;
    return slab(Tag<C2>{}, std::integral_constant<int, 7>{});
  }
  if (x3_is<C3>(Hin, Win, Cin, KH, KW, S, u8in) && X3_WG3_TILE) {
    if (xlo <= 0) return -22;
    const long nsamp = (long)T * E;
    long spw = (nsamp * P + X3_WG3_TARGET - 1) / X3_WG3_TARGET;   // ~X3_WG3_TARGET workgroups over the launch
    if (spw < 4) spw = 4;
    conv_wgrad_tile_x3<C3><<<dim3((unsigned)((nsamp + spw - 1) / spw), P, 2), WT3<C3>::NT, 0, st>>>(
        (const uint16_t*)X, xlo, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br,
        (int)spw, is, gs, gamax, g_fx_accum);
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
  if (x3_is<C3>(Hin, Win, Cin, KH, KW, S, u8in)) {
    if (xlo <= 0) return -22;
    const long rows = (long)T * E * C3::HOWO;
    long rpc = (rows + 15) / 16;
    rpc = (rpc + X3_WG_RB - 1) / X3_WG_RB * X3_WG_RB;
    if (rpc < X3_WG_RB * 4) rpc = X3_WG_RB * 4;
    conv_wgrad_x3<C3><<<dim3((unsigned)((rows + rpc - 1) / rpc), P), 512, 0, st>>>(
        (const bf16_t*)X, xlo, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br,
        (int)rpc, is, gs, gamax, g_fx_accum);
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
  return 0;
}

int x3_conv_dgrad(const float* Gr, const void* bits, const float* flat, long w_off, int chunk, const int* ai,
                  const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH, int KW, int S, int P,
                  int E, int T, long br, float gs, float* dX, const float* gamax, float* gamax_out, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 || P <= 0 ||
      E <= 0 || T <= 0 || br <= 0 || w_off < 0 || layer < 0 || !gamax) return -22;
  if (M > 2 * X3_NCT) return 0;
  const int nsamp = T * E;
  // P-scaled grid for the 4x4/s2 layer's input gradient (P = 8: 127 -> 119 us); the 3x3 layer keeps 32 chunks per
  // path (100 -> 110 us when scaled)
  const long dgt = x3_is<C2>(Hin, Win, Cin, KH, KW, S, 0) ? X3_DG_TARGET : X3_DG3_TARGET;
  int spw = dgt > 0 ? (int)(((long)nsamp * P + dgt - 1) / dgt) : (nsamp + 31) / 32;
  if (spw < 2) spw = 2;
  const dim3 grid((unsigned)((nsamp + spw - 1) / spw), P, X3_DG_GSPLIT);
#define DGX(Gx)                                                                                                    \
  if (x3_is<Gx>(Hin, Win, Cin, KH, KW, S, 0)) {                                                                    \
    if (X3_DG_V0) {                                                                                                \
      if (X3_DG_FOLD == 2)                                                                                         \
        conv_dgrad_x3v0<Gx, false, true><<<dim3(grid.x, P), 256, 0, st>>>(                          \
            Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, spw, gamax,      \
            gamax_out, X3_PRESPLIT);                                                                               \
      else                                                                                                         \
        conv_dgrad_x3v0<Gx><<<dim3(grid.x, P), 256, 0, st>>>(                                       \
            Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, spw, gamax,      \
            gamax_out, X3_PRESPLIT);                                                                               \
    } else if (X3_DG_FOLD == 2 && X3_DG_BAL) {     /* the same workgroup count, cost-balanced, 1-D */          \
      const size_t pad = X3_DG_CAP ? lds_cap_pad<conv_dgrad_x3<Gx, false, true, true>, 2>() : 0;                  \
      conv_dgrad_x3<Gx, false, true, true><<<dim3(grid.x * P), 256, pad, st>>>(                                    \
          Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, spw, gamax,        \
          gamax_out, X3_PRESPLIT);                                                                                 \
    } else if (X3_DG_FOLD == 2) {                                                                                  \
      const size_t pad = X3_DG_CAP ? lds_cap_pad<conv_dgrad_x3<Gx, false, true>, 2>() : 0;                        \
      conv_dgrad_x3<Gx, false, true><<<grid, 256, pad, st>>>(Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac,  \
                                                             layer, L, M, P, E, T, br, gs, dX, spw, gamax,          \
                                                             gamax_out, X3_PRESPLIT);                               \
    } else if (X3_DG_W3) {                                                                                         \
      const size_t pad = X3_DG_CAP ? lds_cap_pad<conv_dgrad_x3<Gx, true, false>, 2>() : 0;                        \
      conv_dgrad_x3<Gx, true><<<grid, 256, pad, st>>>(Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, \
                                                      L, M, P, E, T, br, gs, dX, spw, gamax, gamax_out,              \
                                                      X3_PRESPLIT);                                                 \
    } else {                                                                                                       \
      const size_t pad = X3_DG_CAP ? lds_cap_pad<conv_dgrad_x3<Gx, false, false>, 2>() : 0;                       \
      conv_dgrad_x3<Gx><<<grid, 256, pad, st>>>(Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M,  \
                                                P, E, T, br, gs, dX, spw, gamax, gamax_out, X3_PRESPLIT);            \
    }                                                                                                              \
    const int rc = (int)hipGetLastError();                                                                         \
    return rc ? -rc : 1;                                                                                           \
  }
  DGX(C2) DGX(C3)
#undef DGX
  return 0;
}

// ylo = 0: fp32 output (last layer); > 0: bf16 hi/lo planes
int x3_fc_fwd(const void* X, long xlo, int ldx, void* Y, long ylo, void* bits, const void* Wc, long wlo,
              const float* flat, long bias_off, int chunk, const int* ai, const int* ac, int layer, int L, int M, int K,
              int KP, int Cout, int P, int E, int T, int t0, long br, float os, hipStream_t st) {
  if (ldx <= 0 || chunk <= 0 || L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      br <= 0 || bias_off < 0 || layer < 0 || t0 < 0 || xlo <= 0 || ylo < 0 || wlo <= 0) return -22;
  if (M > X3_MAXM || KP % 32 != 0 || Cout % 64 != 0 || ldx % 8 != 0 || ldx < K || (long)T * E > 32) return 0;
  const dim3 grid(1, Cout / 64, P);
  if ((X3_FC_RT1 == 1 || (X3_FC_RT1 == 2 && (long)P * (Cout / 64) <= 64)) && (long)T * E > 16 && KP == 256) {
    // 16-row workgroups: twice the grid for small populations (8 paths: fc2 16.1 -> 12.8 us; at 64 paths 16.9 ->
    // 22.5, so auto only while the 32-row grid has <= 64 workgroups)
    const dim3 g1((unsigned)((T * E + 15) / 16), Cout / 64, P);
    if (ylo == 0)
      fc_fwd_x3<1, 4, 8, true><<<g1, 256, 0, st>>>((const uint16_t*)X, xlo, ldx, Y, ylo, (uint16_t*)bits,
                                                  (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, layer, L, M, K,
                                                  KP, Cout, P, E, T, t0, br, 1.f / (float)(1 << X3_W0_SHIFT), os);
    else
      fc_fwd_x3<1, 4, 8, false><<<g1, 256, 0, st>>>((const uint16_t*)X, xlo, ldx, Y, ylo, (uint16_t*)bits,
                                                   (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, layer, L, M,
                                                   K, KP, Cout, P, E, T, t0, br, 1.f / (float)(1 << X3_W0_SHIFT), os);
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
#define FCX(RT_, D_, NKS_, OF_)                                                                                      \
  fc_fwd_x3<RT_, D_, NKS_, OF_><<<grid, 256, 0, st>>>((const uint16_t*)X, xlo, ldx, Y, ylo, (uint16_t*)bits,        \
                                                      (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, layer, \
                                                      L, M, K, KP, Cout, P, E, T, t0, br,                               \
                                                      1.f / (float)(1 << X3_W0_SHIFT), os)
  const bool of = ylo == 0;
  if (X3_FC_KS >= 2 && (long)T * E > 16) {
#define FKS(D_, NKS_, OF_, KS_)                                                                                      \
  fc_fwd_ks_x3<2, D_, NKS_, OF_, KS_><<<grid, 256 * KS_, 0, st>>>(                                                  \
      (const uint16_t*)X, xlo, ldx, Y, ylo, (uint16_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, \
      layer, L, M, K, KP, Cout, P, E, T, t0, br, 1.f / (float)(1 << X3_W0_SHIFT), os)
    if (of) FKS(2, 0, true, 2); else FKS(2, 0, false, 2);     // (KS = 4 needs <= 128 VGPRs: spills)
#undef FKS
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
  if ((long)T * E <= 16) {
    if (of) FCX(1, 4, 0, true); else FCX(1, 4, 0, false);
  } else if (KP == 1408 && X3_FC_D <= 2) {
    if (of) FCX(2, 2, 44, true); else FCX(2, 2, 44, false);
  } else if (KP == 1408) {
    if (of) FCX(2, 4, 44, true); else FCX(2, 4, 44, false);
  } else if (KP == 256) {
    if (of) FCX(2, 4, 8, true); else FCX(2, 4, 8, false);
  } else {
    if (of) FCX(2, 4, 0, true); else FCX(2, 4, 0, false);
  }
#undef FCX
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

// the last fc layer + heads of one rollout step (fc_heads_fwd_x3); 0 = shape not covered (the caller runs the two
// launches).  logits / value / actions: step t's [B] rows.
int x3_fc_heads_fwd(const void* X, long xlo, int ldx, float* Y, void* bits, const void* Wc, long wlo,
                    const float* flat, long bias_off, int chunk, const int* ai, const int* ac, int layer, int L, int M,
                    int K, int KP, int Cout, int P, int E, int t0, long br, float os, long pw, long pb, long vw,
                    long vb, int A, float* logits, float* value, int* actions, unsigned seed, const long long* ctr,
                    int t, int Tsteps, int greedy, unsigned rb, hipStream_t st) {
  if (!X || !Y || !bits || !Wc || !flat || !ai || !ac || !logits || !value || !actions || !ctr || ldx <= 0 ||
      chunk <= 0 || L <= 0 || M <= 0 || P <= 0 || E <= 0 || t0 < 0 || br <= 0 || bias_off < 0 || xlo <= 0 ||
      wlo <= 0 || A <= 0) return -22;
  if (M > X3_MAXM || Cout != 256 || K != 256 || KP != 256 || ldx % 8 != 0 || ldx < KP || E > 32 || A > 8) return 0;
#define FHX(D_)                                                                                                    \
  fc_heads_fwd_x3<8, D_><<<dim3((unsigned)((E + 15) / 16), (unsigned)P), 256, 0, st>>>(                             \
      (const uint16_t*)X, xlo, ldx, Y, (uint16_t*)bits, (const uint16_t*)Wc, wlo, flat, bias_off, chunk, ai, ac, layer, \
      L, M, P, E, t0, br, 1.f / (float)(1 << X3_W0_SHIFT), os, pw, pb, vw, vb, A, logits, value, actions, seed, ctr, t,  \
      Tsteps, greedy, rb)
  if (X3_FH_D >= 3) FHX(3); else FHX(2);
#undef FHX
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

// module-major fc forward (fc_fwd_mm_x3 + fc_slot_sum_x3); Ys: fp32 [M][P*T*E][256] slot planes
int x3_fc_fwd_mm(const void* X, long xlo, int ldx, void* Y, long ylo, void* bits, const void* Wc, long wlo,
                 const float* flat, long bias_off, int chunk, const int* ac, const int* ai, const int* inv_path,
                 const int* inv_slot,
                 const int* inv_cnt, float* Ys, int layer, int L, int M, int K, int KP, int Cout, int P, int E, int T,
                 int t0, long br, float os, hipStream_t st) {
  if (ldx <= 0 || chunk <= 0 || L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      br <= 0 || bias_off < 0 || layer < 0 || t0 < 0 || xlo <= 0 || ylo < 0 || wlo <= 0 || !Ys || !inv_path ||
      !inv_slot || !inv_cnt || !ai || !ac) return -22;
  if (M > X3_MAXM || KP % 32 != 0 || Cout != 256 || ldx % 8 != 0 || ldx < KP || (long)T * E > 32) return 0;
  const int R = T * E, tpp = (R + 15) / 16;
  const float isc = 1.f / (float)(1 << X3_W0_SHIFT);
  if (X3_FC_MMV >= 3) {
    // k split in KS (2, or 4 for X3_FC_MMV >= 4): partial planes Ys[KS][M][P*R][256], then bias + ReLU + bits +
    // slot sum in fc_slot_sum2_x3
    int ks = X3_FC_MMV >= 4 ? 4 : 2;
    if (X3_FC_KS_PARTS > 0) ks = X3_FC_KS_PARTS;
    // 4 parts up to 768 rows, else 3 (layer A/B, profiles/r5/ab_ks*.json: 8 paths 22.0 (8 parts) -> 21.6, 16 paths
    // 27.9 (2) -> 23.9, 24 paths 28.7 (2) / 26.1 (3) / 24.8 (4); 32 paths 29.3 (2) / 28.7 (3) / 33.9 (4); 64 paths
    // 48.1 (2) / 46.1 (3) / 51.5 (4) us: at two workgroups per CU, 3 parts keep the ~280 units of 64 paths in one
    // round of 512 slots where 4 parts spill into a second)
    else if (X3_FC_MMV == 3) ks = (long)P * R <= 768 ? 4 : 3;
    while (ks > 2 && (KP / 32) / ks < 2) ks >>= 1;           // every part keeps >= 2 k-steps
    const int umax = (ks * M * 2 * ((P * R + 127) / 128) + 7) / 8 * 8;
    const unsigned g2 = (unsigned)(((long)P * R * 32 + 255) / 256);
#define MM2KS(KS_)                                                                                                \
    {                                                                                                             \
      if (KP == 256)                                                                                              \
        fc_fwd_mm2_x3<8, 3, KS_><<<umax, 512, 0, st>>>((const uint16_t*)X, xlo, ldx, Ys, (uint16_t*)bits,          \
                                                       (const uint16_t*)Wc, wlo, flat, bias_off, chunk, inv_path,  \
                                                       inv_slot, inv_cnt, layer, M, KP, P, E, T, t0, br, isc);     \
      else                                                                                                        \
        fc_fwd_mm2_x3<0, 3, KS_><<<umax, 512, 0, st>>>((const uint16_t*)X, xlo, ldx, Ys, (uint16_t*)bits,          \
                                                       (const uint16_t*)Wc, wlo, flat, bias_off, chunk, inv_path,  \
                                                       inv_slot, inv_cnt, layer, M, KP, P, E, T, t0, br, isc);     \
      int rc_ = (int)hipGetLastError();                                                                           \
      if (rc_) return -rc_;                                                                                       \
      if (ylo == 0)                                                                                               \
        fc_slot_sum2_x3<true, KS_><<<g2, 256, 0, st>>>(Ys, ai, ac, flat, bias_off, chunk, (uint16_t*)bits, br,     \
                                                       layer, L, M, P, E, T, t0, Y, 0, os);                        \
      else                                                                                                        \
        fc_slot_sum2_x3<false, KS_><<<g2, 256, 0, st>>>(Ys, ai, ac, flat, bias_off, chunk, (uint16_t*)bits, br,    \
                                                        layer, L, M, P, E, T, t0, Y, ylo, os);                     \
    }
    if (ks == 8) MM2KS(8) else if (ks == 4) MM2KS(4) else if (ks == 3) MM2KS(3) else MM2KS(2)
#undef MM2KS
    const int rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  } else if (X3_FC_MMV >= 2) {
    const int umax = (M * 2 * ((P * R + 127) / 128) + 7) / 8 * 8;    // every module on every path: an upper bound
    if (KP == 256)
      fc_fwd_mm2_x3<8, 3, 1><<<umax, 512, 0, st>>>((const uint16_t*)X, xlo, ldx, Ys, (uint16_t*)bits,
                                                   (const uint16_t*)Wc, wlo, flat, bias_off, chunk, inv_path, inv_slot,
                                                   inv_cnt, layer, M, KP, P, E, T, t0, br, isc);
    else
      fc_fwd_mm2_x3<0, 3, 1><<<umax, 512, 0, st>>>((const uint16_t*)X, xlo, ldx, Ys, (uint16_t*)bits,
                                                   (const uint16_t*)Wc, wlo, flat, bias_off, chunk, inv_path, inv_slot,
                                                   inv_cnt, layer, M, KP, P, E, T, t0, br, isc);
  } else {
    const int umax = M * ((P * tpp + 3) / 4) * 2;    // x 2 column slices (fc_fwd_mm_x3 NH)
    const int nwg = (umax + 7) / 8 * 8;
#define FMM(NKS_)                                                                                                 \
  fc_fwd_mm_x3<NKS_><<<nwg, 512, 0, st>>>((const uint16_t*)X, xlo, ldx, Ys, (uint16_t*)bits, (const uint16_t*)Wc, \
                                          wlo, flat, bias_off, chunk, inv_path, inv_slot, inv_cnt, layer, M, KP, P, E, \
                                          T, t0, br, isc)
    if (KP == 256) FMM(8); else FMM(0);      // (a constant 44-step loop spills: runtime count for fc1)
#undef FMM
  }
  int rc = (int)hipGetLastError();
  if (rc) return -rc;
  const long thr = (long)P * R * 32;
  const unsigned g2 = (unsigned)((thr + 255) / 256);
  if (ylo == 0)
    fc_slot_sum_x3<true><<<g2, 256, 0, st>>>(Ys, ac, layer, L, P, E, T, t0, Y, 0, os);
  else
    fc_slot_sum_x3<false><<<g2, 256, 0, st>>>(Ys, ac, layer, L, P, E, T, t0, Y, ylo, os);
  rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

int x3_fc_dgrad(const float* G, const void* bits, const void* WcT, long wlo, const int* ai, const int* ac, int layer,
                int L, int M, int K, int KP, int Cout, int P, int E, int T, long br, float gs, float* dX, void* Gm,
                long gmlo, const float* gamax, float* gamax_out, hipStream_t st) {
  if (L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 || br <= 0 || layer < 0 ||
      wlo <= 0 || gmlo < 0 || (Gm && gmlo <= 0) || !gamax) return -22;
  if (M > X3_MAXM || Cout != 256) return 0;
  if (X3_FC_DG_GEMM && Gm != nullptr) {
    const int R = T * E;
    const long thr = (long)P * R * (256 / 8);
    fc_gm_x3<256><<<(unsigned)((thr + 255) / 256), 256, 0, st>>>(G, (const uint16_t*)bits, ac, layer, L, P, E, T, br,
                                                                  gs, (bf16_t*)Gm, gmlo, gamax);
    int rc = (int)hipGetLastError();
    if (rc) return -rc;
    const int nrb = (R + 127) / 128, ncb = (K + 255) / 256;
    const unsigned nwg = (unsigned)((P * nrb * ncb + 7) / 8 * 8);
#define DGG(W3_, FOLD_)                                                                                           \
    fc_dgrad_gemm_x3<256, W3_, FOLD_><<<nwg, 512, 0, st>>>((const bf16_t*)Gm, gmlo, (const bf16_t*)WcT, wlo, ai, ac, \
                                                           layer, L, M, K, KP, P, E, T, br, dX, nrb, ncb, gamax,     \
                                                           gamax_out)
    if (X3_DG_FOLD == 2) DGG(false, 2);
    else if (X3_DG_W3 && X3_DG_FOLD) DGG(true, 1);
    else if (X3_DG_W3) DGG(true, 0);
    else if (X3_DG_FOLD) DGG(false, 1);
    else DGG(false, 0);
#undef DGG
    rc = (int)hipGetLastError();
    return rc ? -rc : 1;
  }
  const int nchunks = (K + 127) / 128;
  const int split = nchunks >= 8 ? 2 : 1;
  const int per = (nchunks + split - 1) / split;
  const int nrowb = (int)(((long)T * E + 63) / 64);
  const int nwg = (nrowb * P * split + 7) / 8 * 8;
  fc_dgrad_x3<256><<<nwg, 512, 0, st>>>(G, (const uint16_t*)bits, (const bf16_t*)WcT, wlo, ai, ac, layer, L, M, K, KP,
                                        P, E, T, br, gs, dX, per, nrowb, split, (bf16_t*)Gm, gmlo, gamax, gamax_out);
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

int x3_fc_wgrad_gm(const void* X, long xlo, int ldx, const void* Gm, long gmlo, float* grad, long w_off, long b_off,
                   int chunk, const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int M, int Pmax,
                   int K, int Cout, int P, int E, int T, long br, int nsplit, const float* gamax, hipStream_t st) {
  if (ldx <= 0 || chunk <= 0 || M <= 0 || Pmax <= 0 || K <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 || br <= 0 ||
      nsplit <= 0 || w_off < 0 || b_off < 0 || layer < 0 || xlo <= 0 || gmlo <= 0 || !gamax) return -22;
  if (Cout != 256 || ldx % 8 != 0 || K % 8 != 0) return 0;
  if (X3_FCW_KT == 256 && K > 256) {
    // 256-wide k tiles: the masked gradient Gm (1 KB per row) is re-read once per k tile -- 6 instead of 11 times at
    // K = 1408
    const int kt = (K + 255) / 256;
    fc_wgrad_gm_x3<256, 256><<<kt * M * nsplit, 512, 0, st>>>((const bf16_t*)X, xlo, ldx, (const bf16_t*)Gm, gmlo,
                                                              grad, w_off, b_off, chunk, inv_path, inv_slot, inv_cnt,
                                                              layer, M, Pmax, K, P, E, T, br, nsplit, gamax,
                                                              g_fx_accum);
  } else {
    const int kt = (K + 127) / 128;
    fc_wgrad_gm_x3<256><<<kt * M * nsplit, 512, 0, st>>>((const bf16_t*)X, xlo, ldx, (const bf16_t*)Gm, gmlo, grad,
                                                         w_off, b_off, chunk, inv_path, inv_slot, inv_cnt, layer, M,
                                                         Pmax, K, P, E, T, br, nsplit, gamax, g_fx_accum);
  }
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

int x3_fc_wgrad(const void* X, long xlo, int ldx, const float* G, const void* bits, float* grad, long w_off,
                long b_off, int chunk, const int* inv_path, const int* inv_slot, const int* inv_cnt, int layer, int M,
                int Pmax, int K, int Cout, int P, int E, int T, long br, float gs, const float* gamax, hipStream_t st) {
  if (ldx <= 0 || chunk <= 0 || M <= 0 || Pmax <= 0 || K <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 || br <= 0 ||
      w_off < 0 || b_off < 0 || layer < 0 || xlo <= 0 || !gamax) return -22;
  if (Cout % 16 != 0 || ldx % 8 != 0) return 0;
  const int tiles = ((K + 63) / 64) * ((Cout + 63) / 64) * M;
  int nsplit = (X3_FCW_TARGET + tiles - 1) / tiles;
  nsplit = nsplit < 1 ? 1 : (nsplit > Pmax ? Pmax : nsplit);
  fc_wgrad_x3<<<dim3((K + 63) / 64, (Cout + 63) / 64, M * nsplit), 256, 0, st>>>(
      (const bf16_t*)X, xlo, ldx, G, (const uint16_t*)bits, grad, w_off, b_off, chunk, inv_path, inv_slot, inv_cnt,
      layer, M, Pmax, K, Cout, P, E, T, br, gs, nsplit, gamax, g_fx_accum);
  const int rc = (int)hipGetLastError();
  return rc ? -rc : 1;
}

// G16 amax of an fp32 gradient tensor: *amax = max(*amax, max |g|) (grid-stride; the caller zeroes it when a new
// backward starts: x3_amax_reset)
__global__ __launch_bounds__(256) void x3_amax_kernel(const float* __restrict__ g, long n, float* __restrict__ amax) {
  float m = 0.f;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (long)gridDim.x * 256 * 4) {
    if (i + 3 < n) {
      const float4 v = *reinterpret_cast<const float4*>(g + i);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    } else {
      for (long j = i; j < n; ++j) m = fmaxf(m, fabsf(g[j]));
    }
  }
  g16_flush_amax_wg(m, amax);
}
__global__ void x3_amax_reset_kernel(float* __restrict__ amax, int n) {
  if ((int)threadIdx.x < n) amax[threadIdx.x] = 0.f;
}
int x3_amax(const float* g, long n, float* amax, hipStream_t st) {
  if (!g || !amax || n <= 0) return -22;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  x3_amax_kernel<<<(unsigned)blocks, 256, 0, st>>>(g, n, amax);
  return (int)hipGetLastError();
}
int x3_amax_reset(float* amax, int n, hipStream_t st) {
  if (!amax || n <= 0 || n > 64) return -22;
  x3_amax_reset_kernel<<<1, 64, 0, st>>>(amax, n);
  return (int)hipGetLastError();
}

// fp16-pair range status of the last rollout (X3_RANGE_ACT) and weight refresh (X3_RANGE_W) -> *out (float, for the
// all-reduced counters slot); both flags reset
int x3_status_fold(void* wstatus, float* out, hipStream_t st) {
  if (!wstatus || !out) return -22;
  x3_status_fold_kernel<<<1, 64, 0, st>>>((uint32_t*)wstatus, out);
  return (int)hipGetLastError();
}

// n layers, meta[i] = {w_off, chunk, K, KP, Cout}, Wc[i] / WcT[i] (WcT[i] may be null); one launch
int x3_refresh_weights_all(const float* flat, int n, const long* meta, void* const* Wc, void* const* WcT, int M,
                           int f16, void* status, hipStream_t st) {
  if (n <= 0 || n > X3_REFRESH_MAXL || !meta || !Wc || !WcT || M <= 0 || f16 < 0) return -22;
  RefreshSet rs{};
  long blocks = 0;
  for (int i = 0; i < n; ++i) {
    const long* m = meta + 5 * i;
    if (m[1] <= 0 || m[2] <= 0 || m[3] <= 0 || m[4] <= 0 || m[0] < 0 || m[3] < m[2] || !Wc[i]) return -22;
    rs.w_off[i] = m[0];
    rs.chunk[i] = (int)m[1]; rs.K[i] = (int)m[2]; rs.KP[i] = (int)m[3]; rs.Cout[i] = (int)m[4];
    rs.Wc[i] = (uint16_t*)Wc[i];
    rs.WcT[i] = (uint16_t*)WcT[i];
    rs.b0[i] = (int)blocks;
    blocks += (long)M * ((m[3] + 31) / 32) * ((m[4] + 63) / 64);
    if (blocks > 0x7FFFFFFFL) return -22;
  }
  rs.b0[n] = (int)blocks;
  rs.n = n; rs.M = M; rs.f16 = f16;
  refresh_x3_all_kernel<<<(unsigned)blocks, 256, 0, st>>>(flat, rs, (uint32_t*)status);
  return (int)hipGetLastError();
}

int x3_refresh_weights(const float* flat, long w_off, int chunk, int K, int KP, int Cout, int M, void* Wc, void* WcT,
                       int f16, void* status, hipStream_t st) {
  if (chunk <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || M <= 0 || w_off < 0 || f16 < 0 || KP < K) return -22;
  const long blocks = (long)M * ((KP + 31) / 32) * ((Cout + 63) / 64);
  if (blocks > 0x7FFFFFFFL) return -22;
  refresh_x3_kernel<<<(unsigned)blocks, 256, 0, st>>>(flat, w_off, chunk, K, KP, Cout, M, (uint16_t*)Wc,
                                                      (uint16_t*)WcT, f16, (uint32_t*)status);
  return (int)hipGetLastError();
}
}
