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
#include <type_traits>

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

// Path-local row r = (s, pos) with s = t*E + e.  Advancing by a stage of n rows
// (n < HOWO) needs at most one wrap: no divisions inside the main loops.
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

// The ReLU-bit word of a lane: byte r = byte k of row r's 64-lane ballot.  One v_perm_b32 per row on the SGPR
// ballot pair, its selector (byte k into byte r, 0x0C -> 0x00 elsewhere) one v_lshl_or_b32 -- instead of a
// 64-bit shift, mask, shift and or per row.  Selectors are formed at use: holding them cost the bf16 conv layers
// (128-VGPR budget at 4 waves/SIMD) 40 spilled VGPRs.
DEVI uint32_t relu_bits_word(const uint64_t (&bal)[4], uint32_t k) {
  uint32_t w = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    w |= __builtin_amdgcn_perm((uint32_t)(bal[r] >> 32), (uint32_t)bal[r],
                               (k << (8 * r)) | (0x0C0C0C0Cu & ~(0xFFu << (8 * r))));
  return w;
}

template <bool U8IN>
DEVI s8v ld8(const void* X, long off) {
  s8v r;
  if constexpr (U8IN) {
    r = u8x8_to_bf16(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + off));
  } else {
    r = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + off);
  }
  return r;
}

// ===========================================================================
// forward: grid = (ceil(T*E*HOWO / 256), P); each wave loops over 32-row tiles
// ===========================================================================
// NT = 32-row tiles per wave: a workgroup covers NT*128 rows and stages the path's
// active weights in LDS once for all of them.
//
// RING (first layer only): X is the frame ring [P*E][nslots][HIN*WIN] uint8 instead of packed
// 4-channel stacks; channel c of sample (t, b) reads frame slot t + max(c, fc[t][b]) of env b
// (fc = first valid channel after an episode reset, written by the env step).  A sample's four
// planes are one contiguous 77 KB run, as a packed stack was.  k is channel-major
// (k = (c*KH + kh)*KW + kw) so each A fragment is 8 consecutive pixels of one kernel row of one
// frame plane: still one 8-byte load.  Wc holds the weights in that k order.
template <class G, int NT, bool RING = false, bool F16 = false>
__global__ __launch_bounds__(256, G::U8 ? 3 : 4) void conv_fwd_fast(const void* __restrict__ X, bf16_t* __restrict__ Y,
                                                     uint8_t* __restrict__ bits, const bf16_t* __restrict__ Wc,
                                                     const float* __restrict__ flat, long bias_off, int chunk,
                                                     const int* __restrict__ act_idx, const int* __restrict__ act_cnt,
                                                     int layer, int L, int M, int P, int E, int T, int t0,
                                                     long bits_rows, float in_scale, float out_scale,
                                                     const uint8_t* __restrict__ fcv = nullptr, int nslots = 0,
                                                     const float* __restrict__ hcorr = nullptr) {
  static_assert(!RING || (G::U8 && G::CIN == 4 && G::KW == 8 && G::K == 256), "ring input: 8x8x4 uint8 layer");
  // F16 (uint8 input only): fp16 MFMA on (1024 + pixel) operands built with one v_perm per 2 pixels;
  // Wc then holds fp16 weights and hcorr[module*8 + map] = sum_k w_k (the offset's contribution)
  static_assert(!F16 || G::U8, "fp16-offset operands are for uint8 inputs");
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
  // compile-time column-tile count per instantiation (see conv_wgrad_slab)
  auto run = [&](auto ncc) {
    constexpr int NC = decltype(ncc)::value;
    const int Rtot = T * E * G::HOWO;
    const int PE = P * E;
    const int w = tid >> 6, l = tid & 63;
    const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
    // ReLU-bit byte of this lane's (row quad q, slot half h) in each row's 64-lane ballot: byte 2q + h
    const uint32_t bkey = (uint32_t)(2 * q + h);
    // one step per launch (the rollout, trunk()): global row = rowbase + path-local row, no iterator needed
    // (uint8 affine path only: in the bf16 layers' 128-VGPR budget the extra live values spilled)
    const bool lin = T == 1;
    const long rowbase = ((long)t0 * PE + (long)p * E) * G::HOWO;
    // lane rows: A-operand rows (rbase + 16i + c16) and epilogue rows (rbase + 16i + 4q + r)
    constexpr int FF_ROWS = NT * 128;
    const int rfirst = blockIdx.x * FF_ROWS + w * 32;
    RowIt ait[2], eit[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rowit_init(ait[i], rfirst + i * 16 + c16, E, G::HOWO);
      rowit_init(eit[i], rfirst + i * 16 + 4 * q, E, G::HOWO);
    }
    constexpr int NK = G::KP / 32;
    using ARaw = typename std::conditional<G::U8, uint2, s8v>::type;
    ARaw araw[2][NK];
    // issue the global loads of one 32-row tile (2 MFMA row tiles x NK k-steps) into registers
    // RING: the first-valid-channel bytes of every tile this wave will touch, loaded once up
    // front (a per-tile byte load would sit on the dependency path of that tile's X loads and
    // expose its latency on every tile)
    uint64_t fcw[2] = {0ull, 0ull};
    if constexpr (RING) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        RowIt it = ait[i];
#pragma unroll
        for (int tl = 0; tl < NT; ++tl) {
          if (it.r < Rtot) fcw[i] |= (uint64_t)fcv[rowit_sample(it, p, E, PE, t0)] << (8 * tl);
          rowit_adv(it, 128, E, G::HOWO);
        }
      }
    }
    auto load_tile = [&](int rbase) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool va = rbase < Rtot && ait[i].r < Rtot;
        const int oh = ait[i].pos / G::WO, ow = ait[i].pos - oh * G::WO;
        if constexpr (RING) {
          const int fc = (int)((fcw[i] >> (8 * ((rbase - rfirst) >> 7))) & 0xFFull);
          const long slot0 = (long)(p * E + ait[i].e) * nslots + t0 + ait[i].t;
          const long pix = (long)(oh * G::S * G::WIN + ow * G::S);
          // channel c's plane base with this lane's kernel row (grp) folded in; k-step kk then
          // reads plane kk/2 at the compile-time row offset (kk&1)*4 rows -> immediate offsets
          const uint8_t* pc[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            pc[c] = reinterpret_cast<const uint8_t*>(X) + (slot0 + max(c, fc)) * (long)(G::HIN * G::WIN) + pix +
                    grp * G::WIN;
          rowit_adv(ait[i], 128, E, G::HOWO);
          if (va) {
#pragma unroll
            for (int kk = 0; kk < NK; ++kk)
              araw[i][kk] = *reinterpret_cast<const uint2*>(pc[kk >> 1] + (kk & 1) * 4 * G::WIN);
          } else {
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) araw[i][kk] = make_uint2(0u, 0u);
          }
          continue;
        }
        const long xb = rowit_sample(ait[i], p, E, PE, t0) * (long)G::IN_ELEMS +
                        (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN;
        rowit_adv(ait[i], 128, E, G::HOWO);
        if constexpr (G::KW * G::CIN == 32 && G::K == G::KP) {
          // one kernel row per 32-k block: the lane offset is koff(grp) and block kk adds the
          // compile-time row stride -> one 64-bit address per row half, immediate load offsets
          using El = typename std::conditional<G::U8, uint8_t, bf16_t>::type;
          const El* src = reinterpret_cast<const El*>(X) + xb + G::koff(grp);
          if (va) {
#pragma unroll
            for (int kk = 0; kk < NK; ++kk)
              araw[i][kk] = *reinterpret_cast<const ARaw*>(src + kk * G::WIN * G::CIN);
          } else {
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) araw[i][kk] = ARaw{};
          }
          continue;
        }
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int off = G::koff(kk * 4 + grp);
          if constexpr (G::U8) {
            araw[i][kk] = make_uint2(0u, 0u);
            if (va && off >= 0) araw[i][kk] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xb + off);
          } else {
            araw[i][kk] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
            if (va && off >= 0) araw[i][kk] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xb + off);
          }
        }
      }
    };
    // affine uint8 layer (conv1 on packed stacks): per-tile row addresses only, fragments loaded per k-step
    constexpr bool AFF8 = !RING && G::U8 && G::KW * G::CIN == 32 && G::K == G::KP;
    using El = typename std::conditional<G::U8, uint8_t, bf16_t>::type;
    const El* asrc[2];
    // rows past the end read row 0 of the path's first sample instead: their 16-row halves are never stored
    auto aff_addr = [&]() {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool va = ait[i].r < Rtot;
        const int oh = ait[i].pos / G::WO, ow = ait[i].pos - oh * G::WO;
        const long xb = va ? rowit_sample(ait[i], p, E, PE, t0) * (long)G::IN_ELEMS +
                                 (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN
                           : rowit_sample(RowIt{0, 0, 0, 0}, p, E, PE, t0) * (long)G::IN_ELEMS;
        asrc[i] = reinterpret_cast<const El*>(X) + xb + G::koff(grp);
        rowit_adv(ait[i], 128, E, G::HOWO);
      }
    };
    // uint8 first layer: the first tile's A loads do not depend on LDS, so they are issued before the
    // weight staging and its barrier and their latency overlaps the Wc gather (nct is uniform over the
    // block, so every thread reaches the barrier).  Not for the bf16 layers: at their 128-VGPR budget
    // the longer live range spills, and that build wrote wrong ReLU bits for conv2
    // (scripts/diag_conv_bits.py, docs/PERF.md).
    if constexpr (AFF8) {
      aff_addr();
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) araw[i][kk] = *reinterpret_cast<const ARaw*>(asrc[i] + kk * G::WIN * G::CIN);
    } else if constexpr (G::U8) {
      load_tile(rfirst);
    }
    for (int i = tid; i < NC * 16 * G::KC; i += 256) {
      const int col = i / G::KC, kc = i - col * G::KC;
      const int slot = col >> 3;
      s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (slot < cnt) v = *reinterpret_cast<const s8v*>(Wc + ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8);
      *reinterpret_cast<s8v*>(Ws + col * KPs + kc * 8) = v;
    }
    if (tid < NCT * 16) {
      float bv = 0.f;
      if ((tid >> 3) < cnt) {
        bv = flat[bias_off + (long)mods[tid >> 3] * chunk + (tid & 7)];
        if constexpr (F16) bv -= 1024.f * in_scale * hcorr[mods[tid >> 3] * 8 + (tid & 7)];
      }
      bias_s[tid] = bv;
    }
    __syncthreads();
    if constexpr (!G::U8) load_tile(rfirst);
    if constexpr (AFF8) {
      // one 32-row tile; RELOAD (AFF8 only): the next tile's fragments are loaded into the same registers
      auto do_tile = [&](const int tile, const int rbase, auto reload_c) {
        constexpr bool RELOAD = decltype(reload_c)::value;
        f4v acc[2][NC];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
        // MFMAs of k-step kk on this tile's (converted) fragments
        auto kstep = [&](const s8v& a0, const s8v& a1, int kk) {
          const int kc = kk * 4 + grp;
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const s8v b = *reinterpret_cast<const s8v*>(Ws + (ct * 16 + c16) * KPs + kc * 8);
            if constexpr (F16) {
              acc[0][ct] = mfma16_f16(a0, b, acc[0][ct]);
              acc[1][ct] = mfma16_f16(a1, b, acc[1][ct]);
            } else {
              acc[0][ct] = mfma16(a0, b, acc[0][ct]);
              acc[1][ct] = mfma16(a1, b, acc[1][ct]);
            }
          }
        };
        // ONE register set: k-step kk's raw fragments are converted, then the same registers are
        // reloaded with the NEXT tile's k-step kk before this step's MFMAs issue -- the loads stay in
        // flight for the rest of the k loop and the epilogue, and no fragment is ever copied (the
        // two-set pipeline below costs ~2 v_mov per fragment dword per tile)
        if constexpr (RELOAD) aff_addr();
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          s8v a0, a1;
          if constexpr (F16) {
            a0 = u8x8_to_f16off(araw[0][kk]);
            a1 = u8x8_to_f16off(araw[1][kk]);
          } else {
            a0 = u8x8_to_bf16(araw[0][kk]);
            a1 = u8x8_to_bf16(araw[1][kk]);
          }
          if constexpr (RELOAD) {
            araw[0][kk] = *reinterpret_cast<const ARaw*>(asrc[0] + kk * G::WIN * G::CIN);
            araw[1][kk] = *reinterpret_cast<const ARaw*>(asrc[1] + kk * G::WIN * G::CIN);
          }
          kstep(a0, a1, kk);
          // keep program order per k-step: the scheduler otherwise hoists every conversion to the top of
          // the tile (one wait for all 16 fragments) and sinks every reload to its end
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r16 = rbase + i * 16;
          long grow4;
          if (lin) {
            grow4 = rowbase + r16 + 4 * q;
          } else {
            const RowIt e0 = eit[i];
            rowit_adv(eit[i], 128, E, G::HOWO);
            grow4 = rowit_sample(e0, p, E, PE, t0) * G::HOWO + e0.pos;
          }
          if (r16 >= Rtot) continue;
          float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            // slots >= cnt have zero weights and bias (staged that way), so v == 0 and they never fire
            const int slot = ct * 2 + h;
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
            // rows 4q..4q+3 of this tile are consecutive global rows (E*HOWO % 16 == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) Y[(grow4 + r) * 8 + ch] = f2bf(sum[r] * out_scale);
          }
        }
      };
      // the reloading body runs while a next tile exists; the last tile is peeled (no reloads), so the
      // fragment registers carry no conditional value across iterations (that cost a copy of the set)
      // fully unrolled (NT - 1 reloading tiles): a rolled loop's back-edge made the wait-count pass drain
      // every load in flight at the end of each tile
      int tile = 0;
#pragma unroll
      for (; tile + 1 < FF_ROWS / 128; ++tile) {
        const int rbase = rfirst + tile * 128;
        if (rbase + 128 >= Rtot) break;
        do_tile(tile, rbase, std::true_type{});
      }
      const int rbase = rfirst + tile * 128;
      if (rbase < Rtot) do_tile(tile, rbase, std::false_type{});
    } else {
      for (int tile = 0; tile < FF_ROWS / 128; ++tile) {
        const int rbase = rfirst + tile * 128;
        if (rbase >= Rtot) break;
        // raw fragments of this tile; the uint8 -> bf16 conversion happens per k-step next to its
        // MFMAs (holding all converted fragments cost 64 VGPRs and capped occupancy at 2 waves)
        ARaw cur[2][NK];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) cur[i][kk] = araw[i][kk];
        if (tile + 1 < FF_ROWS / 128) load_tile(rbase + 128);     // next tile in flight during MFMAs + epilogue
        f4v acc[2][NC];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) acc[i][ct] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const int kc = kk * 4 + grp;
          s8v a0, a1;
          if constexpr (F16) {
            a0 = u8x8_to_f16off(cur[0][kk]);
            a1 = u8x8_to_f16off(cur[1][kk]);
          } else if constexpr (G::U8) {
            a0 = u8x8_to_bf16(cur[0][kk]);
            a1 = u8x8_to_bf16(cur[1][kk]);
          } else {
            a0 = cur[0][kk];
            a1 = cur[1][kk];
          }
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            const s8v b = *reinterpret_cast<const s8v*>(Ws + (ct * 16 + c16) * KPs + kc * 8);
            if constexpr (F16) {
              acc[0][ct] = mfma16_f16(a0, b, acc[0][ct]);
              acc[1][ct] = mfma16_f16(a1, b, acc[1][ct]);
            } else {
              acc[0][ct] = mfma16(a0, b, acc[0][ct]);
              acc[1][ct] = mfma16(a1, b, acc[1][ct]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r16 = rbase + i * 16;
          const RowIt e0 = eit[i];
          rowit_adv(eit[i], 128, E, G::HOWO);
          if (r16 >= Rtot) continue;
          float sum[4] = {0.f, 0.f, 0.f, 0.f};
          const long grow4 = rowit_sample(e0, p, E, PE, t0) * G::HOWO + e0.pos;
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) {
            {
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
          if (h == 0) {
            // rows 4q..4q+3 of this tile are consecutive global rows (E*HOWO % 16 == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) Y[(grow4 + r) * 8 + ch] = f2bf(sum[r] * out_scale);
          }
        }
      }
    }
  };
  switch (nct) {
    case 0:   // empty layer: zero weights -> zero output, cheapest instantiation
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 3: run(std::integral_constant<int, 3>{}); break;
    case 4: run(std::integral_constant<int, 4>{}); break;
    default: run(std::integral_constant<int, NCT>{}); break;
  }
}

template <class G, int OB>
struct Slab {
  static constexpr int RL = G::WIN * G::CIN;               // input row length (elements)
  static constexpr int PS = G::S * G::CIN;                 // position stride within a row
  static constexpr int SEG = G::KW * G::CIN;               // one kernel row of k
  static constexpr int NB = (G::HO + OB - 1) / OB;         // bands per sample
  static constexpr int NPOS = OB * G::WO;                  // positions per (full) band
  static constexpr int KS = (NPOS + 31) / 32;              // MFMA k-steps per stage
  static constexpr int SR = (OB - 1) * G::S + G::KH;       // slab rows
  static constexpr int SLAB = SR * RL;                     // slab elements
  static constexpr int SLABP = SLAB + 64;                  // + zeroed slack for padded positions
  static constexpr int NG8 = SLAB / 8;                     // 8-element groups per slab
  static constexpr int XIT = (NG8 + 255) / 256;
  static_assert(SEG == 32 && PS == 16, "slab wgrad needs KW*CIN == 32 and S*CIN == 16");
  static_assert(SLAB % 8 == 0, "slab must be a whole number of 8-element groups");
};

// ===========================================================================
// forward, LDS-slab implicit im2col (KW*CIN == 32, S*CIN == 16 geometries).
// grid = (chunks, P); 256 threads.  The path's active module weights are staged
// once in LDS (B fragments), so the unit loop only streams the input: per unit (one sample's band of OB output rows) the touched input rows
// are one contiguous range, copied + converted once into LDS (double-buffered,
// register prefetch); each A fragment (8 consecutive k of one position = one
// 16-byte run of a kernel row) is a single ds_read_b128 from the slab.
// Epilogue: bias + ReLU + ReLU bits (ballot) + module sum, as conv_fwd_fast.
// ===========================================================================
template <class G, int OB>
__global__ __launch_bounds__(256, 2) void conv_fwd_slab(const void* __restrict__ X, bf16_t* __restrict__ Y,
                                                        uint8_t* __restrict__ bits, const bf16_t* __restrict__ Wc,
                                                        const float* __restrict__ flat, long bias_off, int chunk,
                                                        const int* __restrict__ act_idx,
                                                        const int* __restrict__ act_cnt, int layer, int L, int M,
                                                        int P, int E, int T, int t0, long bits_rows, int units_per_wg,
                                                        float in_scale, float out_scale) {
  using SB = Slab<G, OB>;
  constexpr int NK = G::KP / 32;                           // = KH (one kernel row per k-step)
  constexpr int NRT = (SB::NPOS + 15) / 16;                // 16-row tiles per unit
  constexpr int RTW = (NRT + 3) / 4;                       // row tiles per wave
  static_assert(NK == G::KH, "one kernel row per 32-wide k-step");
  constexpr int KPs = G::KP + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Ws[NCT * 16 * KPs];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][SB::SLABP];
  __shared__ float bias_s[NCT * 16];
  __shared__ int mods[MAXM_F];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  for (int i = tid; i < 2 * 64; i += 256) Xs[i >> 6][SB::SLAB + (i & 63)] = 0;
  __syncthreads();
  if (tid < NCT * 16) bias_s[tid] = (tid >> 3) < cnt ? flat[bias_off + (long)mods[tid >> 3] * chunk + (tid & 7)] : 0.f;
  // active module weights staged once: Ws[col = slot*8 + map][k] (B operand rows)
  for (int i = tid; i < nct * 16 * G::KC; i += 256) {
    const int col = i / G::KC, kc = i - col * G::KC;
    const int slot = col >> 3;
    s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (slot < cnt) v = *reinterpret_cast<const s8v*>(Wc + ((long)(mods[slot] * 8 + (col & 7))) * G::KP + kc * 8);
    *reinterpret_cast<s8v*>(Ws + col * KPs + kc * 8) = v;
  }
  const int PE = P * E;
  const int nunits = T * E * SB::NB;
  const int u_beg = blockIdx.x * units_per_wg;
  const int u_end = min(nunits, u_beg + units_per_wg);
  // per-lane A offsets (row = position rho = tile*16 + c16) and epilogue rows (tile*16 + 4q + r)
  int aoff[RTW];
#pragma unroll
  for (int i = 0; i < RTW; ++i) {
    int rho = (w + 4 * i) * 16 + c16;
    if (rho >= SB::NPOS) rho = 0;
    const int ob = rho / G::WO, ow = rho - ob * G::WO;
    aoff[i] = ob * G::S * SB::RL + ow * SB::PS + 8 * grp;
  }
  using XRaw = typename std::conditional<G::U8, uint2, s8v>::type;
  XRaw xr[SB::XIT];
  auto load_stage = [&](int u) {
    const int s = u / SB::NB, band = u - s * SB::NB;
    const long sg = sample_global(p, s, E, PE, t0);
    const int ih0 = band * OB * G::S;
    const int navail = min(SB::SR, G::HIN - ih0) * SB::RL;
    const long xbase = sg * (long)G::IN_ELEMS + (long)ih0 * SB::RL;
#pragma unroll
    for (int j = 0; j < SB::XIT; ++j) {
      const int gi = tid + 256 * j;
      const int e0 = gi * 8;
      if constexpr (G::U8) {
        xr[j] = make_uint2(0u, 0u);
        if (gi < SB::NG8 && e0 < navail)
          xr[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xbase + e0);
      } else {
        xr[j] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
        if (gi < SB::NG8 && e0 < navail)
          xr[j] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xbase + e0);
      }
    }
  };
  if (u_beg < u_end) load_stage(u_beg);
  int buf = 0;
  for (int u = u_beg; u < u_end; ++u, buf ^= 1) {
#pragma unroll
    for (int j = 0; j < SB::XIT; ++j) {
      const int gi = tid + 256 * j;
      if (gi < SB::NG8) {
        s8v v;
        if constexpr (G::U8) v = u8x8_to_bf16(xr[j]);
        else v = xr[j];
        *reinterpret_cast<s8v*>(&Xs[buf][gi * 8]) = v;
      }
    }
    __syncthreads();
    const int s = u / SB::NB, band = u - s * SB::NB;
    const long sg = sample_global(p, s, E, PE, t0);
    const long grow0 = sg * G::HOWO + (long)band * OB * G::WO;     // global row of position 0 of the band
    const int npos = min(OB, G::HO - band * OB) * G::WO;
    if (u + 1 < u_end) load_stage(u + 1);
    const bf16_t* xs = Xs[buf];
#pragma unroll
    for (int i = 0; i < RTW; ++i) {
      const int rt = w + 4 * i;
      if (rt >= NRT) break;
      f4v acc[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[ct] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const s8v a = *reinterpret_cast<const s8v*>(xs + kk * SB::RL + aoff[i]);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          if (ct < nct) {
            const s8v b = *reinterpret_cast<const s8v*>(Ws + (ct * 16 + c16) * KPs + kk * 32 + 8 * grp);
            acc[ct] = mfma16(a, b, acc[ct]);
          }
      }
      float sum[4] = {0.f, 0.f, 0.f, 0.f};
      const int rho0 = rt * 16 + 4 * q;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        if (ct < nct) {
          const int slot = ct * 2 + h;
          const bool sv = slot < cnt;
          const float bb = bias_s[ct * 16 + c16];
          uint32_t word = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[ct][r] * in_scale + bb;
            const bool pos = sv && v > 0.f;
            sum[r] += pos ? v : 0.f;
            const uint64_t bal = __ballot(pos);
            word |= (uint32_t)((bal >> (16 * q + 8 * h)) & 0xFFull) << (8 * r);
          }
          if (ch == 0 && sv) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (rho0 + r < npos) bits[(long)slot * bits_rows + grow0 + rho0 + r] = (uint8_t)(word >> (8 * r));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
      if (h == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (rho0 + r < npos) Y[(grow0 + rho0 + r) * 8 + ch] = f2bf(sum[r] * out_scale);
      }
    }
    // no trailing barrier: the next unit writes the other buffer, and this one is only rewritten
    // after every wave has passed the next unit's post-write barrier (i.e. finished this unit)
  }
}

// ===========================================================================
// forward, whole-image staging (first layer, uint8 frames): grid = (2*T*E, P).
// A workgroup owns one half of one sample's output rows; the input rows that half
// touches (~84 rows x 480 B of uint8) are copied into LDS ONCE with 16-byte loads
// (all issued before the barrier: maximal memory-level parallelism), so every input
// byte crosses L2 once per workgroup instead of KH*KW/S^2 = 4 times.  A fragments are
// ds_read_b64 of 2 pixels x 4 channels (8 consecutive k of one kernel row) converted
// u8 -> bf16 once per 16-position tile and reused by every active column tile; B comes
// straight from the 8 KB/path bf16 weight copy (L1/L2 resident).  ~40 KB LDS -> 3-4
// workgroups per CU overlap one another's load and MFMA phases.
// ===========================================================================
template <class G>
struct Half {
  static constexpr int RL = G::WIN * G::CIN;                       // bytes per input row
  static constexpr int OH0 = (G::HO + 1) / 2;                      // output rows of the first half
  static constexpr int IR_MAX = (OH0 - 1) * G::S + G::KH;          // input rows per half (max)
  static constexpr int BYTES = IR_MAX * RL;
};

template <class G>
__global__ __launch_bounds__(256, 3) void conv_fwd_img(const uint8_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                       uint8_t* __restrict__ bits, const bf16_t* __restrict__ Wc,
                                                       const float* __restrict__ flat, long bias_off, int chunk,
                                                       const int* __restrict__ act_idx,
                                                       const int* __restrict__ act_cnt, int layer, int L, int M, int P,
                                                       int E, int T, int t0, long bits_rows, float in_scale,
                                                       float out_scale) {
  using H = Half<G>;
  static_assert(G::U8 && G::KW * G::CIN == 32 && G::S * G::CIN == 16, "uint8 first-layer geometry");
  constexpr int NK = G::KP / 32;                                  // = KH
  __shared__ __attribute__((aligned(16))) uint8_t Xs[H::BYTES + 64];
  __shared__ float bias_s[NCT * 16];
  __shared__ int mods[MAXM_F];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15, q = grp, h = c16 >> 3, ch = l & 7;
  const int s = blockIdx.x >> 1, half = blockIdx.x & 1;
  const int oh_beg = half ? H::OH0 : 0, oh_end = half ? G::HO : H::OH0;
  const int ih_beg = oh_beg * G::S;
  const int nbytes = min(H::BYTES, (G::HIN - ih_beg) * H::RL);
  const long sg = sample_global(p, s, E, P * E, t0);
  // (1) issue the image copy first (16 B per load), then the weights
  const uint8_t* src = X + sg * (long)G::IN_ELEMS + (long)ih_beg * H::RL;
  for (int i = tid * 16; i < nbytes; i += 256 * 16)
    *reinterpret_cast<uint4*>(Xs + i) = *reinterpret_cast<const uint4*>(src + i);
  if (tid < 4) *reinterpret_cast<uint4*>(Xs + H::BYTES + tid * 16) = make_uint4(0u, 0u, 0u, 0u);
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  __syncthreads();
  if (tid < NCT * 16) bias_s[tid] = (tid >> 3) < cnt ? flat[bias_off + (long)mods[tid >> 3] * chunk + (tid & 7)] : 0.f;
  __syncthreads();
  const int npos = (oh_end - oh_beg) * G::WO;
  const int ntile = (npos + 15) / 16;
  const long grow0 = sg * G::HOWO + (long)oh_beg * G::WO;
  for (int tile = w; tile < ntile; tile += 4) {
    int rho = tile * 16 + c16;
    const bool rv = rho < npos;
    if (!rv) rho = 0;
    const int ob = rho / G::WO, ow = rho - ob * G::WO;
    const uint8_t* ap = Xs + ob * G::S * H::RL + ow * (G::S * G::CIN) + 8 * grp;
    // A fragments of this 16-position tile for all k-steps: converted once, reused by every column tile
    s8v a[NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) a[kk] = u8x8_to_bf16(*reinterpret_cast<const uint2*>(ap + kk * H::RL));
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
    const int rho0 = tile * 16 + 4 * q;
    for (int ct = 0; ct < nct; ++ct) {           // runtime loop: only the active column tiles, few live registers
      f4v acc = {0.f, 0.f, 0.f, 0.f};
      const int slot = ct * 2 + h;
      const bool sv = slot < cnt;
      // B straight from the (L1/L2-resident, 8 KB per path) bf16 weight copy
      const bf16_t* bp = Wc + ((long)(mods[sv ? slot : 0] * 8 + ch)) * G::KP + 8 * grp;
      s8v bfr[NK];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
        bfr[kk] = sv ? *reinterpret_cast<const s8v*>(bp + kk * 32) : (s8v){0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) acc = mfma16(a[kk], bfr[kk], acc);
      const float bb = bias_s[ct * 16 + c16];
      uint32_t word = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[r] * in_scale + bb;
        const bool pos = sv && v > 0.f;
        sum[r] += pos ? v : 0.f;
        const uint64_t bal = __ballot(pos);
        word |= (uint32_t)((bal >> (16 * q + 8 * h)) & 0xFFull) << (8 * r);
      }
      if (ch == 0 && sv) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (rho0 + r < npos) bits[(long)slot * bits_rows + grow0 + rho0 + r] = (uint8_t)(word >> (8 * r));
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
    if (h == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (rho0 + r < npos) Y[(grow0 + rho0 + r) * 8 + ch] = f2bf(sum[r] * out_scale);
    }
  }
}

// ===========================================================================
// wgrad: grid = (nchunks, P), 512 threads (8 waves), 32-row stages, register
// prefetch + double-buffered LDS: one barrier per stage; stage i+1's global
// loads are in flight while the MFMAs of stage i run.
//   A = im2col(X)^T  (m = k index, reduction = rows)  -> ds_read_b64_tr_b16
//   B = masked G      (reduction = rows, n = slot*8+map) -> ds_read_b64_tr_b16
// ===========================================================================
#define WG_RB 32
#define WG_NT 512
template <class G>
__global__ __launch_bounds__(WG_NT, 4) void conv_wgrad_fast(const void* __restrict__ X, const float* __restrict__ Gr,
                                                         const uint8_t* __restrict__ bits, float* __restrict__ grad,
                                                         long w_off, long b_off, int chunk,
                                                         const int* __restrict__ act_idx,
                                                         const int* __restrict__ act_cnt, int layer, int L, int M,
                                                         int P, int E, int T, long bits_rows, int rows_per_chunk,
                                                         float in_scale, float g_scale) {
  constexpr int XS = G::KP + 8;
  constexpr int GS = NCT * 16 + 8;
  constexpr int NMT = G::KP / 16;
  constexpr int NW = WG_NT / 64;
  constexpr int MPW = (NMT + NW - 1) / NW;
  constexpr int XIT = (WG_RB * G::KC + WG_NT - 1) / WG_NT;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][WG_RB * XS];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][WG_RB * GS];
  __shared__ float dbias[NCT * 16];
  __shared__ int mods[MAXM_F];
  __shared__ __attribute__((aligned(16))) uint32_t mtab[256 * 8];   // byte -> 8 x (0 | 0xFFFFFFFF)
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x;
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  if (tid < NCT * 16) dbias[tid] = 0.f;
  for (int i = tid; i < 256 * 8; i += WG_NT) mtab[i] = ((i >> 3) >> (i & 7)) & 1u ? 0xFFFFFFFFu : 0u;
  for (int i = tid; i < 2 * WG_RB * GS; i += WG_NT) (&Gs[0][0])[i] = 0;
  static_assert(G::HOWO > WG_RB, "row iterator assumes one wrap per stage");
  const int Rtot = T * E * G::HOWO;          // host asserts < 2^31
  const int PE = P * E;
  const int r_begin = blockIdx.x * rows_per_chunk;
  const int r_end = min(Rtot, r_begin + rows_per_chunk);
  const int w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  const int gslot = tid & 15, grow = tid >> 4;     // G staging role (fixed slot per thread)
  const bool gact = gslot < cnt;
  float bpart[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  f4v acc[MPW][NCT];
#pragma unroll
  for (int a = 0; a < MPW; ++a)
#pragma unroll
    for (int b = 0; b < NCT; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};

  // ---- prefetch registers: two sets, stages s+1 and s+2 in flight while stage s computes ----
  using XRaw = typename std::conditional<G::U8, uint2, s8v>::type;
  XRaw xr[2][XIT];
  bool xv[2][XIT];
  float4 g0r[2], g1r[2];
  uint32_t gbr[2] = {0u, 0u};
  bool gv[2] = {false, false};

  // per-item row iterators (rows advance by WG_RB per stage)
  RowIt xit[XIT];
  int xkoff[XIT];
#pragma unroll
  for (int j = 0; j < XIT; ++j) {
    const int it = tid + WG_NT * j;
    const int row = it / G::KC, kc = it - row * G::KC;
    xkoff[j] = (it < WG_RB * G::KC) ? G::koff(kc) : -1;
    rowit_init(xit[j], (int)r_begin + row, E, G::HOWO);
  }
  RowIt git;
  rowit_init(git, (int)r_begin + grow, E, G::HOWO);

  auto load_stage = [&](const int k) {
#pragma unroll
    for (int j = 0; j < XIT; ++j) {
      xv[k][j] = xkoff[j] >= 0 && xit[j].r < r_end;
      if (xv[k][j]) {
        const int oh = xit[j].pos / G::WO, ow = xit[j].pos - oh * G::WO;
        const long xo = rowit_sample(xit[j], p, E, PE, 0) * (long)G::IN_ELEMS +
                        (long)(oh * G::S * G::WIN + ow * G::S) * G::CIN + xkoff[j];
        if constexpr (G::U8)
          xr[k][j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xo);
        else
          xr[k][j] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xo);
      }
      rowit_adv(xit[j], WG_RB, E, G::HOWO);
    }
    gv[k] = gact && git.r < r_end;
    if (gv[k]) {
      const long go = rowit_sample(git, p, E, PE, 0) * G::HOWO + git.pos;
      g0r[k] = *reinterpret_cast<const float4*>(Gr + go * 8);
      g1r[k] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
      gbr[k] = bits[(long)gslot * bits_rows + go];
    }
    rowit_adv(git, WG_RB, E, G::HOWO);
  };
  auto write_stage = [&](const int buf) {   // register set k == LDS buffer buf
#pragma unroll
    for (int j = 0; j < XIT; ++j) {
      const int it = tid + WG_NT * j;
      if (it < WG_RB * G::KC) {
        const int row = it / G::KC, kc = it - row * G::KC;
        s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (xv[buf][j]) {
          if constexpr (G::U8)
            v = u8x8_to_bf16(xr[buf][j]);
          else
            v = xr[buf][j];
        }
        *reinterpret_cast<s8v*>(&Xs[buf][row * XS + kc * 8]) = v;
      }
    }
    if (gact) {
      s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (gv[buf]) {
        // ReLU-bit byte -> 8 fp32 AND masks from the LDS table (one b128 x2 read, 8 v_and)
        const uint4 m0 = *reinterpret_cast<const uint4*>(&mtab[gbr[buf] * 8]);
        const uint4 m1 = *reinterpret_cast<const uint4*>(&mtab[gbr[buf] * 8 + 4]);
        float gg[8] = {__uint_as_float(__float_as_uint(g0r[buf].x) & m0.x), __uint_as_float(__float_as_uint(g0r[buf].y) & m0.y),
                       __uint_as_float(__float_as_uint(g0r[buf].z) & m0.z), __uint_as_float(__float_as_uint(g0r[buf].w) & m0.w),
                       __uint_as_float(__float_as_uint(g1r[buf].x) & m1.x), __uint_as_float(__float_as_uint(g1r[buf].y) & m1.y),
                       __uint_as_float(__float_as_uint(g1r[buf].z) & m1.z), __uint_as_float(__float_as_uint(g1r[buf].w) & m1.w)};
#pragma unroll
        for (int c = 0; c < 8; ++c) bpart[c] += gg[c];
        v = f32x8_to_bf16(gg);
      }
      *reinterpret_cast<s8v*>(&Gs[buf][grow * GS + gslot * 8]) = v;
    }
  };

  // Stage s uses register set and LDS buffer s & 1.  Writing buffer b at stage s is safe: every
  // wave finished its stage s-2 MFMAs (same buffer) before the barrier of stage s-1.
  auto compute = [&](const int buf) {
    const bf16_t* xs = Xs[buf];
    const bf16_t* gs = Gs[buf];
    s8v bfr[NCT];
#pragma unroll
    for (int nt = 0; nt < NCT; ++nt) {
      if (nt < nct) {
        const s4v v0 = lds_tr16(gs + (8 * grp + q) * GS + nt * 16 + 4 * pp);
        const s4v v1 = lds_tr16(gs + (8 * grp + 4 + q) * GS + nt * 16 + 4 * pp);
        bfr[nt] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
    }
#pragma unroll
    for (int mi = 0; mi < MPW; ++mi) {
      const int mt = w + NW * mi;
      if (mt < NMT) {
        const s4v v0 = lds_tr16(xs + (8 * grp + q) * XS + mt * 16 + 4 * pp);
        const s4v v1 = lds_tr16(xs + (8 * grp + 4 + q) * XS + mt * 16 + 4 * pp);
        const s8v afr = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int nt = 0; nt < NCT; ++nt)
          if (nt < nct) acc[mi][nt] = mfma16(afr, bfr[nt], acc[mi][nt]);
      }
    }
  };
  auto stage = [&](const int k, const int rb) {
    write_stage(k);
    __syncthreads();
    if (rb + 2 * WG_RB < r_end) load_stage(k);
    compute(k);
  };
  __syncthreads();
  if (r_begin < r_end) load_stage(0);
  if (r_begin + WG_RB < r_end) load_stage(1);
  for (int rb = r_begin; rb < r_end; rb += 2 * WG_RB) {
    stage(0, rb);
    if (rb + WG_RB < r_end) stage(1, rb + WG_RB);
  }
  const int h = i16 >> 3, ch = l & 7;
#pragma unroll
  for (int mi = 0; mi < MPW; ++mi) {
    const int mt = w + NW * mi;
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
              if (k < G::K) atomicAdd(&grad[base + (long)k * 8 + ch], acc[mi][nt][r] * (in_scale * g_scale));
            }
          }
        }
      }
    }
  }
  if (gact) {
#pragma unroll
    for (int c = 0; c < 8; ++c) atomicAdd(&dbias[gslot * 8 + c], bpart[c] * g_scale);
  }
  __syncthreads();
  if (tid < cnt * 8) atomicAdd(&grad[b_off + (long)mods[tid >> 3] * chunk + (tid & 7)], dbias[tid]);
}

// ===========================================================================
// wgrad, LDS-slab implicit im2col (geometries with KW*CIN == 32 and S*CIN == 16:
// the 160x120x4/8x8/s4 and 39x29x8/4x4/s2 layers).  A stage is a band of OB output
// rows of one sample: the input rows it touches are ONE contiguous range of the
// image, copied (and u8->bf16 converted) once into LDS; the MFMA A operand
// (im2col^T: m = k, reduction = position) is read straight out of that slab with
// ds_read_b64_tr_b16 -- position rows are 16 elements apart and the 32 k of one
// kernel row are contiguous, so no im2col copy is ever materialised (each input
// byte is converted once per stage instead of KH*KW/S^2 times).  Positions of the
// band are packed densely into 32-row MFMA k-steps.  Masked G (ReLU bits) goes to
// LDS as bf16 as before.  Register prefetch of the next stage + double-buffered LDS.
// grid = (chunks, P); 256 threads; each workgroup reduces a contiguous range of
// (sample, band) units and atomically adds its partial dW/db.
// ===========================================================================

// PF = stages of global loads in flight (register sets).  PF=2 keeps stage u+2's
// loads in flight while stage u computes: one stage of MFMA work (~256 cycles
// per wave) is far shorter than an HBM round trip, so with PF=1 every stage
// waited on its own prefetch.  X loads are branch-free (clamped address, zeroed
// at write time) so hipcc can count vmcnt across the two sets.
//
// RING: X is the frame ring (see conv_fwd_fast); a stage loads 8 pixels of each of the 4
// channel planes per thread and interleaves them into the packed (pixel, channel) slab at
// LDS-write time, so the slab layout and every MFMA operand read are unchanged.
// GT = float, or bf16_t when the layer's output gradient was written in bf16 (conv_dgrad_mfma OT = bf16_t)
template <class G, int OB, int PF, bool RING = false, typename GT = float>
__global__ __launch_bounds__(256, 3) void conv_wgrad_slab(const void* __restrict__ X, const GT* __restrict__ Gr,
                                                          const uint8_t* __restrict__ bits, float* __restrict__ grad,
                                                          long w_off, long b_off, int chunk,
                                                          const int* __restrict__ act_idx,
                                                          const int* __restrict__ act_cnt, int layer, int L, int M,
                                                          int P, int E, int T, long bits_rows, int units_per_wg,
                                                          float in_scale, float g_scale,
                                                          const uint8_t* __restrict__ fcv = nullptr,
                                                          int nslots = 0) {
  using SB = Slab<G, OB>;
  static_assert(!RING || (G::U8 && G::CIN == 4 && G::WIN % 8 == 0), "ring input: uint8 4-channel first layer");
  constexpr int NGP = SB::SR * G::WIN / 8;                 // ring: 8-pixel groups per slab
  constexpr int XIT4 = (NGP + 255) / 256;
  constexpr int GS = NCT * 16 + 8;
  constexpr int NMT = G::KP / 16;
  constexpr int MPW = NMT / 4;
  constexpr int GROWS = SB::KS * 32;
  constexpr int GIT = (GROWS * 4 + 255) / 256;             // (row, slot-group) items per thread
  __shared__ __attribute__((aligned(16))) bf16_t Xs[2][SB::SLABP];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][GROWS * GS];
  __shared__ float dbias[NCT * 16];
  __shared__ int mods[MAXM_F];
  constexpr int FCS = RING ? 1024 : 1;
  __shared__ uint8_t fcs[FCS];     // RING: first-valid channel of this workgroup's samples
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  if (cnt == 0) return;
  const int nct = (cnt + 1) >> 1;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, i16 = l & 15, q = i16 >> 2, pp = i16 & 3;
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  const int s_first = (blockIdx.x * units_per_wg) / SB::NB;
  if constexpr (RING) {
    // staged once: a per-stage global byte load would expose its latency ahead of the X loads
    const int s_last = min(T * E, (blockIdx.x * units_per_wg + units_per_wg + SB::NB - 1) / SB::NB);
    for (int i = tid; i < s_last - s_first && i < FCS; i += 256) {
      fcs[i] = fcv[sample_global(p, s_first + i, E, P * E, 0)];
    }
  }
  if (tid < NCT * 16) dbias[tid] = 0.f;
  for (int i = tid; i < 2 * GROWS * GS; i += 256) (&Gs[0][0])[i] = 0;
  for (int i = tid; i < 2 * 64; i += 256) Xs[i >> 6][SB::SLAB + (i & 63)] = 0;
  const int PE = P * E;
  const int nunits = T * E * SB::NB;
  const int u_beg = blockIdx.x * units_per_wg;
  const int u_end = min(nunits, u_beg + units_per_wg);
  // per-lane A-operand position offsets inside the slab for each k-step (two 4-row halves)
  int aoff[SB::KS][2];
#pragma unroll
  for (int ks = 0; ks < SB::KS; ++ks)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      int rho = ks * 32 + 8 * grp + 4 * hf + q;
      if (rho >= SB::NPOS) rho = 0;                     // padded position: G row is zero
      const int ob = rho / G::WO, ow = rho - ob * G::WO;
      aoff[ks][hf] = ob * G::S * SB::RL + ow * SB::PS + 4 * pp;
    }
  // The column-tile count is a compile-time constant in each instantiation: the
  // MFMA / LDS-read loops are branch-free and fully unrolled (a runtime `nt < nct`
  // guard around every MFMA made hipcc emit a scalar branch per MFMA and
  // serialise the operand reads behind them).
  auto run = [&](auto ncc) {
    constexpr int NC = decltype(ncc)::value;
    float acc_b[3][8];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc_b[k][c] = 0.f;
    f4v acc[MPW][NC];
#pragma unroll
    for (int a = 0; a < MPW; ++a)
#pragma unroll
      for (int b = 0; b < NC; ++b) acc[a][b] = {0.f, 0.f, 0.f, 0.f};

    using XRaw = typename std::conditional<G::U8, uint2, s8v>::type;
    struct Regs {
      XRaw xr[RING ? 1 : SB::XIT];
      uint2 xq[RING ? XIT4 : 1][4];
      // G rows: fp32 as two float4; bf16 kept raw (one uint4) until write_stage, so the load stays in flight
      float4 g0r[sizeof(GT) == 2 ? 1 : GIT], g1r[sizeof(GT) == 2 ? 1 : GIT];
      uint4 graw[sizeof(GT) == 2 ? GIT : 1];
      uint32_t gbr[GIT][3];
      bool gvr[GIT];
      int navail;
    };
    Regs R[PF];

    // stages are loaded strictly in unit order (both PF modes): the (t, e, band) of the next
    // unit is advanced incrementally instead of dividing by the runtime E at every stage
    int it_band, it_e, it_t;
    {
      const int s0 = u_beg / SB::NB;
      it_band = u_beg - s0 * SB::NB;
      it_t = s0 / E;
      it_e = s0 - it_t * E;
    }
    auto load_stage = [&](Regs& Rg, int u) {
      (void)u;
      const int band = it_band, ut = it_t, ue = it_e;
      const int s = ut * E + ue;
      const long sg = (long)ut * PE + (long)p * E + ue;
      if (++it_band == SB::NB) {
        it_band = 0;
        if (++it_e == E) { it_e = 0; ++it_t; }
      }
      const int ih0 = band * OB * G::S;
      const int navail = min(SB::SR, G::HIN - ih0) * SB::RL;   // elements inside the image
      Rg.navail = navail;
      if constexpr (RING) {
        const int fc = (int)fcs[s - s_first];
        const long slot0 = (long)(p * E + ue) * nslots + ut;
        const int npx = min(SB::SR, G::HIN - ih0) * G::WIN;        // pixels inside the image
        Rg.navail = npx;
#pragma unroll
        for (int j = 0; j < XIT4; ++j) {
          const int gi = tid + 256 * j;
          const int e0 = (gi < NGP && gi * 8 < npx) ? gi * 8 : 0;   // clamped, zeroed at write time
#pragma unroll
          for (int c = 0; c < 4; ++c)
            Rg.xq[j][c] = *reinterpret_cast<const uint2*>(
                reinterpret_cast<const uint8_t*>(X) + (slot0 + max(c, fc)) * (long)(G::HIN * G::WIN) +
                (long)ih0 * G::WIN + e0);
        }
      }
      const long xbase = sg * (long)G::IN_ELEMS + (long)ih0 * SB::RL;
#pragma unroll
      for (int j = 0; j < (RING ? 0 : SB::XIT); ++j) {
        const int gi = tid + 256 * j;
        const int e0 = (gi < SB::NG8 && gi * 8 < navail) ? gi * 8 : 0;   // clamped, zeroed at write time
        if constexpr (G::U8)
          Rg.xr[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + xbase + e0);
        else
          Rg.xr[j] = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + xbase + e0);
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
          if constexpr (sizeof(GT) == 2) {
            Rg.graw[j] = *reinterpret_cast<const uint4*>(Gr + go * 8);
          } else {
            Rg.g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
            Rg.g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
          }
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int slot = sub + 4 * k;
            Rg.gbr[j][k] = slot < cnt ? bits[(long)slot * bits_rows + go] : 0u;
          }
        }
      }
    };
    auto write_stage = [&](const Regs& Rg, int buf) {
      if constexpr (RING) {
#pragma unroll
        for (int j = 0; j < XIT4; ++j) {
          const int gi = tid + 256 * j;
          if (gi < NGP) {
            const bool valid = gi * 8 < Rg.navail;
            // 4x4 byte transposes (channel-planar -> pixel-interleaved), 8 v_perm_b32 per 4 pixels
            uint32_t px[8];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const uint32_t A = hh ? Rg.xq[j][0].y : Rg.xq[j][0].x, B = hh ? Rg.xq[j][1].y : Rg.xq[j][1].x;
              const uint32_t C = hh ? Rg.xq[j][2].y : Rg.xq[j][2].x, D = hh ? Rg.xq[j][3].y : Rg.xq[j][3].x;
              const uint32_t t0 = __builtin_amdgcn_perm(B, A, 0x05010400u);    // A0 B0 A1 B1
              const uint32_t t1 = __builtin_amdgcn_perm(B, A, 0x07030602u);    // A2 B2 A3 B3
              const uint32_t t2 = __builtin_amdgcn_perm(D, C, 0x05010400u);    // C0 D0 C1 D1
              const uint32_t t3 = __builtin_amdgcn_perm(D, C, 0x07030602u);    // C2 D2 C3 D3
              px[4 * hh + 0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);     // A0 B0 C0 D0
              px[4 * hh + 1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);     // A1 B1 C1 D1
              px[4 * hh + 2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
              px[4 * hh + 3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
            }
#pragma unroll
            for (int pr = 0; pr < 4; ++pr) {       // pixels 2pr, 2pr+1: (pixel, channel) bytes
              s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
              if (valid) v = u8x8_to_bf16(make_uint2(px[2 * pr], px[2 * pr + 1]));
              *reinterpret_cast<s8v*>(&Xs[buf][gi * 32 + pr * 8]) = v;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < (RING ? 0 : SB::XIT); ++j) {
        const int gi = tid + 256 * j;
        if (gi < SB::NG8) {
          s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
          if (gi * 8 < Rg.navail) {
            if constexpr (G::U8) v = u8x8_to_bf16(Rg.xr[j]);
            else v = Rg.xr[j];
          }
          *reinterpret_cast<s8v*>(&Xs[buf][gi * 8]) = v;
        }
      }
#pragma unroll
      for (int j = 0; j < GIT; ++j) {
        const int it = tid + 256 * j;
        if (it >= GROWS * 4) continue;
        const int rho = it >> 2, sub = it & 3;
        float gg[8];
        if constexpr (sizeof(GT) == 2) {
          const uint32_t u[4] = {Rg.graw[j].x, Rg.graw[j].y, Rg.graw[j].z, Rg.graw[j].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gg[2 * e] = __uint_as_float(u[e] << 16);
            gg[2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u);
          }
        } else {
          gg[0] = Rg.g0r[j].x; gg[1] = Rg.g0r[j].y; gg[2] = Rg.g0r[j].z; gg[3] = Rg.g0r[j].w;
          gg[4] = Rg.g1r[j].x; gg[5] = Rg.g1r[j].y; gg[6] = Rg.g1r[j].z; gg[7] = Rg.g1r[j].w;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int slot = sub + 4 * k;
          if (slot < 2 * NC) {
            float m[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) m[c] = (Rg.gvr[j] && ((Rg.gbr[j][k] >> c) & 1u)) ? gg[c] : 0.f;
#pragma unroll
            for (int c = 0; c < 8; ++c) acc_b[k][c] += m[c];
            *reinterpret_cast<s8v*>(&Gs[buf][rho * GS + slot * 8]) = f32x8_to_bf16(m);
          }
        }
      }
    };
    auto compute_stage = [&](int buf) {
      const bf16_t* xs = Xs[buf];
      const bf16_t* gs = Gs[buf];
#pragma unroll
      for (int ks = 0; ks < SB::KS; ++ks) {
        s8v bfr[NC];
#pragma unroll
        for (int nt = 0; nt < NC; ++nt) {
          const s4v v0 = lds_tr16(gs + (ks * 32 + 8 * grp + q) * GS + nt * 16 + 4 * pp);
          const s4v v1 = lds_tr16(gs + (ks * 32 + 8 * grp + 4 + q) * GS + nt * 16 + 4 * pp);
          bfr[nt] = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        }
#pragma unroll
        for (int mi = 0; mi < MPW; ++mi) {
          const int mt = w * MPW + mi;
          const int kb = (mt * 16 / SB::SEG) * SB::RL + (mt * 16) % SB::SEG;     // kernel row kh, k offset
          const s4v v0 = lds_tr16(xs + kb + aoff[ks][0]);
          const s4v v1 = lds_tr16(xs + kb + aoff[ks][1]);
          const s8v afr = (s8v){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
          for (int nt = 0; nt < NC; ++nt) acc[mi][nt] = mfma16(afr, bfr[nt], acc[mi][nt]);
        }
      }
    };
    __syncthreads();
    // PF=2 only for <= 4 active modules (NC <= 2): with the NC=5 accumulators two register sets spilled
    if constexpr (PF == 1 || NC > 2) {
      // the last stage is peeled so the reload in the loop body is unconditional: a conditional reload is a
      // loop-carried phi and the compiler copied the whole register set (~140 v_mov per stage) to merge it
      if (u_beg < u_end) load_stage(R[0], u_beg);
      int u = u_beg, buf = 0;
      for (; u + 1 < u_end; ++u, buf ^= 1) {
        write_stage(R[0], buf);
        __syncthreads();
        load_stage(R[0], u + 1);
        compute_stage(buf);
      }
      if (u < u_end) {
        write_stage(R[0], buf);
        __syncthreads();
        compute_stage(buf);
      }
    } else {
      // stage u lives in register set (u - u_beg) & 1 and LDS buffer (u - u_beg) & 1.  The main loop reloads
      // unconditionally (a conditional reload is a loop-carried phi: the compiler copied both register sets
      // every stage); the last 0-3 stages run in the straight-line tail.
      if (u_beg < u_end) load_stage(R[0], u_beg);
      if (u_beg + 1 < u_end) load_stage(R[1], u_beg + 1);
      int u = u_beg;
      for (; u + 3 < u_end; u += 2) {
        write_stage(R[0], 0);
        __syncthreads();
        load_stage(R[0], u + 2);
        compute_stage(0);
        write_stage(R[1], 1);
        __syncthreads();
        load_stage(R[1], u + 3);
        compute_stage(1);
      }
      const int rem = u_end - u;
      if (rem >= 1) {
        write_stage(R[0], 0);
        __syncthreads();
        if (rem >= 3) load_stage(R[0], u + 2);
        compute_stage(0);
      }
      if (rem >= 2) {
        write_stage(R[1], 1);
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
        const int slot = nt * 2 + h;
        if (slot < cnt) {
          const long base = w_off + (long)mods[slot] * chunk;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = mt * 16 + 4 * grp + r;
            if (k < G::K) atomicAdd(&grad[base + (long)k * 8 + ch], acc[mi][nt][r] * (in_scale * g_scale));
          }
        }
      }
    }
    // bias: this thread's partials for slots (tid & 3) + 4k
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int slot = (tid & 3) + 4 * k;
      if (slot < cnt) {
#pragma unroll
        for (int c = 0; c < 8; ++c) atomicAdd(&dbias[slot * 8 + c], acc_b[k][c] * g_scale);
      }
    }
    __syncthreads();
  };
  switch (nct) {
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 3: run(std::integral_constant<int, 3>{}); break;
    case 4: run(std::integral_constant<int, 4>{}); break;
    default: run(std::integral_constant<int, NCT>{}); break;
  }
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

// ===========================================================================
// dgrad on MFMA (Cin = Cout = 8): "superpixel" implicit GEMM.
// For stride S the S x S input pixels (S*i+ph, S*j+pw) of superpixel (i, j) read the SAME
// output-gradient positions (i-ta, j-tb) through different taps (kh = ph + S*ta,
// kw = pw + S*tb), so one GEMM row = one superpixel, N = (ph, pw, ci) = 8*S*S
// (32 for the 4x4/s2 layer: two full 16-wide MFMA tiles), K = (tap, slot, c).
// Per sample the masked gradient of the active modules (G & ReLU bits, bf16) is
// staged in LDS once (every element feeds up to KH*KW/S^2 rows through the A
// fragments); the per-path weight matrix B[k][n] is staged once per workgroup.
// grid = (chunks, P), 256 threads; waves take 16-superpixel row tiles.
// ===========================================================================
#define DG_NSMAX 12          // active slots rounded up to a multiple of 4 (M <= 10)
// LDS layouts (MI355X_MICROARCH.md LDS table: ds_read_b128 serves lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... -- lanes c16 and grp mix inside a group, so a plain padded stride cannot be
// conflict-free for both):
//  Gs: one position's [slot][c] block is 96 elements (48 dwords, no pad); slot a of position pos sits at
//      a ^ ((pos >> 1) & 3) within its 4-slot group.  A-fragment reads (16 consecutive positions x 4 k-chunks)
//      and the staging ds_write_b128s are then bank-conflict-free for every base position (the previous
//      52-dword padded stride cost 2x on the reads: 3.9 conflicts per LDS instruction in r2_s3_pmc_mem.md).
//  Bs: row n of a k-step is 32 elements (no pad) with k-chunk q at q ^ ((n >> 1) & 3): conflict-free reads.
#define DG_PSTR (DG_NSMAX * 8)
DEVI int dg_swz(int i) { return (i >> 1) & 3; }
template <class G>
struct DGM {
  static constexpr int S = G::S;
  static constexpr int NA = (G::KH + S - 1) / S;            // taps per axis and class
  static constexpr int NTAP = NA * NA;
  static constexpr int NI = (G::HIN + S - 1) / S, NJ = (G::WIN + S - 1) / S;
  static constexpr int NSP = NI * NJ;                       // superpixels per sample
  static constexpr int NRT = (NSP + 15) / 16;               // row tiles
  static constexpr int NN = 8 * S * S;                      // real N
  static constexpr int NT = (NN + 15) / 16;                 // n tiles
  static constexpr int KSMAX = NTAP * DG_NSMAX / 4;         // 32-wide k-steps at 12 slots
};

// OT = float, or bf16_t for the first layer's input gradient (read only by the slab wgrad, which rounds it to
// bf16 for its MFMAs anyway): half of the largest activation-gradient stream of the update (1.48 GB fp32 at
// the bench shape) is never written or re-read.
// GT = float, or bf16_t when this layer's output gradient was itself stored in bf16 by the next layer's dgrad.
template <class G, typename OT = float, typename GT = float>
__global__ __launch_bounds__(256, 2) void conv_dgrad_mfma(const GT* __restrict__ Gr, const uint8_t* __restrict__ bits,
                                                          const float* __restrict__ flat, long w_off, int chunk,
                                                          const int* __restrict__ act_idx,
                                                          const int* __restrict__ act_cnt, int layer, int L, int M,
                                                          int P, int E, int T, long bits_rows, float g_scale,
                                                          OT* __restrict__ dX, int samples_per_wg) {
  using D = DGM<G>;
  constexpr int S = D::S;
  // [pos][slot (swizzled)][c], plus one zeroed block read by out-of-image taps
  __shared__ __attribute__((aligned(16))) bf16_t Gs[(G::HOWO + 1) * DG_PSTR];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[D::KSMAX * D::NT * 16 * 32];   // [ks][n][k (32), swizzled]
  __shared__ int mods[MAXM_F];
  constexpr int NTAPP = (D::NTAP + 3) & ~3;
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
  if (tid < MAXM_F) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
  __syncthreads();
  const int ns4 = (cnt + 3) >> 2;                  // 32-wide k-steps per tap
  const int KS = D::NTAP * ns4;
  // B[k][n]: k = (tap*ns4*4 + a)*8 + c, n = (ph*S + pw)*8 + ci  ->  W_a[kh][kw][ci][c]
  for (int it = tid; it < KS * D::NT * 16 * 4; it += 256) {
    const int kk8 = it & 3, rest = it >> 2;        // 8-wide k chunk within the step
    const int n = rest % (D::NT * 16), ks = rest / (D::NT * 16);
    const int tap = ks / ns4, a = (ks - tap * ns4) * 4 + kk8;
    const int ta = tap / D::NA, tb = tap - ta * D::NA;
    const int cls = n >> 3, ci = n & 7, ph = cls / S, pw = cls - ph * S;
    const int kh = ph + S * ta, kw = pw + S * tb;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (n < D::NN && a < cnt && kh < G::KH && kw < G::KW) {
      const float* wp = flat + w_off + (long)mods[a] * chunk + ((kh * G::KW + kw) * 8 + ci) * 8;
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = wp[c];
    }
    *reinterpret_cast<s8v*>(Bs + (ks * D::NT * 16 + n) * 32 + (kk8 ^ dg_swz(n)) * 8) = f32x8_to_bf16(v);
  }
  // staging role: one thread per output position (the G row is shared by all slots), all slots' bits
  const int nslot = ns4 * 4;
  constexpr int GIT = (G::HOWO + 255) / 256;
  // G rows: fp32 as two float4; bf16 kept raw (one uint4) and converted at staging time
  float4 g0r[sizeof(GT) == 2 ? 1 : GIT], g1r[sizeof(GT) == 2 ? 1 : GIT];
  uint4 graw[sizeof(GT) == 2 ? GIT : 1];
  uint8_t gbr[GIT][DG_NSMAX];
  auto load_sample = [&](int s) {
    const long sg = sample_global(p, s, E, PE, 0);
#pragma unroll
    for (int j = 0; j < GIT; ++j) {
      const int pos = tid + 256 * j;
      if (pos < G::HOWO) {
        const long go = sg * G::HOWO + pos;
        if constexpr (sizeof(GT) == 2) {
          graw[j] = *reinterpret_cast<const uint4*>(Gr + go * 8);
        } else {
          g0r[j] = *reinterpret_cast<const float4*>(Gr + go * 8);
          g1r[j] = *reinterpret_cast<const float4*>(Gr + go * 8 + 4);
        }
#pragma unroll
        for (int a = 0; a < DG_NSMAX; ++a) gbr[j][a] = a < cnt ? bits[(long)a * bits_rows + go] : (uint8_t)0;
      }
    }
  };
  // Sample-independent geometry, formed once per workgroup in two small LDS tables instead of once per sample
  // in registers (that per-sample index math was ~3/4 of this kernel's VALU work):
  //   atap[sp][tap]: LDS element offset of the A fragment of superpixel row sp and tap for k-chunk 0, with the
  //             position's swizzle in bits 3-4 (position blocks are 96 elements, so those bits are free): the
  //             lane's k-chunk grp is then one XOR (grp << 3).  Out-of-image taps point at the zero block HOWO.
  //   etab[sp]: epilogue superpixel sp -> dX offset S*(io*WIN + jo)*8, bit 14 / 15 set when class offset
  //             ph = 1 / pw = 1 stays inside the image; 0xFFFF past the last superpixel
  static_assert(S <= 2, "dgrad class limits are packed for strides 1 and 2");
  static_assert((G::HOWO + 1) * DG_PSTR < (1 << 16) && DG_PSTR % 32 == 0, "atap offset / swizzle fields");
  static_assert((S * (D::NI - 1) * G::WIN + S * (D::NJ - 1)) * 8 < (1 << 14), "etab offset field");
  for (int sp = tid; sp < D::NRT * 16; sp += 256) {
    const int ii = sp / D::NJ, jj = sp - ii * D::NJ;
#pragma unroll
    for (int tap = 0; tap < NTAPP; ++tap) {
      const int ta = tap / D::NA, tb = tap - ta * D::NA;
      const int oh = ii - ta, ow = jj - tb;
      const bool ok = tap < D::NTAP && sp < D::NSP && oh >= 0 && oh < G::HO && ow >= 0 && ow < G::WO;
      const int apos = ok ? oh * G::WO + ow : G::HOWO;
      atap[sp * NTAPP + tap] = (uint16_t)(apos * DG_PSTR + (dg_swz(apos) << 3));
    }
    etab[sp] = sp < D::NSP ? (uint16_t)((S * ii * G::WIN + S * jj) * 8 | ((S * ii + 1 < G::HIN) << 14) |
                                        ((S * jj + 1 < G::WIN) << 15))
                           : (uint16_t)0xFFFF;
  }
  for (int i = tid; i < DG_PSTR; i += 256) Gs[G::HOWO * DG_PSTR + i] = 0;
  // the lane's columns n = nt*16 + c16 -> (ph*WIN + pw)*8 + ci and its class offsets (ph, pw)
  int nofs[D::NT], nph[D::NT], npw[D::NT];
#pragma unroll
  for (int nt = 0; nt < D::NT; ++nt) {
    const int n = nt * 16 + c16;
    const int cls = n >> 3, ci = n & 7;
    nph[nt] = n < D::NN ? cls / S : 9;            // 9: padding column, never stored
    npw[nt] = cls - (cls / S) * S;
    nofs[nt] = ((cls / S) * G::WIN + npw[nt]) * 8 + ci;
  }
  load_sample(s_beg);
  for (int s = s_beg; s < s_end; ++s) {
    __syncthreads();                               // previous sample's LDS reads done
#pragma unroll
    for (int j = 0; j < GIT; ++j) {
      const int pos = tid + 256 * j;
      if (pos < G::HOWO) {
        if (sizeof(GT) == 2 && g_scale == 1.f) {
          // bf16 G, unit scale: mask the raw bf16 words with the ReLU bits directly (v_bfe_i32 sign-extends a
          // bit to 0 / ~0, v_bfi merges the two halves) -- 4 VALU per channel pair instead of unpack, select,
          // repack
          const uint32_t u[4] = {graw[j].x, graw[j].y, graw[j].z, graw[j].w};
#pragma unroll
          for (int a = 0; a < DG_NSMAX; ++a) {
            if (a < nslot) {
              const uint32_t b = gbr[j][a];
              uint4 o;
              uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)b, 2 * e, 1);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)b, 2 * e + 1, 1);
                ow[e] = u[e] & ((lo & 0xFFFFu) | (hi & 0xFFFF0000u));
              }
              *reinterpret_cast<uint4*>(Gs + pos * DG_PSTR + (a ^ dg_swz(pos)) * 8) = o;
            }
          }
          continue;
        }
        float gg[8];
        if constexpr (sizeof(GT) == 2) {
          const uint32_t u[4] = {graw[j].x, graw[j].y, graw[j].z, graw[j].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gg[2 * e] = __uint_as_float(u[e] << 16) * g_scale;
            gg[2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u) * g_scale;
          }
        } else {
          gg[0] = g0r[j].x * g_scale; gg[1] = g0r[j].y * g_scale; gg[2] = g0r[j].z * g_scale;
          gg[3] = g0r[j].w * g_scale; gg[4] = g1r[j].x * g_scale; gg[5] = g1r[j].y * g_scale;
          gg[6] = g1r[j].z * g_scale; gg[7] = g1r[j].w * g_scale;
        }
#pragma unroll
        for (int a = 0; a < DG_NSMAX; ++a) {
          if (a < nslot) {
            const int b = (int)gbr[j][a];
            float m[8];
#pragma unroll
            for (int c = 0; c < 8; ++c)
              m[c] = __uint_as_float(__float_as_uint(gg[c]) & (uint32_t)__builtin_amdgcn_sbfe(b, c, 1));
            *reinterpret_cast<s8v*>(Gs + pos * DG_PSTR + (a ^ dg_swz(pos)) * 8) = f32x8_to_bf16(m);
          }
        }
      }
    }
    __syncthreads();
    if (s + 1 < s_end) load_sample(s + 1);
    const long sg = sample_global(p, s, E, PE, 0);
    OT* __restrict__ dXs = dX + sg * (long)(G::HIN * G::WIN * 8);
    for (int rt = w; rt < D::NRT; rt += 4) {
      const uint16_t* tp = atap + (rt * 16 + c16) * NTAPP;
      f4v acc[D::NT];
#pragma unroll
      for (int nt = 0; nt < D::NT; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
      // k = (tap, slot group): the tap loop is compile-time (no per-step divisions by the runtime slot count --
      // they made this kernel SALU-bound); the A address of a tap is one table entry XOR the lane's k-chunk
#pragma unroll
      for (int tap = 0; tap < D::NTAP; ++tap) {
        const bf16_t* ap = Gs + ((int)tp[tap] ^ (grp << 3));
        const bf16_t* bp = Bs + (tap * ns4 * D::NT * 16 + c16) * 32 + (grp ^ dg_swz(c16)) * 8;
        for (int a4 = 0; a4 < ns4; ++a4) {
          const s8v af = *reinterpret_cast<const s8v*>(ap + a4 * 32);
#pragma unroll
          for (int nt = 0; nt < D::NT; ++nt) {
            const s8v bf = *reinterpret_cast<const s8v*>(bp + (a4 * D::NT * 16 + nt * 16) * 32);
            acc[nt] = mfma16(af, bf, acc[nt]);
          }
        }
      }
      // epilogue: row (superpixel) = rt*16 + 4*grp + r, n = nt*16 + c16 -> pixel (S*io + ph, S*jo + pw), map ci
      // 4 consecutive superpixel entries of this lane's epilogue rows: one 8-byte LDS read
      const uint2 e4 = *reinterpret_cast<const uint2*>(etab + rt * 16 + 4 * grp);
      const uint32_t ev[4] = {e4.x & 0xFFFFu, e4.x >> 16, e4.y & 0xFFFFu, e4.y >> 16};
#pragma unroll
      for (int nt = 0; nt < D::NT; ++nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t v = ev[r];
          // ph / pw are 0 or 1 (S <= 2): a class offset of 1 needs the in-image bit; 0xFFFF = no superpixel
          const bool okh = nph[nt] == 0 || (nph[nt] == 1 && ((v >> 14) & 1u));
          const bool okw = npw[nt] == 0 || ((v >> 15) & 1u);
          if (v != 0xFFFFu && okh && okw) {
            if constexpr (sizeof(OT) == 2) dXs[(int)(v & 0x3FFFu) + nofs[nt]] = f2bf(acc[nt][r]);
            else dXs[(int)(v & 0x3FFFu) + nofs[nt]] = acc[nt][r];
          }
        }
      }
    }
  }
}

template <class G, typename OT = float, typename GT = float>
static int dgrad_mfma_t(const GT* Gr, const void* bits, const float* flat, long w_off, int chunk, const int* ai,
                        const int* ac, int layer, int L, int M, int P, int E, int T, long br, float gs, OT* dX,
                        hipStream_t st) {
  const int nsamp = T * E;
  int spw = (nsamp + 31) / 32;                     // ~32 workgroups per path
  if (spw < 2) spw = 2;
  dim3 grid((unsigned)((nsamp + spw - 1) / spw), P);
  conv_dgrad_mfma<G, OT, GT><<<grid, 256, 0, st>>>(Gr, (const uint8_t*)bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E,
                                               T, br, gs, dX, spw);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
static int FWD_NT = 4;         // 32-row tiles per wave in conv_fwd_fast (4 -> 512 rows per workgroup); the uint8
                               // first layer uses twice as many (capped at 16): conv1 85.3 -> 82.6 us per step at 8,
                               // while conv2 / conv3 lose at 8 (18.0 -> 22.6, 14.8 -> 20.7 us: too few workgroups)
// uint8 first layer: fp16-offset MFMA operands (1 v_perm per 2 pixels) instead of u8 -> f32 -> bf16 converts.
// Off only for A/B runs and for the exact-equality tests against the bf16 alternative kernels.
static int F16_FWD = 1;
static int WGRAD_PF = 2;       // register sets of slab-wgrad loads in flight (1 or 2; 2: 1617 -> 1464 us conv1)

template <class G, int NT, bool RING = false>
static void fwd_launch(const void* X, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                       int chunk, const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, int t0,
                       long br, float is, float os, hipStream_t st, const uint8_t* fcv = nullptr,
                       int nslots = 0, const float* hcorr = nullptr) {
  const long rows = (long)T * E * G::HOWO;
  dim3 grid((unsigned)((rows + NT * 128 - 1) / (NT * 128)), P);
  if constexpr (G::U8) {
    if (hcorr) {
      conv_fwd_fast<G, NT, RING, true><<<grid, 256, 0, st>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat,
                                                             bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br,
                                                             is, os, fcv, nslots, hcorr);
      return;
    }
  }
  conv_fwd_fast<G, NT, RING, false><<<grid, 256, 0, st>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat,
                                                          bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is,
                                                          os, fcv, nslots, nullptr);
}

template <class G>
static int fwd_t(const void* X, void* Y, void* bits, const void* Wc, const float* flat, long bias_off, int chunk,
                 const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, int t0, long br,
                 float is, float os, hipStream_t st, const float* hcorr = nullptr) {
  const int nt = G::U8 ? (FWD_NT >= 8 ? 16 : 2 * FWD_NT) : FWD_NT;
  if (nt >= 16)
    fwd_launch<G, 16>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st,
                      nullptr, 0, hcorr);
  else if (nt >= 8)
    fwd_launch<G, 8>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st,
                     nullptr, 0, hcorr);
  else if (nt >= 4)
    fwd_launch<G, 4>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st,
                     nullptr, 0, hcorr);
  else
    fwd_launch<G, 2>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st,
                     nullptr, 0, hcorr);
  return (int)hipGetLastError();
}

template <class G>
static int wgrad_t(const void* X, const float* Gr, const void* bits, float* grad, long w_off, long b_off, int chunk,
                   const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, long br, float is,
                   float gs, hipStream_t st) {
  const long rows = (long)T * E * G::HOWO;
  // 16 chunks per path: P*16 workgroups of 512 threads, whole 32-row stages
  long rpc = (rows + 15) / 16;
  rpc = (rpc + WG_RB - 1) / WG_RB * WG_RB;
  if (rpc < WG_RB * 4) rpc = WG_RB * 4;
  dim3 grid((unsigned)((rows + rpc - 1) / rpc), P);
  conv_wgrad_fast<G><<<grid, WG_NT, 0, st>>>(X, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai, ac, layer, L,
                                           M, P, E, T, br, (int)rpc, is, gs);
  return (int)hipGetLastError();
}

template <class G>
static int fwd_img_t(const void* X, void* Y, void* bits, const void* Wc, const float* flat, long bias_off, int chunk,
                     const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, int t0, long br,
                     float is, float os, hipStream_t st) {
  dim3 grid((unsigned)(2 * T * E), P);
  conv_fwd_img<G><<<grid, 256, 0, st>>>((const uint8_t*)X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat,
                                        bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os);
  return (int)hipGetLastError();
}

template <class G, int OB>
static int fwd_slab_t(const void* X, void* Y, void* bits, const void* Wc, const float* flat, long bias_off, int chunk,
                      const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, int t0, long br,
                      float is, float os, hipStream_t st) {
  using SB = Slab<G, OB>;
  const long units = (long)T * E * SB::NB;
  long upw = (units + 15) / 16;                 // ~16 workgroups per path
  if (upw < 4) upw = 4;
  dim3 grid((unsigned)((units + upw - 1) / upw), P);
  conv_fwd_slab<G, OB><<<grid, 256, 0, st>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat, bias_off, chunk,
                                             ai, ac, layer, L, M, P, E, T, t0, br, (int)upw, is, os);
  return (int)hipGetLastError();
}

template <class G, int OB, bool RING = false, typename GT = float>
static int wgrad_slab_t(const void* X, const GT* Gr, const void* bits, float* grad, long w_off, long b_off,
                        int chunk, const int* ai, const int* ac, int layer, int L, int M, int P, int E, int T, long br,
                        float is, float gs, hipStream_t st, const uint8_t* fcv = nullptr, int nslots = 0) {
  using SB = Slab<G, OB>;
  const long units = (long)T * E * SB::NB;
  // ~24 workgroups per path (>= 1.5K workgroups at P=64), at least 8 units each
  long upw = (units + 23) / 24;
  if (upw < 8) upw = 8;
  dim3 grid((unsigned)((units + upw - 1) / upw), P);
  if (WGRAD_PF >= 2)
    conv_wgrad_slab<G, OB, 2, RING, GT><<<grid, 256, 0, st>>>(X, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai,
                                                          ac, layer, L, M, P, E, T, br, (int)upw, is, gs, fcv, nslots);
  else
    conv_wgrad_slab<G, OB, 1, RING, GT><<<grid, 256, 0, st>>>(X, Gr, (const uint8_t*)bits, grad, w_off, b_off, chunk, ai,
                                                          ac, layer, L, M, P, E, T, br, (int)upw, is, gs, fcv, nslots);
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

static int SLAB_WGRAD = 1;
static int DGRAD_MFMA = 1;
// measured slower than conv_fwd_fast at the rollout shape (2.28M vs 2.81M frames/s end to end): off by default
static int IMG_FWD = 0;
static int WGRAD_OB = 2;      // output rows per slab-wgrad stage for the first layer (2 or 3)
// The slab forward streams one band per barrier and is latency-bound at rollout batch sizes
// (rocprof: 451 us vs 128 us/step for conv_fwd_fast): kept for shapes/batches where it wins, off by default.
static int SLAB_FWD = 0;

extern "C" {
void fast_conv_set_slab(int on) { SLAB_WGRAD = on; }
void fast_conv_set_slab_fwd(int on) { SLAB_FWD = on; }
void fast_conv_set_dgrad_mfma(int on) { DGRAD_MFMA = on; }
void fast_conv_set_img_fwd(int on) { IMG_FWD = on; }
void fast_conv_set_wgrad_ob(int ob) { WGRAD_OB = ob; }
void fast_conv_set_fwd_nt(int nt) { FWD_NT = nt; }
void fast_conv_set_wgrad_pf(int pf) { WGRAD_PF = pf; }
void fast_conv_set_f16_fwd(int on) { F16_FWD = on; }

// return 1 if handled by a fast kernel, 0 if the shape is not specialised, <0 on error
// uint8 layers: Wc must be the fp16 weight copy and hcorr[M*8] its per-column sums (launch_refresh_weights_f16);
// the img / slab experiments still take the bf16 copy in Wc_bf16
int fast_conv_fwd(const void* X, int u8in, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                  int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH,
                  int KW, int S, int P, int E, int T, int t0, long br, float is, float os, const float* hcorr,
                  const void* Wc_bf16, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      P <= 0 || E <= 0 || T <= 0 || br <= 0 || u8in < 0 || bias_off < 0 || layer < 0 || t0 < 0) return -22;
  if (M > 2 * NCT) return 0;
  if (u8in && (!F16_FWD || !hcorr)) {      // bf16 operands: the bf16 weight copy, no offset correction
    Wc = Wc_bf16;
    hcorr = nullptr;
  }
#define FWD(Gx)                                                                                              \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, u8in)) {                                                        \
    if ((E * Gx::HOWO) % 16) return -2;                                                                      \
    const int rc = fwd_t<Gx>(X, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os, st, \
                             hcorr);                                                                         \
    return rc ? -rc : 1;                                                                                     \
  }
  if (IMG_FWD && is_shape<C1>(Hin, Win, Cin, KH, KW, S, u8in)) {
    const int rc = fwd_img_t<C1>(X, Y, bits, Wc_bf16, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is,
                                 os, st);
    return rc ? -rc : 1;
  }
  if (SLAB_FWD && is_shape<C1>(Hin, Win, Cin, KH, KW, S, u8in)) {
    const int rc = fwd_slab_t<C1, 2>(X, Y, bits, Wc_bf16, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br,
                                     is, os, st);
    return rc ? -rc : 1;
  }
  FWD(C1) FWD(C2) FWD(C3)
#undef FWD
  return 0;
}

int fast_conv_wgrad(const void* X, int u8in, const float* Gr, const void* bits, float* grad, long w_off, long b_off,
                    int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win, int Cin,
                    int KH, int KW, int S, int P, int E, int T, long br, float is, float gs, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      P <= 0 || E <= 0 || T <= 0 || br <= 0 || u8in < 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (M > 2 * NCT) return 0;
#define WG(Gx)                                                                                                 \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, u8in)) {                                                          \
    const int rc = wgrad_t<Gx>(X, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is, gs, st); \
    return rc ? -rc : 1;                                                                                       \
  }
  if (SLAB_WGRAD && is_shape<C1>(Hin, Win, Cin, KH, KW, S, u8in)) {
    int rc;
    if (WGRAD_OB == 3)
      rc = wgrad_slab_t<C1, 3>(X, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is, gs, st);
    else
      rc = wgrad_slab_t<C1, 2>(X, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is, gs, st);
    return rc ? -rc : 1;
  }
  if (SLAB_WGRAD && is_shape<C2>(Hin, Win, Cin, KH, KW, S, u8in)) {
    const int rc = wgrad_slab_t<C2, 7>(X, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is, gs,
                                       st);
    return rc ? -rc : 1;
  }
  WG(C1) WG(C2) WG(C3)
#undef WG
  return 0;
}

// First layer on the frame ring (160x120 uint8 planes, 4 channels, 8x8/s4): fc = first valid
// channel per (step, sample) [T+1][P*E] uint8.  Wc must be channel-major (launch_refresh_weights_cmajor).
// frames [P*E][nslots][160*120] uint8 with nslots >= t0 + T + 3 (rollout: T_roll + 4 slots)
// Wc: channel-major fp16 weights with hcorr (fp16-offset path) or channel-major bf16 with hcorr = null
int fast_conv1_ring_fwd(const void* frames, const void* fc, void* Y, void* bits, const void* Wc, const float* flat,
                        long bias_off, int chunk, const int* ai, const int* ac, int layer, int L, int M, int P, int E,
                        int T, int t0, int nslots, long br, float is, float os, const float* hcorr,
                        const void* Wc_bf16, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || P <= 0 || E <= 0 || T <= 0 || nslots <= 0 || br <= 0 || bias_off < 0 ||
      layer < 0 || t0 < 0) return -22;
  if (M > 2 * NCT) return -22;
  if ((E * C1::HOWO) % 16) return -2;
  if (nslots < t0 + T + 3) return -33;
  if (!F16_FWD || !hcorr) {
    Wc = Wc_bf16;
    hcorr = nullptr;
  }
  const uint8_t* f = (const uint8_t*)fc;
  if (FWD_NT >= 8)
    fwd_launch<C1, 8, true>(frames, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os,
                            st, f, nslots, hcorr);
  else
    fwd_launch<C1, 4, true>(frames, Y, bits, Wc, flat, bias_off, chunk, ai, ac, layer, L, M, P, E, T, t0, br, is, os,
                            st, f, nslots, hcorr);
  return (int)hipGetLastError();
}

int fast_conv1_ring_wgrad(const void* frames, const void* fc, const float* Gr, const void* bits, float* grad,
                          long w_off, long b_off, int chunk, const int* ai, const int* ac, int layer, int L, int M,
                          int P, int E, int T, int nslots, long br, float is, float gs, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || P <= 0 || E <= 0 || T <= 0 || nslots <= 0 || br <= 0 || w_off < 0 ||
      b_off < 0 || layer < 0) return -22;
  if (M > 2 * NCT) return -22;
  if (nslots < T + 3) return -33;
  if ((long)T * E / 24 + 3 > 1024) return -34;   // samples per workgroup vs the LDS first-channel table
  const uint8_t* f = (const uint8_t*)fc;
  if (WGRAD_OB == 3)
    return wgrad_slab_t<C1, 3, true>(frames, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is,
                                     gs, st, f, nslots);
  return wgrad_slab_t<C1, 2, true>(frames, Gr, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E, T, br, is,
                                   gs, st, f, nslots);
}

int fast_conv_dgrad(const float* Gr, const void* bits, const float* flat, long w_off, int chunk, const int* ai,
                    const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH, int KW, int S, int P,
                    int E, int T, long br, float gs, float* dX, hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      P <= 0 || E <= 0 || T <= 0 || br <= 0 || w_off < 0 || layer < 0) return -22;
#define DG(Gx)                                                                                          \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, 0)) {                                                      \
    const int rc = dgrad_t<Gx>(Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, st); \
    return rc ? -rc : 1;                                                                                \
  }
  if (M <= 10 && DGRAD_MFMA) {
    if (is_shape<C2>(Hin, Win, Cin, KH, KW, S, 0)) {
      const int rc = dgrad_mfma_t<C2>(Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, st);
      return rc ? -rc : 1;
    }
    if (is_shape<C3>(Hin, Win, Cin, KH, KW, S, 0)) {
      const int rc = dgrad_mfma_t<C3>(Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, gs, dX, st);
      return rc ? -rc : 1;
    }
  }
  DG(C2) DG(C3)
#undef DG
  return 0;
}

// bf16 activation gradients between the conv layers: the MFMA dgrad reads its G and writes its dX in fp32
// or bf16 (flags), the slab wgrad reads a bf16 G (reference geometries only: 160x120x4 / 8x8 s4,
// 39x29x8 / 4x4 s2, 18x13x8 / 3x3 s1).  1: handled, 0: not specialised (the caller must then keep that
// gradient in fp32), <0: error.
int fast_conv_dgrad_bf16(const void* Gr, int g_bf16, const void* bits, const float* flat, long w_off, int chunk,
                         const int* ai, const int* ac, int layer, int L, int M, int Hin, int Win, int Cin, int KH,
                         int KW, int S, int P, int E, int T, long br, float gs, void* dX, int dx_bf16,
                         hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      P <= 0 || E <= 0 || T <= 0 || br <= 0 || g_bf16 < 0 || w_off < 0 || layer < 0 || dx_bf16 < 0) return -22;
  if (M > 10 || !DGRAD_MFMA) return 0;
#define DGB(Gx)                                                                                               \
  if (is_shape<Gx>(Hin, Win, Cin, KH, KW, S, 0)) {                                                            \
    int rc;                                                                                                   \
    if (g_bf16 && dx_bf16)                                                                                    \
      rc = dgrad_mfma_t<Gx, bf16_t, bf16_t>((const bf16_t*)Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, \
                                            br, gs, (bf16_t*)dX, st);                                         \
    else if (g_bf16)                                                                                          \
      rc = dgrad_mfma_t<Gx, float, bf16_t>((const bf16_t*)Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, \
                                           br, gs, (float*)dX, st);                                           \
    else if (dx_bf16)                                                                                         \
      rc = dgrad_mfma_t<Gx, bf16_t, float>((const float*)Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, \
                                           br, gs, (bf16_t*)dX, st);                                          \
    else                                                                                                      \
      rc = dgrad_mfma_t<Gx, float, float>((const float*)Gr, bits, flat, w_off, chunk, ai, ac, layer, L, M, P, E, T, br, \
                                          gs, (float*)dX, st);                                                \
    return rc ? -rc : 1;                                                                                      \
  }
  DGB(C2) DGB(C3)
#undef DGB
  return 0;
}

int fast_conv_wgrad_bf16g(const void* X, int u8in, const void* Gr, const void* bits, float* grad, long w_off,
                          long b_off, int chunk, const int* ai, const int* ac, int layer, int L, int M, int Hin,
                          int Win, int Cin, int KH, int KW, int S, int P, int E, int T, long br, float is, float gs,
                          hipStream_t st) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      P <= 0 || E <= 0 || T <= 0 || br <= 0 || u8in < 0 || w_off < 0 || b_off < 0 || layer < 0) return -22;
  if (M > 2 * NCT || !SLAB_WGRAD) return 0;
  const bf16_t* g = (const bf16_t*)Gr;
  if (is_shape<C2>(Hin, Win, Cin, KH, KW, S, u8in)) {
    const int rc = wgrad_slab_t<C2, 7, false, bf16_t>(X, g, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M, P, E,
                                                       T, br, is, gs, st);
    return rc ? -rc : 1;
  }
  if (!is_shape<C1>(Hin, Win, Cin, KH, KW, S, u8in)) return 0;
  const int rc = WGRAD_OB == 3
                     ? wgrad_slab_t<C1, 3, false, bf16_t>(X, g, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M,
                                                          P, E, T, br, is, gs, st)
                     : wgrad_slab_t<C1, 2, false, bf16_t>(X, g, bits, grad, w_off, b_off, chunk, ai, ac, layer, L, M,
                                                          P, E, T, br, is, gs, st);
  return rc ? -rc : 1;
}
}
