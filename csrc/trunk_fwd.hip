// PathNet trunk forward on CDNA4 MFMA.
//
// Reference graph (game_ac_network.py:182-201 / 378-426): every module of a
// layer is computed densely, ReLU'd, multiplied by its 0/1 path mask and the
// M results are summed.  Here only the ACTIVE modules of each path are
// computed: a workgroup owns a tile of rows of ONE path, reads that path's
// compacted module list (act_idx/act_cnt) and runs an indexed grouped GEMM
// over those modules; bias + ReLU + the per-layer module SUM happen in the
// epilogue (in registers + one lane shuffle), and the ReLU sign of every
// (row, module, channel) is kept as one bit for the backward pass (ballot).
//
// conv layers: implicit GEMM, rows = (sample, oh, ow), k = (kh, kw, cin),
//   columns = active-module x 8 output maps (two modules per 16-wide MFMA
//   tile).  The uint8 frame stack is read directly (exact in bf16); the
//   1/255 of game_state.py:49-50 is folded into the epilogue (in_scale).
// fc layers: grouped GEMM over active modules, 64x64 (or 32x64) tiles.
#include "common.h"

#define FWD_BM 64
#define MAXM 16          // max modules per layer supported by the kernels
#define MAX_CT 8         // max 16-wide column tiles per conv layer (= 16 modules of 8 maps)

struct ConvGeom {
  int Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP;
};

template <bool U8IN>
DEVI s8v load_a8(const void* X, long off) {
  s8v r;
  if constexpr (U8IN) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(X) + off);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // u8 -> f32 -> bf16 is exact for 0..255 (8 significant bits)
      r[j] = (short)(__float_as_uint((float)((v.x >> (8 * j)) & 0xFFu)) >> 16);
      r[j + 4] = (short)(__float_as_uint((float)((v.y >> (8 * j)) & 0xFFu)) >> 16);
    }
  } else {
    r = *reinterpret_cast<const s8v*>(reinterpret_cast<const bf16_t*>(X) + off);
  }
  return r;
}

// ---------------------------------------------------------------------------
// conv forward.  grid = (ceil(T*E*Ho*Wo / 64), P), block 256.
// X  : [T'][P*E][Hin*Win*Cin] (uint8 or bf16), Y: [T'][P*E][Ho*Wo*8] bf16
// bits: [M][bits_rows] uint8 (bit c = ReLU>0 of map c of that module slot)
// Wc : [M][8][KP] bf16 (k contiguous, zero padded)
// ---------------------------------------------------------------------------
template <bool U8IN>
__global__ __launch_bounds__(256) void conv_fwd_kernel(
    const void* __restrict__ X, bf16_t* __restrict__ Y, uint8_t* __restrict__ bits,
    const bf16_t* __restrict__ Wc, const float* __restrict__ flat, long bias_off, int chunk,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
    ConvGeom g, int P, int E, int T, int t0, long bits_rows, float in_scale, float out_scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.y;
  const int cnt = act_cnt[p * L + layer];
  const int nct = (cnt + 1) >> 1;
  const int ncol = nct * 16;
  const int KPs = g.KP + 8;                       // padded LDS row (bank spread)
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem);   // [ncol][KPs]
  const int ncap = ((M + 1) >> 1) * 16;           // column capacity (all modules active)
  int* koff = reinterpret_cast<int*>(smem + (size_t)ncap * KPs * 2);           // [KP/8]
  float* bias_s = reinterpret_cast<float*>(koff + g.KP / 8);                   // [ncap]
  int* mods = reinterpret_cast<int*>(bias_s + ncap);                           // [MAXM]

  const int tid = threadIdx.x;
  if (tid < MAXM) mods[tid] = tid < cnt ? act_idx[(p * L + layer) * M + tid] : 0;
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
  __syncthreads();
  const int kvec = g.KP / 8;
  for (int i = tid; i < ncol * kvec; i += 256) {
    const int col = i / kvec, kc = i - col * kvec;
    const int slot = col >> 3, c = col & 7;
    s8v v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (slot < cnt) v = *reinterpret_cast<const s8v*>(Wc + ((long)(mods[slot] * 8 + c)) * g.KP + kc * 8);
    *reinterpret_cast<s8v*>(Ws + col * KPs + kc * 8) = v;
  }
  for (int i = tid; i < ncol; i += 256) {
    const int slot = i >> 3;
    bias_s[i] = slot < cnt ? flat[bias_off + (long)mods[slot] * chunk + (i & 7)] : 0.f;
  }
  __syncthreads();

  const int HoWo = g.Ho * g.Wo;
  const long Rtot = (long)T * E * HoWo;
  const int PE = P * E;
  const int w = tid >> 6, l = tid & 63;
  const long rbase = (long)blockIdx.x * FWD_BM + w * 16;
  if (rbase >= Rtot) return;

  // this lane's A row
  const long ra = rbase + (l & 15);
  const bool va = ra < Rtot;
  long xbase = 0;
  {
    const long rr = va ? ra : rbase;
    const int s = (int)(rr / HoWo);
    const int pos = (int)(rr - (long)s * HoWo);
    const int oh = pos / g.Wo, ow = pos - oh * g.Wo;
    const long sg = sample_global(p, s, E, PE, t0);
    xbase = sg * (long)(g.Hin * g.Win * g.Cin) + (long)(oh * g.S * g.Win + ow * g.S) * g.Cin;
  }
  f4v acc[MAX_CT];
#pragma unroll
  for (int ct = 0; ct < MAX_CT; ++ct) acc[ct] = {0.f, 0.f, 0.f, 0.f};

  const int grp = l >> 4;
  for (int kk = 0; kk < g.KP; kk += 32) {
    const int k0 = kk + 8 * grp;
    const int off = koff[k0 >> 3];
    s8v a = {0, 0, 0, 0, 0, 0, 0, 0};
    if (va && off >= 0) a = load_a8<U8IN>(X, xbase + off);
#pragma unroll
    for (int ct = 0; ct < MAX_CT; ++ct) {
      if (ct < nct) {
        const s8v b = *reinterpret_cast<const s8v*>(Ws + (ct * 16 + (l & 15)) * KPs + k0);
        acc[ct] = mfma16(a, b, acc[ct]);
      }
    }
  }

  // epilogue: bias, ReLU, ReLU bits, module sum
  const int q = l >> 4, c16 = l & 15, h = c16 >> 3, ch = l & 7;
  float sum[4] = {0.f, 0.f, 0.f, 0.f};
  // global bit-row of rows rbase+4q .. +3 (4-aligned, never crosses a sample block: host asserts E*HoWo % 16 == 0)
  long grow4 = 0;
  {
    const long r4 = rbase + 4 * q;
    const int s = (int)(r4 / HoWo);
    const int pos = (int)(r4 - (long)s * HoWo);
    grow4 = sample_global(p, s, E, PE, t0) * HoWo + pos;
  }
#pragma unroll
  for (int ct = 0; ct < MAX_CT; ++ct) {
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
      if (ch == 0 && sv) *reinterpret_cast<uint32_t*>(bits + (long)slot * bits_rows + grow4) = word;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) sum[r] += __shfl_xor(sum[r], 8, 64);
  if (h == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = rbase + 4 * q + r;
      if (row < Rtot) {
        const int s = (int)(row / HoWo);
        const int pos = (int)(row - (long)s * HoWo);
        const long sg = sample_global(p, s, E, PE, t0);
        Y[(sg * HoWo + pos) * 8 + ch] = f2bf(sum[r] * out_scale);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fc forward (indexed grouped GEMM).  grid = (ceil(T*E/BM), Cout/64, P).
// X: [T'][P*E][ldx] bf16 (zero padded to ldx >= K, ldx % 8 == 0)
// Y: [T'][P*E][Cout] bf16;  bits16: [M][bits_rows][Cout/16] uint16
// Wc: [M][Cout][KP] bf16
// 4 waves as 2 (rows) x 2 (cols); wave tile (BM/2) x 32.
// ---------------------------------------------------------------------------
template <int BM>
__global__ __launch_bounds__(256) void fc_fwd_kernel(
    const bf16_t* __restrict__ X, int ldx, bf16_t* __restrict__ Y, uint16_t* __restrict__ bits,
    const bf16_t* __restrict__ Wc, const float* __restrict__ flat, long bias_off, int chunk,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
    int K, int KP, int Cout, int P, int E, int T, int t0, long bits_rows, float out_scale) {
  constexpr int RT = BM / 32;  // row tiles (16) per wave
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * BM + wr * (BM / 2);
  const int col0 = blockIdx.y * 64 + wc * 32;
  if (row0 >= Rtot || col0 >= Cout) return;
  const int grp = l >> 4, c16 = l & 15;

  // A rows for this lane
  long xrow[RT];
  bool xv[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const long r = row0 + i * 16 + c16;
    xv[i] = r < Rtot;
    xrow[i] = sample_global(p, (int)(xv[i] ? r : row0), E, PE, t0) * ldx;
  }
  float sum[RT][2][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[i][j][r] = 0.f;

  for (int a = 0; a < cnt; ++a) {
    const int mod = act_idx[(p * L + layer) * M + a];
    const bf16_t* Wm = Wc + (long)mod * Cout * KP;
    f4v acc[RT][2];
#pragma unroll
    for (int i = 0; i < RT; ++i) { acc[i][0] = {0.f, 0.f, 0.f, 0.f}; acc[i][1] = {0.f, 0.f, 0.f, 0.f}; }
    for (int kk = 0; kk < KP; kk += 32) {
      const int k0 = kk + 8 * grp;
      s8v av[RT];
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        av[i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
        if (xv[i] && k0 < K) av[i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const s8v b = *reinterpret_cast<const s8v*>(Wm + (long)(col0 + j * 16 + c16) * KP + k0);
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i][j] = mfma16(av[i], b, acc[i][j]);
      }
    }
    // epilogue of this module: bias + relu + bits + accumulate
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + j * 16 + c16;
      const float bb = flat[bias_off + (long)mod * chunk + col];
#pragma unroll
      for (int i = 0; i < RT; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r] + bb;
          const bool pos = v > 0.f;
          sum[i][j][r] += pos ? v : 0.f;
          const uint64_t bal = __ballot(pos);
          const long row = row0 + i * 16 + 4 * grp + r;
          if (c16 == 0 && row < Rtot) {
            const long sg = sample_global(p, (int)row, E, PE, t0);
            bits[((long)a * bits_rows + sg) * (Cout / 16) + (col0 + j * 16) / 16] =
                (uint16_t)((bal >> (16 * grp)) & 0xFFFFull);
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + i * 16 + 4 * grp + r;
      if (row < Rtot) {
        const long sg = sample_global(p, (int)row, E, PE, t0);
#pragma unroll
        for (int j = 0; j < 2; ++j) Y[sg * Cout + col0 + j * 16 + c16] = f2bf(sum[i][j][r] * out_scale);
      }
    }
}

// ---------------------------------------------------------------------------
// fc forward for the rollout (<= 32 rows per path): MODULE-PER-WAVE.
// grid = (ceil(T*E/32), Cout/64, P); wave w computes the full 32x64 tile for
// module slots w, w+4, ... (per-module bias+ReLU+bits in registers), the 4
// waves' module sums meet in LDS.  Each wave runs a register double-buffered
// K loop (next k-step's A/B fragments in flight during this step's 8 MFMAs),
// so a path's active modules stream their weights in parallel instead of one
// after another -- the per-step fc layers are latency-bound, not FLOP-bound.
// ---------------------------------------------------------------------------
//
// D = k-steps of A/B fragments in flight per wave.  The grid is one workgroup per (path, 64
// columns) -- one wave per SIMD -- so registers are free and a deep prefetch ring cuts the
// latency chain of the 44-step K loop (fc1: K = 1408) by D.
// NKS > 0: compile-time k-step count (fc1 / fc2 of the pixel trunk): the K loop is fully unrolled, so no
// loop back-edge makes the wait-count pass drain the register ring (it emitted vmcnt(0) at the back-edge
// of the rolled loop, which serialised one memory latency per D k-steps).
template <int RT, int D, int NKS = 0>
__global__ __launch_bounds__(256) void fc_fwd_mw_kernel(
    const bf16_t* __restrict__ X, int ldx, bf16_t* __restrict__ Y, uint16_t* __restrict__ bits,
    const bf16_t* __restrict__ Wc, const float* __restrict__ flat, long bias_off, int chunk,
    const int* __restrict__ act_idx, const int* __restrict__ act_cnt, int layer, int L, int M,
    int K, int KP, int Cout, int P, int E, int T, int t0, long bits_rows, float out_scale) {
  __shared__ float part[4][32][64 + 1];
  const int p = blockIdx.z;
  const int cnt = act_cnt[p * L + layer];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int grp = l >> 4, c16 = l & 15;
  const long Rtot = (long)T * E;
  const int PE = P * E;
  const long row0 = (long)blockIdx.x * 32;
  const int col0 = blockIdx.y * 64;
  long xrow[RT];
  bool xv[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const long r = row0 + i * 16 + c16;
    xv[i] = r < Rtot;
    xrow[i] = sample_global(p, (int)(xv[i] ? r : row0), E, PE, t0) * ldx;
  }
  float sum[RT][4][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[i][j][r] = 0.f;
  const int nwords = Cout / 16;
  // global sample rows of this lane's epilogue rows, once (not a runtime division by E per bit store)
  long sgb[RT][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long row = row0 + i * 16 + 4 * grp + r;
      sgb[i][r] = sample_global(p, (int)(row < Rtot ? row : row0), E, PE, t0);
    }
  for (int a = w; a < cnt; a += 4) {
    const int mod = act_idx[(p * L + layer) * M + a];
    const bf16_t* Wm = Wc + (long)mod * Cout * KP + (long)(col0 + c16) * KP + 8 * grp;
    f4v acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
    s8v an[D][RT], bn[D][4];
    // rows past Rtot read a valid row (their outputs are never stored); K padding (K < KP) reads zeros
    auto load = [&](s8v (&ad)[RT], s8v (&bd)[4], int kk) {
      const int k0 = kk + 8 * grp;
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if (K == KP) {
          ad[i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
        } else {
          ad[i] = (s8v){0, 0, 0, 0, 0, 0, 0, 0};
          if (k0 < K) ad[i] = *reinterpret_cast<const s8v*>(X + xrow[i] + k0);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) bd[j] = *reinterpret_cast<const s8v*>(Wm + (long)j * 16 * KP + kk);
    };
    auto mma = [&](const s8v (&ad)[RT], const s8v (&bd)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i][j] = mfma16(ad[i], bd[j], acc[i][j]);
    };
    // D-deep register ring WITHOUT copies: slot d's MFMAs issue, then the same registers are reloaded
    // with k-step s + d + D.  The main loop reloads unconditionally (no loop-carried conditional value,
    // which made the compiler copy the whole ring every step); the last < 2D k-steps are peeled.
    const int nks = NKS > 0 ? NKS : KP / 32;
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d < nks) load(an[d], bn[d], d * 32);
    int s = 0;
#pragma unroll
    for (; s + 2 * D <= nks; s += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        mma(an[d], bn[d]);
        load(an[d], bn[d], (s + d + D) * 32);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + d < nks) {
        mma(an[d], bn[d]);
        if (s + d + D < nks) load(an[d], bn[d], (s + d + D) * 32);
      }
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (s + D + d < nks) mma(an[d], bn[d]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bb = flat[bias_off + (long)mod * chunk + col0 + j * 16 + c16];
#pragma unroll
      for (int i = 0; i < RT; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r] + bb;
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
  // 256 threads: 32 rows x 64 cols -> 8 outputs each (one row, 8 consecutive cols)
  const int orow = tid >> 3, oc = (tid & 7) * 8;
  const long row = row0 + orow;
  if (orow < RT * 16 && row < Rtot) {
    const long sg = sample_global(p, (int)row, E, PE, t0);
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      o[c] = (part[0][orow][oc + c] + part[1][orow][oc + c] + part[2][orow][oc + c] + part[3][orow][oc + c]) *
             out_scale;
    *reinterpret_cast<s8v*>(Y + sg * Cout + col0 + oc) = f32x8_to_bf16(o);
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
#define FC_MW_D 4

extern "C" {

size_t conv_fwd_smem(int KP, int M) {
  if (KP <= 0 || M <= 0) return 0;
  const int ncap = ((M + 1) >> 1) * 16;
  return (size_t)ncap * (KP + 8) * 2 + (KP / 8) * 4 + ncap * 4 + MAXM * 4;
}

int launch_conv_fwd(const void* X, int u8in, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                    int chunk, const int* act_idx, const int* act_cnt, int layer, int L, int M, int Hin, int Win,
                    int Cin, int KH, int KW, int S, int Ho, int Wo, int K, int KP, int P, int E, int T, int t0,
                    long bits_rows, float in_scale, float out_scale, hipStream_t stream) {
  if (chunk <= 0 || L <= 0 || M <= 0 || Hin <= 0 || Win <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || S <= 0 ||
      Ho <= 0 || Wo <= 0 || K <= 0 || KP <= 0 || P <= 0 || E <= 0 || T <= 0 || bits_rows <= 0 || u8in < 0 ||
      bias_off < 0 || layer < 0 || t0 < 0) return -22;
  if (M > MAXM || KP % 32 != 0 || (E * Ho * Wo) % 16 != 0) return -1;
  ConvGeom g{Hin, Win, Cin, KH, KW, S, Ho, Wo, K, KP};
  const long rows = (long)T * E * Ho * Wo;
  dim3 grid((unsigned)((rows + FWD_BM - 1) / FWD_BM), P);
  const size_t sm = conv_fwd_smem(KP, M);
  if (u8in)
    conv_fwd_kernel<true><<<grid, 256, sm, stream>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat, bias_off,
                                                      chunk, act_idx, act_cnt, layer, L, M, g, P, E, T, t0, bits_rows,
                                                      in_scale, out_scale);
  else
    conv_fwd_kernel<false><<<grid, 256, sm, stream>>>(X, (bf16_t*)Y, (uint8_t*)bits, (const bf16_t*)Wc, flat,
                                                       bias_off, chunk, act_idx, act_cnt, layer, L, M, g, P, E, T, t0,
                                                       bits_rows, in_scale, out_scale);
  return (int)hipGetLastError();
}

int launch_fc_fwd(const void* X, int ldx, void* Y, void* bits, const void* Wc, const float* flat, long bias_off,
                  int chunk, const int* act_idx, const int* act_cnt, int layer, int L, int M, int K, int KP, int Cout,
                  int P, int E, int T, int t0, long bits_rows, float out_scale, hipStream_t stream) {
  if (ldx <= 0 || chunk <= 0 || L <= 0 || M <= 0 || K <= 0 || KP <= 0 || Cout <= 0 || P <= 0 || E <= 0 || T <= 0 ||
      bits_rows <= 0 || bias_off < 0 || layer < 0 || t0 < 0) return -22;
  if (M > MAXM || KP % 32 != 0 || Cout % 32 != 0 || ldx % 8 != 0) return -1;
  const long rows = (long)T * E;
  if (rows <= 32 && Cout % 64 == 0) {
    dim3 grid(1, Cout / 64, P);
#define FC_MW(RT_, NKS_)                                                                                       \
  fc_fwd_mw_kernel<RT_, FC_MW_D, NKS_><<<grid, 256, 0, stream>>>(                                            \
      (const bf16_t*)X, ldx, (bf16_t*)Y, (uint16_t*)bits, (const bf16_t*)Wc, flat, bias_off, chunk, act_idx,  \
      act_cnt, layer, L, M, K, KP, Cout, P, E, T, t0, bits_rows, out_scale)
    if (rows <= 16)
      FC_MW(1, 0);
    else if (KP == 1408)
      FC_MW(2, 44);          // fc1 of the pixel trunk (conv3 output 8 x 11 x 16)
    else if (KP == 256)
      FC_MW(2, 8);           // fc2 (256 -> 256)
    else
      FC_MW(2, 0);
#undef FC_MW
  } else if (rows <= 32) {
    dim3 grid((unsigned)((rows + 31) / 32), (Cout + 63) / 64, P);
    fc_fwd_kernel<32><<<grid, 256, 0, stream>>>((const bf16_t*)X, ldx, (bf16_t*)Y, (uint16_t*)bits,
                                                (const bf16_t*)Wc, flat, bias_off, chunk, act_idx, act_cnt, layer, L,
                                                M, K, KP, Cout, P, E, T, t0, bits_rows, out_scale);
  } else {
    dim3 grid((unsigned)((rows + 63) / 64), (Cout + 63) / 64, P);
    fc_fwd_kernel<64><<<grid, 256, 0, stream>>>((const bf16_t*)X, ldx, (bf16_t*)Y, (uint16_t*)bits,
                                                (const bf16_t*)Wc, flat, bias_off, chunk, act_idx, act_cnt, layer, L,
                                                M, K, KP, Cout, P, E, T, t0, bits_rows, out_scale);
  }
  return (int)hipGetLastError();
}
}
