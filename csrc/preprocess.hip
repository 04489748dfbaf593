// Standalone frame preprocessing for externally rendered RGB frames (SURVEY.md K15 + K16):
// reference game_state.py:41-50,66,78 -- cv2.cvtColor (fixed-point luma) + cv2.resize
// INTER_LINEAR 210x160 -> 160x120 (11-bit weights) + 4-deep frame stack, newest last.
// Bit-exact with envs/pong.py:preprocess_frames (the torch oracle).
//
// One workgroup per env: the 210x160 gray image is built ONCE in LDS from 12-byte RGB
// quads (4 pixels per thread-iteration), then every output pixel reads its 4 taps from LDS;
// the new frame is pushed into the uint32-per-pixel stack with 16-byte loads/stores
// ((in >> 8) | f << 24, or f * 0x01010101 where the episode just reset).
#include "common.h"

namespace pre {
constexpr int SH = 210, SW = 160, OH = 160, OW = 120;
}

__global__ __launch_bounds__(256) void rgb_stack_push_kernel(const uint8_t* __restrict__ rgb,
                                                             const uint32_t* __restrict__ obs_in,
                                                             uint32_t* __restrict__ obs_out,
                                                             const uint8_t* __restrict__ reset,
                                                             const int* __restrict__ tables, int wr, int wg, int wb) {
  using namespace pre;
  __shared__ int tab[8 * 160];
  __shared__ uint32_t gray[SH * SW / 4];
  const int env = blockIdx.x;
  for (int i = threadIdx.x; i < 8 * 160; i += 256) tab[i] = tables[i];
  const uint8_t* src = rgb + (long)env * SH * SW * 3;
  for (int q4 = threadIdx.x; q4 < SH * SW / 4; q4 += 256) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + q4 * 12);   // 4 RGB pixels = 12 bytes
    const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];
    const uint8_t b[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                           (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                           (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
    uint32_t wv = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int g = ((int)b[3 * e] * wr + (int)b[3 * e + 1] * wg + (int)b[3 * e + 2] * wb + 8192) >> 14;
      wv |= (uint32_t)g << (8 * e);
    }
    gray[q4] = wv;
  }
  __syncthreads();
  const uint8_t* g8 = reinterpret_cast<const uint8_t*>(gray);
  const bool rs = reset != nullptr && reset[env];
  const uint4* in4 = reinterpret_cast<const uint4*>(obs_in) + (long)env * (OH * OW / 4);
  uint4* out4 = reinterpret_cast<uint4*>(obs_out) + (long)env * (OH * OW / 4);
  for (int q = threadIdx.x; q < OH * OW / 4; q += 256) {
    const int y = q / (OW / 4), x0 = (q - y * (OW / 4)) * 4;
    const int ys0 = tab[0 * 160 + y], ys1 = tab[1 * 160 + y], cy0 = tab[2 * 160 + y], cy1 = tab[3 * 160 + y];
    uint32_t f4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = x0 + e;
      const int xs0 = tab[4 * 160 + x], xs1 = tab[5 * 160 + x], cx0 = tab[6 * 160 + x], cx1 = tab[7 * 160 + x];
      const int ra = g8[ys0 * SW + xs0] * cx0 + g8[ys0 * SW + xs1] * cx1;
      const int rb = g8[ys1 * SW + xs0] * cx0 + g8[ys1 * SW + xs1] * cx1;
      int v = (ra * cy0 + rb * cy1 + (1 << 21)) >> 22;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      f4[e] = (uint32_t)v;
    }
    uint4 o;
    if (rs) {
      o = make_uint4(f4[0] * 0x01010101u, f4[1] * 0x01010101u, f4[2] * 0x01010101u, f4[3] * 0x01010101u);
    } else {
      const uint4 i = in4[q];
      o = make_uint4((i.x >> 8) | (f4[0] << 24), (i.y >> 8) | (f4[1] << 24), (i.z >> 8) | (f4[2] << 24),
                     (i.w >> 8) | (f4[3] << 24));
    }
    out4[q] = o;
  }
}

extern "C" int launch_rgb_stack_push(const void* rgb, const void* obs_in, void* obs_out, const void* reset,
                                     const int* tables, int N, int wr, int wg, int wb, hipStream_t stream) {
  rgb_stack_push_kernel<<<N, 256, 0, stream>>>((const uint8_t*)rgb, (const uint32_t*)obs_in, (uint32_t*)obs_out,
                                               (const uint8_t*)reset, tables, wr, wg, wb);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Rectangle-list renderer + preprocessing + stack push for the pixel games whose logic runs in
// torch (envs/atari_games.py): each game emits its scene as [N][R][4] int16 rectangles
// (y0, x0, h, w; h*w == 0 = hidden) painted in order with one gray level per rectangle slot.
// One workgroup per env rasterises the scene into an LDS gray image (below), then resizes + pushes
// as above.
// Replaces N x R full-frame boolean mask ops of the torch renderer.
// ---------------------------------------------------------------------------
// Painter's order without a barrier per rectangle: thread t owns source row t (SH = 210 <= 256 threads) and walks
// the whole rectangle list (staged once in LDS) painting only its own row, so every pixel is written by one thread
// in list order.  (One barrier per visible rectangle cost 224 barriers per env for Alien: 260 us per step at 2048
// envs.)  RING: the resized frame goes to frames + env * frame_stride (one 19.2 KB plane of the engine's frame ring)
// with the next stack's first valid channel fc_out = reset ? 3 : max(fc_in - 1, 0); otherwise it is pushed into the
// packed uint32-per-pixel stack.
#define RECT_MAX 512
// BANDED (the default): the rectangle walk per row visits only the rectangles that overlap the row's 8-row band --
// a per-band bit mask over the rectangle indices, set by one thread per rectangle (LDS atomicOr), walked in index
// (painter's) order by find-first-set -- instead of all R (Alien: ~210 rectangles, ~30 per band); the gray image rows
// are padded to 164 bytes (41 dwords: the 64 rows a wave paints fall on 64 distinct banks, where 160 bytes put 8 rows
// on each bank) and filled a dword at a time between the ragged ends.  The image is the same byte for byte.
constexpr int RECT_BAND = 8;
constexpr int RECT_NBAND = (pre::SH + RECT_BAND - 1) / RECT_BAND;
constexpr int RECT_MW = RECT_MAX / 32;

template <bool RING, bool BANDED = true>
__global__ __launch_bounds__(256) void rects_push_kernel(const int16_t* __restrict__ rects,
                                                         const uint8_t* __restrict__ rect_gray, int R, int bg,
                                                         const uint32_t* __restrict__ obs_in,
                                                         uint32_t* __restrict__ obs_out,
                                                         const uint8_t* __restrict__ reset,
                                                         const int* __restrict__ tables, uint8_t* __restrict__ frames,
                                                         long frame_stride, const uint8_t* __restrict__ fc_in,
                                                         uint8_t* __restrict__ fc_out) {
  using namespace pre;
  constexpr int RS = BANDED ? SW + 4 : SW;         // gray row stride (bytes)
  __shared__ int tab[8 * 160];
  __shared__ uint32_t gray[SH * RS / 4];
  __shared__ uint2 rs_[RECT_MAX];                  // (y0 | y1 << 16, x0 | x1 << 16), clamped; empty -> y1 = y0
  __shared__ uint8_t rg_[RECT_MAX];
  __shared__ uint32_t bmask[BANDED ? RECT_NBAND * RECT_MW : 1];
  const int env = blockIdx.x;
  const int nw = (R + 31) >> 5;
  for (int i = threadIdx.x; i < 8 * 160; i += 256) tab[i] = tables[i];
  if constexpr (BANDED) {
    for (int i = threadIdx.x; i < RECT_NBAND * RECT_MW; i += 256) bmask[i] = 0u;
    __syncthreads();
  }
  const int16_t* rr = rects + (long)env * R * 4;
  for (int r = threadIdx.x; r < R; r += 256) {
    int y0 = rr[r * 4 + 0], x0 = rr[r * 4 + 1];
    int y1 = y0 + rr[r * 4 + 2], x1 = x0 + rr[r * 4 + 3];
    y0 = max(y0, 0); x0 = max(x0, 0); y1 = min(y1, SH); x1 = min(x1, SW);
    if (y1 <= y0 || x1 <= x0) y1 = y0 = 0;
    rs_[r] = make_uint2((uint32_t)y0 | ((uint32_t)y1 << 16), (uint32_t)x0 | ((uint32_t)x1 << 16));
    rg_[r] = rect_gray[r];
    if constexpr (BANDED) {
      if (y1 > y0)
        for (int b = y0 / RECT_BAND; b <= (y1 - 1) / RECT_BAND; ++b) atomicOr(&bmask[b * RECT_MW + (r >> 5)], 1u << (r & 31));
    }
  }
  __syncthreads();
  uint8_t* g8 = reinterpret_cast<uint8_t*>(gray);
  const int row = threadIdx.x;
  if (row < SH) {
    uint32_t* rw = gray + row * (RS / 4);
    const uint32_t bg4 = (uint32_t)bg * 0x01010101u;
    for (int i = 0; i < SW / 4; ++i) rw[i] = bg4;
    uint8_t* r8 = g8 + row * RS;
    auto paint = [&](int r) {
      const uint2 b = rs_[r];                      // one broadcast LDS read per rectangle
      if (row < (int)(b.x & 0xFFFFu) || row >= (int)(b.x >> 16)) return;
      const int x0 = (int)(b.y & 0xFFFFu), x1 = (int)(b.y >> 16);
      const uint8_t g = rg_[r];
      if constexpr (BANDED) {
        const int a0 = (x0 + 3) & ~3, a1 = x1 & ~3;
        if (a0 >= a1) {
          for (int x = x0; x < x1; ++x) r8[x] = g;
        } else {
          for (int x = x0; x < a0; ++x) r8[x] = g;
          const uint32_t g4 = (uint32_t)g * 0x01010101u;
          for (int x = a0; x < a1; x += 4) rw[x >> 2] = g4;
          for (int x = a1; x < x1; ++x) r8[x] = g;
        }
      } else {
        for (int x = x0; x < x1; ++x) r8[x] = g;
      }
    };
    if constexpr (BANDED) {
      const uint32_t* bm = bmask + (row / RECT_BAND) * RECT_MW;
      for (int wi = 0; wi < nw; ++wi) {
        uint32_t m = bm[wi];
        while (m) {
          const int r = wi * 32 + __builtin_ctz(m);
          m &= m - 1;
          paint(r);
        }
      }
    } else {
      for (int r = 0; r < R; ++r) paint(r);
    }
  }
  __syncthreads();
  const bool rs = reset != nullptr && reset[env];
  if (RING && threadIdx.x == 0) fc_out[env] = rs ? 3 : (uint8_t)max((int)fc_in[env] - 1, 0);
  const uint4* in4 = reinterpret_cast<const uint4*>(obs_in) + (long)env * (OH * OW / 4);
  uint4* out4 = reinterpret_cast<uint4*>(obs_out) + (long)env * (OH * OW / 4);
  uint32_t* fo = RING ? reinterpret_cast<uint32_t*>(frames + (long)env * frame_stride) : nullptr;
  for (int q = threadIdx.x; q < OH * OW / 4; q += 256) {
    const int y = q / (OW / 4), x0 = (q - y * (OW / 4)) * 4;
    const int ys0 = tab[0 * 160 + y], ys1 = tab[1 * 160 + y], cy0 = tab[2 * 160 + y], cy1 = tab[3 * 160 + y];
    uint32_t f4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = x0 + e;
      const int xs0 = tab[4 * 160 + x], xs1 = tab[5 * 160 + x], cx0 = tab[6 * 160 + x], cx1 = tab[7 * 160 + x];
      const int ra = g8[ys0 * RS + xs0] * cx0 + g8[ys0 * RS + xs1] * cx1;
      const int rb = g8[ys1 * RS + xs0] * cx0 + g8[ys1 * RS + xs1] * cx1;
      int v = (ra * cy0 + rb * cy1 + (1 << 21)) >> 22;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      f4[e] = (uint32_t)v;
    }
    if constexpr (RING) {
      // the 4 new pixels as one word (a v_perm: the shift / or form of this packing came out with a wrong byte 2
      // from this kernel's build, tests/test_games_hip.py test_hip_game_frame_ring_matches_packed_stacks)
      fo[q] = __builtin_amdgcn_perm(f4[3] << 16 | f4[2], f4[1] << 16 | f4[0], 0x06040200u);
    } else {
    uint4 o;
    if (rs) {
      o = make_uint4(f4[0] * 0x01010101u, f4[1] * 0x01010101u, f4[2] * 0x01010101u, f4[3] * 0x01010101u);
    } else {
      const uint4 i = in4[q];
      o = make_uint4((i.x >> 8) | (f4[0] << 24), (i.y >> 8) | (f4[1] << 24), (i.z >> 8) | (f4[2] << 24),
                     (i.w >> 8) | (f4[3] << 24));
    }
    out4[q] = o;
    }
  }
}

// 0 = the per-row walk over every rectangle, 2 = banded, 1 = auto: banded from RECT_BANDED_MIN rectangles.  Measured
// at 2048 envs (scripts/diag/rects_phases.py, us per launch, banded vs walk): Alien (224 rectangles) 93 vs 114,
// Centipede (332) 59 vs 105, Breakout (113) 115 vs 98, SpaceInvaders (40) 41 vs 53; 35 with no rectangles
static int g_rects_banded = 1;
#define RECT_BANDED_MIN 160
extern "C" void rects_set_banded(int v) { g_rects_banded = v; }
static bool rects_banded(int R) { return g_rects_banded == 2 || (g_rects_banded == 1 && R >= RECT_BANDED_MIN); }

extern "C" int launch_rects_stack_push(const void* rects, const void* rect_gray, int R, int bg, const void* obs_in,
                                       void* obs_out, const void* reset, const int* tables, int N,
                                       hipStream_t stream) {
  if (R < 0 || R > RECT_MAX || N <= 0) return -22;
  if (rects_banded(R))
    rects_push_kernel<false, true><<<N, 256, 0, stream>>>((const int16_t*)rects, (const uint8_t*)rect_gray, R, bg,
                                                          (const uint32_t*)obs_in, (uint32_t*)obs_out,
                                                          (const uint8_t*)reset, tables, nullptr, 0, nullptr, nullptr);
  else
    rects_push_kernel<false, false><<<N, 256, 0, stream>>>((const int16_t*)rects, (const uint8_t*)rect_gray, R, bg,
                                                           (const uint32_t*)obs_in, (uint32_t*)obs_out,
                                                           (const uint8_t*)reset, tables, nullptr, 0, nullptr, nullptr);
  return (int)hipGetLastError();
}

// frame-ring form: frames = the engine ring's plane of this step for env 0 ([B][slots][160*120], frame_stride bytes
// between envs); fc_in / fc_out [B] uint8
extern "C" int launch_rects_ring_push(const void* rects, const void* rect_gray, int R, int bg, void* frames,
                                      long frame_stride, const void* fc_in, void* fc_out, const void* reset,
                                      const int* tables, int N, hipStream_t stream) {
  if (R < 0 || R > RECT_MAX || N <= 0 || frame_stride < 160 * 120 || frame_stride % 4 || !fc_in || !fc_out ||
      !frames)
    return -22;
  if (rects_banded(R))
    rects_push_kernel<true, true><<<N, 256, 0, stream>>>((const int16_t*)rects, (const uint8_t*)rect_gray, R, bg,
                                                         nullptr, nullptr, (const uint8_t*)reset, tables,
                                                         (uint8_t*)frames, frame_stride, (const uint8_t*)fc_in,
                                                         (uint8_t*)fc_out);
  else
    rects_push_kernel<true, false><<<N, 256, 0, stream>>>((const int16_t*)rects, (const uint8_t*)rect_gray, R, bg,
                                                          nullptr, nullptr, (const uint8_t*)reset, tables,
                                                          (uint8_t*)frames, frame_stride, (const uint8_t*)fc_in,
                                                          (uint8_t*)fc_out);
  return (int)hipGetLastError();
}
