// On-device vectorised environments (bit-identical to envs/pong.py, envs/cartpole.py).
//
// pong_step: ONE launch per agent step for all envs.  One workgroup per env:
//   * physics for `frameskip` sub-frames (integer 1/16-px fixed point, wave-
//     uniform scalar code), reward/done/auto-reset with random no-op delay;
//   * render + gray + bilinear resize fused: each thread produces output
//     pixels of the 160x120 frame by evaluating the scene analytically at the
//     4 bilinear source pixels of the (never materialised) 210x160 RGB frame
//     -- game_state.py:41-50 (cvtColor + cv2.resize INTER_LINEAR, 11-bit
//     fixed-point weights);
//   * frame-stack push (game_state.py:78): out = (in >> 8) | f << 24 per pixel
//     (uint32 = 4 uint8 channels, newest last), or f*0x01010101 after a reset.
// This replaces ALE + OpenCV + the 4-deep numpy stack of the reference.
#include "common.h"

// phase stamps for the diagnostic probe (scripts/probe_env.hip defines PONG_STAMP); no-op here
#ifndef PONG_STAMP
#define PONG_STAMP(i)
#endif
#ifndef PONG_LOOP_STAMP
#define PONG_LOOP_STAMP(it, slow)
#endif

namespace pong {
constexpr int SCREEN_W = 160;
constexpr int OBS_H = 160, OBS_W = 120;
constexpr int TOP = 34, BOTTOM = 194, WALL_TOP0 = 24;
constexpr int PADDLE_H = 16, PADDLE_W = 4, BALL_W = 2, BALL_H = 4;
constexpr int PLAYER_X = 140, CPU_X = 16, U = 16;
constexpr int PLAYER_SPEED = 40, CPU_SPEED = 28, SERVE_VX = 32, MAX_VX = 64, MAX_VY = 40;
constexpr int SERVE_DELAY = 16, WIN_SCORE = 21;
constexpr int DIGIT_SCALE = 4, SCORE_ROW0 = 2;
enum { BX, BY, VX, VY, PY, CY, PS, CS, SERVE, STEPS, EPRET, NSTATE = 12 };
__constant__ int DIGITS[10] = {0b111101101101111, 0b010110010010111, 0b111001111100111, 0b111001111001111,
                               0b101101111001001, 0b111100111001111, 0b111100111101111, 0b111001001001001,
                               0b111101111101111, 0b111101111001111};

DEVI int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

DEVI uint32_t rnd(uint32_t seed, uint32_t env, uint32_t counter, uint32_t stream, uint32_t n) {
  return env_rand_u32(seed, env, counter, stream) % n;
}

struct St {
  int s[NSTATE];
};

DEVI int subframe(St& st, int up, int down, uint32_t seed, uint32_t env, uint32_t counter) {
  int* s = st.s;
  s[PY] = clampi(s[PY] - up * PLAYER_SPEED + down * PLAYER_SPEED, TOP * U, (BOTTOM - PADDLE_H) * U);
  const bool serving = s[SERVE] > 0;
  const bool chase = !serving && s[VX] < 0;
  const int target = chase ? s[BY] + (BALL_H * U) / 2 - (PADDLE_H * U) / 2 : ((TOP + BOTTOM) / 2 - PADDLE_H / 2) * U;
  const int dy = clampi(target - s[CY], -CPU_SPEED, CPU_SPEED);
  s[CY] = clampi(s[CY] + dy, TOP * U, (BOTTOM - PADDLE_H) * U);
  if (serving) s[SERVE] -= 1;
  if (serving && s[SERVE] == 0) {
    s[BX] = 78 * U;
    s[BY] = (TOP + 20 + (int)rnd(seed, env, counter, 0, BOTTOM - TOP - 40 - BALL_H)) * U;
    s[VX] = rnd(seed, env, counter, 1, 2) == 0 ? -SERVE_VX : SERVE_VX;
    s[VY] = (int)rnd(seed, env, counter, 2, 49) - 24;
  }
  const bool move = !serving;
  const int bx = s[BX], by = s[BY];
  int vx = s[VX], vy = s[VY];
  int nx = bx + vx, ny = by + vy;
  if (ny < TOP * U) { ny = 2 * TOP * U - ny; vy = -vy; }
  if (ny + BALL_H * U > BOTTOM * U) { ny = 2 * (BOTTOM - BALL_H) * U - ny; vy = -vy; }
  const int face = PLAYER_X * U;
  const bool hit_p = (vx > 0) && (bx + BALL_W * U <= face) && (nx + BALL_W * U > face) &&
                     (ny + BALL_H * U > s[PY]) && (ny < s[PY] + PADDLE_H * U);
  if (hit_p) {
    const int off = (ny + (BALL_H * U) / 2) - (s[PY] + (PADDLE_H * U) / 2);
    nx = face - BALL_W * U;
    vx = -min(abs(vx) + 1, MAX_VX);
    vy = clampi((off * 3) / 16, -MAX_VY, MAX_VY);
  }
  const int cface = (CPU_X + PADDLE_W) * U;
  const bool hit_c = (vx < 0) && (bx >= cface) && (nx < cface) && (ny + BALL_H * U > s[CY]) &&
                     (ny < s[CY] + PADDLE_H * U);
  if (hit_c) {
    const int coff = (ny + (BALL_H * U) / 2) - (s[CY] + (PADDLE_H * U) / 2);
    nx = cface;
    vx = min(abs(vx) + 1, MAX_VX);
    vy = clampi((coff * 3) / 16, -MAX_VY, MAX_VY);
  }
  const bool p_pt = move && (nx + BALL_W * U < 0);
  const bool c_pt = move && (nx > SCREEN_W * U);
  const int reward = p_pt ? 1 : (c_pt ? -1 : 0);
  s[PS] += p_pt;
  s[CS] += c_pt;
  if (p_pt || c_pt) s[SERVE] = SERVE_DELAY;
  if (move) { s[BX] = nx; s[BY] = ny; s[VX] = vx; s[VY] = vy; }
  return reward;
}

DEVI void reset_state(St& st, uint32_t seed, uint32_t env, uint32_t counter, int no_op_max, int frameskip) {
  int* s = st.s;
  const int mid = ((TOP + BOTTOM) / 2 - PADDLE_H / 2) * U;
  s[PS] = s[CS] = s[STEPS] = s[EPRET] = 0;
  s[PY] = s[CY] = mid;
  s[SERVE] = 1 + (int)rnd(seed, env, counter, 3, (uint32_t)((no_op_max + 1) * frameskip));
  s[BX] = 78 * U;
  s[BY] = (TOP + BOTTOM) / 2 * U;
  s[VX] = s[VY] = 0;
}

struct Scene {
  int cy, py, bx, by, vis;
  int dmask[4];           // 3x5 glyph bits of cpu tens / ones, player tens / ones (0 = not shown)
  int g_bg, g_wall, g_cpu, g_player, g_ball;
};

// glyph bits are resolved once per workgroup (Scene::dmask): a per-tap DIGITS[] load put a
// scalar-memory round trip on every evaluated score pixel
DEVI bool digit_lit(int mask, int r, int c, int x0) {
  const int dc = c - x0, dr = r - SCORE_ROW0;
  if (dc < 0 || dr < 0) return false;
  const int lc = dc / DIGIT_SCALE, lr = dr / DIGIT_SCALE;
  if (lc >= 3 || lr >= 5) return false;
  return (mask >> (14 - (lr * 3 + lc))) & 1;
}

// scene colour of source row r ignoring the digits, paddles and ball
DEVI int static_gray(const Scene& S, int r) {
  if (r < WALL_TOP0) return S.g_bg;
  return (r < TOP || r >= BOTTOM) ? S.g_wall : S.g_bg;
}

// score band (source rows SCORE_ROW0 .. +5*DIGIT_SCALE, digit columns 24..51 and 104..131) as
// per-source-pixel gray levels, built once per workgroup in LDS
constexpr int BAND_R = 5 * DIGIT_SCALE, BAND_C = 56;
constexpr int DL_R = 18;    // output rows of the per-workgroup score-digit box (rows 0..16 reach a digit)
// The score-digit boxes depend on one score each (the cpu box, output x 16..39, only reaches the cpu digits; the
// player box, x 76..99, only the player's) and on the env's constant colours and resize tables, so they are built
// once per env object (launch_pong_digit_tables) into the tail of the tables buffer: [side][score][DL_R][6 words].
// Per step the kernel copies its two 18 x 24 boxes instead of evaluating 864 pixels x 4 taps per workgroup.
constexpr int TAB_INTS = 8 * 160, DL_SCORES = WIN_SCORE + 1, DL_WORDS = DL_R * 6;
constexpr int TABLES_INTS = TAB_INTS + 2 * DL_SCORES * DL_WORDS;

DEVI int band_col(int c) { return (c >= 24 && c < 52) ? c - 24 : ((c >= 104 && c < 132) ? c - 104 + 28 : -1); }

// playfield-side scene colour, branch-free (walls / background + ball > player > cpu): the quad
// loop's per-pixel path only ever sees paddle / ball rows (digit pixels come from dlut)
DEVI int scene_gray_pf(const Scene& S, int r, int c) {
  int g = (r < TOP || r >= BOTTOM) ? (r < WALL_TOP0 ? S.g_bg : S.g_wall) : S.g_bg;
  const bool play = r >= TOP && r < BOTTOM;
  g = (play && c >= CPU_X && c < CPU_X + PADDLE_W && r >= S.cy && r < S.cy + PADDLE_H) ? S.g_cpu : g;
  g = (play && c >= PLAYER_X && c < PLAYER_X + PADDLE_W && r >= S.py && r < S.py + PADDLE_H) ? S.g_player : g;
  g = (play && S.vis && c >= S.bx && c < S.bx + BALL_W && r >= S.by && r < S.by + BALL_H) ? S.g_ball : g;
  return g;
}

// scene_gray_pf factored by axis: bit k of tap_rows(r) / tap_cols(c) = source row r / column c lies in rectangle k
// (0 cpu paddle, 1 player paddle, 2 ball; rows outside the playfield in none), so scene_gray_pf(S, r, c) ==
// tap_gray(S, tap_rows(r) & tap_cols(c), static colour of row r) (the same priority: ball > player > cpu)
DEVI int tap_rows(const Scene& S, int r) {
  const bool play = r >= TOP && r < BOTTOM;
  return play ? ((r >= S.cy && r < S.cy + PADDLE_H ? 1 : 0) | (r >= S.py && r < S.py + PADDLE_H ? 2 : 0) |
                 (S.vis && r >= S.by && r < S.by + BALL_H ? 4 : 0))
              : 0;
}
DEVI int tap_cols(const Scene& S, int c) {
  return (c >= CPU_X && c < CPU_X + PADDLE_W ? 1 : 0) | (c >= PLAYER_X && c < PLAYER_X + PADDLE_W ? 2 : 0) |
         (c >= S.bx && c < S.bx + BALL_W ? 4 : 0);
}
DEVI int tap_gray(const Scene& S, int m, int stat) {
  return (m & 4) ? S.g_ball : ((m & 2) ? S.g_player : ((m & 1) ? S.g_cpu : stat));
}

DEVI int scene_gray(const Scene& S, const uint8_t* band, int r, int c) {
  if (r < WALL_TOP0) {
    const int bc = band_col(c);
    return (r >= SCORE_ROW0 && r < SCORE_ROW0 + BAND_R && bc >= 0) ? (int)band[(r - SCORE_ROW0) * BAND_C + bc] : S.g_bg;
  }
  if (r < TOP || r >= BOTTOM) return S.g_wall;
  if (S.vis && c >= S.bx && c < S.bx + BALL_W && r >= S.by && r < S.by + BALL_H) return S.g_ball;
  if (c >= PLAYER_X && c < PLAYER_X + PADDLE_W && r >= S.py && r < S.py + PADDLE_H) return S.g_player;
  if (c >= CPU_X && c < CPU_X + PADDLE_W && r >= S.cy && r < S.cy + PADDLE_H) return S.g_cpu;
  return S.g_bg;
}
}  // namespace pong

namespace pong {
// byte offset of output quad xq in a dlut row (the score-digit boxes: quads 4..9 and 19..24), -1 outside them
DEVI int digit_quad(int xq) {
  return xq >= 4 && xq < 10 ? (xq - 4) * 4 : (xq >= 19 && xq < 25 ? 24 + (xq - 19) * 4 : -1);
}

// The 4 new-frame pixels of output quad (y, xq) (row word ri = rowinfo[y]): the row's static value, the
// score-digit box from dlut, or -- on paddle / ball rows whose columns touch the same rectangle -- the 4 taps
// evaluated analytically (all 4 pixels' taps and weights in 4 vector LDS reads, branch-free).
DEVI void quad_gray(const Scene& S, int y, int xq, int ri, const int* tab, const int* colmask, const int* quadmask,
                    const uint8_t* dlut, uint32_t* f4) {
  const uint32_t vr = (uint32_t)(ri & 0xFF);
  f4[0] = f4[1] = f4[2] = f4[3] = vr;
  const int rm = ri >> 8;
  const int dq = digit_quad(xq);
  if (y < DL_R && dq >= 0) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(&dlut[y * 48 + dq]);
    f4[0] = w & 0xFFu; f4[1] = (w >> 8) & 0xFFu; f4[2] = (w >> 16) & 0xFFu; f4[3] = w >> 24;
  } else if (rm && (rm & quadmask[xq])) {
    const int ys0 = tab[0 * 160 + y], ys1 = tab[1 * 160 + y], cy0 = tab[2 * 160 + y], cy1 = tab[3 * 160 + y];
    const int4 xs0v = *reinterpret_cast<const int4*>(&tab[4 * 160 + xq * 4]);
    const int4 xs1v = *reinterpret_cast<const int4*>(&tab[5 * 160 + xq * 4]);
    const int4 cx0v = *reinterpret_cast<const int4*>(&tab[6 * 160 + xq * 4]);
    const int4 cx1v = *reinterpret_cast<const int4*>(&tab[7 * 160 + xq * 4]);
    const int4 cmv = *reinterpret_cast<const int4*>(&colmask[xq * 4]);
    const int xs0a[4] = {xs0v.x, xs0v.y, xs0v.z, xs0v.w}, xs1a[4] = {xs1v.x, xs1v.y, xs1v.z, xs1v.w};
    const int cx0a[4] = {cx0v.x, cx0v.y, cx0v.z, cx0v.w}, cx1a[4] = {cx1v.x, cx1v.y, cx1v.z, cx1v.w};
    const int cma[4] = {cmv.x, cmv.y, cmv.z, cmv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ra = scene_gray_pf(S, ys0, xs0a[e]) * cx0a[e] + scene_gray_pf(S, ys0, xs1a[e]) * cx1a[e];
      const int rb = scene_gray_pf(S, ys1, xs0a[e]) * cx0a[e] + scene_gray_pf(S, ys1, xs1a[e]) * cx1a[e];
      int v = (ra * cy0 + rb * cy1 + (1 << 21)) >> 22;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      f4[e] = (rm & cma[e]) ? (uint32_t)v : f4[e];
    }
  }
}

// quad_gray's analytic branch from the per-tap row / column rectangle bits (scene_tables rowtap / coltap): the same
// taps, weights and rounding, ~4 logic ops per tap instead of scene_gray_pf's three rectangle tests
DEVI void quad_gray_taps(const Scene& S, int y, int xq, int ri, const int* tab, const int* colmask,
                         const int* rowtap, const int* coltap, uint32_t* f4) {
  const int rm = ri >> 8;
  const int rt = rowtap[y];
  const int rb0 = rt & 7, rb1 = (rt >> 3) & 7, st0 = (rt >> 8) & 0xFF, st1 = (rt >> 16) & 0xFF;
  const int cy0 = tab[2 * 160 + y], cy1 = tab[3 * 160 + y];
  const int4 ctv = *reinterpret_cast<const int4*>(&coltap[xq * 4]);
  const int4 cx0v = *reinterpret_cast<const int4*>(&tab[6 * 160 + xq * 4]);
  const int4 cx1v = *reinterpret_cast<const int4*>(&tab[7 * 160 + xq * 4]);
  const int4 cmv = *reinterpret_cast<const int4*>(&colmask[xq * 4]);
  const int cta[4] = {ctv.x, ctv.y, ctv.z, ctv.w};
  const int cx0a[4] = {cx0v.x, cx0v.y, cx0v.z, cx0v.w}, cx1a[4] = {cx1v.x, cx1v.y, cx1v.z, cx1v.w};
  const int cma[4] = {cmv.x, cmv.y, cmv.z, cmv.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c0 = cta[e] & 7, c1 = cta[e] >> 3;
    const int ra = tap_gray(S, rb0 & c0, st0) * cx0a[e] + tap_gray(S, rb0 & c1, st0) * cx1a[e];
    const int rb = tap_gray(S, rb1 & c0, st1) * cx0a[e] + tap_gray(S, rb1 & c1, st1) * cx1a[e];
    int v = (ra * cy0 + rb * cy1 + (1 << 21)) >> 22;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    f4[e] = (rm & cma[e]) ? (uint32_t)v : f4[e];
  }
}

// One env step's game physics on wave 0 of the env's workgroup (scalar code, frameskip sub-frames, reward,
// done, auto-reset); publishes the new state + done flag to LDS phys[] and writes the per-env outputs.
// fc_in != nullptr (frame ring): fc_out = done ? 3 : max(fc_in - 1, 0).
DEVI void physics_wave0(int env, int* __restrict__ state, uint32_t* __restrict__ counter, const int* __restrict__ actions,
                        int n_actions, uint32_t seed, int frameskip, int max_steps, int no_op_max, int* phys,
                        float* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                        float* __restrict__ epret_out, const uint8_t* __restrict__ fc_in,
                        uint8_t* __restrict__ fc_out, uint32_t id_base, int act_in = -1) {
  // RNG identity of the env: its GLOBAL index (id_base = first env of this rank), so a population sharded over
  // any number of ranks draws the same random streams as on one GPU
  const uint32_t rid = id_base + (uint32_t)env;
  St st;
#pragma unroll
  for (int i = 0; i < NSTATE; ++i) st.s[i] = __builtin_amdgcn_readfirstlane(state[env * NSTATE + i]);
  uint32_t ctr = (uint32_t)__builtin_amdgcn_readfirstlane((int)counter[env]);
  // act_in >= 0: the action sampled in this workgroup (pong_step_kernel HEADS), else the engine's action buffer
  int a = act_in >= 0 ? act_in : __builtin_amdgcn_readfirstlane(actions[env]);
  if (a >= n_actions || a < 0) a = 0;                    // game_state.py:38-39
  const int up = (a == 2 || a == 4), down = (a == 3 || a == 5);
  int reward = 0;
  for (int f = 0; f < frameskip; ++f) reward += subframe(st, up, down, seed, rid, ctr);
  ctr += 1;
  st.s[STEPS] += 1;
  st.s[EPRET] += reward;
  const bool done = st.s[PS] >= WIN_SCORE || st.s[CS] >= WIN_SCORE || st.s[STEPS] >= max_steps;
  const int epret = st.s[EPRET];
  if (done) {
    reset_state(st, seed, rid, ctr, no_op_max, frameskip);
    ctr += 1;
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NSTATE; ++i) {
      state[env * NSTATE + i] = st.s[i];
      phys[i] = st.s[i];
    }
    phys[NSTATE] = done ? 1 : 0;
    counter[env] = ctr;
    reward_out[env] = (float)reward;
    done_out[env] = done ? 1 : 0;
    epret_out[env] = done ? (float)epret : 0.f;
    if (fc_in) fc_out[env] = done ? 3 : (uint8_t)max((int)fc_in[env] - 1, 0);
  }
}

// Per-workgroup scene tables of the fused render (pong_step_kernel): the row / column
// rectangle masks, per-row static colour, score band and score-digit box.  Contains two barriers.
// dl: the precomputed digit boxes (tables tail), or nullptr to evaluate them here (launch_pong_digit_tables)
template <int NTH>
DEVI void scene_tables(const St& st, Scene& S, const int* tab, int* rowinfo, int* colmask, int* quadmask,
                       uint8_t* band, uint8_t* dlut, int g_bg, int g_wall, int g_cpu, int g_player, int g_ball,
                       const uint32_t* __restrict__ dl = nullptr, int* rowtap = nullptr, int* coltap = nullptr) {
  S.cy = st.s[CY] >> 4;   // floor division by U=16 (values are non-negative)
  S.py = st.s[PY] >> 4;
  S.bx = st.s[BX] >= 0 ? st.s[BX] / U : -((-st.s[BX] + U - 1) / U);   // floor
  S.by = st.s[BY] >= 0 ? st.s[BY] / U : -((-st.s[BY] + U - 1) / U);
  S.vis = st.s[SERVE] == 0;
  {
    const int cs_t = st.s[CS] / 10, cs_o = st.s[CS] % 10, ps_t = st.s[PS] / 10, ps_o = st.s[PS] % 10;
    S.dmask[0] = cs_t > 0 ? DIGITS[cs_t] : 0;        // tens digit only when non-zero
    S.dmask[1] = DIGITS[cs_o];
    S.dmask[2] = ps_t > 0 ? DIGITS[ps_t] : 0;
    S.dmask[3] = DIGITS[ps_o];
  }
  S.g_bg = g_bg; S.g_wall = g_wall; S.g_cpu = g_cpu; S.g_player = g_player; S.g_ball = g_ball;
  // source rectangles [r0, r1) x [c0, c1): cpu digits, player digits, ball, player, cpu
  const int by0 = S.vis ? S.by : -1000, by1 = S.vis ? S.by + BALL_H : -1000;   // matches no row when hidden
  const int R0[5] = {SCORE_ROW0, SCORE_ROW0, by0, S.py, S.cy};
  const int R1[5] = {SCORE_ROW0 + 5 * DIGIT_SCALE, SCORE_ROW0 + 5 * DIGIT_SCALE, by1, S.py + PADDLE_H,
                     S.cy + PADDLE_H};
  const int C0[5] = {24, 104, S.bx, PLAYER_X, CPU_X};
  const int C1[5] = {40 + 3 * DIGIT_SCALE, 120 + 3 * DIGIT_SCALE, S.bx + BALL_W, PLAYER_X + PADDLE_W,
                     CPU_X + PADDLE_W};
  const bool pre = dl != nullptr && st.s[CS] >= 0 && st.s[CS] < DL_SCORES && st.s[PS] >= 0 && st.s[PS] < DL_SCORES;
  if (pre) {
    // the two boxes of this step's scores: row yy = 6 cpu-box words then 6 player-box words (dlut[yy][48] bytes)
    for (int i = threadIdx.x; i < DL_R * 12; i += NTH) {
      const int yy = i / 12, wd = i - yy * 12, side = wd >= 6 ? 1 : 0;
      const int sc = side ? st.s[PS] : st.s[CS];
      *reinterpret_cast<uint32_t*>(&dlut[yy * 48 + wd * 4]) = dl[((side * DL_SCORES + sc) * DL_R + yy) * 6 + wd - side * 6];
    }
  }
  for (int i = threadIdx.x; !pre && i < BAND_R * BAND_C; i += NTH) {
    const int r = SCORE_ROW0 + i / BAND_C, bc = i - (i / BAND_C) * BAND_C;
    const int c = bc < 28 ? 24 + bc : 104 + (bc - 28);
    int g = S.g_bg;
    if (digit_lit(S.dmask[0], r, c, 24) || digit_lit(S.dmask[1], r, c, 40)) g = S.g_cpu;
    else if (digit_lit(S.dmask[2], r, c, 104) || digit_lit(S.dmask[3], r, c, 120)) g = S.g_player;
    band[i] = (uint8_t)g;
  }
  for (int i = threadIdx.x; i < OBS_H + OBS_W; i += NTH) {
    if (i < OBS_H) {
      const int ys0 = tab[0 * 160 + i], ys1 = tab[1 * 160 + i], cy0 = tab[2 * 160 + i], cy1 = tab[3 * 160 + i];
      int m = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) m |= (ys1 >= R0[k] && ys0 < R1[k]) ? (1 << k) : 0;
      int v = (static_gray(S, ys0) * cy0 + static_gray(S, ys1) * cy1 + 1024) >> 11;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      rowinfo[i] = v | (m << 8);
      if (rowtap) rowtap[i] = tap_rows(S, ys0) | (tap_rows(S, ys1) << 3) | (static_gray(S, ys0) << 8) |
                              (static_gray(S, ys1) << 16);
    } else {
      const int x = i - OBS_H;
      const int xs0 = tab[4 * 160 + x], xs1 = tab[5 * 160 + x];
      int m = 0;
#pragma unroll
      for (int k = 0; k < 5; ++k) m |= (xs1 >= C0[k] && xs0 < C1[k]) ? (1 << k) : 0;
      colmask[x] = m;
      if (coltap) coltap[x] = tap_cols(S, xs0) | (tap_cols(S, xs1) << 3);
    }
  }
  __syncthreads();
  if (threadIdx.x < OBS_W / 4)
    quadmask[threadIdx.x] = colmask[4 * threadIdx.x] | colmask[4 * threadIdx.x + 1] | colmask[4 * threadIdx.x + 2] |
                            colmask[4 * threadIdx.x + 3];
  // score-digit output box (rows < DL_R, quads 4..9 and 19..24 = x 16..39 and 76..99: every output
  // pixel whose taps can reach a digit), each pixel evaluated once per workgroup from the LDS band
  // map instead of inside the (divergent) quad loop
  for (int i = threadIdx.x; !pre && i < DL_R * 48; i += NTH) {
    const int yy = i / 48, lx = i - yy * 48;
    const int x = lx < 24 ? 16 + lx : 76 + (lx - 24);
    const int ys0 = tab[0 * 160 + yy], ys1 = tab[1 * 160 + yy], cy0 = tab[2 * 160 + yy], cy1 = tab[3 * 160 + yy];
    const int xs0 = tab[4 * 160 + x], xs1 = tab[5 * 160 + x], cx0 = tab[6 * 160 + x], cx1 = tab[7 * 160 + x];
    const int ra = scene_gray(S, band, ys0, xs0) * cx0 + scene_gray(S, band, ys0, xs1) * cx1;
    const int rb = scene_gray(S, band, ys1, xs0) * cx0 + scene_gray(S, band, ys1, xs1) * cx1;
    const int v = (ra * cy0 + rb * cy1 + (1 << 21)) >> 22;
    dlut[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
  __syncthreads();
}
}  // namespace pong

// The actor-critic heads + Gumbel-max sampling of ONE sample, folded into the env step of that sample
// (pong_step_kernel HEADS): the arithmetic of heads.hip heads_fwd_s16_kernel<8, float> -- 16 feature slices of 16
// features each summed in order with packed FMAs (common.h heads_fma), the slices summed in order -- so logits,
// value and the sampled action are bit-identical to the separate heads launch.  F = 256, A <= 8, fp32 features.
struct HeadsArgs {
  const float* feat;            // [B][256] step t's features
  const float* flat;            // parameter store
  long pw, pb, vw, vb;          // heads offsets in flat
  int A;
  float* logits;                // step t's [B][A]
  float* value;                 // [B]
  int* actions;                 // [B]
  uint32_t seed, rb;
  const long long* ctr;
  int t, T;
};
DEVI int heads_sample_one(const HeadsArgs& h, int b, float* red) {
  constexpr int F = 256, AM = 8, AW = AM + 1, FQ = F / 16;
  // thread (slice fs, output j), 144 of them: the slice's 16 features in order, one fused multiply-add each -- the
  // lane arithmetic of heads_fwd_s16_kernel's packed FMAs -- with every load of the chain issued up front
  if (threadIdx.x < 16 * AW) {
    const int fs = threadIdx.x / AW, j = threadIdx.x - fs * AW;
    const float* fr = h.feat + (long)b * F + fs * FQ;
    float x[FQ], wv[FQ];
#pragma unroll
    for (int k = 0; k < FQ; ++k) {
      const int f = fs * FQ + k;
      x[k] = fr[k];
      wv[k] = j == AM ? h.flat[h.vw + f] : (j < h.A ? h.flat[h.pw + (long)f * h.A + j] : 0.f);
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < FQ; ++k) acc = __builtin_fmaf(x[k], wv[k], acc);
    red[fs * AW + j] = acc;
  }
  __syncthreads();
  // lanes j < 9 of wave 0: output j's slice sum in slice order, bias, Gumbel key; the first maximum wins (the
  // sequential strict-greater scan of heads_fwd_s16_kernel)
  __shared__ int act_s;
  if (threadIdx.x < 64) {
    const int j = threadIdx.x;
    float v = 0.f;
    if (j < AW)
      for (int k = 0; k < 16; ++k) v += red[k * AW + j];
    float sc = -3.0e38f;
    if (j < h.A) {
      const uint32_t stepkey = (uint32_t)(h.ctr[0] * h.T + h.t);
      const float lg = v + h.flat[h.pb + j];
      h.logits[(long)b * h.A + j] = lg;
      const float g = lg - __logf(-__logf(sample_u01(h.seed, stepkey, h.rb + (uint32_t)b, (uint32_t)j)));
      if (g > sc) sc = g;                                     // (a NaN key never wins, as in the scan)
    }
    if (j == AM) h.value[b] = v + h.flat[h.vb];
    int bj = j < h.A ? j : 64;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float osc = __shfl_xor(sc, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (osc > sc || (osc == sc && oj < bj)) { sc = osc; bj = oj; }
    }
    if (j == 0) {
      const int best = bj < h.A ? bj : 0;
      h.actions[b] = best;
      act_s = best;
    }
  }
  __syncthreads();
  return act_s;
}

// state [B][12] int32, counter [B] uint32, actions [B] int32 (any int; >= n_actions remapped to 0)
// obs_in/obs_out [B][160*120] uint32 (4 stacked uint8 frames), tables [8][160] int32
//
// RING: instead of pushing into a packed stack, write ONLY the new 160x120 frame plane
// (frame_out [B][160*120] uint8, 19.2 KB per env instead of a 77 KB stack read + 77 KB
// stack write) and the next stack's first valid channel: fc_out = done ? 3 : max(fc_in-1, 0)
// (a reset stack repeats the fresh frame in all 4 channels; see conv_fwd_fast RING).
template <bool RING, bool HEADS = false>
__global__ __launch_bounds__(256, 8) void pong_step_kernel(int* __restrict__ state, uint32_t* __restrict__ counter,
                                                        const int* __restrict__ actions, int n_actions,
                                                        const uint32_t* __restrict__ obs_in,
                                                        uint32_t* __restrict__ obs_out, const int* __restrict__ tables,
                                                        float* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                        float* __restrict__ epret_out, uint32_t seed, int frameskip,
                                                        int max_steps, int no_op_max, int g_bg, int g_wall, int g_cpu,
                                                        int g_player, int g_ball,
                                                        const uint8_t* __restrict__ fc_in = nullptr,
                                                        uint8_t* __restrict__ fc_out = nullptr,
                                                        long out_stride = 0, int b0 = 0, uint32_t id_base = 0,
                                                        HeadsArgs ha = HeadsArgs{}) {
  using namespace pong;
  __shared__ __attribute__((aligned(16))) int tab[8 * 160];
  const int env = b0 + blockIdx.x;
  PONG_STAMP(0);
  for (int i = threadIdx.x; i < 8 * 160; i += 256) tab[i] = tables[i];
  int act_in = -1;
  if constexpr (HEADS) {
    __shared__ float hred[16 * 9];
    act_in = heads_sample_one(ha, env, hred);              // (its barriers also publish tab[])
  }
  // --- physics: wave 0 only (scalar code; the 4 waves of a workgroup share ONE scalar unit per
  // CU with the other workgroups there, so running it redundantly in every wave made the SALU the
  // kernel's bottleneck), published through LDS ---
  __shared__ int phys[NSTATE + 4];
  if (threadIdx.x < 64)
    physics_wave0(env, state, counter, actions, n_actions, seed, frameskip, max_steps, no_op_max, phys, reward_out,
                  done_out, epret_out, RING ? fc_in : nullptr, fc_out, id_base, act_in);
  PONG_STAMP(1);
  __syncthreads();    // tab[] staged and the new state published
  PONG_STAMP(2);
  St st;
#pragma unroll
  for (int i = 0; i < NSTATE; ++i) st.s[i] = __builtin_amdgcn_readfirstlane(phys[i]);
  const bool done = __builtin_amdgcn_readfirstlane(phys[NSTATE]) != 0;
  // --- fused render + gray + resize + stack push ---
  // Every source pixel outside five rectangles (the two score-digit blocks, the ball and the two
  // paddles) has its row's static colour (background or wall band), so an output pixel none of
  // whose 4 bilinear taps falls in a rectangle is the per-row constant vrow[y] -- the same
  // fixed-point blend, since the horizontal weights sum to 2048.  Per workgroup, one pass over
  // the 160 rows and 120 columns tabulates vrow and the rectangles each output row / column can
  // touch; a quad then costs one LDS read unless its row touches a rectangle, and only pixels
  // whose row AND column touch the same rectangle evaluate their 4 taps analytically.
  // Packed mode: one 16-byte load of the old stack + one 16-byte store of the new per quad
  // (frame-stack push (in >> 8) | f << 24); ring mode: one 4-byte store of the new frame.
  __shared__ int rowinfo[OBS_H];     // vrow | (rect mask << 8)
  __shared__ __attribute__((aligned(16))) int colmask[OBS_W];
  __shared__ int quadmask[OBS_W / 4];    // OR of the 4 columns' masks per quad
  __shared__ uint8_t band[BAND_R * BAND_C];
  __shared__ __attribute__((aligned(4))) uint8_t dlut[DL_R * 48];
  __shared__ int rowtap[RING ? OBS_H : 1];
  __shared__ __attribute__((aligned(16))) int coltap[RING ? OBS_W : 4];
  Scene S;
  scene_tables<256>(st, S, tab, rowinfo, colmask, quadmask, band, dlut, g_bg, g_wall, g_cpu, g_player, g_ball,
                    reinterpret_cast<const uint32_t*>(tables + TAB_INTS), RING ? rowtap : nullptr,
                    RING ? coltap : nullptr);
  PONG_STAMP(3);
  constexpr int NQ = OBS_H * OBS_W / 4, QR = OBS_W / 4;      // quads per frame / per row
  if constexpr (RING) {
    // Four quads per thread at a time, their row words, quad masks and digit-box words read from LDS up front: at
    // one workgroup per CU (8 paths x 32 envs) the walk of one quad at a time -- dependent LDS round trips and a
    // branch per quad -- took ~850 cycles per quad and was the kernel's critical path
    // (scripts/probe_env.hip).  Same pixels: a quad is its row's static value, its digit-box word, or quad_gray's
    // analytic taps when its row and columns touch the same rectangle.
    uint32_t* outw = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(obs_out) + (long)env * out_stride);
    for (int q0 = threadIdx.x; q0 < NQ; q0 += 4 * 256) {
      PONG_LOOP_STAMP((q0 >> 10), 0);
      int yk[4], xk[4], rik[4], qmk[4];
      uint32_t dwk[4];
      bool dk[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = min(q0 + 256 * k, NQ - 1);
        yk[k] = q / QR;
        xk[k] = q - yk[k] * QR;
        rik[k] = rowinfo[yk[k]];
        qmk[k] = quadmask[xk[k]];
        const int dq = digit_quad(xk[k]);
        dk[k] = yk[k] < DL_R && dq >= 0;
        dwk[k] = *reinterpret_cast<const uint32_t*>(&dlut[min(yk[k], DL_R - 1) * 48 + max(dq, 0)]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = q0 + 256 * k;
        if (q < NQ) {
          uint32_t wv = (uint32_t)(rik[k] & 0xFF) * 0x01010101u;
          if (dk[k]) {
            wv = dwk[k];
          } else if ((rik[k] >> 8) & qmk[k]) {
            uint32_t f4[4] = {wv & 0xFFu, wv & 0xFFu, wv & 0xFFu, wv & 0xFFu};
            quad_gray_taps(S, yk[k], xk[k], rik[k], tab, colmask, rowtap, coltap, f4);
            wv = f4[0] | (f4[1] << 8) | (f4[2] << 16) | (f4[3] << 24);
          }
          outw[q] = wv;
        }
      }
    }
    PONG_STAMP(4);
    return;
  }
  const uint4* in4 = reinterpret_cast<const uint4*>(obs_in) + (long)env * (OBS_H * OBS_W / 4);
  uint4* out4 = reinterpret_cast<uint4*>(obs_out) + (long)env * (OBS_H * OBS_W / 4);
  uint32_t* outw = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(obs_out) + (long)env * out_stride);
  // The old-stack loads of the next TWO items are in flight during this item's render work: with one
  // load ahead per thread the whole chip held ~8 MB of loads in flight, about half of what HBM's
  // bandwidth x latency needs, and the packed-stack kernel ran at ~4.5 TB/s.  Each item is owned by
  // one thread, so obs_in == obs_out stays correct.
  static_assert(256 % QR == 16 && 256 / QR == 8, "quad walk below assumes 30 quads per row");
  uint4 nxt = make_uint4(0u, 0u, 0u, 0u), nxt2 = nxt;
  if (!RING && !done) {
    nxt = in4[min((int)threadIdx.x, NQ - 1)];
    nxt2 = in4[min((int)threadIdx.x + 256, NQ - 1)];
  }
  int y = (int)threadIdx.x / QR, xq = (int)threadIdx.x - y * QR;
  int ri_next = rowinfo[y];            // row word of the next quad, read one iteration ahead
  for (int q = threadIdx.x; q < NQ; q += 256) {
    PONG_LOOP_STAMP((q >> 8), rowinfo[y] >> 8);
    const uint4 cur = nxt;
    nxt = nxt2;
    if (!RING && !done) nxt2 = in4[min(q + 512, NQ - 1)];     // (clamped, unconditional: no loop-carried phi)
    const int ri = ri_next;
    {
      int yn = y + 8 + (xq + 16 >= QR ? 1 : 0);
      ri_next = rowinfo[yn < OBS_H ? yn : OBS_H - 1];
    }
    uint32_t f4[4];
    quad_gray(S, y, xq, ri, tab, colmask, quadmask, dlut, f4);
    if constexpr (RING) {
      outw[q] = f4[0] | (f4[1] << 8) | (f4[2] << 16) | (f4[3] << 24);
    } else {
      uint4 o;
      if (done) {
        o = make_uint4(f4[0] * 0x01010101u, f4[1] * 0x01010101u, f4[2] * 0x01010101u, f4[3] * 0x01010101u);
      } else {
        const uint4 i = cur;
        o = make_uint4((i.x >> 8) | (f4[0] << 24), (i.y >> 8) | (f4[1] << 24), (i.z >> 8) | (f4[2] << 24),
                       (i.w >> 8) | (f4[3] << 24));
      }
      out4[q] = o;
    }
    xq += 16;
    y += 8;
    if (xq >= QR) { xq -= QR; ++y; }
  }
  PONG_STAMP(4);
}

// Frame ring, small populations: the env step as two launches -- physics (one wave per env) and the render split
// over `split` workgroups per env (each builds the scene tables and renders 1/split of the quads).  The fused kernel
// is one workgroup per env, so at B = 256 envs (8 paths x 32) its ~20 us per-workgroup critical path (physics,
// scene tables, 19 quads per thread) is the whole step; the split shortens the render walk and takes the physics
// off the render's path.  Same physics, same pixels (bit-identical to pong_step_kernel<true>).
__global__ __launch_bounds__(64) void pong_physics_kernel(int* __restrict__ state, uint32_t* __restrict__ counter,
                                                         const int* __restrict__ actions, int n_actions,
                                                         float* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                         float* __restrict__ epret_out, uint32_t seed, int frameskip,
                                                         int max_steps, int no_op_max, const uint8_t* __restrict__ fc_in,
                                                         uint8_t* __restrict__ fc_out, uint32_t id_base, int b0) {
  __shared__ int phys[pong::NSTATE + 4];
  pong::physics_wave0(b0 + (int)blockIdx.x, state, counter, actions, n_actions, seed, frameskip, max_steps, no_op_max, phys,
                      reward_out, done_out, epret_out, fc_in, fc_out, id_base);
}

__global__ __launch_bounds__(256, 8) void pong_render_ring_kernel(const int* __restrict__ state,
                                                                 const int* __restrict__ tables,
                                                                 uint8_t* __restrict__ frame_out, long out_stride,
                                                                 int split, int g_bg, int g_wall, int g_cpu,
                                                                 int g_player, int g_ball, int b0) {
  using namespace pong;
  __shared__ __attribute__((aligned(16))) int tab[8 * 160];
  __shared__ int rowinfo[OBS_H];
  __shared__ __attribute__((aligned(16))) int colmask[OBS_W];
  __shared__ int quadmask[OBS_W / 4];
  __shared__ uint8_t band[BAND_R * BAND_C];
  __shared__ __attribute__((aligned(4))) uint8_t dlut[DL_R * 48];
  const int env = b0 + (int)blockIdx.y;
  for (int i = threadIdx.x; i < 8 * 160; i += 256) tab[i] = tables[i];
  St st;
#pragma unroll
  for (int i = 0; i < NSTATE; ++i) st.s[i] = __builtin_amdgcn_readfirstlane(state[env * NSTATE + i]);
  __syncthreads();                                   // tab[] staged
  Scene S;
  scene_tables<256>(st, S, tab, rowinfo, colmask, quadmask, band, dlut, g_bg, g_wall, g_cpu, g_player, g_ball,
                    reinterpret_cast<const uint32_t*>(tables + TAB_INTS));
  constexpr int NQ = OBS_H * OBS_W / 4, QR = OBS_W / 4;
  const int per = (NQ + split - 1) / split;
  const int q0 = (int)blockIdx.x * per, q1 = min(NQ, q0 + per);
  uint32_t* outw = reinterpret_cast<uint32_t*>(frame_out + (long)env * out_stride);
  int q = q0 + (int)threadIdx.x;
  int y = q / QR, xq = q - (q / QR) * QR;
  for (; q < q1; q += 256) {
    uint32_t f4[4];
    quad_gray(S, y, xq, rowinfo[y], tab, colmask, quadmask, dlut, f4);
    outw[q] = f4[0] | (f4[1] << 8) | (f4[2] << 16) | (f4[3] << 24);
    xq += 16;
    y += 8;
    if (xq >= QR) { xq -= QR; ++y; }
  }
}

// The score-digit boxes of every score (launch_pong_digit_tables): workgroup sc evaluates the scene of a state with
// both scores = sc (the ball hidden; the boxes never reach the playfield) with the per-step code path, then stores
// its cpu box as side 0 / score sc and its player box as side 1 / score sc in the tables tail.
__global__ __launch_bounds__(256) void pong_digit_tables_kernel(int* __restrict__ tables, int g_bg, int g_wall,
                                                                int g_cpu, int g_player, int g_ball) {
  using namespace pong;
  __shared__ __attribute__((aligned(16))) int tab[TAB_INTS];
  __shared__ int rowinfo[OBS_H];
  __shared__ __attribute__((aligned(16))) int colmask[OBS_W];
  __shared__ int quadmask[OBS_W / 4];
  __shared__ uint8_t band[BAND_R * BAND_C];
  __shared__ __attribute__((aligned(4))) uint8_t dlut[DL_R * 48];
  for (int i = threadIdx.x; i < TAB_INTS; i += 256) tab[i] = tables[i];
  St st;
#pragma unroll
  for (int i = 0; i < NSTATE; ++i) st.s[i] = 0;
  st.s[CS] = st.s[PS] = (int)blockIdx.x;
  st.s[SERVE] = 1;
  __syncthreads();                                   // tab[] staged
  Scene S;
  scene_tables<256>(st, S, tab, rowinfo, colmask, quadmask, band, dlut, g_bg, g_wall, g_cpu, g_player, g_ball);
  uint32_t* out = reinterpret_cast<uint32_t*>(tables + TAB_INTS);
  for (int i = threadIdx.x; i < DL_R * 12; i += 256) {
    const int yy = i / 12, wd = i - yy * 12, side = wd >= 6 ? 1 : 0;
    out[((side * DL_SCORES + (int)blockIdx.x) * DL_R + yy) * 6 + wd - side * 6] =
        *reinterpret_cast<const uint32_t*>(&dlut[yy * 48 + wd * 4]);
  }
}

// ---------------------------------------------------------------------------
// CartPole-v1: thread per env. state [B][4] f32, steps [B] i32, epret [B] f32,
// counter [B] u32; writes obs bf16 [B][8] (zero padded) for the trunk.
// ---------------------------------------------------------------------------
__global__ void cartpole_step_kernel(float* __restrict__ state, int* __restrict__ steps, float* __restrict__ epret,
                                     uint32_t* __restrict__ counter, const int* __restrict__ actions, int B,
                                     uint32_t seed, uint32_t id_base, int max_steps, float* __restrict__ obs_f32,
                                     bf16_t* __restrict__ obs_bf16, float* __restrict__ reward_out,
                                     uint8_t* __restrict__ done_out, float* __restrict__ epret_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float g = 9.8f, mc = 1.0f, mp = 0.1f, tm = mc + mp, len = 0.5f, pml = mp * len, fm = 10.0f, tau = 0.02f;
  const float th_thr = 12.f * 2.f * 3.14159265358979323846f / 360.f, x_thr = 2.4f;
  float x = state[b * 4 + 0], xd = state[b * 4 + 1], th = state[b * 4 + 2], thd = state[b * 4 + 3];
  const float force = actions[b] == 1 ? fm : -fm;
  const float ct = cosf(th), st = sinf(th);
  const float temp = (force + pml * thd * thd * st) / tm;
  const float thacc = (g * st - ct * temp) / (len * (4.0f / 3.0f - mp * ct * ct / tm));
  const float xacc = temp - pml * thacc * ct / tm;
  x = x + tau * xd;
  xd = xd + tau * xacc;
  th = th + tau * thd;
  thd = thd + tau * thacc;
  const int n = steps[b] + 1;
  const bool fell = x < -x_thr || x > x_thr || th < -th_thr || th > th_thr;
  const bool done = fell || n >= max_steps;
  const float er = epret[b] + 1.0f;
  uint32_t ctr = counter[b];
  reward_out[b] = 1.0f;
  done_out[b] = done;
  epret_out[b] = done ? er : 0.f;
  if (done) {
    float u[4];
    for (int s = 0; s < 4; ++s) u[s] = (float)(env_rand_u32(seed, id_base + (uint32_t)b, ctr, (uint32_t)s) >> 8) * (1.0f / 16777216.0f);
    x = u[0] * 0.1f - 0.05f; xd = u[1] * 0.1f - 0.05f; th = u[2] * 0.1f - 0.05f; thd = u[3] * 0.1f - 0.05f;
    ctr += 1;
  }
  counter[b] = ctr;
  steps[b] = done ? 0 : n;
  epret[b] = done ? 0.f : er;
  state[b * 4 + 0] = x; state[b * 4 + 1] = xd; state[b * 4 + 2] = th; state[b * 4 + 3] = thd;
  if (obs_f32) { obs_f32[b * 4 + 0] = x; obs_f32[b * 4 + 1] = xd; obs_f32[b * 4 + 2] = th; obs_f32[b * 4 + 3] = thd; }
  if (obs_bf16) {
    uint4 o;
    o.x = pack2bf(x, xd);
    o.y = pack2bf(th, thd);
    o.z = 0;
    o.w = 0;
    *reinterpret_cast<uint4*>(obs_bf16 + (long)b * 8) = o;
  }
}



extern "C" {
int launch_pong_step(void* state, void* counter, const int* actions, int n_actions, const void* obs_in, void* obs_out,
                     const int* tables, float* reward, void* done, float* epret, int B, unsigned seed, int frameskip,
                     int max_steps, int no_op_max, int g_bg, int g_wall, int g_cpu, int g_player, int g_ball,
                     int b0, unsigned id_base, hipStream_t stream) {
  if (n_actions <= 0 || B <= 0 || frameskip < 0 || max_steps < 0 || no_op_max < 0 || g_bg < 0 || g_wall < 0 ||
      g_cpu < 0 || g_player < 0 || g_ball < 0 || b0 < 0) return -22;
  // envs [b0, B): one path group of the split rollout (runtime/engine.py); per-env state and RNG keys are global
  if (b0 < 0 || b0 >= B) return -22;
  pong_step_kernel<false><<<B - b0, 256, 0, stream>>>((int*)state, (uint32_t*)counter, actions, n_actions,
                                                      (const uint32_t*)obs_in, (uint32_t*)obs_out, tables, reward,
                                                      (uint8_t*)done, epret, seed, frameskip, max_steps, no_op_max,
                                                      g_bg, g_wall, g_cpu, g_player, g_ball, nullptr, nullptr, 0, b0,
                                                      id_base);
  return (int)hipGetLastError();
}

// frame-ring variant: frame_out = env 0's new frame (160*120 uint8), env b's at + b*out_stride bytes;
// fc_in/fc_out [B] uint8.  Envs [b0, B) only (one path group of the split rollout, runtime/engine.py): every index
// (state, RNG key, frame, fc) stays global.
static int pong_ring_launch(void* state, void* counter, const int* actions, int n_actions, void* frame_out,
                            long out_stride, const void* fc_in, void* fc_out, const int* tables, float* reward,
                            void* done, float* epret, int B, unsigned seed, int frameskip, int max_steps,
                            int no_op_max, int g_bg, int g_wall, int g_cpu, int g_player, int g_ball, unsigned id_base,
                            int b0, int split, hipStream_t stream) {
  if (n_actions <= 0 || out_stride <= 0 || B <= 0 || frameskip < 0 || max_steps < 0 || no_op_max < 0 || g_bg < 0 ||
      g_wall < 0 || g_cpu < 0 || g_player < 0 || g_ball < 0 || b0 < 0 || b0 >= B || split > 64) return -22;
  if (out_stride < 160 * 120 || out_stride % 16) return -22;
  if (split <= 1) {
    pong_step_kernel<true><<<B - b0, 256, 0, stream>>>((int*)state, (uint32_t*)counter, actions, n_actions, nullptr,
                                                       (uint32_t*)frame_out, tables, reward, (uint8_t*)done, epret,
                                                       seed, frameskip, max_steps, no_op_max, g_bg, g_wall, g_cpu,
                                                       g_player, g_ball, (const uint8_t*)fc_in, (uint8_t*)fc_out,
                                                       out_stride, b0, id_base);
    return (int)hipGetLastError();
  }
  if (!fc_in || !fc_out) return -22;
  // the same step in two launches (physics, then the render over `split` workgroups per env)
  pong_physics_kernel<<<B - b0, 64, 0, stream>>>((int*)state, (uint32_t*)counter, actions, n_actions, reward,
                                                 (uint8_t*)done, epret, seed, frameskip, max_steps, no_op_max,
                                                 (const uint8_t*)fc_in, (uint8_t*)fc_out, id_base, b0);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  pong_render_ring_kernel<<<dim3((unsigned)split, (unsigned)(B - b0)), 256, 0, stream>>>(
      (const int*)state, tables, (uint8_t*)frame_out, out_stride, split, g_bg, g_wall, g_cpu, g_player, g_ball, b0);
  return (int)hipGetLastError();
}

// the ring step of envs [b0, b1) with the heads + sampling of each env's sample in the same workgroup
// (pong_step_kernel<true, true>); feat: step t's [B][256] fp32 features
int launch_pong_heads_step_ring(void* state, void* counter, int n_actions, void* frame_out, long out_stride,
                                const void* fc_in, void* fc_out, const int* tables, float* reward, void* done,
                                float* epret, int b1, unsigned seed, int frameskip, int max_steps, int no_op_max,
                                int g_bg, int g_wall, int g_cpu, int g_player, int g_ball, unsigned id_base, int b0,
                                const float* feat, int F, const float* flat, long pw, long pb, long vw, long vb,
                                float* logits, float* value, int* actions, unsigned hseed, const long long* ctr, int t,
                                int T, unsigned rb, hipStream_t stream) {
  if (n_actions <= 0 || n_actions > 8 || F != 256 || out_stride < 160 * 120 || out_stride % 16 || b1 <= 0 || b0 < 0 ||
      b0 >= b1 || !feat || !flat || !logits || !value || !actions || !ctr || !fc_in || !fc_out || frameskip < 0 ||
      max_steps < 0 || no_op_max < 0 || g_bg < 0 || g_wall < 0 || g_cpu < 0 || g_player < 0 || g_ball < 0)
    return -22;
  HeadsArgs ha{feat, flat, pw, pb, vw, vb, n_actions, logits, value, actions, hseed, rb, ctr, t, T};
  pong_step_kernel<true, true><<<b1 - b0, 256, 0, stream>>>(
      (int*)state, (uint32_t*)counter, actions, n_actions, nullptr, (uint32_t*)frame_out, tables, reward,
      (uint8_t*)done, epret, seed, frameskip, max_steps, no_op_max, g_bg, g_wall, g_cpu, g_player, g_ball,
      (const uint8_t*)fc_in, (uint8_t*)fc_out, out_stride, b0, id_base, ha);
  return (int)hipGetLastError();
}

int launch_pong_step_ring(void* state, void* counter, const int* actions, int n_actions, void* frame_out,
                          long out_stride, const void* fc_in, void* fc_out, const int* tables, float* reward,
                          void* done, float* epret, int B, unsigned seed, int frameskip, int max_steps, int no_op_max,
                          int g_bg, int g_wall, int g_cpu, int g_player, int g_ball, unsigned id_base,
                          hipStream_t stream) {
  return pong_ring_launch(state, counter, actions, n_actions, frame_out, out_stride, fc_in, fc_out, tables, reward,
                          done, epret, B, seed, frameskip, max_steps, no_op_max, g_bg, g_wall, g_cpu, g_player, g_ball,
                          id_base, 0, 1, stream);
}

// envs [b0, b1) of the ring step; split <= 1: the fused kernel, else physics + a render over `split` workgroups/env
int launch_pong_step_ring_split(void* state, void* counter, const int* actions, int n_actions, void* frame_out,
                                long out_stride, const void* fc_in, void* fc_out, const int* tables, float* reward,
                                void* done, float* epret, int b1, unsigned seed, int frameskip, int max_steps,
                                int no_op_max, int g_bg, int g_wall, int g_cpu, int g_player, int g_ball,
                                unsigned id_base, int b0, int split, hipStream_t stream) {
  return pong_ring_launch(state, counter, actions, n_actions, frame_out, out_stride, fc_in, fc_out, tables, reward,
                          done, epret, b1, seed, frameskip, max_steps, no_op_max, g_bg, g_wall, g_cpu, g_player, g_ball,
                          id_base, b0, split, stream);
}

// tables: [TAB_INTS resize tables | digit boxes]; fills the digit boxes from the resize tables (every Pong step
// launcher reads a tables buffer of pong_tables_ints() ints filled by this)
int pong_tables_ints() { return pong::TABLES_INTS; }
int launch_pong_digit_tables(int* tables, int g_bg, int g_wall, int g_cpu, int g_player, int g_ball,
                             hipStream_t stream) {
  if (!tables || g_bg < 0 || g_wall < 0 || g_cpu < 0 || g_player < 0 || g_ball < 0) return -22;
  pong_digit_tables_kernel<<<pong::DL_SCORES, 256, 0, stream>>>(tables, g_bg, g_wall, g_cpu, g_player, g_ball);
  return (int)hipGetLastError();
}

int launch_cartpole_step(float* state, int* steps, float* epret, void* counter, const int* actions, int B,
                         unsigned seed, unsigned id_base, int max_steps, float* obs_f32, void* obs_bf16,
                         float* reward, void* done, float* epret_out, hipStream_t stream) {
  if (B <= 0 || max_steps < 0) return -22;
  cartpole_step_kernel<<<(B + 255) / 256, 256, 0, stream>>>(state, steps, epret, (uint32_t*)counter, actions, B, seed,
                                                            id_base, max_steps, obs_f32, (bf16_t*)obs_bf16, reward,
                                                            (uint8_t*)done, epret_out);
  return (int)hipGetLastError();
}
}
