// On-device game logic for the synthetic Atari-style suite (envs/atari_games.py):
// Breakout, SpaceInvaders, Alien / MsPacman, Centipede.
//
// ONE thread per env runs the whole agent step: `frameskip` physics sub-frames,
// reward / done / episode return, the auto-reset of finished envs, and the scene
// (the per-env rectangle list in painter's order, int16 y0/x0/h/w) that
// rects_stack_push (csrc/preprocess.hip) rasterises, converts to gray, resizes and
// pushes into the frame stack.  So a game step is two launches and no torch ops;
// the torch implementation (atari_games.py) stays the bit-exact oracle
// (tests/test_games_hip.py).
//
// State: int32 [N][NS] per game, one row per env (the kernel keeps the row in
// registers).  Boolean grids are bit-packed (bricks 108 b, aliens 36 b, maze eggs
// 143 b, mushrooms 320 b).  The field order of every game is mirrored by
// `HIP_FIELDS` of its class in envs/atari_games.py.
//
// Integer semantics follow torch: `//` and `%` are floor division / floor modulo,
// the counter-based RNG (env_rand_u32) is shared with envs/base.py.
#include "common.h"

namespace games {

DEVI int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
DEVI int fdiv(int a, int b) {            // python a // b
  const int q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}
DEVI int fmodi(int a, int b) {           // python a % b
  const int r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? r + b : r;
}
DEVI int iabs(int v) { return v < 0 ? -v : v; }
DEVI bool getbit(const int* w, int i) { return ((uint32_t)w[i >> 5] >> (i & 31)) & 1u; }
DEVI void setbit(int* w, int i, bool v) {
  const uint32_t m = 1u << (i & 31);
  w[i >> 5] = (int)(v ? ((uint32_t)w[i >> 5] | m) : ((uint32_t)w[i >> 5] & ~m));
}
DEVI void fill_bits(int* w, int nbits) {
  for (int i = 0; i < (nbits + 31) / 32; ++i) {
    const int rem = nbits - 32 * i;
    w[i] = rem >= 32 ? -1 : (int)((1u << rem) - 1u);
  }
}
DEVI bool any_bits(const int* w, int nbits) {
  bool a = false;
  for (int i = 0; i < (nbits + 31) / 32; ++i) a |= w[i] != 0;
  return a;
}

struct Rng {
  uint32_t seed, env, counter;
  DEVI int rand(uint32_t stream, uint32_t n) const { return (int)(env_rand_u32(seed, env, counter, stream) % n); }
};

DEVI void rect(int16_t* r, int i, int y0, int x0, int h, int w) {
  r[4 * i + 0] = (int16_t)clampi(y0, -32768, 32767);
  r[4 * i + 1] = (int16_t)clampi(x0, -32768, 32767);
  r[4 * i + 2] = (int16_t)clampi(h, -32768, 32767);
  r[4 * i + 3] = (int16_t)clampi(w, -32768, 32767);
}

// --------------------------------------------------------------------------- Breakout
struct Breakout {
  static constexpr int U = 16, ROWS = 6, COLS = 18, NB = ROWS * COLS;
  static constexpr int BRICK_Y0 = 57, BRICK_H = 6, BRICK_W = 8, BRICK_X0 = 8, PADDLE_Y = 189, PADDLE_W = 16;
  enum { PX, BX, BY, VX, VY, INPLAY, LIVES, BR, COUNTER = BR + 4, STEPS, EPRET, NS };
  static constexpr int R = 3 + NB + 2;
  static DEVI int row_reward(int r) { return r < 2 ? 7 : (r < 4 ? 4 : 1); }
  static DEVI void reset(int* s, const Rng&) {
    fill_bits(s + BR, NB);
    s[PX] = 72 * U;
    s[INPLAY] = 0;
    s[LIVES] = 5;
  }
  static DEVI int physics(int* s, int a, const Rng& g) {
    const int right = a == 2, left = a == 3;
    s[PX] = clampi(s[PX] + (right - left) * 6 * U, 8 * U, (152 - PADDLE_W) * U);
    bool inplay = s[INPLAY] != 0;
    const bool serve = !inplay && a == 1;
    const int dirn = g.rand(0, 2) == 0 ? -1 : 1;
    if (serve) {
      s[BX] = s[PX] + (PADDLE_W / 2) * U;
      s[BY] = 120 * U;
      s[VX] = dirn * (24 + g.rand(1, 12));
      s[VY] = 40;
    }
    inplay = inplay || serve;
    int nx = s[BX] + s[VX], ny = s[BY] + s[VY];
    if ((nx < 8 * U || nx > 150 * U) && inplay) s[VX] = -s[VX];
    nx = clampi(nx, 8 * U, 150 * U);
    const bool hit_top = ny < 32 * U;
    if (hit_top && inplay) s[VY] = iabs(s[VY]);
    if (hit_top) ny = 32 * U;
    const int cy = fdiv(fdiv(ny, U) - BRICK_Y0, BRICK_H), cx = fdiv(fdiv(nx, U) - BRICK_X0, BRICK_W);
    const bool inb = cy >= 0 && cy < ROWS && cx >= 0 && cx < COLS && inplay;
    const int cyc = clampi(cy, 0, ROWS - 1), cxc = clampi(cx, 0, COLS - 1);
    const bool b = getbit(s + BR, cyc * COLS + cxc);
    const bool hitb = inb && b;
    const int reward = hitb ? row_reward(cyc) : 0;
    setbit(s + BR, cyc * COLS + cxc, b && !hitb);
    if (hitb) s[VY] = -s[VY];
    const int nyu = fdiv(ny, U);
    const bool onp = s[VY] > 0 && nyu >= PADDLE_Y - 4 && nyu < PADDLE_Y + 2 && nx >= s[PX] - 2 * U &&
                     nx <= s[PX] + (PADDLE_W + 2) * U;
    const int off = nx - (s[PX] + (PADDLE_W / 2) * U);
    if (onp && inplay) {
      s[VX] = clampi(fdiv(off * 3, 16), -48, 48);
      s[VY] = -iabs(s[VY]);
    }
    const bool lost = inplay && ny > 200 * U;
    s[LIVES] -= lost;
    inplay = inplay && !lost;
    if (inplay) {
      s[BX] = nx;
      s[BY] = ny;
    }
    s[INPLAY] = inplay;
    return reward;
  }
  static DEVI bool over(const int* s) { return s[LIVES] <= 0 || !any_bits(s + BR, NB); }
  static DEVI void scene(const int* s, int16_t* r) {
    rect(r, 0, 17, 0, 15, 160);
    rect(r, 1, 17, 0, 179, 8);
    rect(r, 2, 17, 152, 179, 8);
    for (int i = 0; i < NB; ++i)
      rect(r, 3 + i, BRICK_Y0 + (i / COLS) * BRICK_H, BRICK_X0 + (i % COLS) * BRICK_W, getbit(s + BR, i) ? BRICK_H : 0,
           BRICK_W);
    rect(r, 3 + NB, PADDLE_Y, fdiv(s[PX], U), 4, PADDLE_W);
    rect(r, 4 + NB, fdiv(s[BY], U), fdiv(s[BX], U), s[INPLAY] ? 4 : 0, 2);
  }
};

// --------------------------------------------------------------------------- SpaceInvaders
struct SpaceInvaders {
  static constexpr int AR = 6, AC = 6;
  enum { FX, FY, FDIR, TICK, PX, LIVES, SX, SY, SHOT, BXP, BYP, BOMB, ALIVE, COUNTER = ALIVE + 2, STEPS, EPRET, NS };
  static constexpr int R = 1 + AR * AC + 3;
  static DEVI void reset(int* s, const Rng&) {
    fill_bits(s + ALIVE, AR * AC);
    s[FX] = 22;
    s[FY] = 40;
    s[FDIR] = 1;
    s[TICK] = 0;
    s[PX] = 76;
    s[LIVES] = 3;
    s[SHOT] = 0;
    s[BOMB] = 0;
  }
  static DEVI bool alive(const int* s, int r, int c) { return getbit(s + ALIVE, r * AC + c); }
  static DEVI int physics(int* s, int a, const Rng& g) {
    const int right = a == 2 || a == 4, left = a == 3 || a == 5;
    const bool fire = a == 1 || a == 4 || a == 5;
    s[PX] = clampi(s[PX] + 2 * (right - left), 20, 133);
    bool shot = s[SHOT] != 0;
    const bool new_shot = fire && !shot;
    if (new_shot) {
      s[SX] = s[PX] + 3;
      s[SY] = 182;
    }
    shot = shot || new_shot;
    s[SY] -= 4 * shot;
    shot = shot && s[SY] > 20;
    // formation march every 4 sub-frames (column occupancy taken BEFORE this sub-frame's hit, as the oracle)
    s[TICK] += 1;
    const bool move = fmodi(s[TICK], 4) == 0;
    int cols = 0;
    for (int c = 0; c < AC; ++c)
      for (int r = 0; r < AR; ++r) cols |= (alive(s, r, c) ? 1 : 0) << c;
    int leftmost = AC, rightmost = -1;
    for (int c = AC - 1; c >= 0; --c)
      if ((cols >> c) & 1) leftmost = c;
    for (int c = 0; c < AC; ++c)
      if ((cols >> c) & 1) rightmost = c;
    const int xl = s[FX] + 16 * leftmost, xr = s[FX] + 16 * rightmost + 8;
    const bool edge = move && ((s[FDIR] > 0 && xr >= 150) || (s[FDIR] < 0 && xl <= 10));
    if (edge) s[FDIR] = -s[FDIR];
    s[FY] += 4 * edge;
    if (move && !edge) s[FX] += s[FDIR];
    // shot vs aliens
    const int col = fdiv(s[SX] - s[FX], 16), row = fdiv(s[SY] - s[FY], 18);
    const bool inx = fmodi(s[SX] - s[FX], 16) < 8, iny = fmodi(s[SY] - s[FY], 18) < 10;
    const bool ok = shot && col >= 0 && col < AC && row >= 0 && row < AR && inx && iny;
    const int colc = clampi(col, 0, AC - 1), rowc = clampi(row, 0, AR - 1);
    const bool al = alive(s, rowc, colc);
    const bool hit = ok && al;
    setbit(s + ALIVE, rowc * AC + colc, al && !hit);
    const int reward = hit ? 30 - 5 * rowc : 0;
    shot = shot && !hit;
    // alien bomb
    bool bomb = s[BOMB] != 0;
    bool drop = !bomb && g.rand(4, 64) == 0 && cols != 0;
    const int bc = g.rand(5, AC);
    const bool has = (cols >> bc) & 1;
    int lowest = -1;
    for (int r = 0; r < AR; ++r)
      if (alive(s, r, bc)) lowest = r;
    drop = drop && has;
    if (drop) {
      s[BXP] = s[FX] + 16 * bc + 4;
      s[BYP] = s[FY] + 18 * lowest + 10;
    }
    bomb = bomb || drop;
    s[BYP] += 2 * bomb;
    const bool hitp = bomb && s[BYP] >= 185 && s[BYP] < 193 && s[BXP] >= s[PX] && s[BXP] < s[PX] + 7;
    s[LIVES] -= hitp;
    s[BOMB] = bomb && !hitp && s[BYP] < 196;
    s[SHOT] = shot;
    if (!any_bits(s + ALIVE, AR * AC)) {      // wave cleared: a new formation marches in from the top
      fill_bits(s + ALIVE, AR * AC);
      s[FX] = 22;
      s[FY] = 40;
      s[FDIR] = 1;
    }
    return reward;
  }
  static DEVI bool over(const int* s) {
    int lowest_row = -1;
    for (int r = 0; r < AR; ++r)
      for (int c = 0; c < AC; ++c)
        if (alive(s, r, c)) lowest_row = r;
    const bool invaded = s[FY] + 18 * lowest_row + 10 >= 180;
    return s[LIVES] <= 0 || invaded;
  }
  static DEVI void scene(const int* s, int16_t* r) {
    rect(r, 0, 195, 0, 2, 160);
    for (int i = 0; i < AR * AC; ++i)
      rect(r, 1 + i, s[FY] + 18 * (i / AC), s[FX] + 16 * (i % AC), getbit(s + ALIVE, i) ? 10 : 0, 8);
    rect(r, 1 + AR * AC, 185, s[PX], 8, 7);
    rect(r, 2 + AR * AC, s[SY], s[SX], s[SHOT] ? 6 : 0, 1);
    rect(r, 3 + AR * AC, s[BYP], s[BXP], s[BOMB] ? 6 : 0, 1);
  }
};

// --------------------------------------------------------------------------- Alien / MsPacman
// 13 x 11 maze (envs/atari_games.py MAZE): bit x of row y set = wall
__constant__ int MAZE_ROWS[11] = {0x1FFF, 0x1041, 0x175D, 0x1001, 0x15F5, 0x1445, 0x175D, 0x1001, 0x175D, 0x1041, 0x1FFF};
struct AlienBase {
  static constexpr int H = 11, W = 13, NA = 3, CW = 12, CH = 16, Y0 = 20, X0 = 2, NWALL = 77;
  enum { PY, PX, AY, AX = AY + NA, LIVES = AX + NA, TICK, DOTS, COUNTER = DOTS + 5, STEPS, EPRET, NS };
  static constexpr int R = NWALL + H * W + 1 + NA;
  static DEVI bool wall(int y, int x) { return (MAZE_ROWS[clampi(y, 0, H - 1)] >> clampi(x, 0, W - 1)) & 1; }
  static DEVI int dy(int j) { return j == 1 ? -1 : (j == 4 ? 1 : 0); }       // none, up, right, left, down
  static DEVI int dx(int j) { return j == 2 ? 1 : (j == 3 ? -1 : 0); }
  static DEVI int amap(int a) {
    const int m[18] = {0, 0, 1, 2, 3, 4, 1, 1, 4, 4, 1, 2, 3, 4, 1, 1, 4, 4};
    return m[a];
  }
  static DEVI void start(int k, int& y, int& x) {
    y = k == 2 ? 9 : 1;
    x = k == 0 ? 1 : (k == 1 ? 11 : 6);
  }
  static DEVI void reset(int* s, const Rng&) {
    for (int i = 0; i < 5; ++i) s[DOTS + i] = 0;
    for (int i = 0; i < H * W; ++i) setbit(s + DOTS, i, !wall(i / W, i % W));
    s[PY] = 7;
    s[PX] = 6;
    setbit(s + DOTS, 7 * W + 6, false);
    for (int k = 0; k < NA; ++k) start(k, s[AY + k], s[AX + k]);
    s[LIVES] = 3;
    s[TICK] = 0;
  }
  static DEVI int physics(int* s, int a, const Rng& g) {
    s[TICK] += 1;
    const bool step_now = fmodi(s[TICK], 2) == 0;
    const int di = amap(a);
    const int ny = s[PY] + dy(di), nx = s[PX] + dx(di);
    if (step_now && !wall(ny, nx)) {
      s[PY] = ny;
      s[PX] = nx;
    }
    const int cell = s[PY] * W + s[PX];
    int reward = getbit(s + DOTS, cell) ? 10 : 0;
    setbit(s + DOTS, cell, false);
    const bool amove = fmodi(s[TICK], 4) == 0;
    for (int k = 0; k < NA; ++k) {
      const int y = s[AY + k], x = s[AX + k];
      int by = y, bx = x, bd = 1 << 20;
      const int r = g.rand(6 + k, 4);
      for (int j = 1; j < 5; ++j) {
        const int cy = y + dy(j), cx = x + dx(j);
        int d = iabs(cy - s[PY]) + iabs(cx - s[PX]);
        if (r == j - 1) d -= 2;
        if (!wall(cy, cx) && d < bd) {
          by = cy;
          bx = cx;
          bd = d;
        }
      }
      if (amove) {
        s[AY + k] = by;
        s[AX + k] = bx;
      }
    }
    bool caught = false;
    for (int k = 0; k < NA; ++k) caught |= s[AY + k] == s[PY] && s[AX + k] == s[PX];
    s[LIVES] -= caught;
    if (caught)
      for (int k = 0; k < NA; ++k) start(k, s[AY + k], s[AX + k]);
    if (!any_bits(s + DOTS, H * W)) reward += 500;
    return reward;
  }
  static DEVI bool over(const int* s) { return s[LIVES] <= 0 || !any_bits(s + DOTS, H * W); }
  static DEVI void scene(const int* s, int16_t* r) {
    int n = 0;
    for (int i = 0; i < H * W; ++i)
      if (wall(i / W, i % W)) rect(r, n++, Y0 + (i / W) * CH, X0 + (i % W) * CW, CH, CW);
    for (int i = 0; i < H * W; ++i)
      rect(r, NWALL + i, Y0 + (i / W) * CH + CH / 2, X0 + (i % W) * CW + CW / 2, getbit(s + DOTS, i) ? 2 : 0, 2);
    rect(r, NWALL + H * W, Y0 + s[PY] * CH + 3, X0 + s[PX] * CW + 3, 10, 6);
    for (int k = 0; k < NA; ++k) rect(r, NWALL + H * W + 1 + k, Y0 + s[AY + k] * CH + 2, X0 + s[AX + k] * CW + 2, 12, 8);
  }
};
struct Alien : AlienBase {};
struct MsPacman : AlienBase {};

// --------------------------------------------------------------------------- Centipede
struct Centipede {
  static constexpr int NSEG = 10, GH = 20, GW = 16;
  enum { MUSH, SY = MUSH + 10, SX = SY + NSEG, SDIR = SX + NSEG, SALIVE = SDIR + NSEG, PX, SHOT, SHX, SHY, LIVES, TICK,
         COUNTER, STEPS, EPRET, NS };
  static constexpr int R = GH * GW + NSEG + 2;
  static DEVI int amap_h(int a) {
    const int m[18] = {0, 0, 0, 1, -1, 0, 1, -1, 1, -1, 0, 0, 1, -1, 0, 1, -1, 1};
    return m[a];
  }
  static DEVI bool afire(int a) { return a == 1 || a >= 10; }
  static DEVI bool salive(const int* s, int k) { return (s[SALIVE] >> k) & 1; }
  static DEVI void reset(int* s, const Rng& g) {
    for (int i = 0; i < 10; ++i) s[MUSH + i] = 0;
    for (int k = 0; k < GH * GW / 16; ++k) {
      const int r = g.rand(10 + k, 100);
      const int pos = min(k * 16 + r % 16, GH * GW - 1);
      if (pos < (GH - 3) * GW) setbit(s + MUSH, pos, r < 60);
    }
    for (int k = 0; k < NSEG; ++k) {
      s[SY + k] = 0;
      s[SX + k] = max(GW - 1 - k, 0);
      s[SDIR + k] = -1;
    }
    s[SALIVE] = (1 << NSEG) - 1;
    s[PX] = 76;
    s[SHOT] = 0;
    s[LIVES] = 3;
    s[TICK] = 0;
  }
  static DEVI int physics(int* s, int a, const Rng&) {
    s[PX] = clampi(s[PX] + 2 * amap_h(a), 4, 152);
    bool shot = s[SHOT] != 0;
    const bool fire = afire(a) && !shot;
    if (fire) {
      s[SHX] = s[PX] + 2;
      s[SHY] = 180;
    }
    shot = shot || fire;
    s[SHY] -= 6 * shot;
    shot = shot && s[SHY] > 20;
    const int gy = clampi(fdiv(s[SHY] - 20, 8), 0, GH - 1), gx = clampi(fdiv(s[SHX], 10), 0, GW - 1);
    const int cell = gy * GW + gx;
    const bool m0 = getbit(s + MUSH, cell);
    const bool hm = shot && m0;
    setbit(s + MUSH, cell, m0 && !hm);
    int reward = hm;
    shot = shot && !hm;
    int hits = 0, alive = s[SALIVE];
    for (int k = 0; k < NSEG; ++k) {
      const bool hs = shot && ((alive >> k) & 1) && s[SY + k] == gy && s[SX + k] == gx;
      hits += hs;
      if (hs) alive &= ~(1 << k);
    }
    reward += 10 * hits;
    s[SALIVE] = alive;
    if (hits) setbit(s + MUSH, cell, true);
    shot = shot && hits == 0;
    s[TICK] += 1;
    const bool tick3 = fmodi(s[TICK], 3) == 0;
    for (int k = 0; k < NSEG; ++k) {
      const bool mv = tick3 && salive(s, k);
      const int nx = s[SX + k] + s[SDIR + k];
      const bool blocked = nx < 0 || nx >= GW || getbit(s + MUSH, s[SY + k] * GW + clampi(nx, 0, GW - 1));
      if (mv && blocked) {
        s[SY + k] = min(s[SY + k] + 1, GH - 1);
        s[SDIR + k] = -s[SDIR + k];
      }
      if (mv && !blocked) s[SX + k] = nx;
    }
    bool reach = false;
    for (int k = 0; k < NSEG; ++k) reach |= salive(s, k) && s[SY + k] >= GH - 1;
    s[LIVES] -= reach;
    if (reach)
      for (int k = 0; k < NSEG; ++k) {
        s[SY + k] = 0;
        s[SX + k] = max(GW - 1 - k, 0);
        s[SDIR + k] = -1;
      }
    if (s[SALIVE] == 0) {
      s[SALIVE] = (1 << NSEG) - 1;
      for (int k = 0; k < NSEG; ++k) s[SY + k] = 0;
    }
    s[SHOT] = shot;
    return reward;
  }
  static DEVI bool over(const int* s) { return s[LIVES] <= 0; }
  static DEVI void scene(const int* s, int16_t* r) {
    for (int i = 0; i < GH * GW; ++i)
      rect(r, i, 20 + (i / GW) * 8, (i % GW) * 10, getbit(s + MUSH, i) ? 8 : 0, 10);
    for (int k = 0; k < NSEG; ++k)
      rect(r, GH * GW + k, 20 + s[SY + k] * 8 + 1, s[SX + k] * 10 + 1, salive(s, k) ? 6 : 0, 8);
    rect(r, GH * GW + NSEG, 184, s[PX], 8, 4);
    rect(r, GH * GW + NSEG + 1, s[SHY], s[SHX], s[SHOT] ? 6 : 0, 1);
  }
};

// --------------------------------------------------------------------------- driver
// mode 0: agent step (actions), mode 1: reset_where(mask).  One thread per env.
template <class G>
__global__ __launch_bounds__(64) void game_step_kernel(int* __restrict__ state, const int* __restrict__ actions,
                                                       const uint8_t* __restrict__ mask, int mode, int n_actions, int N,
                                                       uint32_t seed, uint32_t id_base, int frameskip, int max_steps,
                                                       float* __restrict__ reward, uint8_t* __restrict__ done,
                                                       float* __restrict__ epret, int16_t* __restrict__ rects) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  int s[G::NS];
  int* row = state + (long)e * G::NS;
  for (int i = 0; i < G::NS; ++i) s[i] = row[i];
  Rng g{seed, id_base + (uint32_t)e, (uint32_t)s[G::COUNTER]};   // RNG identity: the global env index
  if (mode == 0) {
    int a = actions[e];
    if (a >= n_actions || a < 0) a = 0;
    int rw = 0;
    for (int f = 0; f < frameskip; ++f) rw += G::physics(s, a, g);
    s[G::COUNTER] += 1;
    s[G::STEPS] += 1;
    s[G::EPRET] += rw;
    const bool d = G::over(s) || s[G::STEPS] >= max_steps;
    reward[e] = (float)rw;
    done[e] = d;
    epret[e] = d ? (float)s[G::EPRET] : 0.f;
    if (d) {
      g.counter = (uint32_t)s[G::COUNTER];
      G::reset(s, g);
      s[G::STEPS] = 0;
      s[G::EPRET] = 0;
      s[G::COUNTER] += 1;
    }
  } else if (mask[e]) {
    G::reset(s, g);
    s[G::STEPS] = 0;
    s[G::EPRET] = 0;
    s[G::COUNTER] += 1;
  }
  for (int i = 0; i < G::NS; ++i) row[i] = s[i];
  G::scene(s, rects + (long)e * G::R * 4);
}

template <class G>
static int launch(void* state, const void* actions, const void* mask, int mode, int n_actions, int N, uint32_t seed,
                  uint32_t id_base, int frameskip, int max_steps, void* reward, void* done, void* epret, void* rects, hipStream_t st) {
  game_step_kernel<G><<<(N + 63) / 64, 64, 0, st>>>((int*)state, (const int*)actions, (const uint8_t*)mask, mode,
                                                    n_actions, N, seed, id_base, frameskip, max_steps, (float*)reward,
                                                    (uint8_t*)done, (float*)epret, (int16_t*)rects);
  return (int)hipGetLastError();
}

}  // namespace games

// game ids: 0 Breakout, 1 SpaceInvaders, 2 Alien, 3 MsPacman, 4 Centipede
extern "C" int game_layout(int game, int* ns, int* nrects) {
  using namespace games;
  switch (game) {
    case 0: *ns = Breakout::NS; *nrects = Breakout::R; return 0;
    case 1: *ns = SpaceInvaders::NS; *nrects = SpaceInvaders::R; return 0;
    case 2: *ns = Alien::NS; *nrects = Alien::R; return 0;
    case 3: *ns = MsPacman::NS; *nrects = MsPacman::R; return 0;
    case 4: *ns = Centipede::NS; *nrects = Centipede::R; return 0;
  }
  return -1;
}

extern "C" int launch_game_step(int game, void* state, const void* actions, const void* mask, int mode, int n_actions,
                                int N, uint32_t seed, uint32_t id_base, int frameskip, int max_steps, void* reward, void* done,
                                void* epret, void* rects, hipStream_t st) {
  using namespace games;
  switch (game) {
    case 0: return launch<Breakout>(state, actions, mask, mode, n_actions, N, seed, id_base, frameskip, max_steps, reward, done, epret, rects, st);
    case 1: return launch<SpaceInvaders>(state, actions, mask, mode, n_actions, N, seed, id_base, frameskip, max_steps, reward, done, epret, rects, st);
    case 2: return launch<Alien>(state, actions, mask, mode, n_actions, N, seed, id_base, frameskip, max_steps, reward, done, epret, rects, st);
    case 3: return launch<MsPacman>(state, actions, mask, mode, n_actions, N, seed, id_base, frameskip, max_steps, reward, done, epret, rects, st);
    case 4: return launch<Centipede>(state, actions, mask, mode, n_actions, N, seed, id_base, frameskip, max_steps, reward, done, epret, rects, st);
  }
  return -1;
}
