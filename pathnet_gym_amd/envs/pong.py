"""Synthetic Atari-style Pong, vectorised on device (the headline workload).

gym/ALE are not installed in this image, so the
framework ships its own Pong with the Atari screen geometry: 210x160x3 uint8
RGB frames, the 6-action Pong action set (NOOP, FIRE, RIGHT=up, LEFT=down,
RIGHTFIRE, LEFTFIRE), +1/-1 rewards, episode ends when a side reaches 21
(or after 10000 agent steps, gym's Pong TimeLimit).  A scripted opponent
tracks the ball with a capped speed so the game is winnable.

Physics is INTEGER (1/16 px fixed point) and the RNG is the counter-based
Wang hash of ``envs/base.py``, so the torch implementation below and the
fused HIP kernel (``csrc/envs.hip``: physics + render + gray + bilinear
resize + frame-stack push in one launch) produce bit-identical frames.

Preprocessing follows ``game_state.py:37-51,66,78``: gray (cv2 fixed-point
luma; ``gray="bgr"`` reproduces the reference's BGR2GRAY-on-RGB quirk),
bilinear resize to H=160, W=120 (cv2 INTER_LINEAR half-pixel mapping with
11-bit fixed-point weights), stack 4 frames newest-last along channels.  The
model consumes the uint8 stack and folds the /255 into its first layer.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .base import VecEnv, env_rand_u32

# ---- screen / game constants (pixels) ----
SCREEN_H, SCREEN_W = 210, 160
OBS_H, OBS_W = 160, 120
TOP, BOTTOM = 34, 194
WALL_TOP0, WALL_BOT1 = 24, 210
PADDLE_H, PADDLE_W = 16, 4
BALL_W, BALL_H = 2, 4
PLAYER_X, CPU_X = 140, 16
U = 16                         # subpixel units
PLAYER_SPEED = 40              # units / subframe
CPU_SPEED = 28
SERVE_VX = 32
MAX_VX = 64
MAX_VY = 40
SERVE_DELAY = 16               # subframes
WIN_SCORE = 21
MAX_STEPS = 10000

COLOR_BG = (144, 72, 17)
COLOR_WALL = (236, 236, 236)
COLOR_CPU = (213, 130, 74)
COLOR_PLAYER = (92, 186, 92)
COLOR_BALL = (236, 236, 236)

# 3x5 digit font, row-major bits (bit 14 = top-left)
DIGITS = [0b111101101101111, 0b010110010010111, 0b111001111100111, 0b111001111001111,
          0b101101111001001, 0b111100111001111, 0b111100111101111, 0b111001001001001,
          0b111101111101111, 0b111101111001111]
DIGIT_SCALE = 4
SCORE_ROW0 = 2
CPU_SCORE_X = (24, 40)
PLAYER_SCORE_X = (104, 120)

# state columns
BX, BY, VX, VY, PY, CY, PS, CS, SERVE, STEPS, EPRET = range(11)
NSTATE = 12

GRAY_RGB = (4899, 9617, 1868)     # cv2 fixed-point luma (R, G, B), >>14


def linear_table(dst: int, src: int):
    """cv2 INTER_LINEAR source indices + 11-bit weights for one axis."""
    scale = src / dst
    s0 = np.zeros(dst, np.int32)
    s1 = np.zeros(dst, np.int32)
    c0 = np.zeros(dst, np.int32)
    for d in range(dst):
        f = (d + 0.5) * scale - 0.5
        s = math.floor(f)
        f -= s
        if s < 0:
            s, f = 0, 0.0
        if s >= src - 1:
            s, f = src - 1, 0.0
        s0[d] = s
        s1[d] = min(s + 1, src - 1)
        c0[d] = int(round((1.0 - f) * 2048))
    c1 = 2048 - c0
    return s0, s1, c0, c1


def resize_tables():
    """(rows: s0,s1,c0,c1 [160]), (cols: s0,s1,c0,c1 [120]) as one int32 [8, 160] array."""
    ry = linear_table(OBS_H, SCREEN_H)
    rx = linear_table(OBS_W, SCREEN_W)
    t = np.zeros((8, OBS_H), np.int32)
    for i in range(4):
        t[i, :OBS_H] = ry[i]
        t[4 + i, :OBS_W] = rx[i]
    return t


def gray_weights(gray: str):
    r, g, b = GRAY_RGB
    return (b, g, r) if gray == "bgr" else (r, g, b)


def _digit_on(score, rows, cols, x0s):
    """bool [N, H, W]: pixel lies on a lit segment of the 2-digit score."""
    on = torch.zeros(score.shape[0], rows.shape[1], cols.shape[2], dtype=torch.bool, device=score.device)
    font = torch.tensor(DIGITS, dtype=torch.int64, device=score.device)
    tens = torch.div(score, 10, rounding_mode="trunc")
    ones = score - tens * 10
    for which, dig in ((0, tens), (1, ones)):
        x0 = x0s[which]
        lc = torch.div(cols - x0, DIGIT_SCALE, rounding_mode="floor")
        lr = torch.div(rows - SCORE_ROW0, DIGIT_SCALE, rounding_mode="floor")
        inside = (lc >= 0) & (lc < 3) & (lr >= 0) & (lr < 5)
        bit = 14 - (lr.clamp(0, 4) * 3 + lc.clamp(0, 2))
        bits = font[dig.long()][:, None, None]
        lit = ((bits >> bit) & 1) == 1
        show = (dig > 0) | torch.tensor(which == 1, device=score.device)
        on |= inside & lit & show[:, None, None]
    return on


def render_rgb(state: torch.Tensor) -> torch.Tensor:
    """[N, NSTATE] int64 -> [N, 210, 160, 3] uint8 RGB frames."""
    N = state.shape[0]
    dev = state.device
    rows = torch.arange(SCREEN_H, device=dev)[None, :, None]
    cols = torch.arange(SCREEN_W, device=dev)[None, None, :]
    img = torch.empty(N, SCREEN_H, SCREEN_W, 3, dtype=torch.uint8, device=dev)
    img[:] = torch.tensor(COLOR_BG, dtype=torch.uint8, device=dev)

    def paint(mask, color):
        img[mask] = torch.tensor(color, dtype=torch.uint8, device=dev)

    wall = ((rows >= WALL_TOP0) & (rows < TOP)) | (rows >= BOTTOM)
    paint(wall.expand(N, SCREEN_H, SCREEN_W), COLOR_WALL)
    cy = torch.div(state[:, CY], U, rounding_mode="floor")[:, None, None]
    py = torch.div(state[:, PY], U, rounding_mode="floor")[:, None, None]
    cpu = (cols >= CPU_X) & (cols < CPU_X + PADDLE_W) & (rows >= cy) & (rows < cy + PADDLE_H)
    paint(cpu, COLOR_CPU)
    ply = (cols >= PLAYER_X) & (cols < PLAYER_X + PADDLE_W) & (rows >= py) & (rows < py + PADDLE_H)
    paint(ply, COLOR_PLAYER)
    bx = torch.div(state[:, BX], U, rounding_mode="floor")[:, None, None]
    by = torch.div(state[:, BY], U, rounding_mode="floor")[:, None, None]
    vis = (state[:, SERVE] == 0)[:, None, None]
    ball = vis & (cols >= bx) & (cols < bx + BALL_W) & (rows >= by) & (rows < by + BALL_H)
    paint(ball, COLOR_BALL)
    paint(_digit_on(state[:, CS], rows, cols, CPU_SCORE_X), COLOR_CPU)
    paint(_digit_on(state[:, PS], rows, cols, PLAYER_SCORE_X), COLOR_PLAYER)
    return img


def preprocess_frames(rgb: torch.Tensor, tables: torch.Tensor, gray: str = "rgb") -> torch.Tensor:
    """[N,210,160,3] uint8 -> [N,160,120] uint8: fixed-point gray + bilinear resize (K15)."""
    wr, wg, wb = gray_weights(gray)
    x = rgb.to(torch.int64)
    g = (x[..., 0] * wr + x[..., 1] * wg + x[..., 2] * wb + 8192) >> 14   # [N,210,160]
    t = tables.to(rgb.device).long()
    ys0, ys1, cy0, cy1 = t[0], t[1], t[2], t[3]
    xs0, xs1, cx0, cx1 = t[4, :OBS_W], t[5, :OBS_W], t[6, :OBS_W], t[7, :OBS_W]
    r0 = g[:, ys0]          # [N,160,160]
    r1 = g[:, ys1]
    a = r0[:, :, xs0] * cx0 + r0[:, :, xs1] * cx1    # [N,160,120]
    b = r1[:, :, xs0] * cx0 + r1[:, :, xs1] * cx1
    out = (a * cy0[None, :, None] + b * cy1[None, :, None] + (1 << 21)) >> 22
    return out.clamp(0, 255).to(torch.uint8)


class PongVec(VecEnv):
    id = "Pong"
    reward_threshold = 18.0          # "solved" criterion used for generations-to-solve
    max_episode_steps = MAX_STEPS

    def __init__(self, num_envs: int, device="cpu", seed: int = 0, frameskip: int = 4,
                 gray: str = "rgb", backend: str = "torch", no_op_max: int = 6):
        self.num_envs = num_envs
        self.num_actions = 6
        self.obs_shape = (OBS_H, OBS_W, 4)
        self.obs_dtype = torch.uint8
        self.device = torch.device(device)
        self.frameskip = frameskip
        self.gray = gray
        self.backend = backend
        self.no_op_max = no_op_max
        self.state = torch.zeros(num_envs, NSTATE, dtype=torch.int64, device=self.device)
        self.counter = torch.zeros(num_envs, dtype=torch.int64, device=self.device)
        self.env_id = torch.arange(num_envs, dtype=torch.int64, device=self.device)
        self.tables = torch.from_numpy(resize_tables()).to(self.device)
        self.obs = torch.zeros(num_envs, OBS_H, OBS_W, 4, dtype=torch.uint8, device=self.device)
        self.seed(seed)

    def seed(self, seed: int):
        self.seed_int = seed & 0xFFFFFFFF
        self._seed = torch.tensor(self.seed_int, dtype=torch.int64, device=self.device)
        self.counter.zero_()

    # -- rng -------------------------------------------------------------------
    def _rand(self, stream: int, n: int) -> torch.Tensor:
        """uniform integer in [0, n) per env (consumes counter at the caller)."""
        h = env_rand_u32(self._seed, self.env_id, self.counter, stream)
        return h % n

    # -- dynamics --------------------------------------------------------------
    def _serve(self, st, mask):
        """Launch the ball from the centre for envs in mask (stream 0..2)."""
        y = (TOP + 20 + self._rand(0, BOTTOM - TOP - 40 - BALL_H)) * U
        dirn = torch.where(self._rand(1, 2) == 0, -SERVE_VX, SERVE_VX)
        vy = self._rand(2, 49) - 24
        st[:, BX] = torch.where(mask, torch.full_like(st[:, BX], 78 * U), st[:, BX])
        st[:, BY] = torch.where(mask, y, st[:, BY])
        st[:, VX] = torch.where(mask, dirn, st[:, VX])
        st[:, VY] = torch.where(mask, vy, st[:, VY])

    def _subframe(self, st, up, down):
        reward = torch.zeros(st.shape[0], dtype=torch.int64, device=st.device)
        # player paddle
        py = st[:, PY] - up * PLAYER_SPEED + down * PLAYER_SPEED
        st[:, PY] = py.clamp(TOP * U, (BOTTOM - PADDLE_H) * U)
        # cpu paddle: chase the ball when it approaches, else re-centre
        serving = st[:, SERVE] > 0
        chase = (~serving) & (st[:, VX] < 0)
        target = torch.where(chase, st[:, BY] + (BALL_H * U) // 2 - (PADDLE_H * U) // 2,
                             torch.full_like(st[:, CY], ((TOP + BOTTOM) // 2 - PADDLE_H // 2) * U))
        dy = (target - st[:, CY]).clamp(-CPU_SPEED, CPU_SPEED)
        st[:, CY] = (st[:, CY] + dy).clamp(TOP * U, (BOTTOM - PADDLE_H) * U)
        # serve countdown
        st[:, SERVE] = torch.where(serving, st[:, SERVE] - 1, st[:, SERVE])
        launch = serving & (st[:, SERVE] == 0)
        self._serve(st, launch)
        move = ~serving
        bx, by, vx, vy = st[:, BX], st[:, BY], st[:, VX], st[:, VY]
        nx = bx + vx
        ny = by + vy
        # walls
        hit_top = ny < TOP * U
        ny = torch.where(hit_top, 2 * TOP * U - ny, ny)
        vy = torch.where(hit_top, -vy, vy)
        hit_bot = ny + BALL_H * U > BOTTOM * U
        ny = torch.where(hit_bot, 2 * (BOTTOM - BALL_H) * U - ny, ny)
        vy = torch.where(hit_bot, -vy, vy)
        # player paddle face
        face = PLAYER_X * U
        cross = (vx > 0) & (bx + BALL_W * U <= face) & (nx + BALL_W * U > face)
        over = (ny + BALL_H * U > st[:, PY]) & (ny < st[:, PY] + PADDLE_H * U)
        hit_p = cross & over
        off = (ny + (BALL_H * U) // 2) - (st[:, PY] + (PADDLE_H * U) // 2)
        nvy = torch.div(off * 3, 16, rounding_mode="trunc").clamp(-MAX_VY, MAX_VY)
        nx = torch.where(hit_p, torch.full_like(nx, face - BALL_W * U), nx)
        vx = torch.where(hit_p, -(vx.abs() + 1).clamp(max=MAX_VX), vx)
        vy = torch.where(hit_p, nvy, vy)
        # cpu paddle face
        cface = (CPU_X + PADDLE_W) * U
        ccross = (vx < 0) & (bx >= cface) & (nx < cface)
        cover = (ny + BALL_H * U > st[:, CY]) & (ny < st[:, CY] + PADDLE_H * U)
        hit_c = ccross & cover
        coff = (ny + (BALL_H * U) // 2) - (st[:, CY] + (PADDLE_H * U) // 2)
        cvy = torch.div(coff * 3, 16, rounding_mode="trunc").clamp(-MAX_VY, MAX_VY)
        nx = torch.where(hit_c, torch.full_like(nx, cface), nx)
        vx = torch.where(hit_c, (vx.abs() + 1).clamp(max=MAX_VX), vx)
        vy = torch.where(hit_c, cvy, vy)
        # scoring
        p_pt = move & (nx + BALL_W * U < 0)
        c_pt = move & (nx > SCREEN_W * U)
        reward = torch.where(p_pt, 1, torch.where(c_pt, -1, 0)).to(torch.int64)
        st[:, PS] += p_pt.long()
        st[:, CS] += c_pt.long()
        scored = p_pt | c_pt
        st[:, SERVE] = torch.where(scored, torch.full_like(st[:, SERVE], SERVE_DELAY), st[:, SERVE])
        st[:, BX] = torch.where(move, nx, st[:, BX])
        st[:, BY] = torch.where(move, ny, st[:, BY])
        st[:, VX] = torch.where(move, vx, st[:, VX])
        st[:, VY] = torch.where(move, vy, st[:, VY])
        return reward

    def _reset_state(self, mask):
        st = self.state
        z = torch.zeros_like(st[:, 0])
        mid = torch.full_like(z, ((TOP + BOTTOM) // 2 - PADDLE_H // 2) * U)
        for c in (PS, CS, STEPS, EPRET):
            st[:, c] = torch.where(mask, z, st[:, c])
        st[:, PY] = torch.where(mask, mid, st[:, PY])
        st[:, CY] = torch.where(mask, mid, st[:, CY])
        # random no-op start: a random serve delay (ref: U{0..no_op_max} no-op steps, game_state.py:57-60)
        delay = 1 + self._rand(3, (self.no_op_max + 1) * self.frameskip)
        st[:, SERVE] = torch.where(mask, delay, st[:, SERVE])
        st[:, BX] = torch.where(mask, torch.full_like(z, 78 * U), st[:, BX])
        st[:, BY] = torch.where(mask, torch.full_like(z, (TOP + BOTTOM) // 2 * U), st[:, BY])
        st[:, VX] = torch.where(mask, z, st[:, VX])
        st[:, VY] = torch.where(mask, z, st[:, VY])

    def frame(self) -> torch.Tensor:
        """Current preprocessed single frame [N,160,120] uint8."""
        return preprocess_frames(render_rgb(self.state), self.tables, self.gray)

    def render(self) -> torch.Tensor:
        """RGB frames [N,210,160,3] (gym ``render('rgb_array')``)."""
        return render_rgb(self.state)

    def stagger_scores(self, max_left: int = 3):
        """Benchmark helper (bench.py): start every env's CURRENT episode at a random late score -- the CPU needs
        1..max_left more points and the player has a random 0..20 -- so episodes end, fitness windows fill and GA
        tournaments fire within the first few hundred agent steps instead of after a whole 21-point game.  Frame
        work per step is unchanged; only the first episode of each env is shortened.  Call before the first
        engine update (the HIP state buffer is updated in place, its address stays the one the graphs use)."""
        if hasattr(self, "_st32"):
            from ..ops import envs as henv
            henv.pong_sync_from_device(self)
        left = self._rand(7, max_left) + 1
        self.state[:, CS] = WIN_SCORE - left
        self.state[:, PS] = self._rand(8, WIN_SCORE)
        self.state[:, EPRET] = self.state[:, PS] - self.state[:, CS]
        self.counter += 1
        if hasattr(self, "_st32"):
            self._st32.copy_(self.state.to(torch.int32))
            self._ctr32.copy_(self.counter.to(torch.int32))

    def reset(self):
        allm = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
        self.reset_where(allm)
        return self.obs.clone()

    def reset_where(self, mask):
        hip_state = hasattr(self, "_st32")
        if hip_state:
            from ..ops import envs as henv
            henv.pong_sync_from_device(self)
        self._reset_state(mask)
        self.counter += mask.long()
        f = self.frame()
        stack = f[..., None].expand(-1, -1, -1, 4)
        self.obs = torch.where(mask[:, None, None, None], stack, self.obs)
        if hip_state:
            henv.pong_sync_to_device(self)

    # the ring step takes an env range (the split rollout steps one path group per launch, runtime/engine.py)
    ring_ranges = True

    # ... and the heads + sampling of each env's sample folded into its step (runtime/engine.py fused env heads)
    ring_heads = True

    def step_ring_heads_into(self, feat, flat, heads, logits, value, actions, seed, ctr, t, T, row_base, frames, slot,
                             fc_in, fc_out, reward, done, epret):
        """Engine frame-ring step with the actor-critic heads of step t folded in (ops/envs.py)."""
        from ..ops import envs as henv
        henv.pong_heads_step_ring_into(self, feat, flat, heads, logits, value, actions, seed, ctr, t, T, row_base,
                                       frames, slot, fc_in, fc_out, reward, done, epret)

    def step_ring_into(self, actions, frames, slot, fc_in, fc_out, reward, done, epret, b0: int = 0, b1=None):
        """Engine frame-ring step (HIP only): write frames[:, slot] + the next first valid channel, envs [b0, b1)."""
        from ..ops import envs as henv
        henv.pong_step_ring_into(self, actions, frames, slot, fc_in, fc_out, reward, done, epret, b0=b0, b1=b1)

    def step(self, actions: torch.Tensor):
        if self.backend == "hip":
            from ..ops import envs as henv
            return henv.pong_step(self, actions, self.obs)
        a = actions.long()
        a = torch.where(a >= self.num_actions, torch.zeros_like(a), a)   # game_state.py:38-39 remap
        up = ((a == 2) | (a == 4)).long()
        down = ((a == 3) | (a == 5)).long()
        st = self.state
        reward = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)
        for _ in range(self.frameskip):
            reward += self._subframe(st, up, down)
        self.counter += 1
        st[:, STEPS] += 1
        st[:, EPRET] += reward
        done = (st[:, PS] >= WIN_SCORE) | (st[:, CS] >= WIN_SCORE) | (st[:, STEPS] >= self.max_episode_steps)
        ep_return = torch.where(done, st[:, EPRET], torch.zeros_like(reward)).float()
        # auto-reset finished envs (physics only), then render ONE frame for everybody
        self._reset_state(done)
        self.counter += done.long()
        f = self.frame()
        pushed = torch.cat([self.obs[..., 1:], f[..., None]], dim=3)
        fresh = f[..., None].expand(-1, -1, -1, 4)
        self.obs = torch.where(done[:, None, None, None], fresh, pushed)
        return self.obs.clone(), reward.float(), done, {"episode_return": ep_return}
