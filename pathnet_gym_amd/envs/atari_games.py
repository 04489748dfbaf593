"""Synthetic Atari-style games for the multi-task suite (Pong -> Breakout -> SpaceInvaders -> Alien).

BASELINE.json config 5 names a 4-task Atari suite; the reference's task
lists are Atari ids (``constants.py:12-15``: MsPacman, Alien, Centipede).
ALE is not available in this image, so each game is a small on-device
vectorised re-creation with the Atari screen geometry (210x160x3 uint8 RGB)
and the same preprocessing/stacking pipeline as Pong
(``envs/pong.py:preprocess_frames``):

* ``Breakout``      4 actions (NOOP, FIRE, RIGHT, LEFT); 6x18 bricks worth
                    7/7/4/4/1/1 by row, 5 lives, FIRE serves.
* ``SpaceInvaders`` 6 actions (NOOP, FIRE, RIGHT, LEFT, RIGHTFIRE, LEFTFIRE);
                    6x6 marching formation worth 30..5 by row, one player
                    shot and one alien bomb in flight, 3 lives; a cleared
                    wave is followed by a new one (the game ends on lives, an
                    invasion or 4500 agent steps: one wave alone was cleared by
                    a random policy).
* ``Alien`` / ``MsPacman``  18 / 9 actions; 13x11 maze with eggs (+10) and
                    three chasing aliens, 3 lives, clearing the maze +500.
* ``Centipede``     18 actions; a 10-segment centipede snaking down through
                    mushrooms, shots worth 10 (segment) / 1 (mushroom).

All dynamics are integer and the randomness uses the counter-based hash
RNG of ``envs/base.py`` (same convention as Pong).  The game logic runs as
torch ops on any device; a step has no host synchronisation and commits its
state in place, so the engine captures it in the rollout hipGraph like the
HIP envs.  On the GPU the frame is not rendered by torch at all: each game
describes its scene as a rectangle list (``Scene``) that one fused kernel
rasterises, preprocesses and pushes into the frame stack.

With ``backend="hip"`` on a GPU the game logic itself runs in ``csrc/games.hip``
(one thread per env: physics sub-frames, reward/done, auto-reset and the scene),
so an agent step is two launches; the torch code above stays the bit-exact
oracle (``tests/test_games_hip.py``).  The packed int32 kernel state is then the
source of truth and ``sync_from_device()`` refreshes the torch state tensors.
"""
from __future__ import annotations

import torch

from .base import VecEnv, env_rand_u32
from .pong import OBS_H, OBS_W, SCREEN_H, SCREEN_W, preprocess_frames, resize_tables

BG = (0, 0, 0)


class Scene:
    """Ordered list of per-env rectangles (painter's order) with one RGB colour per rectangle slot.

    Games describe a frame with ``add`` (one rectangle per env) and ``add_many`` (a batch of R
    rectangles, e.g. a brick grid); hidden rectangles have h == 0.  The same scene feeds the torch
    renderer (``PixelGameVec.draw``, the oracle) and the fused HIP rasteriser
    (``csrc/preprocess.hip:rects_stack_push``).
    """

    def __init__(self, n: int, device):
        self.n, self.device = n, device
        self.parts, self.colors = [], []

    def _t(self, v):
        if isinstance(v, torch.Tensor):
            return v.to(torch.int64)
        # python scalar -> device fill kernel (no host->device copy: capturable in a hipGraph)
        return torch.full((), int(v), dtype=torch.int64, device=self.device)

    def add(self, y0, x0, h, w, color, visible=None):
        y0, x0, h, w = [self._t(v).reshape(-1).expand(self.n) for v in (y0, x0, h, w)]
        if visible is not None:
            h = torch.where(visible, h, torch.zeros_like(h))
        self.parts.append(torch.stack([y0, x0, h, w], -1)[:, None])
        self.colors.append(tuple(color))

    def add_many(self, y0, x0, h, w, colors, visible=None):
        """y0/x0/h/w: [R] or [N, R]; colors: R RGB tuples; visible: [N, R] bool."""
        R = len(colors)

        def full(v):
            t = self._t(v)
            return t.expand(self.n, R) if t.dim() == 0 else (t[None].expand(self.n, R) if t.dim() == 1 else t)
        y0, x0, h, w = [full(v) for v in (y0, x0, h, w)]
        if visible is not None:
            h = torch.where(visible, h, torch.zeros_like(h))
        self.parts.append(torch.stack([y0, x0, h, w], -1))
        self.colors.extend(tuple(c) for c in colors)

    def geometry(self) -> torch.Tensor:
        return torch.cat(self.parts, 1)                    # [N, R, 4] int64


class PixelGameVec(VecEnv):
    """Common driver: state tensors, frame stack, auto-reset, RGB render -> preprocessing."""
    graph_safe = True          # no host syncs / host->device copies inside a step; state updated in place
    n_actions = 4
    max_steps = 27000
    HIP_GAME = None            # game id of csrc/games.hip (None: torch physics + HIP rasteriser)
    # state fields in csrc/games.hip order ("i": one int, "vec": [N, k] ints, "mask": [N, k] bools as one
    # bitmask int, "bits": bool grid bit-packed into 32-bit words); counter/steps/epret follow
    HIP_FIELDS: tuple = ()

    def __init__(self, num_envs: int, device="cpu", seed: int = 0, frameskip: int = 4, gray: str = "rgb",
                 backend: str = "torch", no_op_max: int = 7):
        self.num_envs = num_envs
        self.num_actions = self.n_actions
        self.obs_shape = (OBS_H, OBS_W, 4)
        self.obs_dtype = torch.uint8
        self.device = torch.device(device)
        self.frameskip = frameskip
        self.gray = gray
        self.backend = backend
        self.no_op_max = no_op_max
        self.max_episode_steps = self.max_steps
        self.env_id = torch.arange(num_envs, dtype=torch.int64, device=self.device)
        self.counter = torch.zeros(num_envs, dtype=torch.int64, device=self.device)
        self.tables = torch.from_numpy(resize_tables()).to(self.device)
        self.rows = torch.arange(SCREEN_H, device=self.device)[None, :, None]
        self.cols = torch.arange(SCREEN_W, device=self.device)[None, None, :]
        self.steps = torch.zeros(num_envs, dtype=torch.int64, device=self.device)
        self.epret = torch.zeros(num_envs, dtype=torch.int64, device=self.device)
        self.obs = torch.zeros(num_envs, OBS_H, OBS_W, 4, dtype=torch.uint8, device=self.device)
        self._colors = {}
        self.init_state()
        # per-env state tensors are updated IN PLACE at the end of every step (_commit), so a
        # captured step (hipGraph) keeps reading and writing the same storage on replay
        self._persist = {k: v for k, v in vars(self).items()
                         if isinstance(v, torch.Tensor) and v.dim() >= 1 and v.shape[0] == num_envs
                         and k not in ("obs", "env_id")}
        self._hip = False
        self.seed(seed)
        if self.backend == "hip" and self.device.type == "cuda" and self.HIP_GAME is not None:
            self._hip_setup()

    # -- helpers -------------------------------------------------------------
    def seed(self, seed: int):
        self.seed_int = seed & 0xFFFFFFFF
        self._seed = torch.tensor(self.seed_int, dtype=torch.int64, device=self.device)
        self.counter.zero_()
        if self._hip:
            self._st32[:, self._st32.shape[1] - 3] = 0

    # -- HIP game logic (csrc/games.hip) ------------------------------------------------
    def _fields(self):
        return tuple(self.HIP_FIELDS) + (("counter", "i"), ("steps", "i"), ("epret", "i"))

    def _hip_pack(self) -> torch.Tensor:
        """torch state -> int32 [N, NS] kernel state (bit-packed grids, two's-complement words)."""
        N = self.num_envs
        cols = []
        for name, kind in self._fields():
            t = getattr(self, name).reshape(N, -1).long()
            if kind in ("i", "vec"):
                cols.append(t)
            elif kind == "mask":
                cols.append((t << torch.arange(t.shape[1], device=self.device)).sum(1, keepdim=True))
            else:                                           # bits
                n = t.shape[1]
                k = (n + 31) // 32
                t = torch.nn.functional.pad(t, (0, 32 * k - n)).view(N, k, 32)
                cols.append((t << torch.arange(32, device=self.device)).sum(2))
        v = torch.cat(cols, 1) & 0xFFFFFFFF
        return torch.where(v >= 2 ** 31, v - 2 ** 32, v).to(torch.int32).contiguous()

    def sync_from_device(self):
        """Refresh the torch state tensors from the HIP kernel state (no-op on the torch path)."""
        if not self._hip:
            return
        N = self.num_envs
        v = self._st32.long()
        j = 0
        for name, kind in self._fields():
            t = getattr(self, name)
            if kind == "i":
                new = v[:, j]
                j += 1
            elif kind == "vec":
                k = t.reshape(N, -1).shape[1]
                new = v[:, j:j + k]
                j += k
            elif kind == "mask":
                k = t.reshape(N, -1).shape[1]
                new = (v[:, j:j + 1] >> torch.arange(k, device=self.device)) & 1
                j += 1
            else:
                n = t.reshape(N, -1).shape[1]
                k = (n + 31) // 32
                w = v[:, j:j + k] & 0xFFFFFFFF
                new = ((w[:, :, None] >> torch.arange(32, device=self.device)) & 1).reshape(N, 32 * k)[:, :n]
                j += k
            if name == "counter":
                new = new & 0xFFFFFFFF
            t.copy_(new.reshape(t.shape).to(t.dtype))

    def _hip_setup(self):
        from ..ops import envs as henv
        from .pong import gray_weights
        ns, nr = henv.game_layout(self.HIP_GAME)
        self._st32 = self._hip_pack()
        if self._st32.shape[1] != ns:
            raise RuntimeError(f"{self.HIP_GAME}: HIP_FIELDS pack to {self._st32.shape[1]} ints, kernel expects {ns}")
        colors = self.scene().colors
        if len(colors) != nr:
            raise RuntimeError(f"{self.HIP_GAME}: scene has {len(colors)} rectangles, kernel writes {nr}")
        wr, wg, wb = gray_weights(self.gray)
        lum = lambda c: (c[0] * wr + c[1] * wg + c[2] * wb + 8192) >> 14      # noqa: E731  cv2 fixed-point luma
        self._gray_tab = torch.tensor([lum(c) for c in colors], dtype=torch.uint8, device=self.device)
        self._bg_gray = int(lum(BG))
        N = self.num_envs
        self._rects = torch.zeros(N, nr, 4, dtype=torch.int16, device=self.device)
        self._tab32 = self.tables.to(torch.int32).contiguous()
        self._rw = torch.zeros(N, dtype=torch.float32, device=self.device)
        self._dn = torch.zeros(N, dtype=torch.uint8, device=self.device)
        self._ep = torch.zeros(N, dtype=torch.float32, device=self.device)
        self._hip = True

    def _hip_run(self, actions, mask, reward, done, epret):
        from ..ops import envs as henv
        henv.game_step(self.HIP_GAME, self._st32, actions, mask, self.num_actions, self.seed_int, self.frameskip,
                       int(self.max_episode_steps), reward, done, epret, self._rects, id_base=self.id_base)

    def _hip_push(self, obs_in, obs_out, reset_u8):
        from ..ops import envs as henv
        henv.rects16_stack_push(self._rects, self._gray_tab, self._bg_gray, obs_in, obs_out, reset_u8, self._tab32)

    def _commit(self):
        for k, p in self._persist.items():
            t = getattr(self, k)
            if t is not p:
                p.copy_(t)
                setattr(self, k, p)

    def rand(self, stream: int, n: int) -> torch.Tensor:
        return env_rand_u32(self._seed, self.env_id, self.counter, stream) % n

    def color(self, c):
        if c not in self._colors:
            self._colors[c] = torch.tensor(c, dtype=torch.uint8, device=self.device)
        return self._colors[c]

    def rect(self, y0, x0, h, w):
        """bool [N,210,160] for per-env rectangles (y0/x0 [N] pixel tensors or ints)."""
        y0 = torch.as_tensor(y0, device=self.device).reshape(-1, 1, 1)
        x0 = torch.as_tensor(x0, device=self.device).reshape(-1, 1, 1)
        return (self.rows >= y0) & (self.rows < y0 + h) & (self.cols >= x0) & (self.cols < x0 + w)

    def where_set(self, t, mask, v):
        return torch.where(mask, torch.full_like(t, v), t)

    # -- to implement ------------------------------------------------------------
    def init_state(self):
        raise NotImplementedError

    def reset_state(self, mask):
        raise NotImplementedError

    def physics(self, a):
        """one sub-frame; returns int64 reward [N]"""
        raise NotImplementedError

    def game_over(self):
        raise NotImplementedError

    def scene(self) -> Scene:
        raise NotImplementedError

    def draw(self, img):
        """Torch renderer (oracle): paint the scene's rectangles in order."""
        sc = self.scene()
        geo = sc.geometry()
        for r, c in enumerate(sc.colors):
            y0, x0, h, w = geo[:, r].unbind(-1)
            y0, x0, h, w = y0[:, None, None], x0[:, None, None], h[:, None, None], w[:, None, None]
            m = (self.rows >= y0) & (self.rows < y0 + h) & (self.cols >= x0) & (self.cols < x0 + w)
            img[m] = self.color(c)

    # -- VecEnv API ----------------------------------------------------------------
    def render(self) -> torch.Tensor:
        img = torch.empty(self.num_envs, SCREEN_H, SCREEN_W, 3, dtype=torch.uint8, device=self.device)
        img[:] = self.color(BG)
        self.draw(img)
        return img

    def frame(self):
        return preprocess_frames(self.render(), self.tables, self.gray)

    def reset(self):
        allm = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
        self.reset_where(allm)
        return self.obs.clone()

    def reset_where(self, mask):
        if self._hip:
            m8 = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            self._hip_run(None, m8, self._rw, self._dn, self._ep)
            out = torch.empty_like(self.obs)
            self._hip_push(self.obs, out, m8)
            self.obs = out
            return
        self.reset_state(mask)
        self.steps = torch.where(mask, torch.zeros_like(self.steps), self.steps)
        self.epret = torch.where(mask, torch.zeros_like(self.epret), self.epret)
        self.counter += mask.long()
        self._commit()
        self.obs = self._push(self.obs, mask)

    def _push(self, obs_in, reset, obs_out=None):
        """Render, preprocess and push the new frame: fused HIP kernel (backend 'hip') or the torch oracle."""
        if self.backend == "hip":
            from ..ops import envs as henv
            out = obs_out if obs_out is not None else torch.empty_like(obs_in)
            sc = self.scene()
            henv.rects_stack_push(sc.geometry(), sc.colors, BG, obs_in, out, reset, self.tables, self.gray)
            return out
        f = self.frame()
        pushed = torch.cat([obs_in.reshape(self.obs.shape)[..., 1:], f[..., None]], dim=3)
        new = torch.where(reset[:, None, None, None], f[..., None].expand(-1, -1, -1, 4), pushed)
        if obs_out is not None:
            obs_out.copy_(new.reshape(obs_out.shape))
            return obs_out
        return new

    def _advance(self, actions):
        """Physics for one agent step (frameskip sub-frames) + auto-reset; returns (reward, done, ep_return)."""
        a = actions.long().to(self.device)
        a = torch.where((a >= self.num_actions) | (a < 0), torch.zeros_like(a), a)   # game_state.py:38-39
        reward = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)
        for _ in range(self.frameskip):
            reward += self.physics(a)
        self.counter += 1
        self.steps += 1
        self.epret += reward
        done = self.game_over() | (self.steps >= self.max_episode_steps)
        ep_return = torch.where(done, self.epret, torch.zeros_like(self.epret)).float()
        self.reset_state(done)
        self.steps = torch.where(done, torch.zeros_like(self.steps), self.steps)
        self.epret = torch.where(done, torch.zeros_like(self.epret), self.epret)
        self.counter += done.long()
        self._commit()
        return reward, done, ep_return

    def step(self, actions):
        if self._hip:
            a = actions.to(device=self.device, dtype=torch.int32).contiguous()
            self._hip_run(a, None, self._rw, self._dn, self._ep)
            out = torch.empty_like(self.obs)
            self._hip_push(self.obs, out, self._dn)
            self.obs = out
            return out.clone(), self._rw.clone(), self._dn.bool(), {"episode_return": self._ep.clone()}
        reward, done, ep_return = self._advance(actions)
        self.obs = self._push(self.obs, done)
        return self.obs.clone(), reward.float(), done, {"episode_return": ep_return}

    @property
    def supports_ring(self) -> bool:
        """The engine's frame ring (runtime/engine.py) needs the HIP game logic + renderer."""
        return bool(getattr(self, "_hip", False))

    def step_ring_into(self, actions, frames, slot, fc_in, fc_out, reward, done, epret):
        """Engine frame-ring step (HIP only): game logic, then the scene rasterised straight into the ring plane
        frames[:, slot] with the next stack's first valid channel (csrc/preprocess.hip rects_push_kernel<true>)."""
        if not self.supports_ring:
            raise RuntimeError(f"{self.id}: the frame ring needs the HIP game backend")
        from ..ops import envs as henv
        a = actions if actions.dtype == torch.int32 and actions.is_contiguous() else \
            actions.to(torch.int32).contiguous()
        direct = (reward.dtype == torch.float32 and done.dtype == torch.uint8 and epret.dtype == torch.float32
                  and reward.is_contiguous() and done.is_contiguous() and epret.is_contiguous())
        rw, dn, ep = (reward, done, epret) if direct else (self._rw, self._dn, self._ep)
        self._hip_run(a, None, rw, dn, ep)
        henv.rects16_ring_push(self._rects, self._gray_tab, self._bg_gray, frames, slot, fc_in, fc_out,
                               dn.reshape(-1), self._tab32)
        if not direct:
            reward.copy_(rw.view(reward.shape))
            done.copy_(dn.view(done.shape).to(done.dtype))
            epret.copy_(ep.view(epret.shape))

    def step_into(self, actions, obs_in, obs_out, reward, done, epret):
        """Engine hook: torch physics + render, then (backend 'hip') ONE fused kernel that preprocesses the
        frame and pushes it from the engine's obs slot t straight into slot t+1.  With the HIP game logic
        the whole step is two launches writing the engine's reward/done/return rows directly."""
        if self._hip:
            a = actions if actions.dtype == torch.int32 and actions.is_contiguous() else \
                actions.to(torch.int32).contiguous()
            direct = (reward.dtype == torch.float32 and done.dtype == torch.uint8 and epret.dtype == torch.float32
                      and reward.is_contiguous() and done.is_contiguous() and epret.is_contiguous())
            rw, dn, ep = (reward, done, epret) if direct else (self._rw, self._dn, self._ep)
            self._hip_run(a, None, rw, dn, ep)
            self._hip_push(obs_in.view(self.obs.shape), obs_out.view(self.obs.shape), dn.reshape(-1))
            if not direct:
                reward.copy_(rw.view(reward.shape))
                done.copy_(dn.view(done.shape).to(done.dtype))
                epret.copy_(ep.view(epret.shape))
            self.obs = obs_out.view(self.obs.shape)
            return
        r, d, ep = self._advance(actions)
        self._push(obs_in.view(self.obs.shape), d, obs_out.view(self.obs.shape))
        self.obs = obs_out.view(self.obs.shape)
        reward.copy_(r.float())
        done.copy_(d.to(done.dtype))
        epret.copy_(ep)


# ===========================================================================
class BreakoutVec(PixelGameVec):
    id = "Breakout"
    n_actions = 4
    reward_threshold = 30.0
    HIP_GAME = "Breakout"
    HIP_FIELDS = (("px", "i"), ("bx", "i"), ("by", "i"), ("vx", "i"), ("vy", "i"), ("inplay", "i"), ("lives", "i"),
                  ("bricks", "bits"))
    U = 16
    ROWS, COLS = 6, 18
    BRICK_Y0, BRICK_H, BRICK_W, BRICK_X0 = 57, 6, 8, 8
    ROW_REWARD = (7, 7, 4, 4, 1, 1)
    ROW_COLOR = ((200, 72, 72), (198, 108, 58), (180, 122, 48), (162, 162, 42), (72, 160, 72), (66, 72, 200))
    PADDLE_Y, PADDLE_W = 189, 16

    def init_state(self):
        N = self.num_envs
        d = self.device
        self.bricks = torch.ones(N, self.ROWS, self.COLS, dtype=torch.bool, device=d)
        self.px = torch.zeros(N, dtype=torch.int64, device=d)
        self.bx = torch.zeros(N, dtype=torch.int64, device=d)
        self.by = torch.zeros(N, dtype=torch.int64, device=d)
        self.vx = torch.zeros(N, dtype=torch.int64, device=d)
        self.vy = torch.zeros(N, dtype=torch.int64, device=d)
        self.inplay = torch.zeros(N, dtype=torch.bool, device=d)
        self.lives = torch.zeros(N, dtype=torch.int64, device=d)
        self.rew = torch.tensor(self.ROW_REWARD, dtype=torch.int64, device=d)

    def reset_state(self, m):
        self.bricks = torch.where(m[:, None, None], torch.ones_like(self.bricks), self.bricks)
        self.px = self.where_set(self.px, m, 72 * self.U)
        self.inplay = torch.where(m, torch.zeros_like(self.inplay), self.inplay)
        self.lives = self.where_set(self.lives, m, 5)

    def physics(self, a):
        U = self.U
        right = (a == 2).long()
        left = (a == 3).long()
        self.px = (self.px + (right - left) * 6 * U).clamp(8 * U, (152 - self.PADDLE_W) * U)
        serve = (~self.inplay) & (a == 1)
        dirn = torch.where(self.rand(0, 2) == 0, -1, 1)
        self.bx = torch.where(serve, self.px + (self.PADDLE_W // 2) * U, self.bx)
        self.by = self.where_set(self.by, serve, 120 * U)
        self.vx = torch.where(serve, dirn * (24 + self.rand(1, 12)), self.vx)
        self.vy = self.where_set(self.vy, serve, 40)
        self.inplay = self.inplay | serve
        nx, ny = self.bx + self.vx, self.by + self.vy
        hitx = (nx < 8 * U) | (nx > 150 * U)
        self.vx = torch.where(hitx & self.inplay, -self.vx, self.vx)
        nx = nx.clamp(8 * U, 150 * U)
        hit_top = ny < 32 * U
        self.vy = torch.where(hit_top & self.inplay, self.vy.abs(), self.vy)
        ny = torch.where(hit_top, 32 * U, ny)
        # bricks
        cy = torch.div(ny // U - self.BRICK_Y0, self.BRICK_H, rounding_mode="floor")
        cx = torch.div(nx // U - self.BRICK_X0, self.BRICK_W, rounding_mode="floor")
        inb = (cy >= 0) & (cy < self.ROWS) & (cx >= 0) & (cx < self.COLS) & self.inplay
        cyc, cxc = cy.clamp(0, self.ROWS - 1), cx.clamp(0, self.COLS - 1)
        b = self.bricks[torch.arange(self.num_envs, device=self.device), cyc, cxc]
        hitb = inb & b
        reward = torch.where(hitb, self.rew[cyc], torch.zeros_like(cy))
        self.bricks[torch.arange(self.num_envs, device=self.device), cyc, cxc] = b & ~hitb
        self.vy = torch.where(hitb, -self.vy, self.vy)
        # paddle
        onp = (self.vy > 0) & (ny // U >= self.PADDLE_Y - 4) & (ny // U < self.PADDLE_Y + 2) & \
              (nx >= self.px - 2 * U) & (nx <= self.px + (self.PADDLE_W + 2) * U)
        off = (nx - (self.px + (self.PADDLE_W // 2) * U))
        self.vx = torch.where(onp & self.inplay, (off * 3 // 16).clamp(-48, 48), self.vx)
        self.vy = torch.where(onp & self.inplay, -self.vy.abs(), self.vy)
        lost = self.inplay & (ny > 200 * U)
        self.lives = self.lives - lost.long()
        self.inplay = self.inplay & ~lost
        self.bx = torch.where(self.inplay, nx, self.bx)
        self.by = torch.where(self.inplay, ny, self.by)
        return reward

    def game_over(self):
        return (self.lives <= 0) | (~self.bricks.view(self.num_envs, -1).any(1))

    def scene(self) -> Scene:
        sc = Scene(self.num_envs, self.device)
        wall = (142, 142, 142)
        sc.add(17, 0, 15, 160, wall)
        sc.add(17, 0, 179, 8, wall)
        sc.add(17, 152, 179, 8, wall)
        r = torch.arange(self.ROWS, device=self.device).repeat_interleave(self.COLS)
        c = torch.arange(self.COLS, device=self.device).repeat(self.ROWS)
        sc.add_many(self.BRICK_Y0 + r * self.BRICK_H, self.BRICK_X0 + c * self.BRICK_W, self.BRICK_H, self.BRICK_W,
                    [self.ROW_COLOR[i // self.COLS] for i in range(self.ROWS * self.COLS)],
                    visible=self.bricks.reshape(self.num_envs, -1))
        red = (200, 72, 72)
        sc.add(self.PADDLE_Y, self.px // self.U, 4, self.PADDLE_W, red)
        sc.add(self.by // self.U, self.bx // self.U, 4, 2, red, visible=self.inplay)
        return sc


# ===========================================================================
class SpaceInvadersVec(PixelGameVec):
    id = "SpaceInvaders"
    n_actions = 6
    reward_threshold = 300.0
    # waves repeat, so a good player's episode is unbounded: 4500 agent steps (18000 frames, 5 minutes of play)
    # bound it, as ALE's frame limit bounds the real game
    max_steps = 4500
    HIP_GAME = "SpaceInvaders"
    HIP_FIELDS = (("fx", "i"), ("fy", "i"), ("fdir", "i"), ("tick", "i"), ("px", "i"), ("lives", "i"), ("sx", "i"),
                  ("sy", "i"), ("shot", "i"), ("bxp", "i"), ("byp", "i"), ("bomb", "i"), ("alive", "bits"))
    AR, AC = 6, 6
    ROW_REWARD = (30, 25, 20, 15, 10, 5)

    def init_state(self):
        N, d = self.num_envs, self.device
        z = lambda: torch.zeros(N, dtype=torch.int64, device=d)
        self.alive = torch.ones(N, self.AR, self.AC, dtype=torch.bool, device=d)
        self.fx, self.fy, self.fdir, self.tick = z(), z(), z(), z()
        self.px, self.lives = z(), z()
        self.sx, self.sy = z(), z()
        self.shot = torch.zeros(N, dtype=torch.bool, device=d)
        self.bxp, self.byp = z(), z()
        self.bomb = torch.zeros(N, dtype=torch.bool, device=d)
        self.rew = torch.tensor(self.ROW_REWARD, dtype=torch.int64, device=d)

    def reset_state(self, m):
        self.alive = torch.where(m[:, None, None], torch.ones_like(self.alive), self.alive)
        for name, v in (("fx", 22), ("fy", 40), ("fdir", 1), ("tick", 0), ("px", 76), ("lives", 3)):
            setattr(self, name, self.where_set(getattr(self, name), m, v))
        self.shot = self.shot & ~m
        self.bomb = self.bomb & ~m

    def physics(self, a):
        N, d = self.num_envs, self.device
        ar = torch.arange(N, device=d)
        right = ((a == 2) | (a == 4)).long()
        left = ((a == 3) | (a == 5)).long()
        fire = (a == 1) | (a == 4) | (a == 5)
        self.px = (self.px + 2 * (right - left)).clamp(20, 133)
        new_shot = fire & ~self.shot
        self.sx = torch.where(new_shot, self.px + 3, self.sx)
        self.sy = torch.where(new_shot, torch.full_like(self.sy, 182), self.sy)
        self.shot = self.shot | new_shot
        self.sy = self.sy - 4 * self.shot.long()
        self.shot = self.shot & (self.sy > 20)
        # formation march every 4 sub-frames
        self.tick += 1
        move = (self.tick % 4) == 0
        alive_cols = self.alive.any(1)                                        # [N, AC]
        ci = torch.arange(self.AC, device=d)
        leftmost = torch.where(alive_cols, ci, self.AC).min(1).values
        rightmost = torch.where(alive_cols, ci, -1).max(1).values
        xl = self.fx + 16 * leftmost
        xr = self.fx + 16 * rightmost + 8
        edge = move & (((self.fdir > 0) & (xr >= 150)) | ((self.fdir < 0) & (xl <= 10)))
        self.fdir = torch.where(edge, -self.fdir, self.fdir)
        self.fy = self.fy + 4 * edge.long()
        self.fx = self.fx + torch.where(move & ~edge, self.fdir, torch.zeros_like(self.fx))
        # shot vs aliens
        col = torch.div(self.sx - self.fx, 16, rounding_mode="floor")
        row = torch.div(self.sy - self.fy, 18, rounding_mode="floor")
        inx = ((self.sx - self.fx) % 16) < 8
        iny = ((self.sy - self.fy) % 18) < 10
        ok = self.shot & (col >= 0) & (col < self.AC) & (row >= 0) & (row < self.AR) & inx & iny
        colc, rowc = col.clamp(0, self.AC - 1), row.clamp(0, self.AR - 1)
        hit = ok & self.alive[ar, rowc, colc]
        self.alive[ar, rowc, colc] = self.alive[ar, rowc, colc] & ~hit
        reward = torch.where(hit, self.rew[rowc], torch.zeros_like(self.px))
        self.shot = self.shot & ~hit
        # alien bomb
        drop = ~self.bomb & (self.rand(4, 64) == 0) & alive_cols.any(1)
        bc = self.rand(5, self.AC)
        has = alive_cols[ar, bc]
        lowest = torch.where(self.alive[ar, :, bc], torch.arange(self.AR, device=d)[None], -1).max(1).values
        drop = drop & has
        self.bxp = torch.where(drop, self.fx + 16 * bc + 4, self.bxp)
        self.byp = torch.where(drop, self.fy + 18 * lowest + 10, self.byp)
        self.bomb = self.bomb | drop
        self.byp = self.byp + 2 * self.bomb.long()
        hitp = self.bomb & (self.byp >= 185) & (self.byp < 193) & (self.bxp >= self.px) & (self.bxp < self.px + 7)
        self.lives = self.lives - hitp.long()
        self.bomb = self.bomb & ~hitp & (self.byp < 196)
        # wave cleared: a new formation marches in from the top (the game ends on lives or an invasion only)
        cleared = ~self.alive.view(N, -1).any(1)
        self.alive = torch.where(cleared[:, None, None], torch.ones_like(self.alive), self.alive)
        self.fx = self.where_set(self.fx, cleared, 22)
        self.fy = self.where_set(self.fy, cleared, 40)
        self.fdir = self.where_set(self.fdir, cleared, 1)
        return reward

    def game_over(self):
        lowest_row = torch.where(self.alive.any(2), torch.arange(self.AR, device=self.device)[None], -1).max(1).values
        invaded = (self.fy + 18 * lowest_row + 10) >= 180
        return (self.lives <= 0) | invaded

    def scene(self) -> Scene:
        sc = Scene(self.num_envs, self.device)
        sc.add(195, 0, 2, 160, (80, 89, 22))
        green, olive = (50, 132, 50), (134, 134, 29)
        r = torch.arange(self.AR, device=self.device).repeat_interleave(self.AC)
        c = torch.arange(self.AC, device=self.device).repeat(self.AR)
        sc.add_many(self.fy[:, None] + 18 * r[None], self.fx[:, None] + 16 * c[None], 10, 8,
                    [olive if (i // self.AC) % 2 else green for i in range(self.AR * self.AC)],
                    visible=self.alive.reshape(self.num_envs, -1))
        sc.add(185, self.px, 8, 7, (50, 132, 50))
        sc.add(self.sy, self.sx, 6, 1, (142, 142, 142), visible=self.shot)
        sc.add(self.byp, self.bxp, 6, 1, (200, 200, 200), visible=self.bomb)
        return sc


# ===========================================================================
MAZE = [
    "#############",
    "#.....#.....#",
    "#.###.#.###.#",
    "#...........#",
    "#.#.#####.#.#",
    "#.#...#...#.#",
    "#.###.#.###.#",
    "#...........#",
    "#.###.#.###.#",
    "#.....#.....#",
    "#############",
]


class AlienVec(PixelGameVec):
    """Maze game: eggs + 3 chasing aliens (Alien: 18 actions; MsPacman: 9 actions)."""
    id = "Alien"
    n_actions = 18
    reward_threshold = 400.0
    HIP_GAME = "Alien"
    HIP_FIELDS = (("py", "i"), ("px", "i"), ("ay", "vec"), ("ax", "vec"), ("lives", "i"), ("tick", "i"),
                  ("dots", "bits"))
    CW, CH, Y0, X0 = 12, 16, 20, 2
    NA = 3
    MOVE_EVERY = 2

    def init_state(self):
        N, d = self.num_envs, self.device
        walls = torch.tensor([[ch == "#" for ch in row] for row in MAZE], device=d)
        self.walls = walls
        self.H, self.W = walls.shape
        self.dots = torch.zeros(N, self.H, self.W, dtype=torch.bool, device=d)
        self.py, self.px = torch.zeros(N, dtype=torch.int64, device=d), torch.zeros(N, dtype=torch.int64, device=d)
        self.ay = torch.zeros(N, self.NA, dtype=torch.int64, device=d)
        self.ax = torch.zeros(N, self.NA, dtype=torch.int64, device=d)
        self.lives = torch.zeros(N, dtype=torch.int64, device=d)
        self.tick = torch.zeros(N, dtype=torch.int64, device=d)
        self.dy = torch.tensor([0, -1, 0, 0, 1], device=d)      # none, up, right, left, down
        self.dx = torch.tensor([0, 0, 1, -1, 0], device=d)
        # action -> direction index (ALE: 2 UP 3 RIGHT 4 LEFT 5 DOWN; diagonals/fire variants fold onto them)
        amap = [0, 0, 1, 2, 3, 4, 1, 1, 4, 4, 1, 2, 3, 4, 1, 1, 4, 4]
        self.amap = torch.tensor(amap[: self.n_actions], device=d)
        self.start_a = torch.tensor([[1, 1], [1, 11], [9, 6]], device=d)

    def reset_state(self, m):
        self.dots = torch.where(m[:, None, None], (~self.walls)[None].expand_as(self.dots), self.dots)
        self.py = self.where_set(self.py, m, 7)
        self.px = self.where_set(self.px, m, 6)
        self.dots[:, 7, 6] &= ~m
        self.ay = torch.where(m[:, None], self.start_a[:, 0][None].expand_as(self.ay), self.ay)
        self.ax = torch.where(m[:, None], self.start_a[:, 1][None].expand_as(self.ax), self.ax)
        self.lives = self.where_set(self.lives, m, 3)
        self.tick = self.where_set(self.tick, m, 0)

    def _free(self, y, x):
        return ~self.walls[y.clamp(0, self.H - 1), x.clamp(0, self.W - 1)]

    def physics(self, a):
        N, d = self.num_envs, self.device
        ar = torch.arange(N, device=d)
        self.tick += 1
        step_now = (self.tick % self.MOVE_EVERY) == 0
        di = self.amap[a]
        ny, nx = self.py + self.dy[di], self.px + self.dx[di]
        ok = step_now & self._free(ny, nx)
        self.py = torch.where(ok, ny, self.py)
        self.px = torch.where(ok, nx, self.px)
        eat = self.dots[ar, self.py, self.px]
        self.dots[ar, self.py, self.px] = False
        reward = eat.long() * 10
        # aliens: every other move, step towards the player (random tie-break / 25% random move)
        amove = (self.tick % (2 * self.MOVE_EVERY)) == 0
        for k in range(self.NA):
            y, x = self.ay[:, k], self.ax[:, k]
            best_y, best_x = y.clone(), x.clone()
            best_d = torch.full_like(y, 1 << 20)
            r = self.rand(6 + k, 4)
            for j in range(1, 5):
                cy, cx = y + self.dy[j], x + self.dx[j]
                free = self._free(cy, cx)
                dist = (cy - self.py).abs() + (cx - self.px).abs()
                dist = torch.where(r == (j - 1), dist - 2, dist)          # a little randomness
                better = free & (dist < best_d)
                best_y = torch.where(better, cy, best_y)
                best_x = torch.where(better, cx, best_x)
                best_d = torch.where(better, dist, best_d)
            self.ay[:, k] = torch.where(amove, best_y, y)
            self.ax[:, k] = torch.where(amove, best_x, x)
        caught = ((self.ay == self.py[:, None]) & (self.ax == self.px[:, None])).any(1)
        self.lives = self.lives - caught.long()
        # respawn aliens on a catch
        self.ay = torch.where(caught[:, None], self.start_a[:, 0][None].expand_as(self.ay), self.ay)
        self.ax = torch.where(caught[:, None], self.start_a[:, 1][None].expand_as(self.ax), self.ax)
        cleared = ~self.dots.view(N, -1).any(1)
        reward = reward + cleared.long() * 500
        return reward

    def game_over(self):
        return (self.lives <= 0) | (~self.dots.view(self.num_envs, -1).any(1))

    def scene(self) -> Scene:
        sc = Scene(self.num_envs, self.device)
        if not hasattr(self, "_walls_yx"):          # static maze walls, built once (outside any capture)
            cells = [(y, x) for y in range(self.H) for x in range(self.W) if MAZE[y][x] == "#"]
            self._walls_yx = (torch.tensor([self.Y0 + y * self.CH for y, _ in cells], device=self.device),
                              torch.tensor([self.X0 + x * self.CW for _, x in cells], device=self.device))
        wy, wx = self._walls_yx
        sc.add_many(wy, wx, self.CH, self.CW, [(84, 92, 214)] * wy.shape[0])
        # eggs: 2x2 pixels at cell centres
        yy = torch.arange(self.H, device=self.device).repeat_interleave(self.W)
        xx = torch.arange(self.W, device=self.device).repeat(self.H)
        sc.add_many(self.Y0 + yy * self.CH + self.CH // 2, self.X0 + xx * self.CW + self.CW // 2, 2, 2,
                    [(223, 183, 85)] * (self.H * self.W), visible=self.dots.reshape(self.num_envs, -1))
        sc.add(self.Y0 + self.py * self.CH + 3, self.X0 + self.px * self.CW + 3, 10, 6, (132, 144, 252))
        sc.add_many(self.Y0 + self.ay * self.CH + 2, self.X0 + self.ax * self.CW + 2, 12, 8,
                    [(252, 144, 144)] * self.NA)
        return sc


class MsPacmanVec(AlienVec):
    id = "MsPacman"
    n_actions = 9
    reward_threshold = 500.0
    HIP_GAME = "MsPacman"


# ===========================================================================
class CentipedeVec(PixelGameVec):
    id = "Centipede"
    n_actions = 18
    reward_threshold = 3000.0
    HIP_GAME = "Centipede"
    HIP_FIELDS = (("mush", "bits"), ("sy", "vec"), ("sx", "vec"), ("sdir", "vec"), ("salive", "mask"), ("px", "i"),
                  ("shot", "i"), ("shx", "i"), ("shy", "i"), ("lives", "i"), ("tick", "i"))
    NS = 10
    GH, GW = 20, 16          # mushroom grid (8 px rows x 10 px cols in the field rows 20..180)

    def init_state(self):
        N, d = self.num_envs, self.device
        self.mush = torch.zeros(N, self.GH, self.GW, dtype=torch.bool, device=d)
        self.sy = torch.zeros(N, self.NS, dtype=torch.int64, device=d)     # segment grid row
        self.sx = torch.zeros(N, self.NS, dtype=torch.int64, device=d)     # segment grid col
        self.sdir = torch.zeros(N, self.NS, dtype=torch.int64, device=d)
        self.salive = torch.zeros(N, self.NS, dtype=torch.bool, device=d)
        self.px = torch.zeros(N, dtype=torch.int64, device=d)
        self.shot = torch.zeros(N, dtype=torch.bool, device=d)
        self.shx = torch.zeros(N, dtype=torch.int64, device=d)
        self.shy = torch.zeros(N, dtype=torch.int64, device=d)
        self.lives = torch.zeros(N, dtype=torch.int64, device=d)
        self.tick = torch.zeros(N, dtype=torch.int64, device=d)
        self.amap_h = torch.tensor([0, 0, 0, 1, -1, 0, 1, -1, 1, -1, 0, 0, 1, -1, 0, 1, -1, 1, -1][:18], device=d)
        self.afire = torch.tensor([0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1], device=d).bool()

    def reset_state(self, m):
        N = self.num_envs
        r = torch.stack([self.rand(10 + k, 100) for k in range(self.GH * self.GW // 16)], 1)     # sparse field
        field = torch.zeros(N, self.GH * self.GW, dtype=torch.bool, device=self.device)
        pos = (torch.arange(r.shape[1], device=self.device)[None] * 16 + r % 16).clamp(max=self.GH * self.GW - 1)
        field.scatter_(1, pos, (r < 60))
        field = field.view(N, self.GH, self.GW)
        field[:, self.GH - 3:] = False
        self.mush = torch.where(m[:, None, None], field, self.mush)
        k = torch.arange(self.NS, device=self.device)[None]
        self.sy = torch.where(m[:, None], torch.zeros_like(self.sy), self.sy)
        self.sx = torch.where(m[:, None], (self.GW - 1 - k).expand_as(self.sx).clamp(min=0), self.sx)
        self.sdir = torch.where(m[:, None], -torch.ones_like(self.sdir), self.sdir)
        self.salive = torch.where(m[:, None], torch.ones_like(self.salive), self.salive)
        self.px = self.where_set(self.px, m, 76)
        self.shot = self.shot & ~m
        self.lives = self.where_set(self.lives, m, 3)
        self.tick = self.where_set(self.tick, m, 0)

    def physics(self, a):
        N, d = self.num_envs, self.device
        ar = torch.arange(N, device=d)
        self.px = (self.px + 2 * self.amap_h[a]).clamp(4, 152)
        fire = self.afire[a] & ~self.shot
        self.shx = torch.where(fire, self.px + 2, self.shx)
        self.shy = torch.where(fire, torch.full_like(self.shy, 180), self.shy)
        self.shot = self.shot | fire
        self.shy = self.shy - 6 * self.shot.long()
        self.shot = self.shot & (self.shy > 20)
        gy = torch.div(self.shy - 20, 8, rounding_mode="floor").clamp(0, self.GH - 1)
        gx = torch.div(self.shx, 10, rounding_mode="floor").clamp(0, self.GW - 1)
        reward = torch.zeros(N, dtype=torch.int64, device=d)
        hm = self.shot & self.mush[ar, gy, gx]
        self.mush[ar, gy, gx] = self.mush[ar, gy, gx] & ~hm
        reward += hm.long()
        self.shot = self.shot & ~hm
        hs = self.shot[:, None] & self.salive & (self.sy == gy[:, None]) & (self.sx == gx[:, None])
        anyhs = hs.any(1)
        reward += 10 * hs.sum(1)
        self.salive = self.salive & ~hs
        # a hit segment leaves a mushroom
        self.mush[ar, gy, gx] = self.mush[ar, gy, gx] | anyhs
        self.shot = self.shot & ~anyhs
        # centipede moves every 3 sub-frames
        self.tick += 1
        mv = ((self.tick % 3) == 0)[:, None] & self.salive
        nx = self.sx + self.sdir
        blocked = (nx < 0) | (nx >= self.GW)
        nxc = nx.clamp(0, self.GW - 1)
        blocked = blocked | self.mush[ar[:, None], self.sy, nxc]
        self.sy = torch.where(mv & blocked, (self.sy + 1).clamp(max=self.GH - 1), self.sy)
        self.sdir = torch.where(mv & blocked, -self.sdir, self.sdir)
        self.sx = torch.where(mv & ~blocked, nx, self.sx)
        reach = (self.salive & (self.sy >= self.GH - 1)).any(1)
        self.lives = self.lives - reach.long()
        k = torch.arange(self.NS, device=d)[None]
        self.sy = torch.where(reach[:, None], torch.zeros_like(self.sy), self.sy)
        self.sx = torch.where(reach[:, None], (self.GW - 1 - k).expand_as(self.sx).clamp(min=0), self.sx)
        self.sdir = torch.where(reach[:, None], -torch.ones_like(self.sdir), self.sdir)
        # wave cleared -> new centipede
        cleared = ~self.salive.any(1)
        self.salive = self.salive | cleared[:, None]
        self.sy = torch.where(cleared[:, None], torch.zeros_like(self.sy), self.sy)
        return reward

    def game_over(self):
        return self.lives <= 0

    def scene(self) -> Scene:
        sc = Scene(self.num_envs, self.device)
        gy = torch.arange(self.GH, device=self.device).repeat_interleave(self.GW)
        gx = torch.arange(self.GW, device=self.device).repeat(self.GH)
        sc.add_many(20 + gy * 8, gx * 10, 8, 10, [(181, 83, 40)] * (self.GH * self.GW),
                    visible=self.mush.reshape(self.num_envs, -1))
        sc.add_many(20 + self.sy * 8 + 1, self.sx * 10 + 1, 6, 8, [(184, 70, 162)] * self.NS, visible=self.salive)
        sc.add(184, self.px, 8, 4, (181, 108, 224))
        sc.add(self.shy, self.shx, 6, 1, (181, 108, 224), visible=self.shot)
        return sc


GAMES = {"Breakout": BreakoutVec, "SpaceInvaders": SpaceInvadersVec, "Alien": AlienVec, "MsPacman": MsPacmanVec,
         "Centipede": CentipedeVec}


def make_game(name: str, **kw) -> PixelGameVec:
    return GAMES[name](**kw)
