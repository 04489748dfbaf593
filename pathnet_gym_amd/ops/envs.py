"""HIP env stepping (``csrc/envs.hip``) for the on-device environments.

Two entry points per env:
* ``*_step_into``: engine path -- reads obs slot t, writes slot t+1 and the
  reward/done/episode-return rows of the rollout buffers in ONE launch;
* ``*_step``: the generic VecEnv API (allocates outputs), used by tests to
  compare bit-for-bit against the torch implementation.
"""
from __future__ import annotations

import os

import ctypes

import torch

from . import _lib


def _id_base(env) -> int:
    """Global index of the env's first instance: the RNG identity of instance b is id_base + b, so a population
    sharded over ranks draws the same random streams as on one GPU (envs/base.py VecEnv.set_id_base)."""
    return int(getattr(env, "id_base", 0)) & 0xFFFFFFFF


# ------------------------------------------------------------------ Pong
def pong_sync_to_device(env):
    """(Re)build the int32 kernel state from the torch (int64) state."""
    env._st32 = env.state.to(torch.int32).contiguous()
    env._ctr32 = env.counter.to(torch.int32).contiguous()
    env._tab32 = pong_tables(env)


def pong_tables(env) -> torch.Tensor:
    """The Pong step kernels' tables buffer: the [8][160] resize tables followed by the score-digit boxes of every
    score (csrc/envs.hip launch_pong_digit_tables, built here once per env object)."""
    if not hasattr(env, "_gray"):
        env._gray = _gray_consts(env)
    g = env._gray
    lib = _lib.lib()
    tab = torch.zeros(int(lib.pong_tables_ints()), dtype=torch.int32, device=env.tables.device)
    tab[: 8 * 160] = env.tables.to(torch.int32).reshape(-1)
    _lib.call("launch_pong_digit_tables", tab.data_ptr(), g[0], g[1], g[2], g[3], g[4], _lib.stream())
    return tab


def pong_sync_from_device(env):
    env.state = env._st32.to(torch.int64)
    env.counter = env._ctr32.to(torch.int64) & 0xFFFFFFFF


def _gray_consts(env):
    from ..envs import pong as pg
    wr, wg, wb = pg.gray_weights(env.gray)

    def g(c):
        return (c[0] * wr + c[1] * wg + c[2] * wb + 8192) >> 14
    return [g(pg.COLOR_BG), g(pg.COLOR_WALL), g(pg.COLOR_CPU), g(pg.COLOR_PLAYER), g(pg.COLOR_BALL)]


def pong_step_into(env, actions, obs_in, obs_out, reward, done, epret, b0: int = 0, b1=None):
    """One step of envs [b0, b1) (default all; the split rollout steps one path group per call)."""
    B = env.num_envs
    b1 = B if b1 is None else b1
    if not 0 <= b0 < b1 <= B:
        raise ValueError(f"pong_step_into: env range [{b0}, {b1}) outside [0, {B})")
    if not hasattr(env, "_st32"):
        pong_sync_to_device(env)
    _lib.check(actions, torch.int32, (B,), name="actions")
    _lib.check(obs_in, torch.uint8, numel=B * 160 * 120 * 4, name="obs_in")
    _lib.check(obs_out, torch.uint8, numel=B * 160 * 120 * 4, name="obs_out")
    _lib.check(reward, torch.float32, numel=B, name="reward")
    _lib.check(done, torch.uint8, numel=B, name="done")
    _lib.check(epret, torch.float32, numel=B, name="epret")
    if not hasattr(env, "_gray"):
        env._gray = _gray_consts(env)
    g = env._gray
    _lib.call("launch_pong_step", env._st32.data_ptr(), env._ctr32.data_ptr(), actions.data_ptr(), env.num_actions,
              obs_in.data_ptr(), obs_out.data_ptr(), env._tab32.data_ptr(), reward.data_ptr(), done.data_ptr(),
              epret.data_ptr(), b1, env.seed_int, env.frameskip, env.max_episode_steps,
              env.no_op_max, g[0], g[1], g[2], g[3], g[4], b0, _id_base(env), _lib.stream())


def pong_step_ring_into(env, actions, frames, slot, fc_in, fc_out, reward, done, epret, b0: int = 0, b1=None):
    """Frame-ring engine path: write only the new newest frame plane frames[:, slot] of the ring
    [B][slots][160*120] and the next stack's first valid channel (csrc/envs.hip RING;
    runtime/engine.py frame ring).  Envs [b0, b1) only (default all): one path group of the split rollout."""
    B = env.num_envs
    b1 = B if b1 is None else b1
    if not 0 <= b0 < b1 <= B:
        raise ValueError(f"pong_step_ring_into: env range [{b0}, {b1}) outside [0, {B})")
    if not hasattr(env, "_st32"):
        pong_sync_to_device(env)
    _lib.check(actions, torch.int32, (B,), name="actions")
    _lib.check(frames, torch.uint8, name="frames")
    if frames.dim() != 3 or frames.shape[0] != B or frames.shape[2] != 160 * 120 or not 0 <= slot < frames.shape[1]:
        raise ValueError(f"frames {tuple(frames.shape)} / slot {slot} do not match [{B}, slots, 19200]")
    _lib.check(fc_in, torch.uint8, numel=B, name="fc_in")
    _lib.check(fc_out, torch.uint8, numel=B, name="fc_out")
    _lib.check(reward, torch.float32, numel=B, name="reward")
    _lib.check(done, torch.uint8, numel=B, name="done")
    _lib.check(epret, torch.float32, numel=B, name="epret")
    if not hasattr(env, "_gray"):
        env._gray = _gray_consts(env)
    g = env._gray
    _lib.call("launch_pong_step_ring_split", env._st32.data_ptr(), env._ctr32.data_ptr(), actions.data_ptr(),
              env.num_actions, frames[0, slot].data_ptr(), frames.stride(0), fc_in.data_ptr(), fc_out.data_ptr(),
              env._tab32.data_ptr(),
              reward.data_ptr(), done.data_ptr(), epret.data_ptr(), b1, env.seed_int, env.frameskip,
              env.max_episode_steps, env.no_op_max, g[0], g[1], g[2], g[3], g[4], _id_base(env), b0,
              ring_split(b1 - b0), _lib.stream())


def pong_heads_step_ring_into(env, feat, flat, heads, logits, value, actions, seed, ctr, t, T, row_base, frames, slot,
                              fc_in, fc_out, reward, done, epret):
    """The frame-ring step of every env with the actor-critic heads + Gumbel-max sampling of its sample folded into
    the same workgroup (csrc/envs.hip pong_step_kernel<true, true>): feat [B, 256] fp32 = step t's trunk features,
    heads = the parameter offsets {pw, pb, vw, vb}; writes logits [B, A], value [B] and actions [B] exactly as
    HipPathNet.heads_fwd would, then steps the env with those actions."""
    B = env.num_envs
    if not hasattr(env, "_st32"):
        pong_sync_to_device(env)
    _lib.check(feat, torch.float32, (B, 256), name="feat")
    _lib.check(logits, torch.float32, numel=B * env.num_actions, name="logits")
    _lib.check(value, torch.float32, numel=B, name="value")
    _lib.check(actions, torch.int32, (B,), name="actions")
    _lib.check(frames, torch.uint8, name="frames")
    if frames.dim() != 3 or frames.shape[0] != B or frames.shape[2] != 160 * 120 or not 0 <= slot < frames.shape[1]:
        raise ValueError(f"frames {tuple(frames.shape)} / slot {slot} do not match [{B}, slots, 19200]")
    for tns, nm in ((fc_in, "fc_in"), (fc_out, "fc_out"), (done, "done")):
        _lib.check(tns, torch.uint8, numel=B, name=nm)
    for tns, nm in ((reward, "reward"), (epret, "epret")):
        _lib.check(tns, torch.float32, numel=B, name=nm)
    if not hasattr(env, "_gray"):
        env._gray = _gray_consts(env)
    g = env._gray
    _lib.call("launch_pong_heads_step_ring", env._st32.data_ptr(), env._ctr32.data_ptr(), env.num_actions,
              frames[0, slot].data_ptr(), frames.stride(0), fc_in.data_ptr(), fc_out.data_ptr(), env._tab32.data_ptr(),
              reward.data_ptr(), done.data_ptr(), epret.data_ptr(), B, env.seed_int, env.frameskip,
              env.max_episode_steps, env.no_op_max, g[0], g[1], g[2], g[3], g[4], _id_base(env), 0,
              feat.data_ptr(), 256, flat.data_ptr(), heads["pw"], heads["pb"], heads["vw"], heads["vb"],
              logits.data_ptr(), value.data_ptr(), actions.data_ptr(), seed & 0xFFFFFFFF, ctr.data_ptr(), t, T,
              int(row_base) & 0xFFFFFFFF, _lib.stream())


def ring_split(B: int) -> int:
    """Render workgroups per env of the frame-ring Pong step (csrc/envs.hip launch_pong_step_ring_split).  Default 1:
    the fused one-workgroup-per-env kernel.  Measured at 8 paths x 32 envs (profiles/r5/): physics 5.4 + split-4
    render 18.5 us vs 20.5 us fused -- a render workgroup's latency is its scene tables, not its quad walk -- so the
    split is kept for A/B runs only (PATHNET_PONG_SPLIT=N)."""
    v = os.environ.get("PATHNET_PONG_SPLIT")
    return max(1, int(v)) if v is not None else 1


def pong_step(env, actions, obs):
    B = env.num_envs
    dev = obs.device
    out = torch.empty_like(obs)
    reward = torch.empty(B, dtype=torch.float32, device=dev)
    done = torch.empty(B, dtype=torch.uint8, device=dev)
    epret = torch.empty(B, dtype=torch.float32, device=dev)
    pong_step_into(env, actions.to(torch.int32).contiguous(), obs.contiguous(), out, reward, done, epret)
    env.obs = out
    return out.clone(), reward, done.bool(), {"episode_return": epret}


# ------------------------------------------------------------------ CartPole
def cartpole_sync_to_device(env):
    env._steps32 = env.steps.to(torch.int32).contiguous()
    env._ctr32 = env.counter.to(torch.int32).contiguous()
    env.state = env.state.contiguous()
    env.ep_ret = env.ep_ret.contiguous()


def cartpole_step_into(env, actions, obs_bf16_out, reward, done, epret, obs_f32_out=None):
    B = env.num_envs
    if not hasattr(env, "_steps32"):
        cartpole_sync_to_device(env)
    _lib.check(actions, torch.int32, (B,), name="actions")
    if obs_bf16_out is not None:
        _lib.check(obs_bf16_out, torch.bfloat16, numel=B * 8, name="obs_bf16")
    _lib.call("launch_cartpole_step", env.state.data_ptr(), env._steps32.data_ptr(), env.ep_ret.data_ptr(),
              env._ctr32.data_ptr(), actions.data_ptr(), B, env.seed_int, _id_base(env),
              env.max_episode_steps, _lib.ptr(obs_f32_out), _lib.ptr(obs_bf16_out), reward.data_ptr(),
              done.data_ptr(), epret.data_ptr(), _lib.stream())


def cartpole_step(env, actions):
    B = env.num_envs
    dev = env.state.device
    obs = torch.empty(B, 4, dtype=torch.float32, device=dev)
    reward = torch.empty(B, dtype=torch.float32, device=dev)
    done = torch.empty(B, dtype=torch.uint8, device=dev)
    epret = torch.empty(B, dtype=torch.float32, device=dev)
    cartpole_step_into(env, actions.to(torch.int32).contiguous(), None, reward, done, epret, obs_f32_out=obs)
    return obs, reward, done.bool(), {"episode_return": epret}


def obs_to_bf16_padded(obs_f32: torch.Tensor) -> torch.Tensor:
    """[B, d<=8] float -> [B, 8] bf16 zero padded (trunk input for vector envs)."""
    B, d = obs_f32.shape
    out = torch.zeros(B, 8, dtype=torch.bfloat16, device=obs_f32.device)
    out[:, :d] = obs_f32.to(torch.bfloat16)
    return out


# ------------------------------------------------------------------ RGB frame preprocessing (K15/K16)
def rgb_stack_push(rgb: torch.Tensor, obs_in: torch.Tensor, obs_out: torch.Tensor, reset, tables: torch.Tensor,
                   gray: str = "rgb"):
    """[N,210,160,3] uint8 frames -> gray + bilinear 160x120 + push into the uint8 [N,160,120,4] stack.

    ``reset`` (bool/uint8 [N] or None): rows whose stack is re-filled with the new frame (episode start).
    Bit-exact with ``envs/pong.py:preprocess_frames`` + the torch stack push.
    """
    from ..envs.pong import gray_weights
    N = rgb.shape[0]
    _lib.check(rgb, torch.uint8, shape=(N, 210, 160, 3), name="rgb")
    _lib.check(obs_out, torch.uint8, numel=N * 160 * 120 * 4, name="obs_out")
    _lib.check(obs_in, torch.uint8, numel=N * 160 * 120 * 4, name="obs_in")
    tab = tables.to(device=rgb.device, dtype=torch.int32).contiguous()
    r8 = None
    if reset is not None:
        r8 = _lib.check(reset.to(torch.uint8).contiguous(), torch.uint8, numel=N, name="reset")
    wr, wg, wb = gray_weights(gray)
    _lib.call("launch_rgb_stack_push", rgb.data_ptr(), obs_in.data_ptr(), obs_out.data_ptr(), _lib.ptr(r8),
              tab.data_ptr(), N, int(wr), int(wg), int(wb), _lib.stream())


def rects_stack_push(geom: torch.Tensor, colors, bg, obs_in: torch.Tensor, obs_out: torch.Tensor, reset,
                     tables: torch.Tensor, gray: str = "rgb"):
    """Rasterise a rectangle scene ([N, R, 4] y0/x0/h/w, painter's order) + preprocess + stack push on device."""
    from ..envs.pong import gray_weights
    N, R = geom.shape[0], geom.shape[1]
    _lib.check(obs_out, torch.uint8, numel=N * 160 * 120 * 4, name="obs_out")
    _lib.check(obs_in, torch.uint8, numel=N * 160 * 120 * 4, name="obs_in")
    g16 = geom.clamp(-32768, 32767).to(torch.int16).contiguous()
    wr, wg, wb = gray_weights(gray)
    lum = lambda c: (c[0] * wr + c[1] * wg + c[2] * wb + 8192) >> 14      # noqa: E731  cv2 fixed-point luma
    key = (tuple(colors), gray, str(geom.device))
    cache = rects_stack_push.__dict__.setdefault("_gray", {})
    if key not in cache:
        cache[key] = torch.tensor([lum(c) for c in colors], dtype=torch.uint8, device=geom.device)
    tab = tables.to(device=geom.device, dtype=torch.int32).contiguous()
    r8 = None if reset is None else _lib.check(reset.to(torch.uint8).contiguous(), torch.uint8, numel=N, name="reset")
    _lib.call("launch_rects_stack_push", g16.data_ptr(), cache[key].data_ptr(), R, int(lum(bg)), obs_in.data_ptr(),
              obs_out.data_ptr(), _lib.ptr(r8), tab.data_ptr(), N, _lib.stream())


# ------------------------------------------------------------------ synthetic Atari-style games (csrc/games.hip)
GAME_IDS = {"Breakout": 0, "SpaceInvaders": 1, "Alien": 2, "MsPacman": 3, "Centipede": 4}


def game_layout(game: str):
    """(ints of state per env, rectangles per scene) of a HIP game."""
    ns, nr = ctypes.c_int(0), ctypes.c_int(0)
    _lib.call("game_layout", GAME_IDS[game], ctypes.byref(ns), ctypes.byref(nr))
    return ns.value, nr.value


def game_step(game: str, state: torch.Tensor, actions, mask, n_actions: int, seed: int, frameskip: int,
              max_steps: int, reward: torch.Tensor, done: torch.Tensor, epret: torch.Tensor, rects: torch.Tensor,
              id_base: int = 0):
    """One launch: agent step of every env (``actions`` int32 [N]) or, with ``mask`` (uint8 [N]) instead,
    ``reset_where``; writes reward/done/episode-return rows and the int16 scene [N, R, 4]."""
    N = state.shape[0]
    ns, nr = game_layout(game)
    _lib.check(state, torch.int32, (N, ns), name="state")
    _lib.check(rects, torch.int16, (N, nr, 4), name="rects")
    _lib.check(reward, torch.float32, numel=N, name="reward")
    _lib.check(done, torch.uint8, numel=N, name="done")
    _lib.check(epret, torch.float32, numel=N, name="epret")
    if actions is not None:
        _lib.check(actions, torch.int32, (N,), name="actions")
    if mask is not None:
        _lib.check(mask, torch.uint8, (N,), name="mask")
    _lib.call("launch_game_step", GAME_IDS[game], state.data_ptr(), _lib.ptr(actions), _lib.ptr(mask),
              0 if mask is None else 1, n_actions, N, seed & 0xFFFFFFFF, id_base & 0xFFFFFFFF, frameskip, max_steps,
              reward.data_ptr(),
              done.data_ptr(), epret.data_ptr(), rects.data_ptr(), _lib.stream())


def rects16_stack_push(rects: torch.Tensor, gray_tab: torch.Tensor, bg_gray: int, obs_in: torch.Tensor,
                       obs_out: torch.Tensor, reset, tables32: torch.Tensor):
    """``rects_stack_push`` for a scene that is already int16 [N, R, 4] with a precomputed per-rectangle gray
    table (the HIP games write their scene that way; no conversions, capturable)."""
    N, R = rects.shape[0], rects.shape[1]
    _lib.check(rects, torch.int16, (N, R, 4), name="rects")
    _lib.check(gray_tab, torch.uint8, (R,), name="gray_tab")
    _lib.check(obs_out, torch.uint8, numel=N * 160 * 120 * 4, name="obs_out")
    _lib.check(obs_in, torch.uint8, numel=N * 160 * 120 * 4, name="obs_in")
    _lib.check(tables32, torch.int32, name="tables")
    if reset is not None:
        _lib.check(reset, torch.uint8, numel=N, name="reset")
    _lib.call("launch_rects_stack_push", rects.data_ptr(), gray_tab.data_ptr(), R, int(bg_gray), obs_in.data_ptr(),
              obs_out.data_ptr(), _lib.ptr(reset), tables32.data_ptr(), N, _lib.stream())


def rects16_ring_push(rects: torch.Tensor, gray_tab: torch.Tensor, bg_gray: int, frames: torch.Tensor, slot: int,
                      fc_in: torch.Tensor, fc_out: torch.Tensor, reset, tables32: torch.Tensor):
    """Frame-ring form of ``rects16_stack_push`` (csrc/preprocess.hip rects_push_kernel<true>): write only the new
    plane frames[:, slot] of the engine's ring [N][slots][160*120] and the next stack's first valid channel
    fc_out = reset ? 3 : max(fc_in - 1, 0) (runtime/engine.py frame ring)."""
    N, R = rects.shape[0], rects.shape[1]
    _lib.check(rects, torch.int16, (N, R, 4), name="rects")
    _lib.check(gray_tab, torch.uint8, (R,), name="gray_tab")
    _lib.check(frames, torch.uint8, name="frames")
    if frames.dim() != 3 or frames.shape[0] != N or frames.shape[2] != 160 * 120 or not 0 <= slot < frames.shape[1]:
        raise ValueError(f"frames {tuple(frames.shape)} / slot {slot} do not match [{N}, slots, 19200]")
    _lib.check(fc_in, torch.uint8, numel=N, name="fc_in")
    _lib.check(fc_out, torch.uint8, numel=N, name="fc_out")
    _lib.check(tables32, torch.int32, name="tables")
    if reset is not None:
        _lib.check(reset, torch.uint8, numel=N, name="reset")
    _lib.call("launch_rects_ring_push", rects.data_ptr(), gray_tab.data_ptr(), R, int(bg_gray),
              frames[0, slot].data_ptr(), frames.stride(0), fc_in.data_ptr(), fc_out.data_ptr(), _lib.ptr(reset),
              tables32.data_ptr(), N, _lib.stream())
