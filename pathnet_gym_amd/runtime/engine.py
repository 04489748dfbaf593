"""HIP rollout/update engine: static buffers + hipGraph-captured update.

One A2C update of the local population (P paths x E envs, T steps) is a
fixed sequence of kernel launches on one stream:

  for t in 0..T-1:                                   (rollout)
      trunk fwd layer 0..L-1   (obs[t] -> acts[l][t], ReLU bits)
      heads fwd + Gumbel-max sample  (logits[t], values[t], actions[t])
      env step                 (obs[t] -> obs[t+1], rewards/dones/epret[t])
  trunk+heads fwd on obs[T] (greedy) -> bootstrap value
  fitness update (per-path last-episode return) + counters
  a2c_grad                     (reverse scan + analytic loss gradient)
  memset grad; heads bwd; for l = L-1..0: wgrad_l (+ dgrad_l)
  -------------------------------- fused RCCL all-reduce (outside the graph)
  clip + RMSProp + refresh bf16 weight copies; obs[0] <- obs[T]; ctr += 1

All shapes and addresses are static (genotype changes only rewrite the
compacted index tensors in place), so the two halves are captured once as
hipGraphs (``torch.cuda.graph`` over our ctypes launches) and replayed:
~(T*(L+2)+2L+6) launches become two graph launches per update.  This is
the MI355X replacement for the reference's per-step ``sess.run`` over gRPC
(SURVEY.md call sites C1-C3).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..ops import _lib
from ..ops import envs as henv


# hipGraph capture mode: thread-local, so other threads' HIP calls stay legal during a capture.  The RCCL process
# group's watchdog thread polls the completion events of earlier collectives; under the default global mode a poll
# that lands inside a capture fails with hipErrorStreamCaptureUnsupported and aborts the process (seen when a second
# trainer captured its graphs after the first one's all-reduces: bench.py strong / per-rank windows, in-run solve).
CAPTURE_MODE = "thread_local"


def loss_scale(cfg) -> float:
    """grad_scale x (1 / world size when rank_reduction == "mean"): the factor on every sample's loss weight."""
    a2c = cfg.a2c
    world = 1
    if getattr(a2c, "rank_reduction", "sum") == "mean":
        import torch.distributed as dist
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    return float(getattr(a2c, "grad_scale", 1.0)) / world


class HipEngine:
    def __init__(self, model, env, cfg, opt, seed: int = 1, row_base: int = 0):
        self.model = model
        self.hip = model.hip
        self.env = env
        self.cfg = cfg
        self.opt = opt
        self.seed = seed & 0xFFFFFFFF
        # global index of this rank's first env: action sampling draws the RNG of global sample row_base + b, so
        # a population sharded over ranks samples exactly what one GPU would (trainer: rank * P * E)
        self.row_base = int(row_base)
        a2c = cfg.a2c
        self.T = T = a2c.t_max
        self.P = P = model.P
        self.E = E = cfg.envs_per_path
        self.B = B = P * E
        self.A = A = model.cfg.num_actions
        dev = model.device
        self.device = dev
        hp = self.hip
        self.pixels = hp.pixels
        # Frame ring (Pong, standard 160x120x4 trunk): the rollout keeps T+4 single frame planes
        # instead of T+1 packed 4-frame stacks; stack t = frames t..t+3 (newest last) with the
        # channels before fc[t] replaced by the first valid frame after an episode reset.  The env
        # step writes 19.2 KB per env instead of reading + writing a 77 KB stack.
        self.ring = bool(self.pixels and getattr(cfg, "frame_ring", True) and hp.ring_ok and _lib.USE_FAST
                         and hasattr(env, "step_ring_into") and getattr(env, "supports_ring", True))
        # observation double buffer (non-ring): the rollout of parity q reads bufs[q][0..T-1] and its last
        # env step writes the NEXT rollout's step-0 input straight into bufs[1-q][0] (the bootstrap forward
        # reads it there), so no obs[0] <- obs[T] copy of the whole stack batch (157 MB at the bench shape)
        # runs per update; one rollout hipGraph per parity, the parity flips after every optimizer step
        self._obs_bufs = None
        self._par = 0
        if self.ring:
            H, W, C = model.cfg.input_shape
            hp.enable_ring()
            self.HW = H * W
            # fp32x: a MODULAR ring of 2T slots (T >= 4): the rollout of parity q starts at base slot q*T, step t's
            # channel k is slot (q*T + t + max(k, fc[t])) mod 2T, so the next rollout's first stack is already in
            # place (no per-update copy of the last 4 planes: 157 MB, 51 us at 64 paths); other modes copy them
            nsl = 2 * T if (hp.x3 and T >= 4) else T + 4
            self.frames = torch.zeros(B, nsl, H * W, dtype=torch.uint8, device=dev)   # env-major: a stack is contiguous
            self.fc = torch.zeros(T + 1, B, dtype=torch.uint8, device=dev)
        elif self.pixels:
            H, W, C = model.cfg.input_shape
            self._obs_bufs = [torch.zeros(T, B, H * W * C, dtype=torch.uint8, device=dev) for _ in range(2)]
        elif hp.f32:
            self._obs_bufs = [torch.zeros(T, B, hp.geoms[0].ldx, dtype=torch.float32, device=dev) for _ in range(2)]
        else:
            self._obs_bufs = [torch.zeros(T, B, 8, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        self.acts, self.bits, self.bits_rows, self.grads = [], [], [], []
        # conv-layer output gradients kept in bf16 where the specialised dgrad / wgrad kernels take them
        # (grads[0] is 1.5 GB and grads[1] 0.3 GB in fp32 at the bench shape)
        bf16_grads = hp.grad_bf16_layers(self.ring)
        for l, g in enumerate(hp.geoms):
            self.acts.append(hp.alloc_act(l, (T + 1, B, g.out_feat)))
            b, rows = hp.alloc_bits(l, T + 1, B)
            self.bits.append(b)
            self.bits_rows.append(rows)
            self.grads.append(torch.zeros(T * B, g.out_feat, dtype=torch.bfloat16 if l in bf16_grads else torch.float32,
                                          device=dev))
        self.logits = torch.zeros(T + 1, B, A, device=dev)
        self.values = torch.zeros(T + 1, B, device=dev)
        self.actions = torch.zeros(T + 1, B, dtype=torch.int32, device=dev)
        self.rewards = torch.zeros(T, B, device=dev)
        self.dones = torch.zeros(T, B, dtype=torch.uint8, device=dev)
        self.epret = torch.zeros(T, B, device=dev)
        self.dlogits = torch.zeros(T, B, A, device=dev)
        self.dvalue = torch.zeros(T, B, device=dev)
        self.stats = torch.zeros(4, device=dev)          # a2c_grad: loss_pi, loss_v, entropy sum
        self.grad_flat = torch.zeros_like(model.store.flat, requires_grad=False)
        self.fitness = torch.full((P,), -1000.0, device=dev)
        # windowed fitness (GAConfig.fitness == "mean"): episodes / return sum since the path's last tournament
        self.fit_window = cfg.ga.window_for(E)
        self.fit_cnt = torch.zeros(P, device=dev)
        self.fit_sum = torch.zeros(P, device=dev)
        self.counters = torch.zeros(4, device=dev)
        self.path_part = torch.zeros(P, 2, device=dev)     # per-path (episodes, return sum) of the last rollout
        self.ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr = torch.zeros(2, dtype=torch.float32, device=dev)      # {lr, skip}
        # the lr anneal on device (optimizer tail, csrc/ga.hip opt_tail_kernel): {lr0, max_t, mode, frames per update,
        # frames done on the anneal clock}; the tail writes the next update's lr into self.lr, so the steady-state update
        # needs no host fill (optimizer_step re-seeds it whenever the host's clock is not the one the device predicted)
        world = 1
        import torch.distributed as _dist
        if _dist.is_available() and _dist.is_initialized():
            world = _dist.get_world_size()
        self.frames_per_update = T * P * E * world
        self.lr_sched = torch.tensor([float(a2c.lr), float(a2c.max_time_step), 0.0 if a2c.lr_anneal == "none" else 1.0,
                                      float(self.frames_per_update), 0.0], dtype=torch.float64, device=dev)
        self._next_t = None
        self._skip_set = False
        self.weight = ((1.0 / E) if a2c.env_reduction == "mean_env" else 1.0) * loss_scale(cfg)
        # end of the first layer's parameters (the overlapped exchange's second bucket, runtime/engine.py split)
        self._l0_end = max((s.offset + s.numel for s in model.store.layout.segments if s.layer == 0), default=0)
        # optimizer block table (segments split into <= 8192-element blocks)
        self._build_opt_tables()
        self.g_rollout = None
        self.g_opt = None
        self.ga_dev = None
        # overlapped all-reduce (TrainConfig.overlap_allreduce, world > 1): the rollout graph is captured as a head
        # (everything but the first layer's backward) and a tail (that backward), replayed around the bucket-1
        # all-reduce (parallel/comm.py exchange_async_split)
        self.split = False
        # LSTM nets: fused HIP LSTM cell (csrc/lstm.hip) when the widths are multiples of 64; otherwise
        # the hybrid path (HIP trunk + autograd LSTM/heads/loss, dL/dfeat fed back to the HIP trunk backward)
        self.lstm_hip = hp.lstm is not None
        self.hybrid = bool(model.cfg.use_lstm) and not self.lstm_hip
        self.lstm_state = model.init_state(B) if self.hybrid else None
        if self.lstm_hip:
            F, H = hp.lstm["F"], hp.lstm["H"]
            ldt = hp.lstm_dtype                  # bf16 (bf16 engine) or fp32 (fp32x: csrc/lstm_x3.hip)
            hp.lstm_prepare(T)
            self.hst = torch.zeros(T + 2, B, H, dtype=ldt, device=dev)   # slot t = state entering step t
            self.cst = torch.zeros(T + 2, B, H, device=dev)
            self.gates = torch.zeros(T, B, 4 * H, device=dev)
            self.xh = torch.zeros(T, B, F + H, dtype=ldt, device=dev)
            self.dz = torch.zeros(T, B, 4 * H, device=dev)
            self.dh_heads = torch.zeros(T, B, H, device=dev)
            self.dh_rec = torch.zeros(2, B, H, device=dev)
            self.dc_rec = torch.zeros(2, B, H, device=dev)
        # torch-implemented games (envs/atari_games.py) are stepped eagerly, outside hipGraphs
        self.env_graph_safe = getattr(env, "graph_safe", True)
        self.use_graph = bool(cfg.use_graph) and not self.hybrid and self.env_graph_safe
        # the heads + sampling of rollout steps 0..T-1 folded into the env step (frame-ring Pong, fp32 features):
        # one launch per step less (csrc/envs.hip pong_step_kernel HEADS)
        self.fuse_env_heads = (self.ring and getattr(env, "ring_heads", False) and hp.feat_dtype == torch.float32
                               and not self.lstm_hip and not self.hybrid and self.env_graph_safe
                               and model.cfg.num_actions <= 8 and hp.geoms[-1].out_feat == 256
                               and os.environ.get("PATHNET_FUSE_ENV_HEADS", "1") != "0")
        self.auto_group_max_paths = int(os.environ.get("PATHNET_AUTO_GROUP_MAX_PATHS", "0"))
        self.groups = self._rollout_groups(getattr(cfg, "rollout_groups", 0))
        self.side_streams = [torch.cuda.Stream(device=dev) for _ in range(self.groups - 1)]
        self.ring_mod = bool(self.ring and hp.x3 and self.groups == 1 and T >= 4 and self.frames.shape[1] == 2 * T)
        if self.groups > 1 and self.ring:
            for g in range(self.groups):
                p0, np_ = self._group_range(g)
                hp.prepare_group(p0, np_, rows=np_ * E)
        self.load_obs(env)

    def _rollout_groups(self, want: int) -> int:
        """Path groups of the split rollout (TrainConfig.rollout_groups): each group's forward + env step chain
        runs on its own stream (a branch of the rollout hipGraph).  Needs per-range launches: the Pong kernels
        (pong_step_into / pong_step_ring_into b0/b1), the trunk forward (HipPathNet.layer_fwd row0/p0; on the frame
        ring, fp32x: ring_fwd / conv23_fwd at the group's base and the module-major fc forward on the group's own
        inverse lists) and the heads (heads_fwd b0/b1).  0 = auto = one group: two were 3 % slower at 64 paths in
        bf16 (round 1), and on the fp32x frame ring (profiles/r5/groups_sweep.md) 3.43 (1) / 3.45 (2) / 3.81 (4) ms
        at 8 paths, 4.31 / 4.37 / 4.76 at 16, 6.13 / 6.33 at 32: a 4-path group's kernels take as long as the
        8-path ones (their latency is one workgroup's chain) and two concurrent chains run ~1.55x, not 2x, the
        work of one.  PATHNET_AUTO_GROUP_MAX_PATHS=N makes auto pick two groups at <= N paths."""
        packed = (self.pixels and not self.ring and not hasattr(self.env, "step_into"))
        ring = self.ring and self.hip.x3 and getattr(self.env, "ring_ranges", False)
        ok = (packed or ring) and not self.lstm_hip and not self.hybrid and self.env_graph_safe
        if want == 0:
            want = 2 if (ring and ok and self.P <= self.auto_group_max_paths and self.P % 2 == 0) else 1
        if want > 1 and (not ok or self.P % want != 0):
            raise ValueError(f"rollout_groups={want} needs a packed-stack pixel env (or the fp32x frame ring with a "
                             f"ranged env step) without LSTM and paths ({self.P}) divisible by it")
        return max(1, want)

    # -- observation double buffer -------------------------------------------
    @property
    def obs(self):
        """[T, B, ...] observations of the current rollout (steps 0..T-1); None with the frame ring."""
        return None if self._obs_bufs is None else self._obs_bufs[self._par]

    @property
    def rbase(self) -> int:
        """Base slot of the running rollout in the modular frame ring (parity x T), 0 otherwise."""
        return self._par * self.T if self.ring_mod else 0

    def _slot(self, t: int) -> int:
        """Frame-ring slot of plane t of the running rollout (t = 0..T+3: step t's newest channel is plane t + 3)."""
        return (self.rbase + t) % self.frames.shape[1] if self.ring_mod else t

    @property
    def _parities(self) -> bool:
        """Two rollout graphs, one per parity (observation double buffer, or the modular frame ring)."""
        return self._obs_bufs is not None or self.ring_mod

    def _obs_at(self, t: int) -> torch.Tensor:
        """Input of step t (t == T: the bootstrap input = the next rollout's step 0, in the other buffer)."""
        return self._obs_bufs[self._par][t] if t < self.T else self._obs_bufs[1 - self._par][0]

    def _obs_x(self, t: int):
        """(buffer, first global row) of step t's observations for a trunk launch."""
        if t < self.T:
            return self._obs_bufs[self._par], t * self.B
        return self._obs_bufs[1 - self._par], 0

    # ------------------------------------------------------------------
    def load_obs(self, env):
        """Copy the env's current observation into slot 0."""
        o = env.obs if self.pixels else None
        if self.pixels:
            self.set_obs_stack0(o.reshape(self.B, -1))
        elif self.hip.f32:
            self.obs[0].copy_(env.state.float().reshape(self.B, -1))
        else:
            self.obs[0].copy_(henv.obs_to_bf16_padded(env.state.float()))

    # -- packed-stack views of the observation buffers (tests, checkpoints) -------
    def obs_stack(self, t: int) -> torch.Tensor:
        """Stack of step t as [B, H*W*4] uint8 (pixel-major, channel-minor, newest frame last)."""
        if not self.ring:
            return self._obs_at(t)
        B = self.B
        dev = self.device
        c = torch.arange(4, device=dev)
        idx = (self.rbase + t + torch.maximum(c[None, :], self.fc[t].long()[:, None])) % self.frames.shape[1]
        planes = self.frames[torch.arange(B, device=dev)[:, None], idx]           # [B, 4, H*W]
        return planes.permute(0, 2, 1).reshape(B, -1).contiguous()

    def obs_stacks(self, n: Optional[int] = None) -> torch.Tensor:
        """Stacks of steps 0..n-1 (default T+1) as [n, B, H*W*4] uint8 (or the vector obs)."""
        n = self.T + 1 if n is None else n
        if not self.ring:
            return self.obs[:n] if n <= self.T else torch.cat([self.obs, self._obs_at(self.T)[None]])[:n]
        return torch.stack([self.obs_stack(t) for t in range(n)])

    def set_obs_stack0(self, stack: torch.Tensor):
        """Install a packed [B, H*W*4] stack as the observation entering step 0."""
        if not self.ring:
            self.obs[0].copy_(stack.reshape(self.B, -1))
            return
        st = stack.reshape(self.B, self.HW, 4)
        for c in range(4):
            self.frames[:, self._slot(c)].copy_(st[:, :, c])
        self.fc[0].zero_()

    def _build_opt_tables(self):
        segs = self.model.store.layout.segments
        seg_id, beg, end, blk0 = [], [], [], []
        BLK = 8192
        for i, s in enumerate(segs):
            blk0.append(len(seg_id))
            o = s.offset
            while o < s.offset + s.numel:
                e = min(o + BLK, s.offset + s.numel)
                seg_id.append(i)
                beg.append(o)
                end.append(e)
                o = e
        blk0.append(len(seg_id))
        dev = self.device
        self.blk_seg = torch.tensor(seg_id, dtype=torch.int32, device=dev)
        self.blk_beg = torch.tensor(beg, dtype=torch.int64, device=dev)
        self.blk_end = torch.tensor(end, dtype=torch.int64, device=dev)
        self.seg_blk0 = torch.tensor(blk0, dtype=torch.int32, device=dev)
        self.nblk = len(seg_id)
        self.partial = torch.zeros(self.nblk + 1, dtype=torch.float32, device=dev)
        # 1.0 when the last optimizer step found a non-finite (all-reduced) gradient and skipped itself
        self.opt_status = torch.zeros(1, dtype=torch.float32, device=dev)
        # [loss_pi, loss_v, entropy, spare, previous optimizer step skipped] read back per update (pipelined mode)
        self.report = torch.zeros(5, dtype=torch.float32, device=dev)
        self.trainable_u8 = self.opt.seg_trainable.to(torch.uint8)

    def refresh_trainable(self):
        self.trainable_u8.copy_(self.opt.seg_trainable.to(torch.uint8))

    # ------------------------------------------------------------------
    def _group_range(self, grp):
        """(first path, path count) of path group grp (None: the whole population)."""
        if grp is None:
            return 0, self.P
        pg = self.P // self.groups
        return grp * pg, pg

    def _env_step(self, t, grp=None, heads=False):
        """Env step t (``heads``: with step t's heads + sampling folded in, fuse_env_heads)."""
        env = self.env
        if heads:
            m = self.model
            h = m.store.layout.heads[m.task if m.cfg.per_task_heads else 0]
            env.step_ring_heads_into(self.acts[-1][t], m.store.flat, h, self.logits[t], self.values[t],
                                     self.actions[t], self.seed, self.ctr, t, self.T + 1, self.row_base, self.frames,
                                     self._slot(t + 4), self.fc[t], self.fc[t + 1], self.rewards[t], self.dones[t],
                                     self.epret[t])
            return
        if grp is not None:
            p0, np_ = self._group_range(grp)
            if self.ring:
                env.step_ring_into(self.actions[t], self.frames, t + 4, self.fc[t], self.fc[t + 1], self.rewards[t],
                                   self.dones[t], self.epret[t], b0=p0 * self.E, b1=(p0 + np_) * self.E)
                return
            henv.pong_step_into(env, self.actions[t], self._obs_at(t), self._obs_at(t + 1), self.rewards[t],
                                self.dones[t], self.epret[t], b0=p0 * self.E, b1=(p0 + np_) * self.E)
            return
        if self.ring:
            env.step_ring_into(self.actions[t], self.frames, self._slot(t + 4), self.fc[t], self.fc[t + 1],
                               self.rewards[t], self.dones[t], self.epret[t])
        elif hasattr(env, "step_into"):
            env.step_into(self.actions[t], self._obs_at(t), self._obs_at(t + 1), self.rewards[t], self.dones[t],
                          self.epret[t])
        elif self.pixels:
            henv.pong_step_into(env, self.actions[t], self._obs_at(t), self._obs_at(t + 1), self.rewards[t],
                                self.dones[t], self.epret[t])
        elif self.hip.f32:
            henv.cartpole_step_into(env, self.actions[t], None, self.rewards[t], self.dones[t], self.epret[t],
                                    obs_f32_out=self._obs_at(t + 1))
        else:
            henv.cartpole_step_into(env, self.actions[t], self._obs_at(t + 1), self.rewards[t], self.dones[t],
                                    self.epret[t])

    def _trunk_step(self, t, grp=None, skip_last=False):
        """Trunk forward of step t (one path group, or all); ``skip_last``: every layer but the last (the caller runs
        the last layer fused with the heads)."""
        hp = self.hip
        nl = len(hp.geoms) - (1 if skip_last else 0)
        if self.ring:
            if grp is None:
                p0, np_, t0, row0 = 0, self.P, t, 0
                hp.ring_fwd(self.frames, self.fc, self.acts[0], self.bits[0], self.P, self.E, 1, t, self.bits_rows[0],
                            rbase=self.rbase)
            else:
                # one path group: every launch at the group's first row of step t, the kernels at t0 = 0
                p0, np_ = self._group_range(grp)
                t0, row0 = 0, t * self.B + p0 * self.E
                hp.ring_fwd(self.frames, self.fc, self.acts[0], self.bits[0], self.P, self.E, 1, t, self.bits_rows[0],
                            p0=p0, np_=np_)
            l = 1
            while l < nl:
                if l + 1 < nl and hp.conv23_fwd(l, self.acts[l - 1], self.acts[l], self.bits[l],
                                                           self.bits_rows[l], self.acts[l + 1], self.bits[l + 1],
                                                           self.bits_rows[l + 1], np_, self.E, 1, t0, row0=row0, p0=p0):
                    l += 2
                    continue
                hp.layer_fwd(l, self.acts[l - 1], self.acts[l], self.bits[l], np_, self.E, 1, t0, self.bits_rows[l],
                             row0=row0, p0=p0)
                l += 1
            return
        p0, np_ = self._group_range(grp)
        x, xrow0 = self._obs_x(t)
        row0 = t * self.B + p0 * self.E
        for l in range(nl):
            hp.layer_fwd(l, x, self.acts[l], self.bits[l], np_, self.E, 1, 0, self.bits_rows[l], row0=row0, p0=p0,
                         xrow0=xrow0 + p0 * self.E if l == 0 else None)
            x = self.acts[l]

    def _bwd_side_stream(self):
        """Side stream of the backward (fp32x, small populations): layer l's weight gradient runs there while the
        main stream computes its input gradient and the layers below -- the input-gradient chain is the critical
        path.  Measured (profiles/r5/kwin_p*_bwd_side.md): the concurrent kernels contend instead of overlapping at
        every population size (8 paths 3.59 -> 3.70 ms, 16 paths 4.63 -> 5.24 ms; the fc1 weight gradient 106 ->
        228 us), as two streams did at 64 paths in round 1, so it is off; PATHNET_BWD_STREAMS=2 turns it on."""
        import os
        on = os.environ.get("PATHNET_BWD_STREAMS") == "2"
        if not (on and self.hip.x3 and not self.hybrid):
            return None
        if getattr(self, "_bwd_side", None) is None:
            self._bwd_side = torch.cuda.Stream(device=self.device)
        return self._bwd_side

    def _layer_bwd_all(self, T, lo: int = 0, hi: Optional[int] = None):
        """Backward of layers hi-1 .. lo (default: all).  With a side stream (fp32x, small P) every layer's weight
        gradient is forked off after the main stream has issued that layer's input gradient (fc layers: which also
        writes the masked gradient the weight gradient reads; the last layer: the G16 amax) and joined at the end."""
        hp = self.hip
        P, E = self.P, self.E
        hi = len(hp.geoms) if hi is None else hi
        side = self._bwd_side_stream()
        main = torch.cuda.current_stream() if side is not None else None
        forked = False
        for l in range(hi - 1, lo - 1, -1):
            if l == 0 and self.ring:
                hp.ring_wgrad(self.frames, self.fc, self.grads[0], self.bits[0], self.grad_flat, P, E, T,
                              self.bits_rows[0], rbase=self.rbase)
                continue
            X = self.obs if l == 0 else self.acts[l - 1]
            dX = self.grads[l - 1] if l > 0 else None
            if side is None or dX is None:
                hp.layer_bwd(l, X, self.grads[l], self.bits[l], self.grad_flat, dX, P, E, T, self.bits_rows[l])
                continue
            hp.layer_bwd(l, X, self.grads[l], self.bits[l], self.grad_flat, dX, P, E, T, self.bits_rows[l], part="d")
            side.wait_stream(main)
            forked = True
            with torch.cuda.stream(side):
                hp.layer_bwd(l, X, self.grads[l], self.bits[l], self.grad_flat, dX, P, E, T, self.bits_rows[l],
                             part="w")
        if forked:
            main.wait_stream(side)

    def _fused_heads(self) -> bool:
        """fp32x rollout steps: the last fc layer, the heads and the sampling in one launch (HipPathNet.fc_heads_fwd)."""
        hp = self.hip
        L = len(hp.geoms)
        return (hp.x3 and hp.fuse_heads and not self.lstm_hip and not self.hybrid and L > 1
                and hp.geoms[-1].kind == "fc" and hp.geoms[-1].Cout == 256 and hp.geoms[-1].K == 256
                and self.E <= 32 and self.A <= 8)

    def _forward_step(self, t, greedy=False, grp=None, heads=True):
        """Forward of step t; ``heads`` False: the trunk only (the env step runs the heads, fuse_env_heads)."""
        hp = self.hip
        if not heads:
            self._trunk_step(t, grp)
            return
        if grp is None and self._fused_heads():
            self._trunk_step(t, None, skip_last=True)
            L = len(hp.geoms)
            if hp.fc_heads_fwd(self.acts[L - 2], self.acts[L - 1], self.bits[L - 1], self.bits_rows[L - 1],
                               self.logits[t], self.values[t], self.actions[t], self.seed, self.ctr, t, self.T + 1,
                               self.P, self.E, t, greedy=greedy, task=self.model.task, row_base=self.row_base):
                return
            hp.layer_fwd(L - 1, self.acts[L - 2], self.acts[L - 1], self.bits[L - 1], self.P, self.E, 1, t,
                         self.bits_rows[L - 1])
            hp.heads_fwd(self.acts[L - 1][t], self.logits[t], self.values[t], self.actions[t], self.seed, self.ctr, t,
                         self.T + 1, greedy=greedy, task=self.model.task, row_base=self.row_base)
            return
        self._trunk_step(t, grp)
        feat = self.acts[-1][t]
        if grp is not None:
            p0, np_ = self._group_range(grp)
            hp.heads_fwd(feat, self.logits[t], self.values[t], self.actions[t], self.seed, self.ctr, t, self.T + 1,
                         greedy=greedy, task=self.model.task, b0=p0 * self.E, b1=(p0 + np_) * self.E,
                         row_base=self.row_base)
            return
        if self.lstm_hip:
            # state entering step t: slot t, reset where the previous step ended an episode
            # (slot 0 is pre-masked by the carry at the end of the previous update)
            last = t >= self.T
            hp.lstm_fwd(feat, self.hst[t], self.cst[t], self.dones[t - 1] if t > 0 else None, self.hst[t + 1],
                        self.cst[t + 1], None if last else self.gates[t], None if last else self.xh[t])
            feat = self.hst[t + 1]
        hp.heads_fwd(feat, self.logits[t], self.values[t], self.actions[t], self.seed, self.ctr, t,
                     self.T + 1, greedy=greedy, task=self.model.task, row_base=self.row_base)

    def _rollout_backward_hybrid(self):
        """LSTM nets: HIP trunk fwd/bwd, torch (autograd) LSTM + heads + loss in between."""
        from ..algo.a2c_math import a2c_loss, nstep_returns, sample_actions
        from ..models.pathnet import lstm_cell_ref
        T, P, E, B = self.T, self.P, self.E, self.B
        a2c = self.cfg.a2c
        model = self.model
        st = model.store
        k, bb = st.lstm()
        pw, pb, vw, vb = st.head(model.task)
        h, c = self.lstm_state
        feats, logits_l, values_l = [], [], []
        for t in range(T):
            self._trunk_step(t)
            f = self.acts[-1][t].float().detach().requires_grad_(True)
            feats.append(f)
            h, c = lstm_cell_ref(f, h, c, k, bb)
            logits = h @ pw + pb
            v = (h @ vw + vb).squeeze(-1)
            self.actions[t].copy_(sample_actions(logits.detach()).to(torch.int32))
            self.logits[t].copy_(logits.detach())
            self.values[t].copy_(v.detach())
            self._env_step(t)
            keep = (1.0 - self.dones[t].float())[:, None]
            h, c = h * keep, c * keep
            logits_l.append(logits)
            values_l.append(v)
        with torch.no_grad():
            self._trunk_step(T)
            h2, _ = lstm_cell_ref(self.acts[-1][T].float(), h, c, k, bb)
            vboot = (h2 @ vw + vb).squeeze(-1)
        R, adv = nstep_returns(self.rewards, self.values[:T], self.dones.bool(), vboot, a2c.gamma, a2c.gae_lambda,
                               a2c.reward_clip)
        wt = torch.full((T * B,), self.weight, device=self.device)
        loss, lp, lv, ent = a2c_loss(torch.cat(logits_l), torch.cat(values_l), self.actions[:T].reshape(-1).long(),
                                     R.reshape(-1), adv.reshape(-1), a2c.entropy_beta, a2c.value_coef, wt)
        st.flat.grad = None
        loss.backward()
        self.stats[0], self.stats[1], self.stats[2] = lp, lv, ent * T * B
        self.grads[-1].copy_(torch.cat([f.grad for f in feats]))
        self.grad_flat.zero_()
        self.hip.fx_begin()
        self._layer_bwd_all(T)
        self.hip.fx_end(self.grad_flat)
        tn = st.layout.trunk_numel
        self.grad_flat[tn:] += st.flat.grad[tn:]
        st.flat.grad = None
        self._fitness_update()
        if self.hip.x3:
            self.hip.fold_x3_status(self.counters[3:4])
        self.lstm_state = (h.detach(), c.detach())

    def _rollout_backward_body(self, part: Optional[str] = None):
        """part None: the whole rollout + backward; "head": all of it except the first layer's backward; "tail":
        the first layer's backward only (the overlapped all-reduce runs between them, parallel/comm.py)."""
        hp = self.hip
        if part == "tail":
            hp.fx_begin()
            self._layer_bwd_all(self.T, 0, 1)
            hp.fx_end(self.grad_flat, 0, self._l0_end)
            return
        if self.hybrid:
            return self._rollout_backward_hybrid()
        T, P, E, B = self.T, self.P, self.E, self.B
        a2c = self.cfg.a2c
        hp = self.hip
        if self.lstm_hip:
            hp.lstm_amax_reset()
        if self.groups > 1:
            self._rollout_split()
        else:
            fh = self.fuse_env_heads
            for t in range(T):
                self._forward_step(t, heads=not fh)
                self._env_step(t, heads=fh)
            self._forward_step(T, greedy=True)
        self._fitness_update()
        if hp.x3:
            # fp16-pair range flags of this rollout (+ the last weight refresh) -> the all-reduced counters slot 3
            hp.fold_x3_status(self.counters[3:4])
        self.stats.zero_()
        _lib.call("launch_a2c_grad", self.logits.data_ptr(), self.values.data_ptr(), self.actions.data_ptr(),
                  self.rewards.data_ptr(), self.dones.data_ptr(), self.values[T].data_ptr(), T, B, self.A,
                  a2c.gamma, a2c.gae_lambda, a2c.reward_clip, a2c.entropy_beta, a2c.value_coef, self.weight,
                  self.dlogits.data_ptr(), self.dvalue.data_ptr(), self.stats.data_ptr(), _lib.stream())
        self.grad_flat.zero_()
        L = len(hp.geoms)
        hp.fx_begin()            # deterministic fp32x: weight gradients in fixed point, added to grad_flat below
        if self.lstm_hip:
            self._lstm_backward()
        else:
            feat = self.acts[L - 1][:T].reshape(T * B, -1)
            hp.heads_bwd(feat, self.dlogits.reshape(T * B, -1), self.dvalue.reshape(-1), self.grad_flat,
                         self.grads[L - 1], task=self.model.task)
        self._layer_bwd_all(T, 1 if part == "head" else 0)
        hp.fx_end(self.grad_flat, self._l0_end if part == "head" else 0)

    def _rollout_split(self):
        """The rollout as independent per-path-group chains (forward -> sample -> env step, T times, then the
        bootstrap forward), group g on stream g, forked from and joined back into the current stream.  Under
        graph capture each chain is a branch of the rollout hipGraph.  Every kernel computes exactly what the
        single-stream rollout does for its rows (global RNG keys, same tiling per path), so the result is
        bit-identical; only the overlap changes."""
        T = self.T
        cur = torch.cuda.current_stream()
        streams = [cur] + self.side_streams
        for s in self.side_streams:
            s.wait_stream(cur)
        if self.ring:
            # the groups' module-major fc forwards read inverse lists of their own paths, cut from the population's
            # (which the last optimizer step's device GA, or the host GA, rewrote)
            for g, s in enumerate(streams):
                with torch.cuda.stream(s):
                    self.hip.group_inverse(*self._group_range(g))
        for t in range(T + 1):
            for g, s in enumerate(streams):
                with torch.cuda.stream(s):
                    self._forward_step(t, greedy=(t == T), grp=g)
                    if t < T:
                        self._env_step(t, grp=g)
        for s in self.side_streams:
            cur.wait_stream(s)

    def _fitness_update(self):
        _lib.call("launch_fitness_update", self.dones.data_ptr(), self.epret.data_ptr(), self.T, self.P, self.E,
                  self.fitness.data_ptr(), self.counters.data_ptr(), self.fit_cnt.data_ptr(), self.fit_sum.data_ptr(),
                  self.fit_window, self.path_part.data_ptr(), _lib.stream())

    def reset_fitness(self, fitness_local: torch.Tensor, fired: Optional[torch.Tensor] = None):
        """Install the GA's view of the local fitness; the candidates of tournaments that fired (``fired``,
        bool [P]) restart their episode window."""
        self.fitness.copy_(fitness_local)
        if fired is not None:
            self.fit_cnt.masked_fill_(fired, 0.0)
            self.fit_sum.masked_fill_(fired, 0.0)

    # -- device GA (GAConfig.backend == "device"; algo/ga_device.py mirrors it on the host) --------
    def enable_device_ga(self, pop, comm, p_off: int):
        dev = self.device
        self.ga_dev = dict(
            geno=torch.zeros(pop.P, pop.L, pop.M, dtype=torch.uint8, device=dev),
            frozen=torch.zeros(pop.L, pop.M, dtype=torch.uint8, device=dev),
            slots=torch.full((pop.concurrent, pop.B), -1, dtype=torch.int32, device=dev),
            gen=torch.zeros(1, dtype=torch.int64, device=dev),
            events=torch.zeros(pop.concurrent, 3, dtype=torch.int32, device=dev),
            reset=torch.zeros(pop.P, dtype=torch.uint8, device=dev),      # candidates of the tournaments just fired
            fit=comm.fit_reduced, p_off=p_off, pop=pop,
            # union of the modules the whole population expresses next, minus frozen ones (csrc/comm.hip):
            # read back after every optimizer step to plan the active-path gradient all-reduce
            union=torch.zeros(pop.L * pop.M, dtype=torch.uint8, device=dev),
            union_host=torch.zeros(pop.L * pop.M, dtype=torch.uint8, pin_memory=True))
        self._union_ev = None
        self.ga_upload(pop)

    def ga_upload(self, pop):
        """Host GA state -> device (task start, freeze, checkpoint load); static addresses kept."""
        g = self.ga_dev
        g["geno"].copy_(torch.from_numpy(pop.genotypes.astype(np.uint8)))
        g["frozen"].copy_(torch.from_numpy(pop.frozen.astype(np.uint8)))
        g["slots"].copy_(torch.from_numpy(pop.slots.astype(np.int32)))
        g["gen"].fill_(int(pop.generation))
        g["fit"].copy_(torch.from_numpy(pop.fitness.astype(np.float32)))
        self._union_ev = None          # the last read-back union described the old genotypes

    def _ga_body(self, sync_fitness: bool = True):
        g = self.ga_dev
        pop = g["pop"]
        hp = self.hip
        m = self.model
        st = _lib.stream()
        _lib.call("launch_ga_step", g["geno"].data_ptr(), g["fit"].data_ptr(), g["slots"].data_ptr(),
                  g["gen"].data_ptr(), g["events"].data_ptr(), pop.P, pop.L, pop.M, pop.N, pop.B, pop.concurrent,
                  pop.seed32, g["reset"].data_ptr(), st)
        _lib.call("launch_ga_compact", g["geno"].data_ptr(), g["frozen"].data_ptr(), g["p_off"], self.P, pop.L,
                  pop.M, m.mask.data_ptr(), m.act_idx.data_ptr(), m.act_cnt.data_ptr(), hp.inv_path.data_ptr(),
                  hp.inv_slot.data_ptr(), hp.inv_cnt.data_ptr(), st)
        _lib.call("launch_active_union", g["geno"].data_ptr(), g["frozen"].data_ptr(), pop.P, pop.L, pop.M,
                  g["union"].data_ptr(), st)
        # local fitness <- the GA's view; ONLY the candidates of tournaments that just fired restart their
        # episode window (paths still filling theirs keep accumulating).  sync_fitness False: the optimizer tail
        # does it (launch_opt_tail)
        if not sync_fitness:
            return
        self.fitness.copy_(g["fit"][g["p_off"]:g["p_off"] + self.P])
        if self.fit_window > 0:
            fired = g["reset"][g["p_off"]:g["p_off"] + self.P].bool()
            self.fit_cnt.masked_fill_(fired, 0.0)
            self.fit_sum.masked_fill_(fired, 0.0)

    def _read_union(self):
        """After an optimizer step: start the D2H of the device GA's next module union (outside any graph) -- only
        when the trainer's next exchange plan needs it (``want_union``: a multi-rank run on the exact plan)."""
        if self.ga_dev is None or not getattr(self, "want_union", False):
            self._union_ev = None
            return
        self.ga_dev["union_host"].copy_(self.ga_dev["union"], non_blocking=True)
        self._union_ev = torch.cuda.Event()
        self._union_ev.record()

    def active_union(self):
        """[L, M] bool union of the modules the population expresses in the rollout now running (minus frozen),
        as computed on device by the last optimizer step; None before the first one."""
        if self.ga_dev is None or self._union_ev is None:
            return None
        self._union_ev.synchronize()
        pop = self.ga_dev["pop"]
        return self.ga_dev["union_host"].numpy().reshape(pop.L, pop.M).astype(bool)

    def report_parts(self):
        """(stats [loss_pi, loss_v, entropy, 0], last optimizer step skipped) for the async read-back, the layout of
        report_tensor; the single-rank exchange packs them behind fitness and counters with one cat and one D2H."""
        return (self.stats, self.opt_status)

    def report_tensor(self) -> torch.Tensor:
        """Assemble [loss_pi, loss_v, entropy, 0, last optimizer step skipped] for the async read-back
        (enqueued after the rollout: the skip flag is the PREVIOUS optimizer step's)."""
        self.report[:4].copy_(self.stats)
        self.report[4:5].copy_(self.opt_status)
        return self.report

    def _lstm_backward(self):
        """Heads backward into dL/dh, reverse scan through the fused LSTM cell, then its weight gradient."""
        T, B = self.T, self.B
        hp = self.hip
        H = hp.lstm["H"]
        hp.heads_bwd(self.hst[1:T + 1].reshape(T * B, H), self.dlogits.reshape(T * B, -1), self.dvalue.reshape(-1),
                     self.grad_flat, self.dh_heads.reshape(T * B, H), task=self.model.task)
        dfeat = self.grads[-1].view(T, B, -1)
        for t in range(T - 1, -1, -1):
            cur, nxt = t % 2, (t + 1) % 2
            first = t == T - 1
            hp.lstm_bwd_step(self.dh_heads[t], None if first else self.dh_rec[nxt], None if first else self.dc_rec[nxt],
                             self.dones[t], self.gates[t], self.cst[t + 1], self.cst[t],
                             self.dones[t - 1] if t > 0 else None, self.dz[t], self.dc_rec[cur], dfeat[t],
                             self.dh_rec[cur], t=t)
        hp.lstm_wgrad(self.xh, self.dz, self.grad_flat)

    def lstm_state_tensors(self):
        """Recurrent state carried into the next update (checkpointing)."""
        if self.lstm_hip:
            return self.hst[0].float(), self.cst[0]
        return self.lstm_state

    def load_lstm_state(self, h, c):
        if self.lstm_hip:
            self.hst[0].copy_(h.to(self.hst.dtype))
            self.cst[0].copy_(c)
        elif self.hybrid:
            self.lstm_state = (h.clone(), c.clone())

    def _optimizer_body(self):
        if self.lstm_hip:
            T = self.T
            self.hip.lstm_carry(self.hst[T], self.cst[T], self.dones[T - 1], self.hst[0], self.cst[0])
        o = self.opt
        # non-finite (all-reduced) gradients: the kernel skips the step by itself, identically on every rank,
        # and records it in opt_status (runtime/guard.py counts consecutive skips on the host)
        _lib.call("launch_rmsprop", self.model.store.flat.data_ptr(), self.grad_flat.data_ptr(), o.ms.data_ptr(),
                  o.mom.data_ptr(), self.blk_seg.data_ptr(), self.blk_beg.data_ptr(), self.blk_end.data_ptr(),
                  self.nblk, self.partial.data_ptr(), self.seg_blk0.data_ptr(), self.trainable_u8.data_ptr(),
                  self.lr.data_ptr(), self.opt_status.data_ptr(), o.decay, o.momentum, o.epsilon, o.clip_norm,
                  _lib.stream())
        self.hip.refresh_weights()
        tail = self._tail
        if self.ga_dev is not None:
            self._ga_body(sync_fitness=not tail)
        if self.ring and not self.ring_mod:
            # through an int64 view: 8 bytes per element (the uint8 strided copy ran at ~3.4 TB/s, 92 us per update)
            f64 = self.frames.view(torch.int64) if self.HW % 8 == 0 else self.frames
            src = f64[:, self.T:self.T + 4]
            f64[:, 0:4].copy_(src if self.T >= 4 else src.clone())   # T < 4: the slot ranges overlap
        if tail:
            # the GA's local fitness view, fired windows reset, the ring's fc row carried and the counter advanced:
            # one launch (csrc/ga.hip opt_tail_kernel)
            g = self.ga_dev
            _lib.call("launch_opt_tail", g["fit"].data_ptr(), g["reset"].data_ptr(), g["p_off"], self.P,
                      self.fit_window, self.fitness.data_ptr(), self.fit_cnt.data_ptr(), self.fit_sum.data_ptr(),
                      self.fc[self.T].data_ptr() if self.ring else None, self.fc[0].data_ptr() if self.ring else None,
                      self.B if self.ring else 0, self.ctr.data_ptr(), self.lr_sched.data_ptr(), self.lr.data_ptr(),
                      _lib.stream())
            return
        if self.ring:
            self.fc[0].copy_(self.fc[self.T])
        self.ctr.add_(1)

    # ------------------------------------------------------------------
    def _capture(self):
        # warm up once on a side stream (torch requirement), then capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        par = self._par
        self.g_rollouts = []
        self.g_tails = []
        for q in ((0, 1) if self._parities else (par,)):                  # one rollout graph per parity
            self._par = q
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                self._rollout_backward_body("head" if self.split else None)
            self.g_rollouts.append(g)
            if self.split:
                gt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gt, capture_error_mode=CAPTURE_MODE):
                    self._rollout_backward_body("tail")
                self.g_tails.append(gt)
        self._par = par
        self.g_rollout = self.g_rollouts[0]
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, capture_error_mode=CAPTURE_MODE):
            self._optimizer_body()
        torch.cuda.synchronize()

    def rollout_backward(self, part: Optional[str] = None):
        """Replay (or run) the rollout + backward; with ``split``, part "head" then part "tail"."""
        if part is None and self.split:
            self.rollout_backward("head")
            self.rollout_backward("tail")
            return
        if self.use_graph:
            if self.g_rollout is None:
                # first update eagerly (validates every launch), capture for the next ones
                self._rollout_backward_body(part)
                self._pending_capture = True
                return
            gi = self._par if self._parities else 0
            (self.g_tails[gi] if part == "tail" else self.g_rollouts[gi]).replay()
        else:
            self._rollout_backward_body(part)

    @property
    def _tail(self) -> bool:
        return self.ga_dev is not None and os.environ.get("PATHNET_OPT_TAIL", "1") != "0"

    def optimizer_step(self, lr: float, skip: bool = False, sched_t: Optional[int] = None):
        """``skip``: host-decided skip (tests); non-finite gradients are skipped by the kernel itself.  ``sched_t``: the
        anneal clock (frames) ``lr`` was computed at; with the optimizer tail the device already holds that update's lr
        (it advanced its own clock by one update's frames), so nothing is written unless the clocks disagree (first
        update, checkpoint load, a caller without a clock)."""
        dev_lr = sched_t is not None and self._tail
        if not dev_lr or self._next_t != sched_t:
            self.lr[0:1].fill_(lr)
            if dev_lr:
                self.lr_sched[4:5].fill_(float(sched_t))
        if skip != self._skip_set:
            self.lr[1:2].fill_(1.0 if skip else 0.0)
            self._skip_set = skip
        self._next_t = sched_t + self.frames_per_update if dev_lr else None
        if self.use_graph and self.g_opt is not None:
            self.g_opt.replay()
        else:
            self._optimizer_body()
            if self.use_graph and getattr(self, "_pending_capture", False):
                self._pending_capture = False
                self._capture()
        if self._parities:
            self._par ^= 1          # the next rollout starts from the buffer / ring slots this one's last env step wrote
        self._read_union()

    def stats_host(self):
        return self.stats.cpu().numpy()
