"""Population-parallel PathNet A2C trainer (one process per GPU).

Replaces the reference's worker/coordinator/PS process roles
(``doom_pathnet.py:53-296``, ``a3c_training_thread.py:102-245``) with ONE
synchronous loop per rank:

    update():
      rollout T steps of P_local paths x E envs      (env + policy on device)
      backward through the stored rollout graph      (no recompute)
      ONE fused all-reduce: active grads + fitness + counters   (parallel/comm.py)
      clip-by-norm per tensor + TF RMSProp            (algo/optim.py)
      replicated B-way tournament on the global fitness vector  (algo/ga.py)

Semantic differences from the reference (all
deliberate and documented): synchronous instead of Hogwild; fixed-length
rollouts with done masks instead of cutting at episode end; genotypes only
change at update boundaries; per-task lr anneal by default; frozen mask is
the union over tasks by default.
"""
from __future__ import annotations

import gc
import math
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import FITNESS_PENDING, PERFORMANCE_LOG_INTERVAL, TrainConfig
from ..envs.registry import is_synthetic, make, reward_threshold
from ..models.acnet import ACPathNet
from ..parallel.comm import FusedUpdateComm, GatherBroadcastComm, active_union
from ..parallel.dist import DistContext
from ..runtime.consistency import check_replicas
from ..runtime.guard import NonFiniteGuard, Watchdog
from ..utils.metrics import MetricsLogger
from ..utils.tracing import PhaseTracer, performance_line
from .a2c_math import a2c_loss, nstep_returns, sample_actions_keyed
from .ga import Population
from .optim import RMSPropTF, anneal_lr


def resolve_backend(backend: str, device: torch.device) -> str:
    if backend == "auto":
        return "hip" if device.type == "cuda" else "torch"
    if backend == "hip" and device.type != "cuda":
        raise RuntimeError("backend 'hip' needs a GPU device")
    return backend


@dataclass
class UpdateStats:
    loss_pi: float = 0.0
    loss_v: float = 0.0
    entropy: float = 0.0
    episodes: int = 0
    mean_return: float = float("nan")
    tournaments: int = 0
    best_winner: float = float("nan")
    winner_path: int = -1               # global index of the path that won with best_winner (-1: no tournament)
    steps: int = 0
    skipped: bool = False
    # the update (1-based count) whose optimizer step ``skipped`` refers to: this one when not pipelined; with the
    # pipeline the status arrives one update late, so it names the previous update (flush() reports the last)
    skipped_update: int = -1


class PathNetTrainer:
    def __init__(self, cfg: TrainConfig, device=None, ctx: Optional[DistContext] = None,
                 logger: Optional[MetricsLogger] = None):
        self.cfg = cfg
        self.ctx = ctx or DistContext()
        if device is None:
            device = self.ctx.device
        self.device = torch.device(device)
        self.backend = resolve_backend(cfg.backend, self.device)
        # the torch backend always computes in fp32; the HIP engine uses bf16 (fp16 for the uint8 conv1
        # operands) MFMA with fp32 accumulation and fp32 master weights, or fp32 operands (compute_dtype="fp32")
        if cfg.compute_dtype not in ("bf16", "fp32", "fp32x"):
            raise ValueError(f"compute_dtype {cfg.compute_dtype!r}: expected 'bf16', 'fp32' or 'fp32x'")
        self.compute_dtype = cfg.compute_dtype if self.backend == "hip" else "fp32"
        self.precision_note = None
        if self.compute_dtype == "fp32x":
            from ..ops.pathnet_ops import x3_unsupported_reason
            why = x3_unsupported_reason(cfg.net)
            if why is not None:
                # no split-operand kernels for this geometry: the fp32 engine keeps (and exceeds) fp32x's accuracy
                import warnings
                self.precision_note = f"fp32x -> fp32: {why}"
                warnings.warn(f"compute_dtype fp32x: {why}; running the fp32 engine (csrc/trunk_f32.hip) instead")
                self.compute_dtype = "fp32"
        self.logger = logger
        net = cfg.net
        if cfg.paths_total:
            # strong scaling: a fixed population split over the ranks (cfg.paths is resolved to the local count)
            if cfg.paths_total % self.ctx.world:
                raise ValueError(f"paths_total={cfg.paths_total} is not divisible by the world size {self.ctx.world}")
            cfg.paths = cfg.paths_total // self.ctx.world
        self.P = cfg.paths
        self.E = cfg.envs_per_path
        self.P_total = self.P * self.ctx.world
        self.path_offset = self.ctx.rank * self.P
        # global index of this rank's first env: every env's RNG (dynamics, resets, action sampling) is keyed by its
        # global index and the seeds carry no rank term, so rank r computes exactly envs [env_base, env_base + P*E)
        # of the one-GPU run of the same population (strong scaling reproduces one GPU; weak scaling = the first
        # world * P paths of a bigger population)
        self.env_base = self.path_offset * self.E
        self.device_ga = cfg.ga.backend == "device"
        pop_cls = Population
        if self.device_ga:
            from .ga_device import CounterPopulation
            pop_cls = CounterPopulation      # host mirror of the device GA (identical decisions)
        self.pop = pop_cls(self.P_total, net.L, net.M, net.N, cfg.ga.B, seed=cfg.ga.seed,
                           mutation_kind=cfg.ga.mutation, concurrent=cfg.ga.concurrent_tournaments)
        self.model = ACPathNet(net, self.P, self.device, self.backend, seed=cfg.seed,
                               compute_dtype=self.compute_dtype, deterministic=cfg.deterministic)
        a2c = cfg.a2c
        self.opt = RMSPropTF(self.model.store.layout, self.model.store.flat, a2c.rmsp_alpha, a2c.rmsp_momentum,
                             a2c.rmsp_epsilon, a2c.grad_norm_clip,
                             backend="hip" if self.backend == "hip" else "torch")
        # vars_backup: initial weights used for re-initialisation between tasks (doom_pathnet.py:204-205)
        self.init_flat = self.model.store.flat.detach().clone()
        comm_cls = GatherBroadcastComm if getattr(cfg, "ga_sync", "fused") == "gather_bcast" else FusedUpdateComm
        self.comm = comm_cls(self.ctx, self.model.store.layout, self.P_total, self.P, self.device)
        self.global_step = 0
        self.task_start_step = 0
        self.task_idx = 0
        self.updates = 0
        self.solved_generation: Dict[int, Optional[int]] = {}
        self.task_paths: Dict[int, np.ndarray] = {}
        self.frozen_tasks = set()
        self.env = None
        self.visualizer = None
        self.monitor = None          # envs.monitor.UpdateMonitor (--monitor_dir)
        self._last_vis = 0.0
        self.tracer = PhaseTracer(enabled=True, path=cfg.trace_path, rank=self.ctx.rank)
        self.guard = NonFiniteGuard(cfg.max_nonfinite)
        self.watchdog = Watchdog(cfg.watchdog_s, phase=lambda: self.tracer.current) if cfg.watchdog_s > 0 else None
        self._start_task(0, fresh=True)
        if getattr(cfg, "gc_freeze", True):
            # move everything built so far (torch / numpy / the engine's ~10^5 Python objects) out of the cyclic
            # collector's reach: a full collection every ~70 K allocations otherwise walks all of it, a host pause of
            # tens of ms that the pipelined loop (one update of GPU work queued) cannot hide -- measured as 64-path bench
            # windows drifting 10.4 -> 12.0 ms after ~65 updates (profiles/r6/README.md)
            gc.collect()
            gc.freeze()

    # ------------------------------------------------------------------
    # task sequencing (doom_pathnet.py:178-293)
    # ------------------------------------------------------------------
    def _make_env(self, task_idx: int):
        name = self.cfg.tasks[task_idx]
        seed = self.cfg.seed * 7919 + task_idx * 113
        kw = dict(gray=self.cfg.gray)
        if is_synthetic(name):
            kw["frameskip"] = self.cfg.frameskip
        env_backend = "hip" if self.backend == "hip" else "torch"
        env = make(name, num_envs=self.P * self.E, device=self.device, seed=seed, backend=env_backend, **kw)
        env.set_id_base(self.env_base)
        return env

    def _start_task(self, task_idx: int, fresh: bool = False):
        self.task_idx = task_idx
        self.model.task = task_idx
        if not fresh:
            self.pop.init_genotypes()
        if self.env is not None:
            self.env.close()
        self.env = self._make_env(task_idx)
        self.obs = self.env.reset()
        B = self.P * self.E
        self.lstm_state = self.model.init_state(B)
        self._push_genotypes()
        self.engine = None
        if self.backend == "hip":
            from ..runtime.engine import HipEngine
            self.engine = HipEngine(self.model, self.env, self.cfg, self.opt, seed=self._sample_seed(task_idx),
                                    row_base=self.env_base)
            self.fitness_local = self.engine.fitness
            if self.device_ga:
                self.engine.enable_device_ga(self.pop, self.comm, self.path_offset)
            self._enable_overlap()
        else:
            self.fitness_local = torch.full((self.P,), FITNESS_PENDING, device=self.device)
            self.fit_cnt = torch.zeros(self.P, device=self.device)
            self.fit_sum = torch.zeros(self.P, device=self.device)
        self.task_start_step = self.global_step
        self.solved_generation.setdefault(task_idx, None)
        self._task_gen0 = self.pop.generation

    def _sample_seed(self, task_idx: int) -> int:
        """Key of the action-sampling RNG (identical on every rank; rows are told apart by their global index)."""
        return (self.cfg.seed * 1000003 + task_idx) & 0xFFFFFFFF

    def _enable_overlap(self):
        """TrainConfig.overlap_allreduce: split the HIP update at the first layer so the all-reduce of everything
        else runs during the first layer's weight gradient (parallel/comm.py exchange_async_split)."""
        eng = self.engine
        if not (getattr(self.cfg, "overlap_allreduce", True) and self.ctx.enabled and self.pipelined
                and isinstance(self.comm, FusedUpdateComm) and type(self.comm) is FusedUpdateComm
                and not eng.hybrid and self.device.type == "cuda"):
            return
        segs = self.model.store.layout.segments
        split_off = max(s.offset + s.numel for s in segs if s.layer == 0)
        if any(s.offset < split_off for s in segs if s.layer != 0):
            return                               # layout does not put the first layer first: keep one bucket
        if self.comm.split_off is None:
            self.comm.enable_overlap(split_off)
        eng.split = True

    def _push_genotypes(self):
        expr = self.pop.expressed()
        self.model.set_paths(expr[self.path_offset:self.path_offset + self.P])
        self.comm.plan(expr, self.pop.frozen)

    def end_task(self):
        """Freeze the last winner and re-init every other parameter (doom_pathnet.py:274-293)."""
        self.flush()
        winner = self.pop.best()
        # the path that solved this task, as expressed (its genotype OR the earlier frozen modules)
        self.task_paths[self.task_idx] = self.pop.expressed()[winner].copy()
        frozen = self.pop.freeze(winner, union=self.cfg.ga.freeze_union)
        if self.cfg.net.per_task_heads:
            self.frozen_tasks.add(self.task_idx)          # keep this task's own head with its path
        self.model.set_frozen(frozen)
        self.opt.set_frozen(frozen, self.frozen_tasks)
        keep = np.zeros(self.model.store.layout.numel, bool)
        for s in self.model.store.layout.segments:
            if (s.layer >= 0 and frozen[s.layer, s.module] > 0.5) or (s.task >= 0 and s.task in self.frozen_tasks):
                keep[s.offset:s.offset + s.numel] = True
        keep_t = torch.from_numpy(keep).to(self.device)
        with torch.no_grad():
            f = self.model.store.flat
            f.copy_(torch.where(keep_t, f, self.init_flat))
        if self.backend == "hip":
            self.model.hip.refresh_weights()
            self.engine.refresh_trainable()
            if self.engine.ga_dev is not None:
                self.engine.ga_upload(self.pop)
        return winner, frozen

    # ------------------------------------------------------------------
    # one update
    # ------------------------------------------------------------------
    def rollout_and_backward(self):
        """T env steps for the whole local population + loss.backward()."""
        cfg = self.cfg
        a2c = cfg.a2c
        T, E, P = a2c.t_max, self.E, self.P
        B = P * E
        model, env = self.model, self.env
        logits_l, values_l, actions_l, rewards_l, dones_l = [], [], [], [], []
        state = self.lstm_state
        obs = self.obs
        ep_sum = torch.zeros(P, device=self.device)
        ep_cnt = torch.zeros(P, device=self.device)
        for t in range(T):
            logits, value, state = model.forward(obs, E, state)
            # the HIP heads kernel's keyed Gumbel-max: sample b of this rank = global row env_base + b
            a = sample_actions_keyed(logits, self._sample_seed(self.task_idx), self.updates * (T + 1) + t,
                                     self.env_base)
            obs, r, d, info = env.step(a)
            finished = d.float()
            er = info["episode_return"].float()
            s = (er * finished).view(P, E).sum(1)
            c = finished.view(P, E).sum(1)
            # fitness = return of the most recently finished episode(s) (a3c_training_thread.py:145-147)
            self.fitness_local = torch.where(c > 0, s / c.clamp(min=1.0), self.fitness_local)
            ep_sum += s
            ep_cnt += c
            if state is not None:
                keep = (1.0 - finished)[:, None]
                state = (state[0] * keep, state[1] * keep)
            logits_l.append(logits)
            values_l.append(value)
            actions_l.append(a)
            rewards_l.append(r)
            dones_l.append(d)
        window = cfg.ga.window_for(E)
        if window > 0:   # mean return over the episodes finished since the path's last tournament
            self.fit_cnt += ep_cnt
            self.fit_sum += ep_sum
            self.fitness_local = torch.where(self.fit_cnt >= window, self.fit_sum / self.fit_cnt.clamp(min=1.0),
                                             torch.full_like(self.fit_sum, FITNESS_PENDING))
        with torch.no_grad():
            _, v_boot, _ = model.forward(obs, E, state)
        values = torch.stack(values_l)
        R, adv = nstep_returns(torch.stack(rewards_l), values.detach().float(), torch.stack(dones_l),
                               v_boot.float(), a2c.gamma, a2c.gae_lambda, a2c.reward_clip)
        from ..runtime.engine import loss_scale
        weight = None
        ls = loss_scale(cfg)
        if a2c.env_reduction == "mean_env" or ls != 1.0:
            weight = torch.full((T * B,), (1.0 / E if a2c.env_reduction == "mean_env" else 1.0) * ls,
                                device=self.device)
        loss, lp, lv, ent = a2c_loss(torch.cat(logits_l), values.reshape(-1), torch.cat(actions_l),
                                     R.reshape(-1), adv.reshape(-1), a2c.entropy_beta, a2c.value_coef, weight)
        flat = model.store.flat
        flat.grad = None
        loss.backward()
        self.obs = obs
        if state is not None:
            state = (state[0].detach(), state[1].detach())
        self.lstm_state = state
        nonfinite = (~torch.isfinite(flat.grad)).sum(dtype=torch.float32)
        counters = torch.stack([torch.tensor(float(T * B), device=self.device), ep_cnt.sum(), ep_sum.sum(),
                                nonfinite])
        return flat.grad, counters, (lp, lv, ent)

    @property
    def pipelined(self) -> bool:
        """HIP engine + device GA: host bookkeeping of update u-1 overlaps the GPU work of update u."""
        return bool(self.cfg.pipeline and self.engine is not None and self.engine.ga_dev is not None)

    def update(self) -> UpdateStats:
        lr = anneal_lr(self.cfg.a2c.lr, self.global_step, self.cfg.a2c.max_time_step,
                       self.task_start_step, self.cfg.a2c.lr_anneal)
        self.last_lr = lr                # the learning rate of the optimizer step this update enqueues
        tr = self.tracer
        if self.pipelined:
            return self._update_pipelined(lr)
        if self.engine is not None:
            eng = self.engine
            with tr.phase("rollout_backward"):
                eng.rollout_backward()
            with tr.phase("allreduce"):
                fit_all, csum = self.comm.exchange(eng.grad_flat, eng.fitness, eng.counters)
            with tr.phase("optimizer"):
                eng.optimizer_step(lr)       # skips itself on a non-finite reduced gradient (same on every rank)
            skip = self.guard.check(float(eng.opt_status.item()), self.updates)
            lp, lv, ent = [float(x) for x in eng.stats_host()[:3]]
            ent /= max(1, self.cfg.a2c.t_max * self.P * self.E)
        else:
            with tr.phase("rollout_backward"):
                grad, counters, (lp, lv, ent) = self.rollout_and_backward()
            with tr.phase("allreduce"):
                fit_all, csum = self.comm.exchange(grad, self.fitness_local, counters)
            skip = self.guard.check(float(csum[3]), self.updates)
            if not skip:
                with tr.phase("optimizer"), torch.no_grad():
                    self.opt.step(grad, lr)
        self.global_step += int(csum[0])
        self.updates += 1
        st = self._finish_update(fit_all, csum, (lp, lv, ent), skip, self.global_step)
        st.skipped_update = self.updates if skip else -1
        return st

    def _update_pipelined(self, lr) -> UpdateStats:
        """Enqueue update u (rollout graph, fused reduce, optimizer+GA graph, async D2H), then finish u-1."""
        tr = self.tracer
        eng = self.engine
        with tr.phase("rollout_backward"):
            eng.rollout_backward("head" if eng.split else None)
        with tr.phase("allreduce"):
            if self.ctx.enabled:
                self._plan_exchange(eng)
            if eng.split:
                # bucket 1 (layers >= 1, heads, fitness, counters) is reduced while the first layer's weight
                # gradient runs; bucket 2 (the first layer) after it
                handle = self.comm.exchange_async_split(eng.grad_flat, eng.fitness, eng.counters,
                                                        run_tail=lambda: eng.rollout_backward("tail"),
                                                        extra=eng.report_parts())
            else:
                handle = self.comm.exchange_async(eng.grad_flat, eng.fitness, eng.counters,
                                                  extra=eng.report_parts())
        with tr.phase("optimizer"):
            # non-finite reduced gradient: skipped on device, on every rank; the lr anneal runs on device too (the
            # optimizer tail), the host clock only checks it
            a2c = self.cfg.a2c
            clock = self.global_step - (self.task_start_step if a2c.lr_anneal == "per_task" else 0)
            eng.optimizer_step(lr, sched_t=clock)
        self.global_step += self.cfg.a2c.t_max * self.P * self.E * self.ctx.world
        self.updates += 1
        prev, self._pending = getattr(self, "_pending", None), (handle, self.global_step, self.updates)
        if prev is None:
            return UpdateStats(float("nan"), float("nan"), float("nan"), 0, float("nan"),
                               steps=self.cfg.a2c.t_max * self.P * self.E * self.ctx.world)
        return self._collect(prev)

    # the host mirror's module union covers at least this share of the trainable (non-frozen) modules: all-reduce
    # every trainable module (static plan, no per-update read-back); below it, the exact device union
    static_plan_min_density = 0.9

    def _plan_exchange(self, eng):
        """Plan the gradient all-reduce of the update just enqueued, identically on every rank.

        * Static plan (steady state of a large population): every non-frozen module + heads/LSTM -- the reference's
          own apply set (get_vars_idx, a3c_training_thread.py:190-216; a module no path uses carries a zero
          gradient).  Its ranges change only with the frozen mask, so the update needs no device read-back and no
          Python replanning (``plan_union`` returns on an unchanged key).
        * Exact plan: when the population's union is sparse, only the modules the running rollout expresses, read
          back from the device GA of the previous optimizer step (one small D2H + event wait per update).
        The choice uses the host GA mirror (identical on every rank, one update behind), never a timing-dependent
        read, so ranks always issue the same collective sizes; both plans contain every module the rollout uses."""
        pop = self.pop
        trainable = ~(np.asarray(pop.frozen) > 0.5)
        n_tr = int(trainable.sum())
        mirror = active_union(pop.expressed(), pop.frozen)
        if n_tr == 0 or mirror.sum() >= self.static_plan_min_density * n_tr:
            self.comm.plan_union(trainable)
            self.plan_mode = "static"
            eng.want_union = False
            return
        # exact plan: the union of the previous optimizer step's device GA; read back only while the exact plan is
        # in use, so the first update after a switch takes the static superset instead
        eng.want_union = True
        union = eng.active_union()
        self.comm.plan_union(union if union is not None else trainable)
        self.plan_mode = "exact" if union is not None else "static"

    def _guard_opt(self, flag: float, update: int) -> bool:
        """Feed the device optimizer status of ``update`` to the guard once (pipelined: it arrives late)."""
        if update <= getattr(self, "_opt_checked", 0):
            return False
        self._opt_checked = update
        return self.guard.check(flag, update)

    def _collect(self, pending) -> UpdateStats:
        handle, step_at, u = pending
        with self.tracer.phase("collect"):           # waits for update u's read-back (GPU-bound when it dominates)
            fit_all, csum, stats = self.comm.collect(handle)
        # stats[4]: whether the optimizer step of update u-1 skipped a non-finite gradient (read before the
        # optimizer of update u ran: one-update lag)
        skip = self._guard_opt(float(stats[4]), u - 1) if u > 1 else False
        ent = float(stats[2]) / max(1, self.cfg.a2c.t_max * self.P * self.E)
        st = self._finish_update(fit_all, csum, (float(stats[0]), float(stats[1]), ent), skip, step_at)
        st.skipped_update = u - 1 if skip else -1
        return st

    def flush(self) -> Optional[UpdateStats]:
        """Drain the pipelined update still in flight (task end, checkpoint, end of run); the status of its
        optimizer step (the last one) is read here, so it reaches the guard too."""
        pending = getattr(self, "_pending", None)
        self._pending = None
        self._check_x3_refresh()
        if pending is None:
            return None
        st = self._collect(pending)
        u = pending[2]
        if self.engine is not None and getattr(self.engine, "opt_status", None) is not None:
            if self._guard_opt(float(self.engine.opt_status), u):
                st.skipped, st.skipped_update = True, u
        return st

    def _check_x3_refresh(self):
        """fp32x: fold the range flags raised since the last rollout (the weight refresh of the last optimizer
        step) and raise X3RangeError now -- all-reduced, so every rank raises together -- instead of one update
        late (flush runs at task end and before every checkpoint: no checkpoint holds out-of-range weights)."""
        if self.engine is None or not self.model.hip.x3:
            return
        out = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.model.hip.fold_x3_status(out)
        self.ctx.all_reduce_(out)
        v = float(out.item())
        if v != 0.0:
            from ..runtime.guard import X3RangeError
            raise X3RangeError(v, self.updates, self.ctx.world)

    def _finish_update(self, fit_all, csum, losses, skip, step_at) -> UpdateStats:
        tr = self.tracer
        lp, lv, ent = losses
        if self.engine is not None and self.model.hip.x3 and float(csum[3]) != 0.0:
            # fp32x fp16-pair range flags, all-reduced: every rank raises at the same update
            from ..runtime.guard import X3RangeError
            raise X3RangeError(float(csum[3]), self.updates, self.ctx.world)
        eps = float(csum[1]) if np.isfinite(csum[1]) else 0.0
        st = UpdateStats(float(lp), float(lv), float(ent), int(round(eps)),
                         float(csum[2] / csum[1]) if eps >= 0.5 else float("nan"), steps=int(csum[0]),
                         skipped=skip)
        with tr.phase("ga"):
            events = self.pop.step(fit_all, step_at)
        if isinstance(self.comm, GatherBroadcastComm) and events:
            g = self.comm.broadcast_genotypes(self.pop.genotypes)
            self.pop.genotypes = g
        if events:
            st.tournaments = len(events)
            best_ev = max(events, key=lambda e: e.winner_fitness)
            st.best_winner = best_ev.winner_fitness
            st.winner_path = int(best_ev.winner)
            thr = reward_threshold(self.cfg.tasks[self.task_idx])
            if self.solved_generation.get(self.task_idx) is None and st.best_winner >= thr:
                self.solved_generation[self.task_idx] = self.pop.generation - self._task_gen0
            lo, hi = self.path_offset, self.path_offset + self.P
            if self.engine is not None and self.engine.ga_dev is not None:
                # the device GA already mutated, compacted and reset inside the optimizer graph; without the
                # pipeline the host mirror is current and refreshes the (multi-rank) packing plan, with it the
                # plan comes from the device union instead (this mirror lags one update)
                if not self.pipelined:
                    self.comm.plan(self.pop.expressed(), self.pop.frozen)
            else:
                self._push_genotypes()
            if self.engine is None or self.engine.ga_dev is None:
                fl = torch.from_numpy(self.pop.fitness[lo:hi]).to(self.device)
                # only the candidates of the tournaments that fired restart their episode window
                fired_np = np.zeros(self.P, bool)
                for e in events:
                    for i in e.candidates:
                        if lo <= i < hi:
                            fired_np[i - lo] = True
                fired = torch.from_numpy(fired_np).to(self.device)
                if self.engine is not None:
                    self.engine.reset_fitness(fl, fired)
                else:
                    self.fitness_local.copy_(fl)
                    self.fit_cnt.masked_fill_(fired, 0.0)
                    self.fit_sum.masked_fill_(fired, 0.0)
            if self.visualizer is not None and time.time() - self._last_vis > 10.0:
                from .ga import decode_path
                self.visualizer.show([decode_path(g) for g in self.pop.genotypes], "m")   # visualize.py:90
                self._last_vis = time.time()
            if self.logger is not None and self.ctx.is_main:
                for e in events:
                    # "<step> Step Score: <s>" (doom_pathnet.py:256)
                    self.logger.log("tournament", step=e.step, generation=e.generation, winner=e.winner,
                                    score=e.winner_fitness, candidates=e.candidates, scores=e.scores)
        if self.watchdog is not None:
            self.watchdog.beat()
        if self.cfg.check_every and self.updates % self.cfg.check_every == 0:
            with tr.phase("consistency"):
                check_replicas(self)
        return st

    # ------------------------------------------------------------------
    def train(self, steps_per_task: Optional[int] = None, max_updates: Optional[int] = None,
              checkpoint: Optional[str] = None, checkpoint_every: int = 0):
        """Run the task sequence (doom_pathnet.py:178-293 generalised to K tasks)."""
        steps_per_task = steps_per_task or self.cfg.steps_per_task
        t0 = time.time()
        perf_step, perf_t = self.global_step, t0
        first = self.task_idx
        for task_idx in range(first, len(self.cfg.tasks)):
            if task_idx != self.task_idx:
                self._start_task(task_idx)
            n = 0
            while self.global_step - self.task_start_step < steps_per_task:
                st = self.update()
                n += 1
                if checkpoint and checkpoint_every and self.updates % checkpoint_every == 0:
                    from ..utils import checkpoint as ckpt
                    self.flush()
                    ckpt.save(self, checkpoint)
                # reference throughput line: every PERFORMANCE_LOG_INTERVAL steps (rate-limited to 10 s)
                if self.ctx.is_main and self.logger is not None and self.logger.echo and \
                        self.global_step - perf_step >= PERFORMANCE_LOG_INTERVAL and time.time() - perf_t >= 10.0:
                    perf_step, perf_t = self.global_step, time.time()
                    print(performance_line(self.global_step, perf_t - t0), flush=True)
                if self.logger is not None and self.ctx.is_main and self.updates % 10 == 0:
                    el = time.time() - t0
                    self.logger.log("perf", step=self.global_step, steps_per_sec=self.global_step / max(el, 1e-9),
                                    loss_pi=st.loss_pi, loss_v=st.loss_v, entropy=st.entropy,
                                    mean_return=st.mean_return, generation=self.pop.generation)
                if self.monitor is not None:
                    self.monitor.record(task_idx, self.updates, self.global_step, st.episodes, st.mean_return,
                                        self.pop.generation)
                if max_updates is not None and n >= max_updates:
                    break
            winner, frozen = self.end_task()
            if self.visualizer is not None:
                from .ga import decode_path
                self.visualizer.set_fixed(decode_path(frozen), "r" if task_idx == 0 else "g")   # :276
            if checkpoint:
                from ..utils import checkpoint as ckpt
                ckpt.save(self, checkpoint)
            if self.logger is not None and self.ctx.is_main:
                self.logger.log("freeze", task=task_idx, winner=winner, frozen=frozen.astype(int).tolist(),
                                solved_generation=self.solved_generation.get(task_idx))
        if self.cfg.trace_path:
            self.tracer.dump()
        return self.solved_generation
