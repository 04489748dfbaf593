"""Checkpoint / resume.

The reference's ``tf.train.Saver()`` (``doom_pathnet.py:157``) saves every
global variable: weights, RMSProp slots, genotype masks, flag, global_step,
scores and the frozen path.  It does NOT save the
coordinator's evolvable genotypes, tournament sample, RNG or env state, so a
resume is never exact (and never happens, because ``main`` appends a fresh
timestamp to log_dir, ``doom_pathnet.py:300``).

This checkpoint stores the same logical tensors under stable names PLUS the
state the reference loses, so resume is bit-exact on the same backend:

* ``layer{i}.module{j}.weight|bias``, ``policy.weight`` ..., ``lstm.kernel``
  (TF layouts: conv [kh,kw,cin,cout], fc [din,dout])
* ``<name>/RMSProp`` (ms, init 1.0) and ``<name>/RMSProp_1`` (momentum):
  TF slot naming
* ``ga.*``: genotype table [P,L,M] uint8, frozen mask, fitness, candidate
  sets, generation, MT19937 state
* ``train.*``: global_step, task index (``flag`` = task+1), update count
* per rank ``env.*`` / ``engine.*``: env state, frame stack, LSTM state,
  sampling counter (file ``<path>.rank<r>.safetensors``)

Format: safetensors (no pickle; loaders never execute file content).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import numpy as np
import torch
from safetensors.torch import load_file, save_file

# 1: rounds 1-3.  2: task ids name what they mean today (``Pong-v0`` = the real gym game, ``Pong`` / ``Synth*`` the
# on-device ones) and env / sampling RNG streams are keyed by the global env index (VecEnv.set_id_base)
FORMAT_VERSION = 2


def _t(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x)))


def state_tensors(trainer, light: bool = False) -> Dict[str, torch.Tensor]:
    """``light``: leave out the momentum slots when the momentum coefficient is 0.0 (the reference's setting: TF's
    ApplyRMSProp then only stores the last step in them and never reads them back)."""
    st = trainer.model.store
    out: Dict[str, torch.Tensor] = {}
    skip_mom = light and float(trainer.opt.momentum) == 0.0
    for s in st.layout.segments:
        out[s.name] = _t(st.flat[s.offset:s.offset + s.numel].view(s.shape))
        out[s.name + "/RMSProp"] = _t(trainer.opt.ms[s.offset:s.offset + s.numel].view(s.shape))
        if not skip_mom:
            out[s.name + "/RMSProp_1"] = _t(trainer.opt.mom[s.offset:s.offset + s.numel].view(s.shape))
    out["optim.seg_trainable"] = _t(trainer.opt.seg_trainable.to(torch.uint8))
    out["init_flat"] = _t(trainer.init_flat)
    for k, v in trainer.pop.state_dict().items():
        out["ga." + k] = _t(v)
    out["train.global_step"] = torch.tensor([trainer.global_step], dtype=torch.int64)
    out["train.task_idx"] = torch.tensor([trainer.task_idx], dtype=torch.int64)
    out["train.flag"] = torch.tensor([trainer.task_idx + 1], dtype=torch.int64)
    out["train.updates"] = torch.tensor([trainer.updates], dtype=torch.int64)
    out["train.task_start_step"] = torch.tensor([trainer.task_start_step], dtype=torch.int64)
    out["train.task_gen0"] = torch.tensor([trainer._task_gen0], dtype=torch.int64)
    # continual-learning bookkeeping: finished tasks whose per-task heads are frozen, the expressed path
    # each finished task was solved with, and generations-to-solve per task (-1 = not solved / not run)
    out["train.frozen_tasks"] = torch.tensor(sorted(trainer.frozen_tasks) or [-1], dtype=torch.int64)
    K = len(trainer.cfg.tasks)
    L, M = trainer.cfg.net.L, trainer.cfg.net.M
    paths = np.zeros((K, L, M), np.uint8)
    have = np.zeros(K, np.uint8)
    for t, p in trainer.task_paths.items():
        if 0 <= t < K:
            paths[t] = (np.asarray(p) > 0.5).astype(np.uint8)
            have[t] = 1
    out["train.task_paths"] = torch.from_numpy(paths)
    out["train.task_paths_valid"] = torch.from_numpy(have)
    solved = [-1 if trainer.solved_generation.get(t) is None else int(trainer.solved_generation[t]) for t in range(K)]
    out["train.solved_generation"] = torch.tensor(solved, dtype=torch.int64)
    return out


def _sync_env_from_device(env):
    """Kernel-side env state is authoritative: HIP Pong (csrc/envs.hip) or a HIP synthetic game (csrc/games.hip)."""
    if hasattr(env, "_st32") and hasattr(env, "_ctr32"):
        from ..ops import envs as henv
        henv.pong_sync_from_device(env)
    elif getattr(env, "_hip", False) and hasattr(env, "sync_from_device"):
        env.sync_from_device()


def rank_tensors(trainer, light: bool = False) -> Dict[str, torch.Tensor]:
    """``light``: leave out the frame stacks entering the next rollout (1.3 GB at 512 paths x 32 envs); a load then
    rebuilds every env's stack from its current frame, as at an episode start (resume no longer bit-exact)."""
    env = trainer.env
    out: Dict[str, torch.Tensor] = {}
    _sync_env_from_device(env)
    if hasattr(env, "_steps32"):
        env.steps = env._steps32.long()
        env.counter = env._ctr32.long() & 0xFFFFFFFF
    for name in ("state", "counter", "steps", "ep_ret") + (() if light else ("obs",)):
        if hasattr(env, name) and isinstance(getattr(env, name), torch.Tensor):
            out["env." + name] = _t(getattr(env, name))
    if getattr(env, "_hip", False) and hasattr(env, "_hip_pack"):
        out["env.game_state32"] = _t(env._st32)     # HIP synthetic game: the packed kernel state (csrc/games.hip)
    out["env.seed"] = torch.tensor([env.seed_int], dtype=torch.int64)
    if trainer.engine is not None:
        eng = trainer.engine
        out["engine.ctr"] = _t(eng.ctr)
        if not light:
            out["engine.obs0"] = _t(eng.obs_stack(0))
        out["engine.fitness"] = _t(eng.fitness)
        out["engine.fit_cnt"] = _t(eng.fit_cnt)
        out["engine.fit_sum"] = _t(eng.fit_sum)
    else:
        out["train.obs"] = _t(trainer.obs)
        out["train.fitness_local"] = _t(trainer.fitness_local)
        out["train.fit_cnt"] = _t(trainer.fit_cnt)
        out["train.fit_sum"] = _t(trainer.fit_sum)
    lstm = trainer.engine.lstm_state_tensors() if trainer.engine is not None else trainer.lstm_state
    if lstm is not None:
        out["lstm.h"] = _t(lstm[0])
        out["lstm.c"] = _t(lstm[1])
    return out


def save(trainer, path: str, light: bool = False) -> str:
    """Write ``path`` (rank-0 global state) and ``path.rank<r>.safetensors`` (every rank).  ``light``: a continuation
    checkpoint without the frame stacks and, at momentum 0, the momentum slots (state_tensors / rank_tensors)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    meta = {"format_version": str(FORMAT_VERSION), "config": trainer.cfg.to_json(), "light": str(int(light)),
            "world": str(trainer.ctx.world), "segments": json.dumps([s.name for s in trainer.model.store.layout.segments])}
    if trainer.ctx.is_main:
        save_file(state_tensors(trainer, light), path, metadata=meta)
    save_file(rank_tensors(trainer, light), f"{path}.rank{trainer.ctx.rank}.safetensors", metadata=meta)
    return path


def _restack_current_frame(trainer):
    """Light checkpoints: every env's stack entering the next rollout = its current frame x 4 (episode-start rule)."""
    env = trainer.env
    if not hasattr(env, "frame"):
        return
    _sync_env_from_device(env)
    f = env.frame()                                   # [N, H, W] uint8
    stack = f[..., None].expand(-1, -1, -1, 4).contiguous()
    env.obs = stack
    if trainer.engine is not None:
        trainer.engine.set_obs_stack0(stack.reshape(stack.shape[0], -1))
    else:
        trainer.obs = stack.clone()


def load(trainer, path: str, strict: bool = True):
    """Restore a trainer built with the same config (resume)."""
    d = load_file(path)
    st = trainer.model.store
    dev = st.flat.device
    with torch.no_grad():
        for s in st.layout.segments:
            if s.name not in d:
                if strict:
                    raise KeyError(f"checkpoint misses {s.name}")
                continue
            st.flat[s.offset:s.offset + s.numel].copy_(d[s.name].reshape(-1).to(dev))
            trainer.opt.ms[s.offset:s.offset + s.numel].copy_(d[s.name + "/RMSProp"].reshape(-1).to(dev))
            if s.name + "/RMSProp_1" in d:
                trainer.opt.mom[s.offset:s.offset + s.numel].copy_(d[s.name + "/RMSProp_1"].reshape(-1).to(dev))
            else:                                     # light checkpoint, momentum 0: the slots are never read
                trainer.opt.mom[s.offset:s.offset + s.numel].zero_()
        trainer.opt.seg_trainable.copy_(d["optim.seg_trainable"].bool().to(dev))
        trainer.init_flat.copy_(d["init_flat"].to(dev))
    ga = {k[3:]: v.numpy() for k, v in d.items() if k.startswith("ga.")}
    trainer.pop.load_state_dict(ga)
    task = int(d["train.task_idx"][0])
    if task != trainer.task_idx:
        trainer._start_task(task, fresh=True)
    trainer.global_step = int(d["train.global_step"][0])
    trainer.updates = int(d["train.updates"][0])
    trainer.task_start_step = int(d["train.task_start_step"][0])
    trainer._task_gen0 = int(d["train.task_gen0"][0])
    if "train.frozen_tasks" in d:
        trainer.frozen_tasks = set(int(x) for x in d["train.frozen_tasks"].tolist() if int(x) >= 0)
        valid = d["train.task_paths_valid"].numpy()
        paths = d["train.task_paths"].numpy().astype(np.float32)
        trainer.task_paths = {t: paths[t].copy() for t in range(len(valid)) if valid[t]}
        trainer.solved_generation = {t: (None if int(g) < 0 else int(g))
                                     for t, g in enumerate(d["train.solved_generation"].tolist())
                                     if t <= task or int(g) >= 0}
    frozen = trainer.pop.frozen
    trainer.model.set_frozen(frozen)
    trainer.opt.set_frozen(frozen, trainer.frozen_tasks)
    trainer._push_genotypes()
    rp = f"{path}.rank{trainer.ctx.rank}.safetensors"
    if os.path.exists(rp):
        r = load_file(rp)
        env = trainer.env
        for name in ("state", "counter", "steps", "ep_ret", "obs"):
            if "env." + name in r and hasattr(env, name):
                setattr(env, name, r["env." + name].to(getattr(env, name).device))
        if "env.game_state32" in r and getattr(env, "_hip", False):
            env._st32.copy_(r["env.game_state32"].to(env._st32.device))
            env.sync_from_device()
        elif hasattr(env, "_st32") and hasattr(env, "_ctr32"):
            from ..ops import envs as henv
            henv.pong_sync_to_device(env)
        if hasattr(env, "_steps32"):
            from ..ops import envs as henv
            henv.cartpole_sync_to_device(env)
        if trainer.engine is not None:
            eng = trainer.engine
            eng.ctr.copy_(r["engine.ctr"].to(dev))
            if "engine.obs0" in r:
                eng.set_obs_stack0(r["engine.obs0"].to(dev))
            eng.fitness.copy_(r["engine.fitness"].to(dev))
            if "engine.fit_cnt" in r:
                eng.fit_cnt.copy_(r["engine.fit_cnt"].to(dev))
                eng.fit_sum.copy_(r["engine.fit_sum"].to(dev))
            eng.refresh_trainable()
        elif "train.obs" in r:
            trainer.obs = r["train.obs"].to(dev)
            trainer.fitness_local = r["train.fitness_local"].to(dev)
            if "train.fit_cnt" in r:
                trainer.fit_cnt = r["train.fit_cnt"].to(dev)
                trainer.fit_sum = r["train.fit_sum"].to(dev)
        if "lstm.h" in r:
            if trainer.engine is not None:
                trainer.engine.load_lstm_state(r["lstm.h"].to(dev), r["lstm.c"].to(dev))
            else:
                trainer.lstm_state = (r["lstm.h"].to(dev), r["lstm.c"].to(dev))
    if os.path.exists(rp) and "engine.obs0" not in r and "train.obs" not in r:
        _restack_current_frame(trainer)
    if trainer.backend == "hip":
        trainer.model.hip.refresh_weights()
        if trainer.engine is not None and trainer.engine.ga_dev is not None:
            trainer.engine.ga_upload(trainer.pop)
    return trainer


def read_metadata(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        return dict(f.metadata() or {})


def read_config(path: str):
    """The TrainConfig stored in a checkpoint.  In format-1 checkpoints (written before the rename) the ids of the
    synthetic games (``Pong-v0`` ...: those ids now mean the real gym games, envs/registry.py) are mapped to their
    ``Synth*`` equivalents with a warning; newer checkpoints keep their ids as written."""
    import warnings
    from ..config import TrainConfig
    from ..envs.registry import legacy_synth_id
    meta = read_metadata(path)
    cfg = TrainConfig.from_json(meta["config"])
    if int(meta.get("format_version", "1")) >= 2:
        return cfg
    new = [legacy_synth_id(t) or t for t in cfg.tasks]
    if new != list(cfg.tasks):
        warnings.warn(f"checkpoint tasks {cfg.tasks} use round-1 synthetic ids; mapped to {new}")
        cfg.tasks = new
        cfg.env = legacy_synth_id(cfg.env) or cfg.env
    return cfg


# ---------------------------------------------------------------------------
# TF1 creation-order importer
# ---------------------------------------------------------------------------
def tf_creation_order(cfg) -> List[str]:
    """Names of the reference's trainable tensors in tf.Variable creation order.

    conv W/b per (layer, module) i-major j-minor, then lin W/b per module,
    fc2 (policy), fc3 (value), then the LSTM kernel/bias
    (game_ac_network.py:328-347,397; LSTM variables are created last).
    """
    from ..models.pathnet import ParamLayout
    lay = ParamLayout(cfg)
    names = []
    for l in range(cfg.L):
        for j in range(cfg.M):
            names += [f"layer{l}.module{j}.weight", f"layer{l}.module{j}.bias"]
    names += ["policy.weight", "policy.bias", "value.weight", "value.bias"]
    if cfg.use_lstm:
        names += ["lstm.kernel", "lstm.bias"]
    assert set(names) <= set(lay.by_name)
    return names


def import_tf_arrays(store, arrays: List[np.ndarray]):
    """Load reference weights given as numpy arrays in TF creation order."""
    names = tf_creation_order(store.cfg)
    if len(arrays) != len(names):
        raise ValueError(f"expected {len(names)} arrays, got {len(arrays)}")
    with torch.no_grad():
        for n, a in zip(names, arrays):
            s = store.layout.by_name[n]
            a = np.asarray(a, np.float32)
            if a.size != s.numel:
                raise ValueError(f"{n}: size {a.size} != {s.numel}")
            store.flat[s.offset:s.offset + s.numel].copy_(torch.from_numpy(a.reshape(-1)))
