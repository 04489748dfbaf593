"""Trainer: learning, task sequencing/freeze/re-init, checkpoint resume (CPU, torch backend)."""
import numpy as np
import torch

from pathnet_gym_amd.algo.trainer import PathNetTrainer
from pathnet_gym_amd.config import preset
from pathnet_gym_amd.utils import checkpoint as ckpt


def small_cfg(**kw):
    cfg = preset("cartpole-cpu")
    cfg.paths, cfg.envs_per_path = 4, 4
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def test_cartpole_learns_on_cpu():
    torch.manual_seed(0)
    cfg = small_cfg()
    cfg.paths, cfg.envs_per_path = 8, 8
    tr = PathNetTrainer(cfg)
    rets = []
    for i in range(250):
        st = tr.update()
        if not np.isnan(st.mean_return):
            rets.append(st.mean_return)
    assert np.mean(rets[-20:]) > np.mean(rets[:20]) + 10
    assert tr.pop.generation > 10


def test_end_task_freezes_and_reinitialises():
    cfg = small_cfg(tasks=["CartPole-v1", "CartPole-v1"])
    tr = PathNetTrainer(cfg)
    for _ in range(5):
        tr.update()
    before = tr.model.store.flat.detach().clone()
    winner, frozen = tr.end_task()
    after = tr.model.store.flat.detach()
    lay = tr.model.store.layout
    for s in lay.segments:
        sl = slice(s.offset, s.offset + s.numel)
        if s.layer >= 0 and frozen[s.layer, s.module] > 0.5:
            assert torch.equal(after[sl], before[sl]), s.name              # frozen path kept
        else:
            assert torch.equal(after[sl], tr.init_flat[sl]), s.name       # re-initialised (doom_pathnet.py:290-293)
    # frozen modules excluded from updates in the next task
    tr._start_task(1)
    frozen_before = after.clone()
    for _ in range(3):
        tr.update()
    for s in lay.segments:
        if s.layer >= 0 and frozen[s.layer, s.module] > 0.5:
            sl = slice(s.offset, s.offset + s.numel)
            assert torch.equal(tr.model.store.flat.detach()[sl], frozen_before[sl])
    # frozen modules always expressed in task-2 genotypes
    expr = tr.pop.expressed()
    assert (expr[:, frozen > 0.5] == 1).all()


def test_train_runs_task_sequence():
    cfg = small_cfg(tasks=["CartPole-v1", "CartPole-v1"])
    tr = PathNetTrainer(cfg)
    solved = tr.train(steps_per_task=400)
    assert set(solved) == {0, 1}
    assert tr.task_idx == 1 and tr.pop.frozen.sum() > 0


def test_checkpoint_resume_is_exact(tmp_path):
    cfg = small_cfg()
    torch.manual_seed(0)
    a = PathNetTrainer(cfg)
    for _ in range(4):
        a.update()
    p = str(tmp_path / "ck.safetensors")
    ckpt.save(a, p)
    torch.manual_seed(123)
    for _ in range(3):
        a.update()
    b = PathNetTrainer(cfg)
    ckpt.load(b, p)
    torch.manual_seed(123)
    for _ in range(3):
        b.update()
    assert torch.equal(a.model.store.flat, b.model.store.flat)
    assert np.array_equal(a.pop.genotypes, b.pop.genotypes)
    assert a.global_step == b.global_step


def test_tf_creation_order_importer():
    from pathnet_gym_amd.models.pathnet import ParamStore
    cfg = preset("reference").net
    names = ckpt.tf_creation_order(cfg)
    assert names[0] == "layer0.module0.weight" and names[-1] == "lstm.bias"
    st = ParamStore(cfg, "cpu", seed=0)
    arrays = [np.full(st.layout.by_name[n].shape, i, np.float32) for i, n in enumerate(names)]
    ckpt.import_tf_arrays(st, arrays)
    assert float(st.tensor("layer3.module9.bias")[0]) == names.index("layer3.module9.bias")


def test_windowed_mean_fitness_slows_and_averages_tournaments():
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    gens = {}
    for mode in ("last", "mean"):
        cfg = preset("cartpole-cpu")
        cfg.ga.fitness = mode
        cfg.ga.fitness_window = 4
        tr = PathNetTrainer(cfg)
        for _ in range(40):
            tr.update()
        gens[mode] = tr.pop.generation
        if mode == "mean":
            assert all(s > 0 for e in tr.pop.history for s in e.scores)      # real episode means, never pending
    assert gens["mean"] < gens["last"]


def test_checkpoint_keeps_continual_state_across_resume(tmp_path):
    """Resume inside task 1 with per-task heads: the next end_task must keep task 0's head."""
    cfg = small_cfg(tasks=["CartPole-v1", "CartPole-v1", "CartPole-v1"])
    cfg.net.per_task_heads = True
    cfg.net.num_tasks = 3
    a = PathNetTrainer(cfg)
    for _ in range(3):
        a.update()
    a.end_task()
    a._start_task(1)
    for _ in range(2):
        a.update()
    p = str(tmp_path / "ck.safetensors")
    ckpt.save(a, p)
    b = PathNetTrainer(cfg)
    ckpt.load(b, p)
    assert b.task_idx == 1 and b.frozen_tasks == {0}
    assert set(b.task_paths) == {0} and np.array_equal(b.task_paths[0], a.task_paths[0])
    assert b.solved_generation.get(0) == a.solved_generation.get(0)
    lay = b.model.store.layout
    head0 = [s for s in lay.segments if s.task == 0]
    assert head0 and not any(bool(b.opt.seg_trainable[lay.segments.index(s)]) for s in head0)
    before = b.model.store.flat.detach().clone()
    b.update()
    b.end_task()
    after = b.model.store.flat.detach()
    for s in head0:
        sl = slice(s.offset, s.offset + s.numel)
        assert torch.equal(after[sl], before[sl]), s.name          # task-0 head neither trained nor re-initialised
    assert b.frozen_tasks == {0, 1} and set(b.task_paths) == {0, 1}


def test_windowed_fitness_windows_restart_only_for_tournament_candidates():
    """A tournament firing must not wipe the episode windows of paths that are still filling theirs."""
    cfg = preset("cartpole-cpu")
    cfg.paths, cfg.envs_per_path = 8, 4
    cfg.ga.fitness = "mean"
    cfg.ga.fitness_window = 6
    tr = PathNetTrainer(cfg)
    fired_any = False
    for _ in range(120):
        before = tr.fit_cnt.clone()
        st = tr.update()
        if st.tournaments:
            fired_any = True
            cands = set(i for e in tr.pop.history[-st.tournaments:] for i in e.candidates)
            for p in range(tr.P):
                if p not in cands:
                    assert float(tr.fit_cnt[p]) >= float(before[p])      # still accumulating
                else:
                    assert float(tr.fit_cnt[p]) == 0.0
    assert fired_any


def test_compute_dtype_and_deterministic_flags():
    """--compute_dtype / --deterministic reach the config, survive the checkpoint JSON, and bad dtypes fail early;
    the torch backend always computes in fp32."""
    import pytest
    from pathnet_gym_amd.cli import build_parser, config_from_args
    from pathnet_gym_amd.config import TrainConfig
    a = build_parser().parse_args(["train", "--preset", "pong", "--compute_dtype", "fp32", "--deterministic", "1"])
    cfg = config_from_args(a)
    assert cfg.compute_dtype == "fp32" and cfg.deterministic
    c2 = TrainConfig.from_json(cfg.to_json())
    assert c2.compute_dtype == "fp32" and c2.deterministic
    bad = preset("cartpole-cpu")
    bad.compute_dtype = "fp16"
    with pytest.raises(ValueError):
        PathNetTrainer(bad, device="cpu")
    ok = preset("cartpole-cpu")
    ok.compute_dtype = "bf16"
    assert PathNetTrainer(ok, device="cpu").compute_dtype == "fp32"


def test_checkpoint_format_version_gates_legacy_task_id_mapping(tmp_path):
    """Format-1 checkpoints (rounds 1-3) named the synthetic games Pong-v0 ...; read_config maps those ids to Synth*.
    Format-2 checkpoints keep their ids: Pong-v0 now means the real gym game."""
    import torch
    from safetensors.torch import save_file
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.utils import checkpoint as ckpt
    cfg = preset("cartpole-cpu")
    cfg.tasks = ["Pong-v0", "Breakout-v0"]
    cfg.env = "Pong-v0"
    for ver, want in (("1", ["SynthPong-v0", "SynthBreakout-v0"]), ("2", ["Pong-v0", "Breakout-v0"])):
        p = str(tmp_path / f"v{ver}.safetensors")
        save_file({"x": torch.zeros(1)}, p, metadata={"format_version": ver, "config": cfg.to_json()})
        assert ckpt.read_config(p).tasks == want, ver
    assert ckpt.FORMAT_VERSION == 2
