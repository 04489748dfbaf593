"""CLI entry points and the supervised transfer workload (CPU)."""
import json
import subprocess
import sys

import numpy as np
import torch

from pathnet_gym_amd.algo.supervised import SupervisedPathNet, make_digits, supervised_config


def test_digit_data_shapes():
    X, y = make_digits("mnist", 20, 0)
    assert X.shape == (20, 3072) and y.shape == (20,) and float(X.min()) >= 0 and float(X.max()) <= 1
    X2, y2 = make_digits("svhn", 20, 1)
    assert X2.shape == (20, 3072)


def test_supervised_pathnet_learns_and_freezes():
    cfg = supervised_config(L=2, M=6, N=2, width=16)
    sp = SupervisedPathNet(cfg, population=8, num_tasks=2, device="cpu", seed=0)
    data = make_digits("mnist", 512, 0)
    accs = []
    for gen in range(6):
        acc = sp.train_generation(data, 0, steps=15, batch=16, lr=0.05, gen=gen)
        sp.pop.step(acc.astype(np.float32), gen)
        accs.append(acc.max())
    assert accs[-1] > 0.5
    w = int(np.argmax(acc))
    before = sp.store.flat.detach().clone()
    sp.end_task(w)
    assert sp.frozen.sum() > 0
    # task 2: frozen modules unchanged by training
    data2 = make_digits("svhn", 256, 1)
    sp.pop.init_genotypes()
    sp.train_generation(data2, 1, steps=3, batch=8, lr=0.05, gen=0)
    fe = sp.frozen_elems
    assert torch.equal(sp.store.flat.detach()[fe], before[fe])


def _cli(*args, timeout=300):
    r = subprocess.run([sys.executable, "-m", "pathnet_gym_amd.cli", *args], capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_cli_info_and_train_eval(tmp_path):
    info = json.loads(_cli("info", "--preset", "reference").strip().splitlines()[-1])
    assert info["params"] == 4173955
    ck = str(tmp_path / "c.safetensors")
    _cli("train", "--preset", "cartpole-cpu", "--worker_hosts_num", "4", "--steps_per_task", "800",
         "--checkpoint", ck, "--log_dir", str(tmp_path / "tb") + "/")
    out = json.loads(_cli("eval", "--preset", "cartpole-cpu", "--worker_hosts_num", "4", "--checkpoint", ck,
                          "--max_steps", "300").strip().splitlines()[-1])
    assert len(out["returns"]) == 4
    png = _cli("visualize", "--checkpoint", ck, "--out", str(tmp_path / "g.png")).strip()
    assert png.endswith("g.png")


def test_frozen_mode_available_lets_paths_skip_frozen_modules():
    """frozen_mode 'or' expresses the frozen path in every task-2 path (reference RL semantics); 'available'
    trains task-2 paths on their own genotypes only; frozen parameters stay fixed in both."""
    cfg = supervised_config(L=2, M=6, N=2, width=16)
    for mode in ("or", "available"):
        sp = SupervisedPathNet(cfg, population=8, num_tasks=2, device="cpu", seed=0, frozen_mode=mode)
        data = make_digits("mnist", 256, 0)
        acc = sp.train_generation(data, 0, steps=2, batch=8, lr=0.05, gen=0)
        before = sp.store.flat.detach().clone()
        sp.end_task(int(np.argmax(acc)))
        sp.pop.init_genotypes()
        paths = sp.paths()
        frozen = sp.frozen > 0.5
        if mode == "or":
            assert np.all(paths[:, frozen] == 1)
        else:
            assert np.array_equal(paths, (sp.pop.genotypes > 0.5).astype(np.float32))
            assert not np.all(paths[:, frozen] == 1)
        sp.train_generation(make_digits("svhn", 128, 1), 1, steps=2, batch=8, lr=0.05, gen=0, clip=5.0)
        assert torch.equal(sp.store.flat.detach()[sp.frozen_elems], before[sp.frozen_elems])
