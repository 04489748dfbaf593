"""Supervised PathNet: sequential transfer with module locking (MNIST -> SVHN).

BASELINE.json config 4.  The reference only keeps the leftovers of the
upstream supervised PathNet scripts (``pathnet.py:10-18,65-76,100-196``,
``input_data.py``): FC modules, the heterogeneous ``module2`` (skip / FC+ReLU /
residual by module index), ``select_two_candi`` binary tournaments and
parameter backup/restore.  This module rebuilds that workload on the shared
engine pieces:

* population of P paths trained in ONE batched forward (dense-masked PathNet
  trunk; every path gets its own minibatch), gradients summed over paths
  (shared modules, Hogwild-equivalent), plain SGD as in the supervised
  scripts;
* fitness = accuracy of the path on a held-out batch after its training
  steps; binary tournament (B=2) with the same mutation operator;
* task end: freeze the best path, re-initialise every other parameter, new
  task = new classification head, evolution restarts with the frozen modules
  always expressed.

Data: no dataset download is possible here, so both tasks are synthetic and
shape-compatible: ``mnist`` = 28x28 white-on-black bitmap digits with random
scale/shift/stroke/noise padded to 32x32x3; ``svhn`` = 32x32x3 coloured digits
on coloured backgrounds with neighbouring distractor digits.  Both are 10-way.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from ..config import LayerSpec, PathNetConfig
from ..models.pathnet import ParamStore, trunk_forward_ref
from .ga import Population

FONT5x7 = [
    "01110 10001 10011 10101 11001 10001 01110", "00100 01100 00100 00100 00100 00100 01110",
    "01110 10001 00001 00010 00100 01000 11111", "11111 00010 00100 00010 00001 10001 01110",
    "00010 00110 01010 10010 11111 00010 00010", "11111 10000 11110 00001 00001 10001 01110",
    "00110 01000 10000 11110 10001 10001 01110", "11111 00001 00010 00100 01000 01000 01000",
    "01110 10001 10001 01110 10001 10001 01110", "01110 10001 10001 01111 00001 00010 01100",
]


def _glyphs(device):
    g = torch.zeros(10, 7, 5, device=device)
    for d, s in enumerate(FONT5x7):
        for r, row in enumerate(s.split()):
            for c, ch in enumerate(row):
                g[d, r, c] = float(ch == "1")
    return g


def make_digits(kind: str, n: int, seed: int, device="cpu"):
    """Synthetic digit dataset -> (X [n, 32*32*3] float in [0,1], y [n] long)."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=gen)
    glyph = _glyphs("cpu")
    img = torch.zeros(n, 3, 32, 32)
    for i in range(n):
        if kind == "mnist":
            s = int(torch.randint(3, 5, (1,), generator=gen))
            g = F.interpolate(glyph[y[i]][None, None], scale_factor=s, mode="nearest")[0, 0]
            if torch.rand(1, generator=gen) < 0.5:      # thicker stroke
                g = torch.clamp(g + torch.roll(g, 1, 1), 0, 1)
            h, w = g.shape
            oy = 2 + int(torch.randint(0, max(1, 28 - h + 1), (1,), generator=gen))
            ox = 2 + int(torch.randint(0, max(1, 28 - w + 1), (1,), generator=gen))
            oy, ox = min(oy, 32 - h), min(ox, 32 - w)
            img[i, :, oy:oy + h, ox:ox + w] = g
            img[i] += 0.1 * torch.randn(3, 32, 32, generator=gen)
            img[i, 1:] = img[i, :1]          # gray replicated to 3 channels
        else:   # svhn-like
            bg = torch.rand(3, generator=gen)
            fg = (bg + 0.35 + 0.3 * torch.rand(3, generator=gen)) % 1.0
            img[i] = bg[:, None, None]
            s = 3
            for k, (dx, lab) in enumerate(((-13, int(torch.randint(0, 10, (1,), generator=gen))), (0, int(y[i])),
                                           (13, int(torch.randint(0, 10, (1,), generator=gen))))):
                g = F.interpolate(glyph[lab][None, None], scale_factor=s, mode="nearest")[0, 0]
                h, w = g.shape
                oy = 5 + int(torch.randint(-2, 3, (1,), generator=gen))
                ox = 16 - w // 2 + dx + int(torch.randint(-1, 2, (1,), generator=gen))
                y0, y1, x0, x1 = max(oy, 0), min(oy + h, 32), max(ox, 0), min(ox + w, 32)
                if x1 <= x0:
                    continue
                gg = g[y0 - oy:y1 - oy, x0 - ox:x1 - ox]
                region = img[i, :, y0:y1, x0:x1]
                img[i, :, y0:y1, x0:x1] = region * (1 - gg) + fg[:, None, None] * gg
            img[i] += 0.08 * torch.randn(3, 32, 32, generator=gen)
    X = img.clamp(0, 1).permute(0, 2, 3, 1).reshape(n, -1)     # NHWC flatten
    return X.to(device), y.to(device)


def supervised_config(L=3, M=10, N=3, width=20, din=32 * 32 * 3, module2=True):
    """FC PathNet; layers >0 use module2 types (j%3: skip / fc / residual, pathnet.py:137-168)."""
    layers = [LayerSpec("fc", width)]
    for _ in range(L - 1):
        layers.append(LayerSpec("fc", width, module_types=[0, 1, 2] if module2 else None))
    return PathNetConfig(L=L, M=M, N=N, input_shape=(din,), layers=layers, trunk_scale="none", num_actions=10)


def supervised_conv_config(M=10, N=3, width=64, maps=(16, 32)):
    """conv_module PathNet (pathnet.py:170-183): conv 5x5/2 -> conv 3x3/2 -> fc, M modules per layer."""
    layers = [LayerSpec("conv", maps[0], kernel=5, stride=2), LayerSpec("conv", maps[1], kernel=3, stride=2),
              LayerSpec("fc", width)]
    return PathNetConfig(L=3, M=M, N=N, input_shape=(32, 32, 3), layers=layers, trunk_scale="none", num_actions=10)


class SupervisedPathNet:
    def __init__(self, cfg: PathNetConfig, population: int, num_tasks: int, device, seed=1, B=2, backend="auto",
                 frozen_mode: str = "or"):
        """frozen_mode "or": frozen modules are always expressed (the reference's OR with fixed_path, as in RL);
        "available": a later task's genotypes may or may not select them (the PathNet paper's transfer
        setting); frozen parameters are never updated either way."""
        if frozen_mode not in ("or", "available"):
            raise ValueError(frozen_mode)
        self.frozen_mode = frozen_mode
        self.cfg = cfg
        self.P = population
        self.device = torch.device(device)
        # "hip": the typed-module FC kernels (csrc/typed_fc.hip, K19); "torch": the dense masked oracle
        self.backend = ("hip" if self.device.type == "cuda" else "torch") if backend == "auto" else backend
        self.store = ParamStore(cfg, self.device, seed)
        self.store.flat.requires_grad_(True)
        self.init_flat = self.store.flat.detach().clone()
        F_ = cfg.layers[-1].out
        g = torch.Generator().manual_seed(seed + 17)
        self.heads = [(torch.empty(F_, 10).uniform_(-1 / math.sqrt(F_), 1 / math.sqrt(F_), generator=g).to(device)
                       .requires_grad_(True), torch.zeros(10, device=device, requires_grad=True))
                      for _ in range(num_tasks)]
        self.pop = Population(population, cfg.L, cfg.M, cfg.N, B=B, seed=seed, concurrent=max(1, population // B))
        self.frozen = np.zeros((cfg.L, cfg.M), np.float32)
        self.frozen_elems = torch.zeros_like(self.store.flat, dtype=torch.bool)

    def logits(self, X, masks, rows_per_path, task):
        """X rows grouped by path: masks [P, L, M], row r -> path r // rows_per_path."""
        if self.backend == "hip":
            from ..ops.typed_fc import typed_trunk_forward
            feat = typed_trunk_forward(self.store, X, masks, rows_per_path)
        else:
            feat = trunk_forward_ref(self.store, X, masks.repeat_interleave(rows_per_path, 0))
        W, b = self.heads[task]
        return feat @ W + b

    def train_generation(self, data, task, steps, batch, lr, gen, clip: float = 0.0):
        """``steps`` SGD steps of every path on its own minibatch.  ``clip`` > 0: clip the global gradient norm
        (trunk + head) per step; without it the first steps of a later task can explode when frozen modules
        meet the new input distribution."""
        X, y = data
        n = X.shape[0]
        P = self.P
        masks = torch.from_numpy(self.paths()).to(self.device)
        g = torch.Generator(device="cpu").manual_seed(1000003 * gen + task)
        for _ in range(steps):
            idx = torch.randint(0, n, (P * batch,), generator=g).to(self.device)
            logit = self.logits(X[idx], masks, batch, task)
            loss = F.cross_entropy(logit, y[idx], reduction="sum") / batch
            self.store.flat.grad = None
            W, b = self.heads[task]
            W.grad = None
            b.grad = None
            loss.backward()
            with torch.no_grad():
                gflat = self.store.flat.grad.masked_fill(self.frozen_elems, 0.0)
                scale = lr / P
                if clip > 0:
                    norm = torch.sqrt(gflat.square().sum() + W.grad.square().sum() + b.grad.square().sum()) / P
                    scale = scale * float(torch.clamp(clip / (norm + 1e-12), max=1.0))
                self.store.flat.sub_(scale * gflat)
                W.sub_(scale * W.grad)
                b.sub_(scale * b.grad)
        # fitness: accuracy of every path on a fresh evaluation batch
        with torch.no_grad():
            idx = torch.randint(0, n, (P * batch * 4,), generator=g).to(self.device)
            pred = self.logits(X[idx], masks, batch * 4, task).argmax(-1)
            acc = (pred == y[idx]).float().view(P, -1).mean(1)
        return acc.cpu().numpy()

    def paths(self) -> np.ndarray:
        """[P, L, M] module masks the population trains and is evaluated with."""
        if self.frozen_mode == "or":
            return self.pop.expressed()
        return (self.pop.genotypes > 0.5).astype(np.float32)

    @torch.no_grad()
    def test_accuracy(self, path: np.ndarray, data, task: int, chunk: int = 512) -> float:
        """Accuracy of ONE path (expressed genotype [L, M]) on held-out data."""
        X, y = data
        m = torch.from_numpy(np.asarray(path, np.float32))[None].to(self.device)
        correct = 0
        for i in range(0, X.shape[0], chunk):
            xb = X[i:i + chunk]
            correct += int((self.logits(xb, m, xb.shape[0], task).argmax(-1) == y[i:i + chunk]).sum())
        return correct / X.shape[0]

    def end_task(self, winner: int):
        frozen = self.pop.freeze(winner, union=True)
        self.frozen = frozen
        keep = torch.zeros_like(self.frozen_elems)
        for s in self.store.layout.segments:
            if s.layer >= 0 and frozen[s.layer, s.module] > 0.5:
                keep[s.offset:s.offset + s.numel] = True
        self.frozen_elems = keep
        with torch.no_grad():
            self.store.flat.copy_(torch.where(keep, self.store.flat, self.init_flat))


def _progress(task, gen, best, t0):
    import sys
    print(f"[supervised] {task} generation {gen} best path accuracy {best:.3f} t={time.time() - t0:.0f}s",
          file=sys.stderr, flush=True)


def run_supervised_transfer(a) -> Dict:
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    tasks = [t.strip() for t in a.tasks.split(",")]
    arch = getattr(a, "arch", "fc")
    if arch == "conv":
        cfg = supervised_conv_config(a.M, a.N, a.width)
        cfg.input_shape = (32, 32, 3)
    else:
        cfg = supervised_config(a.L, a.M, a.N, a.width)
    n_train = getattr(a, "train_size", 4096)
    sizes = [int(v) for v in str(getattr(a, "train_sizes", "") or "").split(",") if v.strip()]
    n_of = lambda ti: sizes[min(ti, len(sizes) - 1)] if sizes else n_train      # noqa: E731
    frozen_mode = getattr(a, "frozen_mode", "or")
    sp = SupervisedPathNet(cfg, a.population, len(tasks), device, a.seed, a.B, frozen_mode=frozen_mode)
    out = {"tasks": tasks, "arch": arch, "train_sizes": [n_of(i) for i in range(len(tasks))], "per_task": [],
           "config": {"L": cfg.L, "M": cfg.M, "N": cfg.N, "layers": [(sp_.kind, sp_.out, sp_.kernel, sp_.stride)
                                                                     for sp_ in cfg.layers],
                      "population": a.population, "B": a.B, "generations": a.generations,
                      "steps_per_gen": a.steps_per_gen, "batch": a.batch, "lr": a.lr, "seed": a.seed,
                      "backend": sp.backend, "frozen_mode": frozen_mode}}
    t0 = time.time()
    gsz = [int(v) for v in str(getattr(a, "task_generations", "") or "").split(",") if v.strip()]
    gens_of = lambda ti: gsz[min(ti, len(gsz) - 1)] if gsz else a.generations      # noqa: E731
    eval_every = int(getattr(a, "eval_every", 0) or 0)
    out["config"].update(task_generations=[gens_of(i) for i in range(len(tasks))], eval_every=eval_every)

    clip = getattr(a, "clip", 0.0)
    standardize = getattr(a, "standardize", False)
    out["config"].update(clip=clip, standardize=standardize)

    def shaped(X):
        return X.reshape(X.shape[0], 32, 32, 3) if arch == "conv" else X

    def prep(train, test):
        """Per-task, per-channel standardisation with the TRAINING set's statistics."""
        (X, y), (Xt, yt) = train, test
        if standardize:
            c = X.reshape(X.shape[0], -1, 3)
            mu, sd = c.mean((0, 1)), c.std((0, 1)) + 1e-6
            X = ((c - mu) / sd).reshape(X.shape)
            Xt = ((Xt.reshape(Xt.shape[0], -1, 3) - mu) / sd).reshape(Xt.shape)
        return (shaped(X), y), (shaped(Xt), yt)

    for ti, name in enumerate(tasks):
        data, test = prep(make_digits(name, n_of(ti), a.seed * 31 + ti, device),
                          make_digits(name, 2048, a.seed * 31 + ti + 7919, device))
        if ti > 0:
            sp.pop.rng = np.random.RandomState(a.seed * 7919 + ti)     # the paired control replays this draw
            sp.pop.init_genotypes()
        best_hist, test_curve = [], []
        for gen in range(gens_of(ti)):
            acc = sp.train_generation(data, ti, a.steps_per_gen, a.batch, a.lr, gen, clip)
            sp.pop.step(acc.astype(np.float32), gen)
            best_hist.append(float(acc.max()))
            if eval_every and ti == len(tasks) - 1 and (gen + 1) % eval_every == 0:
                # held-out accuracy of the generation's best path: the learning-speed curve of the PathNet paper's
                # transfer comparison (the paired control records the same curve)
                test_curve.append([gen + 1, sp.test_accuracy(sp.paths()[int(np.argmax(acc))], test, ti)])
            _progress(name, gen, best_hist[-1], t0)
        winner = int(np.argmax(acc))
        test_acc = sp.test_accuracy(sp.paths()[winner], test, ti)
        sp.end_task(winner)
        out["per_task"].append({"task": name, "best_accuracy": best_hist[-1], "test_accuracy": test_acc,
                                "curve": best_hist, "test_curve": test_curve,
                                "frozen": sp.frozen.astype(int).tolist()})
    if getattr(a, "control", False) and len(tasks) > 1:
        # transfer check: the last task learned from scratch (no frozen source path), same budget.  paired (default):
        # common random numbers -- the same initial parameters and task head, the same minibatch and GA random
        # streams and the same initial genotypes as the transfer run's last task, so the ONLY difference is the
        # frozen source modules; otherwise an independent seed (seed + 1000)
        last = len(tasks) - 1
        paired = bool(getattr(a, "paired_control", 1))
        if paired:
            ctl = SupervisedPathNet(cfg, a.population, len(tasks), device, a.seed, a.B)
            ctl.pop.rng = np.random.RandomState(a.seed * 7919 + last)
            ctl.pop.init_genotypes()
            task_c = last
        else:
            ctl = SupervisedPathNet(cfg, a.population, 1, device, a.seed + 1000, a.B)
            task_c = 0
        data, test = prep(make_digits(tasks[-1], n_of(last), a.seed * 31 + last, device),
                          make_digits(tasks[-1], 2048, a.seed * 31 + last + 7919, device))
        hist, ctl_curve = [], []
        for gen in range(gens_of(last)):
            acc = ctl.train_generation(data, task_c, a.steps_per_gen, a.batch, a.lr, gen, clip)
            ctl.pop.step(acc.astype(np.float32), gen)
            hist.append(float(acc.max()))
            if eval_every and (gen + 1) % eval_every == 0:
                ctl_curve.append([gen + 1, ctl.test_accuracy(ctl.paths()[int(np.argmax(acc))], test, task_c)])
            _progress(tasks[-1] + " (scratch)", gen, hist[-1], t0)
        out["control"] = {"task": tasks[-1], "best_accuracy": hist[-1], "curve": hist, "paired": paired,
                          "test_curve": ctl_curve,
                          "test_accuracy": ctl.test_accuracy(ctl.paths()[int(np.argmax(acc))], test, task_c)}
        if ctl_curve:
            tr_c = out["per_task"][-1]["test_curve"]
            out["transfer_auc"] = {"transfer": float(np.mean([v for _, v in tr_c])),
                                   "from_scratch": float(np.mean([v for _, v in ctl_curve]))}
        thr = getattr(a, "target_accuracy", 0.9)
        first = lambda c: next((i for i, v in enumerate(c) if v >= thr), None)     # noqa: E731
        out["generations_to_accuracy"] = {"threshold": thr, "transfer": first(out["per_task"][-1]["curve"]),
                                          "from_scratch": first(hist)}
    out["seconds"] = time.time() - t0
    return out
