#!/usr/bin/env python3
"""Headline benchmark: env frames/s (whole node), Pong PathNet, 1..8 GPUs.

BASELINE.json metric "env frames/sec (whole node) + generations-to-solve,
Pong PathNet 1/2/4/8 GPU"; config "Atari Pong pixels, L=3 conv + 2 fc x
N=10 modules, population split across 8xMI355X".

One timed step = one full A2C update of the local population on every rank:
T=20 env steps of P paths x E envs (on-device Pong: physics + render + gray
+ resize + frame stack), PathNet forward (active modules only) + sampling,
bootstrap, loss gradient, backward, ONE fused RCCL all-reduce of
active-module gradients + fitness + counters, clip + RMSProp, GA
tournaments.  Nothing is skipped inside the timed region.

A "frame" is one agent-environment step (one observation), i.e. the same
unit as the reference's 63 global steps/s (aliencentipede.txt);
the synthetic Pong repeats each action for `frameskip`=4 emulator sub-frames
that are NOT counted.  Weak scaling: P paths per GPU, fixed.

Precision: the headline runs the fp32x engine (``--dtype fp32x``, reported as "dtype": "fp32x" with the
bound "max_rel_err_per_layer": 2e-5): the reference trains in fp32 (game_ac_network.py:89-110) and fp32x
matches a float64 autograd truth to < 2e-5 per layer (fp16 hi+lo operand pairs, gradients as scaled fp16 pairs,
three MFMAs per product, csrc/trunk_x3.hip; tests/test_x3_engine.py).  The bf16 engine is timed on the same config as
``value_bf16``.

Timing: after W warmup updates, ``--windows`` (default 3) back-to-back windows of EXACTLY K updates, each
bracketed by barrier + synchronize; every window's time is the max over ranks; the reported time is the
median window (``windows_ms_per_step`` lists all of them, ``spread_pct`` = (max - min) / median).

Strong scaling (the half of the metric that frames/s cannot show): the default run is weak scaling, P paths
per GPU.  ``strong_scaling`` additionally times the FIXED 64-path population split over the N ranks
(TrainConfig.paths_total: 64 / N paths per GPU, the same GA over P_total and the same summed gradient, env and
sampling RNG keyed by the global env index -- tests/test_distributed.py shows 4 ranks reproduce one process),
i.e. the per-update latency that divides the wall time of a solve (solves take 20-34 K updates whatever the
frame count, profiles/solve/README.md).  It reports the predicted seconds to solve (committed updates-to-solve
x measured ms/update; labelled a prediction) and, on more than one GPU, one in-run strong-mode solve under a
wall cap (the stop decision is collective, so ranks never disagree).  ``--scaling strong`` makes the strong
config the headline instead.

Steady state: every env's first episode starts at a random late score
(PongVec.stagger_scores), so fitness windows fill and tournaments fire inside
the timed window (``generations_in_timed_window``).  After it, one
generations-to-solve seed runs on a fresh trainer under a hard wall cap
(``generations_to_solve_in_run``); ``generations_to_solve`` lists every
committed multi-seed record of exactly this config (scripts/solve.py).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

``--gpus N`` > 1 without torchrun's WORLD_SIZE in the environment launches its own N ranks (like the reference's
auto_run.sh:6-14, which starts every process of its cluster itself): ``torch.distributed.run`` on 127.0.0.1 as a
CHILD process, started before this process imports torch or touches the GPU; rank 0's JSON line goes straight to
this process's stdout and the exit code is the launcher's.  Under torchrun, a WORLD_SIZE different from ``--gpus``
is an error (exit 2), so an N-GPU record can never come from a different number of ranks.

Per-rank strong-scaling shapes (one GPU): the 1-GPU run also times the per-rank shapes of the strong-scaling
split, P_total / N paths x E envs for N = 2, 4, 8 (3 windows each), and reports ``strong_scaling.per_rank`` with a
predicted seconds-to-solve per N: committed one-GPU updates-to-solve x (measured per-rank ms + a modelled ring
all-reduce of the gradient over xGMI).  A prediction, labelled as one.

Build provenance: on one GPU, a cold build of every csrc/*.hip into a scratch directory runs in a niced background
process during the run (``python -m pathnet_gym_amd._build --verify``); ``build.verified`` reports whether the cold
objects and library are byte-identical to the loaded ones (the build is reproducible: explicit compilation-unit
ids, relative paths).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

BASELINE_STEPS_PER_SEC = 63.0     # reference steady-state global agent steps/s


SOLVE_KEYS = ("preset", "paths_per_gpu", "envs_per_path", "t_max", "N", "B", "trunk_scale", "env_reduction", "lr",
              "entropy_beta", "gae_lambda", "fitness", "concurrent_tournaments", "dtype", "rmsp_epsilon")


def solve_key(cfg, preset_name: str) -> dict:
    """The fields of a scripts/solve.py record that must equal the bench config for its
    generations-to-solve to be reported next to the bench's frames/s."""
    return {"preset": preset_name, "paths_per_gpu": cfg.paths, "envs_per_path": cfg.envs_per_path,
            "t_max": cfg.a2c.t_max, "N": cfg.net.N, "B": cfg.ga.B, "trunk_scale": cfg.net.trunk_scale,
            "env_reduction": cfg.a2c.env_reduction, "lr": round(float(cfg.a2c.lr), 8),
            "entropy_beta": cfg.a2c.entropy_beta, "gae_lambda": cfg.a2c.gae_lambda, "fitness": cfg.ga.fitness,
            "concurrent_tournaments": cfg.ga.concurrent_tournaments, "dtype": cfg.compute_dtype,
            "rmsp_epsilon": cfg.a2c.rmsp_epsilon}


def equivalent_builds(sources: str, root: str) -> dict:
    """Builds whose committed records count for the build ``sources``: itself, and every build linked to it by a
    reproducing certificate in root/build_equivalence.json (scripts/certify_build.py: a committed deterministic seed
    re-run on the newer build gave the same generations, updates, frames and held-out mean), transitively.  Returns
    {sha: certificate or None}."""
    try:
        certs = [c for c in json.loads(open(os.path.join(root, "build_equivalence.json")).read())
                 if c.get("reproduces") and c.get("from") and c.get("to")]
    except (OSError, ValueError):
        certs = []
    out, todo = {sources: None}, [sources]
    while todo:
        cur = todo.pop()
        for c in certs:
            for a, b in ((c["from"], c["to"]), (c["to"], c["from"])):
                if a == cur and b not in out:
                    out[b] = c
                    todo.append(b)
    return out


def solve_records(key: dict, n_gpus: int, sources: str = None, root: str = None):
    """The committed solve runs (profiles/solve/*.json, written by scripts/solve.py --out) of exactly this config on
    ``n_gpus`` GPUs, under the v2 criterion (algo/solve.py: the task horizon where the lr anneal reaches 0, a held-out
    confirmation of the winning path) and built from the same sources as the running library (``sources``, the
    build's sources_sha256; None = any build), ONE record per distinct seed (the latest).  Runs that stopped on a wall
    limit before the horizon without solving say nothing about the horizon and are listed apart.  The statistic is the
    median over seeds with "unsolved at horizon" counted as infinite: null unless most seeds solved."""
    import glob
    from pathnet_gym_amd.algo.solve import CRITERION
    root = root or os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "solve")
    by_seed, excluded = {}, {"other_config": 0, "pre_v2_criterion": 0, "other_build": 0, "wall_limited": 0}
    equiv = equivalent_builds(sources, root) if sources is not None else {}
    for f in sorted(glob.glob(os.path.join(root, "*.json"))):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        if not isinstance(d, dict):                 # build_equivalence.json
            continue
        c = d.get("config") or {}
        if d.get("metric") != "generations_to_solve" or d.get("n_gpus") != n_gpus or not c.get("ga", True) \
                or c.get("same_path"):
            continue
        c = dict(c, dtype=c.get("dtype", "bf16"), lr=round(float(c.get("lr", 0.0)), 8),
                 rmsp_epsilon=c.get("rmsp_epsilon", 0.1))
        if any(c.get(k) != key[k] for k in SOLVE_KEYS):
            excluded["other_config"] += 1
            continue
        if d.get("criterion") != CRITERION:
            excluded["pre_v2_criterion"] += 1
            continue
        rec_sha = (d.get("build") or {}).get("sources_sha256")
        if sources is not None and rec_sha not in equiv:
            excluded["other_build"] += 1
            continue
        if not d.get("solved") and d.get("stopped") != "horizon":
            excluded["wall_limited"] += 1
            continue
        r = {"seed": c.get("seed"), "solved": bool(d.get("solved")), "generations": d.get("generations_to_solve"),
             "updates": d.get("updates_to_solve"), "frames": d.get("frames_to_solve"),
             "seconds": d.get("train_seconds_to_solve") or d.get("seconds_to_solve"), "lr_at_solve": d.get("lr_at_solve"),
             "heldout_mean": d.get("heldout_mean"), "winner_fitness": d.get("winner_fitness"),
             "unconfirmed_candidates": sum(1 for x in d.get("candidates", []) if not x.get("confirmed")),
             "stopped": d.get("stopped"), "deterministic": bool(c.get("deterministic")),
             "finished_at": d.get("finished_at", 0.0), "file": os.path.relpath(f, os.path.dirname(root)),
             "build": rec_sha}
        old = by_seed.get(r["seed"])
        if old is None or r["finished_at"] >= old["finished_at"]:
            by_seed[r["seed"]] = r
    runs = [by_seed[k] for k in sorted(by_seed, key=lambda x: (x is None, x))]
    if not runs:
        return {"value": None, "note": "no v2-criterion scripts/solve.py run of exactly this config and build is "
                "committed", "config": key, "excluded": excluded, "build_sources_sha256": sources}
    inf = float("inf")
    gens = sorted(r["generations"] if r["solved"] else inf for r in runs)
    upd = sorted(r["updates"] if r["solved"] else inf for r in runs)
    med = statistics.median(gens)
    solved = [g for g in gens if g != inf]
    return {"value": None if med == inf else med,
            "statistic": "median over distinct seeds, unsolved-at-horizon counted as infinite (null unless most "
                         "seeds solved)",
            "min": min(solved) if solved else None, "max": max(gens) if gens[-1] != inf else "unsolved",
            "updates_median": None if statistics.median(upd) == inf else statistics.median(upd),
            "solved_seeds": len(solved), "seeds": len(runs), "runs": runs, "config": key, "excluded": excluded,
            "build_sources_sha256": sources,
            "equivalent_builds": {k: (v or {}).get("committed_file") for k, v in equiv.items() if k != sources},
            "criterion": CRITERION}


def build_trainer(args, ctx, dtype: str, stagger: bool, paths_total: int = 0):
    """The bench trainer; ``paths_total`` > 0: strong scaling (that population split over the ranks)."""
    from pathnet_gym_amd.config import preset
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset(args.preset)
    if args.env:
        cfg.env = args.env
        cfg.tasks = [args.env] + [t for t in cfg.tasks if t != args.env]
    cfg.paths = args.paths
    cfg.paths_total = paths_total
    cfg.envs_per_path = args.envs
    cfg.a2c.t_max = args.tmax
    cfg.backend = args.backend
    cfg.use_graph = not args.no_graph
    # fp32x: the first layer reads the frame ring (env 70 -> 39 us per step; conv1 forward / weight gradient +6 % /
    # +7 %; window 11.42 -> 11.15 ms, profiles/r3/kwin_x3_v19*.md); bf16 keeps packed stacks (a wash there, docs/PERF.md)
    cfg.frame_ring = args.ring or (dtype == "fp32x" and not args.packed)
    # concurrent tournaments: paths/16 of the population one GA sees per update -- per rank in weak scaling (the GA
    # takes the same number of tournaments per update on 1, 2, 4 and 8 GPUs), of P_total in strong scaling (exactly
    # the one-GPU GA)
    cfg.ga.concurrent_tournaments = args.concurrent or max(1, (paths_total or cfg.paths) // 16)
    cfg.ga.backend = args.ga_backend
    cfg.compute_dtype = dtype
    cfg.deterministic = args.deterministic
    cfg.rollout_groups = args.rollout_groups
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx)
    if stagger and hasattr(tr.env, "stagger_scores"):
        tr.env.stagger_scores()
    return cfg, tr


def gpu_telemetry() -> dict:
    """GPU clock / power / temperature now (torch.cuda's SMI queries, amdsmi on ROCm); {} where unavailable."""
    import torch
    out = {}
    if not torch.cuda.is_available():
        return out
    for k, f in (("sclk_mhz", "clock_rate"), ("power", "power_draw"), ("temp_c", "temperature")):
        try:
            out[k] = getattr(torch.cuda, f)()
        except Exception:
            pass
    return out


def timed_windows(tr, ctx, steps: int, warmup: int, windows: int = 1, markers: bool = False, info=None,
                  mark_window: int = 0):
    """W untimed updates, then ``windows`` back-to-back windows of EXACTLY K updates, each between barrier +
    synchronize on both sides; a window's time is the max over ranks.  Returns [(seconds, frames, generations)].
    ``info`` (a list): per window, the GPU telemetry sampled while its last updates still run (before the drain) and
    the population's mean active modules per layer (mutation can grow a path; the work per update follows it)."""
    import torch

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        ctx.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(warmup):
        tr.update()
    tr.flush()
    out = []
    for w in range(windows):
        sync()
        gen0 = tr.pop.generation
        step0 = tr.global_step
        if markers and w == mark_window:
            from pathnet_gym_amd.ops import _lib as _plib
            _plib.call("launch_prof_marker", 1, _plib.stream())
        host0 = dict(tr.tracer.totals_ms)
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.update()
        tel = gpu_telemetry() if info is not None else None
        tr.flush()                               # drain the pipelined host bookkeeping of the last update
        if markers and w == mark_window:
            _plib.call("launch_prof_marker", 2, _plib.stream())
        sync()
        dt = ctx.max_scalar(time.perf_counter() - t0)
        out.append((dt, tr.global_step - step0, tr.pop.generation - gen0))   # whole-job agent steps
        if info is not None:
            ex = tr.pop.expressed()
            tel["active_modules_per_layer"] = [round(float(x), 3) for x in ex.sum(axis=2).mean(axis=0)]
            # the widest path per layer: a path of more than 4 (or 6) active modules runs extra passes in some kernels
            tel["active_modules_max_per_layer"] = [int(x) for x in ex.sum(axis=2).max(axis=0)]
            tel["ms"] = round(dt / steps * 1e3, 3)
            # host milliseconds per update in each phase of the pipelined loop (utils/tracing.py): "collect" is the
            # wait for the previous update's read-back, i.e. GPU-bound time; the rest is host work
            tel["host_ms_per_update"] = {k: round((v - host0.get(k, 0.0)) / steps, 3)
                                         for k, v in tr.tracer.totals_ms.items() if v - host0.get(k, 0.0) > 0}
            info.append(tel)
    return out


def window_summary(wins, steps: int) -> dict:
    ms = [w[0] / steps * 1e3 for w in wins]
    med = statistics.median(ms)
    return {"ms": med, "all": [round(x, 3) for x in ms],
            "spread_pct": round((max(ms) - min(ms)) / med * 100.0, 2) if med > 0 else 0.0,
            "frames": wins[0][1], "generations": sum(w[2] for w in wins)}


def in_run_solve(args, ctx, dtype: str, cap_s: float, paths_total: int = 0) -> dict:
    """One seed of generations-to-solve on a FRESH trainer of the bench config, observed inside this run under a hard
    wall cap (scripts/solve.py is the multi-seed version), with the criterion of algo/solve.py: a tournament winner at
    the reward threshold, confirmed by a held-out evaluation of its path, before the task horizon.  Every rank takes
    the same decisions (replicated GA, rank 0's held-out mean, a collective wall-cap check every 32 updates)."""
    from pathnet_gym_amd.algo.solve import SolveTracker
    a = argparse.Namespace(**vars(args))
    if args.solve_deterministic and ctx.world == 1 and dtype == "fp32x":
        # the committed seeds ran in the deterministic mode (bit-reproducible): this run repeats one of them exactly
        a.deterministic = True
    cfg, tr = build_trainer(a, ctx, dtype, stagger=False, paths_total=paths_total)
    t0 = time.time()
    last = [t0]

    def progress(c=None):
        now = time.time()
        if ctx.is_main and (c is not None or now - last[0] > 30):     # stderr: the JSON line stays the only stdout line
            last[0] = now
            print(f"[bench] solve t={now - t0:.0f}s generation={tr.pop.generation} frames={tr.global_step} "
                  f"updates={tr.updates} best_winner={trk.best:.2f}" + (f" candidate={c}" if c else ""),
                  file=sys.stderr, flush=True)

    trk = SolveTracker(tr, wall_s=cap_s, log=progress)
    while not trk.observe(tr.update()):
        progress()
    tr.flush()
    out = {"seed": cfg.seed, "cap_s": round(cap_s, 1), "paths_per_gpu": cfg.paths, "paths_total": tr.P_total,
           "deterministic": bool(tr.model.hip is not None and tr.model.hip.reproducible)}
    out.update(trk.record())
    return out


def compare_with_committed(run: dict, records: dict) -> dict:
    """The in-run solve against the committed record of the same seed (same config, build and criterion): in the
    deterministic mode one seed defines a run, so generations, updates and the held-out mean must be equal."""
    if not run or not run.get("deterministic"):
        return {"compared": False, "reason": "the in-run solve was not deterministic"}
    same = [r for r in (records or {}).get("runs", []) if r.get("seed") == run.get("seed") and r.get("deterministic")]
    if not same:
        return {"compared": False, "reason": "no committed deterministic record of this seed, config and build"}
    r = same[0]
    if run.get("stopped") != "solved":
        return {"compared": True, "file": r["file"], "reproduces": False, "reason": f"in-run solve {run.get('stopped')}"}
    eq = (run.get("generations_to_solve") == r.get("generations") and run.get("updates_to_solve") == r.get("updates")
          and run.get("heldout_mean") == r.get("heldout_mean"))
    return {"compared": True, "file": r["file"], "reproduces": bool(eq),
            "committed": {"generations": r.get("generations"), "updates": r.get("updates"),
                          "heldout_mean": r.get("heldout_mean")}}


def committed_updates_to_solve(key: dict, sources: str = None) -> list:
    """Optimizer updates each committed solved seed (solve_records: v2 criterion, this build) of the one-GPU bench
    config needed."""
    rec = solve_records(key, 1, sources)
    return sorted(int(r["updates"]) for r in rec.get("runs", []) if r["solved"] and r["updates"])


def self_launch(n: int) -> int:
    """``--gpus N`` > 1 outside torchrun: run ``torch.distributed.run --nproc-per-node N`` on 127.0.0.1 over this same
    command line as a child process (this process never imports torch or touches the GPU) and return its exit code.
    The ranks inherit stdout, so rank 0's JSON line is this process's only stdout line."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver (RCCL peer access)
    print(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def under_profiler() -> bool:
    """rocprofv3 (or another tool) preloads a library that initialises the GPU in every process it enters, so a
    child started from here would count as an exec after GPU initialisation: no background build then."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def start_build_verify():
    """Cold-build every source in a background child process at the lowest CPU priority (build provenance; collected
    by finish_build_verify).  The child is this interpreter itself (no `nice` / shell hop in between)."""
    import subprocess
    import tempfile
    out = tempfile.NamedTemporaryFile("w+", suffix=".json", delete=False)
    cmd = [sys.executable, "-m", "pathnet_gym_amd._build", "--verify", "--jobs", "8"]
    p = subprocess.Popen(cmd, stdout=out, stderr=subprocess.STDOUT, cwd=os.path.dirname(os.path.abspath(__file__)),
                         preexec_fn=lambda: os.nice(19))
    return p, out, time.time()


def finish_build_verify(h, wait_s: float = 240.0) -> dict:
    p, out, t0 = h
    try:
        p.wait(timeout=wait_s)
    except Exception:
        p.kill()
        p.wait()
        return {"status": f"not finished {wait_s:.0f} s after the run (killed)"}
    out.seek(0)
    lines = [l for l in out.read().splitlines() if l.startswith("{")]
    os.unlink(out.name)
    if p.returncode != 0 or not lines:
        return {"status": f"failed (rc {p.returncode})"}
    d = json.loads(lines[-1])
    d["status"] = "ok"
    return d


# modelled ring all-reduce of the fp32 gradient over xGMI (per-rank strong-scaling prediction on one GPU): RCCL ring,
# 2 (N - 1) steps of ALLREDUCE_STEP_US latency plus 2 (N - 1) / N x bytes at ALLREDUCE_BUS_GBS bus bandwidth.  A
# model, not a measurement (no multi-GPU node here); the overlapped exchange hides part of it behind the first
# layer's weight gradient, which the model ignores (conservative).
ALLREDUCE_STEP_US = 10.0
ALLREDUCE_BUS_GBS = 150.0


def allreduce_model_ms(n: int, nbytes: int) -> float:
    if n <= 1:
        return 0.0
    return (2 * (n - 1) * ALLREDUCE_STEP_US * 1e-6 + 2.0 * (n - 1) / n * nbytes / (ALLREDUCE_BUS_GBS * 1e9)) * 1e3


def per_rank_shapes(args, ctx, numel: int, upd: list, headline_ms: float) -> dict:
    """One GPU: time the per-rank shape of the strong-scaling split for each N in --per-rank-shapes --
    paths_total / N paths x E envs, with the GA taking the whole population's paths_total / 16 concurrent
    tournaments -- in ``--windows`` windows, and predict seconds-to-solve on N GPUs from it."""
    import torch
    out = {}
    med = upd[len(upd) // 2] if upd else None
    for n in [int(x) for x in str(args.per_rank_shapes).strip("'\"").split(",") if x.strip()]:
        if n <= 1 or args.paths_total % n:
            continue
        a = argparse.Namespace(**vars(args))
        a.paths = args.paths_total // n
        a.concurrent = args.concurrent or max(1, args.paths_total // 16)
        _, trn = build_trainer(a, ctx, args.dtype, not args.no_stagger)
        w = window_summary(timed_windows(trn, ctx, args.steps, args.warmup, args.windows), args.steps)
        del trn
        torch.cuda.empty_cache() if torch.cuda.is_available() else None
        ar = allreduce_model_ms(n, 4 * numel)
        r = {"paths_per_gpu": a.paths, "envs_per_path": args.envs, "ms_per_update": round(w["ms"], 3),
             "windows_ms": w["all"], "spread_pct": w["spread_pct"], "allreduce_model_ms": round(ar, 3),
             "predicted_speedup_vs_1gpu": round(headline_ms / (w["ms"] + ar), 2)}
        if med:
            r["predicted_seconds_to_solve"] = round(med * (w["ms"] + ar) / 1e3, 1)
        out[str(n)] = r
    return {"measured_on": "1 GPU, each per-rank shape run alone", "by_n_gpus": out,
            "allreduce_model": f"ring: 2(N-1) x {ALLREDUCE_STEP_US:g} us + 2(N-1)/N x {4 * numel} B at "
                               f"{ALLREDUCE_BUS_GBS:g} GB/s bus bandwidth (modelled, not measured)",
            "prediction": "median committed one-GPU updates-to-solve x (measured per-rank ms/update + modelled "
                          "all-reduce); strong mode computes the one-GPU GA and summed gradient, so it needs the same "
                          "updates.  A prediction, not a measured multi-GPU solve"}


def reference_preset_windows(args, ctx) -> dict:
    """The reference's OWN default network (USE_LSTM=True, constants.py:30-31: L=4 = 3 conv + linear 1408->256, M=10,
    N=4, BasicLSTMCell(256), game_ac_network.py:303-521; 18-way head, ACTION_SIZEZ) on its first task (synthetic
    Alien, aliencentipede.txt) at the bench's paths x envs, same dtype, windows and warmup as the headline."""
    from pathnet_gym_amd.config import preset
    a = argparse.Namespace(**vars(args))
    a.preset = "reference"
    a.env = None
    cfg, trr = build_trainer(a, ctx, args.dtype, False)
    tele = []
    w = window_summary(timed_windows(trr, ctx, args.steps, args.warmup, args.windows, info=tele), args.steps)
    net = cfg.net
    out = {"preset": "reference", "env": cfg.tasks[0], "dtype": trr.compute_dtype,
           "model": f"PathNet L={net.L} (conv 8x8/4, 4x4/2, 3x3/1 + fc {net.layers[-1].out}) x M={net.M}, N={net.N}, "
                    f"LSTM {net.lstm_size}, {net.num_actions} actions",
           "paths_per_gpu": cfg.paths, "envs_per_path": cfg.envs_per_path, "t_max": cfg.a2c.t_max,
           "ms_per_update": round(w["ms"], 3), "windows_ms": w["all"], "spread_pct": w["spread_pct"],
           "frames_per_sec": round(w["frames"] / (w["ms"] * args.steps / 1e3), 1),
           "frame_ring": bool(getattr(trr.engine, "ring", False)), "lstm_hip": bool(trr.engine.lstm_hip),
           # per window: clock, and the population's mean / widest active-module count per layer (a path of more than
           # 4 modules in the 3x3 layer still lengthens its weight gradient, docs/PERF.md)
           "windows_telemetry": [{k: t.get(k) for k in ("ms", "sclk_mhz", "active_modules_per_layer",
                                                        "active_modules_max_per_layer")} for t in tele]}
    del trr
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--windows", type=int, default=3, help="timed windows of --steps updates (median reported)")
    ap.add_argument("--paths", type=int, default=64, help="paths per GPU (weak scaling)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="headline: weak (--paths per GPU) or strong (--paths-total split over the GPUs)")
    ap.add_argument("--paths-total", type=int, default=64,
                    help="strong scaling: the fixed population split over the GPUs (the one-GPU bench population)")
    ap.add_argument("--envs", type=int, default=32, help="envs per path (multiple of 16)")
    ap.add_argument("--tmax", type=int, default=20)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--ring", action="store_true", help="frame ring (single-frame writes) instead of packed stacks")
    ap.add_argument("--packed", action="store_true", help="fp32x: packed 4-frame stacks instead of the frame ring")
    ap.add_argument("--preset", default="pong")
    ap.add_argument("--env", default=None, help="train this task of the preset's suite instead of its first task")
    ap.add_argument("--kernel-opt", action="append", default=[],
                    help="kernel switch NAME=VALUE (fast_conv_set_*), for A/B measurements")
    ap.add_argument("--dtype", default="fp32x", choices=["bf16", "fp32", "fp32x"],
                    help="HIP engine compute dtype.  fp32x (headline): fp32-accurate split operands (fp16 / bf16 "
                         "hi+lo pairs, 3 MFMAs per product, <= 2e-5 per layer vs a plain fp32 oracle, "
                         "csrc/trunk_x3.hip); fp32: fp32 MFMA operands (csrc/trunk_f32.hip); bf16: bf16 operands")
    ap.add_argument("--deterministic", action="store_true", help="fixed-order gradient reductions (bit-reproducible)")
    ap.add_argument("--rollout-groups", type=int, default=0,
                    help="path groups stepped on their own streams in the rollout (0 = auto, 1 = one stream)")
    ap.add_argument("--ga-backend", default="device", choices=["device", "host"],
                    help="device: GA kernels inside the update graph + pipelined host bookkeeping")
    ap.add_argument("--concurrent", type=int, default=None,
                    help="concurrent tournaments (default: paths/16 -- per rank in weak scaling, so the GA takes the "
                         "same number of tournaments per update on 1, 2, 4 and 8 GPUs; of P_total in strong scaling)")
    ap.add_argument("--no-stagger", action="store_true",
                    help="start every env at 0-0 (default: random late scores, so tournaments fire inside the window)")
    ap.add_argument("--solve-seconds", type=float, default=None,
                    help="after the timed windows, run one generations-to-solve seed on a fresh trainer for at most "
                         "this long (default: one GPU, the bench config, what is left of a 560 s run, at most 480 s; "
                         "several GPUs, the strong-scaling config, what is left of 480 s, at most 300 s; 0 = off)")
    ap.add_argument("--solve-deterministic", type=int, default=1,
                    help="one GPU, fp32x: run the in-run solve in the deterministic mode, so it repeats the committed "
                         "record of its seed exactly (reported as generations_to_solve_in_run.vs_committed)")
    ap.add_argument("--compare-bf16", type=int, default=None,
                    help="also time the bf16 engine on the same config (default: on for one GPU)")
    ap.add_argument("--reference-preset", type=int, default=None,
                    help="also time the reference's own LSTM network (preset 'reference'; default: on for one GPU)")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling windows on several GPUs")
    ap.add_argument("--prof-window", action="store_true",
                    help="launch marker kernels around the first timed window (scripts/prof_window.py summarises the "
                         "rocprofv3 kernel trace between them)")
    ap.add_argument("--prof-window-index", type=int, default=0, help="--prof-window: which timed window to mark")
    ap.add_argument("--per-rank-shapes", default="2,4,8",
                    help="one GPU: also time the strong-scaling per-rank shapes paths_total/N for these N ('' = off)")
    ap.add_argument("--no-verify-build", action="store_true",
                    help="skip the background cold build that checks the loaded library against the sources")
    args = ap.parse_args()
    t_start = time.time()
    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is None and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    if ws_env is not None and int(ws_env) != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={ws_env}: refusing to report an {args.gpus}-GPU record from "
              f"{ws_env} ranks", file=sys.stderr, flush=True)
        sys.exit(2)
    verify_h = None
    if args.backend == "hip" and int(ws_env or 1) == 1 and not args.no_verify_build and not args.prof_window \
            and not under_profiler():
        verify_h = start_build_verify()

    import torch

    from pathnet_gym_amd.parallel.dist import init_distributed

    build_info = None
    if args.backend == "hip":
        from pathnet_gym_amd import _build
        build_info = _build.build_info(_build.build())

    if args.kernel_opt:
        from pathnet_gym_amd.ops import _lib
        for kv in args.kernel_opt:
            k, v = kv.split("=")
            lib = _lib.lib()
            (getattr(lib, k) if hasattr(lib, k) and "_set_" in k else getattr(lib, "fast_conv_set_" + k))(int(v))
    ctx = init_distributed()
    world = ctx.world
    single = world == 1 and not args.prof_window
    if args.scaling == "strong" and args.paths_total % world:
        raise SystemExit(f"--paths-total {args.paths_total} is not divisible by {world} GPUs")
    head_total = args.paths_total if args.scaling == "strong" else 0
    compare = args.compare_bf16 if args.compare_bf16 is not None else int(single and args.dtype != "bf16")
    stagger = not args.no_stagger
    cfg, tr = build_trainer(args, ctx, args.dtype, stagger, paths_total=head_total)
    verified = None
    if verify_h is not None:
        # the cold build (8 niced hipcc jobs) runs while torch imports and the trainer builds; it is joined HERE, so
        # no compiler competes with any timed window
        verified = finish_build_verify(verify_h)
        verify_h = None
    tele = []
    wins = timed_windows(tr, ctx, args.steps, args.warmup, args.windows, markers=args.prof_window, info=tele,
                         mark_window=min(args.prof_window_index, args.windows - 1))
    ws = window_summary(wins, args.steps)
    dt = ws["ms"] * args.steps / 1e3
    value = ws["frames"] / dt
    x3 = tr.compute_dtype == "fp32x"
    rec = {
        "metric": "env_frames_per_sec_whole_node_pong_pathnet",
        "value": round(value, 1),
        "unit": "env frames/s (agent steps, all GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ws["ms"], 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": round(value / BASELINE_STEPS_PER_SEC, 1),
        "dtype": tr.compute_dtype,
        "compute": {"fp32x": "fp32-accurate split operands: fp16 hi+lo pairs (forward), fp16 hi+lo pairs of G * 2^e "
                             "(gradients, one power of two per layer from the amax), 3 MFMAs per product, "
                             "sign-alternating accumulation in the input gradients, fp32 accumulation and master "
                             "weights; < 2e-5 relative per layer vs a float64 autograd truth, at most plain fp32's own "
                             "error on ill-conditioned layers (tests/test_x3_engine.py)",
                    "fp32": "fp32 MFMA operands (v_mfma_f32_16x16x4_f32)",
                    "bf16": "bf16/fp16 MFMA operands, fp32 accumulation (reduced precision)"}[tr.compute_dtype],
        "max_rel_err_per_layer": 2e-5 if x3 else (1e-5 if tr.compute_dtype == "fp32" else None),
        "windows": args.windows,
        "windows_ms_per_step": ws["all"],
        "spread_pct": ws["spread_pct"],
        "windows_telemetry": tele,
        "data": (f"synthetic: on-device Atari-style {cfg.tasks[0]} simulator (210x160 RGB -> gray 160x120 x4 "
                 "stack), random-init weights") if len(cfg.net.input_shape) == 3 else
                f"synthetic: on-device {cfg.tasks[0]}, random-init weights",
        "config": {
            "model": f"PathNet {cfg.net.L} layers ("
                     + " + ".join(f"{sp.kind} {sp.out}" + (f" {sp.kernel}x{sp.kernel}/{sp.stride}"
                                                             if sp.kind == "conv" else "")
                                  for sp in cfg.net.layers)
                     + f") x M={cfg.net.M} modules, N={cfg.net.N}, A2C T={cfg.a2c.t_max}, B={cfg.ga.B} tournament",
            "global_batch": cfg.paths * cfg.envs_per_path * world * cfg.a2c.t_max,
            "seq_len": cfg.a2c.t_max,
            "parallelism": f"dp{world} (population split: {cfg.paths} paths x {cfg.envs_per_path} envs per GPU"
                           + (f", {tr.P_total} paths in total)" if head_total else ")"),
            "backend": args.backend,
            "hipgraph": cfg.use_graph,
            "frame_ring": bool(getattr(tr.engine, "ring", False)),
            "rollout_groups": int(getattr(tr.engine, "groups", 1)),
            "ga": f"{cfg.ga.backend} (B={cfg.ga.B}, {cfg.ga.concurrent_tournaments} concurrent tournaments, "
                  f"fitness {cfg.ga.fitness} over {cfg.ga.window_for(cfg.envs_per_path)} episodes)",
            "pipelined": bool(tr.pipelined),
            "overlap_allreduce": bool(getattr(tr.engine, "split", False)),
            "deterministic": bool(getattr(tr.model.hip, "reproducible", False)),
            "episode_stagger": stagger,
        },
        "generations_in_timed_window": int(wins[0][2]),
        "generations_in_timed_windows": int(ws["generations"]),
    }
    if build_info is not None:
        rec["build"] = build_info
    if getattr(tr, "precision_note", None):
        rec["precision_note"] = tr.precision_note
    tr_numel = int(tr.model.store.layout.numel)
    del tr
    if compare:
        _, trb = build_trainer(args, ctx, "bf16", stagger, paths_total=head_total)
        wb = window_summary(timed_windows(trb, ctx, args.steps, args.warmup, args.windows), args.steps)
        rec["value_bf16"] = round(wb["frames"] / (wb["ms"] * args.steps / 1e3), 1)
        rec["ms_per_step_bf16"] = round(wb["ms"], 3)
        rec["windows_ms_per_step_bf16"] = wb["all"]
        del trb
    torch.cuda.empty_cache() if torch.cuda.is_available() else None
    ref_on = args.reference_preset if args.reference_preset is not None else int(single and args.preset == "pong")
    if ref_on:
        rec["reference_preset"] = reference_preset_windows(args, ctx)
        torch.cuda.empty_cache() if torch.cuda.is_available() else None
    # strong scaling: the one-GPU population (64 paths) split over the ranks
    key = solve_key(cfg, args.preset)
    key1 = dict(key, paths_per_gpu=args.paths_total, concurrent_tournaments=max(1, args.paths_total // 16))
    sources = (build_info or {}).get("sources_sha256")
    upd = committed_updates_to_solve(key1, sources)
    strong = None
    if args.scaling == "strong" or (world == 1 and args.paths == args.paths_total):
        strong = {"ms_per_update": round(ws["ms"], 3), "windows_ms": ws["all"], "same_as_headline": True}
    elif not args.no_strong and args.paths_total % world == 0:
        _, trs = build_trainer(args, ctx, args.dtype, stagger, paths_total=args.paths_total)
        wst = window_summary(timed_windows(trs, ctx, args.steps, args.warmup, args.windows), args.steps)
        strong = {"ms_per_update": round(wst["ms"], 3), "windows_ms": wst["all"], "spread_pct": wst["spread_pct"],
                  "frames_per_sec": round(wst["frames"] / (wst["ms"] * args.steps / 1e3), 1)}
        del trs
        torch.cuda.empty_cache() if torch.cuda.is_available() else None
    if strong is not None:
        strong.update(paths_total=args.paths_total, paths_per_gpu=args.paths_total // world,
                      envs_per_path=args.envs, n_gpus=world)
        if upd:
            med = upd[len(upd) // 2]
            strong["committed_updates_to_solve_1gpu"] = upd
            strong["predicted_seconds_to_solve"] = round(med * strong["ms_per_update"] / 1e3, 1)
            strong["prediction"] = ("median committed one-GPU updates-to-solve of this config x the measured strong-"
                                    "scaling ms/update on these n_gpus (the strong run computes the one-GPU run's GA "
                                    "and summed gradient, so it needs the same updates); a prediction, not a measured "
                                    "solve")
        if world == 1 and args.scaling == "weak" and args.per_rank_shapes and args.paths == args.paths_total:
            strong["per_rank"] = per_rank_shapes(args, ctx, tr_numel, upd, ws["ms"])
        rec["strong_scaling"] = strong
    # the metric's second half: one seed observed in this run (one GPU: the bench config; several GPUs: the strong
    # config, whose updates are what more GPUs shorten), plus every committed multi-seed record of this config
    solve_s = args.solve_seconds
    if solve_s is None:
        # one GPU: up to 480 s within a 560 s run (seed 1 needs 34-40 K updates of ~10.6 ms); several: the strong config
        # solves in ~20-40 K updates of a few ms,
        # so up to 300 s within a 480 s run
        cap, budget = (480.0, 560.0) if world == 1 else (300.0, 480.0)
        solve_s = cap if (single or (world > 1 and strong is not None)) else 0.0
        solve_s = max(0.0, min(solve_s, budget - ctx.max_scalar(time.time() - t_start)))
    if solve_s > 0:
        strong_solve = world > 1 and args.scaling == "weak"
        r = in_run_solve(args, ctx, args.dtype, solve_s, paths_total=args.paths_total if strong_solve else head_total)
        if strong_solve:
            rec["strong_scaling"]["in_run_solve"] = r
        else:
            rec["generations_to_solve_in_run"] = r
    if verified is not None:
        rec.setdefault("build", {})["verified"] = verified
    if ctx.is_main:
        rec["generations_to_solve"] = solve_records(key, world, sources)
        if rec.get("generations_to_solve_in_run") is not None:
            rec["generations_to_solve_in_run"]["vs_committed"] = compare_with_committed(
                rec["generations_to_solve_in_run"], rec["generations_to_solve"])
        print(json.dumps(rec), flush=True)
    ctx.destroy()


if __name__ == "__main__":
    main()
