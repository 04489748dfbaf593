"""Command line interface (``python -m pathnet_gym_amd.cli <cmd> ...`` or ``mipath``).

Flag names follow the reference (``doom_pathnet.py:306-361``): --L --M --N
--B --kernel_num --stride_size --log_dir --monitor_dir --worker_hosts_num
--ps_hosts_num --hostname --st_port_num --job_name --task_index.  The
cluster flags are accepted for drop-in compatibility but the topology comes
from ``torch.distributed.run`` (one process per GPU, no parameter server):
``--worker_hosts_num`` maps to the population size.  The RL constants of
``constants.py`` are flags too.

Commands
  train       population-parallel PathNet A2C + GA over the task sequence
  eval        greedy rollouts of every path (or the frozen path) of a checkpoint
  visualize   path-graph PNG of a checkpoint's population (visualize.py)
  supervised  PathNet supervised transfer (MNIST -> SVHN-shaped synthetic data)
  info        print the network / parameter / FLOP summary of a preset
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def build_parser():
    ap = argparse.ArgumentParser(prog="mipath", description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p):
        p.add_argument("--preset", default="pong", help="cartpole-cpu | cartpole | pong | atari4 | reference")
        # reference flags (doom_pathnet.py:309-361)
        p.add_argument("--ps_hosts_num", type=int, default=None, help="accepted, ignored (no parameter server)")
        p.add_argument("--worker_hosts_num", type=int, default=None, help="population size (paths per rank)")
        p.add_argument("--hostname", default=None, help="accepted, ignored (use torchrun --master-addr)")
        p.add_argument("--st_port_num", type=int, default=None, help="accepted, ignored (use --master-port)")
        p.add_argument("--job_name", default=None, help="accepted, ignored (every rank is a worker)")
        p.add_argument("--task_index", type=int, default=None, help="accepted, ignored (RANK env var)")
        p.add_argument("--log_dir", default=None)
        p.add_argument("--monitor_dir", default=None,
                       help="write gym-Monitor-style per-update episode records (envs/monitor.py)")
        p.add_argument("--M", type=int, default=None)
        p.add_argument("--L", type=int, default=None)
        p.add_argument("--N", type=int, default=None)
        p.add_argument("--kernel_num", default=None, help='e.g. "8,4,3"')
        p.add_argument("--stride_size", default=None, help='e.g. "4,2,1"')
        p.add_argument("--fc", default=None, help='linear PathNet layer widths, e.g. "256,256"')
        p.add_argument("--B", type=int, default=None, help="tournament size")
        # framework flags
        p.add_argument("--paths", type=int, default=None, help="paths per rank (weak scaling)")
        p.add_argument("--paths_total", type=int, default=None,
                       help="strong scaling: this fixed population split over the ranks (paths = paths_total / world)")
        p.add_argument("--scaling", default=None, choices=["weak", "strong"],
                       help="strong: --paths_total (default: --paths) is the whole population, split over the ranks")
        p.add_argument("--envs_per_path", type=int, default=None)
        p.add_argument("--tasks", default=None, help='comma list, e.g. "Pong,Breakout"')
        p.add_argument("--backend", default=None, choices=["auto", "hip", "torch"])
        p.add_argument("--seed", type=int, default=None)
        p.add_argument("--use_lstm", type=int, default=None)
        p.add_argument("--trunk_scale", default=None, choices=["M", "none"],
                       help="divide the trunk output by M (reference FF net) or not (reference LSTM net)")
        p.add_argument("--no_graph", action="store_true")
        p.add_argument("--compute_dtype", default=None, choices=["bf16", "fp32", "fp32x"],
                       help="HIP engine operand precision: fp32 (fp32 MFMA operands, csrc/trunk_f32.hip, bit-"
                            "reproducible), fp32x (fp32-accurate fp16 hi+lo pairs, csrc/trunk_x3.hip + lstm_x3.hip, "
                            "< 2e-5 per layer vs a float64 truth), bf16")
        p.add_argument("--deterministic", type=int, default=None,
                       help="1: fixed-order gradient reductions (bit-reproducible updates)")
        # RL constants (constants.py)
        p.add_argument("--t_max", type=int, default=None)
        p.add_argument("--gamma", type=float, default=None)
        p.add_argument("--gae_lambda", type=float, default=None)
        p.add_argument("--entropy_beta", type=float, default=None)
        p.add_argument("--lr", type=float, default=None)
        p.add_argument("--lr_anneal", default=None, choices=["per_task", "global", "none"])
        p.add_argument("--rmsp_alpha", type=float, default=None)
        p.add_argument("--rmsp_epsilon", type=float, default=None)
        p.add_argument("--grad_norm_clip", type=float, default=None)
        p.add_argument("--max_time_step", type=int, default=None)
        p.add_argument("--env_reduction", default=None, choices=["sum", "mean_env"])
        p.add_argument("--rank_reduction", default=None, choices=["sum", "mean"])
        p.add_argument("--grad_scale", type=float, default=None)
        p.add_argument("--mutation", default=None, choices=["ref", "down"])
        p.add_argument("--concurrent_tournaments", type=int, default=None)
        p.add_argument("--freeze_union", type=int, default=None)
        p.add_argument("--gray", default=None, choices=["rgb", "bgr"])
        p.add_argument("--frameskip", type=int, default=None)
        p.add_argument("--ga_sync", default=None, choices=["fused", "gather_bcast"])
        p.add_argument("--ga_backend", default=None, choices=["host", "device"],
                       help="host: reference MT19937 GA; device: counter-hash GA kernel inside the update graph")
        p.add_argument("--fitness", default=None, choices=["last", "mean"],
                       help="last: latest episode return (reference); mean: mean over a window of episodes")
        p.add_argument("--fitness_window", type=int, default=None, help="episodes per tournament entry (0 = envs)")
        p.add_argument("--check_every", type=int, default=None, help="replica-consistency check interval (updates)")
        p.add_argument("--max_nonfinite", type=int, default=None, help="consecutive skipped non-finite updates")
        p.add_argument("--watchdog_s", type=float, default=None, help="abort if an update hangs this long")
        p.add_argument("--trace", default=None, help="write a Chrome trace of update phases to this path")

    t = sub.add_parser("train")
    common(t)
    t.add_argument("--steps_per_task", type=int, default=None, help="agent steps per task (all ranks)")
    t.add_argument("--max_updates", type=int, default=None)
    t.add_argument("--checkpoint", default=None, help="checkpoint path written at task ends / every --checkpoint_every")
    t.add_argument("--checkpoint_every", type=int, default=0, help="updates between checkpoints")
    t.add_argument("--resume", default=None)
    t.add_argument("--init_from_tf", default=None,
                   help="reference tf.train.Saver checkpoint prefix (model.ckpt-N) to start from (utils/tf_checkpoint.py)")
    t.add_argument("--graphs", action="store_true", help="dump path-graph PNGs per tournament (visualize.py)")

    e = sub.add_parser("eval")
    common(e)
    e.add_argument("--checkpoint", required=True)
    e.add_argument("--episodes", type=int, default=1)
    e.add_argument("--max_steps", type=int, default=2000)

    v = sub.add_parser("visualize")
    v.add_argument("--checkpoint", required=True)
    v.add_argument("--out", default="./data/graphs/population.png")

    s = sub.add_parser("supervised")
    s.add_argument("--tasks", default="mnist,svhn")
    s.add_argument("--generations", type=int, default=50)
    s.add_argument("--population", type=int, default=64)
    s.add_argument("--B", type=int, default=2)
    s.add_argument("--L", type=int, default=3)
    s.add_argument("--M", type=int, default=10)
    s.add_argument("--N", type=int, default=3)
    s.add_argument("--width", type=int, default=20)
    s.add_argument("--arch", default="fc", choices=["fc", "conv"], help="fc: module2 FC modules; conv: conv_module")
    s.add_argument("--train_size", type=int, default=4096, help="training samples per task")
    s.add_argument("--train_sizes", default="", help="per-task training-set sizes, e.g. 4096,256 (overrides --train_size)")
    s.add_argument("--frozen_mode", default="or", choices=["or", "available"],
                   help="or: frozen modules always expressed (reference RL semantics); available: selectable by later paths")
    s.add_argument("--clip", type=float, default=5.0, help="global gradient-norm clip per SGD step (0: off)")
    s.add_argument("--standardize", type=int, default=1, help="per-task per-channel input standardisation")
    s.add_argument("--task_generations", default="",
                   help="per-task generation budgets, e.g. 50,10 (overrides --generations)")
    s.add_argument("--eval_every", type=int, default=0,
                   help="held-out accuracy of the best path every K generations of the last task and the control")
    s.add_argument("--steps_per_gen", type=int, default=50)
    s.add_argument("--batch", type=int, default=16)
    s.add_argument("--lr", type=float, default=0.05)
    s.add_argument("--seed", type=int, default=1)
    s.add_argument("--device", default=None)
    s.add_argument("--control", action="store_true", help="also learn the last task from scratch (transfer check)")
    s.add_argument("--paired_control", type=int, default=1,
                   help="1: the control replays the transfer run's last-task random streams (same init, head, "
                        "minibatches, GA draws): only the frozen source modules differ; 0: independent seed")
    s.add_argument("--target_accuracy", type=float, default=0.9)
    s.add_argument("--log_dir", default=None)

    i = sub.add_parser("info")
    i.add_argument("--preset", default="pong")
    return ap


def config_from_args(a):
    from .config import LayerSpec, preset, reference_pixel_layers
    cfg = preset(a.preset)
    net = cfg.net
    rebuild = False
    if a.L is not None:
        net.L = a.L
        rebuild = True
    if a.M is not None:
        net.M = a.M
    if a.N is not None:
        net.N = a.N
    if a.kernel_num or a.stride_size or a.fc or rebuild:
        if net.layers and net.layers[0].kind == "conv":
            ks = tuple(int(x) for x in (a.kernel_num or "8,4,3").split(","))
            ss = tuple(int(x) for x in (a.stride_size or "4,2,1").split(","))
            fc = tuple(int(x) for x in (a.fc or ",".join(str(l.out) for l in net.layers if l.kind == "fc")).split(","))
            net.layers = reference_pixel_layers(net.L, ks, ss, fc=fc)
        elif a.fc:
            net.layers = [LayerSpec("fc", int(x)) for x in a.fc.split(",")]
        net.L = len(net.layers)
    if a.use_lstm is not None:
        net.use_lstm = bool(a.use_lstm)
        if net.use_lstm:
            net.trunk_scale = "none"
    if getattr(a, "trunk_scale", None):
        net.trunk_scale = a.trunk_scale
    if a.B is not None:
        cfg.ga.B = a.B
    pop = a.paths if a.paths is not None else a.worker_hosts_num
    if pop is not None:
        cfg.paths = pop
    if getattr(a, "paths_total", None):
        cfg.paths_total = a.paths_total
    elif getattr(a, "scaling", None) == "strong":
        cfg.paths_total = cfg.paths
    for k in ("envs_per_path", "backend", "seed", "log_dir", "gray", "frameskip"):
        v = getattr(a, k, None)
        if v is not None:
            setattr(cfg, k, v)
    if a.tasks:
        cfg.tasks = [t.strip() for t in a.tasks.split(",")]
        cfg.env = cfg.tasks[0]
        net.num_tasks = len(cfg.tasks)
    for k, attr in (("t_max", "t_max"), ("gamma", "gamma"), ("gae_lambda", "gae_lambda"),
                    ("entropy_beta", "entropy_beta"), ("lr", "lr"), ("lr_anneal", "lr_anneal"),
                    ("rmsp_alpha", "rmsp_alpha"), ("rmsp_epsilon", "rmsp_epsilon"),
                    ("grad_norm_clip", "grad_norm_clip"), ("max_time_step", "max_time_step"),
                    ("env_reduction", "env_reduction"), ("rank_reduction", "rank_reduction"),
                    ("grad_scale", "grad_scale")):
        v = getattr(a, k, None)
        if v is not None:
            setattr(cfg.a2c, attr, v)
    if a.mutation is not None:
        cfg.ga.mutation = a.mutation
    if a.concurrent_tournaments is not None:
        cfg.ga.concurrent_tournaments = a.concurrent_tournaments
    if a.freeze_union is not None:
        cfg.ga.freeze_union = bool(a.freeze_union)
    if getattr(a, "no_graph", False):
        cfg.use_graph = False
    if getattr(a, "compute_dtype", None):
        cfg.compute_dtype = a.compute_dtype
    if getattr(a, "deterministic", None) is not None:
        cfg.deterministic = bool(a.deterministic)
    if getattr(a, "ga_sync", None):
        cfg.ga_sync = a.ga_sync
    if getattr(a, "steps_per_task", None):
        cfg.steps_per_task = a.steps_per_task
    if getattr(a, "ga_backend", None):
        cfg.ga.backend = a.ga_backend
    if getattr(a, "fitness", None):
        cfg.ga.fitness = a.fitness
    if getattr(a, "fitness_window", None) is not None:
        cfg.ga.fitness_window = a.fitness_window
    for k in ("check_every", "max_nonfinite", "watchdog_s"):
        if getattr(a, k, None) is not None:
            setattr(cfg, k, getattr(a, k))
    if getattr(a, "trace", None):
        cfg.trace_path = a.trace
    cfg.net.__post_init__()
    return cfg


def cmd_train(a):
    import torch
    from .algo.trainer import PathNetTrainer
    from .parallel.dist import init_distributed
    from .utils import checkpoint as ckpt
    from .utils.metrics import MetricsLogger
    cfg = config_from_args(a)
    ctx = init_distributed()
    if cfg.backend in ("auto", "hip") and ctx.device.type == "cuda":
        from . import _build
        _build.build()
    log_dir = (cfg.log_dir or "./data/tensorboard/") + str(int(time.time()))   # doom_pathnet.py:300
    logger = MetricsLogger(os.path.join(log_dir, f"events.rank{ctx.rank}.jsonl"), echo=ctx.is_main,
                           tensorboard_dir=log_dir if ctx.is_main else None)
    tr = PathNetTrainer(cfg, device=ctx.device, ctx=ctx, logger=logger)
    if a.resume:
        ckpt.load(tr, a.resume)
    if getattr(a, "init_from_tf", None):
        from .utils.tf_checkpoint import import_reference_checkpoint
        info = import_reference_checkpoint(tr, a.init_from_tf)
        logger.log("tf_import", **{k: v for k, v in info.items() if k != "genotypes"})
    if a.graphs and ctx.is_main:
        from .utils.visualize import GraphVisualize
        tr.visualizer = GraphVisualize([cfg.net.M] * cfg.net.L, out_dir=os.path.join(log_dir, "graphs"))
    if getattr(a, "monitor_dir", None):
        from .envs.monitor import UpdateMonitor
        tr.monitor = UpdateMonitor(a.monitor_dir, rank=ctx.rank)
    logger.log("config", config=json.loads(cfg.to_json()), world=ctx.world, backend=tr.backend)
    solved = tr.train(max_updates=a.max_updates, checkpoint=a.checkpoint, checkpoint_every=a.checkpoint_every)
    if a.checkpoint:
        ckpt.save(tr, a.checkpoint)
    logger.log("done", global_step=tr.global_step, generations=tr.pop.generation, solved_generation=solved)
    logger.close()
    ctx.destroy()


def cmd_eval(a):
    from .algo.evaluate import evaluate_checkpoint
    cfg = config_from_args(a)
    res = evaluate_checkpoint(cfg, a.checkpoint, episodes=a.episodes, max_steps=a.max_steps)
    print(json.dumps(res))


def cmd_visualize(a):
    from safetensors.torch import load_file
    from .utils.visualize import GraphVisualize
    d = load_file(a.checkpoint)
    g = d["ga.genotypes"].numpy()
    fr = d["ga.frozen"].numpy()
    P, L, M = g.shape
    vis = GraphVisualize([M] * L, out_dir=os.path.dirname(os.path.abspath(a.out)))
    from .algo.ga import decode_path
    if fr.any():
        vis.set_fixed(decode_path(fr), "r")
    path = vis.show([decode_path(x) for x in g], "m", filename=a.out)
    print(path)


def cmd_supervised(a):
    from .algo.supervised import run_supervised_transfer
    res = run_supervised_transfer(a)
    print(json.dumps(res))


def cmd_info(a):
    from .config import preset
    from .models.pathnet import count_params, forward_flops_per_sample
    cfg = preset(a.preset)
    n = cfg.net
    print(json.dumps({"preset": a.preset, "layers": [(l.kind, l.out, l.kernel, l.stride) for l in n.layers],
                      "shapes": [list(map(list, s[:2])) for s in n.layer_shapes()], "params": count_params(n),
                      "fwd_mflop_dense": forward_flops_per_sample(n) / 1e6,
                      "fwd_mflop_N_active": forward_flops_per_sample(n, [n.N] * n.L) / 1e6}))


def main(argv=None):
    a = build_parser().parse_args(argv)
    {"train": cmd_train, "eval": cmd_eval, "visualize": cmd_visualize, "supervised": cmd_supervised,
     "info": cmd_info}[a.cmd](a)


if __name__ == "__main__":
    main()
