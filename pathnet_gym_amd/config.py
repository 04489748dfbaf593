"""Configuration: reference hyper-parameters + MI355X presets.

Reference defaults live in ``constants.py`` (module-level constants) and the
argparse flags of ``doom_pathnet.py:306-361``.  Here they are one dataclass
tree so a run is fully described by one object (and one JSON blob in the
checkpoint).  Every field cites where its default comes from.
"""
from __future__ import annotations

import dataclasses
import json
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# Reference constants (ref constants.py:4-32)
# ---------------------------------------------------------------------------
LOCAL_T_MAX = 20                 # constants.py:4
RMSP_ALPHA = 0.99                # constants.py:5
RMSP_EPSILON = 0.1               # constants.py:6
CHECKPOINT_DIR = "checkpoints"   # constants.py:7 (unused by the reference)
INITIAL_ALPHA_LOW = 1e-4         # constants.py:8
INITIAL_ALPHA_HIGH = 1e-2        # constants.py:9
PARALLEL_SIZE = 8                # constants.py:11 (unused by the reference)
ROMZ = ["MsPacman-v0", "Alien-v0"]   # constants.py:14
ACTION_SIZEZ = [9, 18]               # constants.py:15
ACTION_SPACE_TYPE = "full"           # constants.py:16
INITIAL_ALPHA_LOG_RATE = 0.4226      # constants.py:24
GAMMA = 0.99                         # constants.py:25
ENTROPY_BETA = 0.01                  # constants.py:26
MAX_TIME_STEP = 4 * 10 ** 6          # constants.py:27
GRAD_NORM_CLIP = 40.0                # constants.py:28
USE_LSTM = True                      # constants.py:30
USE_PATHNET = True                   # constants.py:32
FITNESS_PENDING = -1000.0            # doom_pathnet.py:133,248,267 sentinel
PERFORMANCE_LOG_INTERVAL = 1000      # a3c_training_thread.py:23
DEVICE_TASK_STEPS = 2 * 10 ** 9      # per-task horizon for on-device presets (~20 min/GPU at 1.6M frames/s)


def log_uniform(lo: float, hi: float, rate: float) -> float:
    """Geometric interpolation used for lr0 (ref doom_pathnet.py:47-51)."""
    log_lo = math.log(lo)
    log_hi = math.log(hi)
    return math.exp(log_lo * (1 - rate) + log_hi * rate)


@dataclass
class LayerSpec:
    """One PathNet layer = M parallel modules of one kind.

    kind: "conv" (VALID conv, NHWC, TF kernel layout [kh,kw,cin,cout]) or
          "fc" (dense [din,dout]).
    Reference: conv layers ``game_ac_network.py:328-335`` (8 maps each),
    linear layer ``:340-341`` (1408->256).
    """
    kind: str
    out: int                      # output channels (conv) / width (fc) per module
    kernel: int = 1               # conv kernel size (square)
    stride: int = 1               # conv stride
    module_types: Optional[List[int]] = None   # supervised module2 types per module (pathnet.py:137-168)


@dataclass
class PathNetConfig:
    """Super-network topology (ref flags --L --M --N --kernel_num --stride_size)."""
    L: int = 4                                   # doom_pathnet.py:352
    M: int = 10                                  # doom_pathnet.py:350
    N: int = 4                                   # doom_pathnet.py:354
    input_shape: Tuple[int, ...] = (160, 120, 4)  # H,W,C (game_ac_network.py:376)
    layers: List[LayerSpec] = field(default_factory=list)
    # FF net divides the summed trunk output by M (game_ac_network.py:194);
    # LSTM net does not (:394).  "M" | "none".
    trunk_scale: str = "M"
    use_lstm: bool = False
    lstm_size: int = 256                          # game_ac_network.py:397
    num_actions: int = 18                         # max(ACTION_SIZEZ) unified head (:344)
    per_task_heads: bool = False                  # paper semantics (commented at :150-151)
    num_tasks: int = 2

    def __post_init__(self):
        if not self.layers:
            self.layers = reference_pixel_layers(self.L)
        self.L = len(self.layers)
        self.layers = [l if isinstance(l, LayerSpec) else LayerSpec(**l) for l in self.layers]
        self.input_shape = tuple(self.input_shape)

    # ---- derived geometry ----
    def layer_shapes(self):
        """Per layer: (in_shape, out_shape, K (=fan_in), cin) with NHWC shapes."""
        shapes = []
        cur = tuple(self.input_shape)
        for spec in self.layers:
            if spec.kind == "conv":
                H, W, C = cur
                Ho = (H - spec.kernel) // spec.stride + 1
                Wo = (W - spec.kernel) // spec.stride + 1
                if Ho <= 0 or Wo <= 0:
                    raise ValueError(f"conv layer produces empty output from {cur}")
                out = (Ho, Wo, spec.out)
                K = spec.kernel * spec.kernel * C
                shapes.append((cur, out, K, C))
            elif spec.kind == "fc":
                din = int(math.prod(cur))
                out = (spec.out,)
                shapes.append((cur, out, din, din))
            else:
                raise ValueError(spec.kind)
            cur = out
        return shapes

    @property
    def feature_dim(self) -> int:
        return int(math.prod(self.layer_shapes()[-1][1]))

    def to_dict(self):
        return dataclasses.asdict(self)

    @staticmethod
    def from_dict(d):
        d = dict(d)
        d["layers"] = [LayerSpec(**l) for l in d["layers"]]
        return PathNetConfig(**d)


def reference_pixel_layers(L: int = 4, kernels: Sequence[int] = (8, 4, 3),
                           strides: Sequence[int] = (4, 2, 1), maps: int = 8,
                           fc: Sequence[int] = (256,)) -> List[LayerSpec]:
    """Reference trunk: L-1 conv layers (8 maps) + linear PathNet layer(s) of 256.

    ``doom_pathnet.py:356,358`` kernel "8,4,3" stride "4,2,1";
    ``game_ac_network.py:321`` feature_num=[8,8,8]; ``:341`` 256-wide linear.
    """
    nconv = L - len(fc)
    if nconv > len(kernels):
        raise ValueError("reference builder supports at most len(kernel_num) conv layers")
    layers = [LayerSpec("conv", maps, kernels[i], strides[i]) for i in range(nconv)]
    layers += [LayerSpec("fc", w) for w in fc]
    return layers


@dataclass
class A2CConfig:
    t_max: int = LOCAL_T_MAX
    gamma: float = GAMMA
    gae_lambda: float = 1.0            # 1.0 == reference n-step return (a3c_training_thread.py:170-180)
    entropy_beta: float = ENTROPY_BETA
    value_coef: float = 0.5            # 0.5*l2_loss == 0.25*sum(r-v)^2 (game_ac_network.py:56)
    reward_clip: float = 1.0           # a3c_training_thread.py:136
    # loss reduction over envs of one path: "sum" (ref: sum over everything)
    # or "mean_env" (sum over time, mean over the E envs of a path, sum over paths)
    env_reduction: str = "mean_env"
    # gradient reduction over ranks: "sum" (each rank's paths count like the reference's Hogwild workers: the update
    # grows with the population) or "mean" (the all-reduced gradient is divided by the world size, so an 8-GPU
    # update has the scale of a 1-GPU one -- measured: profiles/solve/README.md, "8-GPU population on one GPU")
    rank_reduction: str = "sum"
    grad_scale: float = 1.0            # extra factor on the loss weight (1 / world emulates "mean" on one GPU)
    lr: float = log_uniform(INITIAL_ALPHA_LOW, INITIAL_ALPHA_HIGH, INITIAL_ALPHA_LOG_RATE)
    lr_anneal: str = "per_task"        # "per_task" | "global" (ref quirk) | "none"
    max_time_step: int = MAX_TIME_STEP
    rmsp_alpha: float = RMSP_ALPHA
    rmsp_epsilon: float = RMSP_EPSILON
    rmsp_momentum: float = 0.0
    grad_norm_clip: float = GRAD_NORM_CLIP


@dataclass
class GAConfig:
    B: int = 3                          # doom_pathnet.py:360 (paper: 2)
    mutation: str = "ref"               # "ref" (pathnet.py:50-63) | "down" (pathnet.py:32-48)
    concurrent_tournaments: int = 1     # 1 == reference single tournament at a time
    fitness: str = "last"               # "last" episode return (ref) | "mean" over a window of episodes
    fitness_window: int = 0             # "mean": episodes per tournament entry (0 = envs_per_path)
    freeze_union: bool = True           # keep union of frozen paths across tasks (paper); False = ref quirk
    backend: str = "host"               # "host": reference MT19937 GA | "device": counter-hash GA kernel in the graph
    seed: int = 1                       # doom_pathnet.py:104 tf.set_random_seed(1)

    def window_for(self, envs_per_path: int) -> int:
        """Episodes a path must finish before it can enter a tournament (0 = reference 'last episode')."""
        if self.fitness != "mean":
            return 0
        return self.fitness_window if self.fitness_window > 0 else max(1, envs_per_path)


@dataclass
class TrainConfig:
    env: str = "Pong"
    tasks: List[str] = field(default_factory=lambda: ["Pong"])
    paths: int = 64                     # paths per rank (weak scaling: the population grows with the ranks)
    # strong scaling: a FIXED population of paths_total paths split over the ranks (paths = paths_total / world).
    # Envs and action sampling are keyed by the global env index (VecEnv.set_id_base, heads row_base) and the
    # GA and the summed gradient run over the same P_total, so any world size computes the one-GPU run of the
    # same seed -- more GPUs shorten each update instead of growing it.  0 = weak scaling (``paths`` per rank)
    paths_total: int = 0
    envs_per_path: int = 16
    net: PathNetConfig = field(default_factory=PathNetConfig)
    a2c: A2CConfig = field(default_factory=A2CConfig)
    ga: GAConfig = field(default_factory=GAConfig)
    backend: str = "auto"               # "hip" | "torch" | "auto"
    # HIP engine operand precision: "bf16" (bf16/fp16 MFMA operands, fp32 accumulation + master weights) or
    # "fp32" (fp32 activations and operands on v_mfma_f32_16x16x4_f32, csrc/trunk_f32.hip) -- the reference
    # computes in fp32 (game_ac_network.py:89-110)
    compute_dtype: str = "bf16"
    # fixed-order gradient reductions everywhere (no fp32 atomics): one seed reproduces every update bit for
    # bit.  Always on with compute_dtype="fp32"; in bf16 it routes the weight gradients through the ordered
    # fp32 kernels (slower: see docs/PERF.md)
    deterministic: bool = False
    use_graph: bool = True
    frame_ring: bool = False            # HIP Pong: single-frame ring instead of packed stacks (runtime/engine.py).
                                        # bf16: 13.06 vs 12.73 ms/update (the conv1 planar loads cost more than the
                                        # env saves); fp32x: 11.15 vs 11.42 ms (LDS-staged first layer, bench default)
    # HIP engine rollout: the population is stepped as this many path groups on their own HIP streams (one
    # branch each inside the rollout hipGraph) so one group's latency-bound fc / heads launches can overlap
    # the other group's env / conv1 launches (runtime/engine.py; packed-stack pixel envs without LSTM).
    # Bit-identical to one stream.  Measured at the bench shape: 9.70 (1) vs 10.00 (2) vs 10.81 (4) ms per
    # update -- every rollout kernel already fills the GPU -- so 0 (auto) = 1.
    rollout_groups: int = 0
    seed: int = 1
    log_dir: str = "./data/tensorboard/"
    steps_per_task: int = MAX_TIME_STEP
    checkpoint_every: int = 0
    frameskip: int = 4
    gray: str = "rgb"                   # "rgb" luma | "bgr" (reference cv2.COLOR_BGR2GRAY on RGB quirk)
    # failure / race detection and tracing (runtime/guard.py, runtime/consistency.py, utils/tracing.py)
    check_every: int = 0                # replica-consistency check interval in updates (0 = off)
    max_nonfinite: int = 3              # consecutive non-finite updates tolerated (skipped) before raising
    watchdog_s: float = 0.0             # abort if no update completes for this long (0 = off)
    trace_path: Optional[str] = None    # Chrome-trace JSON of update phases
    # HIP engine + device GA: overlap the host bookkeeping of update u-1 with the GPU work of update u
    # (stats / tournament events are reported one update late; flush() drains the last one)
    pipeline: bool = True
    # multi-rank HIP engine: all-reduce everything but the first layer's gradient while that layer's weight-gradient
    # kernel runs (two async buckets, parallel/comm.py); False = one bucket after the whole backward
    overlap_allreduce: bool = True
    # gc.freeze() once the trainer is built (algo/trainer.py): the objects of the setup leave the cyclic collector, whose
    # full collections otherwise stall the pipelined update loop by tens of ms every ~70 updates
    gc_freeze: bool = True

    def to_json(self):
        return json.dumps(dataclasses.asdict(self))

    @staticmethod
    def from_json(s):
        d = json.loads(s)
        d["net"] = PathNetConfig.from_dict(d["net"])
        d["a2c"] = A2CConfig(**d["a2c"])
        d["ga"] = GAConfig(**d["ga"])
        return TrainConfig(**d)


# ---------------------------------------------------------------------------
# Presets (BASELINE.json configs)
# ---------------------------------------------------------------------------
def preset(name: str) -> TrainConfig:
    name = name.lower()
    if name in ("cartpole-cpu", "cartpole_cpu"):
        # BASELINE config 1: CartPole-v1, L=2 x N=4 MLP PathNet, binary tournament, CPU
        net = PathNetConfig(L=2, M=4, N=2, input_shape=(4,),
                            layers=[LayerSpec("fc", 32), LayerSpec("fc", 32)],
                            trunk_scale="none", num_actions=2)
        return TrainConfig(env="CartPole-v1", tasks=["CartPole-v1"], paths=4, envs_per_path=8,
                           net=net, ga=GAConfig(B=2), backend="torch", compute_dtype="fp32",
                           use_graph=False, a2c=A2CConfig(t_max=5, lr=7e-3, lr_anneal="none"))
    if name == "cartpole":
        # BASELINE config 2: 64 path-parallel A2C workers on one MI355X, bf16
        net = PathNetConfig(L=2, M=4, N=2, input_shape=(4,),
                            layers=[LayerSpec("fc", 32), LayerSpec("fc", 32)],
                            trunk_scale="none", num_actions=2)
        return TrainConfig(env="CartPole-v1", tasks=["CartPole-v1"], paths=64, envs_per_path=16,
                           net=net, ga=GAConfig(B=2), a2c=A2CConfig(t_max=5, lr=7e-3, lr_anneal="none"))
    if name == "pong":
        # BASELINE config 3 (headline): Pong pixels, L=3 conv + 2 fc x M=10 modules, N=4 (doom_pathnet.py:354).
        # Two choices make it learn (profiles/solve/ablation_r2/README.md):
        #  * GA fitness = mean return of the last E episodes of a path (window = envs per path): a path
        #    enters a tournament about once per episode of each of its E envs, the timescale of a reference
        #    worker that plays one env (a "last episode" fitness made tournaments E x more frequent and the
        #    mutated copies of the winner churned every path's modules before anything was learned);
        #  * no /M on the trunk output: the reference's default network (USE_LSTM=True, constants.py:30)
        #    does not divide by M (game_ac_network.py:394); only its FF variant does (:194).
        net = PathNetConfig(L=5, M=10, N=4, input_shape=(160, 120, 4),
                            layers=reference_pixel_layers(5, fc=(256, 256)),
                            trunk_scale="none", num_actions=6)
        # MAX_TIME_STEP (4e6, constants.py:27) is ~17 h of the reference's 63 steps/s but only ~2.5 s
        # at on-device throughput, so the per-task anneal horizon is sized in frames for this engine.
        return TrainConfig(env="Pong", tasks=["Pong"], paths=64, envs_per_path=32, net=net,
                           ga=GAConfig(B=3, fitness="mean"), steps_per_task=DEVICE_TASK_STEPS,
                           a2c=A2CConfig(max_time_step=DEVICE_TASK_STEPS))
    if name in ("atari4", "atari-suite"):
        # BASELINE config 5: 4-task suite with unified 18-way head (same GA fitness / trunk scale as "pong")
        net = PathNetConfig(L=5, M=10, N=4, input_shape=(160, 120, 4),
                            layers=reference_pixel_layers(5, fc=(256, 256)),
                            trunk_scale="none", num_actions=18, num_tasks=4)
        return TrainConfig(env="Pong", tasks=["Pong", "Breakout", "SpaceInvaders", "Alien"],
                           paths=64, envs_per_path=32, net=net, steps_per_task=DEVICE_TASK_STEPS,
                           ga=GAConfig(B=3, fitness="mean"),
                           a2c=A2CConfig(max_time_step=DEVICE_TASK_STEPS))
    if name in ("reference", "ref"):
        # the reference's own default network and experiment: L=4 (3 conv + 1 linear 1408->256), M=10, N=4,
        # BasicLSTMCell(256) (USE_LSTM=True, constants.py:30; game_ac_network.py:303-521), 18-way head
        # (ACTION_SIZEZ, constants.py:15), LOCAL_T_MAX=20 (constants.py:4), Alien -> Centipede
        # (aliencentipede.txt:55-93).  The reference's 9 one-env workers become 64 paths x 16 envs, the HIP
        # engine's shape (runtime/engine.py, csrc/lstm.hip); the same GA fitness as "pong" (mean of the last E).
        net = PathNetConfig(L=4, M=10, N=4, use_lstm=True, trunk_scale="none", num_actions=18)
        return TrainConfig(env="Alien", tasks=["Alien", "Centipede"], paths=64, envs_per_path=16, net=net,
                           ga=GAConfig(B=3, fitness="mean"), steps_per_task=DEVICE_TASK_STEPS,
                           a2c=A2CConfig(t_max=20, max_time_step=DEVICE_TASK_STEPS))
    raise KeyError(name)
