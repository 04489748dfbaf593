"""fp32x engine mode (split-bf16 operands, csrc/trunk_x3.hip) on an MI355X.

The reference computes in fp32 (TF default dtype, game_ac_network.py:89-110).  The fp32x mode keeps every activation
as a (hi, lo) bf16 pair and every product as three bf16 MFMAs; it must match a PLAIN fp32 PyTorch oracle to <= 2e-5
relative per layer (forward and whole-update gradient), and a gradient wiring error of 2 % in a single module must
be detected by the same comparison.
"""
import numpy as np
import pytest
import torch

from pathnet_gym_amd.algo.a2c_math import a2c_loss, nstep_returns
from pathnet_gym_amd.algo.ga import get_geopath
from pathnet_gym_amd.config import LayerSpec, PathNetConfig, preset
from pathnet_gym_amd.models.acnet import ACPathNet
from pathnet_gym_amd.models.pathnet import ParamStore, heads_ref, trunk_forward_ref
from pathnet_gym_amd.ops.pathnet_ops import x2_alloc, x2_lo, x2_value

pytestmark = pytest.mark.gpu
DEV = "cuda"
X3_LAYER_TOL = 2e-5


def rel(a, b):
    a = a.double().flatten()
    b = b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-12))


def masks_with_edges(P, L, M, N, seed=0):
    rng = np.random.RandomState(seed)
    m = np.stack([get_geopath(L, M, N, rng) for _ in range(P)])
    m[0, 1, :] = 0          # empty layer
    m[1, :, :] = 1          # every module active: 5 column tiles -> two LDS passes per layer
    m[2, 0, :] = 0
    m[2, 0, M - 1] = 1      # one (odd) module
    return m


def pixel_cfg(scale="M"):
    return PathNetConfig(L=5, M=10, N=4, input_shape=(160, 120, 4),
                         layers=[LayerSpec("conv", 8, 8, 4), LayerSpec("conv", 8, 4, 2), LayerSpec("conv", 8, 3, 1),
                                 LayerSpec("fc", 256), LayerSpec("fc", 256)],
                         trunk_scale=scale, num_actions=6)


def test_x2_pair_helpers(hip_lib):
    t = x2_alloc((3, 5), DEV)
    assert x2_lo(t) == 15 and x2_lo(t[1]) == 15
    v = torch.rand(3, 5, device=DEV)
    full = torch.empty(0, dtype=torch.float16, device=DEV).set_(t.untyped_storage(), 0, (2, 3, 5), (15, 5, 1))
    hi = v.half()
    full[0].copy_(hi)
    full[1].copy_((v - hi.float()).half())
    assert rel(x2_value(t), v) < 1e-6
    with pytest.raises(ValueError):
        x2_lo(torch.zeros(4, dtype=torch.float16, device=DEV)[:1].expand(4))


def test_x3_weight_pairs_reconstruct_fp32(hip_lib):
    cfg = pixel_cfg()
    m = ACPathNet(cfg, 2, DEV, "hip", seed=5, compute_dtype="fp32x")
    hp = m.hip
    st = m.store
    flat = st.flat.detach()
    for l, g in enumerate(hp.geoms):
        W = flat[g.w_off:g.w_off + hp.M * g.chunk].view(hp.M, g.chunk)[:, :g.K * g.Cout].view(hp.M, g.K, g.Cout)
        pair = hp.Wc[l].float()
        rec = (pair[0] + pair[1])[:, :, :g.K].transpose(1, 2)
        # forward copy and WcT (fc input gradient): fp16 pairs of W * 2^8 (22 significant bits)
        rec = rec / 256.0
        assert rel(rec, W) < 1e-7, (l, rel(rec, W))
        if hp.WcT[l] is not None:
            pt = hp.WcT[l].float()
            assert hp.WcT[l].dtype == torch.float16
            assert rel((pt[0] + pt[1])[:, :g.K] / 256.0, W) < 1e-7
            # the third piece (X3_DG_W3 input gradients): hi + lo + third == W to fp32 accuracy (exact but for
            # weights below ~2^-13, whose third piece is an fp16 subnormal)
            p3 = hp.WcT[l].double()
            assert rel((p3[0] + p3[1] + p3[2])[:, :g.K] / 256.0, W.double()) < 3e-9
    assert int(hp.x3_status.item()) == 0


def test_x3_trunk_forward_matches_plain_fp32_oracle(hip_lib):
    cfg = pixel_cfg()
    P, E = 4, 16
    m = ACPathNet(cfg, P, DEV, "hip", seed=3, compute_dtype="fp32x")
    m.set_paths(masks_with_edges(P, cfg.L, cfg.M, cfg.N))
    assert m.hip.x3 and m.hip.Wc[1].shape[0] == 2
    g = torch.Generator(device="cpu").manual_seed(0)
    obs = torch.randint(0, 256, (P * E, 160, 120, 4), generator=g, dtype=torch.uint8).to(DEV)
    feat = m.hip.trunk(obs, E)
    with torch.no_grad():
        ref = trunk_forward_ref(m.store, obs.float() / 255.0, m.mask.repeat_interleave(E, 0))
    errs = []
    for p in range(P):
        sl = slice(p * E, (p + 1) * E)
        if ref[sl].norm() == 0:
            assert feat[sl].norm() == 0, p
            continue
        errs.append(rel(feat[sl], ref[sl]))
    print("fp32x trunk forward vs fp32 oracle, per path:", [f"{e:.2e}" for e in errs])
    assert max(errs) < X3_LAYER_TOL, errs


def _oracle_grad(tr, eng, dtype=torch.float32):
    """Autograd of the A2C loss over the engine's stored rollout: plain fp32, or float64 (the truth the fp32x engine
    and the plain fp32 oracle are both measured against)."""
    cfg = tr.cfg
    T, B = eng.T, eng.B
    a2c = cfg.a2c
    flat = tr.model.store.flat.detach().clone().to(dtype).requires_grad_(True)
    st = ParamStore(cfg.net, DEV, flat=flat)
    x = eng.obs_stacks().reshape((T + 1) * B, 160, 120, 4).to(dtype) / 255.0
    mask = tr.model.mask.repeat_interleave(eng.E, 0).repeat(T + 1, 1, 1).to(dtype)
    feat = trunk_forward_ref(st, x, mask)
    logits, values = heads_ref(st, feat)
    assert rel(logits[:T * B], eng.logits[:T].reshape(-1, eng.A)) < 1e-5
    assert rel(values, eng.values[:T + 1].reshape(-1)) < 1e-5
    R, adv = nstep_returns(eng.rewards, eng.values[:T], eng.dones.bool(), eng.values[T], a2c.gamma,
                           a2c.gae_lambda, a2c.reward_clip)
    loss, _, _, _ = a2c_loss(logits[:T * B], values[:T * B], eng.actions[:T].reshape(-1).long(),
                             R.reshape(-1).to(dtype), adv.reshape(-1).to(dtype), a2c.entropy_beta, a2c.value_coef,
                             torch.full((T * B,), eng.weight, device=DEV, dtype=dtype))
    loss.backward()
    return flat.grad


def _oracles(fn, tr, eng):
    """(float64 truth, plain fp32 oracle) of one stored rollout."""
    return fn(tr, eng, torch.float64), fn(tr, eng, torch.float32)


def check_layers(label, tr, g_hip, g64, g32, tol=lambda k: X3_LAYER_TOL):
    """Per-layer budget against the float64 truth: < 2e-5, or -- on a layer whose gradient is ill-conditioned in the
    forward values (the policy head: the A2C policy gradient cancels across samples, so the 1e-7 differences between
    any fp32 forward and the float64 forward come back amplified) -- no worse than 1.25x the plain fp32 oracle's own
    error against that truth.  Every number is printed."""
    e64 = layer_errors(tr, g_hip, g64)
    o32 = layer_errors(tr, g32, g64)
    e32 = layer_errors(tr, g_hip, g32)
    print(f"{label} per layer: vs float64", {k: f"{v:.2e}" for k, v in e64.items()},
          "| plain fp32 oracle vs float64", {k: f"{v:.2e}" for k, v in o32.items()},
          "| fp32x vs plain fp32", {k: f"{v:.2e}" for k, v in e32.items()})
    for k, v in e64.items():
        assert v < max(tol(k), 1.25 * o32[k]), (k, v, o32[k])
    return e64


def layer_errors(tr, g_hip, g_ref):
    parts = {}
    for s in tr.model.store.layout.segments:
        key = s.layer if s.layer >= 0 else s.name.split(".")[0]
        parts.setdefault(key, []).append((g_hip[s.offset:s.offset + s.numel], g_ref[s.offset:s.offset + s.numel]))
    return {k: rel(torch.cat([a for a, _ in v]), torch.cat([b for _, b in v])) for k, v in parts.items()}


@pytest.fixture(scope="module")
def x3_rollout(hip_lib):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.compute_dtype = "fp32x"
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    assert tr.compute_dtype == "fp32x" and eng.acts[-1].dtype == torch.float32 and not eng.ring
    tr.env.max_episode_steps = 5
    tr.update()
    tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    return (tr, eng, *_oracles(_oracle_grad, tr, eng), eng.grad_flat.clone())


def test_x3_engine_gradient_vs_plain_fp32_oracle(x3_rollout):
    tr, eng, g_ref, g32, g_hip = x3_rollout
    check_layers("fp32x engine", tr, g_hip, g_ref, g32)


def test_x3_gradient_check_detects_a_two_percent_module_error(x3_rollout):
    """Negative control: one active module's weight gradient scaled by 1.02 must fail the per-layer budget."""
    tr, eng, g_ref, _, g_hip = x3_rollout
    hp = tr.model.hip
    for l, g in enumerate(hp.geoms):
        act = np.nonzero(tr.model.mask[0, l].cpu().numpy() > 0.5)[0]
        j = int(act[0]) if len(act) else int(np.nonzero(tr.model.mask[1, l].cpu().numpy() > 0.5)[0][0])
        bad = g_hip.clone()
        seg = slice(g.w_off + j * g.chunk, g.w_off + j * g.chunk + g.K * g.Cout)
        bad[seg] *= 1.02
        err = layer_errors(tr, bad, g_ref)[l]
        assert err > X3_LAYER_TOL, (l, err)


@pytest.fixture(scope="module")
def x3_ring_rollout(hip_lib):
    """The x3_rollout update with the first layer on the frame ring (engine.frame_ring: T+4 single frames per env;
    csrc/trunk_x3.hip conv1_fwd_band_x2 / conv_wgrad_slab_x3 RING), episode resets inside the rollout."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    assert tr.compute_dtype == "fp32x" and eng.ring
    tr.env.max_episode_steps = 5
    tr.update()
    tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    assert eng.dones.any()
    return (tr, eng, *_oracles(_oracle_grad, tr, eng), eng.grad_flat.clone())


def test_x3_frame_ring_gradient_vs_plain_fp32_oracle(x3_ring_rollout):
    tr, eng, g_ref, g32, g_hip = x3_ring_rollout
    check_layers("fp32x frame-ring engine", tr, g_hip, g_ref, g32)


def test_x3_frame_ring_forward_bit_equal_to_packed(x3_ring_rollout):
    """The ring forward stages the same packed band in LDS as the packed-stack kernel: its outputs and ReLU bits
    must equal the packed kernel's on the reconstructed stacks bit for bit (resets included)."""
    tr, eng, _, _, _ = x3_ring_rollout
    hp = tr.model.hip
    T, B = eng.T, eng.B
    g = hp.geoms[0]
    stacks = eng.obs_stacks(T + 1).contiguous()
    Y = hp.alloc_act(0, (T + 1, B, g.out_feat))
    bits, rows = hp.alloc_bits(0, T + 1, B)
    hp.layer_fwd(0, stacks, Y, bits, eng.P, eng.E, T + 1, 0, rows)
    torch.cuda.synchronize()
    assert rows == eng.bits_rows[0]
    assert torch.equal(x2_value(Y), x2_value(eng.acts[0]))
    # ReLU bits: slots < the path's active-module count (slots past it keep whatever an earlier path set wrote)
    cnt = tr.model.act_cnt.view(eng.P, -1)[:, 0].cpu()
    hw = g.HWo
    for p in range(eng.P):
        for t in range(T + 1):
            r0 = (t * B + p * eng.E) * hw
            k = int(cnt[p])
            assert torch.equal(bits[:k, r0:r0 + eng.E * hw], eng.bits[0][:k, r0:r0 + eng.E * hw]), (p, t)


@pytest.mark.parametrize("E", [16, 32])
@pytest.mark.parametrize("variant", ["split_k", "module_major", "module_major_ks1", "module_major_regs",
                                     "module_major_ks2", "module_major_ks4", "module_major_ks8", "rows16"])
def test_x3_fc_forward_variants_match_path_major(hip_lib, E, variant):
    """fc_fwd_ks_x3 (two waves per module, partial sums meet in LDS), fc_fwd_mm2_x3 (module-major LDS tiles, one or
    two k parts; the two-part form leaves bias / ReLU / bits to fc_slot_sum2_x3) and fc_fwd_mm_x3 (one workgroup per module
    x 64 rows, slot planes summed in slot order) and fc_fwd_x3 in 16-row workgroups (rows16) == the path-major
    fc_fwd_x3 up to summation order: outputs to fp32 rounding, relu bits equal but for exact ties."""
    from pathnet_gym_amd.ops import _lib
    cfg = pixel_cfg()
    P = 5
    m = ACPathNet(cfg, P, DEV, "hip", seed=7, compute_dtype="fp32x")
    m.set_paths(masks_with_edges(P, cfg.L, cfg.M, cfg.N, seed=4))
    hp = m.hip
    g = torch.Generator(device="cpu").manual_seed(2)
    obs = torch.randint(0, 256, (P * E, 160, 120, 4), generator=g, dtype=torch.uint8).to(DEV)
    outs = []
    lib = _lib.lib()
    lib.fast_conv_set_x3_fc_mmv({"module_major_regs": 1, "module_major_ks1": 2}.get(variant, 3))
    # k parts of the two-part module-major form: fixed 2 / 4 / 8, or 0 = auto (8 at these small row counts)
    lib.fast_conv_set_x3_fc_ks_parts(int(variant[-1]) if variant[-3:-1] == "ks" and variant[-1] in "248" else 0)
    hp.fc_fwd_mm_min_k = 0
    for ref in (False, True):
        hp.fc_fwd_mm = variant.startswith("module_major") and not ref
        lib.fast_conv_set_x3_fc_ks(1 if ref or variant.startswith("module_major") or variant == "rows16" else 2)
        # rows16: the path-major kernel in 16-row workgroups (forced) vs 32-row ones
        lib.fast_conv_set_x3_fc_rt1(1 if variant == "rows16" and not ref else 0)
        acts, bits = [], []
        x = obs
        for l, geo in enumerate(hp.geoms):
            Y = hp.alloc_act(l, (1, P * E, geo.out_feat))
            b, rows = hp.alloc_bits(l, 1, P * E)
            hp.layer_fwd(l, x, Y, b, P, E, 1, 0, rows)
            acts.append(Y)
            bits.append(b)
            x = Y
        torch.cuda.synchronize()
        outs.append(([x2_value(a) if a.dtype == torch.float16 else a.clone() for a in acts], [b.clone() for b in bits]))
    hp.fc_fwd_mm = True
    hp.fc_fwd_mm_min_k = 1024
    lib.fast_conv_set_x3_fc_mmv(3)
    lib.fast_conv_set_x3_fc_ks(1)
    lib.fast_conv_set_x3_fc_ks_parts(0)
    lib.fast_conv_set_x3_fc_rt1(2)
    for l in (3, 4):
        a, b = outs[0][0][l], outs[1][0][l]
        assert rel(a, b) < 1e-6, (l, rel(a, b))
        same = (outs[0][1][l] == outs[1][1][l]).float().mean().item()
        assert same > 0.999, (l, same)


def test_x3_backward_side_stream_matches_one_stream(hip_lib, monkeypatch):
    """Small populations run every layer's weight gradient on a side stream (runtime/engine.py _layer_bwd_all): the
    first update's gradient equals the one-stream backward's to fp32 rounding (float atomics in both); the captured
    graphs replay.  (Off by default: measured slower; PATHNET_BWD_STREAMS=2.)"""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    grads = {}
    for mode in ("1", "2"):
        monkeypatch.setenv("PATHNET_BWD_STREAMS", mode)
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 4
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        cfg.ga.backend = "device"
        tr = PathNetTrainer(cfg, device=DEV)
        tr.env.max_episode_steps = 5
        eng = tr.engine
        assert (eng._bwd_side_stream() is not None) == (mode == "2")
        tr.update()                           # eager; the graphs are captured at its end
        torch.cuda.synchronize()
        grads[mode] = eng.grad_flat.clone()
        for _ in range(2):
            tr.update()                       # graph replays
        tr.flush()
        torch.cuda.synchronize()
        assert eng.g_opt is not None and torch.isfinite(tr.model.store.flat).all()
    assert rel(grads["2"], grads["1"]) < 1e-6, rel(grads["2"], grads["1"])


@pytest.mark.parametrize("T", [1, 3])
def test_x3_fused_conv23_forward_bit_equal(hip_lib, T):
    """conv23_fwd_tile_x3 (conv2 + conv3 forward in one launch, csrc/trunk_x3.hip) == two conv_fwd_tile_x3 launches,
    bit for bit: activations (both fp16 planes) and ReLU bits, including a path with every module active (multi-pass
    accumulation through global memory) and a path with an empty layer."""
    cfg = pixel_cfg()
    P, E = 4, 16
    m = ACPathNet(cfg, P, DEV, "hip", seed=11, compute_dtype="fp32x")
    m.set_paths(masks_with_edges(P, cfg.L, cfg.M, cfg.N, seed=6))   # path 1: all 10 modules (multi-pass), path 0: none
    hp = m.hip
    g = torch.Generator(device="cpu").manual_seed(5)
    obs = torch.randint(0, 256, (T * P * E, 160, 120, 4), generator=g, dtype=torch.uint8).to(DEV)
    X0 = hp.alloc_act(0, (T, P * E, hp.geoms[0].out_feat))
    b0, r0 = hp.alloc_bits(0, T, P * E)
    hp.layer_fwd(0, obs, X0, b0, P, E, T, 0, r0)
    outs = []
    for fused in (False, True):
        Y1 = hp.alloc_act(1, (T, P * E, hp.geoms[1].out_feat))
        Y2 = hp.alloc_act(2, (T, P * E, hp.geoms[2].out_feat))
        b1, r1 = hp.alloc_bits(1, T, P * E)
        b2, r2 = hp.alloc_bits(2, T, P * E)
        if fused:
            assert hp.conv23_fwd(1, X0, Y1, b1, r1, Y2, b2, r2, P, E, T, 0)
        else:
            hp.layer_fwd(1, X0, Y1, b1, P, E, T, 0, r1)
            hp.layer_fwd(2, Y1, Y2, b2, P, E, T, 0, r2)
        torch.cuda.synchronize()
        outs.append([x2_value(Y1), x2_value(Y2), b1.clone(), b2.clone(), Y1.clone(), Y2.clone()])
    cnt = m.act_cnt.view(P, -1).cpu()
    for i in (0, 1, 4, 5):
        assert torch.equal(outs[0][i], outs[1][i]), i
    for bi, l, hw in ((2, 1, hp.geoms[1].HWo), (3, 2, hp.geoms[2].HWo)):
        for p in range(P):
            k = int(cnt[p, l])
            for t in range(T):
                r = (t * P * E + p * E) * hw
                assert torch.equal(outs[0][bi][:k, r:r + E * hw], outs[1][bi][:k, r:r + E * hw]), (l, p, t)


@pytest.mark.parametrize("arm", ["swapped", "tile", "tile_pair", "band", "band_pipe"])
@pytest.mark.parametrize("T", [1, 2])
def test_x3_conv_forward_swapped_epilogue_matches_rows_as_a(hip_lib, T, arm):
    """conv_epi_sw (weights as the MFMA A operand: one xor-32 module-pair sum, nibble ReLU bits, 8-byte stores; the
    first layer with fp16(1024 + v) pixels and the offset folded into the bias) == the rows-as-A epilogue: conv2/3
    bit-identical, conv1 to fp32 rounding of the offset sum; ReLU bits equal but for near-zero ties.  T = 2 runs the
    multi-step row walk (backward-style launches), T = 1 the rollout's linear rows.  arm "tile": conv_fwd_tile_x3
    (one sample's input staged in LDS, im2col fragments read from it) against conv_fwd_x3 for conv2/conv3."""
    from pathnet_gym_amd.ops import _lib
    cfg = pixel_cfg()
    P, E = 5, 16
    m = ACPathNet(cfg, P, DEV, "hip", seed=11, compute_dtype="fp32x")
    m.set_paths(masks_with_edges(P, cfg.L, cfg.M, cfg.N, seed=6))
    hp = m.hip
    g = torch.Generator(device="cpu").manual_seed(5)
    obs = torch.randint(0, 256, (T * P * E, 160, 120, 4), generator=g, dtype=torch.uint8).to(DEV)
    lib = _lib.lib()
    outs = []
    for sw in (0, 3):
        if arm == "tile_pair":       # conv2/3 tile: two position tiles per weight-fragment read vs one
            lib.fast_conv_set_x3_fwd_sw(1)
            lib.fast_conv_set_x3_c1_band(1)
            lib.fast_conv_set_x3_fwd_tile(2 if sw else 1)
        elif arm == "band_pipe":     # conv1 band: next k-step's LDS fragments in flight vs one k-step at a time
            lib.fast_conv_set_x3_fwd_sw(1)
            lib.fast_conv_set_x3_fwd_tile(1)
            lib.fast_conv_set_x3_c1_band(1)
            lib.fast_conv_set_x3_c1_pipe(1 if sw else 0)
        elif arm == "band":          # conv1: input band in LDS vs conv1_fwd_x2 (both swapped epilogue, folded offset)
            lib.fast_conv_set_x3_fwd_sw(1)
            lib.fast_conv_set_x3_fwd_tile(1)
            lib.fast_conv_set_x3_c1_band(1 if sw else 0)
        elif arm == "tile":
            lib.fast_conv_set_x3_c1_band(0)
            lib.fast_conv_set_x3_fwd_sw(0)
            lib.fast_conv_set_x3_fwd_tile(1 if sw else 0)
        else:
            lib.fast_conv_set_x3_c1_band(0)
            lib.fast_conv_set_x3_fwd_tile(0)
            lib.fast_conv_set_x3_fwd_sw(sw)
        acts, bits = [], []
        x = obs
        for l in range(3):
            geo = hp.geoms[l]
            Y = hp.alloc_act(l, (T, P * E, geo.out_feat))
            b, rows = hp.alloc_bits(l, T, P * E)
            hp.layer_fwd(l, x, Y, b, P, E, T, 0, rows)
            acts.append(Y)
            bits.append(b)
            x = Y
        torch.cuda.synchronize()
        outs.append(([x2_value(a) for a in acts], [b.clone() for b in bits]))
    lib.fast_conv_set_x3_fwd_sw(1)
    lib.fast_conv_set_x3_fwd_tile(3)         # the default: paired tiles for conv2, single for conv3
    lib.fast_conv_set_x3_c1_band(1)
    lib.fast_conv_set_x3_c1_pipe(0)
    for l in range(3):
        a, b = outs[0][0][l], outs[1][0][l]
        if arm in ("band_pipe", "tile_pair"):   # the same products in the same order
            assert torch.equal(a, b) and torch.equal(outs[0][1][l], outs[1][1][l]), l
        e = rel(b, a)
        same = (outs[0][1][l] == outs[1][1][l]).float().mean().item()
        print(f"layer {l}: rel {e:.2e}, relu-bit bytes equal {same:.6f}")
        assert e < 3e-6, (l, e)
        assert same > 0.999, (l, same)


def test_x3_conv3_wgrad_tile_matches_im2col_rows(x3_rollout):
    """conv_wgrad_tile_x3 (one sample per stage: the input tile converted once, im2col^T read straight from it with
    transposed LDS reads; a path's passes of 4 slots in separate workgroups, blockIdx.z) == conv_wgrad_x3 (32-row
    im2col stages) up to fp32 summation order, weights and biases; the all-modules path runs 3 passes."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, g_hip = x3_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    l = 2
    g = hp.geoms[l]
    seg = slice(g.w_off, g.w_off + hp.M * g.chunk)
    outs = []
    for tile in (0, 1):
        lib.fast_conv_set_x3_wg3_tile(tile)
        eng.grad_flat.zero_()
        hp.layer_bwd(l, eng.acts[l - 1], eng.grads[l], eng.bits[l], eng.grad_flat, eng.grads[l - 1], eng.P, eng.E,
                     eng.T, eng.bits_rows[l])
        torch.cuda.synchronize()
        outs.append(eng.grad_flat[seg].clone())
    lib.fast_conv_set_x3_wg3_tile(1)
    assert outs[0].norm() > 0
    e = rel(outs[1], outs[0])
    print(f"conv3 wgrad tile vs im2col rows: rel {e:.2e}")
    assert e < 1e-6, e
    assert rel(outs[1], g_hip[seg]) < 1e-6


@pytest.mark.parametrize("l", [1, 2, 3, 4])
def test_x3_dgrad_accumulation_variants_match_plain_chain(x3_rollout, l):
    """Input gradients (conv_dgrad_x3 / fc_dgrad_gemm_x3) in the shipped sign-alternating accumulation (FOLD 2: odd
    k-steps on negated operands, summed from zero and subtracted) and with the weights as three fp16 pieces (W3) ==
    the plain MFMA chain up to fp32 rounding; the weight gradient is untouched."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, g_hip = x3_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    g = hp.geoms[l]
    seg = slice(g.w_off, g.w_off + hp.M * g.chunk)
    dxs, gws = [], []
    for fold, w3 in ((0, 0), (2, 0), (0, 1)):
        lib.fast_conv_set_x3_dg_fold(fold)
        lib.fast_conv_set_x3_dg_w3(w3)
        eng.grad_flat.zero_()
        dX = eng.grads[l - 1]
        dX.fill_(float("nan"))
        hp.layer_bwd(l, eng.acts[l - 1], eng.grads[l], eng.bits[l], eng.grad_flat, dX, eng.P, eng.E, eng.T,
                     eng.bits_rows[l])
        torch.cuda.synchronize()
        dxs.append(dX[:eng.T * eng.B].clone())
        gws.append(eng.grad_flat[seg].clone())
    lib.fast_conv_set_x3_dg_fold(2)              # the defaults
    lib.fast_conv_set_x3_dg_w3(0)
    assert dxs[0].norm() > 0
    for name, d, gw in (("fold 2", dxs[1], gws[1]), ("three weight pieces", dxs[2], gws[2])):
        assert torch.isfinite(d).all()
        e = rel(d, dxs[0])
        print(f"layer {l} input gradient, {name} vs plain chain: rel {e:.2e}")
        assert 0 < e < 1e-6, (name, e)
        assert rel(gw, gws[0]) < 1e-6


@pytest.mark.parametrize("l", [1, 2])
def test_x3_dgrad_presplit_staging_bit_equal(x3_rollout, l):
    """conv_dgrad_x3 staging the output gradient's fp16 pair once per position and masking it per slot (X3_PRESPLIT,
    csrc/trunk_x3.hip mask_pair8) == masking the fp32 values and splitting per slot: the split of 0 is (0, 0), so the
    input gradient is bit-identical."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, _ = x3_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    dxs = []
    for on in (0, 1):
        lib.fast_conv_set_x3_presplit(on)
        dX = eng.grads[l - 1]
        dX.fill_(float("nan"))
        hp.layer_bwd(l, eng.acts[l - 1], eng.grads[l], eng.bits[l], torch.zeros_like(eng.grad_flat), dX, eng.P,
                     eng.E, eng.T, eng.bits_rows[l], part="d")
        torch.cuda.synchronize()
        dxs.append(dX[:eng.T * eng.B].clone())
    lib.fast_conv_set_x3_presplit(1)
    assert torch.isfinite(dxs[0]).all() and dxs[0].norm() > 0
    assert torch.equal(dxs[0], dxs[1])


@pytest.mark.parametrize("l", [1, 2])
def test_x3_dgrad_group_outer_and_split_bit_equal(x3_rollout, l):
    """conv_dgrad_x3 with the slot groups outermost (each group's weights staged once per workgroup), with the samples
    of a path of > 4 active slots split over gridDim.z, and on the cost-balanced 1-D schedule whose workgroups span
    paths (BAL, the default) == the round-6 kernel (conv_dgrad_x3v0: groups inside the sample loop, weights restaged
    per sample): one workgroup computes a sample's dX in group order either way, so the input gradient and its amax
    are bit-identical.  masks_with_edges has an all-modules path (3 slot groups)."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, _ = x3_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    assert int(tr.model.act_cnt.view(eng.P, -1)[:, l].max()) > 8
    outs = []
    for v0, gsplit, bal in ((1, 1, 0), (0, 1, 0), (0, 2, 0), (0, 1, 1)):
        lib.fast_conv_set_x3_dg_v0(v0)
        lib.fast_conv_set_x3_dg_gsplit(gsplit)
        lib.fast_conv_set_x3_dg_bal(bal)
        dX = eng.grads[l - 1]
        dX.fill_(float("nan"))
        hp.gamax.zero_()
        hp.layer_bwd(l, eng.acts[l - 1], eng.grads[l], eng.bits[l], torch.zeros_like(eng.grad_flat), dX, eng.P,
                     eng.E, eng.T, eng.bits_rows[l], part="d")
        torch.cuda.synchronize()
        outs.append((dX[:eng.T * eng.B].clone(), hp.gamax.clone()))
    lib.fast_conv_set_x3_dg_v0(0)                # the defaults
    lib.fast_conv_set_x3_dg_gsplit(2)
    lib.fast_conv_set_x3_dg_bal(1)
    assert torch.isfinite(outs[0][0]).all() and outs[0][0].norm() > 0
    for d, am in outs[1:]:
        assert torch.equal(d, outs[0][0]) and torch.equal(am, outs[0][1])


@pytest.mark.parametrize("l", [3, 4])
def test_x3_fc_dgrad_gemm_matches_streaming_kernel(x3_rollout, l):
    """fc_gm_x3 + fc_dgrad_gemm_x3 (per-path GEMM over (slot, column) with LDS-staged 128 x 256 tiles) == fc_dgrad_x3
    (64-row workgroups streaming the weights): input gradient to fp32 summation order, weight gradient (which reads
    the same Gm) equal up to its own float atomics."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, g_hip = x3_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    g = hp.geoms[l]
    seg = slice(g.w_off, g.w_off + hp.M * g.chunk)
    dxs, gws = [], []
    for gemm in (0, 1):
        lib.fast_conv_set_x3_fc_dg_gemm(gemm)
        eng.grad_flat.zero_()
        dX = eng.grads[l - 1]
        dX.fill_(float("nan"))
        hp.layer_bwd(l, eng.acts[l - 1], eng.grads[l], eng.bits[l], eng.grad_flat, dX, eng.P, eng.E, eng.T,
                     eng.bits_rows[l])
        torch.cuda.synchronize()
        dxs.append(dX[:eng.T].clone())
        gws.append(eng.grad_flat[seg].clone())
    lib.fast_conv_set_x3_fc_dg_gemm(1)
    assert torch.isfinite(dxs[1]).all() and dxs[0].norm() > 0
    e = rel(dxs[1], dxs[0])
    print(f"fc layer {l} dgrad GEMM vs streaming: rel {e:.2e}, weight gradient rel {rel(gws[1], gws[0]):.2e}")
    assert e < 1e-6, e
    assert rel(gws[1], gws[0]) < 1e-6


def _shipped_trainer(paths=3, envs=16, tmax=4, seed=1):
    """The bench path at a small shape: fp32x, frame ring, hipGraph capture + replay, device GA, pipelined."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = paths, envs, tmax
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.use_graph = True
    cfg.ga.backend = "device"
    cfg.seed = seed
    tr = PathNetTrainer(cfg, device=DEV)
    assert tr.engine.ring and tr.engine.use_graph and tr.pipelined
    return tr


def test_x3_shipped_graph_path_gradient_vs_plain_fp32_oracle(hip_lib):
    """What the bench runs: eager first update + capture, graph replays, then one more replay of the captured rollout
    graph whose gradient is compared against the plain fp32 autograd oracle on the same stored rollout."""
    tr = _shipped_trainer()
    eng = tr.engine
    tr.env.max_episode_steps = 5                 # episode resets inside the rollouts
    for _ in range(4):
        tr.update()
    tr.flush()
    assert eng.g_rollout is not None and eng.g_opt is not None
    eng.rollout_backward()                       # a replay of the captured rollout + backward graph
    torch.cuda.synchronize()
    assert eng.dones.any()
    check_layers("fp32x shipped graph path", tr, eng.grad_flat, *_oracles(_oracle_grad, tr, eng))


@pytest.mark.parametrize("what", ["activation", "weight"])
def test_x3_range_overflow_raises_named_error(hip_lib, what):
    """fp16-pair range guard: an fc activation driven past 65504 (bias 1e5) or a first-layer weight past 128 (x 2^8
    = 32768) must surface as X3RangeError naming the cause, through the all-reduced counters of the graph path."""
    from pathnet_gym_amd.runtime.guard import X3RangeError
    tr = _shipped_trainer()
    tr.update()
    tr.update()
    tr.flush()                                   # in range so far
    st = tr.model.store
    with torch.no_grad():
        for j in range(tr.cfg.net.M):
            if what == "activation":
                s = st.layout.by_name[f"layer3.module{j}.bias"]
                st.flat[s.offset:s.offset + s.numel] = 1e5
            else:
                s = st.layout.by_name[f"layer0.module{j}.weight"]
                st.flat[s.offset:s.offset + 4] = 1e3
    tr.model.hip.refresh_weights()
    if what == "weight":
        # the refresh's flag is caught by flush() itself (task end / before a checkpoint), not one update late
        with pytest.raises(X3RangeError, match=r"weight x 2\^8"):
            tr.flush()
        tr.model.hip.refresh_weights()
    with pytest.raises(X3RangeError, match="activation" if what == "activation" else r"weight x 2\^8"):
        for _ in range(3):
            tr.update()
        tr.flush()


def test_optimizer_tail_one_launch_matches_torch_ops(hip_lib, monkeypatch):
    """The optimizer graph's tail in one launch (csrc/ga.hip opt_tail_kernel: the GA's local fitness view, fired
    windows reset, the ring's fc row carried, the update counter) == the torch ops it replaces, over updates whose
    tournaments fire (short episodes), through the graph capture and replays."""
    runs = []
    for tail in ("0", "1"):
        monkeypatch.setenv("PATHNET_OPT_TAIL", tail)
        tr = _shipped_trainer(paths=4, envs=16, tmax=3)
        tr.cfg.a2c.lr = 0.0
        tr.env.max_episode_steps = 4
        e = tr.engine
        snaps = []
        for _ in range(6):
            tr.update()
            torch.cuda.synchronize()
            snaps.append((e.fitness.clone(), e.fit_cnt.clone(), e.fit_sum.clone(), e.fc.clone(), e.ctr.clone(),
                          e.ga_dev["geno"].clone()))
        tr.flush()
        runs.append(snaps)
    assert any(bool(x[1].eq(0).any()) for x in runs[1][2:])
    for u, (a, b) in enumerate(zip(*runs)):
        for k, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (u, k)


def test_x3_refresh_all_layers_one_launch_bit_equal(hip_lib):
    """Every layer's fp16-pair weight copies in one launch (x3_refresh_weights_all) == one launch per layer
    (x3_refresh_weights), Wc and WcT bit for bit, after random weights."""
    from pathnet_gym_amd.ops import _lib
    tr = _shipped_trainer()
    hp = tr.model.hip
    with torch.no_grad():
        tr.model.store.flat.normal_(0, 0.05)
    hp.refresh_weights()
    torch.cuda.synchronize()
    a = [w.clone() for w in hp.Wc] + [w.clone() for w in hp.WcT if w is not None]
    for w in list(hp.Wc) + [w for w in hp.WcT if w is not None]:
        w.zero_()
    flat = tr.model.store.flat
    for l, g in enumerate(hp.geoms):
        _lib.call("x3_refresh_weights", flat.data_ptr(), g.w_off, g.chunk, g.K, g.KP, g.Cout, hp.M,
                  hp.Wc[l].data_ptr(), _lib.ptr(hp.WcT[l]), 1, hp.x3_status.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    b = [w.clone() for w in hp.Wc] + [w.clone() for w in hp.WcT if w is not None]
    assert len(a) == len(b) and any(x.abs().sum() > 0 for x in a)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


# ---------------------------------------------------------------------------------------------------------------
# the reference's default network (BasicLSTMCell(256) after the L=4 trunk, constants.py:30) in fp32x:
# csrc/lstm_x3.hip against a plain fp32 autograd oracle of the whole update
# ---------------------------------------------------------------------------------------------------------------
def _oracle_grad_lstm(tr, eng, dtype=torch.float32):
    from pathnet_gym_amd.models.pathnet import lstm_cell_ref
    cfg = tr.cfg
    T, B = eng.T, eng.B
    a2c = cfg.a2c
    flat = tr.model.store.flat.detach().clone().to(dtype).requires_grad_(True)
    st = ParamStore(cfg.net, DEV, flat=flat)
    x = eng.obs_stacks().reshape((T + 1) * B, 160, 120, 4).to(dtype) / 255.0
    mask = tr.model.mask.repeat_interleave(eng.E, 0).repeat(T + 1, 1, 1).to(dtype)
    feat = trunk_forward_ref(st, x, mask).view(T + 1, B, -1)
    k, bb = st.lstm()
    h, c = eng.hst[0].to(dtype), eng.cst[0].to(dtype)      # state entering step 0 (pre-masked by the carry)
    hs = []
    for t in range(T + 1):
        if t > 0:
            keep = (1.0 - eng.dones[t - 1].to(dtype))[:, None]
            h, c = h * keep, c * keep
        h, c = lstm_cell_ref(feat[t], h, c, k, bb)
        hs.append(h)
    hcat = torch.stack(hs).reshape((T + 1) * B, -1)
    assert rel(hcat[:T * B], eng.hst[1:T + 1].reshape(T * B, -1)) < X3_LAYER_TOL
    logits, values = heads_ref(st, hcat, tr.model.task)
    assert rel(logits[:T * B], eng.logits[:T].reshape(-1, eng.A)) < 1e-5
    assert rel(values, eng.values[:T + 1].reshape(-1)) < 1e-5
    R, adv = nstep_returns(eng.rewards, eng.values[:T], eng.dones.bool(), eng.values[T], a2c.gamma,
                           a2c.gae_lambda, a2c.reward_clip)
    loss, _, _, _ = a2c_loss(logits[:T * B], values[:T * B], eng.actions[:T].reshape(-1).long(),
                             R.reshape(-1).to(dtype), adv.reshape(-1).to(dtype), a2c.entropy_beta, a2c.value_coef,
                             torch.full((T * B,), eng.weight, device=DEV, dtype=dtype))
    loss.backward()
    return flat.grad


@pytest.fixture(scope="module", params=[("eager", "Alien"), ("graph", "Alien"), ("eager", "Pong")],
                ids=["eager-Alien", "graph-Alien", "eager-Pong"])
def x3_lstm_rollout(hip_lib, request):
    """The `reference` preset (L=4 trunk + LSTM 256, 18 actions) at a small shape in fp32x: the fused split-operand
    LSTM (no autograd hybrid), device GA (Alien: packed stacks); "graph": hipGraph capture + replays, the last replay compared."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    mode, task = request.param
    cfg = preset("reference")
    cfg.tasks = [task] + [t for t in cfg.tasks if t != task]
    cfg.env = task
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = True
    cfg.use_graph = mode == "graph"
    cfg.ga.backend = "device"
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    assert eng.lstm_hip and not eng.hybrid and eng.hst.dtype == torch.float32
    assert eng.use_graph == (mode == "graph")
    tr.env.max_episode_steps = 5
    for _ in range(3 if cfg.use_graph else 1):
        tr.update()
    tr.flush()
    if not cfg.use_graph:
        tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
    else:
        assert eng.g_rollout is not None
    eng.rollout_backward()
    torch.cuda.synchronize()
    assert eng.dones.any()
    return (tr, eng, *_oracles(_oracle_grad_lstm, tr, eng), eng.grad_flat.clone(), task)


def test_x3_lstm_engine_gradient_vs_plain_fp32_oracle(x3_lstm_rollout):
    tr, eng, g_ref, g32, g_hip, task = x3_lstm_rollout
    err = check_layers(f"fp32x LSTM engine ({task})", tr, g_hip, g_ref, g32)
    assert "lstm" in err


def test_x3_lstm_gradient_check_detects_a_two_percent_error(x3_lstm_rollout):
    """Negative control: the LSTM kernel's (and bias') gradient scaled by 1.02 must fail the per-layer budget."""
    tr, eng, g_ref, _, g_hip, _ = x3_lstm_rollout
    for name in ("lstm.kernel", "lstm.bias"):
        s = tr.model.store.layout.by_name[name]
        bad = g_hip.clone()
        bad[s.offset:s.offset + s.numel] *= 1.02
        assert layer_errors(tr, bad, g_ref)["lstm"] > X3_LAYER_TOL, name


@pytest.mark.parametrize("ncx,pf", [(2, 1), (2, 2)])
def test_x3_conv1_ring_wgrad_two_tile_passes_match_default(x3_ring_rollout, ncx, pf):
    """conv_wgrad_slab_x3 with 2 column tiles per pass (3 waves / SIMD, the default; the all-modules path of
    masks_with_edges takes 3 passes) == the 3-tile form, weights and biases, up to float-atomic order."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, g_hip = x3_ring_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    g = hp.geoms[0]
    seg = slice(g.w_off, g.w_off + hp.M * g.chunk)
    outs = []
    for arm in ("default", "variant"):
        lib.fast_conv_set_x3_c1_wg_ncx(ncx if arm == "variant" else 3)
        lib.fast_conv_set_x3_wgrad_pf(pf if arm == "variant" else 3)
        eng.grad_flat.zero_()
        hp.ring_wgrad(eng.frames, eng.fc, eng.grads[0], eng.bits[0], eng.grad_flat, eng.P, eng.E, eng.T,
                      eng.bits_rows[0], rbase=eng.rbase)
        torch.cuda.synchronize()
        outs.append(eng.grad_flat[seg].clone())
    lib.fast_conv_set_x3_c1_wg_ncx(2)            # the defaults
    lib.fast_conv_set_x3_wgrad_pf(3)
    assert outs[0].norm() > 0
    e = rel(outs[1], outs[0])
    print(f"conv1 ring wgrad ncx={ncx} pf={pf} vs default: rel {e:.2e}")
    assert e < 1e-6, e
    assert rel(outs[0], g_hip[seg]) < 1e-6


def test_x3_conv1_ring_wgrad_env_major_matches_step_major(x3_ring_rollout):
    """conv_wgrad_slab_x3 on the frame ring with its units in env-major order (X3_C1_EMAJ, the atomic-mode default: a
    workgroup walks one env's consecutive steps) == the step-major order, weights and biases, up to float-atomic order;
    the deterministic mode always runs the step-major partition (test_x3_deterministic_*)."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, g_hip = x3_ring_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    g = hp.geoms[0]
    seg = slice(g.w_off, g.w_off + hp.M * g.chunk)
    outs = []
    for emaj in (0, 1):
        lib.fast_conv_set_x3_c1_emaj(emaj)
        eng.grad_flat.zero_()
        hp.ring_wgrad(eng.frames, eng.fc, eng.grads[0], eng.bits[0], eng.grad_flat, eng.P, eng.E, eng.T,
                      eng.bits_rows[0], rbase=eng.rbase)
        torch.cuda.synchronize()
        outs.append(eng.grad_flat[seg].clone())
    lib.fast_conv_set_x3_c1_emaj(1)               # the default
    assert outs[0].norm() > 0
    e = rel(outs[1], outs[0])
    print(f"conv1 ring wgrad env-major vs step-major: rel {e:.2e}")
    assert e < 1e-6, e
    assert rel(outs[1], g_hip[seg]) < 1e-6


@pytest.mark.parametrize("opt", ["f16b", "sb1", "bal"])
def test_x3_conv1_band_f16_staging_bit_equal(x3_ring_rollout, opt):
    """conv1_fwd_band_x2 F16B (the band converted to fp16 once while staged, X3_C1_F16B, the default) == the
    double-buffered per-read conversion, SB1 (one band buffer, three workgroups per CU, X3_C1_SB1) == the
    default, and BAL (the cost-balanced 1-D schedule whose workgroups span paths, X3_C1_BAL, the default; the
    all-modules path runs 3 passes) == the per-path grid: the same MFMA operands and pass order per band, so outputs
    and ReLU bits agree bit for bit."""
    from pathnet_gym_amd.ops import _lib
    tr, eng, _, _, _ = x3_ring_rollout
    hp = tr.model.hip
    lib = _lib.lib()
    setter = getattr(lib, "fast_conv_set_x3_c1_" + opt)
    outs = []
    for on in (0, 1):
        setter(on)
        eng.acts[0].zero_()
        eng.bits[0].zero_()
        for t in range(eng.T):
            hp.ring_fwd(eng.frames, eng.fc, eng.acts[0], eng.bits[0], eng.P, eng.E, 1, t, eng.bits_rows[0],
                        rbase=eng.rbase)
        torch.cuda.synchronize()
        outs.append((eng.acts[0].clone(), eng.bits[0].clone()))
    setter(1 if opt in ("f16b", "bal") else 0)  # the defaults
    assert outs[0][0].float().abs().sum() > 0
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("graph", [False, True])
def test_x3_fused_fc_heads_bit_equal(hip_lib, monkeypatch, graph):
    """fc_heads_fwd_x3 (the last fc layer + heads + Gumbel-max sampling of a rollout step in one launch,
    csrc/trunk_x3.hip) == fc_fwd_x3 + heads_fwd_s16_kernel: features, ReLU bits, logits, values and sampled actions
    bit for bit, over several updates (zero learning rate, so the float-atomic gradient order cannot leak into the
    compared rollouts) through the eager update, the capture and replays."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    runs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("PATHNET_X3_FUSE_HEADS", fuse)
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 32, 5
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        cfg.use_graph = graph
        cfg.ga.backend = "device"
        cfg.a2c.lr = 0.0
        tr = PathNetTrainer(cfg, device=DEV)
        e = tr.engine
        assert e._fused_heads() == (fuse == "1")
        tr.env.max_episode_steps = 7
        snaps = []
        for _ in range(3):
            tr.update()
            torch.cuda.synchronize()
            snaps.append((e.acts[-1].clone(), e.bits[-1].clone(), e.logits.clone(), e.values.clone(),
                          e.actions.clone()))
        tr.flush()
        runs.append(snaps)
    assert runs[0][0][2].abs().sum() > 0
    for u, (a, b) in enumerate(zip(*runs)):
        for k, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (u, ("feat", "bits", "logits", "values", "actions")[k])


@pytest.mark.parametrize("graph", [False, True])
def test_x3_env_step_with_folded_heads_bit_equal(hip_lib, monkeypatch, graph):
    """The frame-ring Pong step with the heads + Gumbel-max sampling of each env's sample folded into its workgroup
    (csrc/envs.hip pong_step_kernel<true, true>, engine fuse_env_heads) == heads_fwd_s16_kernel + the ring step:
    logits, values, actions, frames, rewards and dones bit for bit over several updates (zero learning rate),
    through the eager update, the capture and replays, across episode resets."""
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    runs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("PATHNET_FUSE_ENV_HEADS", fuse)
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 4, 16, 5
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        cfg.use_graph = graph
        cfg.ga.backend = "device"
        cfg.a2c.lr = 0.0
        tr = PathNetTrainer(cfg, device=DEV)
        e = tr.engine
        assert e.fuse_env_heads == (fuse == "1")
        tr.env.max_episode_steps = 7
        snaps = []
        for _ in range(3):
            tr.update()
            torch.cuda.synchronize()
            snaps.append((e.logits.clone(), e.values.clone(), e.actions.clone(), e.frames.clone(), e.rewards.clone(),
                          e.dones.clone(), e.fc.clone()))
        tr.flush()
        runs.append(snaps)
    assert runs[0][0][0].abs().sum() > 0 and runs[0][-1][5].any()
    names = ("logits", "values", "actions", "frames", "rewards", "dones", "fc")
    for u, (a, b) in enumerate(zip(*runs)):
        for k, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (u, names[k])


# ---------------------------------------------------------------------------------------------------------------
# deterministic fp32x (TrainConfig.deterministic): int64 fixed-point weight-gradient accumulation (csrc/common.h gacc)
# ---------------------------------------------------------------------------------------------------------------
def _det_rollout(ring: bool, deterministic: bool):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    cfg = preset("pong")
    cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 3, 16, 4
    cfg.use_graph = False
    cfg.compute_dtype = "fp32x"
    cfg.frame_ring = ring
    cfg.deterministic = deterministic
    tr = PathNetTrainer(cfg, device=DEV)
    eng = tr.engine
    assert eng.ring == ring and tr.model.hip.fx_det == deterministic
    tr.env.max_episode_steps = 5
    tr.update()
    tr.model.set_paths(masks_with_edges(3, cfg.net.L, cfg.net.M, cfg.net.N, seed=2))
    eng._rollout_backward_body()
    torch.cuda.synchronize()
    return tr, eng


@pytest.mark.parametrize("ring", [False, True])
def test_x3_deterministic_gradient_vs_float64_truth(hip_lib, ring):
    """The fixed-point accumulation keeps the fp32x budget against the float64 autograd truth on every layer (packed
    stacks: conv1 / conv2 slab, conv3 tile and fc weight gradients; frame ring: the conv1 ring weight gradient), and
    matches the fp32-atomic mode to fp32 rounding; the accumulator is left zeroed and the range word clear."""
    tr, eng = _det_rollout(ring, True)
    g_det = eng.grad_flat.clone()
    check_layers(f"fp32x deterministic ({'ring' if ring else 'packed'})", tr, g_det, *_oracles(_oracle_grad, tr, eng))
    assert int(tr.model.hip._fxbuf.abs().sum()) == 0
    tr.model.hip.check_x3_status()
    _, eng2 = _det_rollout(ring, True)             # an identical second trainer: the same rollout, the same bits
    assert torch.equal(eng2.grad_flat, g_det)


def test_x3_deterministic_200_updates_bit_identical(hip_lib):
    """Two runs of one seed on the shipped path (frame ring, hipGraphs, device GA, pipelined) give bit-identical
    weights, optimizer slots and genotypes after 200 updates (the fp32-atomic default differs between runs)."""
    def run():
        from pathnet_gym_amd.algo.trainer import PathNetTrainer
        cfg = preset("pong")
        cfg.paths, cfg.envs_per_path, cfg.a2c.t_max = 8, 16, 5
        cfg.compute_dtype = "fp32x"
        cfg.frame_ring = True
        cfg.use_graph = True
        cfg.ga.backend = "device"
        cfg.ga.concurrent_tournaments = 2
        cfg.deterministic = True
        tr = PathNetTrainer(cfg, device=DEV)
        assert tr.engine.ring and tr.engine.use_graph and tr.pipelined and tr.model.hip.reproducible
        tr.env.max_episode_steps = 7                    # episodes end, fitness windows fill, tournaments fire
        for _ in range(200):
            tr.update()
        tr.flush()
        torch.cuda.synchronize()
        return (tr.model.store.flat.detach().clone(), tr.opt.ms.clone(), tr.engine.ga_dev["geno"].clone(),
                tr.pop.generation)
    a, b = run(), run()
    assert a[3] > 0, "no tournament fired"
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]) and a[3] == b[3]


def test_device_lr_schedule_matches_host_anneal(hip_lib):
    """The optimizer tail advances the lr anneal on device (csrc/ga.hip opt_tail_kernel): after every update the lr
    waiting for the next one equals the host's anneal_lr (fp32) at the next clock, and no host fill was needed."""
    from pathnet_gym_amd.algo.optim import anneal_lr
    tr = _shipped_trainer(paths=4, envs=16, tmax=5)
    tr.cfg.a2c.max_time_step = 4000                # a short anneal: the lr moves every update and reaches 0
    eng = tr.engine
    eng.lr_sched[1] = 4000.0
    for u in range(14):
        tr.update()
        torch.cuda.synchronize()
        nxt = anneal_lr(tr.cfg.a2c.lr, tr.global_step - tr.task_start_step, 4000, 0, "per_task")
        assert float(eng.lr[0]) == float(np.float32(nxt)), (u, float(eng.lr[0]), nxt)
        assert eng._next_t == tr.global_step - tr.task_start_step
    tr.flush()
    assert float(eng.lr[0]) == 0.0
