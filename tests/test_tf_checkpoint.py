"""TF1 Saver V2 bundle reader/writer and the reference-name importer (utils/tf_checkpoint.py)."""
import numpy as np
import pytest
import torch

from pathnet_gym_amd.utils import tf_checkpoint as tfc


def test_crc32c_check_value_and_chunked_combination():
    assert tfc.crc32c(b"123456789") == 0xE3069283           # CRC-32C (Castagnoli) check value
    d = np.random.RandomState(0).bytes(70_001)
    assert tfc.crc32c_np(d, chunk=256) == tfc.crc32c(d)


def test_bundle_roundtrip(tmp_path):
    rng = np.random.RandomState(1)
    tensors = {f"scope/v{i:03d}": np.asarray(rng.randn(*(rng.randint(1, 5, size=rng.randint(0, 3)))), np.float32)
               for i in range(300)}                             # > one 4 KB block of index entries
    tensors["global_step"] = np.array(12345, np.int64)
    tensors["mask"] = np.array([1, 0, 1], np.int32)
    tensors["big"] = rng.randn(300, 70).astype(np.float32)
    p = str(tmp_path / "model.ckpt-7")
    tfc.write_bundle(p, tensors)
    back = tfc.read_bundle(p)
    assert set(back) == set(tensors)
    for k, v in tensors.items():
        assert back[k].dtype == v.dtype and back[k].shape == v.shape and np.array_equal(back[k], v), k
    # corrupting a data byte is caught by the per-tensor CRC32C
    raw = bytearray(open(p + ".data-00000-of-00001", "rb").read())
    raw[-3] ^= 0xFF
    open(p + ".data-00000-of-00001", "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        tfc.read_bundle(p)


def _reference_like_checkpoint(cfg, workers, rng):
    """Variables named the way the reference's graph names them."""
    from pathnet_gym_amd.models.pathnet import ParamLayout
    from pathnet_gym_amd.utils.checkpoint import tf_creation_order
    lay = ParamLayout(cfg)
    t = {}
    k = 0
    expect = {}
    for name in tf_creation_order(cfg):
        shape = lay.by_name[name].shape
        v = rng.randn(*shape).astype(np.float32)
        tf_name = "net_0/Variable" + (f"_{k}" if k else "")
        t[tf_name] = v
        t[tf_name + "/RMSPropApplier"] = np.full(shape, 0.5, np.float32)
        t[tf_name + "/RMSPropApplier_1"] = np.full(shape, 0.25, np.float32)
        expect[name] = v
        k += 1
    genos = (rng.rand(workers, cfg.L, cfg.M) < 0.5).astype(np.float32)
    for g in genos.reshape(-1):
        t[f"net_0/Variable_{k}"] = np.array(g, np.float32)
        k += 1
    t["global_step"] = np.array(4242.0, np.float32)
    t["flag"] = np.array(2.0, np.float32)
    t["score"] = np.array(-21.0, np.float32)
    for i in range(workers):
        t[f"score{i}"] = np.array(-1000.0 if i % 2 else float(i), np.float32)
    fixed = np.zeros((cfg.L, cfg.M), np.float32)
    fixed[0, 1] = fixed[1, 3] = 1
    for i in range(cfg.L):
        for j in range(cfg.M):
            t[f"fixed_path{i}-{j}"] = np.array(fixed[i, j], np.float32)
    return t, expect, genos, fixed


def test_import_reference_checkpoint(tmp_path):
    from pathnet_gym_amd.algo.trainer import PathNetTrainer
    from pathnet_gym_amd.config import preset
    cfg = preset("cartpole-cpu")
    cfg.paths = 4
    tr = PathNetTrainer(cfg)
    t, expect, genos, fixed = _reference_like_checkpoint(cfg.net, 6, np.random.RandomState(2))
    p = str(tmp_path / "ref.ckpt")
    tfc.write_bundle(p, t)
    out = tfc.import_reference_checkpoint(tr, p)
    assert out["mapped"] == len(expect) and out["genotype_slots"] == 6 and out["global_step"] == 4242
    assert out["task"] == 1
    st = tr.model.store
    for name, v in expect.items():
        assert np.array_equal(st.tensor(name).detach().numpy(), v.reshape(st.tensor(name).shape)), name
        s = st.layout.by_name[name]
        assert float(tr.opt.ms[s.offset]) == 0.5 and float(tr.opt.mom[s.offset]) == 0.25
    assert np.array_equal(tr.pop.genotypes, genos[:4])
    assert np.array_equal(tr.pop.frozen, fixed)
    assert tr.pop.fitness[0] == 0.0 and tr.pop.fitness[1] == -1000.0
    # frozen modules are excluded from updates after the import
    s = st.layout.by_name["layer0.module1.weight"]
    assert not bool(tr.opt.seg_trainable[st.layout.segments.index(s)])
    tr.update()
    assert torch.equal(st.tensor("layer0.module1.weight").detach(), torch.from_numpy(expect["layer0.module1.weight"]))
