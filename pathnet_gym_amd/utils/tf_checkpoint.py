"""TF1 ``tf.train.Saver`` (V2 tensor-bundle) checkpoints: reader, writer, importer.

The reference saves every global variable with ``saver = tf.train.Saver()`` through the Supervisor
(``doom_pathnet.py:157-164``) into ``<prefix>.index`` + ``<prefix>.data-00000-of-00001``.  TensorFlow
is not installed here, so this module implements the on-disk format directly, with no TF code and no
pickle:

* ``<prefix>.index`` is a LevelDB-format SSTable: data blocks of prefix-compressed
  ``(key, value)`` entries with restart points, a block trailer (compression byte + masked
  CRC32C), an index block of block handles, an empty metaindex block, and a 48-byte footer ending
  in the magic ``0xdb4775248b80fb57``.  Key ``""`` holds a ``BundleHeaderProto``; every other key is a
  tensor name whose value is a ``BundleEntryProto`` (dtype, shape, shard, offset, size, crc32c).
* ``<prefix>.data-SSSSS-of-NNNNN`` holds the raw little-endian tensor bytes.

The protobuf messages are decoded by hand (varint / length-delimited fields), as is CRC32C.

``import_reference_checkpoint`` maps the reference's variable names onto this engine's state (SURVEY.md
Appendix A):
* ``net_0/Variable``, ``net_0/Variable_1``, ... in creation order: conv W/b per (layer, module), then
  the linear-layer W/b, the policy head, the value head, then the L x M genotype-mask scalars of every
  worker slot (``game_ac_network.py:317-352``); ``net_0/basic_lstm_cell/{kernel,bias}`` (``:434-438``);
* ``<var>/RMSPropApplier`` (rms, init 1.0) and ``<var>/RMSPropApplier_1`` (momentum) slots
  (``rmsprop_applier.py:34-39``, slot_creator naming);
* ``global_step``, ``flag`` (task gate = task + 1), ``score{i}`` (fitness, -1000 pending) and
  ``fixed_path{i}-{j}`` (frozen mask) (``doom_pathnet.py:116-142``).

Parity with files written by real TensorFlow is unpinned (no TF checkpoint ships with the reference); the
reader follows the published format and is tested on bundles written by ``write_bundle``.
"""
from __future__ import annotations

import os
import re
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

MAGIC = 0xDB4775248B80FB57
DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 6: np.int8, 9: np.int64, 10: np.bool_,
      19: np.float16}
DT_INV = {np.dtype(v): k for k, v in DT.items()}

# ---------------------------------------------------------------------------
# CRC32C (Castagnoli) + LevelDB masking
# ---------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


_POLY = 0x82F63B78
_TAB_NP = np.array(_CRC_TABLE, dtype=np.uint32)


def _gf2_times(mat, vec: int) -> int:
    s, i = 0, 0
    while vec:
        if vec & 1:
            s ^= mat[i]
        vec >>= 1
        i += 1
    return s


def _shift_zeros(crc: int, nbytes: int) -> int:
    """CRC state after appending ``nbytes`` zero bytes (zlib's crc32_combine operator squaring)."""
    if nbytes <= 0:
        return crc
    odd = [_POLY] + [1 << (n - 1) for n in range(1, 32)]
    even = [_gf2_times(odd, odd[n]) for n in range(32)]
    odd = [_gf2_times(even, even[n]) for n in range(32)]
    while True:
        even = [_gf2_times(odd, odd[n]) for n in range(32)]
        if nbytes & 1:
            crc = _gf2_times(even, crc)
        nbytes >>= 1
        if not nbytes:
            return crc
        odd = [_gf2_times(even, even[n]) for n in range(32)]
        if nbytes & 1:
            crc = _gf2_times(odd, crc)
        nbytes >>= 1
        if not nbytes:
            return crc


_SHIFT_OPS = {}


def crc32c_np(data: bytes, chunk: int = 1024) -> int:
    """CRC32C of a large buffer: numpy over ``chunk``-byte pieces in parallel, then zlib-style combination."""
    buf = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    n = len(buf) // chunk
    if n < 4:
        return crc32c(bytes(buf))
    x = buf[:n * chunk].reshape(n, chunk)
    st = np.full(n, 0xFFFFFFFF, np.uint32)
    for j in range(chunk):
        st = _TAB_NP[(st ^ x[:, j]) & 0xFF] ^ (st >> 8)
    parts = (st ^ 0xFFFFFFFF).tolist()
    op = _SHIFT_OPS.get(chunk)
    if op is None:
        op = _SHIFT_OPS[chunk] = [_shift_zeros(1 << i, chunk) for i in range(32)]
    crc = parts[0]
    for c in parts[1:]:
        crc = _gf2_times(op, crc) ^ c
    rest = bytes(buf[n * chunk:])
    if rest:
        crc = _shift_zeros(crc, len(rest)) ^ crc32c(rest)
    return crc


def mask_crc(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------
# varints / protobuf wire format
# ---------------------------------------------------------------------------
def _uvarint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v, i
        shift += 7


def _put_uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _pb_fields(buf: bytes):
    """Yield (field_number, wire_type, value) of a serialized message."""
    i = 0
    while i < len(buf):
        tag, i = _uvarint(buf, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _uvarint(buf, i)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, i)[0]
            i += 8
        elif wt == 2:
            n, i = _uvarint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, i)[0]
            i += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _pb_varint(f: int, v: int) -> bytes:
    return _put_uvarint(f << 3) + _put_uvarint(v & 0xFFFFFFFFFFFFFFFF)


def _pb_bytes(f: int, b: bytes) -> bytes:
    return _put_uvarint((f << 3) | 2) + _put_uvarint(len(b)) + b


def _pb_fixed32(f: int, v: int) -> bytes:
    return _put_uvarint((f << 3) | 5) + struct.pack("<I", v)


def _decode_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None}
    for f, wt, v in _pb_fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for f2, _, v2 in _pb_fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, v3 in _pb_fields(v2):
                        if f3 == 1:
                            size = v3 - (1 << 64) if v3 >= (1 << 63) else v3
                    e["shape"].append(size)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = v
        elif f == 7:
            raise ValueError("sliced (partitioned) variables are not supported")
    return e


def _encode_entry(dtype: int, shape, shard: int, offset: int, size: int, crc: int) -> bytes:
    shp = b"".join(_pb_bytes(2, _pb_varint(1, int(d))) for d in shape)
    out = _pb_varint(1, dtype) + _pb_bytes(2, shp)
    if shard:
        out += _pb_varint(3, shard)
    if offset:
        out += _pb_varint(4, offset)
    out += _pb_varint(5, size) + _pb_fixed32(6, crc)
    return out


# ---------------------------------------------------------------------------
# SSTable
# ---------------------------------------------------------------------------
def _read_block(data: bytes, off: int, size: int, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    block = data[off:off + size]
    ctype = data[off + size]
    if ctype != 0:
        raise ValueError("compressed SSTable blocks are not supported (TF bundles are uncompressed)")
    if verify:
        want = struct.unpack_from("<I", data, off + size + 1)[0]
        got = mask_crc(crc32c(block + bytes([ctype])))
        if want != got:
            raise ValueError(f"block checksum mismatch at {off}")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    out, i, last = [], 0, b""
    while i < end:
        shared, i = _uvarint(block, i)
        nonshared, i = _uvarint(block, i)
        vlen, i = _uvarint(block, i)
        key = last[:shared] + block[i:i + nonshared]
        i += nonshared
        out.append((key, block[i:i + vlen]))
        i += vlen
        last = key
    return out


def read_sstable(path: str, verify: bool = True) -> Dict[bytes, bytes]:
    data = open(path, "rb").read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != MAGIC:
        raise ValueError(f"{path}: not a LevelDB/TF table (bad magic)")
    footer = data[len(data) - 48:]
    _, i = _uvarint(footer, 0)
    _, i = _uvarint(footer, i)                     # metaindex handle (unused)
    ioff, i = _uvarint(footer, i)
    isize, i = _uvarint(footer, i)
    out = {}
    for _, handle in _read_block(data, ioff, isize, verify):
        boff, j = _uvarint(handle, 0)
        bsize, _ = _uvarint(handle, j)
        for k, v in _read_block(data, boff, bsize, verify):
            out[k] = v
    return out


def _build_block(entries: List[Tuple[bytes, bytes]], restart_every: int = 16) -> bytes:
    out = bytearray()
    restarts = []
    last = b""
    for n, (k, v) in enumerate(entries):
        if n % restart_every == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(last), len(k)) and last[shared] == k[shared]:
                shared += 1
        out += _put_uvarint(shared) + _put_uvarint(len(k) - shared) + _put_uvarint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def write_sstable(path: str, items: Dict[bytes, bytes], block_bytes: int = 4096):
    keys = sorted(items)
    out = bytearray()
    index = []

    def emit(block: bytes) -> bytes:
        off = len(out)
        out.extend(block)
        out.append(0)
        out.extend(struct.pack("<I", mask_crc(crc32c(block + b"\x00"))))
        return _put_uvarint(off) + _put_uvarint(len(block))

    cur, size = [], 0
    for k in keys:
        cur.append((k, items[k]))
        size += len(k) + len(items[k])
        if size >= block_bytes:
            index.append((cur[-1][0], emit(_build_block(cur))))
            cur, size = [], 0
    if cur:
        index.append((cur[-1][0], emit(_build_block(cur))))
    meta = emit(_build_block([]))
    idx = emit(_build_block(index, restart_every=1))
    footer = meta + idx
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(out)


# ---------------------------------------------------------------------------
# tensor bundle
# ---------------------------------------------------------------------------
def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    """All tensors of ``<prefix>.index`` / ``<prefix>.data-*`` as numpy arrays (no code execution)."""
    table = read_sstable(prefix + ".index", verify)
    header = table.get(b"", b"")
    nshards = 1
    for f, _, v in _pb_fields(header):
        if f == 1:
            nshards = v
        elif f == 2 and v != 0:
            raise ValueError("big-endian bundles are not supported")
    shards = {}
    out = {}
    for k, v in table.items():
        if k == b"":
            continue
        e = _decode_entry(v)
        dt = DT.get(e["dtype"])
        if dt is None:
            raise ValueError(f"{k!r}: unsupported dtype enum {e['dtype']}")
        sid = e["shard_id"]
        if sid not in shards:
            shards[sid] = open(f"{prefix}.data-{sid:05d}-of-{nshards:05d}", "rb").read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if verify and e["crc32c"] is not None and mask_crc(crc32c_np(raw)) != e["crc32c"]:
            raise ValueError(f"{k!r}: tensor checksum mismatch")
        out[k.decode()] = np.frombuffer(raw, dtype=dt).reshape(e["shape"]).copy()
    return out


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]):
    """Write a single-shard V2 bundle (used for tests and for exporting to TF-format tools)."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)) or ".", exist_ok=True)
    data = bytearray()
    items = {}
    for name in sorted(tensors):
        a = np.array(tensors[name], order="C", copy=True)          # keeps 0-d scalars 0-d
        if a.dtype not in DT_INV:
            raise ValueError(f"{name}: dtype {a.dtype} not representable")
        raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        items[name.encode()] = _encode_entry(DT_INV[a.dtype], a.shape, 0, len(data), len(raw),
                                             mask_crc(crc32c_np(raw)))
        data.extend(raw)
    items[b""] = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1))        # num_shards=1, version{producer=1}
    with open(f"{prefix}.data-00000-of-00001", "wb") as f:
        f.write(data)
    write_sstable(prefix + ".index", items)


# ---------------------------------------------------------------------------
# reference name mapping
# ---------------------------------------------------------------------------
_VAR_RE = re.compile(r"^net_0/Variable(?:_(\d+))?$")


def reference_variables(tensors: Dict[str, np.ndarray]) -> List[str]:
    """``net_0/Variable[_k]`` names in creation order (TF suffixes count up from the unsuffixed first one)."""
    names = [n for n in tensors if _VAR_RE.match(n)]
    return sorted(names, key=lambda n: int(_VAR_RE.match(n).group(1) or 0))


def import_reference_checkpoint(trainer, prefix: str, verify: bool = True) -> dict:
    """Load a reference Saver checkpoint into a trainer built with the matching topology.

    Returns a summary (tensors mapped, genotype slots found, control state).  The LSTM variables map
    only when the trainer's net has an LSTM; RMSProp slots map when present.
    """
    import torch
    from .checkpoint import tf_creation_order
    t = read_bundle(prefix, verify)
    cfg = trainer.cfg.net
    store = trainer.model.store
    names = tf_creation_order(cfg)
    lstm_names = [n for n in names if n.startswith("lstm.")]
    dense_names = [n for n in names if not n.startswith("lstm.")]
    order = reference_variables(t)
    params = [n for n in order if t[n].ndim > 0]
    masks = [n for n in order if t[n].ndim == 0]
    if len(params) != len(dense_names):
        raise ValueError(f"checkpoint has {len(params)} non-scalar net_0 variables, this topology needs "
                         f"{len(dense_names)}")
    tf_of = dict(zip(dense_names, params))
    if cfg.use_lstm:
        tf_of["lstm.kernel"] = "net_0/basic_lstm_cell/kernel"
        tf_of["lstm.bias"] = "net_0/basic_lstm_cell/bias"
    mapped = 0
    with torch.no_grad():
        for ours, theirs in tf_of.items():
            s = store.layout.by_name[ours]
            a = t[theirs].astype(np.float32)
            if a.size != s.numel:
                raise ValueError(f"{theirs} -> {ours}: {a.size} != {s.numel} elements")
            sl = slice(s.offset, s.offset + s.numel)
            store.flat[sl].copy_(torch.from_numpy(a.reshape(-1)))
            for suffix, buf in (("/RMSPropApplier", trainer.opt.ms), ("/RMSPropApplier_1", trainer.opt.mom)):
                if theirs + suffix in t:
                    buf[sl].copy_(torch.from_numpy(t[theirs + suffix].astype(np.float32).reshape(-1)))
            mapped += 1
        trainer.init_flat.copy_(store.flat.detach())
    L, M = cfg.L, cfg.M
    out = {"mapped": mapped, "genotype_slots": len(masks) // (L * M) if masks else 0}
    if masks and len(masks) % (L * M) == 0:
        g = np.array([float(t[n]) for n in masks], np.float32).reshape(-1, L, M)
        out["genotypes"] = g
        P = trainer.pop.P
        k = min(P, g.shape[0])
        trainer.pop.genotypes[:k] = (g[:k] > 0.5).astype(np.float32)
    frozen = np.zeros((L, M), np.float32)
    have_fixed = False
    for i in range(L):
        for j in range(M):
            n = f"fixed_path{i}-{j}"
            if n in t:
                frozen[i, j] = float(t[n])
                have_fixed = True
    if have_fixed:
        trainer.pop.frozen = (frozen > 0.5).astype(np.float32)
        trainer.model.set_frozen(trainer.pop.frozen)
        trainer.opt.set_frozen(trainer.pop.frozen, trainer.frozen_tasks)
    if "global_step" in t:
        trainer.global_step = int(float(t["global_step"]))
        out["global_step"] = trainer.global_step
    if "flag" in t:
        out["task"] = max(0, int(float(t["flag"])) - 1)
    scores = [(int(m.group(1)), float(t[n])) for n in t for m in [re.match(r"^score(\d+)$", n)] if m]
    if scores:
        fit = trainer.pop.fitness
        for i, v in scores:
            if i < len(fit):
                fit[i] = v
    trainer._push_genotypes()
    if trainer.backend == "hip":
        trainer.model.hip.refresh_weights()
        if trainer.engine is not None:
            trainer.engine.refresh_trainable()
            if trainer.engine.ga_dev is not None:
                trainer.engine.ga_upload(trainer.pop)
    return out
