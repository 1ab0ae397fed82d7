"""TF 1.x tensor-bundle checkpoints without TensorFlow (SURVEY.md §8(f) row 3,
Appendix D): read the reference's ``save/*.index`` + ``.data-00000-of-00001``
files and write new ones in the same format (the ``save_every`` cadence of
train.py:330-343).

Format (reproduced byte for byte; tests/test_checkpoint.py re-encodes the
reference's own checkpoints):
  * ``.data``: the tensors' raw little-endian bytes back to back, in key order;
  * ``.index``: a LevelDB-format table — one data block of prefix-compressed
    entries (restart point every 16 entries), an empty metaindex block, an
    index block whose single key is the short successor of the last key, each
    block followed by a type byte and a masked CRC32C, and a 48-byte footer
    (two varint block handles padded to 40 bytes + the table magic).  The
    first entry (empty key) is a BundleHeaderProto {num_shards 1, version
    {producer 1}}; the others map tensor names to BundleEntryProto {dtype,
    shape, offset, size, crc32c (masked, of the tensor bytes)}.

Host-side data-format code (no GPU): device tensors are copied to/from the
host around it.
"""
from __future__ import annotations

import os
import struct

import numpy as np

DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64}
DTYPE_ENUM = {np.dtype(v): k for k, v in DTYPES.items()}
TABLE_MAGIC = 0xDB4775248B80FB57
BLOCK_SIZE = 262144          # TF's table options: every reference checkpoint is one block
RESTART_INTERVAL = 16

# ---------------------------------------------------------------------------
# CRC32C (Castagnoli) and LevelDB's CRC mask
# ---------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ (0x82F63B78 if _c & 1 else 0)
    _CRC_TABLE.append(_c)


def crc32c(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def mask_crc(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------
# varints / protobuf fields
# ---------------------------------------------------------------------------
def _varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        c = v & 0x7F
        v >>= 7
        if v:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _proto_fields(b):
    i, out = 0, {}
    while i < len(b):
        tag, i = _varint(b, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        else:
            raise ValueError(f"protobuf wire type {wt}")
        out.setdefault(f, []).append(v)
    return out


def _field_varint(field: int, v: int) -> bytes:
    return _enc_varint(field << 3) + _enc_varint(v)


def _field_bytes(field: int, b: bytes) -> bytes:
    return _enc_varint((field << 3) | 2) + _enc_varint(len(b)) + b


# ---------------------------------------------------------------------------
# LevelDB table blocks
# ---------------------------------------------------------------------------
def _block_entries(buf):
    nrest = struct.unpack_from("<I", buf, len(buf) - 4)[0]
    end = len(buf) - 4 - 4 * nrest
    i, key, out = 0, b"", []
    while i < end:
        shared, i = _varint(buf, i)
        nonshared, i = _varint(buf, i)
        vlen, i = _varint(buf, i)
        key = key[:shared] + buf[i:i + nonshared]
        i += nonshared
        out.append((key, buf[i:i + vlen]))
        i += vlen
    return out


def _build_block(entries, restart_interval=RESTART_INTERVAL) -> bytes:
    buf = bytearray()
    restarts = [0]
    last = b""
    counter = 0
    for key, val in entries:
        if counter >= restart_interval:
            restarts.append(len(buf))
            counter = 0
            shared = 0
        else:
            shared = 0
            lim = min(len(last), len(key))
            while shared < lim and last[shared] == key[shared]:
                shared += 1
        buf += _enc_varint(shared) + _enc_varint(len(key) - shared) + _enc_varint(len(val))
        buf += key[shared:] + val
        last = key
        counter += 1
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def _short_successor(key: bytes) -> bytes:
    for i, c in enumerate(key):
        if c != 0xFF:
            return key[:i] + bytes([c + 1])
    return key


def _short_separator(start: bytes, limit: bytes) -> bytes:
    n = min(len(start), len(limit))
    i = 0
    while i < n and start[i] == limit[i]:
        i += 1
    if i < n:
        c = start[i]
        if c < 0xFF and c + 1 < limit[i]:
            return start[:i] + bytes([c + 1])
    return start


def _handle(off: int, size: int) -> bytes:
    return _enc_varint(off) + _enc_varint(size)


# ---------------------------------------------------------------------------
# bundles
# ---------------------------------------------------------------------------
def read_bundle(prefix: str, with_meta: bool = False):
    """{name: array} of a TF tensor bundle (`prefix`.index / .data-00000-of-00001).
    with_meta: also return {name: (offset, size, crc32c)}."""
    idx = open(prefix + ".index", "rb").read()
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    footer = idx[-48:]
    if struct.unpack_from("<Q", footer, 40)[0] != TABLE_MAGIC:
        raise ValueError(f"{prefix}.index: not a LevelDB table")
    _, j = _varint(footer, 0)
    _, j = _varint(footer, j)
    ioff, j = _varint(footer, j)
    isz, j = _varint(footer, j)
    tensors, meta = {}, {}
    for _, handle in _block_entries(idx[ioff:ioff + isz]):
        off, k = _varint(handle, 0)
        sz, k = _varint(handle, k)
        for key, val in _block_entries(idx[off:off + sz]):
            if not key:
                continue                                   # BundleHeaderProto
            fl = _proto_fields(val)
            dtype = fl.get(1, [0])[0]
            shape = [_proto_fields(dm).get(1, [0])[0]
                     for dm in _proto_fields(fl[2][0]).get(2, [])] if 2 in fl else []
            o, n = fl.get(4, [0])[0], fl.get(5, [0])[0]
            crc = struct.unpack("<I", fl[6][0])[0] if 6 in fl else None
            if dtype not in DTYPES:
                raise ValueError(f"{key!r}: unsupported dtype enum {dtype}")
            arr = np.frombuffer(data[o:o + n], dtype=np.dtype(DTYPES[dtype]).newbyteorder("<"))
            tensors[key.decode()] = arr.reshape(shape).astype(DTYPES[dtype])
            meta[key.decode()] = (o, n, crc)
    return (tensors, meta) if with_meta else tensors


def write_bundle(prefix: str, tensors: dict):
    """Write `tensors` ({name: array}; float32/float64/int32/int64) as a TF
    tensor bundle at `prefix` (tensors stored in key order, as TF's saver
    does).  Returns the list of names written."""
    names = sorted(tensors, key=lambda s: s.encode())
    data = bytearray()
    entries = [(b"", _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1)))]
    for name in names:
        arr = np.asarray(tensors[name])
        if arr.dtype not in DTYPE_ENUM:
            raise ValueError(f"{name}: dtype {arr.dtype} not supported")
        raw = np.ascontiguousarray(arr).astype(arr.dtype.newbyteorder("<")).tobytes()
        shape = b"".join(_field_bytes(2, _field_varint(1, int(d)) if d else b"")
                         for d in arr.shape)
        val = _field_varint(1, DTYPE_ENUM[arr.dtype]) + _field_bytes(2, shape)
        if len(data):
            val += _field_varint(4, len(data))
        if len(raw):
            val += _field_varint(5, len(raw))
        val += struct.pack("<B", (6 << 3) | 5) + struct.pack("<I", mask_crc(crc32c(raw)))
        entries.append((name.encode(), val))
        data += raw
    # table: data blocks of <= BLOCK_SIZE bytes, metaindex, index, footer
    out = bytearray()
    index_entries = []
    block, last_key = [], b""

    def flush(next_key):
        nonlocal block
        raw = _build_block(block)
        off = len(out)
        out.extend(raw + b"\x00" + struct.pack("<I", mask_crc(crc32c(raw + b"\x00"))))
        sep = _short_separator(block[-1][0], next_key) if next_key is not None \
            else _short_successor(block[-1][0])
        index_entries.append((sep, _handle(off, len(raw))))
        block = []

    for k, v in entries:
        if block and sum(len(a) + len(b) + 3 for a, b in block) >= BLOCK_SIZE:
            flush(k)
        block.append((k, v))
        last_key = k
    if block:
        flush(None)
    meta_raw = _build_block([])
    meta_off = len(out)
    out.extend(meta_raw + b"\x00" + struct.pack("<I", mask_crc(crc32c(meta_raw + b"\x00"))))
    idx_raw = _build_block(index_entries, restart_interval=1)
    idx_off = len(out)
    out.extend(idx_raw + b"\x00" + struct.pack("<I", mask_crc(crc32c(idx_raw + b"\x00"))))
    footer = _handle(meta_off, len(meta_raw)) + _handle(idx_off, len(idx_raw))
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
    out.extend(footer)
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    with open(prefix + ".index", "wb") as f:
        f.write(bytes(out))
    return names


# G2KParams field -> (variable scope, variable name) in the reference's graph:
# weight_input/{weight_i, weight_ii} (train.py:167-175), krnl_weights/{weight_v,
# bias_v, weight_o, weight_c} (models/g2k_lstm_mcr.py:38-69), krnl_embed/weight_r
# (models/g2k_lstm_mcr.py:71-76).  TF uniquifies a scope opened again in the same
# graph as <scope>_<k>; the reference opens them once per batch, so its
# checkpoints hold krnl_weights_288/weight_v ... krnl_weights_307/weight_v.
REF_NAMES = {
    "Wi": ("weight_input", "weight_i"),
    "Wii": ("weight_input", "weight_ii"),
    "Wv": ("krnl_weights", "weight_v"),
    "bv": ("krnl_weights", "bias_v"),
    "Wo": ("krnl_weights", "weight_o"),
    "Wc": ("krnl_weights", "weight_c"),
    "Wr": ("krnl_embed", "weight_r"),
    "head": ("nll_head", "head"),      # the build's NLL head (no reference counterpart)
}


def _scope(scope: str, k: int) -> str:
    return scope if k == 0 else f"{scope}_{k}"


def ref_name(field: str, k: int = 0) -> str:
    scope, var = REF_NAMES[field]
    return f"{_scope(scope, k)}/{var}"


def checkpoint_prefix(save_dir: str, d: int, e: int, b: int, num_batches: int) -> str:
    """The reference's checkpoint path for dataset d, epoch e, batch b
    (train.py:332-341: g2k_MPC_model_kfold_train_{d}_{e}_{b}.ckpt, saved with
    global_step = e * num_batches + b)."""
    return os.path.join(save_dir, f"g2k_MPC_model_kfold_train_{d}_{e}_{b}.ckpt-{e * num_batches + b}")


def save_due(e: int, b: int, num_batches: int, save_every: int) -> bool:
    """train.py:330: a checkpoint whenever (e * num_batches + b) % save_every == 0."""
    return (e * num_batches + b) % save_every == 0


def save_params(prefix: str, params, scope_index: int = 0, extras: dict | None = None,
                dtype=np.float64):
    """Checkpoint a G2KParams (torch tensors, any device) under the reference's
    variable names (REF_NAMES; scopes suffixed _<scope_index> when > 0), in the
    reference's dtype (float64: tf.float64 variables), then point the
    directory's ``checkpoint`` state file at it (tf.train.Saver.save).
    ``extras``: more {name: array} for the bundle (e.g. the last frame's
    krnl_weights/cost).  Returns the names written."""
    from dataclasses import fields
    t = {ref_name(f.name, scope_index): getattr(params, f.name).detach().cpu().numpy().astype(dtype)
         for f in fields(params) if getattr(params, f.name) is not None}
    t.update(extras or {})
    names = write_bundle(prefix, t)
    write_state(os.path.dirname(os.path.abspath(prefix)), prefix)
    return names


def _scope_indices(names) -> list[int]:
    out = set()
    for n in names:
        scope = n.split("/")[0]
        if scope == "krnl_weights":
            out.add(0)
        elif scope.startswith("krnl_weights_") and scope[13:].isdigit():
            out.add(int(scope[13:]))
    return sorted(out)


def load_params(prefix: str, scope_index: int | None = None, nmax: int | None = None,
                device="cpu"):
    """G2KParams (float32) from a bundle with the reference's variable names:
    our own save_params output or a reference checkpoint.  ``scope_index``:
    which <scope>_<k> instance (default: the last one, the reference's final
    batch).  ``nmax``: pad the pedestrian axis (Wi rows, Wo columns) with
    zeros to this width (the reference sizes them by the batch's num_nodes)."""
    import torch

    from .frame_step import G2KParams
    from dataclasses import fields
    t = read_bundle(prefix)
    ks = _scope_indices(t)
    if not ks:
        raise KeyError(f"{prefix}: no krnl_weights scope")
    k = ks[-1] if scope_index is None else scope_index
    vals = {}
    for f in fields(G2KParams):
        name = ref_name(f.name, k)
        if f.name == "head":                 # optional (NLL-trained checkpoints only)
            if name in t:
                vals["head"] = np.asarray(t[name], dtype=np.float32)
            continue
        if name not in t:
            raise KeyError(f"{prefix}: {name} missing")
        vals[f.name] = np.asarray(t[name], dtype=np.float32)
    n = vals["Wi"].shape[0]
    if nmax is not None and nmax > n:
        vals["Wi"] = np.concatenate([vals["Wi"], np.zeros((nmax - n, vals["Wi"].shape[1]), np.float32)], 0)
        vals["Wo"] = np.concatenate([vals["Wo"], np.zeros((vals["Wo"].shape[0], nmax - n), np.float32)], 1)
    return G2KParams(**{kk: torch.from_numpy(np.ascontiguousarray(v)).to(device) for kk, v in vals.items()})


def write_state(save_dir: str, prefix: str):
    """The ``checkpoint`` state file tf.train.Saver.save writes next to the
    bundles (a CheckpointState text proto; the reference's Saver is created per
    save, so it lists the one path; train.py:383 reads it back)."""
    path = os.path.abspath(prefix)
    with open(os.path.join(save_dir, "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{path}"\nall_model_checkpoint_paths: "{path}"\n')


def read_state(save_dir: str) -> str | None:
    """tf.train.get_checkpoint_state(save_dir).model_checkpoint_path (train.py:
    383): the latest prefix, relative paths taken from save_dir; None without a
    state file."""
    p = os.path.join(save_dir, "checkpoint")
    if not os.path.exists(p):
        return None
    for line in open(p):
        key, _, val = line.partition(":")
        if key.strip() == "model_checkpoint_path":
            path = val.strip().strip('"')
            return path if os.path.isabs(path) else os.path.join(save_dir, path)
    return None


def epoch_of(prefix: str) -> int:
    """The epoch in a checkpoint path, as train.py:387-389 parses it (the
    second `_<digits>` group)."""
    import re
    return int(re.findall(r"_[0-9]+", prefix)[1].replace("_", ""))
