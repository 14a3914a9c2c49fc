"""Offline reader / writer of TensorFlow checkpoint-V2 tensor bundles
(SURVEY.md 8f row 3), so a model the reference trained (tf.train.Saver,
genericNeuralNet.py:149, 410; experiments.py:75-82) can be loaded here without
TensorFlow.

A bundle ``<prefix>`` is two files:
  * ``<prefix>.index`` -- a LevelDB-format table (sorted keys, prefix-compressed
    data blocks with restart arrays, a 5-byte block trailer of compression type +
    masked crc32c, an index block of block handles, and a 48-byte footer ending in
    the magic 0xdb4775248b80fb57).  Key "" holds a BundleHeaderProto; every other
    key is a variable name whose value is a BundleEntryProto {dtype = 1,
    shape = 2, shard_id = 3, offset = 4, size = 5, crc32c = 6 (fixed32, masked)};
  * ``<prefix>.data-SSSSS-of-NNNNN`` -- the tensors' raw little-endian bytes.
Protobuf wire format and crc32c (Castagnoli) are decoded here by hand; no
TensorFlow / protobuf runtime is used.  The reference's variable names are
``embedding_layer/embedding_users`` ... (matrix_factorization.py:30-36,
NCF.py:29-41); Adam slots are ``<var>/Adam`` and ``<var>/Adam_1``, the powers
``beta1_power`` / ``beta2_power`` (gnn:432-440).

Parity is unpinned against real reference checkpoints: the reference ships none
(its trained models are absent); the format is pinned by the
crc32c check value and round trips through write_checkpoint.
"""
import os
import struct

import numpy as np

MAGIC = 0xDB4775248B80FB57
# tensorflow/core/framework/types.proto DataType -> numpy
DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
          10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DT_OF = {np.dtype(v): k for k, v in DTYPES.items()}

# ---------------------------------------------------------------- crc32c
_POLY = 0x82F63B78
_TABLE = []
for _n in range(256):
    _c = _n
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)
_TABLE = np.array(_TABLE, np.uint32)


def crc32c(data, crc=0):
    """CRC-32C (Castagnoli), the checksum of LevelDB blocks and TF bundle entries."""
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in bytes(data):
        crc = int(t[(crc ^ b) & 0xFF]) ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def mask(crc):
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- varint / protobuf
def _varint(buf, pos):
    out, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        out |= (b & 0x7F) << shift
        if b < 0x80:
            return out, pos
        shift += 7


def _enc_varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fields(buf):
    """Protobuf wire decode: yields (field number, wire type, value)."""
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        yield fn, wt, v


def parse_entry(buf):
    """BundleEntryProto -> dict(dtype, shape, shard_id, offset, size, crc32c)."""
    e = dict(dtype=0, shape=[], shard_id=0, offset=0, size=0, crc32c=None, slices=False)
    for fn, wt, v in _fields(buf):
        if fn == 1:
            e["dtype"] = v
        elif fn == 2:
            for f2, _, d in _fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, s in _fields(d):
                        if f3 == 1:
                            size = s
                    e["shape"].append(size)
        elif fn == 3:
            e["shard_id"] = v
        elif fn == 4:
            e["offset"] = v
        elif fn == 5:
            e["size"] = v
        elif fn == 6:
            e["crc32c"] = struct.unpack("<I", v)[0]
        elif fn == 7:
            e["slices"] = True
    return e


def _enc_entry(dtype, shape, offset, size, crc):
    dims = b"".join(b"\x12" + _enc_varint(len(d)) + d for d in
                    (b"\x08" + _enc_varint(int(s)) for s in shape))
    out = b"\x08" + _enc_varint(dtype)
    out += b"\x12" + _enc_varint(len(dims)) + dims
    if offset:
        out += b"\x20" + _enc_varint(offset)
    if size:
        out += b"\x28" + _enc_varint(size)
    out += b"\x35" + struct.pack("<I", crc)
    return out


# ---------------------------------------------------------------- LevelDB table
def _block_entries(block):
    n_restarts = struct.unpack("<I", block[-4:])[0]
    end = len(block) - 4 - 4 * n_restarts
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        non_shared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + bytes(block[pos:pos + non_shared])
        pos += non_shared
        yield key, bytes(block[pos:pos + vlen])
        pos += vlen


def _read_block(data, offset, size, verify=True):
    block = data[offset:offset + size]
    trailer = data[offset + size:offset + size + 5]
    if len(trailer) != 5:
        raise ValueError("truncated table block")
    if trailer[0] != 0:
        raise ValueError("compressed table blocks (type %d) are not supported" % trailer[0])
    if verify and mask(crc32c(block + trailer[:1])) != struct.unpack("<I", trailer[1:5])[0]:
        raise ValueError("table block checksum mismatch")
    return block


def read_index(path, verify=True):
    """All (key, value) pairs of a LevelDB-format table file, in key order."""
    data = open(path, "rb").read()
    if len(data) < 48 or struct.unpack("<Q", data[-8:])[0] != MAGIC:
        raise ValueError("%s is not a LevelDB table (bad footer magic)" % path)
    footer = data[-48:]
    _, pos = _varint(footer, 0)
    _, pos = _varint(footer, pos)          # metaindex handle (unused)
    ioff, pos = _varint(footer, pos)
    isz, pos = _varint(footer, pos)
    out = []
    for _, handle in _block_entries(_read_block(data, ioff, isz, verify)):
        boff, p = _varint(handle, 0)
        bsz, _ = _varint(handle, p)
        out.extend(_block_entries(_read_block(data, boff, bsz, verify)))
    return out


def _build_block(entries, restart_interval=16):
    buf, restarts, last = bytearray(), [], b""
    for n, (k, v) in enumerate(entries):
        if n % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        buf += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def write_index(path, entries, block_bytes=4096):
    """Write sorted (key, value) pairs as an uncompressed LevelDB-format table."""
    out = bytearray()
    index = []
    chunk, size = [], 0

    def flush():
        nonlocal chunk, size
        if not chunk:
            return
        blk = _build_block(chunk)
        off = len(out)
        out.extend(blk + b"\x00" + struct.pack("<I", mask(crc32c(blk + b"\x00"))))
        index.append((chunk[-1][0], _enc_varint(off) + _enc_varint(len(blk))))
        chunk, size = [], 0

    for k, v in entries:
        chunk.append((k, v))
        size += len(k) + len(v)
        if size >= block_bytes:
            flush()
    flush()
    meta = _build_block([])
    moff = len(out)
    out.extend(meta + b"\x00" + struct.pack("<I", mask(crc32c(meta + b"\x00"))))
    iblk = _build_block(index, restart_interval=1)
    ioff = len(out)
    out.extend(iblk + b"\x00" + struct.pack("<I", mask(crc32c(iblk + b"\x00"))))
    footer = _enc_varint(moff) + _enc_varint(len(meta)) + _enc_varint(ioff) + _enc_varint(len(iblk))
    footer = footer + b"\x00" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(bytes(out))


# ---------------------------------------------------------------- bundles
def list_variables(prefix):
    """[(name, shape, numpy dtype)] of a checkpoint (tf.train.list_variables)."""
    out = []
    for k, v in read_index(prefix + ".index"):
        if k == b"":
            continue
        e = parse_entry(v)
        out.append((k.decode(), tuple(e["shape"]), DTYPES.get(e["dtype"])))
    return out


def read_checkpoint(prefix, names=None, verify=True):
    """{variable name: numpy array} of a TF checkpoint-V2 bundle (all variables, or names)."""
    num_shards = 1
    entries = {}
    for k, v in read_index(prefix + ".index", verify):
        if k == b"":
            for fn, _, val in _fields(v):
                if fn == 1:
                    num_shards = val
            continue
        entries[k.decode()] = parse_entry(v)
    want = entries if names is None else {n: entries[n] for n in names}
    shards = {}
    out = {}
    for name, e in want.items():
        if e["slices"]:
            raise ValueError("partitioned variable %s is not supported" % name)
        if e["dtype"] not in DTYPES:
            raise ValueError("variable %s has unsupported dtype %d" % (name, e["dtype"]))
        sid = e["shard_id"]
        if sid not in shards:
            shards[sid] = open("%s.data-%05d-of-%05d" % (prefix, sid, num_shards), "rb").read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(raw) != e["size"]:
            raise ValueError("variable %s is truncated in its data shard" % name)
        if verify and e["crc32c"] is not None and mask(crc32c(raw)) != e["crc32c"]:
            raise ValueError("variable %s fails its crc32c check" % name)
        out[name] = np.frombuffer(raw, dtype=np.dtype(DTYPES[e["dtype"]]).newbyteorder("<")).reshape(
            e["shape"]).copy()
    return out


def write_checkpoint(prefix, tensors):
    """Write {name: array} as a single-shard TF checkpoint-V2 bundle (tf.train.Saver layout)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    data = bytearray()
    entries = []
    for name in sorted(tensors):
        a = np.asarray(tensors[name], order="C")      # keeps 0-d (ascontiguousarray would not)
        dt = DT_OF.get(a.dtype)
        if dt is None:
            raise ValueError("unsupported dtype %s" % a.dtype)
        raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        entries.append((name.encode(), _enc_entry(dt, a.shape, len(data), len(raw), mask(crc32c(raw)))))
        data += raw
    header = b"\x08\x01"                       # num_shards = 1, little endian, version {}
    write_index(prefix + ".index", [(b"", header)] + entries)
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
