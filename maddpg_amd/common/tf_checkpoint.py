"""TF1 checkpoints (tensor bundles) for ``U.save_state`` / ``U.load_state``.

The reference saves and restores every variable of the session with
``tf.train.Saver`` (``maddpg/common/tf_util.py:259-273``), which writes a
TF1 *tensor bundle*: ``<prefix>.index`` (a LevelDB-format sorted table of
``BundleEntryProto`` records keyed by variable name, the empty key holding a
``BundleHeaderProto``) and ``<prefix>.data-00000-of-00001`` (the tensors'
raw little-endian bytes at the offsets the entries give, each with a masked
CRC32C).  TensorFlow is not a dependency here, so this module reads and
writes that format directly:

* :func:`read_bundle` / :func:`write_bundle` -- name -> ndarray;
* :func:`state_from_tf1` / :func:`tf1_from_state` -- the mapping between
  the reference's variable names and :meth:`Engine.state_dict` keys.

Variable names (TF1 graph built by ``maddpg/trainer/maddpg.py:113-150`` with
``experiments/train.py:39-46``'s ``mlp_model``; trainer ``i`` is scope
``agent_i``):

* ``agent_i/{p_func,q_func,target_p_func,target_q_func}/fully_connected{,_1,_2}/{weights,biases}``
  (``layers.fully_connected``: weights ``[in, out]``, biases ``[out]``);
* Adam slots ``<var>/Adam`` (m) and ``<var>/Adam_1`` (v) of the p_func and q_func
  variables (``slot_creator``: the primary's op name + the optimizer's name);
* the beta powers, non-slot variables made with ``tf.Variable`` under the
  *name* scope current at ``apply_gradients``: ``agent_i/beta{1,2}_power``
  for q_train's optimizer (created first) and, because re-entering
  ``tf.variable_scope("agent_i")`` in p_train opens name scope ``agent_i_1``,
  ``agent_i_1/beta{1,2}_power`` for p_train's.  The reader does not rely on
  that suffix: it takes the beta-power variables whose name starts with
  ``agent_i/`` or ``agent_i_<k>/`` in creation order (scope suffix, then
  name suffix) -- the first pair is the critic's optimizer, the second the
  actor's.

Parity unpinned: TensorFlow is not importable here and the reference ships
no checkpoint, so the format follows TF's published tensor_bundle / table
layout and the tests check the writer against the reader (and the engine's
state through both).
"""
import os
import re
import struct

import numpy as np

# ---------------------------------------------------------------- CRC32C
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def _crc_scalar(data, crc=0):
    crc ^= 0xFFFFFFFF
    for b in bytes(data):
        crc = _TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _gf2_times(mat, vec):
    s, i = 0, 0
    while vec:
        if vec & 1:
            s ^= mat[i]
        vec >>= 1
        i += 1
    return s


def _zeros_operator(nbytes):
    """32x32 GF(2) matrix (column n = image of bit n) of appending nbytes zero
    bytes to a CRC register: crc(A || B) = op_|B|(crc(A)) ^ crc(B)."""
    one = [_TABLE[(1 << n) & 0xFF] ^ ((1 << n) >> 8) for n in range(32)]
    result = [1 << n for n in range(32)]
    sq = one
    while nbytes:
        if nbytes & 1:
            result = [_gf2_times(sq, c) for c in result]
        nbytes >>= 1
        if nbytes:
            sq = [_gf2_times(sq, c) for c in sq]
    return result


def crc32c(data, crc=0):
    """CRC-32C (Castagnoli), as tensorflow/core/lib/hash/crc32c.  Large inputs
    run as 1024 independent lanes (numpy table lookups) combined with the
    zero-append operator, so an 8 MB checkpoint takes well under a second."""
    b = np.frombuffer(bytes(data), np.uint8)
    K = 1024
    if b.size < 64 * K:
        return _crc_scalar(b.tobytes(), crc)
    L = b.size // K
    lanes = np.ascontiguousarray(b[:K * L].reshape(K, L).T)
    t = np.asarray(_TABLE, np.uint32)
    st = np.full(K, 0xFFFFFFFF, np.uint32)
    for j in range(L):
        st = t[(st ^ lanes[j]) & 0xFF] ^ (st >> 8)
    st ^= np.uint32(0xFFFFFFFF)
    op = _zeros_operator(L)
    acc = _gf2_times(op, crc) ^ int(st[0]) if crc else int(st[0])
    for c in st[1:]:
        acc = _gf2_times(op, acc) ^ int(c)
    return _crc_scalar(b[K * L:].tobytes(), acc)


def crc_mask(crc):
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def crc_unmask(m):
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------- varint / proto
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def _proto_fields(buf):
    """[(field, wire_type, value)] of one message (varint, fixed64, bytes, fixed32)."""
    out, pos = [], 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.append((f, wt, v))
    return out


def _pf_varint(f, v):
    return _varint(f << 3) + _varint(v) if v else b""


def _pf_bytes(f, b):
    return _varint((f << 3) | 2) + _varint(len(b)) + b


# DataType enum (tensorflow/core/framework/types.proto)
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64}
_DT_OF = {np.dtype(v): k for k, v in _DT.items()}


def _entry_proto(dtype, shape, offset, size, crc):
    dims = b"".join(_pf_bytes(2, _pf_varint(1, int(d)) if d else b"") for d in shape)
    return (_pf_varint(1, dtype) + _pf_bytes(2, dims) + _pf_varint(4, offset) + _pf_varint(5, size) +
            _varint((6 << 3) | 5) + struct.pack("<I", crc))


def _parse_entry(buf):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": False}
    for f, _wt, v in _proto_fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for g, _w, d in _proto_fields(v):
                if g == 2:
                    size = 0
                    for h, _x, s in _proto_fields(d):
                        if h == 1:
                            size = s
                    e["shape"].append(size)
                elif g == 3 and d:
                    raise ValueError("unknown-rank tensor in checkpoint")
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = v
        elif f == 7:
            e["slices"] = True
    return e


# ------------------------------------------------------------- sorted table
_MAGIC = 0xDB4775248B80FB57
_RESTART = 16
_BLOCK = 256 * 1024


def _block(entries):
    """LevelDB block: prefix-compressed entries, restart array, count."""
    out, restarts, prev = bytearray(), [], b""
    for i, (k, v) in enumerate(entries):
        shared = 0
        if i % _RESTART == 0:
            restarts.append(len(out))
        else:
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _block_entries(buf):
    nrest = struct.unpack_from("<I", buf, len(buf) - 4)[0]
    end = len(buf) - 4 - 4 * nrest
    out, pos, key = [], 0, b""
    while pos < end:
        shared, pos = _read_varint(buf, pos)
        nonshared, pos = _read_varint(buf, pos)
        vlen, pos = _read_varint(buf, pos)
        key = key[:shared] + bytes(buf[pos:pos + nonshared])
        pos += nonshared
        out.append((key, bytes(buf[pos:pos + vlen])))
        pos += vlen
    return out


def _handle(off, size):
    return _varint(off) + _varint(size)


def _write_table(path, items):
    """items: sorted [(key bytes, value bytes)] -> LevelDB-format table file
    (uncompressed blocks, each with its type byte + masked CRC32C trailer)."""
    f = bytearray()

    def put(block):
        off = len(f)
        f.extend(block)
        trailer = b"\x00"
        f.extend(trailer + struct.pack("<I", crc_mask(crc32c(block + trailer))))
        return off, len(block)

    index, cur, cur_bytes = [], [], 0
    for k, v in items:
        cur.append((k, v))
        cur_bytes += len(k) + len(v)
        if cur_bytes >= _BLOCK:
            off, size = put(_block(cur))
            index.append((cur[-1][0], _handle(off, size)))
            cur, cur_bytes = [], 0
    if cur:
        off, size = put(_block(cur))
        index.append((cur[-1][0], _handle(off, size)))
    meta = put(_block([]))
    idx = put(_block(index))
    footer = _handle(*meta) + _handle(*idx)
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
    f.extend(footer)
    with open(path, "wb") as fh:
        fh.write(bytes(f))


def _read_table(path):
    with open(path, "rb") as fh:
        buf = fh.read()
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != _MAGIC:
        raise ValueError(f"{path}: not a TF1 checkpoint index (bad table magic)")
    footer = buf[len(buf) - 48:]
    _moff, p = _read_varint(footer, 0)
    _msize, p = _read_varint(footer, p)
    ioff, p = _read_varint(footer, p)
    isize, p = _read_varint(footer, p)

    def block_at(off, size):
        if buf[off + size] != 0:
            raise ValueError(f"{path}: compressed table block (type {buf[off + size]}) is not supported")
        blk = buf[off:off + size]
        want = struct.unpack_from("<I", buf, off + size + 1)[0]
        if crc_unmask(want) != crc32c(blk + b"\x00"):
            raise ValueError(f"{path}: table block checksum mismatch")
        return blk

    items = []
    for _k, h in _block_entries(block_at(ioff, isize)):
        off, q = _read_varint(h, 0)
        size, _ = _read_varint(h, q)
        items.extend(_block_entries(block_at(off, size)))
    return items


# ------------------------------------------------------------------ bundle
def _data_path(prefix, shard=0, nshards=1):
    return f"{prefix}.data-{shard:05d}-of-{nshards:05d}"


def is_bundle(prefix):
    return os.path.exists(prefix + ".index")


def write_bundle(prefix, tensors):
    """Write name -> ndarray as a one-shard TF1 tensor bundle at `prefix`
    (`prefix`.index + `prefix`.data-00000-of-00001), keys in sorted order."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    header = _pf_varint(1, 1) + _pf_bytes(3, _pf_varint(1, 1))  # num_shards 1, LITTLE, version {producer 1}
    items = [(b"", header)]
    data = bytearray()
    for name in sorted(tensors):
        a = np.asarray(tensors[name])  # (ascontiguousarray would make a scalar 1-d)
        if a.dtype not in _DT_OF:
            raise TypeError(f"{name}: dtype {a.dtype} not supported")
        raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        items.append((name.encode(), _entry_proto(_DT_OF[a.dtype], a.shape, len(data), len(raw),
                                                  crc_mask(crc32c(raw)))))
        data += raw
    with open(_data_path(prefix), "wb") as fh:
        fh.write(bytes(data))
    _write_table(prefix + ".index", items)
    return prefix


def read_bundle(prefix, verify=True):
    """name -> ndarray of every tensor in the TF1 bundle at `prefix`."""
    items = _read_table(prefix + ".index")
    nshards = 1
    if items and items[0][0] == b"":
        for f, _wt, v in _proto_fields(items[0][1]):
            if f == 1:
                nshards = v
            elif f == 2 and v != 0:
                raise ValueError("big-endian checkpoint is not supported")
    out, shards = {}, {}
    for k, v in items:
        if k == b"":
            continue
        e = _parse_entry(v)
        name = k.decode()
        if e["slices"]:
            raise ValueError(f"{name}: partitioned (sliced) variables are not supported")
        if e["dtype"] not in _DT:
            raise ValueError(f"{name}: dtype enum {e['dtype']} not supported")
        sid = e["shard_id"]
        if sid not in shards:
            with open(_data_path(prefix, sid, nshards), "rb") as fh:
                shards[sid] = fh.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if verify and e["crc32c"] is not None and crc_unmask(e["crc32c"]) != crc32c(raw):
            raise ValueError(f"{name}: data checksum mismatch")
        out[name] = np.frombuffer(raw, np.dtype(_DT[e["dtype"]]).newbyteorder("<")).astype(
            _DT[e["dtype"]]).reshape(e["shape"])
    return out


# ------------------------------------------------- reference variable names
_NET = {"actor": "p_func", "critic": "q_func", "tgt_actor": "target_p_func", "tgt_critic": "target_q_func"}
_LAYER = {"W1": ("fully_connected", "weights"), "b1": ("fully_connected", "biases"),
          "W2": ("fully_connected_1", "weights"), "b2": ("fully_connected_1", "biases"),
          "W3": ("fully_connected_2", "weights"), "b3": ("fully_connected_2", "biases")}
_SLOT = {"m": "Adam", "v": "Adam_1"}


def tf1_name(key):
    """Engine.state_dict key -> the reference's variable name (not the beta powers)."""
    agent, which, k = key.split("/")
    layer, var = _LAYER[k]
    if which in _NET:
        return f"{agent}/{_NET[which]}/{layer}/{var}"
    slot, net = which.split("_")
    return f"{agent}/{_NET[net]}/{layer}/{var}/{_SLOT[slot]}"


def tf1_from_state(sd):
    """Engine.state_dict() -> the reference's {variable name: array}."""
    out = {}
    for key, v in sd.items():
        agent, which, k = key.split("/")
        if k == "beta_power":
            scope = agent if which == "critic" else f"{agent}_1"
            out[f"{scope}/beta1_power"] = np.float32(v[0])
            out[f"{scope}/beta2_power"] = np.float32(v[1])
        else:
            out[tf1_name(key)] = np.asarray(v, np.float32)
    return out


def _beta_vars(tensors, agent):
    """[(beta1 name, beta2 name)] of trainer `agent` in creation order."""
    pat = re.compile(rf"^{re.escape(agent)}(?:_(\d+))?/(?:.*/)?beta([12])_power(?:_(\d+))?$")
    found = {}
    for name in tensors:
        m = pat.match(name)
        if m:
            order = (int(m.group(1) or 0), int(m.group(3) or 0))
            found.setdefault(order, {})[m.group(2)] = name
    return [(d["1"], d["2"]) for _o, d in sorted(found.items()) if "1" in d and "2" in d]


def state_from_tf1(tensors, n_agents, sets):
    """The reference's {variable name: array} -> Engine.state_dict() keys.
    Raises KeyError naming the first variable the checkpoint lacks."""
    sd = {}
    for i in range(n_agents):
        agent = f"agent_{i}"
        for which in sets:
            for k in _LAYER:
                key = f"{agent}/{which}/{k}"
                name = tf1_name(key)
                if name not in tensors:
                    raise KeyError(f"TF1 checkpoint has no variable {name!r}")
                a = np.asarray(tensors[name], np.float32)
                sd[key] = a
        betas = _beta_vars(tensors, agent)
        if len(betas) < 2:
            raise KeyError(f"TF1 checkpoint lacks the two Adam beta-power pairs of {agent}")
        for net, (b1, b2) in zip(("critic", "actor"), betas[:2]):
            sd[f"{agent}/{net}/beta_power"] = np.array([tensors[b1], tensors[b2]], np.float32).reshape(2)
    return sd
