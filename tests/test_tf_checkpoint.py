"""TF1 checkpoint (tensor bundle) reader / writer (maddpg_amd/common/tf_checkpoint.py).

CRC-32C is pinned by the published test vectors (RFC 3720 B.4 and the
"123456789" check value).  The bundle layout itself is parity unpinned (no
TensorFlow here and no checkpoint in the reference): the writer is checked
against the reader, the table against its own structural invariants, and the
name mapping against the reference's variable scopes (maddpg.py:75-150,
train.py:39-46)."""
import struct

import numpy as np
import pytest

from maddpg_amd.common import tf_checkpoint as tfc


def test_crc32c_known_answers():
    assert tfc.crc32c(b"123456789") == 0xE3069283
    assert tfc.crc32c(bytes(32)) == 0x8A9136AA             # RFC 3720 B.4: 32 zero bytes
    assert tfc.crc32c(b"\xff" * 32) == 0x62A8AB43          # 32 bytes of 0xff
    assert tfc.crc32c(bytes(range(32))) == 0x46DD794E      # ascending 0..31
    assert tfc.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C  # descending 31..0


@pytest.mark.parametrize("n", [0, 1, 65535, 65536, 65537, 1024 * 97 + 13, 3_000_001])
def test_crc32c_lanes_match_scalar(n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert tfc.crc32c(data) == tfc._crc_scalar(data)
    # continuation: crc(a || b) from crc(a)
    cut = n // 3
    assert tfc.crc32c(data[cut:], tfc.crc32c(data[:cut])) == tfc._crc_scalar(data)


def test_crc_mask_round_trip():
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert tfc.crc_unmask(tfc.crc_mask(c)) == c
    assert tfc.crc_mask(0) == 0xA282EAD8


def test_bundle_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    t = {
        "agent_0/beta1_power": np.float32(0.81),
        "agent_0/q_func/fully_connected/weights": rng.standard_normal((69, 64)).astype(np.float32),
        "agent_0/q_func/fully_connected/biases": rng.standard_normal(64).astype(np.float32),
        "d": np.arange(7, dtype=np.float64),
        "i": np.arange(12, dtype=np.int32).reshape(3, 4),
        "l": np.array([-(2 ** 40)], np.int64),
        "empty": np.zeros((0, 5), np.float32),
    }
    # > restart interval and > one data block of index entries
    for i in range(300):
        t[f"many/x{i:04d}/a_rather_long_shared_prefix_{'y' * 900}"] = np.full(3, i, np.float32)
    prefix = str(tmp_path) + "/ck/"
    tfc.write_bundle(prefix, t)
    back = tfc.read_bundle(prefix)
    assert set(back) == set(t)
    for k, v in t.items():
        assert back[k].dtype == np.asarray(v).dtype and back[k].shape == np.asarray(v).shape, k
        np.testing.assert_array_equal(back[k], v)
    # the table: footer magic, more than one data block in the index
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack_from("<Q", raw, len(raw) - 8)[0] == 0xDB4775248B80FB57
    items = tfc._read_table(prefix + ".index")
    assert [k for k, _ in items] == sorted(k for k, _ in items) and items[0][0] == b""
    assert len(items) == len(t) + 1


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path) + "/c"
    tfc.write_bundle(prefix, {"w": np.arange(64, dtype=np.float32)})
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[17] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError, match="checksum"):
        tfc.read_bundle(prefix)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[-1] ^= 0xFF
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(ValueError, match="magic"):
        tfc.read_bundle(prefix)


def _state(n, obs=(18, 18), H=8):
    rng = np.random.default_rng(1)
    cin = sum(obs) + 5 * n
    sd = {}
    for i in range(n):
        for w in ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_actor", "m_critic", "v_critic"):
            fin = cin if "critic" in w else obs[i]
            fout = 1 if "critic" in w else 5
            shapes = {"W1": (fin, H), "b1": (H,), "W2": (H, H), "b2": (H,), "W3": (H, fout), "b3": (fout,)}
            for k, s in shapes.items():
                sd[f"agent_{i}/{w}/{k}"] = rng.standard_normal(s).astype(np.float32)
        sd[f"agent_{i}/actor/beta_power"] = np.array([0.9 ** (i + 2), 0.999 ** (i + 2)], np.float32)
        sd[f"agent_{i}/critic/beta_power"] = np.array([0.9 ** (i + 3), 0.999 ** (i + 3)], np.float32)
    return sd


def test_reference_variable_names(tmp_path):
    sd = _state(2)
    t = tfc.tf1_from_state(sd)
    assert "agent_1/q_func/fully_connected_1/weights" in t
    assert "agent_0/p_func/fully_connected_2/biases/Adam_1" in t
    assert "agent_0/target_q_func/fully_connected/weights" in t
    assert t["agent_0/q_func/fully_connected/weights"].shape == (18 + 18 + 10, 8)   # [in, out]
    assert t["agent_1/beta1_power"] == sd["agent_1/critic/beta_power"][0]          # q_train's optimizer
    assert t["agent_1_1/beta2_power"] == sd["agent_1/actor/beta_power"][1]         # p_train's (name scope agent_1_1)
    tfc.write_bundle(str(tmp_path) + "/p", t)
    back = tfc.state_from_tf1(tfc.read_bundle(str(tmp_path) + "/p"), 2,
                              ("actor", "critic", "tgt_actor", "tgt_critic", "m_actor", "v_actor", "m_critic",
                               "v_critic"))
    assert set(back) == set(sd)
    for k in sd:
        np.testing.assert_array_equal(back[k], sd[k], err_msg=k)


def test_beta_powers_found_under_either_suffix():
    sd = _state(1)
    t = tfc.tf1_from_state(sd)
    # the other plausible TF1 naming: both optimizers in name scope agent_0, the second uniquified
    t["agent_0/beta1_power_1"] = t.pop("agent_0_1/beta1_power")
    t["agent_0/beta2_power_1"] = t.pop("agent_0_1/beta2_power")
    back = tfc.state_from_tf1(t, 1, ("actor", "critic"))
    np.testing.assert_array_equal(back["agent_0/critic/beta_power"], sd["agent_0/critic/beta_power"])
    np.testing.assert_array_equal(back["agent_0/actor/beta_power"], sd["agent_0/actor/beta_power"])
    del t["agent_0/q_func/fully_connected/weights"]
    with pytest.raises(KeyError, match="q_func/fully_connected/weights"):
        tfc.state_from_tf1(t, 1, ("actor", "critic"))


def test_shape_unknown_rank_field():
    """TensorShapeProto field 3 (unknown_rank) present but false is a known-rank
    shape; only unknown_rank = true is refused"""
    dims = tfc._pf_bytes(2, tfc._pf_varint(1, 3)) + tfc._pf_bytes(2, tfc._pf_varint(1, 4))
    # an explicit field-3 entry with value 0 (tfc._pf_varint omits zero values, so it is
    # spelled out here): present but false
    zero = tfc._varint(3 << 3) + tfc._varint(0)
    assert zero == b"\x18\x00"
    e = tfc._parse_entry(tfc._pf_varint(1, 1) + tfc._pf_bytes(2, dims + zero))
    assert e["shape"] == [3, 4]
    with pytest.raises(ValueError, match="unknown-rank"):
        tfc._parse_entry(tfc._pf_varint(1, 1) + tfc._pf_bytes(2, tfc._pf_varint(3, 1)))


class _FakeEngine:
    """the attributes Engine.load_state uses, without a GPU"""
    SETS = ("actor", "critic")
    n = 1

    def __init__(self):
        self.loaded = None

    checkpoint_path = staticmethod(lambda f: __import__("maddpg_amd.engine", fromlist=["Engine"]).Engine.checkpoint_path(f))

    def load_state_dict(self, sd):
        self.loaded = sd


def test_load_state_picks_newer_format_and_breaks_a_tie(tmp_path):
    import os

    from maddpg_amd.engine import Engine
    sd = _state(1)
    prefix = str(tmp_path / "ckpt")
    tfc.write_bundle(prefix, tfc.tf1_from_state(sd))
    npz = Engine.checkpoint_path(prefix)
    marked = dict(sd)
    marked["agent_0/actor/W1"] = sd["agent_0/actor/W1"] + 1.0
    np.savez(npz, **marked)
    e = _FakeEngine()
    os.utime(prefix + ".index", (1000, 1000))
    os.utime(npz, (2000, 2000))
    assert Engine.load_state(e, prefix) == npz
    np.testing.assert_array_equal(e.loaded["agent_0/actor/W1"], marked["agent_0/actor/W1"])
    os.utime(npz, (500, 500))
    assert Engine.load_state(e, prefix) == prefix
    np.testing.assert_array_equal(e.loaded["agent_0/actor/W1"], sd["agent_0/actor/W1"])
    # a tie (timestamps kept by a copy / a tar archive): the TF1 bundle, with a warning
    os.utime(npz, (1000, 1000))
    e.loaded = None
    with pytest.warns(UserWarning, match="same modification time"):
        assert Engine.load_state(e, prefix) == prefix
    np.testing.assert_array_equal(e.loaded["agent_0/actor/W1"], sd["agent_0/actor/W1"])
    # nanosecond resolution decides what whole seconds cannot
    os.utime(npz, ns=(1000 * 10**9 + 1, 1000 * 10**9 + 1))
    assert Engine.load_state(e, prefix) == npz


def test_injected_tensor_sizes_are_checked():
    import torch

    from maddpg_amd.engine import Engine
    Engine._sized("idx", None, 1024)
    Engine._sized("idx", torch.zeros(1024), 1024)
    with pytest.raises(ValueError, match="idx: 1000 elements, the update reads 1024"):
        Engine._sized("idx", torch.zeros(1000), 1024)


def test_host_tensors_are_refused_at_the_abi():
    import torch

    from maddpg_amd.engine import Engine
    assert Engine._ptr(None).value is None
    with pytest.raises(ValueError, match="device tensors"):
        Engine._ptr(torch.zeros(4, dtype=torch.int32))
