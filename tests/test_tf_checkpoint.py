"""Offline TF checkpoint-V2 bundle reader/writer (influence/tf_checkpoint.py,
SURVEY.md 8f row 3).  The reference ships no checkpoint, so the format is pinned
by the CRC-32C check value and by write/read round trips; parity with real
reference checkpoints is unpinned."""
import numpy as np
import pytest


def test_crc32c_check_value_and_mask():
    from influence import tf_checkpoint as tfc
    assert tfc.crc32c(b"123456789") == 0xE3069283          # CRC-32C (Castagnoli) check value
    assert tfc.crc32c(b"") == 0
    c = tfc.crc32c(b"influence")
    assert tfc.mask(c) != c


def test_round_trip_reference_names(tmp_path):
    from influence import tf_checkpoint as tfc
    rng = np.random.default_rng(0)
    names = ["embedding_layer/embedding_users", "embedding_layer/embedding_items", "embedding_layer/bias_users",
             "embedding_layer/bias_items", "embedding_layer/global_bias"]
    t = {n: rng.standard_normal(s).astype(np.float32) for n, s in zip(names, [600, 480, 60, 40, 1])}
    for n in names:
        t[n + "/Adam"] = rng.standard_normal(t[n].shape).astype(np.float32)
        t[n + "/Adam_1"] = np.abs(rng.standard_normal(t[n].shape)).astype(np.float32)
    t["beta1_power"] = np.float32(0.9 ** 50)
    t["beta2_power"] = np.float32(0.999 ** 50)
    t["global_step"] = np.int64(49)
    t["h1/weights"] = rng.standard_normal((32, 16)).astype(np.float64)
    prefix = str(tmp_path / "m-checkpoint-49")
    tfc.write_checkpoint(prefix, t)
    got = tfc.read_checkpoint(prefix)
    assert set(got) == set(t)
    for n in t:
        assert got[n].dtype == np.asarray(t[n]).dtype and np.array_equal(got[n], t[n]), n
    lv = dict((n, s) for n, s, _ in tfc.list_variables(prefix))
    assert lv["h1/weights"] == (32, 16) and lv["global_step"] == ()
    # small blocks: many data blocks, prefix-compressed keys across restart points
    tfc.write_index(str(tmp_path / "t.index"), [(("k%05d" % i).encode(), bytes([i % 251]) * (i % 7))
                                               for i in range(400)], block_bytes=64)
    ent = tfc.read_index(str(tmp_path / "t.index"))
    assert [k for k, _ in ent] == [("k%05d" % i).encode() for i in range(400)]
    assert all(v == bytes([i % 251]) * (i % 7) for i, (_, v) in enumerate(ent))


def test_corruption_is_detected(tmp_path):
    from influence import tf_checkpoint as tfc
    prefix = str(tmp_path / "c")
    tfc.write_checkpoint(prefix, {"a": np.arange(100, dtype=np.float32)})
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[17] ^= 0x40
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError):
        tfc.read_checkpoint(prefix)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[-1] ^= 1
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(ValueError):
        tfc.read_checkpoint(prefix)
