"""Pin the oracle against the reference's own known answers and golden outputs.

KATs: util/crc32c_test.cc:12-53, util/crc32c.cc:269-273.  Golden vectors and
the SST fixture were produced by the reference itself (oracle/gen_golden.py).
"""
import numpy as np

from conftest import Oracle  # noqa: F401


def test_published_kats(oracle, golden):
    kat = golden["kat"]
    by_name = {v["name"]: v for v in kat["vectors"]}
    for name, want in kat["published"].items():
        data = bytes.fromhex(by_name[name]["hex"])
        assert oracle.value(data) == want, name
        assert oracle.extend_bitwise(0, data) == want, name


def test_all_kat_vectors_and_masks(oracle, golden):
    for v in golden["kat"]["vectors"]:
        data = bytes.fromhex(v["hex"])
        assert oracle.value(data) == v["value"], v["name"]
        assert oracle.mask(v["value"]) == v["masked"], v["name"]
        assert oracle.unmask(v["masked"]) == v["value"]
    e = golden["kat"]["extend"]
    assert oracle.extend(oracle.value(e["a"].encode()), e["b"].encode()) == e["extend_value"] == e["value"]
    # util/crc32c_test.cc:41 and :47-53
    assert oracle.value(b"a") != oracle.value(b"foo")
    c = oracle.value(b"foo")
    assert oracle.mask(c) != c and oracle.mask(oracle.mask(c)) != c
    assert oracle.unmask(oracle.unmask(oracle.mask(oracle.mask(c)))) == c


def test_sweep_vectors(oracle, golden):
    inp = golden["input"]
    rows = golden["vectors"]["rows"]
    assert len(rows) > 1500
    for off, n, init, crc, masked in rows:
        got = oracle.extend(init, inp[off:off + n])
        assert got == crc, (off, n, init)
        assert oracle.mask(got) == masked


def test_batch_matches_scalar(oracle, golden):
    buf = np.frombuffer(golden["input"], dtype=np.uint8).copy()
    rows = golden["vectors"]["rows"]
    off = [r[0] for r in rows]
    lens = [r[1] for r in rows]
    init = [r[2] for r in rows]
    out, _ = oracle.batch(buf, off, lens, init)
    assert out.tolist() == [r[3] for r in rows]
    outm, _ = oracle.batch(buf, off, lens, init, mask=True)
    assert outm.tolist() == [r[4] for r in rows]


def test_synth_stream_and_long_vectors(oracle, golden):
    # the fixture input.bin is the first 80 KiB of the seed-0x5EED0001 stream
    a = oracle.synth(len(golden["input"]), golden["vectors"]["seed"])
    assert a.tobytes() == golden["input"]
    # unaligned window of the stream equals the slice
    b = oracle.synth(1000, golden["vectors"]["seed"], 24)
    assert b.tobytes() == golden["input"][24:1024]
    for s in golden["stream"]:
        data = oracle.synth(s["len"] + s["byte_offset"] % 8, s["seed"], s["byte_offset"] - s["byte_offset"] % 8)
        data = data[s["byte_offset"] % 8:].tobytes()
        assert oracle.value(data) == s["crc"], s


def test_sst_fixture_trailers(oracle, golden):
    """Every block trailer written by the reference TableBuilder equals
    Mask(Value(contents || type)) (table/table_builder.cc:185-202)."""
    f = golden["sst_bytes"]
    assert len(f) == golden["sst"]["file_size"]
    for blk in golden["sst"]["blocks"]:
        o, n = blk["offset"], blk["size"]
        assert f[o + n] == blk["type"]
        stored = int.from_bytes(f[o + n + 1:o + n + 5], "little")
        assert stored == blk["masked_crc"]
        assert oracle.mask(oracle.value(f[o:o + n + 1])) == stored
    # footer magic (table/format.h:76)
    assert int.from_bytes(f[-8:], "little") == 0xDB4775248B80FB57


def test_oracle_verify_flags_corruption(oracle, golden):
    f = bytearray(golden["sst_bytes"])
    blocks = golden["sst"]["blocks"]
    off = [b["offset"] for b in blocks]
    lens = [b["size"] + 1 for b in blocks]  # contents || type
    buf = np.frombuffer(bytes(f), dtype=np.uint8).copy()
    _, mm = oracle.batch(buf, off, lens, verify=True)
    assert mm.sum() == 0
    victim = 5
    buf[blocks[victim]["offset"] + 100] ^= 0x80  # db/corruption_test.cc:152-154 style flip
    _, mm = oracle.batch(buf, off, lens, verify=True)
    assert mm.tolist() == [1 if i == victim else 0 for i in range(len(blocks))]
