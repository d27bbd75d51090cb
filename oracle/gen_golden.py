#!/usr/bin/env python3
"""Generate golden CRC32C vectors from the REFERENCE implementation.

TEST INFRASTRUCTURE ONLY.  Run in the build container (where /root/reference
exists) after `make -C oracle ref`:

    python oracle/gen_golden.py

It loads oracle/_ref/libref_crc32c.so (the reference util/crc32c.cc compiled
by oracle/Makefile, see ref_shim.cc) and writes data-only fixtures:

  tests/golden/kat.json             util/crc32c_test.cc:12-53 + util/crc32c.cc:269-273
  tests/golden/input.bin            80 KiB of synthetic bytes (splitmix64 stream)
  tests/golden/crc32c_vectors.json  [off, len, init, Extend(init, input[off:off+len]), Mask(.)]
  tests/golden/stream_vectors.json  long spans over the regenerable splitmix64 stream
  tests/golden/sst_small.ldb/.json  SST written and re-verified by the reference TableBuilder
  tests/golden/log_cases.bin/.json  log files written by the reference log::Writer (db/log_test.cc
                                    scenarios + seeded damage) and what log::Reader returns for them

The fixtures hold reference OUTPUTS only; no reference source travels with them.
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(ROOT, "tests", "golden")
SEED = 0x5EED0001
INPUT_LEN = 80 * 1024


def splitmix_stream(seed: int, nbytes: int, byte_offset: int = 0) -> bytes:
    """Bytes [byte_offset, byte_offset+nbytes) of the splitmix64 word stream
    (same definition as oracle/crc32c_oracle.c:oracle_fill_synthetic)."""
    import numpy as np

    w0 = byte_offset // 8
    w1 = (byte_offset + nbytes + 7) // 8
    k = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (k + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    raw = z.astype("<u8").tobytes()
    s = byte_offset - w0 * 8
    return raw[s : s + nbytes]


def main() -> int:
    lib_path = os.path.join(HERE, "_ref", "libref_crc32c.so")
    if not os.path.exists(lib_path):
        subprocess.check_call(["make", "-C", HERE, "ref"])
    ref = ctypes.CDLL(lib_path)
    ref.ref_crc32c_extend.restype = ctypes.c_uint32
    ref.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    ref.ref_crc32c_mask.restype = ctypes.c_uint32
    ref.ref_crc32c_mask.argtypes = [ctypes.c_uint32]

    def ext(init, data):
        return ref.ref_crc32c_extend(init, data, len(data))

    os.makedirs(GOLD, exist_ok=True)

    # --- KATs (inputs as hex, expected from the reference run here) ---
    iscsi = bytes([0x01, 0xC0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x14, 0, 0, 0, 0, 0, 0x04, 0,
                   0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0])
    kat_inputs = {
        "zeros32": bytes(32),
        "ones32": b"\xff" * 32,
        "inc32": bytes(range(32)),
        "dec32": bytes(range(31, -1, -1)),
        "iscsi48": iscsi,
        "TestCRCBuffer": b"TestCRCBuffer",
        "hello world": b"hello world",
        "a": b"a",
        "foo": b"foo",
        "empty": b"",
    }
    kat = {
        "source": "util/crc32c_test.cc:12-53, util/crc32c.cc:269-273; expected values computed by the reference",
        "published": {"zeros32": 0x8A9136AA, "ones32": 0x62A8AB43, "inc32": 0x46DD794E,
                      "dec32": 0x113FDB5C, "iscsi48": 0xD9963A56, "TestCRCBuffer": 0xDCBC59FA},
        "vectors": [{"name": k, "hex": v.hex(), "value": ext(0, v), "masked": ref.ref_crc32c_mask(ext(0, v))}
                    for k, v in kat_inputs.items()],
        "extend": {"a": "hello ", "b": "world", "extend_value": ext(ext(0, b"hello "), b"world"),
                   "value": ext(0, b"hello world")},
    }
    for name, want in kat["published"].items():
        got = ext(0, kat_inputs[name])
        assert got == want, (name, hex(got), hex(want))
    with open(os.path.join(GOLD, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    # --- sweep over a fixed input buffer ---
    buf = splitmix_stream(SEED, INPUT_LEN)
    with open(os.path.join(GOLD, "input.bin"), "wb") as f:
        f.write(buf)
    import random

    rng = random.Random(0x5EED0002)
    vecs = []
    for n in range(0, 131):
        for off in range(8):
            vecs.append((off, n, 0))
    special = [255, 256, 257, 1023, 1024, 1025, 3958, 3959, 3987, 3988, 3992, 4095, 4096, 4097,
               8192, 16383, 16384, 16385, 65535, 65536, 65537]
    for n in special:
        for off in range(8):
            vecs.append((off, n, 0))
            vecs.append((off, n, rng.getrandbits(32)))
    for _ in range(256):  # adversarial: random length, random byte offset, random init
        n = rng.randrange(0, 70000)
        off = rng.randrange(0, INPUT_LEN - n + 1)
        vecs.append((off, n, rng.getrandbits(32) if rng.random() < 0.5 else 0))
    rows = []
    for off, n, init in vecs:
        c = ext(init, buf[off : off + n])
        rows.append([off, n, init, c, ref.ref_crc32c_mask(c)])
    with open(os.path.join(GOLD, "crc32c_vectors.json"), "w") as f:
        json.dump({"seed": SEED, "input": "input.bin", "columns": ["off", "len", "init", "crc", "masked"],
                   "rows": rows}, f, separators=(",", ":"))

    # --- long spans over the regenerable stream (SST index-block sized) ---
    srows = []
    for seed, off, n in [(SEED, 0, 486977), (SEED, 3, 486976), (0x5EED0003, 12345, 1 << 20),
                         (0x5EED0004, 0, 3988 * 64)]:
        data = splitmix_stream(seed, n, off)
        srows.append({"seed": seed, "byte_offset": off, "len": n, "crc": ext(0, data)})
    with open(os.path.join(GOLD, "stream_vectors.json"), "w") as f:
        json.dump(srows, f, indent=1)

    # --- reference-built SST ---
    subprocess.check_call([os.path.join(HERE, "_ref", "sst_fixture"), os.path.join(GOLD, "sst_small.ldb"),
                           os.path.join(GOLD, "sst_small.json"), "64", "980", "4096"])
    # --- reference-written / reference-read log files ---
    subprocess.check_call([os.path.join(HERE, "_ref", "log_fixture"), os.path.join(GOLD, "log_cases")],
                          stderr=subprocess.DEVNULL)  # the reference reader traces every block read to stderr
    print(f"wrote {len(kat['vectors'])} KATs, {len(rows)} sweep vectors, {len(srows)} stream vectors")
    return 0


if __name__ == "__main__":
    sys.exit(main())
