"""Host-side sanitizer runs (CPU only): the engine's host C++ -- the SST walker
(csrc/sst.cc: parses untrusted file bytes), the log scanner / replay
(csrc/log_reader.cc), the host Extend (csrc/crc32c_host.cc) -- and the C-ABI
argument and error paths (csrc/crc32c_capi.hip, crc32c_multi.hip,
crc32c_pipeline.hip, host side), built by tools/sanitize/Makefile with

  * ASan + UBSan (no recovery, leak check on): a seeded mutation test over the
    reference-built SST (tests/golden/sst_small.ldb: bit flips, truncations,
    overlong / overflowing varints in the footer and index handles, byte
    splats) and the reference log cases (tests/golden/log_cases.bin), every
    mutant in an exactly-sized heap block; every entry point's EINVAL and
    (no device) EDEVICE paths.
  * TSan: the C ABI, the host Extend, the test hooks and the SST walker from 8
    threads at once (PrismDB's 8 partition threads).

Driven by tools/sanitize/harness.cc; a report or a failed check fails the
run.  Skipped when ROCm's clang is absent."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")
OUT = os.path.join(ROOT, "build", "sanitize")
GOLD = os.path.join(ROOT, "tests", "golden")

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang++"), reason="needs ROCm clang")


def _env(**kw):
    env = dict(os.environ)
    env.update(kw)
    return env


@pytest.fixture(scope="module")
def asan():
    subprocess.check_call(["make", "-s", "-j8", "-C", SAN, "asan"], stdout=subprocess.DEVNULL)
    return os.path.join(OUT, "asan", "harness")


@pytest.fixture(scope="module")
def tsan():
    subprocess.check_call(["make", "-s", "-j8", "-C", SAN, "tsan"], stdout=subprocess.DEVNULL)
    return os.path.join(OUT, "tsan", "harness")


def _run(cmd, **env):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(**env))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:abort_on_error=0",
            "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_asan_sst_mutations(asan, seed):
    out = _run([asan, "sst", os.path.join(GOLD, "sst_small.ldb"), "3000", str(seed)], **ASAN_ENV)
    assert "3000 mutants" in out
    listed, corrupt = int(out.split()[3]), int(out.split()[5])
    assert listed > 0 and corrupt > 0  # both outcomes exercised


def test_asan_log_mutations(asan):
    out = _run([asan, "log", os.path.join(GOLD, "log_cases.bin"), "200", "7"], **ASAN_ENV)
    assert "200 mutants" in out


def test_asan_abi_paths(asan):
    import torch

    mode = ["nodevice"] if not torch.cuda.is_available() else []
    assert "abi: ok" in _run([asan, "abi"] + mode, **ASAN_ENV)


def test_tsan_eight_threads(tsan):
    out = _run([tsan, "threads", "8", "200", os.path.join(GOLD, "sst_small.ldb")],
               TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    assert "0 failures" in out
