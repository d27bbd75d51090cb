"""Build libprismdb_crc32c.so in-tree with hipcc for gfx950.

    python -m prismdb_amd.build            # build (incremental on mtime)
    python -m prismdb_amd.build --asm      # also dump gfx950 assembly to build/asm/

The shared library holds the HIP kernels, the C ABI (include/prismdb_crc32c.h),
the per-call host surface (leveldb::crc32c::Extend) and the synthetic-data
generator.  It is built in-tree (prismdb_amd/lib/) so gpurun ships it to the
GPU box with the snapshot.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(LIBDIR, "libprismdb_crc32c.so")

ARCH = os.environ.get("PRISMDB_OFFLOAD_ARCH", "gfx950")
HIP_SOURCES = ["crc32c_kernels.hip", "crc32c_direct.hip", "crc32c_capi.hip", "crc32c_multi.hip", "crc32c_pipeline.hip", "synth.hip"]
CXX_SOURCES = ["crc32c_host.cc", "sst.cc", "log_reader.cc"]
HEADERS = ["crc32c_device.h", "crc32c_gf2.h", "crc32c_fold.h"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found; the MI355X engine cannot be built")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)


def build(force: bool = False, asm: bool = False, verbose: bool = False, defines: dict | None = None,
          lib_path: str | None = None, src_dir: str | None = None, obj_dir: str | None = None) -> str:
    """Build the library.  The product is the default; tools/variants.py
    builds measurement variants from a patched copy of the sources
    (`src_dir`, `obj_dir`, `lib_path`), never from knobs in the product
    source."""
    lib_out = lib_path or LIB
    csrc = src_dir or CSRC
    objdir = obj_dir or (OBJDIR if not defines else os.path.join(ROOT, "build", "obj_" + "_".join(
        f"{k}{v}" for k, v in sorted(defines.items()))))
    os.makedirs(os.path.dirname(lib_out), exist_ok=True)
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(csrc, h) for h in HEADERS] + [
        os.path.join(ROOT, "include", "prismdb_crc32c.h"),
        os.path.join(ROOT, "include", "prismdb_synth.h"),
        os.path.join(ROOT, "include", "prismdb_sst.h"),
        os.path.join(ROOT, "include", "prismdb_log.h"),
        os.path.join(ROOT, "include", "util", "crc32c.h"),
    ]
    common = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
    common += [f"-D{k}={v}" for k, v in sorted((defines or {}).items())]
    jobs = []
    objs = []
    for src in HIP_SOURCES + CXX_SOURCES:
        s = os.path.join(csrc, src)
        o = os.path.join(objdir, src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            if src.endswith(".hip"):
                cmd = [hipcc, "-x", "hip", f"--offload-arch={ARCH}", *common, "-c", s, "-o", o]
            else:
                cmd = [hipcc, "-x", "c++", *common, "-c", s, "-o", o]
            jobs.append(cmd)
    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        for cmd in jobs:
            if verbose:
                print(" ".join(cmd))
        list(ex.map(_run, jobs))
    exports = os.path.join(csrc, "exports.map")
    if force or jobs or _stale(lib_out, objs + [exports]):
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", f"-Wl,--version-script={exports}",
              "-o", lib_out, *objs, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    if asm:
        asmdir = os.path.join(ROOT, "build", "asm")
        os.makedirs(asmdir, exist_ok=True)
        for src in HIP_SOURCES:
            _run([hipcc, "-x", "hip", f"--offload-arch={ARCH}", *common, "--cuda-device-only", "-S",
                  os.path.join(csrc, src), "-o", os.path.join(asmdir, src + ".s")])
    return lib_out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asm", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, asm=args.asm, verbose=args.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
