#!/usr/bin/env python3
"""Headline benchmark: batched CRC32C over device-resident 4 KiB SST blocks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--nblocks B] [--strong] [--no-gather] [--e2e]

Workload (BASELINE.json configs[1], "config 2"): per GPU, 16 Mi blocks x 4096 B
(64 GiB) generated on the device from the splitmix64 stream, stride 4096,
base 256-B aligned.  One step = one pass of the engine over the whole batch
(leveldb_crc32c_batch_fixed, one persistent kernel launch) and, for N > 1, an
RCCL gather of the 4-byte results to rank 0 (overlapped with the next pass on
RCCL's own stream; the last one is inside the timed region).
N > 1 runs one process per GPU under torch.distributed.run (weak scaling: each
rank owns a different 64 GiB slice of the global block stream).  Started as
`python bench.py --gpus N` without a launcher (no WORLD_SIZE), bench starts
torch.distributed.run itself with N ranks before anything touches the GPU and
exits with its status; a WORLD_SIZE that disagrees with --gpus is an error.
--strong keeps the total fixed instead (--nblocks blocks in all, nblocks / N
per rank), and --no-gather drops the RCCL gather
(config 5 asks for both).

Printed (rank 0): ONE JSON line with the driver's contract fields plus
  roofline      dominant kernel vs the HBM roofline (HIP events on the launch stream)
  cpu_baseline  the reference crc32c::Value (util/crc32c.cc compiled to
                oracle/_ref/) on this host's cores over a bounded sample of the
                same blocks, also cross-checked bit for bit against the GPU results
  e2e           (with --e2e) host-resident rate incl. pinned H2D/D2H copies
  config5_partitions
                BASELINE configs[4]: each rank one PrismDB partition of ~2.4 M
                SST block spans (143 files), sealed and verified file by file
                through the descriptor path, results gathered to rank 0 over
                RCCL (N > 1); its own GiB/s, never the headline value
                (--no-config5 skips it)
  config5_one_process
                the same partitions from ONE process (rank 0) through
                leveldb_crc32c_batch_multi over all N devices: PrismDB's shape,
                8 partition threads of one process (db/db_impl.h:359,
                util/env_posix.cc:850-890); one RCCL clique of N devices
                (ncclCommInitAll), results gathered to device 0 over xGMI;
                per device its batch and gather times (HIP events on the
                clique streams), each partition's host enqueue start and
                duration, and the clique's ncclCommInitAll wall time
                (--no-multi skips it; at N = 1, --multi-devices picks the
                device count, default 1)
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# (The measured process runs with the library's test hooks off: every leg
# takes the default routes a PrismDB caller gets.  tools/bench_configs.py
# times pinned routes side by side.)

METRIC = "GiB/s CRC32C over device-resident 4 KiB SST blocks; bit-exact vs util/crc32c.cc"
SEED = 0x5EED0001
BLOCK = 4096
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nblocks", type=int, default=1 << 24, help="4 KiB blocks per GPU (--strong: in total)")
    ap.add_argument("--strong", action="store_true", help="strong scaling: --nblocks is the total over all ranks")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: no RCCL gather of the results")
    ap.add_argument("--cpu-sample-blocks", type=int, default=1 << 18)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-seconds of reference work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also measure the host-resident (pinned copy) rate")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 partition leg")
    ap.add_argument("--c5-spans", type=int, default=2_400_000, help="config-5 spans per partition (GPU)")
    # (20, as the headline's steps: at 5 the first call's launch latency and
    # the closing synchronisation were ~1.5 % of a one-process config-5 round)
    ap.add_argument("--c5-steps", type=int, default=20)
    ap.add_argument("--c5-files-per-call", default="7,11,12",
                    help="config-5 compaction legs: SST files per leveldb_crc32c_batch call (comma list; 7 files "
                         "are the most one launch takes below 2^17 spans, 11 the most a sealing or verifying batch "
                         "takes in one launch on 256 CUs, 12 a compaction's input set: 1 file + ~11 overlapping)")
    ap.add_argument("--no-multi", action="store_true", help="skip the one-process batch_multi leg")
    ap.add_argument("--multi-timeout", type=float, default=240.0,
                    help="seconds the batch_multi leg's child process may take before it is stopped")
    ap.add_argument("--multi-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--multi-devices", type=int, default=0,
                    help="at --gpus 1: devices of the one-process batch_multi leg (default 1)")
    ap.add_argument("--cpu-all-blocks", type=int, default=1 << 20,
                    help="cpu_baseline all-cores figure: blocks (config 1: 1 Mi x 4 KiB)")
    return ap.parse_args()


def affinity() -> list:
    return sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))


def cpu_threads() -> int:
    """Threads for the CPU baseline: the cores this process may run on,
    bounded by OMP_NUM_THREADS (16 on the GPU box: its share of the host)."""
    n = len(affinity())
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


def cpu_quota():
    """CPUs the process's cgroup lets it use (CFS quota / period, rounded up;
    the tightest level of its hierarchy), or None without a quota.  cgroup v2
    (cpu.max) and v1 (cpu.cfs_quota_us / cpu.cfs_period_us)."""
    best = None
    try:
        with open("/proc/self/cgroup") as f:
            lines = [ln.strip().split(":", 2) for ln in f if ln.strip()]
    except OSError:
        return None
    for _, ctrl, path in lines:
        if ctrl == "":
            base, files = "/sys/fs/cgroup", ("cpu.max",)
        elif "cpu" in ctrl.split(","):
            base, files = "/sys/fs/cgroup/cpu", ("cpu.cfs_quota_us", "cpu.cfs_period_us")
        else:
            continue
        parts = [p for p in path.split("/") if p]
        for k in range(len(parts), -1, -1):  # the cgroup and each ancestor
            d = os.path.join(base, *parts[:k])
            try:
                if len(files) == 1:
                    with open(os.path.join(d, files[0])) as f:
                        q, per = f.read().split()[:2]
                else:
                    with open(os.path.join(d, files[0])) as f:
                        q = f.read().strip()
                    with open(os.path.join(d, files[1])) as f:
                        per = f.read().strip()
            except (OSError, ValueError):
                continue
            if q in ("max", "-1") or int(per) <= 0:
                continue
            n = max(1, -(-int(q) // int(per)))
            best = n if best is None else min(best, n)
    return best


def all_core_threads():
    """Threads for the config-1 "all host cores" figure: the CPUs the process
    may actually use -- its affinity set, bounded by its cgroup CPU quota, else
    by OMP_NUM_THREADS (the box's CPU share for one GPU).  Threads beyond the
    quota only time-slice: round 4 ran 256 threads on a 16-CPU share and
    measured 47.8 GiB/s against 220.4 on 16."""
    n = len(affinity())
    q = cpu_quota()
    if q is not None:
        return min(n, q), f"cgroup CPU quota {q}, affinity {n}"
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        return min(n, int(env)), f"no cgroup quota; OMP_NUM_THREADS {env}, affinity {n}"
    return n, f"no cgroup quota; affinity {n}"


def _ranges(cpus: list) -> str:
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(f"{cpus[i]}-{cpus[j]}" if j > i else f"{cpus[i]}")
        i = j + 1
    return ",".join(out)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_leg(args, gpu_out, dev_buf) -> dict | None:
    """Reference crc32c::Value timed on the host cores over the first
    cpu_sample_blocks blocks of rank 0's shard (regenerated on the host by the
    oracle's splitmix64 fill); results compared with the GPU.  Plus the
    config-1 figure: 1 Mi x 4 KiB on every core of the affinity
    set, over the device's own bytes copied to the host."""
    import numpy as np

    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    ora_so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(ora_so):
        return None
    ora = ctypes.CDLL(ora_so)
    ora.oracle_fill_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
    nblk = min(args.cpu_sample_blocks, args.nblocks)
    host = np.empty(nblk * BLOCK, dtype=np.uint8)
    ora.oracle_fill_synthetic(host.ctypes.data, host.nbytes, SEED, 0)
    out = np.empty(nblk, dtype=np.uint32)
    threads = cpu_threads()
    if os.path.exists(ref_so):
        kind = "reference"
        lib = ctypes.CDLL(ref_so)
        lib.ref_crc32c_time_blocks.restype = ctypes.c_double
        lib.ref_crc32c_time_blocks.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        accel = int(lib.ref_crc32c_accelerated())

        def run(t, p, arr=host, o=out, nb=nblk):
            return lib.ref_crc32c_time_blocks(arr.ctypes.data, BLOCK, BLOCK, nb, t, p, o.ctypes.data)
    else:
        # oracle/_ref/ (the reference compiled from /root/reference, shipped
        # with the snapshot) is missing: time the C restatement instead, and
        # say so in the line (kind "port", a warning on stderr)
        print("warning: oracle/_ref/libref_crc32c.so is missing; cpu_baseline times the oracle port (kind=port)",
              file=sys.stderr)
        kind = "port"
        accel = 0
        ora.oracle_crc32c_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                                  ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        threads = 1

        def run(t, p, arr=host, o=out, nb=nblk):
            t0 = time.perf_counter()
            for _ in range(p):
                ora.oracle_crc32c_batch_fixed(arr.ctypes.data, BLOCK, BLOCK, nb, 0, o.ctypes.data, 0)
            return time.perf_counter() - t0

    t1 = run(1, 1)  # single-thread calibration pass
    rate1 = nblk * BLOCK / t1 / GIB
    # one pass costs ~t1 CPU-seconds whatever the thread count: aim at cpu_seconds in total
    passes = max(1, int(round(args.cpu_seconds / max(t1, 1e-6))))
    tn = run(threads, passes)
    rate = nblk * BLOCK * passes / tn / GIB
    g = gpu_out[:nblk].cpu().numpy().view(np.uint32)
    agree = int((g == out).sum())
    cpus = affinity()
    res = {
        "value": round(rate, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
        "host_cores_total": os.cpu_count(),
        "affinity": {"count": len(cpus), "cpus": _ranges(cpus)},
        "kind_note": ("the reference's util/crc32c.cc compiled from /root/reference (oracle/_ref/)"
                      if kind == "reference" else
                      "PORT: oracle/_ref/ missing -- the oracle's C restatement on 1 thread, not the reference"),
        "sample": (f"crc32c::Value over the first {nblk} x 4096 B blocks of the same splitmix64 stream "
                   f"(host-resident, {nblk * BLOCK / GIB:.2f} GiB), {passes} passes on {threads} threads "
                   f"(~{tn * threads:.1f} CPU-s); 1 thread: {rate1:.3f} GiB/s"),
        "single_thread_value": round(rate1, 3),
        "path": "HAVE_CRC32C (libcrc32c)" if accel else "portable slicing-by-4 (util/crc32c.cc:276-377)",
        "cpu_model": cpu_model(),
        "agrees_with_gpu": f"{agree}/{nblk}",
    }
    # config 1 as SURVEY 8(d) states it: 1 Mi x 4 KiB at all host cores --
    # the CPUs this process may use (all_core_threads), bytes from the device
    # buffer (the same stream)
    nall = min(args.cpu_all_blocks, args.nblocks)
    if kind == "reference" and nall > 0:
        big = dev_buf[:nall * BLOCK].cpu().numpy()
        oall = np.empty(nall, dtype=np.uint32)
        nthr, why = all_core_threads()
        t_one = max(run(nthr, 1, big, oall, nall), 1e-6)  # one calibration pass
        p_all = max(1, min(64, int(round(2.0 / t_one))))  # ~2 s
        ta = run(nthr, p_all, big, oall, nall)
        ga = gpu_out[:nall].cpu().numpy().view(np.uint32)
        res["all_cores"] = {
            "value": round(nall * BLOCK * p_all / ta / GIB, 3), "unit": "GiB/s", "threads": nthr,
            "threads_from": why,
            "blocks": nall, "passes": p_all, "wall_s": round(ta, 3),
            "sample": f"config 1: crc32c::Value over {nall} x 4096 B host-resident blocks on all {nthr} CPUs "
                      f"this process may use ({why})",
            "agrees_with_gpu": f"{int((ga == oall).sum())}/{nall}",
        }
        del big
    return res


def load_pmc_traffic(nblocks: int):
    """HBM bytes per launch of the span kernel from the committed PMC profile
    (profiles/*pmc*.json, written by tools/pmc_summary.py), if it matches."""
    best = None  # the newest match: rNN round, then the run tag (r05ab after r05g after r05a)

    def order(p):
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(p))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, p)

    paths = glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "*", "*pmc*.json"))
    for p in sorted(paths, key=order):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("nblocks") == nblocks and d.get("hbm_bytes_per_launch"):
            best = dict(d, _path=os.path.relpath(p, ROOT))
    return best


def e2e_leg(args, torch, crc32c, dev) -> dict:
    """Host-resident rate through leveldb_crc32c_batch_host: 4 KiB blocks in
    host memory streamed H2D -> CRC -> results D2H in 64 MiB chunks, 4 in
    flight on separate copy and compute streams.  Measured for a pinned source (direct DMA) and a pageable one
    (staged through the engine's pinned ring), next to the plain pinned H2D
    copy rate of the same bytes.  Never the headline value."""
    import numpy as np

    nblk = 1 << 19  # 2 GiB of 4 KiB blocks
    tmp = torch.empty(nblk * BLOCK, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(tmp, SEED)
    pinned = tmp.cpu().pin_memory()
    pageable = pinned.numpy().copy()
    off = np.arange(nblk, dtype=np.uint64) * BLOCK
    lens = np.full(nblk, BLOCK, dtype=np.uint32)
    ref, _ = crc32c.batch_fixed(tmp, BLOCK, BLOCK, nblk)
    ref = ref.cpu().numpy().view(np.uint32)
    res = {"bytes": nblk * BLOCK, "chunk": "64 MiB per DMA, 4 in flight, copy and compute streams",
           "reps": 3, "stat": "best of reps"}
    for name, src in (("pinned", pinned), ("pageable", pageable)):
        crc32c.batch_host(src, off[:16384], lens[:16384])  # warm the ring
        best, exact = 0.0, True
        for _ in range(3):
            t0 = time.perf_counter()
            got, _ = crc32c.batch_host(src, off, lens)
            best = max(best, nblk * BLOCK / (time.perf_counter() - t0) / GIB)
            exact = exact and bool((got == ref).all())
        res[name] = round(best, 2)
        res[name + "_bit_exact"] = exact
    d = torch.empty_like(tmp)
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nblk * BLOCK / (time.perf_counter() - t0) / GIB)
    res["h2d_copy_only"] = round(best, 2)
    res["unit"] = "GiB/s"
    del tmp, d, pinned, pageable
    res["config4_compaction"] = compaction_leg(torch, crc32c, dev)
    return res


def compaction_leg(torch, crc32c, dev, nfiles: int = 115) -> dict:
    """BASELINE config 4 restated (db_bench cannot build here): the block CRC
    work of a 10 GB YCSB-A run's compactions, host-resident and end to end.
    scripts/config_test_10gb.yml puts ~7.7 GB on flash: ~115 SSTs of 64 MiB,
    each 16 811 data blocks of 3987 B + type byte + 4-byte crc (stride 3992,
    table/table_builder.cc:185-202) and one 486 976-B index block.  The files
    sit in pageable host memory, like ReadBlock's heap buffers
    (table/format.cc:75-79).
      read  (input SSTs)  ReadBlock verify of every block: Unmask(stored) ==
                          Value(contents||type)  (table/format.cc:93-101)
      write (output SSTs) WriteRawBlock's Mask(Value(contents||type)) for every
                          block, stored into the 5-byte trailers by the engine
                          (batch_host with WRITE_TRAILER)
    Both through leveldb_crc32c_batch_host; GiB/s of block bytes incl. all
    copies.  Never the headline value."""
    import numpy as np

    ndata, data_n, stride, index_n = 16811, 3987, 3992, 486976
    file_bytes = ndata * stride + index_n + 5
    g = torch.empty(file_bytes + 8, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(g, SEED ^ 0xC0)
    off1 = np.concatenate([np.arange(ndata, dtype=np.int64) * stride, [ndata * stride]])
    len1 = np.concatenate([np.full(ndata, data_n + 1, dtype=np.int64), [index_n + 1]])
    g[torch.from_numpy(off1 + len1 - 1).to(dev)] = 0  # type byte: kNoCompression
    d_off = torch.from_numpy(off1).to(dev)
    d_len = torch.from_numpy(len1.astype(np.int32)).to(dev)
    crc32c.batch(g, d_off, d_len, mask=True, trailer=True)  # sealed on the device once
    one = g[:file_bytes].cpu().numpy()
    del g, d_off, d_len
    img = np.empty(nfiles * file_bytes, dtype=np.uint8)
    img.reshape(nfiles, file_bytes)[:] = one
    off = (np.arange(nfiles, dtype=np.uint64)[:, None] * file_bytes + off1.astype(np.uint64)[None, :]).reshape(-1)
    lens = np.tile(len1.astype(np.uint32), nfiles)
    tr = (off + lens).astype(np.int64)[:, None] + np.arange(4)[None, :]
    want = img[tr].copy()
    nbytes = int(lens.sum()) + 4 * len(lens)
    crc32c.batch_host(img, off[:20000], lens[:20000], verify=True)  # warm the ring
    res = {"files": nfiles, "blocks": int(len(off)), "block_bytes": nbytes, "source": "pageable",
           "reps": 3, "stat": "best of reps"}
    best, clean = 0.0, True
    for _ in range(3):
        t0 = time.perf_counter()
        _, mm = crc32c.batch_host(img, off, lens, verify=True)
        best = max(best, nbytes / (time.perf_counter() - t0) / GIB)
        clean = clean and int(mm.sum()) == 0
    res["read_verify"] = round(best, 2)
    res["read_all_blocks_verified"] = clean
    # the engine stores each block's trailer into the host image as it seals
    # (WRITE_TRAILER: 4 LE bytes behind each block, table/table_builder.cc:192-197),
    # chunk by chunk while the next chunks are in flight
    best, exact = 0.0, True
    for _ in range(3):
        img[tr] = 0
        t0 = time.perf_counter()
        crc32c.batch_host(img, off, lens, mask=True, trailer=True)
        best = max(best, nbytes / (time.perf_counter() - t0) / GIB)
        exact = exact and bool((img[tr] == want).all())
    res["write_seal"] = round(best, 2)
    res["write_trailers_match_reference_layout"] = exact
    res["unit"] = "GiB/s"
    return res


C5_ND, C5_DATA, C5_STRIDE, C5_INDEX = 16811, 3988, 3992, 486977  # one 64 MiB SST


def _c5_descriptors(nfiles: int):
    """Descriptors of nfiles consecutive SST files of the config-5 layout
    (file f at f * fbytes): offsets, lengths, type-byte positions."""
    import numpy as np

    fbytes = (C5_ND * C5_STRIDE + C5_INDEX + 4 + 255) & ~255
    off1 = np.concatenate([np.arange(C5_ND, dtype=np.int64) * C5_STRIDE, [C5_ND * C5_STRIDE]])
    len1 = np.concatenate([np.full(C5_ND, C5_DATA, dtype=np.int64), [C5_INDEX]])
    off = (np.arange(nfiles, dtype=np.int64)[:, None] * fbytes + off1[None, :]).reshape(-1)
    lens = np.tile(len1, nfiles)
    return fbytes, off, lens, off + lens - 1


def config5_leg(args, torch, dist, crc32c, dev, rank, world) -> dict:
    """BASELINE configs[4] (scripts/config_test_100gb.yml): 8 partitions, ~19.3 M
    block spans, partition p on GPU p -- ~2.4 M spans per GPU, here as the SST
    files that partition's compactions write: nfiles x (16 811 data spans of
    contents||type = 3988 B at stride 3992 + one 486 977-B index span), device-
    resident.  One step = every file of the partition, then (N > 1) one RCCL
    gather of the partition's 4-byte results to rank 0.  Two granularities:
      per file        one leveldb_crc32c_batch per file -- TableBuilder::Finish
                      seals a file (table/table_builder.cc:185-261), ReadBlock
                      verifies a block at a time (table/format.cc:91-102)
      per compaction  one call per --c5-files-per-call files: a compaction's
                      input set verified together (db/version_set.cc:1265-1300
                      opens them as one merging iterator), or its output files
                      sealed together
    Seal = MASK | WRITE_TRAILER (trailers written in place), verify = the
    mismatch vector.  GiB/s of span bytes, whole job (all ranks), max-over-
    ranks timing between barriers.  Checks: verify after seal flags nothing
    and returns the unmasked seal results; 256 spans of file 0 against the
    host leveldb_crc32c_value; the gathered digests."""
    import numpy as np
    from prismdb_amd._lib import lib
    from prismdb_amd.dist import ShardedBatch

    spf = C5_ND + 1
    nfiles = -(-args.c5_spans // spf)
    span_bytes = C5_ND * C5_DATA + C5_INDEX
    fbytes, off_all, len_all, typ = _c5_descriptors(nfiles)
    off1, len1 = off_all[:spf], len_all[:spf]
    buf = torch.empty(nfiles * fbytes, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED ^ 0xC5C5, byte_offset=rank * nfiles * fbytes)
    buf[torch.from_numpy(typ).to(dev)] = 0  # type byte kNoCompression
    kpcs = sorted({max(1, min(int(k), nfiles)) for k in str(args.c5_files_per_call).split(",") if k.strip()})
    kmax = max(kpcs + [1])
    d_off = torch.from_numpy(off_all[:kmax * spf].copy()).to(dev)  # kmax consecutive files from file 0
    d_len = torch.from_numpy(len_all[:kmax * spf].astype(np.int32)).to(dev)
    n = nfiles * spf
    out = torch.empty(n, dtype=torch.int32, device=dev)
    raw = torch.empty(n, dtype=torch.int32, device=dev)
    mm = torch.empty(n, dtype=torch.uint8, device=dev)
    L = lib()
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    base, op, lp = buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr()

    def run(verify, k):
        o = raw.data_ptr() if verify else out.data_ptr()
        fl = 0 if verify else 0x3  # seal: MASK | WRITE_TRAILER
        for f in range(0, nfiles, k):
            m = min(k, nfiles - f) * spf
            rc = L.leveldb_crc32c_batch(base + f * fbytes, op, lp, None, m, o + 4 * f * spf,
                                        (mm.data_ptr() + f * spf) if verify else None, fl, sp)
            if rc != 0:
                raise RuntimeError(f"leveldb_crc32c_batch: {L.leveldb_crc32c_last_error().decode()}")

    shard = ShardedBatch(nblocks_per_rank=n, block_bytes=0, rank=rank, world=world, device=dev, slots=1) \
        if world > 1 else None

    def leg(verify, k):
        res = out if not verify else raw
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.c5_steps)]
        for _ in range(2):
            run(verify, k)
            if shard:
                shard.gather_async(res, 0).wait()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.c5_steps):
            ev[i][0].record(stream)
            run(verify, k)
            ev[i][1].record(stream)
            if shard:
                shard.gather_async(res, 0).wait()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = sum(a.elapsed_time(b) for a, b in ev) / args.c5_steps
        t = torch.tensor([el, kern], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern = float(t[0]), float(t[1])
        calls = -(-nfiles // k)
        d = {"value": round(world * nfiles * span_bytes * args.c5_steps / el / GIB, 2), "unit": "GiB/s",
             "ms_per_step": round(el * 1e3 / args.c5_steps, 3),
             "batch_ms_per_step_max_rank": round(kern, 3),
             "files_per_call": k, "calls_per_step": calls,
             "us_per_call": round(kern * 1e3 / calls, 2),
             "us_per_file": round(kern * 1e3 / nfiles, 2),
             "roofline_frac_per_gpu": round(nfiles * (span_bytes + 4 * spf) / (kern / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        if shard:
            d["gather_check"] = shard.check_gathered(res, 0)
        return d

    seal = leg(False, 1)
    verify = leg(True, 1)
    comp = {str(k): {"seal": leg(False, k), "verify": leg(True, k)} for k in kpcs}
    torch.cuda.synchronize()
    bad = int(mm.sum().item())
    unmasked = (out.to(torch.int64) & 0xFFFFFFFF) - 0xA282EAD8
    unmasked = unmasked & 0xFFFFFFFF
    unmasked = ((unmasked >> 17) | (unmasked << 15)) & 0xFFFFFFFF  # Unmask (util/crc32c.h:34-37)
    same = bool(torch.equal(unmasked, raw.to(torch.int64) & 0xFFFFFFFF))
    host0 = buf[:fbytes].cpu().numpy()
    pick = np.random.default_rng(rank).choice(spf, size=min(256, spf), replace=False)
    r0 = raw[:spf].cpu().numpy().view(np.uint32)
    host_ok = all(crc32c.Value(host0[off1[i]:off1[i] + len1[i]].tobytes()) == int(r0[i]) for i in pick)
    del buf, out, raw, mm
    return {
        "workload": (f"config5: partition {rank} of {world} on GPU {rank}: {nfiles} SST files x ({C5_ND} x "
                     f"{C5_DATA} B @ {C5_STRIDE} + 1 x {C5_INDEX} B) = {n} spans per GPU, one "
                     "leveldb_crc32c_batch per file (seal, verify) or per k files (compaction[k])"
                     + (", RCCL gather of the results to rank 0" if world > 1 else "")),
        "files_per_gpu": nfiles, "spans_per_gpu": n, "span_bytes_per_gpu": nfiles * span_bytes,
        "steps": args.c5_steps, "scaling": "weak",
        "seal": seal, "verify": verify, "compaction": comp,
        "checks": {"verify_after_seal_mismatches": bad, "verify_equals_unmasked_seal": same,
                   "host_value_256_spans_file0": host_ok},
    }


def multi_leg(args, torch, crc32c, ndev: int) -> dict:
    """Config 5 from ONE process, PrismDB's own shape (its 8 partitions are
    threads of one process, db/db_impl.h:359, util/env_posix.cc:850-890):
    partition p = the config-5 SST files of partition p, resident on device p;
    one leveldb_crc32c_batch_multi call per step seals every partition on its
    own device and gathers the 4-byte results to device 0 over RCCL (one
    clique of ndev devices, ncclCommInitAll).  Timed next to the same
    per-device batches issued without the gather.  Checks: the gathered
    vector equals the per-device results concatenated; a verify pass over
    the sealed partitions flags nothing."""
    import numpy as np

    spf = C5_ND + 1
    nfiles = -(-args.c5_spans // spf)
    span_bytes = C5_ND * C5_DATA + C5_INDEX
    fbytes, off_all, len_all, typ = _c5_descriptors(nfiles)
    n = nfiles * spf
    parts, streams = [], []
    for p in range(ndev):
        d = torch.device("cuda", p)
        with torch.cuda.device(d):
            crc32c.device_init(p)
            buf = torch.empty(nfiles * fbytes, dtype=torch.uint8, device=d)
            crc32c.fill_synthetic(buf, SEED ^ 0xC5C5, byte_offset=p * nfiles * fbytes)
            buf[torch.from_numpy(typ).to(d)] = 0
            parts.append((buf, torch.from_numpy(off_all).to(d), torch.from_numpy(len_all.astype(np.int32)).to(d)))
            streams.append(torch.cuda.current_stream(d))
    root = torch.device("cuda", 0)
    out = torch.empty(ndev * n, dtype=torch.int32, device=root)
    mm = torch.empty(ndev * n, dtype=torch.uint8, device=root)
    sep = [torch.empty(n, dtype=torch.int32, device=torch.device("cuda", p)) for p in range(ndev)]

    def sync_all():
        for p in range(ndev):
            torch.cuda.synchronize(p)

    def gathered():
        crc32c.batch_multi(parts, mask=True, trailer=True, out=out, streams=streams, check_bounds=False)

    def separate():
        for p in range(ndev):
            with torch.cuda.device(p):
                crc32c.batch(*parts[p], mask=True, trailer=True, out=sep[p], stream=streams[p], check_bounds=False)

    res = {"devices": ndev, "clique": ndev, "files_per_device": nfiles, "spans_per_device": n,
           "steps": args.c5_steps, "call": "one leveldb_crc32c_batch_multi per step: every partition sealed "
           "(MASK | WRITE_TRAILER) on its device, results gathered to device 0"}
    # Three rounds of c5_steps steps per leg, the legs alternating (a leg
    # timed right after the other ran up to 10 % apart from run to run; the
    # per-call hand-offs cost ~2 %: tools/multi_ab.py, profiles/r05/r05an_multi_ab.json);
    # each leg's median round.
    legs = (("with_gather", gathered), ("without_gather", separate))
    for _, fn in legs:
        fn()
    sync_all()
    rounds = {name: [] for name, _ in legs}
    for r in range(3):
        for name, fn in (legs if r % 2 == 0 else legs[::-1]):
            t0 = time.perf_counter()
            for _ in range(args.c5_steps):
                fn()
            sync_all()
            rounds[name].append(time.perf_counter() - t0)
    for name, fn in legs:
        el = sorted(rounds[name])[1]
        res[name] = {"value": round(ndev * nfiles * span_bytes * args.c5_steps / el / GIB, 2), "unit": "GiB/s",
                     "ms_per_step": round(el * 1e3 / args.c5_steps, 3), "rounds": 3, "stat": "median round"}
        if name == "with_gather":
            # the timing diagnostics below read the second call's phases: it is
            # enqueued while the first runs, as in the timed steps (a call made
            # right after a synchronisation took ~3x the host time)
            fn()
            fn()
            sync_all()
            # the last step's phases on each device (HIP events on the clique
            # streams) and the clique's one-time ncclCommInitAll
            tm = crc32c.multi_timing(list(range(ndev)))
            if tm is not None:
                res["init_ms_ncclCommInitAll"] = tm["init_ms"]
                res[name]["per_device_batch_ms"] = tm["batch_ms"]
                res[name]["per_device_gather_ms"] = tm["gather_ms"]
                res[name]["per_device_GiB_s"] = [round(nfiles * span_bytes / (b / 1e3) / GIB, 1) if b > 0 else None
                                                 for b in tm["batch_ms"]]
            # the same call's host side: when each partition's enqueue started
            # (partitions > 0 on their devices' worker threads) and how long it took
            ht = crc32c.multi_host_timing(list(range(ndev)))
            if ht is not None:
                res[name]["host_enqueue_start_us"] = ht["start_us"]
                res[name]["host_enqueue_us"] = ht["enqueue_us"]
                res[name]["host_call_us"] = ht["call_us"]
    want = torch.cat([t.to(root) for t in sep])
    res["gather_check"] = {"gathered_equals_per_device": bool(torch.equal(out, want)), "entries": int(out.numel())}
    crc32c.batch_multi(parts, verify=True, out=out, mismatch=mm, streams=streams, check_bounds=False)
    sync_all()
    res["verify_after_seal_mismatches"] = int(mm.sum().item())
    del parts, sep, out, mm
    for p in range(ndev):
        with torch.cuda.device(p):
            torch.cuda.empty_cache()
    return res


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks under
    torch.distributed.run from this process, which never touches the GPU
    (no HIP call before the children exist, no exec after one), and return
    their status.  The ranks' rank 0 prints the JSON line."""
    import torch

    have = torch.cuda.device_count()  # counts devices without initialising HIP on this image
    if have and args.gpus > have:
        print(f"error: --gpus {args.gpus} but only {have} devices are visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: no WORLD_SIZE; launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def run_multi_child(args, ndev: int) -> dict:
    """The batch_multi leg in a child process of its own, under a time limit:
    it drives every device through one RCCL clique, and a hang or a fault
    there must not cost the line whose headline was already measured.  (A
    child process, not an exec: this process has initialised the GPU.)"""
    cmd = [sys.executable, os.path.abspath(__file__), "--multi-child", "--multi-devices", str(ndev),
           "--c5-spans", str(args.c5_spans), "--c5-steps", str(args.c5_steps)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.multi_timeout)
    except subprocess.TimeoutExpired:
        return {"devices": ndev, "error": f"batch_multi leg stopped after {args.multi_timeout:.0f} s"}
    for line in reversed(r.stdout.splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                break
    return {"devices": ndev, "error": f"batch_multi child exited {r.returncode}: {r.stderr.strip()[-400:]}"}


def main() -> int:
    args = parse()
    if args.multi_child:  # bench's own child (run_multi_child): the batch_multi leg alone
        import torch

        from prismdb_amd import crc32c

        try:
            res = multi_leg(args, torch, crc32c, args.multi_devices)
        except Exception as e:
            res = {"devices": args.multi_devices, "error": f"{type(e).__name__}: {e}"}
        print(json.dumps(res), flush=True)
        return 0
    # The launch mode is settled before anything touches the GPU.
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        return spawn_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure another world size",
              file=sys.stderr)
        return 2
    if os.environ.get("PRISMDB_BENCH_DRYRUN"):  # tests: the launch alone, no GPU
        # one write(2): lines of concurrent ranks never interleave
        os.write(1, (json.dumps({"dryrun": True, "rank": rank, "world": world, "local_rank": local}) + "\n").encode())
        return 0
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cpu_group = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        # ranks that wait while rank 0 drives every device wait here, on the
        # host (an RCCL barrier would leave a spinning kernel on their device)
        cpu_group = dist.new_group(backend="gloo")

    from prismdb_amd import crc32c
    from prismdb_amd.dist import ShardedBatch

    crc32c.device_init(local)
    nblk = args.nblocks
    if args.strong:
        if args.nblocks % world:
            raise SystemExit(f"--strong: --nblocks {args.nblocks} is not a multiple of {world} ranks")
        nblk = args.nblocks // world
    gather = world > 1 and not args.no_gather
    shard = ShardedBatch(nblocks_per_rank=nblk, block_bytes=BLOCK, rank=rank, world=world, device=dev)
    buf = torch.empty(nblk * BLOCK, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, SEED, byte_offset=shard.first_block * BLOCK)
    outs = [torch.empty(nblk, dtype=torch.int32, device=dev) for _ in range(2)]
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    pending = [None, None]

    def step(i, timed):
        slot = i % 2
        if pending[slot] is not None:
            pending[slot].wait()  # the gather that still reads this output buffer
            pending[slot] = None
        if timed:
            ev[i][0].record(stream)
        crc32c.batch_fixed(buf, BLOCK, BLOCK, nblk, out=outs[slot])
        if timed:
            ev[i][1].record(stream)
        if gather:
            pending[slot] = shard.gather_async(outs[slot], slot)

    for i in range(args.warmup):
        step(i, False)
    for w in pending:
        if w is not None:
            w.wait()
    pending = [None, None]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    for w in pending:
        if w is not None:
            w.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(t[0]), float(t[1])

    total_bytes = world * nblk * BLOCK * args.steps
    value = total_bytes / elapsed / GIB
    algo_bytes = nblk * (BLOCK + 4)  # L read + 4 B result written per block
    achieved = algo_bytes / (kern_ms / 1e3) / 1e9
    # rank-0 results check: gathered results of the last step hold every rank's shard
    gathered_ok = None
    if gather:
        gathered_ok = shard.check_gathered(outs[(args.steps - 1) % 2])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_leg(args, outs[(args.steps - 1) % 2], buf)
    e2e = e2e_leg(args, torch, crc32c, dev) if (args.e2e and rank == 0 and world == 1) else None
    del buf  # the config-2 blocks; the results stay for the checks above
    torch.cuda.empty_cache()
    c5 = None
    if not args.no_config5:
        if world == 1:
            try:  # one rank: a failure here is reported in the line, the headline stands
                c5 = config5_leg(args, torch, dist, crc32c, dev, rank, world)
            except Exception as e:
                c5 = {"error": f"{type(e).__name__}: {e}"}
        else:  # (ranks meet in collectives inside: one rank's exception must end them all)
            c5 = config5_leg(args, torch, dist, crc32c, dev, rank, world)
    multi = None
    if not args.no_multi:
        # one child process of rank 0 drives the devices (all `world` ranks'
        # devices: PrismDB's one-process shape); the ranks free their memory
        # and wait on the host
        del outs
        torch.cuda.empty_cache()
        if world > 1:
            dist.barrier(group=cpu_group)
        if rank == 0:
            # the ranks' devices; at world 1 --multi-devices (default: the
            # one device the caller asked for, not every visible one)
            ndev = world if world > 1 else max(1, args.multi_devices or 1)
            multi = run_multi_child(args, ndev)
        if world > 1:
            dist.barrier(group=cpu_group)

    if rank == 0:
        pmc = load_pmc_traffic(nblk)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device-generated splitmix64 stream, regenerable on host)",
            "config": {
                "workload": "config2: 16Mi x 4096 B blocks per GPU, stride 4096, device-resident (BASELINE.json configs[1])"
                if nblk == 1 << 24 and not args.strong else
                (f"config5 strong scaling: {args.nblocks} x 4096 B blocks in total, {nblk} per GPU, stride 4096, "
                 "device-resident" if args.strong else f"{nblk} x 4096 B blocks per GPU, stride 4096, device-resident"),
                "blocks_per_gpu": nblk,
                "block_bytes": BLOCK,
                "bytes_per_gpu": nblk * BLOCK,
                "parallelism": f"shard{world}" + ("+rccl_gather" if gather else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "traffic_source": (f"{pmc['_path']}: committed rocprofv3 --pmc run of this workload "
                                   "(FETCH_SIZE + WRITE_SIZE per launch, gfx950-corrected), not measured in this run"
                                   if pmc else None),
                "kernel": "crc32c_fixed_kernel<16, false>",
                "kernel_ms": round(kern_ms, 4),
                "kernel_ms_max_rank": round(kern_ms_max, 4),
                "algorithmic_bytes_per_launch": algo_bytes,
            },
            "cpu_baseline": cpu,
        }
        if gathered_ok is not None:
            line["gather_check"] = gathered_ok
        if e2e is not None:
            line["e2e_host_resident"] = e2e
        if c5 is not None:
            line["config5_partitions"] = c5
        if multi is not None:
            line["config5_one_process"] = multi
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
