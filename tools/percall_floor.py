#!/usr/bin/env python3
"""Where a one-SST-file call's time goes, against the launch floor.

    python tools/percall_floor.py build     # here: tools/probe_lib/libfloor_probe.so
                                            #   (+ variants: tools/variants.py build --only direct_ts direct_plain direct_ts_plain)
    python tools/percall_floor.py run       # GPU box: one JSON object

Every row brackets calls on one stream between two probe_stamp kernels (one
wave storing s_memrealtime, 100 MHz) and reports the median over reps of the
bracket in us, minus nothing: rows are read against each other.
  stamp_only            stamp; stamp                     the bracket itself
  null_plain / _ext     stamp; empty kernel; stamp       one-launch grid (CUs x 768), plain
                                                         launch / hipExtLaunchKernel + stop event
  waves                 stamp; waves kernel; stamp       + each wave's entry / exit stamp
  scatter_16811         stamp; 16 811 stores at 3992 B   the trailer stores' dirty lines
  empty_call            a 1-span leveldb_crc32c_batch    (one-launch path)
  file_seal / _verify   one SST file (16 811 x 3988 B @ 3992 + 486 977 B index), one call
  fixed_same_bytes      leveldb_crc32c_batch_fixed over 16 480 x 4096 B (the file's 67.5 MB)
  null_ext_<flags> / null_rec_<flags> / scatter_rec_<flags>_x10
                        the empty kernel with a stop event / a recorded event, and
                        16 811 scattered stores + a recorded event, for events made
                        with hipEventDisableTiming (the product's), | DisableSystemFence,
                        | ReleaseToDevice, or no flags
  <variant>_file_*      the file rows through variants base / ev_nofence / ev_device
                        (the library's own events with those flags)
  file_verify_x10       ten file calls back to back in one bracket (/10: what bench's
                        config5_partitions per-file figure sees)
and, with the direct_ts variants (per-wave stamps), the one-file call's
phases against the bracket: start = first wave entry - first stamp, end =
second stamp - last wave exit, with the stop-event launch and a plain one.
"""
import ctypes
import json
import os
import subprocess
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROBE_DIR = os.path.join(ROOT, "tools", "probe_lib")
PROBE = os.path.join(PROBE_DIR, "libfloor_probe.so")
VLIB = os.path.join(ROOT, "tools", "vlib")
ND, DATA, STRIDE, INDEX = 16811, 3988, 3992, 486977
EVENT_VARIANTS = ("base", "ev_nofence", "ev_device")
EVENT_FLAGS = {"default": 0, "notiming": 2, "nofence": 2 | 0x20000000, "todevice": 2 | 0x40000000}


def build():
    os.makedirs(PROBE_DIR, exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(ROOT, "tools", "floor_probe.hip"), "-o", PROBE])
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "variants.py"), "build", "--only",
                           "direct_ts", "direct_plain", "direct_ts_plain", *EVENT_VARIANTS])


def _lib(path):
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    g = lib.leveldb_crc32c_batch
    g.restype = ctypes.c_int
    g.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_void_p]
    return lib


def run(reps):
    import numpy as np
    import torch

    from prismdb_amd import crc32c
    from prismdb_amd._lib import lib as product

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    P = ctypes.CDLL(PROBE, mode=os.RTLD_LOCAL)
    vp = ctypes.c_void_p
    P.probe_stamp.argtypes = [vp, vp]
    P.probe_null.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
    P.probe_waves.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
    P.probe_scatter.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp]
    P.probe_event_create.argtypes = [vp]
    P.probe_event_create_flags.argtypes = [vp, ctypes.c_uint]
    P.probe_record.argtypes = [vp, vp]
    P.probe_lds.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
    P.probe_read.argtypes = [vp, ctypes.c_uint64, ctypes.c_int, vp, vp]
    ev = ctypes.c_void_p()
    assert P.probe_event_create(ctypes.byref(ev)) == 0
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    stamps = torch.zeros(2 * reps, dtype=torch.int64, device=dev)

    fbytes = ND * STRIDE + INDEX + 4
    buf = torch.empty(fbytes + 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED00F9)
    off = np.concatenate([np.arange(ND, dtype=np.int64) * STRIDE, [ND * STRIDE]])
    lens = np.array([DATA] * ND + [INDEX], dtype=np.int32)
    n = len(off)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    nwaves_direct = 12 * cus
    out = torch.zeros(((n + 3) & ~3) + 16 * nwaves_direct, dtype=torch.int32, device=dev)
    mm = torch.zeros(n, dtype=torch.uint8, device=dev)
    wave_ts = torch.zeros(2 * nwaves_direct, dtype=torch.int64, device=dev)
    L = product()
    crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, out=out[:n], check_bounds=False)  # seal once
    torch.cuda.synchronize()

    def call_batch(lib, verify, m=n):
        rc = lib.leveldb_crc32c_batch(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, m, out.data_ptr(),
                                      mm.data_ptr() if verify else None, 0 if verify else 3, sp)
        if rc != 0:
            lib.leveldb_crc32c_last_error.restype = ctypes.c_char_p
            raise RuntimeError(f"leveldb_crc32c_batch: {rc}: {lib.leveldb_crc32c_last_error()}")

    nfix = (ND * STRIDE + INDEX) // 4096

    def call_fixed():
        assert L.leveldb_crc32c_batch_fixed(buf.data_ptr(), 4096, 4096, nfix, 0, out.data_ptr(), None, 0, sp) == 0

    def bracket(fn, per=1):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        for r in range(reps):
            P.probe_stamp(ctypes.c_void_p(stamps.data_ptr() + 16 * r), sp)
            for _ in range(per):
                fn()
            P.probe_stamp(ctypes.c_void_p(stamps.data_ptr() + 16 * r + 8), sp)
        torch.cuda.synchronize()
        st = stamps.cpu().numpy().reshape(reps, 2)
        d = (st[:, 1] - st[:, 0]) / 100.0 / per
        return {"median_us": round(float(np.median(d)), 2), "p10_us": round(float(np.percentile(d, 10)), 2),
                "p90_us": round(float(np.percentile(d, 90)), 2)}

    rows = {}
    rows["stamp_only"] = bracket(lambda: None)
    rows["null_plain"] = bracket(lambda: P.probe_null(cus, 768, sp, None))
    rows["null_ext"] = bracket(lambda: P.probe_null(cus, 768, sp, ev))
    # the same with events of explicit flags: the product's (DisableTiming), and
    # that | DisableSystemFence / | ReleaseToDevice (agent-scope release)
    scat = torch.zeros(ND * STRIDE // 4 + 64, dtype=torch.int32, device=dev)
    for fname, fl in EVENT_FLAGS.items():
        e2 = ctypes.c_void_p()
        assert P.probe_event_create_flags(ctypes.byref(e2), fl) == 0
        rows[f"null_ext_{fname}"] = bracket(lambda: P.probe_null(cus, 768, sp, e2))
        rows[f"null_rec_{fname}"] = bracket(lambda: (P.probe_null(cus, 768, sp, None), P.probe_record(e2, sp)))
        rows[f"scatter_rec_{fname}_x10"] = bracket(
            lambda: (P.probe_scatter(ctypes.c_void_p(scat.data_ptr()), ND, STRIDE // 4, sp), P.probe_record(e2, sp)),
            per=10)
    rows["waves"] = bracket(lambda: P.probe_waves(cus, 768, ctypes.c_void_p(wave_ts.data_ptr()), sp))
    rows["scatter_16811"] = bracket(lambda: P.probe_scatter(ctypes.c_void_p(scat.data_ptr()), ND, STRIDE // 4, sp))
    for lds in (0, 65536, 163840):
        rows[f"lds_{lds}"] = bracket(lambda: P.probe_lds(cus, 768, lds, ctypes.c_void_p(wave_ts.data_ptr()), sp))
    sink = torch.zeros(65536, dtype=torch.int32, device=dev)
    for g in (cus, 4 * cus, 16 * cus):
        rows[f"read_67MB_grid{g // cus}x"] = bracket(
            lambda: P.probe_read(ctypes.c_void_p(buf.data_ptr()), ND * STRIDE + INDEX, g, ctypes.c_void_p(sink.data_ptr()), sp))
        rows[f"read_67MB_grid{g // cus}x_x10"] = bracket(
            lambda: P.probe_read(ctypes.c_void_p(buf.data_ptr()), ND * STRIDE + INDEX, g, ctypes.c_void_p(sink.data_ptr()), sp),
            per=10)
    one = torch.tensor([8], dtype=torch.int64, device=dev)
    onel = torch.tensor([4], dtype=torch.int32, device=dev)

    def call_empty():
        assert L.leveldb_crc32c_batch(buf.data_ptr(), one.data_ptr(), onel.data_ptr(), None, 1, out.data_ptr(), None,
                                      0, sp) == 0

    rows["empty_call"] = bracket(call_empty)
    rows["file_seal"] = bracket(lambda: call_batch(L, False))
    rows["file_verify"] = bracket(lambda: call_batch(L, True))
    rows["fixed_same_bytes"] = bracket(call_fixed)
    rows["file_verify_x10"] = bracket(lambda: call_batch(L, True), per=10)
    rows["file_seal_x10"] = bracket(lambda: call_batch(L, False), per=10)
    rows["fixed_same_bytes_x10"] = bracket(call_fixed, per=10)
    # The same calls over 24 different files in turn (1.6 GB: past the 256 MB
    # MALL, as bench's config5_partitions walks its 143 files): HBM-bound
    nf = 24
    fstride = (fbytes + 4095) & ~4095  # (file starts 4 KiB aligned: the fixed kernel's fast path needs 4-B alignment)
    big = torch.empty(nf * fstride + 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(big, 0x5EED00FA)
    k = [0]

    def rot(fn):
        def step():
            fn(big.data_ptr() + (k[0] % nf) * fstride)
            k[0] += 1
        return step

    def file_at(verify):
        def f(base):
            rc = L.leveldb_crc32c_batch(base, d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(),
                                        mm.data_ptr() if verify else None, 0 if verify else 3, sp)
            assert rc == 0
        return f

    rows["hbm_file_seal_x24"] = bracket(rot(file_at(False)), per=nf)
    rows["hbm_file_verify_x24"] = bracket(rot(file_at(True)), per=nf)
    rows["hbm_fixed_same_bytes_x24"] = bracket(
        rot(lambda b: L.leveldb_crc32c_batch_fixed(b, 4096, 4096, nfix, 0, out.data_ptr(), None, 0, sp)), per=nf)
    rows["hbm_read_67MB_grid4x_x24"] = bracket(
        rot(lambda b: P.probe_read(ctypes.c_void_p(b), ND * STRIDE + INDEX, 4 * cus, ctypes.c_void_p(sink.data_ptr()), sp)),
        per=nf)
    for name in EVENT_VARIANTS:
        path = os.path.join(VLIB, f"lib_{name}.so")
        if not os.path.exists(path):
            continue
        V = _lib(path)

        def vfile_at(verify, V=V):
            def f(base):
                rc = V.leveldb_crc32c_batch(base, d_off.data_ptr(), d_len.data_ptr(), None, n, out.data_ptr(),
                                            mm.data_ptr() if verify else None, 0 if verify else 3, sp)
                assert rc == 0
            return f
        rows[f"{name}_file_verify_x10"] = bracket(lambda: call_batch(V, True), per=10)
        rows[f"{name}_file_seal_x10"] = bracket(lambda: call_batch(V, False), per=10)
        rows[f"{name}_hbm_file_seal_x24"] = bracket(rot(vfile_at(False)), per=nf)
        rows[f"{name}_hbm_file_verify_x24"] = bracket(rot(vfile_at(True)), per=nf)
    del big
    res = {"cus": cus, "reps": reps, "file_bytes": int(ND * DATA + INDEX), "rows": rows}

    # the null kernel's waves: first entry / last exit against the bracket
    st = stamps
    P.probe_stamp(ctypes.c_void_p(st.data_ptr()), sp)
    P.probe_waves(cus, 768, ctypes.c_void_p(wave_ts.data_ptr()), sp)
    P.probe_stamp(ctypes.c_void_p(st.data_ptr() + 8), sp)
    torch.cuda.synchronize()
    a, b = st[:2].cpu().numpy()
    w = wave_ts[:2 * cus * 12].cpu().numpy().reshape(-1, 2)
    res["waves_phases_us"] = {"start": round((w[:, 0].min() - a) / 100.0, 2),
                              "life": round((w[:, 1].max() - w[:, 0].min()) / 100.0, 2),
                              "end": round((b - w[:, 1].max()) / 100.0, 2)}
    for lds in (0, 163840):  # the first group's entry against the bracket, with and without the LDS
        P.probe_stamp(ctypes.c_void_p(st.data_ptr()), sp)
        P.probe_lds(cus, 768, lds, ctypes.c_void_p(wave_ts.data_ptr()), sp)
        P.probe_stamp(ctypes.c_void_p(st.data_ptr() + 8), sp)
        torch.cuda.synchronize()
        a, b = st[:2].cpu().numpy()
        w = wave_ts[:cus].cpu().numpy()
        res[f"lds_{lds}_phases_us"] = {"first_entry": round((w.min() - a) / 100.0, 2),
                                       "last_entry": round((w.max() - a) / 100.0, 2),
                                       "end_after_last_entry": round((b - w.max()) / 100.0, 2)}

    # the one-file call's phases (per-wave stamps of the direct_ts builds)
    base = (n + 3) & ~3
    for name in ("direct_ts", "direct_ts_plain", "direct_plain"):
        path = os.path.join(VLIB, f"lib_{name}.so")
        if not os.path.exists(path):
            continue
        V = _lib(path)
        if name == "direct_plain":
            res[name] = {"file_verify": bracket(lambda: call_batch(V, True)),
                         "file_verify_x10": bracket(lambda: call_batch(V, True), per=10)}
            continue
        ph = []
        for verify in (False, True):
            for r in range(reps):
                for _ in range(2):
                    call_batch(V, verify)
                P.probe_stamp(ctypes.c_void_p(st.data_ptr()), sp)
                call_batch(V, verify)
                P.probe_stamp(ctypes.c_void_p(st.data_ptr() + 8), sp)
                torch.cuda.synchronize()
                a, b = st[:2].cpu().numpy()
                ts = out[base:base + 16 * nwaves_direct].cpu().numpy().view(np.uint64).reshape(nwaves_direct, 8)
                ts = ts.astype(np.int64)
                live = ts[:, 0] != 0
                first, last = ts[live, 0].min(), ts[live, 5].max()
                drained = ts[live & (ts[:, 6] > 0), 4]
                ph.append((verify, (first - a) / 100.0, (last - first) / 100.0, (b - last) / 100.0,
                           (np.median(drained) - first) / 100.0, (b - a) / 100.0))
        out_ph = {}
        for verify in (False, True):
            v = np.array([p[1:] for p in ph if p[0] == verify])
            out_ph["verify" if verify else "seal"] = {
                k: round(float(np.median(v[:, j])), 2)
                for j, k in enumerate(["start_us", "first_entry_to_last_exit_us", "end_us", "drain_p50_us",
                                       "bracket_us"])}
        res[name] = out_ph
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
