#!/usr/bin/env python3
"""Run one engine variant's fixed kernel back-to-back for a few seconds while
the GPU's power and clocks are sampled (measurement support, not product):

    python tools/power_probe.py --only base nofold --seconds 6

For each variant: kernels/s, GB/s, and the rocm-smi samples taken while it
ran (written raw to gpurun_out/power_<variant>.txt).  Answers whether the
fold's extra VALU/LDS work moves the card onto its power limit.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "vlib")


def sampler(stop, path):
    with open(path, "w") as f:
        while not stop.is_set():
            for cmd in (["rocm-smi", "--showpower", "--showclocks", "--showtemp", "--json"],):
                try:
                    r = subprocess.run(cmd, capture_output=True, text=True, timeout=5)
                    f.write(json.dumps({"t": time.time(), "cmd": cmd[0], "out": r.stdout[-4000:]}) + "\n")
                except Exception as e:  # sampling is best effort
                    f.write(json.dumps({"t": time.time(), "err": str(e)}) + "\n")
            f.flush()
            time.sleep(0.25)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="+", default=["base", "nofold"])
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--gib", type=int, default=64)
    args = ap.parse_args()
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    nblk = (args.gib << 30) // 4096
    buf = torch.empty(nblk * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res = {}
    for name in args.only:
        lib = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        f = lib.leveldb_crc32c_batch_fixed
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        run = lambda: f(buf.data_ptr(), 4096, 4096, nblk, 0, out.data_ptr(), None, 0, sp)
        run()
        torch.cuda.synchronize()
        stop = threading.Event()
        path = os.path.join(ROOT, "gpurun_out", f"power_{name}.txt")
        th = threading.Thread(target=sampler, args=(stop, path))
        th.start()
        t0 = time.time()
        k = 0
        while time.time() - t0 < args.seconds:
            for _ in range(20):
                assert run() == 0
            torch.cuda.synchronize()
            k += 20
        dt = time.time() - t0
        stop.set()
        th.join()
        res[name] = {"launches": k, "ms_per_launch": round(dt / k * 1e3, 3),
                     "GB/s": round(k * nblk * 4100 / dt / 1e9, 1)}
        print(name, res[name], flush=True)
        time.sleep(2.0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
