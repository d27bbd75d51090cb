#!/usr/bin/env python3
"""Repeat config-5-shaped planner calls and check every result against an
independent path: the claimed pair-run tail deals runs in claim order, which
differs from call to call.

    python tools/claim_stress.py [calls]     # GPU box; one JSON line

A: 2.4 M spans of 3988 B at stride 3992 (the pair-run kernel) against the
   fixed kernel over the same blocks (batch_fixed, a different kernel);
B: bench's config-5 partition (143 files, index spans on the segment path),
   sealed into zeroed trailers, then verified: every call's results equal the
   first call's, and the verify pass flags nothing."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(calls):
    import numpy as np
    import torch

    from prismdb_amd import crc32c

    dev = torch.device("cuda", 0)
    crc32c.device_init(0)
    res = {"calls": calls}
    # A
    n = 2404116
    buf = torch.empty(n * 3992 + 64, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0C5A)
    want, _ = crc32c.batch_fixed(buf, 3992, 3988, n, mask=True)
    d_off = torch.arange(n, dtype=torch.int64, device=dev) * 3992
    d_len = torch.full((n,), 3988, dtype=torch.int32, device=dev)
    bad = 0
    for _ in range(calls):
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, check_bounds=False)
        bad += int((out != want).sum().item())
    res["A_pair_vs_fixed_mismatches"] = bad
    del buf, d_off, d_len, want
    # B
    nd, stride, dl, il, nf = 16811, 3992, 3988, 486977, 143
    fb = (nd * stride + il + 4 + 255) & ~255
    off1 = np.concatenate([np.arange(nd, dtype=np.int64) * stride, [nd * stride]])
    len1 = np.concatenate([np.full(nd, dl, dtype=np.int64), [il]])
    off = (np.arange(nf, dtype=np.int64)[:, None] * fb + off1[None, :]).reshape(-1)
    lens = np.tile(len1, nf)
    buf = torch.empty(nf * fb, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0C5B)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    first = None
    diff = flagged = 0
    for _ in range(calls):
        out, _ = crc32c.batch(buf, d_off, d_len, mask=True, trailer=True, check_bounds=False)
        if first is None:
            first = out.clone()
        else:
            diff += int((out != first).sum().item())
        _, mm = crc32c.batch(buf, d_off, d_len, mask=True, verify=True, check_bounds=False)
        flagged += int(mm.sum().item())
    res["B_seal_calls_differing_entries"] = diff
    res["B_verify_flags"] = flagged
    res["ok"] = bad == 0 and diff == 0 and flagged == 0
    print(json.dumps(res))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 50))
