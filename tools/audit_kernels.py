#!/usr/bin/env python3
"""Compile crc32c_kernels.hip to gfx950 assembly (optionally with -D knobs) and
run both inline-asm audits on every kernel in it:

    python tools/audit_kernels.py [-D NAME=VALUE ...]

  * tools/check_inflight.py   in-flight asm-load registers read/copied early
  * tools/check_asm_hazards.py VALU-written SGPR -> asm VMEM within 5 wait states

Also prints each kernel's VGPR / SGPR / spill / LDS figures from the metadata.
Exit status 1 if any audit fails or a kernel spills.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "prismdb_amd", "csrc", "crc32c_kernels.hip")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--keep", help="write the .s here")
    ap.add_argument("--asm", help="audit this .s (e.g. the build's own) instead of compiling")
    ap.add_argument("-q", "--quiet", action="store_true", help="print failing kernels only")
    args = ap.parse_args()
    out = args.asm or args.keep or tempfile.mktemp(suffix=".s")
    if not args.asm:
        cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "--cuda-device-only", "-S", SRC, "-o", out] + [f"-D{d}" for d in args.D]
        subprocess.check_call(cmd)
    text = open(out).read().splitlines()
    # kernel bodies: from "<name>:" (a .globl symbol) to ".Lfunc_end"
    kernels, cur, name = {}, None, None
    globs = {m.group(1) for l in text for m in [re.match(r"\s*\.globl\s+(\S+)", l)] if m}
    for l in text:
        m = re.match(r"^(\S+):\s*(;.*)?$", l)
        if m and m.group(1) in globs:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if l.startswith(".Lfunc_end"):
                kernels[name] = cur
                cur = None
                continue
            cur.append(l)
    bad = 0
    meta = "\n".join(text)
    for k, body in kernels.items():
        with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
            f.write("\n".join(body) + "\n")
            p = f.name
        r1 = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_inflight.py"), p],
                            capture_output=True, text=True)
        r2 = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_hazards.py"), p],
                            capture_output=True, text=True)
        os.unlink(p)
        info = {}
        i0 = meta.find(".name:           " + k + "\n")
        blk = meta[i0:meta.find(".vgpr_spill_count", i0) + 40] if i0 >= 0 else ""
        for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                    "group_segment_fixed_size", "private_segment_fixed_size"):
            v = re.search(r"\." + key + r":\s+(\d+)", blk)
            info[key] = int(v.group(1)) if v else None
        # SGPR spills go to VGPR lanes (v_writelane): reported, not fatal
        spill = (info["vgpr_spill_count"] or 0) + (info["private_segment_fixed_size"] or 0)
        ok = r1.returncode == 0 and r2.returncode == 0 and spill == 0
        bad += not ok
        short = re.sub(r"^_ZN7prismdb3dev", "", k)[:60]
        if not (ok and args.quiet):
            print(f"{'ok ' if ok else 'BAD'} {short:60s} vgpr={info['vgpr_count']} sgpr={info['sgpr_count']} "
                  f"spill={spill} sgpr_spill={info['sgpr_spill_count']} lds={info['group_segment_fixed_size']}")
        if r1.returncode or r2.returncode:
            print((r1.stdout + r1.stderr + r2.stdout + r2.stderr).strip()[:2000])
    if not args.keep and not args.asm:
        os.unlink(out)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
