"""The inline-asm audit of the gfx950 kernels (tools/audit_kernels.py), on CPU:
hipcc cross-compiles crc32c_kernels.hip to assembly and every kernel is checked
for ring registers touched while their asm loads are in flight
(tools/check_inflight.py), VALU-written SGPRs read by an asm load within 5 wait
states (tools/check_asm_hazards.py), and spills.  build() runs the same audit
on the build's own assembly and refuses to finish on a finding."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
@pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")), reason="no hipcc")
def test_kernels_pass_inline_asm_audit():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "audit_kernels.py"), "-q"],
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout + r.stderr


def test_inflight_audit_catches_an_injected_read(tmp_path):
    """A read of an asm-load destination right after the load is reported."""
    asm = "\n".join([
        "k:",
        "\t;;#ASMSTART",
        "\tglobal_load_dword v10, v1, s[2:3] offset:0 nt",
        "\t;;#ASMEND",
        "\tv_mov_b32_e32 v11, v10",
        "\t;;#ASMSTART",
        "\ts_waitcnt vmcnt(0)",
        "\t;;#ASMEND",
        "\ts_endpgm",
    ])
    f = tmp_path / "k.s"
    f.write_text(asm + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_inflight.py"), str(f)],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "in-flight [10]" in r.stdout, r.stdout


def test_inflight_audit_tracks_asm_atomic_returns(tmp_path):
    """An asm atomic with return (sc0) is in flight like a load: a copy of its
    destination before a wait that retires it is reported, a read after is not."""
    def run(lines):
        f = tmp_path / "k.s"
        f.write_text("\n".join(["k:"] + lines + ["\ts_endpgm"]) + "\n")
        return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_inflight.py"), str(f)],
                              capture_output=True, text=True)
    atomic = ["\t;;#ASMSTART", "\tglobal_atomic_add v12, v1, v2, s[4:5] sc0", "\t;;#ASMEND"]
    load = ["\t;;#ASMSTART", "\tglobal_load_dword v10, v1, s[2:3] offset:0 nt", "\t;;#ASMEND"]
    wait = ["\t;;#ASMSTART", "\ts_waitcnt vmcnt(1)", "\t;;#ASMEND"]
    bad = run(atomic + load + ["\tv_mov_b32_e32 v11, v12"] + wait)
    assert bad.returncode == 1 and "in-flight [12]" in bad.stdout, bad.stdout
    good = run(atomic + load + wait + ["\tv_readfirstlane_b32 s6, v12", "\ts_waitcnt vmcnt(0)"])
    assert good.returncode == 0, good.stdout


def test_hazard_audit_catches_valu_sgpr_write(tmp_path):
    """v_readfirstlane into a descriptor SGPR right before an asm buffer load is reported."""
    asm = "\n".join([
        "k:",
        "\tv_readfirstlane_b32 s4, v1",
        "\t;;#ASMSTART",
        "\tbuffer_load_dword v10, v2, s[4:7], 0 offen offset:0 nt",
        "\t;;#ASMEND",
        "\ts_endpgm",
    ])
    f = tmp_path / "k.s"
    f.write_text(asm + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_hazards.py"), str(f)],
                       capture_output=True, text=True)
    assert r.returncode == 1, r.stdout
