"""bench.py's launch contract (CPU; no GPU is touched): `python bench.py
--gpus N` without a launcher starts N ranks under torch.distributed.run
itself, a WORLD_SIZE that disagrees with --gpus is refused, and no run ever
reports a world size it did not measure (the old bench warned
and went on as one rank, so `--gpus 8` printed n_gpus 1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def _json_lines(text):
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except ValueError:
                pass
    return out


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_spawns_n_ranks(n):
    """--gpus N without WORLD_SIZE: N ranks, each told world N (dry run: the
    ranks report and leave before importing torch's GPU side)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)], capture_output=True, text=True, timeout=300,
                       env=_env(PRISMDB_BENCH_DRYRUN="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert sorted(d["rank"] for d in lines) == list(range(n)), r.stdout
    assert all(d["world"] == n for d in lines)
    assert sorted(d["local_rank"] for d in lines) == list(range(n))
    assert "n_gpus" not in r.stdout


def test_world_size_mismatch_refused():
    """WORLD_SIZE set by a launcher but different from --gpus: exit 2, no line."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
    assert _json_lines(r.stdout) == []


def test_gpus_2_without_devices_fails_loudly():
    """The real run (no dry run) on a host without devices: the two spawned
    ranks fail, bench exits non-zero, and nothing claims n_gpus 1."""
    import torch

    if torch.cuda.device_count() > 0:  # (counts devices without initialising HIP)
        pytest.skip("devices visible: this checks the no-device failure path")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, timeout=600, env=_env())
    assert r.returncode != 0
    assert '"n_gpus": 1' not in r.stdout
    assert all("n_gpus" not in d for d in _json_lines(r.stdout))


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_multi_leg_child_reports_instead_of_raising(monkeypatch):
    """The batch_multi leg runs in a child process under a time limit; a child
    that fails (no device here) or runs out of time comes back as an `error`
    entry for the line, never as an exception or a hang of the bench."""
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("devices visible: this checks the failure paths")
    bench = _bench_module()
    monkeypatch.setattr(sys, "argv", [BENCH, "--c5-spans", "1000", "--c5-steps", "1"])
    args = bench.parse()
    res = bench.run_multi_child(args, 1)
    assert res["devices"] == 1 and "error" in res
    args.multi_timeout = 0.01
    res = bench.run_multi_child(args, 2)
    assert res == {"devices": 2, "error": "batch_multi leg stopped after 0 s"}


def test_pmc_summary_picked_is_the_newest():
    """The line's `traffic` comes from the newest committed PMC summary of
    the headline workload: by round, then run tag (r05ab after r05g after
    r05a), not by plain path order (where r05ab sorts before r05g)."""
    import glob
    import re

    bench = _bench_module()
    got = bench.load_pmc_traffic(1 << 24)
    assert got is not None

    def key(p):
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(p))
        return (int(m.group(1)), len(m.group(2)), m.group(2))

    cands = []
    for p in glob.glob(os.path.join(ROOT, "profiles", "*", "r*_pmc.json")):
        with open(p) as f:
            d = json.load(f)
        if d.get("nblocks") == 1 << 24 and d.get("hbm_bytes_per_launch"):
            cands.append(p)
    assert key("r05ab_pmc.json") > key("r05g_pmc.json") > key("r05a_pmc.json")
    assert os.path.basename(got["_path"]) == os.path.basename(max(cands, key=key))
