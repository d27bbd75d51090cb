"""The N>1 path (sharding + gather of 4-byte results + checksum-of-checksums)
exercised with world_size 2 on the gloo backend, on CPU.  The per-rank compute
here is the oracle (the GPU engine is covered by the -m gpu tests); what is
under test is prismdb_amd.dist."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ORACLE_SO, Oracle

BLOCK = 256
NPER = 64
SEED = 0x5EED0001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from prismdb_amd.dist import ShardedBatch

        ora = Oracle(ORACLE_SO)
        sh = ShardedBatch(NPER, BLOCK, rank, world, device="cpu")
        host = ora.synth(NPER * BLOCK, SEED, sh.first_block * BLOCK)
        res = []
        for slot in range(2):  # two in-flight gathers, as bench.py overlaps them
            mine = torch.from_numpy(ora.batch_fixed(host, BLOCK, BLOCK, NPER, init=slot).view(np.int32).copy())
            work = sh.gather_async(mine, slot)
            work.wait()
            chk = sh.check_gathered(mine, slot)
            res.append((chk, sh.gathered(slot).numpy().view(np.uint32).tolist() if rank == 0 else None))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_exactly():
    from prismdb_amd.dist import shard_range

    for total in (0, 1, 7, 1000, 1 << 24):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 4])
def test_gather_gloo(world):
    """world 2 and a 4-rank rehearsal of the path bench.py runs at N = 2..8."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    ora = Oracle(ORACLE_SO)
    glob = ora.synth(world * NPER * BLOCK, SEED)
    for slot in range(2):
        want = ora.batch_fixed(glob, BLOCK, BLOCK, world * NPER, init=slot).tolist()
        chk, gathered = out[0][slot]
        assert chk == {"ranks": world, "digests_match": True}
        assert gathered == want
