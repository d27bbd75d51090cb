"""The N>1 path with the engine in it: two ranks (processes) on the box's
device, each checksumming its own shard through the C ABI -- fixed 4 KiB
blocks (bench.py's config-2 shard) and one SST-shaped descriptor batch
(bench.py's config-5 partition leg: the one-launch path) -- and the results
gathered to rank 0 with prismdb_amd.dist (gloo here: two ranks cannot share
one device under RCCL; bench.py uses the same calls over RCCL, one GPU per
rank).  Rank 0 checks the checksum of checksums and every gathered result
against the oracle over the global stream."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BLOCK = 4096
NPER = 2048
SEED = 0x5EED00F7
ND, DATA, STRIDE, INDEX = 1024, 3988, 3992, 486977  # a small SST-shaped file per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _file_geometry():
    off = np.concatenate([np.arange(ND, dtype=np.int64) * STRIDE, [ND * STRIDE]])
    lens = np.concatenate([np.full(ND, DATA, dtype=np.int64), [INDEX]])
    return off, lens, (ND * STRIDE + INDEX + 4 + 7) // 8 * 8  # (the generator starts at 8-B offsets)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from prismdb_amd import crc32c
        from prismdb_amd.dist import ShardedBatch

        dev = torch.device("cuda", 0)
        crc32c.device_init(0)
        res = {}
        # config-2 shard: blocks [rank * NPER, (rank + 1) * NPER) of the global stream
        sh = ShardedBatch(NPER, BLOCK, rank, world, device="cpu")
        buf = torch.empty(NPER * BLOCK, dtype=torch.uint8, device=dev)
        crc32c.fill_synthetic(buf, SEED, sh.first_block * BLOCK)
        out, _ = crc32c.batch_fixed(buf, BLOCK, BLOCK, NPER)
        mine = out.cpu()
        sh.gather_async(mine, 0).wait()
        res["fixed"] = (sh.check_gathered(mine, 0),
                        sh.gathered(0).numpy().view(np.uint32).tolist() if rank == 0 else None)
        # config-5 partition: one SST-shaped file per rank through descriptors
        off, lens, fbytes = _file_geometry()
        fb = torch.empty(fbytes, dtype=torch.uint8, device=dev)
        crc32c.fill_synthetic(fb, SEED + 1, rank * fbytes)
        fo, _ = crc32c.batch(fb, torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev),
                             mask=True)
        sf = ShardedBatch(len(off), fbytes, rank, world, device="cpu")
        mine = fo.cpu()
        sf.gather_async(mine, 0).wait()
        res["file"] = (sf.check_gathered(mine, 0),
                       sf.gathered(0).numpy().view(np.uint32).tolist() if rank == 0 else None)
        torch.cuda.synchronize()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_engine_and_gather(oracle):
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    glob = oracle.synth(world * NPER * BLOCK, SEED)
    want = oracle.batch_fixed(glob, BLOCK, BLOCK, world * NPER).tolist()
    chk, gathered = out[0]["fixed"]
    assert chk == {"ranks": world, "digests_match": True}
    assert gathered == want
    off, lens, fbytes = _file_geometry()
    files = oracle.synth(world * fbytes, SEED + 1)
    want = []
    for r in range(world):
        raw, _ = oracle.batch(files, (off + r * fbytes).astype(np.uint64), lens.astype(np.uint64))
        want += [oracle.mask(int(c)) for c in raw]
    chk, gathered = out[0]["file"]
    assert chk == {"ranks": world, "digests_match": True}
    assert gathered == want
