"""Multi-GPU sharding of block batches: one process per GPU, results gathered
to rank 0 with one RCCL gather of the 4-byte checksums.

The reference has no collectives; its only parallelism is key-range
partitioning (8 partitions, db/db_impl.h:359, one background thread each,
util/env_posix.cc:850-890).  Here a partition's block batch maps to one GPU:
blocks are independent, so the data path needs no exchange; the single
exchange step is the gather of the u32 results (64 MiB per 16 Mi blocks),
issued asynchronously so it overlaps the next pass on RCCL's stream.
Works with any torch.distributed backend ("nccl" = RCCL on ROCm; "gloo" for the
CPU tests of this logic).
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block range [start, start+count) of `rank` for strong scaling."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


class ShardedBatch:
    """Weak-scaling shard: rank r owns blocks [r*nblocks_per_rank, (r+1)*nblocks_per_rank)
    of the global block stream."""

    def __init__(self, nblocks_per_rank: int, block_bytes: int, rank: int, world: int, device=None,
                 group=None, slots: int = 2):
        self.n = nblocks_per_rank
        self.block_bytes = block_bytes
        self.rank = rank
        self.world = world
        self.group = group
        self.first_block = rank * nblocks_per_rank
        self.recv: Optional[List[List[object]]] = None
        if world > 1 and rank == 0:
            import torch

            self.recv = [[torch.empty(nblocks_per_rank, dtype=torch.int32, device=device) for _ in range(world)]
                         for _ in range(slots)]

    def gather_async(self, out, slot: int = 0):
        """Start the gather of this rank's results (int32 [n]) to rank 0; returns a work handle."""
        import torch.distributed as dist

        return dist.gather(out, self.recv[slot] if self.rank == 0 else None, dst=0, group=self.group,
                           async_op=True)

    def gathered(self, slot: int = 0):
        """Rank 0: the concatenated global result vector of the last gather in `slot`."""
        import torch

        assert self.rank == 0 and self.recv is not None
        return torch.cat(self.recv[slot])

    def check_gathered(self, out, slot: Optional[int] = None) -> dict:
        """Checksum of checksums: every rank publishes (sum, xor) of its own
        results; rank 0 recomputes them over what it received."""
        import torch
        import torch.distributed as dist

        def digest(t):
            v = t.to(torch.int64) & 0xFFFFFFFF
            x = v[0].clone() if v.numel() else torch.zeros((), dtype=torch.int64, device=v.device)
            if v.numel() > 1:
                # xor-reduce via bit counts per bit position (cheap, deterministic)
                bits = torch.stack([((v >> b) & 1).sum() & 1 for b in range(32)])
                x = (bits << torch.arange(32, device=v.device)).sum()
            return torch.stack([v.sum(), x])

        mine = digest(out)
        allv = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(allv, mine, group=self.group)
        if self.rank != 0:
            return {"rank": self.rank}
        if slot is None:
            slot = 0
            for s in range(len(self.recv)):
                if torch.equal(self.recv[s][0], out):
                    slot = s
        got = [digest(t) for t in self.recv[slot]]
        ok = all(torch.equal(a, b) for a, b in zip(allv, got))
        return {"ranks": self.world, "digests_match": bool(ok)}
