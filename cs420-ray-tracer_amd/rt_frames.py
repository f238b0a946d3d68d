"""Pipelined multi-rank frame loop: each rank renders its cyclic
row bands of frame i while frame i-1's shards travel to rank 0.

Two shard buffers per rank and two gather buffers on rank 0 alternate by frame
parity.  Frame i's gather is issued asynchronously (RCCL runs it on the
process group's stream after the render that produced the shard); before
frame i+2 renders into the same buffer the rank's stream waits for that
gather (Work.wait() orders streams, it does not block the host under NCCL),
and rank 0 reassembles frame i then.  So on every rank the render of frame i
overlaps the gather of frame i-1, and the image of frame i is complete once
the loop has drained.
"""
from __future__ import annotations

from typing import Callable, Sequence


def run_frames(dist, steps: int, rank: int, render: Callable[[object], None], shards: Sequence,
               gathered: Sequence | None, unpermute: Callable[[object], None] | None) -> None:
    """render(shard) enqueues frame rendering into `shard`; on rank 0,
    gathered[k] is the list of per-rank receive tensors for buffer k and
    unpermute(gathered_k) enqueues the reassembly of that buffer."""
    works = [None, None]

    def retire(k):
        works[k].wait()
        works[k] = None
        if rank == 0 and unpermute is not None:
            unpermute(gathered[k])

    for i in range(steps):
        k = i & 1
        if works[k] is not None:
            retire(k)  # frame i-2: its shard buffer is free, rank 0 reassembles it
        render(shards[k])
        works[k] = dist.gather(shards[k], gathered[k] if rank == 0 else None, dst=0, async_op=True)
    for i in range(max(0, steps - 2), steps):  # drain in frame order
        k = i & 1
        if works[k] is not None:
            retire(k)
