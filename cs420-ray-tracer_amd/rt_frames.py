"""Pipelined multi-rank frame loop: each rank renders its cyclic
row bands of a batch of frames while the previous batch's shards travel to
rank 0.

Frames are rendered into one of two shard buffers per rank ([batch, R, W, 3]
each) and the buffer's frames are gathered to rank 0 with ONE collective, so
the per-collective host cost is paid once per batch instead of once per frame.
The two buffers alternate by batch parity: a batch's gather is issued
asynchronously (RCCL runs it on the process group's stream after the renders
that produced it); before the buffer is rendered into again the rank's stream
waits for that gather (Work.wait() orders streams, it does not block the host
under NCCL) and rank 0 reassembles the batch's frames then.  So on every rank
the rendering of batch i overlaps the gather of batch i-1, and every frame's
image is complete once the loop has drained.

With `render_batch` the frames of a batch are rendered by ONE call (one
rt_render_frames_async launch), so a rank's slowest tiles of one frame overlap
the other frames' tiles instead of ending every launch.  With `side`, rank 0
reassembles a batch on a second stream (side.begin(k) ... side.end(k)), so the
memory-bound unpermute overlaps the VALU-bound render of the next batch
instead of queueing behind it; side.join(k) orders the next gather into
receive buffer k after that reassembly.
"""
from __future__ import annotations

from typing import Callable, Sequence


def batch_sizes(steps: int, batch: int) -> list[int]:
    """`steps` frames in ceil(steps / batch) launches of near-equal size (the
    larger ones first): 20 frames at batch 16 are two launches of 10, not 16 + 4,
    whose short tail launch would run at a lower per-frame rate."""
    if steps <= 0:
        return []
    k = -(-steps // batch)
    q, r = divmod(steps, k)
    return [q + 1] * r + [q] * (k - r)


def run_frames(dist, steps: int, rank: int, render: Callable[[object], None], shards: Sequence,
               gathered: Sequence | None, unpermute: Callable[[Sequence, int], None] | None,
               batch: int = 1, render_batch: Callable[[object], None] | None = None, side=None) -> None:
    """render(view) enqueues one frame into `view` (a [R, W, 3] slice of a
    shard buffer); shards[k] is buffer k ([batch, R, W, 3]); on rank 0,
    gathered[k] is the list of per-rank receive tensors ([batch, R, W, 3]) for
    buffer k and unpermute(gathered[k], j) enqueues the reassembly of frame j
    of that buffer.  `steps` frames are rendered in batches of at most `batch`
    (batch_sizes: near-equal launches);
    render_batch(view), if given, enqueues all frames of a [n, R, W, 3] view
    at once instead of n render() calls."""
    works = [None, None]
    counts = [0, 0]

    def retire(k):
        works[k].wait()
        works[k] = None
        if rank == 0 and unpermute is not None:
            if side is not None:
                side.begin(k)
            for j in range(counts[k]):
                unpermute(gathered[k], j)
            if side is not None:
                side.end(k)

    done, b = 0, 0
    for n in batch_sizes(steps, batch):
        k = b & 1
        if works[k] is not None:
            retire(k)  # batch b-2: its shard buffer is free, rank 0 reassembles it
        if render_batch is not None:
            render_batch(shards[k][:n])
        else:
            for j in range(n):
                render(shards[k][j])
        recv = [g[:n] for g in gathered[k]] if rank == 0 else None
        if rank == 0 and side is not None:
            side.join(k)  # buffer k's previous batch has been reassembled
        works[k] = dist.gather(shards[k][:n], recv, dst=0, async_op=True)
        counts[k] = n
        done += n
        b += 1
    for i in range(max(0, b - 2), b):  # drain in batch order
        k = i & 1
        if works[k] is not None:
            retire(k)
