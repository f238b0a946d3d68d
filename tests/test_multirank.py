"""CPU-only (gloo, world_size 2 and 3): the multi-GPU data path without GPUs.
Each rank renders its cyclic 8-row bands (with the oracle standing in for the
device kernel), the shards are gathered to rank 0 exactly as bench.py gathers
them over RCCL, and rank 0 reassembles them with the same row mapping as the
unpermute kernel.  The result must equal the reference's golden image, and
the per-rank ray counts must sum to the full frame's."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import golden_rgb, manifest, scene_path

BAND = 8


def unpermute_host(gathered: np.ndarray, H: int, band: int) -> np.ndarray:
    """Row mapping of rtk::unpermute_kernel (csrc/rt_kernel.hip)."""
    G, R, W, _ = gathered.shape
    out = np.empty((H, W, 3), np.uint8)
    for y in range(H):
        b = y // band
        out[y] = gathered[b % G, (b // G) * band + y % band]
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    import rt_hip

    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    rows = rt_hip.rows_for_shard(H, BAND, rank, world)
    rgb, counts, _ = orc.OracleScene(scene_path(m["scene"])).render(
        W, H, D, band=rows.band, first=rows.first, stride=rows.stride, count=rows.count)
    shard = torch.from_numpy(np.frombuffer(rgb, np.uint8).reshape(rows.count, W, 3).copy())
    gathered = torch.empty((world, rows.count, W, 3), dtype=torch.uint8) if rank == 0 else None
    dist.gather(shard, list(gathered.unbind(0)) if rank == 0 else None, dst=0)
    n = torch.tensor([counts["primary"] + counts["shadow"] + counts["reflect"]], dtype=torch.int64)
    dist.all_reduce(n)
    if rank == 0:
        img = unpermute_host(gathered.numpy(), H, BAND)
        q.put((img.tobytes(), int(n.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "complex_97x61_d4"), (3, "simple_800x600_d10")])
def test_gloo_gather_reassembles_golden(world, name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    img, rays = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert img == golden_rgb(name)
    assert rays == sum(manifest()[name]["rays"].values())


class _Side:
    """Records rt_frames' side-stream protocol: begin/end around each batch's
    reassembly, join(k) before buffer k is gathered into again."""

    def __init__(self):
        self.log = []
        self.open = None

    def begin(self, k):
        assert self.open is None
        self.open = k
        self.log.append(("begin", k))

    def end(self, k):
        assert self.open == k
        self.open = None
        self.log.append(("end", k))

    def join(self, k):
        assert self.open is None
        self.log.append(("join", k))


def _pipelined_worker(rank, world, port, batch, q, batched=False):
    """bench.py's pipelined frame loop (rt_frames.run_frames) under gloo: frame f
    of rank r fills its shard with (f, r, row); every reassembled frame must be
    exact and arrive in order, with `batch` frames per gather (steps not a
    multiple of it: the last batch is partial)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rt_frames

    W, H, band, steps = 5, 37, 8, 7
    import rt_hip

    rows = rt_hip.rows_for_shard(H, band, rank, world)
    R = rows.count
    shards = [torch.zeros((batch, R, W, 3), dtype=torch.uint8) for _ in range(2)]
    gathered = ([list(torch.zeros((world, batch, R, W, 3), dtype=torch.uint8).unbind(0)) for _ in range(2)]
                if rank == 0 else None)
    frame = [0]
    seen = []

    def render(shard):
        f = frame[0]
        for k in range(R):
            shard[k] = (f * 16 + rank * 4 + k % 4) % 256
        frame[0] += 1

    def unpermute(g, j):
        # the device unpermute's addressing: frame j of rank r at rows (r * batch + j) * R
        flat = torch.stack(g).reshape(world * batch * R, W, 3)[j * R:]
        img = unpermute_host(np.stack([flat[r * batch * R:r * batch * R + R].numpy() for r in range(world)]), H,
                             band)
        seen.append(img[:, 0, 0].tolist())

    def render_batch(view):  # one call per batch (bench.py's rt_render_frames_async path)
        for j in range(view.shape[0]):
            render(view[j])

    side = _Side() if (batched and rank == 0) else None
    rt_frames.run_frames(dist, steps, rank, render, shards, gathered, unpermute if rank == 0 else None, batch,
                         render_batch if batched else None, side)
    if side is not None:
        # every reassembly is bracketed, and buffer k is joined before each gather into it
        nb = -(-steps // batch)
        assert [e for e in side.log if e[0] == "begin"] == [("begin", b & 1) for b in range(nb)]
        assert [e for e in side.log if e[0] == "join"] == [("join", b & 1) for b in range(nb)]
    if rank == 0:
        q.put(seen)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,batched", [(2, 1, False), (3, 1, False), (2, 4, False), (3, 3, False),
                                                 (2, 4, True), (3, 3, True)])
def test_gloo_pipelined_frames(world, batch, batched):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, batch, q, batched)) for r in range(world)]
    for p in procs:
        p.start()
    seen = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H, band = 37, 8
    assert len(seen) == 7
    for f, col in enumerate(seen):
        want = []
        for y in range(H):
            b = y // band
            r, k = b % world, (b // world) * band + y % band
            want.append((f * 16 + r * 4 + k % 4) % 256)
        assert col == want, f
