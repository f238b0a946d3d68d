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
