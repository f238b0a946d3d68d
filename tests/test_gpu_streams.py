"""Stream ordering of the C-ABI (include/rt_hip.h "Streams"): a context's own
stream is ordered with torch's default (NULL) stream, and rt_set_stream orders
the new stream after the old one.  No host synchronisation between the
producer and the consumer here: these tests fail if the ordering is missing
(the round-1 race of test_unpermute_copy_widths)."""
import numpy as np
import pytest

from conftest import golden_rgb, manifest, scene_path

pytestmark = pytest.mark.gpu


def _delay(torch, n=24):
    """Queue ~tens of ms of work on torch's current stream."""
    x = torch.ones((8 << 20,), dtype=torch.float32, device="cuda:0")
    for _ in range(n):
        x.mul_(1.0000001).add_(1e-7)
    return x


def test_own_stream_orders_with_torch_default_stream():
    import torch
    import rt_hip

    assert torch.cuda.current_stream().cuda_stream == 0, "torch's current stream is expected to be the NULL stream"
    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    r = rt_hip.Renderer(0)  # its own (blocking) stream
    try:
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        torch.cuda.synchronize()
        out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
        _delay(torch)
        out.fill_(77)  # torch's stream, still queued behind the delay when the render is enqueued
        r.render_async(sc.camera(), W, H, D, None, out.data_ptr())
        got = out.cpu().numpy().tobytes()  # torch's stream: must see the finished render
        assert got == golden_rgb(name)
        # the unpermute reads a buffer torch fills and writes one torch zeroes, no host sync between
        G, band = 3, 8
        R = rt_hip.rows_for_shard(H, band, 0, G).count
        src = torch.empty((G * R * W * 3,), dtype=torch.uint8, device="cuda:0")
        dst = torch.empty((H * W * 3,), dtype=torch.uint8, device="cuda:0")
        _delay(torch)
        src.copy_(torch.arange(src.numel(), device="cuda:0").to(torch.uint8))
        dst.zero_()
        r.unpermute(src.data_ptr(), dst.data_ptr(), W, H, band, G, R)
        s = src.cpu().numpy().reshape(G, R, W * 3)
        want = np.stack([s[(y // band) % G][(y // band // G) * band + y % band] for y in range(H)])
        assert dst.cpu().numpy().reshape(H, W * 3).tobytes() == want.tobytes()
    finally:
        r.close()


def test_set_stream_orders_old_before_new():
    import torch
    import rt_hip

    name = "complex_97x61_d4"
    m = manifest()[name]
    W, H, D = m["width"], m["height"], m["depth"]
    r = rt_hip.Renderer(0)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        sc = rt_hip.Scene.load(scene_path(m["scene"]))
        r.upload(sc)
        G, band = 2, 8
        R = rt_hip.rows_for_shard(H, band, 0, G).count
        gathered = torch.zeros((G, R, W, 3), dtype=torch.uint8, device="cuda:0")
        image = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        r.set_stream(a.cuda_stream)
        with torch.cuda.stream(a):
            _delay(torch)  # stream a is busy when the shards are enqueued behind it
        for k in range(G):
            r.render_async(sc.camera(), W, H, D, rt_hip.rows_for_shard(H, band, k, G), gathered[k].data_ptr())
        r.set_stream(b.cuda_stream)  # b must wait for the renders still queued on a
        r.unpermute(gathered.data_ptr(), image.data_ptr(), W, H, band, G, R)
        b.synchronize()
        assert image.cpu().numpy().tobytes() == golden_rgb(name)
    finally:
        r.set_stream(None)
        r.close()
