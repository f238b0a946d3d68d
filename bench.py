#!/usr/bin/env python3
"""bench.py -- Mrays/s of the HIP render loop (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

A step renders ONE frame of the workload: each rank traces its cyclic 8-row
bands through librt_hip.so (on torch's current stream, output resident in
HBM), then the shards are gathered to rank 0 with RCCL (torch.distributed
"nccl" = RCCL over xGMI) and unpermuted into the final PPM-ordered
framebuffer on device.  Frames are rendered in batches of
--frames-per-launch (default 32), one rt_render_frames_async launch per batch,
so the slowest tiles of one frame overlap the other frames' work; for N > 1
a batch renders while the previous batch's shards travel to rank 0 in one
gather.  Every frame is rendered and delivered in full.  Total work per step is fixed
as N grows ("scaling": "strong").  value = rays of the frame x K / max-over-ranks wall
time of the K timed steps.

Also reported:
  roofline      fp64 VALU roof of the render kernels (render_kernel +
                render_deferred): the fp64 FLOPs they EXECUTE per frame (rocprofv3
                PMC: 64 x (ADD + MUL + 2 FMA + TRANS)_F64 wave-instructions,
                profiles/pmc_traffic.json, checked against the kernel sources'
                hash) / the in-stream HIP-event kernel time per frame of the
                timed launches, vs the 78.6 TFLOP/s fp64 vector peak; VALU busy
                and the fp64 share of VALU issue beside it; traffic = HBM bytes
                per launch (FETCH_SIZE x 2, the gfx950 correction, + WRITE_SIZE).
                SURVEY 8(d)'s brute-force count (25 FLOP x spheres x rays) is
                `algorithmic_equivalent`: the kernel prunes pairs exactly, so
                that rate measures the algorithm and exceeds the peak.
  hbm_write     the north star's HBM-write roofline: W*H*3 bytes per frame.
  single_frame  ONE frame of a view the context has not rendered (the camera
                moved per sample: its camera grid built on the device in the
                launch, the tile order rebuilt on the host), one launch, median
                of 5 -- the still frame the reference times (src/main.cpp:139-161):
                in-stream kernel ms and host wall ms.
  moving_camera launches of 32 frames whose camera positions all differ and
                are new to the context (a camera grid per frame built on the
                device in each launch): the batched rate of a moving view.
  e2e           the drop-in path end to end, fresh context: parse + rt_create +
                rt_upload_scene (BVH, light grids) + render (tile order,
                scratch, kernel, D2H) + rt_write_ppm P3 (src/main.cpp:93-163).
  cpu_baseline  the reference's own trace_ray (oracle/_ref/ref_render, built
                from /root/reference/src/main.cpp) on 1 host core, same
                workload, rank 0 at N=1 only; falls back to the C port
                (oracle/liborc.so) when the reference build is absent.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "cs420-ray-tracer_amd")
ORACLE = os.path.join(REPO, "oracle")
sys.path.insert(0, PKG)

METRIC = "Mrays/sec (primary+shadow+reflect) at 1920×1080, 200 spheres, depth 4"
WORKLOADS = {
    # name: (scene, W, H, depth)
    "synth200_1920x1080_d4": ("synth200", 1920, 1080, 4),   # the metric (BASELINE cfg 3')
    "complex_1920x1080_d4": ("complex", 1920, 1080, 4),     # north-star target
    "medium_1920x1080_d2": ("medium", 1920, 1080, 2),       # cfg 2
    "complex_3840x2160_d4": ("complex", 3840, 2160, 4),     # cfg 4
    "synth10k_3840x2160_d6": ("synth10k", 3840, 2160, 6),   # cfg 5
}
FLOP_PER_TEST = 25          # A5 miss path: 3 sub + 5 (a) + 6 (b) + 7 (c) + 4 (disc), SURVEY 8(d)
FLOP_PER_CULL = 34          # rtk::keep(): 3 sub, |v.a| 5, v x a 9, |v x a|^2 5, margin 5, rhs 4, compare 3
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X vector FP64 (spec; 256 CU x 2.4 GHz x 128 FLOP/clk)
HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BAND = 8
# back-to-back warmup launches after the host-side builds (clocks settle; measure());
# BENCH_WARM_BUSY_S overrides it for the A/B that measured it
WARM_BUSY_S = float(os.environ.get("BENCH_WARM_BUSY_S", "0.05"))
# the sources the PMC record in profiles/pmc_traffic.json must have been measured with
KERNEL_SOURCES = ("rt_kernel.hip", "rt_device.h", "rt_cgbuild.h", "rt_bvh.cpp", "rt_bvh.h", "rt_lightgrid.cpp",
                  "rt_lightgrid.h", "rt_sched.cpp", "rt_sched.h", "Makefile")  # Makefile: the compile flags


def kernel_source_sha() -> str:
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(PKG, "csrc", name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count() -> int:
    """GPUs a child process would see, counted in a separate interpreter so
    this (launcher) process never loads the HIP runtime; device_count() does
    not initialise the GPU on this image."""
    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=600)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError):
        return 0


def launch_ranks(n: int, argv: list, child: list | None = None, gpu_count: int | None = None,
                 out=None, poll_s: float = 0.1) -> int:
    """`bench.py --gpus N` without an external launcher: start N rank processes
    of this script (plain child processes -- nothing here has touched the GPU,
    and the parent never execs), one per local GPU, with the env
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT).  Rank 0's
    stdout (the JSON line) is relayed to `out`; every other rank's stdout goes
    to stderr.  Returns 0 only if every rank exits 0; when one fails, the rest
    are terminated and its exit code is returned.  `child` replaces the
    command (tests use a stub); `gpu_count` skips the device probe."""
    import threading

    out = out or sys.stdout
    if gpu_count is None:
        gpu_count = visible_gpu_count()
    if gpu_count < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, this host has {gpu_count}", file=sys.stderr)
        return 2
    cmd = child or [sys.executable, os.path.abspath(__file__)] + list(argv)
    port = str(free_port())
    procs = []
    for i in range(n):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if i == 0 else sys.stderr.fileno()))
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout.read().decode().splitlines()),
                              daemon=True)
    reader.start()
    rc = 0
    while None in [p.poll() for p in procs]:  # poll every rank each round
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(poll_s)
    reader.join(timeout=20)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    for ln in lines:
        print(ln, file=out, flush=True)
    if rc != 0:
        print(f"bench.py: a rank failed (exit {rc}) of {n}", file=sys.stderr)
    return rc


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(scene_file: str, W: int, H: int, D: int, rays_per_frame: int, threads: int = 1) -> dict:
    """Reference render loop on `threads` host cores over the full frame (the sample)."""
    ref = os.path.join(ORACLE, "_ref", "ref_render")
    if os.path.exists(ref):
        out = subprocess.run([ref, scene_file, str(W), str(H), str(D), "--threads", str(threads)],
                             capture_output=True, text=True, timeout=600, check=True).stdout
        secs = float(out.split("Serial time:")[1].split()[0])
        kind, rays = "reference", rays_per_frame
        what = "oracle/_ref/ref_render: the reference's src/main.cpp trace_ray, g++ -O3, full frame"
    else:
        sys.path.insert(0, ORACLE)
        import orc  # checker / CPU-baseline leg only

        _, counts, secs = orc.OracleScene(scene_file).render(W, H, D, threads=threads)
        kind, rays = "port", counts["primary"] + counts["shadow"] + counts["reflect"]
        what = "oracle/liborc.so C restatement, full frame"
    what += ", OpenMP schedule(dynamic) as ray_openmp" if threads > 1 else ""
    return {"value": round(rays / secs / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": kind,
            "sample": f"{what}; {W}x{H} d{D}, {rays} rays in {secs:.3f} s on {threads} thread(s) of {cpu_model()}"}


def moved(rt_hip, cam, dx):
    """A copy of `cam` with its position moved by dx along x (same basis)."""
    c = rt_hip.rt_camera.from_buffer_copy(cam)
    c.position[0] = cam.position[0] + dx
    return c


def median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if len(xs) % 2 else 0.5 * (xs[len(xs) // 2 - 1] + xs[len(xs) // 2])


def info_or_none(r):
    """rt_get_info, or None for an older diagnostic build (RT_HIP_LIB) without it."""
    try:
        return r.info()
    except AttributeError:
        return None


def single_frame(rt_hip, r, cam, W, H, D, rows, out_ptr, samples=5):
    """One-frame launches, each from a camera position the context has not seen
    (moved 1e-3 further along x per sample), after one untimed such launch: the
    reference's timed region (main.cpp:139-161) on a steady-state context.  The
    launch builds its camera grid on the device (in kernel_ms) and its tile
    order on the host (in wall_ms)."""
    import time as _t

    kms, wall, rate = [], [], []
    before = info_or_none(r)
    for k in range(samples + 1):
        c = moved(rt_hip, cam, 1e-3 * (k + 1))
        t0 = _t.perf_counter()
        r.render_async(c, W, H, D, rows, out_ptr)
        st = r.stats()  # waits for the stream
        dt = (_t.perf_counter() - t0) * 1e3
        if k:
            kms.append(st.kernel_ms)
            wall.append(dt)
            rate.append(st.rays / st.kernel_ms / 1e3)
    after = info_or_none(r)
    return {"kernel_ms": round(median(kms), 4), "wall_ms": round(median(wall), 4),
            "mrays_per_s": round(median(rate), 1), "samples": samples,
            "camera_grid_used": bool(after.cam_grid_last) if after else None,
            "camera_grid_builds": after.cam_grid_builds - before.cam_grid_builds if after else None,
            "tile_order_builds": after.tile_order_builds - before.tile_order_builds if after else None,
            "what": "one frame per launch, each from a camera position not rendered before (camera moved 1e-3 per "
                    "sample): camera grid built on the device per launch (in kernel_ms), tile order rebuilt on the "
                    "host per frame (in wall_ms); median of %d" % samples}


def moving_camera(rt_hip, torch, r, cam, W, H, D, rows, shard, F, launches=2):
    """Launches of F frames whose camera positions all differ, and differ from
    every earlier launch's (a sequence moved 1e-3 per frame): each launch builds
    F camera grids on the device (in the timed kernels)."""
    import time as _t

    seqs = [rt_hip.camera_array([moved(rt_hip, cam, 1e-3 * (k * F + f + 1)) for f in range(F)])
            for k in range(launches + 1)]
    R = rows.count
    r.render_frames_async(seqs[0], W, H, D, rows, shard.data_ptr(), R * W * 3)  # untimed: scratch sized
    r.stats()
    torch.cuda.synchronize()
    t0 = _t.perf_counter()
    for k in range(launches):
        r.render_frames_async(seqs[k + 1], W, H, D, rows, shard.data_ptr(), R * W * 3)
    st = r.stats()
    el = _t.perf_counter() - t0
    ktimes = r.kernel_times(launches)
    return {"mrays_per_s": round(st.rays * launches / el / 1e6, 1), "frames": F * launches,
            "ms_per_frame": round(el / (F * launches) * 1e3, 4),
            "kernel_ms_per_frame": round(sum(ktimes) / (F * launches), 4),
            "camera_grid_used": bool(info.cam_grid_last) if (info := info_or_none(r)) else None,
            "what": "%d launches of %d frames, every frame's camera position distinct and new (moved 1e-3 per "
                    "frame): a camera grid per frame built on the device in each launch" % (launches, F)}


def end_to_end(rt_hip, scene_file, W, H, D, device, runs=5):
    """The drop-in path end to end in a fresh context (what ray_hip does):
    parse, rt_create, rt_upload_scene, one synchronous render to host memory,
    rt_write_ppm P3.  Median over `runs` of each part and of the total."""
    import tempfile
    import time as _t

    import numpy as np

    parts = {k: [] for k in ("parse_ms", "create_ms", "upload_ms", "render_ms", "write_p3_ms", "total_ms")}
    up_parts = {k: [] for k in ("bvh_ms", "light_grids_ms", "sphere_grids_ms", "behind_grid_ms")}
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "output_gpu.ppm")
        for _ in range(runs):
            t = [_t.perf_counter()]
            sc = rt_hip.Scene.load(scene_file)
            cam = sc.camera()
            t.append(_t.perf_counter())
            r = rt_hip.Renderer(device)
            t.append(_t.perf_counter())
            r.upload(sc)
            t.append(_t.perf_counter())
            info = info_or_none(r)
            if info is not None:  # rt_upload_scene's builds (host wall time, inside upload_ms)
                for k, v in zip(up_parts, (info.bvh_build_ms, info.light_grid_build_ms, info.sphere_grid_build_ms,
                                           info.behind_grid_build_ms)):
                    up_parts[k].append(v)
            # the image buffer as ray_hip allocates it (uninitialised: the render writes every byte)
            rgb, st = r.render(cam, W, H, D, out=np.empty(W * H * 3, np.uint8))
            t.append(_t.perf_counter())
            rt_hip.write_ppm(out, rgb, W, H)
            t.append(_t.perf_counter())
            r.close()
            for k, (a, b) in zip(list(parts)[:5], zip(t, t[1:])):
                parts[k].append((b - a) * 1e3)
            parts["total_ms"].append((t[-1] - t[0]) * 1e3)
            kernel_ms, rays = st.kernel_ms, st.rays
        size = os.path.getsize(out)
    res = {k: round(median(v), 3) for k, v in parts.items()}
    if all(up_parts.values()):
        res["upload_parts_ms"] = {k: round(median(v), 3) for k, v in up_parts.items()}
    res.update({"kernel_ms": round(kernel_ms, 4), "rays": rays, "p3_bytes": size, "runs": runs,
                "mrays_per_s_end_to_end": round(rays / median(parts["total_ms"]) / 1e3, 1)})
    return res


def golden_check(torch, workload, depth, shards, launches, image, rank):
    """Untimed, after the timed region: the bytes the timed launches produced
    against the reference's own image of this workload (tests/golden/
    manifest.json `sha256_rgb`, rendered by the reference's trace_ray).  At
    N = 1 every frame of the last timed launch (still in its shard buffer);
    for N > 1, rank 0's last reassembled frame.  None when the workload has no
    golden (or the depth is overridden)."""
    if not launches or depth is not None or rank != 0:
        return None
    path = os.path.join(REPO, "tests", "golden", "manifest.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        want = json.load(f).get(workload, {}).get("sha256_rgb")
    if want is None:
        return None
    if image is not None:
        frames = [image.cpu().numpy().tobytes()]
    else:
        last = shards[(len(launches) - 1) & 1][:launches[-1]].cpu().numpy()
        frames = [last[j].tobytes() for j in range(last.shape[0])]
    got = [hashlib.sha256(b).hexdigest() for b in frames]
    return {"frames_checked": len(got), "frames_equal": sum(g == want for g in got),
            "all_equal": all(g == want for g in got), "sha256_rgb": want,
            "what": "every frame of the last timed launch" if image is None else "rank 0's last reassembled frame"}


def measure(rt_hip, torch, dist, workload, steps, warmup, world, rank, device, cull=True, batch=4, dist_on=None,
            depth=None, extras=False):
    import rt_frames

    if dist_on is None:
        dist_on = world > 1
    scene_name, W, H, D = WORKLOADS[workload]
    if depth is not None:
        D = depth
    scene_file = os.path.join(PKG, "scenes", scene_name + ".txt")
    scene = rt_hip.Scene.load(scene_file)
    cam = scene.camera()
    r = rt_hip.Renderer(device)
    r.set_culling(cull)
    r.upload(scene)
    stream = torch.cuda.current_stream()
    r.set_stream(stream.cuda_stream)  # the kernel runs on torch's stream: events and RCCL order with it
    rows = rt_hip.rows_for_shard(H, BAND, rank, world) if dist_on else rt_hip.rt_rows(1, 0, 1, H)
    R = rows.count
    # two shard / gather buffers of `batch` frames each: a batch is rendered by
    # ONE launch (rt_render_frames_async) while the previous one is gathered to
    # rank 0 by one RCCL gather (rt_frames); at N = 1 the batches alternate
    # between the two buffers the same way, without the gather
    F = batch
    shards = [torch.empty((F, R, W, 3), dtype=torch.uint8, device=f"cuda:{device}") for _ in range(2)]
    cams = [cam] * F  # a frame sequence of the metric's view
    gathered = image = None
    if dist_on and rank == 0:
        gathered = [list(torch.empty((world, F, R, W, 3), dtype=torch.uint8, device=f"cuda:{device}").unbind(0))
                    for _ in range(2)]
        image = torch.empty((H, W, 3), dtype=torch.uint8, device=f"cuda:{device}")

    def render(shard):
        r.render_async(cam, W, H, D, rows, shard.data_ptr())

    # the camera arrays of every launch size the loop uses, built before any
    # timing: a launch's host path is then one ctypes call
    cam_arrays = {n: rt_hip.camera_array(cams[:n]) for n in range(2, F + 1)}

    def render_batch(view):  # view: [n, R, W, 3], frame j at view[j]
        n = view.shape[0]
        if n == 1:
            render(view[0])
        else:
            r.render_frames_async(cam_arrays[n], W, H, D, rows, view.data_ptr(), R * W * 3)

    def unpermute(g, j):
        # g: per-rank views of one [world, F, R, W, 3] buffer; frame j of rank r
        # starts (r * F + j) * R rows in, i.e. rank-major with F * R rows per rank
        r.unpermute(g[0].data_ptr() + j * R * W * 3, image.data_ptr(), W, H, BAND, world, F * R)

    class Side:
        """rank 0's reassembly stream (rt_frames.run_frames(side=...)): the unpermute
        kernels run there, overlapping the next batch's render on the main stream."""

        def __init__(self):
            self.main = stream
            self.s = torch.cuda.Stream(device=f"cuda:{device}")
            self.ev = [torch.cuda.Event(), torch.cuda.Event()]

        def begin(self, k):
            self.s.wait_stream(self.main)  # the gather of buffer k (Work.wait ordered it on main)
            r.set_stream(self.s.cuda_stream)

        def end(self, k):
            r.set_stream(self.main.cuda_stream)
            self.ev[k].record(self.s)

        def join(self, k):
            self.main.wait_event(self.ev[k])

    side = Side() if dist_on and rank == 0 else None

    def frames(n):
        if dist_on:
            rt_frames.run_frames(dist, n, rank, render, shards, gathered, unpermute if rank == 0 else None, F,
                                 render_batch, side)
        else:
            for b, m in enumerate(rt_frames.batch_sizes(n, F)):
                render_batch(shards[b & 1][:m])

    # one single-frame launch (untimed): the ray counts of ONE frame of this rank's shard
    render(shards[0][0])
    st = r.stats()  # syncs
    # then at least one full batch: the launch shape of the timed region has
    # run once (scratch sized, tile order and camera grid built) before the
    # clock starts, and the warmup launches are the last GPU work before the
    # barrier: no host work leaves the GPU idle in between (a launch after a
    # 0.38 ms idle gap ran 2.9 % slower than the next, profiles/r3u/trace96);
    # the timed launches' durations are read after the timed region
    frames(max(warmup, F))
    # ... and then back-to-back launches for at least WARM_BUSY_S of GPU time:
    # the first warmup launch waits for the host-side builds (camera grid, tile
    # order: 30-100 ms with the GPU idle), and after an idle gap that long the
    # GPU's clocks need more than one launch to come back -- a 20-frame launch
    # after 20 ms idle runs 8 % slower, after 1 ms or less it does not
    # (profiles/r4e/idle_gap.log) -- so the timed launches would otherwise pay
    # for the build.  Every rank runs the same number of batches (collectives).
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    frames(F)
    torch.cuda.synchronize()
    per_batch = time.perf_counter() - t_w
    warm_extra = int(min(1000, max(0, -(-WARM_BUSY_S // max(per_batch, 1e-6)) - 1)))
    if dist_on:
        n_t = torch.tensor([warm_extra], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(n_t, op=dist.ReduceOp.MAX)
        warm_extra = int(n_t.item())
    for _ in range(warm_extra):
        frames(F)
    info_warm = info_or_none(r)  # the camera grid / tile order the timed launches use (built in warmup), host only
    timed_launches = len(rt_frames.batch_sizes(steps, F)) if steps > 0 else 0
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames(steps)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # one entry per timed launch (F frames each, the last maybe fewer): the most recent ones
    ktimes = r.kernel_times(max(timed_launches, 1))
    kmean = sum(ktimes) / len(ktimes)
    kframe = sum(ktimes) / max(steps, 1)  # kernel time per frame
    my_rays = st.rays
    tests_exact, tests_cull = st.tests_exact, st.tests_cull
    if dist_on:
        t = torch.tensor([elapsed, kframe], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmax = t.tolist()
        per_rank = [torch.zeros(1, dtype=torch.float64, device=f"cuda:{device}") for _ in range(world)]
        dist.all_gather(per_rank, torch.tensor([kframe], dtype=torch.float64, device=f"cuda:{device}"))
        rank_kernel_ms = [round(float(x.item()), 5) for x in per_rank]
        seen_world = dist.get_world_size()
        n = torch.tensor([my_rays], dtype=torch.int64, device=f"cuda:{device}")
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        frame_rays = int(n.item())
    else:
        kmax = kframe
        frame_rays = my_rays
        rank_kernel_ms = [round(kframe, 5)]
        seen_world = 1
    golden = golden_check(torch, workload, depth, shards, rt_frames.batch_sizes(steps, F), image if dist_on else None,
                          rank)
    assembled_ok = None
    if dist_on and rank == 0 and steps > 0:
        # untimed: the last frame reassembled from the gathered shards must equal
        # one full-frame render on this device, byte for byte
        full = torch.empty((H, W, 3), dtype=torch.uint8, device=f"cuda:{device}")
        r.render_async(cam, W, H, D, rt_hip.rt_rows(1, 0, 1, H), full.data_ptr())
        torch.cuda.synchronize()
        assembled_ok = bool(torch.equal(full, image))
    info_timed = info_or_none(r)  # None: an RT_HIP_LIB diagnostic build without rt_get_info
    camera_grid = sphere_grids = behind_grid = scratch = None
    if info_timed is not None and info_warm is not None:
        camera_grid = {"used_by_timed_launches": bool(info_timed.cam_grid_last),
                       "cells_per_face_edge": info_timed.cam_grid_n,
                       "builds_in_warmup": info_warm.cam_grid_builds,
                       "builds_in_timed_region": info_timed.cam_grid_builds - info_warm.cam_grid_builds,
                       "build_ms_total": round(info_warm.cam_grid_build_ms, 2),
                       "tile_order_builds_in_timed_region": info_timed.tile_order_builds - info_warm.tile_order_builds,
                       "upload_ms": round(info_timed.upload_ms, 2)}
        # sphere grids (reflection rays' closest hit), built by rt_upload_scene (in upload_ms)
        sphere_grids = {"grids": info_timed.sphere_grids, "cells_per_face_edge": info_timed.sphere_grid_n,
                        "entries": info_timed.sphere_grid_entries,
                        "build_ms": round(info_timed.sphere_grid_build_ms, 2)}
        # uniform grid (closest hits of scenes above 1,024 spheres), built by rt_upload_scene
        scratch = {"bytes": int(info_timed.scratch_bytes),
                   "what": "device scratch of the context after the timed launches: reflection-stack homes, the "
                           "deferred queue with its slots' stacks, the camera grid, the tile order (rt_info)"}
        behind_grid = {"built": bool(info_timed.behind_grid),
                       "used_by_timed_launches": bool(info_timed.behind_grid_last),
                       "cells": info_timed.behind_grid_cells, "entries": info_timed.behind_grid_entries,
                       "build_ms": round(info_timed.behind_grid_build_ms, 2)}
    extra = {}
    if extras and not dist_on:
        extra["single_frame"] = single_frame(rt_hip, r, cam, W, H, D, rows, shards[0][0].data_ptr())
        extra["moving_camera"] = moving_camera(rt_hip, torch, r, cam, W, H, D, rows, shards[0], F)
    gather_ms = None
    if dist_on and steps > 0:
        # untimed: one batch's RCCL gather to rank 0 alone ("plus the
        # gather time"), mean of 5, in-stream events around the collective
        dist.barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dist.gather(shards[0], gathered[0] if rank == 0 else None, dst=0)
        e1.record()
        torch.cuda.synchronize()
        gather_ms = e0.elapsed_time(e1) / 5
    r.close()
    return {"assembled_ok": assembled_ok, "golden": golden, "scene": scene_name, "scene_file": scene_file, "W": W, "H": H, "D": D, "spheres": scene.num_spheres,
            "lights": scene.num_lights, "frame_rays": frame_rays, "rank_rays": my_rays, "elapsed": elapsed,
            "kernel_ms_mean": kmean, "kernel_ms_per_frame": kframe, "kernel_ms_per_frame_max_rank": kmax,
            "kernel_ms_min": min(ktimes), "frames_per_launch": F,
            "launches_timed": len(ktimes), "rows_per_rank": R, "tests_exact": tests_exact,
            "tests_cull": tests_cull, "cull": cull, "gather_ms_per_batch": gather_ms,
            "rank_kernel_ms_per_frame": rank_kernel_ms, "world_size_seen": seen_world,
            "warmup_frames_rendered": max(warmup, F) + (1 + warm_extra) * F,
            "launch_frames": rt_frames.batch_sizes(steps, F),
            "camera_grid": camera_grid, "sphere_grids": sphere_grids, "behind_grid": behind_grid,
            "scratch": scratch, **extra}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--workload", default="synth200_1920x1080_d4", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-also", action="store_true", help="skip the complex.txt north-star line item")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the single-frame, moving-camera and end-to-end line items (N = 1 only)")
    ap.add_argument("--frames-per-launch", "--frames-per-gather", dest="frames_per_launch", type=int, default=32,
                    help="frames rendered by one kernel launch (rt_render_frames_async, 1..32); for N > 1 also "
                         "the frames per RCCL gather to rank 0 (one collective per batch)")
    ap.add_argument("--force-dist", action="store_true",
                    help="rehearsal: run the N > 1 data path (RCCL process group, shard gather, unpermute) at N = 1")
    ap.add_argument("--depth", type=int, default=None,
                    help="diagnostic: override the workload's depth (the line then no longer measures the metric)")
    ap.add_argument("--brute-force", action="store_true",
                    help="disable the exact per-wave sphere culling: every ray tests every sphere")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: start the ranks here, before anything loads torch
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree",
              file=sys.stderr)
        sys.exit(2)

    # The JSON line is the only thing on stdout: RCCL's banner and any other
    # library output written to fd 1 go to stderr instead.
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch  # loads torch's HIP runtime first; librt_hip.so binds to it
    import torch.distributed as dist
    import rt_hip

    if torch.cuda.device_count() < world:
        print(f"bench.py: WORLD_SIZE={world} needs {world} visible GPUs, rank {rank} sees "
              f"{torch.cuda.device_count()}", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), rank=rank, world_size=world)

    cull = not args.brute_force
    batch = max(1, min(rt_hip.MAX_FRAMES, args.frames_per_launch))
    extras = world == 1 and not args.no_extras
    m = measure(rt_hip, torch, dist, args.workload, args.steps, args.warmup, world, rank, local, cull, batch, dist_on,
                args.depth, extras)
    also = {}
    if not args.no_also and args.workload != "complex_1920x1080_d4":
        a = measure(rt_hip, torch, dist, "complex_1920x1080_d4", max(args.steps // 2, 5), 2, world, rank, local,
                    cull, batch, dist_on, extras=extras)
        also["complex_1920x1080_d4"] = {
            "mrays_per_s": round(a["frame_rays"] * max(args.steps // 2, 5) / a["elapsed"] / 1e6, 2),
            "ms_per_frame": round(a["elapsed"] / max(args.steps // 2, 5) * 1e3, 4),
            "kernel_ms_per_frame": round(a["kernel_ms_per_frame"], 4), "rays_per_frame": a["frame_rays"],
            "target_mrays_per_s": 1000, "frame_equals_golden": a["golden"]["all_equal"] if a["golden"] else None}
        for k in ("single_frame", "moving_camera"):
            if k in a:
                also["complex_1920x1080_d4"][k] = a[k]
    e2e = {}
    if extras and rank == 0:
        for wl in (args.workload, "complex_1920x1080_d4"):
            sn, W_, H_, D_ = WORKLOADS[wl]
            e2e[wl] = end_to_end(rt_hip, os.path.join(PKG, "scenes", sn + ".txt"), W_, H_, D_, local)

    if rank == 0:
        value = m["frame_rays"] * args.steps / m["elapsed"] / 1e6
        k_s = m["kernel_ms_per_frame"] * 1e-3  # launch time / frames per launch
        # executed work of one frame (device counters), not the brute-force count
        flops = FLOP_PER_TEST * m["tests_exact"] + FLOP_PER_CULL * m["tests_cull"]
        test_tflops = flops / k_s / 1e12
        brute = FLOP_PER_TEST * m["spheres"] * m["rank_rays"] / k_s / 1e12
        pmc_rec = {}
        pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pmc_rec = json.load(f).get(args.workload, {})
        # the PMC record is per frame of THIS workload at N = 1; it describes the
        # measured kernel only if it was taken with the same kernel sources
        src_sha = kernel_source_sha()
        pmc_ok = bool(pmc_rec) and pmc_rec.get("kernel_src_sha") == src_sha and world == 1
        fp64_pf = pmc_rec.get("fp64_flops_per_frame") if pmc_ok else None
        if fp64_pf is not None:
            achieved, flops_source = fp64_pf / k_s / 1e12, "pmc"
        else:
            # no PMC record taken on these kernel sources: no hardware fraction is
            # claimed (the device's exact/cull test counters undercount the executed
            # work -- walks, shading, normalisation -- and stay under `executed`)
            achieved, flops_source = None, "none: no PMC record matches the kernel sources"
        traffic = None
        if pmc_ok and "fetch_bytes" in pmc_rec and "write_bytes" in pmc_rec:
            # FETCH_SIZE x 2: MI355X_MICROARCH.md's gfx950 correction; per launch of `batch` frames
            traffic = int((2 * pmc_rec["fetch_bytes"] + pmc_rec["write_bytes"]) * batch)
        out_bytes = m["W"] * m["rows_per_rank"] * 3
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(m["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: scenes/%s.txt (splitmix64 seed 420, SURVEY 8(d) generator) resident in HBM"
                    % m["scene"] if m["scene"].startswith("synth") else "scenes/%s.txt" % m["scene"],
            "config": {"workload": args.workload + (f"_depth{args.depth}_override" if args.depth is not None else ""),
                       "scene": m["scene"], "width": m["W"], "height": m["H"],
                       "depth": m["D"], "spheres": m["spheres"], "lights": m["lights"],
                       "rays_per_frame": m["frame_rays"],
                       **({"assembled_frame_equals_single_gpu_render": m["assembled_ok"]} if dist_on else {}),
                       # untimed: the timed launches' output vs the reference's image (tests/golden)
                       "frame_equals_golden": m["golden"]["all_equal"] if m["golden"] else None,
                       "golden_check": m["golden"],
                       "frames_per_launch": batch,
                       # the slowest rank's kernel time per frame and, for N > 1,
                       # one batch's gather to rank 0 measured alone (overlapped with rendering
                       # in the timed loop)
                       "kernel_ms_per_frame_max_rank": round(m["kernel_ms_per_frame_max_rank"], 4),
                       # what torch.distributed saw: the process group's size and every rank's
                       # kernel time per frame of its shard (rank order)
                       "world_size_seen": m["world_size_seen"],
                       "rank_kernel_ms_per_frame": m["rank_kernel_ms_per_frame"],
                       "launch_frames": m["launch_frames"],
                       "warmup_frames_rendered": m["warmup_frames_rendered"],
                       "kernel_only_mrays_per_s": round(m["frame_rays"] / m["kernel_ms_per_frame_max_rank"] / 1e3,
                                                        1),
                       **({"gather_ms_per_batch": round(m["gather_ms_per_batch"], 4),
                           "gather_ms_per_frame": round(m["gather_ms_per_batch"] / batch, 4)}
                          if m.get("gather_ms_per_batch") is not None else {}),
                       "parallelism": f"rows cyclic {BAND}-row bands x {world} GPU, {batch} frames per launch" +
                                      (f" + RCCL gather to rank 0 every {batch} frames" if dist_on else ""),
                       # the timed frames all see the workload's one camera (the reference renders one fixed
                       # view): the camera grid for that position is built once, in warmup (its cost below);
                       # single_frame / moving_camera are the rates without that assumption
                       "view": "static camera: every frame the scene file's view",
                       "camera_grid": m["camera_grid"], "sphere_grids": m["sphere_grids"],
                       "behind_grid": m["behind_grid"], "scratch": m["scratch"]},
            # achieved = the fp64 FLOPs the render kernels EXECUTE per frame
            # (rocprofv3 PMC, 64 x (ADD + MUL + 2 FMA + TRANS)_F64 wave-instructions,
            # profiles/pmc_traffic.json taken with these kernel sources) over the
            # in-stream kernel time per frame: a hardware fraction of the fp64
            # VALU peak.  One launch renders `batch` frames; rates per launch =
            # per frame.  SURVEY 8(d)'s brute-force count is algorithmic_equivalent.
            "roofline": {"bound": "valu",
                         "achieved": round(achieved, 3) if achieved is not None else None,
                         "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / FP64_VALU_PEAK_TFLOPS, 4) if achieved is not None else None,
                         "traffic": traffic,
                         "kernel": "rtk::render_kernel + rtk::render_deferred (fp64 VALU; no dense contraction, "
                                   "so no MFMA roof)",
                         "flops_source": flops_source,
                         "fp64_flops_per_frame": fp64_pf,
                         "fp64_flops_per_launch": fp64_pf * batch if fp64_pf is not None else None,
                         "per_unit": ("fp64 FLOPs the render kernels executed per frame: rocprofv3 PMC "
                                      "64 x (ADD + MUL + 2 FMA + TRANS)_F64 wave-instructions, "
                                      "profiles/pmc_traffic.json on these kernel sources; x frames per launch"
                                      if fp64_pf is not None else
                                      "none counted: no PMC record on these kernel sources (achieved / frac null; "
                                      "the device's exact + cull test counts are under executed.test_tflops)"),
                         "valu_busy": pmc_rec.get("valu_busy") if pmc_ok else None,
                         "fp64_share_of_valu_insts": pmc_rec.get("fp64_share_of_valu_insts") if pmc_ok else None,
                         "valu_lane_utilization": pmc_rec.get("valu_lane_utilization") if pmc_ok else None,
                         # the PMC FLOP count assumes full exec masks (an upper bound): weighted by the
                         # measured VALU lane utilisation it is the FLOPs on active lanes (an estimate:
                         # the fp64 instructions' own lane occupancy is not counted separately)
                         "lane_weighted": ({
                             "achieved": round(achieved * pmc_rec["valu_lane_utilization"], 3),
                             "frac": round(achieved * pmc_rec["valu_lane_utilization"] / FP64_VALU_PEAK_TFLOPS, 4),
                             "what": "achieved x valu_lane_utilization (SQ_THREAD_CYCLES_VALU / 64 "
                                     "SQ_ACTIVE_INST_VALU): fp64 FLOPs on active lanes"}
                             if pmc_ok and achieved is not None and pmc_rec.get("valu_lane_utilization") else None),
                         "kernel_src_sha": src_sha,
                         "pmc_matches_kernel_src": pmc_ok,
                         # PMC counters per FRAME (scripts/make_pmc_json.py); bytes: fetch (raw) / write per frame
                         "pmc": {k: pmc_rec[k] for k in ("valu_busy", "fp64_flops_per_frame", "fetch_bytes",
                                                         "write_bytes", "hbm_bytes_per_frame", "source",
                                                         "kernel_src_sha") if k in pmc_rec},
                         "algorithmic_equivalent": {
                             "achieved": round(brute, 3), "frac": round(brute / FP64_VALU_PEAK_TFLOPS, 4),
                             "per_unit": f"{FLOP_PER_TEST} FLOP per ray-sphere pair x {m['spheres']} spheres x "
                                         f"{m['rank_rays']} rays per frame (SURVEY 8(d), every ray against every "
                                         f"sphere; the kernel prunes pairs exactly, so this exceeds the peak)",
                             "flops_per_frame": FLOP_PER_TEST * m["spheres"] * m["rank_rays"],
                             "flops_per_launch": FLOP_PER_TEST * m["spheres"] * m["rank_rays"] * batch},
                         "executed": {"exact_tests": m["tests_exact"], "cull_tests": m["tests_cull"],
                                      # a lower bound of the executed fp64 work: 25 FLOP per exact test
                                      # + 34 per cull test (device counters), nothing for walks / shading
                                      "test_tflops": round(test_tflops, 3),
                                      "test_tflops_what": f"lower bound: ({FLOP_PER_TEST} x exact + "
                                                          f"{FLOP_PER_CULL} x cull tests) per frame / kernel time",
                                      "frac_of_brute_force_tests": round(
                                          m["tests_exact"] / max(1, m["spheres"] * m["rank_rays"]), 6)},
                         "culling": m["cull"],
                         "kernel_ms_mean": round(m["kernel_ms_mean"], 4),
                         "kernel_ms_min": round(m["kernel_ms_min"], 4),
                         "kernel_ms_per_frame": round(m["kernel_ms_per_frame"], 4),
                         "frames_per_launch": batch,
                         "launches_timed": m["launches_timed"]},
            "hbm_write": {"achieved": round(out_bytes / k_s / 1e9, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                          "frac": round(out_bytes / k_s / 1e9 / HBM_PEAK_GBPS, 6),
                          "bytes_per_frame": out_bytes, "bytes_per_launch": out_bytes * batch},
            "also": also,
        }
        for k in ("single_frame", "moving_camera"):
            if k in m:
                line[k] = m[k]
        if e2e:
            line["e2e"] = e2e
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(m["scene_file"], m["W"], m["H"], m["D"], m["frame_rays"])
            # ray_openmp's loop on the host cores this job may use (16 on the GPU box)
            line["cpu_baseline_all_cores"] = cpu_baseline(m["scene_file"], m["W"], m["H"], m["D"],
                                                          m["frame_rays"], threads=min(16, os.cpu_count() or 1))
        print(json.dumps(line), file=result_out, flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
