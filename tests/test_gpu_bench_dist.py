"""bench.py's multi-rank data path rehearsed on one GPU (--force-dist: an RCCL
process group of world size 1, the batched shard gather, the device
unpermute): the bench line must carry a frame reassembled from the gathered
shards that equals a direct full-frame render byte for byte."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["1", "4", "16"])
def test_bench_force_dist_reassembles_frame(batch):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29540 + int(batch)))
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--force-dist", "--no-cpu-baseline",
                          "--no-also", "--steps", "7", "--warmup", "1", "--frames-per-launch", batch,
                          "--workload", "medium_1920x1080_d2"],
                         capture_output=True, text=True, timeout=150, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.strip().splitlines()
    assert len(lines) == 1, out.stdout[-2000:]  # RCCL's banner goes to stderr
    line = json.loads(lines[0])
    assert line["config"]["assembled_frame_equals_single_gpu_render"] is True
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["gather_ms_per_batch"] > 0 and line["config"]["kernel_ms_per_frame_max_rank"] > 0


@pytest.mark.gpu
def test_bench_gpus2_launches_ranks_or_fails_fast():
    """`bench.py --gpus 2` with no external launcher: on a box with 2+ GPUs it
    starts two ranks itself (the line says n_gpus 2 and the reassembled frame
    equals a direct render); on a 1-GPU box it exits non-zero at once, with no
    line, instead of measuring one GPU."""
    import torch

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu-baseline",
                          "--no-also", "--steps", "4", "--warmup", "1", "--frames-per-launch", "2",
                          "--workload", "medium_1920x1080_d2"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    if torch.cuda.device_count() < 2:
        assert out.returncode == 2, out.stderr[-2000:]
        assert "visible GPUs" in out.stderr and out.stdout == ""
        return
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["world_size_seen"] == 2
    assert line["config"]["assembled_frame_equals_single_gpu_render"] is True
