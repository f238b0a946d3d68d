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
