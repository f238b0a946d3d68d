"""CPU: bench.py's own rank launcher (`bench.py --gpus N` with no external
launcher) and its refusals.  A stub child stands in for the rank processes:
it records the env it was started with, prints one line, and exits with the
code the test asks for.  The driver's 8-GPU run must never silently measure
one GPU: --gpus N starts N ranks or fails, and a launcher/flag mismatch fails."""
import importlib.util
import io
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO

STUB = r"""
import json, os, sys, time
rank = int(os.environ["RANK"])
with open(os.path.join(sys.argv[1], "rank%d.json" % rank), "w") as f:
    json.dump({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                              "MASTER_ADDR", "MASTER_PORT")}, f)
print(json.dumps({"rank": rank, "line": "result"}), flush=True)
fail = os.environ.get("STUB_FAIL_RANK")
if fail is not None and int(fail) == rank:
    sys.exit(3)
if fail is not None:
    time.sleep(60)  # the others hang: the launcher must end them
"""


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return [sys.executable, str(p), str(tmp_path)]


def test_launcher_starts_n_ranks_with_torchrun_env(stub, tmp_path, monkeypatch):
    monkeypatch.delenv("STUB_FAIL_RANK", raising=False)
    out = io.StringIO()
    rc = _bench().launch_ranks(4, ["--gpus", "4"], child=stub, gpu_count=8, out=out)
    assert rc == 0
    lines = out.getvalue().strip().splitlines()
    assert [json.loads(x)["rank"] for x in lines] == [0]  # only rank 0's stdout is relayed
    envs = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and int(envs[0]["MASTER_PORT"]) > 0


def test_launcher_fails_and_ends_the_other_ranks(stub, monkeypatch):
    monkeypatch.setenv("STUB_FAIL_RANK", "1")
    t0 = time.time()
    rc = _bench().launch_ranks(3, [], child=stub, gpu_count=3, out=io.StringIO())
    assert rc == 3
    assert time.time() - t0 < 30  # ranks 0 and 2 (sleeping 60 s) were terminated


def test_launcher_refuses_more_ranks_than_gpus(stub, tmp_path):
    rc = _bench().launch_ranks(2, [], child=stub, gpu_count=1, out=io.StringIO())
    assert rc == 2
    assert not list(tmp_path.glob("rank*.json"))  # nothing was started


def _run_bench(args, env_extra, drop=()):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env, cwd=REPO)


def test_bench_world_size_mismatch_fails():
    out = _run_bench(["--gpus", "8"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode == 2 and "disagree" in out.stderr
    assert out.stdout == ""


def test_bench_gpus_without_gpus_fails_fast():
    # no GPU in this container: --gpus 2 must not fall back to a 1-GPU line
    out = _run_bench(["--gpus", "2"], {}, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK"))
    assert out.returncode == 2 and "visible GPUs" in out.stderr
    assert out.stdout == ""
