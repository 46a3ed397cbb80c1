"""bench.py --gpus N without torchrun starts N rank processes itself
(bench.launch_ranks) and relays rank 0's JSON line. CPU only: a stub worker
stands in for the GPU ranks; the real script on a CPU box must fail loudly
(no device) rather than time one rank and call it the job."""
import io
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

STUB = r"""
import json, os, sys
out = sys.argv[1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
env = {k: os.environ.get(k) for k in keys}
open(os.path.join(out, "rank%s.json" % env["RANK"]), "w").write(json.dumps(env))
if env["RANK"] == "0":
    print("some log line")
    print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": int(env["WORLD_SIZE"])}))
code = int(os.environ.get("STUB_FAIL_RANK", "-1"))
sys.exit(3 if code == int(env["RANK"]) else 0)
"""


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_gives_each_rank_its_environment(tmp_path, n):
    buf = io.StringIO()
    rc = bench.launch_ranks(n, [], cmd=[sys.executable, "-c", STUB, str(tmp_path)], out=buf)
    assert rc == 0
    envs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(n)]
    assert sorted(int(e["RANK"]) for e in envs) == list(range(n))
    assert all(e["LOCAL_RANK"] == e["RANK"] for e in envs)
    assert {e["WORLD_SIZE"] for e in envs} == {str(n)}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    line = buf.getvalue().strip().splitlines()
    assert len(line) == 1  # only rank 0's result line is relayed
    assert json.loads(line[0])["n_gpus"] == n


def test_launcher_propagates_a_failing_rank(tmp_path):
    env = dict(os.environ, STUB_FAIL_RANK="1")
    buf = io.StringIO()
    rc = bench.launch_ranks(2, [], cmd=[sys.executable, "-c", STUB, str(tmp_path)], env=env, out=buf)
    assert rc == 3
    assert buf.getvalue() == ""


def test_bench_gpus2_on_cpu_fails_loudly():
    """The real script: two ranks start, neither finds a device, the launcher
    exits non-zero and prints no result line."""
    if not os.path.exists(os.path.join(ROOT, "dst-libp2p-test-node_amd", "libgossipsim.so")):
        pytest.skip("libgossipsim.so not built")
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--peers", "1000", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "{" not in r.stdout
    assert "rank" in r.stderr
