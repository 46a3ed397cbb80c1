"""bench.py's N-rank path on the GPU box (`-m gpu`): `--gpus 2` launches two
ranks itself (no torchrun); on a box with fewer GPUs than ranks they share
the device and reduce their timing / counter scalars over gloo. Each rank
simulates its own message shard (message sharding, no data-path collective),
so the line's deliveries are 2 x (messages per rank) x (peers - 1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_message_sharded():
    N, B, K = 20_000, 64, 2
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--peers", str(N), "--batch", str(B),
           "--steps", str(K), "--warmup", "1", "--configs", "0", "--cpu-seconds", "0", "--also-peers", "0",
           "--gossip-check", "0", "--output-steps", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "msg-shard2"
    assert line["dist"]["ranks"] == 2
    assert line["deliveries"] == 2 * K * B * (N - 1)
    assert line["value"] > 0 and line["gossip"]["fallback_batches"] == 0
