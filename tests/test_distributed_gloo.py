"""World-size-2 gloo test of the message-sharded multi-GPU path (CPU only).

Each rank takes its shard with gossipsim.shard_messages (what bench.py does per
GPU), simulates it (here with the CPU oracle standing in for the device, since
no GPU is present), and the counters/timings are reduced with bench.py's own
helpers. The union must equal a single-process run over all messages
bit for bit (messages are independent given the frozen mesh)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, B, STEPS, WORLD = 400, 6, 2, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph():
    import oracle
    p = oracle.params(peers=N, seed=17)
    lat, bw = oracle.topogen_links(5, 50, 150, 40, 130)
    stage = (np.arange(N) % 5).astype(np.uint8)
    row, col, flags = oracle.build_topology(p)
    flags, mesh, cnt, _ = oracle.mesh_converge(p, row, col, flags, stage, lat)
    return p, (row, col, mesh, cnt, stage, lat, bw)


def _worker(rank, port, outdir):
    for q in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dst-libp2p-test-node_amd")):
        sys.path.insert(0, q)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    import bench
    import gossipsim
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    p, (row, col, mesh, cnt, stage, lat, bw) = _graph()
    tcs, tot = [], np.zeros(4)
    for step in range(STEPS):
        t, pub, size = gossipsim.shard_messages(step, rank, WORLD, B, N, 15000)
        tc, hops, st = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, t, pub, size)
        tcs.append((t, tc))
        tot += [st["deliveries"], st["frag_deliveries"], st["relaxations"], st["bytes_alg"]]
    red = bench.allreduce(torch, dist, WORLD, tot.tolist(), dist.ReduceOp.SUM)
    mx = bench.allreduce(torch, dist, WORLD, [float(rank + 1)], dist.ReduceOp.MAX)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), t=np.concatenate([x[0] for x in tcs]),
             tc=np.concatenate([x[1] for x in tcs]), red=np.array(red), mx=np.array(mx))
    dist.barrier()
    dist.destroy_process_group()


def test_message_sharding_world2_matches_single_process(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    import gossipsim
    import oracle
    p, (row, col, mesh, cnt, stage, lat, bw) = _graph()
    M = STEPS * WORLD * B
    t = gossipsim.T0_NS + np.arange(M, dtype=np.uint64) * np.uint64(gossipsim.DELAY_NS)
    pub = (gossipsim.PUBLISHER0 + np.arange(M)) % N
    tc, _, st = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, t, pub, np.full(M, 15000))
    parts = [np.load(os.path.join(tmp_path, "r%d.npz" % r)) for r in range(WORLD)]
    got_t = np.concatenate([x["t"] for x in parts])
    got_tc = np.concatenate([x["tc"] for x in parts])
    order = np.argsort(got_t)
    np.testing.assert_array_equal(got_t[order], t)
    np.testing.assert_array_equal(got_tc[order], tc)
    for x in parts:
        assert list(x["red"]) == [st["deliveries"], st["frag_deliveries"], st["relaxations"], st["bytes_alg"]]
        assert list(x["mx"]) == [2.0]
