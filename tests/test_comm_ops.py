"""Cross-process ranks of the library-driven partitioned run (SURVEY §8e;
include/gossipsim.h gs_comm_init_ops, ABI 10).

gs_comm_init_ops hands every collective of gs_run_partitioned — the per-pass
control all-gather, the record exchange of the list pass (gathered and routed
layouts: k_lpack ranges, per-peer offset / count tables, lp_route_bases
rebasing), the push protocol's count matrix and bucket MIN, the
message-sharded transposition — to the caller's transport, here
torch.distributed gloo between 2 or 3 processes (gossipsim.TorchDistTransport).

CPU suite: the transport itself through gs_comm_check (one all-gather and one
exchange of position-hashed bytes, no device work) at world 2 and 3, and a
corrupting transport is caught. GPU suite: 2 or 3 processes share the one GPU,
each one rank with its own context; the ranks' rows concatenated equal gs_run
bit for bit, for uneven splits, both list-pass exchange layouts, the push
protocol, and a churn batch (message-sharded)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    for q in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dst-libp2p-test-node_amd")):
        if q not in sys.path:
            sys.path.insert(0, q)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


class _Corrupt:
    """A transport that flips one received byte (rank 0's data from rank 1)."""

    def __init__(self, inner):
        self.inner = inner

    def allgather(self, mine):
        return self.inner.allgather(mine)

    def exchange(self, sends, sizes):
        got = self.inner.exchange(sends, sizes)
        if self.inner.rank == 0 and sizes[1]:
            b = bytearray(got[1])
            b[len(b) // 2] ^= 0x40
            got[1] = bytes(b)
        return got


def _check_worker(rank, world, port, outdir):
    _setup(rank, world, port)
    import gossipsim
    tr = gossipsim.TorchDistTransport()
    comm = gossipsim.Comm(nranks=world, rank=rank, device=0, transport=tr)
    comm.check()
    bad = gossipsim.Comm(nranks=world, rank=rank, device=0, transport=_Corrupt(tr))
    try:
        bad.check()
        caught = False
    except gossipsim.GossipSimError:
        caught = True
    np.save(os.path.join(outdir, "r%d.npy" % rank), np.array([1, int(caught)]))
    comm.close()
    bad.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_comm_ops_transport_check(tmp_path, world):
    mp.spawn(_check_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [np.load(os.path.join(tmp_path, "r%d.npy" % r)) for r in range(world)]
    assert all(g[0] == 1 for g in got)
    assert got[0][1] == 1  # rank 0 saw the flipped byte
    assert all(g[1] == 0 for g in got[1:])


# ---- GPU: P processes, one rank each, on the one GPU ----

T0_OFF = 0
CASES = {  # name: (peers, messages, batch, knobs, env)
    "gather": (3001, 48, 32, {}, {}),
    "route": (3001, 48, 32, {}, {"GS_PART_ROUTE": "1"}),
    "push": (2003, 24, 24, {}, {"GS_PART_PUSH": "1"}),
    "f2_route": (2501, 20, 20, {"fragments": 2}, {"GS_PART_ROUTE": "1"}),
    "churn": (1501, 16, 16, {"churn_ppm": 20000, "lazy_gossip": 1, "churn_horizon": 12}, {}),
}


def _case(name):
    import gossipsim
    N, M, B, knobs, env = CASES[name]
    t = gossipsim.T0_NS + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
    sched = (t, (6 + 7 * np.arange(M)) % N, np.full(M, 15000))
    kw = dict(peers=N, batch=B, seed=71, **knobs)
    if "churn_ppm" in knobs:
        kw["hb_phase_ns"] = gossipsim.SHADOW_START_NS
    return kw, sched, env


def _sim(kw):
    import gossipsim
    s = gossipsim.Simulator(**kw)
    s.set_topogen_links(5, 50, 150, 40, 130)
    s.connect_gossipsub_peers()
    s.mesh_converge()
    return s


def _run_worker(rank, world, port, outdir, name):
    _setup(rank, world, port)
    kw, sched, env = _case(name)
    os.environ.update(env)
    import gossipsim
    sim = _sim(kw)
    comm = gossipsim.Comm(nranks=world, rank=rank, device=0, transport=gossipsim.TorchDistTransport())
    comm.check()
    (r,) = comm.run_partitioned([sim], sched)
    st = sim.stats()
    np.savez(os.path.join(outdir, "r%d.npz" % rank), tc=r["t_complete"], hops=r["hops"],
             rng=np.array(r["peer_range"]),
             st=np.array([st["deliveries"], st["relaxations"], st["list_pull_batches"], st["ms_batches"]]))
    comm.close()
    sim.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("gather", 2), ("gather", 3), ("route", 2), ("route", 3), ("push", 3),
                                        ("f2_route", 3), ("churn", 2)])
def test_run_partitioned_across_processes_equals_gs_run(tmp_path, name, world):
    mp.spawn(_run_worker, args=(world, _free_port(), str(tmp_path), name), nprocs=world, join=True)
    parts = [np.load(os.path.join(tmp_path, "r%d.npz" % r)) for r in range(world)]
    kw, sched, env = _case(name)
    N = kw["peers"]
    assert [tuple(p["rng"]) for p in parts] == [(r * N // world, (r + 1) * N // world) for r in range(world)]
    sim = _sim(kw)  # the whole graph in this process (after the ranks left the GPU)
    ref = sim.run(sched)
    rst = sim.stats()
    np.testing.assert_array_equal(np.concatenate([p["tc"] for p in parts], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([p["hops"] for p in parts], axis=1), ref["hops"])
    assert sum(int(p["st"][0]) for p in parts) == rst["deliveries"]
    assert sum(int(p["st"][1]) for p in parts) == rst["relaxations"]
    if name in ("gather", "route", "f2_route"):
        assert all(p["st"][2] > 0 for p in parts)  # the list pass ran on every rank
    if name == "push":
        assert all(p["st"][2] == 0 for p in parts)
    if name == "churn":
        assert all(p["st"][3] > 0 for p in parts)  # message-sharded batches
