"""Probe: two RCCL ranks of gs_comm_init on the one GPU of the box (two
processes, the RCCL id handed over through torch.distributed gloo). RCCL may
refuse two ranks on one device; if it accepts them, gs_run_partitioned over
the two ranks is compared with gs_run bit for bit. Prints one line per rank."""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sim(gossipsim, N, M):
    s = gossipsim.Simulator(peers=N, batch=M, seed=81)
    s.set_topogen_links(5, 50, 150, 40, 130)
    s.connect_gossipsub_peers()
    s.mesh_converge()
    return s


def worker(rank, world, port, outdir):
    for q in (ROOT, os.path.join(ROOT, "dst-libp2p-test-node_amd")):
        sys.path.insert(0, q)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gossipsim
    N, M = 3001, 32
    t = gossipsim.T0_NS + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
    sched = (t, (5 + 11 * np.arange(M)) % N, np.full(M, 15000))
    uid = [gossipsim.Comm.get_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    try:
        comm = gossipsim.Comm(nranks=world, rank=rank, uid=uid[0], device=0)
    except Exception as e:  # RCCL refused: report and leave
        print("rank %d: gs_comm_init refused: %s" % (rank, e), flush=True)
        dist.destroy_process_group()
        return
    sim = _sim(gossipsim, N, M)
    (r,) = comm.run_partitioned([sim], sched)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), tc=r["t_complete"], hops=r["hops"])
    comm.close()
    sim.close()
    dist.barrier()
    if rank == 0:
        ref = _sim(gossipsim, N, M).run(sched)
        parts = [np.load(os.path.join(outdir, "r%d.npz" % q)) for q in range(world)]
        ok = np.array_equal(np.concatenate([p["tc"] for p in parts], axis=1), ref["t_complete"]) and \
            np.array_equal(np.concatenate([p["hops"] for p in parts], axis=1), ref["hops"])
        print("rank 0: two RCCL ranks on one GPU, gs_run_partitioned == gs_run: %s" % ok, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rccl2"
    os.makedirs(out, exist_ok=True)
    mp.spawn(worker, args=(2, _port(), out), nprocs=2, join=True)
