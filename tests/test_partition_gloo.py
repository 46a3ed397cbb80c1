"""World-size-2 gloo test of the peer-partitioned path.

partition.run_partitioned + DistExchange drive the bucket protocol of
include/gossipsim.h (gs_part_begin / scan / relax / finish). On the GPU those
steps are HIP kernels (tests/test_gpu_partition.py); here each rank drives a
numpy restatement of the same four steps for F = 1 (_PartModel, written from
the protocol in csrc/gs_part.h), so the exchange - record all-gather, next-key
MIN reduction, termination - is exercised over real gloo collectives. The
concatenated per-partition results must equal the oracle's single-process
run bit for bit."""
import ctypes
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, M, WORLD, STAGES = 360, 5, 2, 3
INF = (1 << 64) - 1
EMPTY = 0xFFFFFFFF


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph():
    import oracle
    p = oracle.params(peers=N, seed=23)
    lat, bw = oracle.topogen_links(STAGES, 20, 200, 10, 90)
    stage = (np.arange(N) % STAGES).astype(np.uint8)
    row, col, flags = oracle.build_topology(p)
    flags, mesh, cnt, _ = oracle.mesh_converge(p, row, col, flags, stage, lat)
    return p, (row, col, mesh, cnt, stage, lat, bw)


def _sched():
    import gossipsim
    t = gossipsim.T0_NS + np.arange(M, dtype=np.uint64) * np.uint64(gossipsim.DELAY_NS)
    return t, (gossipsim.PUBLISHER0 + np.arange(M)) % N, np.full(M, 15000)


def _words(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_int64 * max(3 * n, 1)).from_address(ptr))[:3 * n]


class _PartModel:
    """numpy restatement of the gs_part_* steps for F = 1 (no uplink fold)."""

    def __init__(self, p, graph, parts, part):
        import oracle
        self.oracle = oracle
        self.p = p
        self.row, self.col, self.mesh, _, self.stage, self.lat, self.bw = graph
        self.u0, self.u1 = part * N // parts, (part + 1) * N // parts
        sb = 1
        while (1 << sb) < N:
            sb += 1
        self.sb, self.tshift = sb, sb + 6

    def _own(self, w):
        return self.u0 <= w < self.u1

    def part_begin(self, schedule):
        t, pub, size = schedule
        self.tpub, self.pub = [int(x) for x in t], [int(x) for x in pub]
        wire = self.oracle.wire_bytes(int(size[0]), self.p.muxer, self.p.signed_msgs)
        self.ser = [(wire * 8_000_000_000 + int(b) - 1) // int(b) for b in self.bw]
        self.delta = int(self.lat.min()) + min(self.ser)
        self.keys = [[INF] * len(t) for _ in range(self.u1 - self.u0)]
        nmin = INF
        for m, pm in enumerate(self.pub):
            if self._own(pm):
                self.keys[pm - self.u0][m] = pm
            sp = self.stage[pm]
            for j, w in enumerate(self.col[self.row[pm]:self.row[pm + 1]]):
                sw = self.stage[w]
                arr = (j + 1) * self.ser[sp] + int(self.lat[sp, sw]) + max(0, self.ser[sw] - self.ser[sp])
                nk = (arr << self.tshift) | (1 << self.sb) | pm
                if self._own(w) and nk < self.keys[w - self.u0][m]:
                    self.keys[w - self.u0][m] = nk
                    nmin = min(nmin, nk)
        return nmin

    def _targets(self, u, src, pm):
        return [int(w) for w in self.mesh[u] if w != EMPTY and w != src and w != pm]

    def part_scan(self, key, ptr, cap):
        lo = ((key >> self.tshift) // self.delta) * self.delta
        self.hi = hi = lo + self.delta
        smask = (1 << self.sb) - 1
        recs, m1 = [], INF
        for i, row in enumerate(self.keys):
            u = self.u0 + i
            for m, k in enumerate(row):
                if k == INF:
                    continue
                t = k >> self.tshift
                if t >= hi:
                    m1 = min(m1, k)
                elif t >= lo and u != self.pub[m] and self._targets(u, k & smask, self.pub[m]):
                    recs.append((k, t, u, m))
        if len(recs) > cap:
            return False, len(recs), m1
        w = _words(ptr, len(recs)).view(np.uint64)
        for q, (k, st, u, m) in enumerate(recs):
            w[3 * q:3 * q + 3] = [k, st, u | (m << 32)]
        return True, len(recs), m1

    def part_relax(self, key, ptr, n):
        w = _words(ptr, n).view(np.uint64)
        smask = (1 << self.sb) - 1
        final = [[k != INF and (k >> self.tshift) < self.hi for k in row] for row in self.keys]
        nmin = INF
        for q in range(n):
            k, start, pu = int(w[3 * q]), int(w[3 * q + 1]), int(w[3 * q + 2])
            u, m = pu & 0xFFFFFFFF, pu >> 32
            hp = (k >> self.sb) & 63
            su = self.stage[u]
            for pos, v in enumerate(self._targets(u, k & smask, self.pub[m]), 1):
                if not self._own(v) or final[v - self.u0][m]:
                    continue
                sv = self.stage[v]
                arr = start + pos * self.ser[su] + int(self.lat[su, sv]) + max(0, self.ser[sv] - self.ser[su])
                nk = (arr << self.tshift) | ((hp + 1) << self.sb) | u
                if nk < self.keys[v - self.u0][m]:
                    self.keys[v - self.u0][m] = nk
                    nmin = min(nmin, nk)
        return nmin

    def part_finish(self, collect=True):
        tc = np.full((len(self.pub), self.u1 - self.u0), INF, np.uint64)
        for i, row in enumerate(self.keys):
            for m, k in enumerate(row):
                if self.u0 + i == self.pub[m]:
                    tc[m, i] = self.tpub[m]
                elif k != INF:
                    tc[m, i] = self.tpub[m] + (k >> self.tshift)
        return {"t_complete": tc}


def _worker(rank, port, outdir):
    for q in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dst-libp2p-test-node_amd")):
        sys.path.insert(0, q)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import partition
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    p, graph = _graph()
    model = _PartModel(p, graph, WORLD, rank)
    bufs = [partition.RecordBuffer(torch.device("cpu"), capacity=8)]  # forces the grow path
    res, info = partition.run_partitioned([model], _sched(), partition.DistExchange(), bufs=bufs)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), tc=res[0]["t_complete"],
             info=np.array([info["buckets"], info["records"]]))
    dist.barrier()
    dist.destroy_process_group()


def test_key_order_map_is_monotone():
    import partition
    ks = [0, 1, 5, (1 << 63) - 1, 1 << 63, INF - 1, INF]
    ss = [partition.key_to_i64(k) for k in ks]
    assert ss == sorted(ss) and all(-(1 << 63) <= s < (1 << 63) for s in ss)
    assert [partition.i64_to_key(s) for s in ss] == ks


def test_peer_partitioned_world2_matches_oracle(tmp_path):
    import oracle
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    p, (row, col, mesh, cnt, stage, lat, bw) = _graph()
    t, pub, size = _sched()
    tc, _, _ = oracle.run(p, row, col, mesh, cnt, stage, lat, bw, bw, t, pub, size)
    parts = [np.load(os.path.join(tmp_path, "r%d.npz" % r)) for r in range(WORLD)]
    np.testing.assert_array_equal(np.concatenate([x["tc"] for x in parts], axis=1), tc)
    assert (parts[0]["info"] == parts[1]["info"]).all() and parts[0]["info"][1] > 0
