"""GPU parity of the peer-partitioned mode.

P partitions live as P contexts on the one GPU and exchange records through
partition.LoopbackExchange; the per-partition results, concatenated over the
peer ranges, must equal the oracle (and gs_run) bit for bit, and the counters
summed over partitions must equal the single-device counters."""
import numpy as np
import pytest

import gossipsim
import oracle
import partition

pytestmark = pytest.mark.gpu
T0 = gossipsim.T0_NS


def _sched(M, N, size=15000, pub0=6):
    t = T0 + np.arange(M, dtype=np.uint64) * np.uint64(1_000_000_000)
    return t, (pub0 + np.arange(M)) % N, np.full(M, size)


def _parts(p, S, links, parts, batch):
    kw = {n: getattr(p, n) for n, _ in oracle.OrParams._fields_}
    kw["batch"] = batch
    sims = []
    for i in range(parts):
        s = gossipsim.Simulator(**kw)
        s.set_topogen_links(S, *links)
        s.connect_gossipsub_peers()
        s.mesh_converge()
        s.set_partition(parts, i)
        sims.append(s)
    return sims


def _check(p, S, links, parts, sched, small_buffers=False):
    import torch
    sims = _parts(p, S, links, parts, len(sched[0]))
    bufs = [partition.RecordBuffer(torch.device("cuda", 0), capacity=16 if small_buffers else 1 << 16)
            for _ in sims]
    res, info = partition.run_partitioned(sims, sched, partition.LoopbackExchange(), bufs=bufs)
    ref = oracle.simulate(p, S, links, sched=sched)
    tc = np.concatenate([r["t_complete"] for r in res], axis=1)
    hops = np.concatenate([r["hops"] for r in res], axis=1)
    np.testing.assert_array_equal(tc, ref["t_complete"])
    np.testing.assert_array_equal(hops, ref["hops"])
    st = [s.stats() for s in sims]
    for k in ("deliveries", "frag_deliveries", "relaxations", "bytes_alg", "latency_sum_ms"):
        assert sum(x[k] for x in st) == ref["stats"][k], k
    assert max(x["latency_max_ms"] for x in st) == ref["stats"]["latency_max_ms"]
    assert all(x["messages"] == len(sched[0]) for x in st)
    return info


@pytest.mark.parametrize("parts,frags", [(1, 1), (2, 1), (3, 2), (4, 4), (2, 3)])
def test_partitioned_matches_oracle(parts, frags):
    p = oracle.params(peers=1200, seed=51, fragments=frags)
    info = _check(p, 5, (50, 150, 40, 130), parts, _sched(16, 1200))
    assert info["buckets"] > 0 and info["records"] > 0


def test_partitioned_grows_record_buffer_and_uneven_ranges():
    p = oracle.params(peers=1001, seed=52)  # 1001 / 3: uneven peer ranges
    _check(p, 3, (20, 200, 10, 90), 3, _sched(9, 1001), small_buffers=True)


def test_partitioned_knobs():
    for kw, S, links in [(dict(peers=600, seed=53, flood_publish=0), 1, (50, 50, 50, 50)),
                         (dict(peers=500, seed=54, muxer=1, signed_msgs=0, d=8, d_lo=6, d_hi=12), 2,
                          (10, 100, 5, 50))]:
        _check(oracle.params(**kw), S, links, 2, _sched(7, kw["peers"]))


@pytest.mark.parametrize("frags", [1, 2])
def test_partitioned_p8_10k_peers(frags):
    """The config #4 split (P = 8) as loop-back partitions on one GPU, 10k peers."""
    p = oracle.params(peers=10_000, seed=57, fragments=frags)
    info = _check(p, 5, (50, 150, 40, 130), 8, _sched(8, 10_000))
    assert info["buckets"] > 0


def test_partitioned_unsupported_modes_fail_loudly():
    """Lazy gossip runs in partitioned mode only as the proven no-op (every part
    checks its peers at gs_part_finish); a heartbeat at the publish instant
    makes IWANTs possible and the batch fails instead of dropping them.
    IDONTWANT and per-peer traffic are refused at gs_part_begin."""
    p = oracle.params(peers=300, seed=55, lazy_gossip=1, hb_phase_ns=T0 % 1_000_000_000)
    (s,) = _parts(p, 1, (50, 50, 50, 50), 1, 4)
    with pytest.raises(gossipsim.GossipSimError, match="GS_EUNSUPPORTED"):
        partition.run_partitioned([s], _sched(4, 300), partition.LoopbackExchange())
    p = oracle.params(peers=300, seed=56, idontwant=1000)
    (s,) = _parts(p, 1, (50, 50, 50, 50), 1, 4)
    with pytest.raises(gossipsim.GossipSimError, match="GS_EUNSUPPORTED"):
        s.part_begin(_sched(4, 300))
    with pytest.raises(gossipsim.GossipSimError, match="GS_ESTATE"):
        s.part_relax(1, 0, 0)
    p = oracle.params(peers=300, seed=57)
    (s,) = _parts(p, 1, (50, 50, 50, 50), 1, 4)
    s.set_traffic(True)  # no traffic pass in partitioned mode
    with pytest.raises(gossipsim.GossipSimError, match="GS_EUNSUPPORTED"):
        s.part_begin(_sched(4, 300))


# ---- the library-driven protocol behind the C ABI (gs_comm_*, gs_run_partitioned) ----

def _whole(p, S, links, sched, batch):
    sims = _parts(p, S, links, 1, batch)
    return sims[0].run(sched), sims[0].stats()


@pytest.mark.parametrize("parts,frags,batch", [(2, 1, 16), (3, 2, 16), (8, 1, 16), (4, 3, 6)])
def test_run_partitioned_local_comm_equals_gs_run(parts, frags, batch):
    """gs_run_partitioned with gs_comm_init_local: P parts on one GPU, records
    routed only to the parts owning a target; bit-identical to gs_run (several
    batches when batch < messages) and to the oracle, counters summed over parts."""
    p = oracle.params(peers=3000, seed=58, fragments=frags)
    sched = _sched(16, 3000)
    ref, rst = _whole(p, 5, (50, 150, 40, 130), sched, batch)
    sims = _parts(p, 5, (50, 150, 40, 130), parts, batch)
    comm = gossipsim.Comm(local_parts=parts)
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ref["hops"])
    st = [s.stats() for s in sims]
    for k in ("deliveries", "frag_deliveries", "relaxations", "bytes_alg", "latency_sum_ms"):
        assert sum(x[k] for x in st) == rst[k], k
    assert sum(x["gossip_noop_msgs"] for x in st) == 16 * parts
    ora = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
    np.testing.assert_array_equal(ref["t_complete"], ora["t_complete"])
    comm.close()


@pytest.mark.parametrize("mode", ["gather", "route", "route_copy", "push"])
@pytest.mark.parametrize("parts,frags,batch", [(2, 1, 64), (5, 2, 32), (8, 1, 1024), (12, 2, 32), (16, 1, 64)])
def test_run_partitioned_list_pass_and_push_protocol(monkeypatch, mode, parts, frags, batch):
    """gs_run_partitioned runs each part's rows on the list pass (records
    exchanged between passes: routed to the parts owning a receiver, stored
    straight into the destination contexts — the loop-back default — or
    through send segments and copies as ranks do (GS_PART_DIRECT=0), or with
    GS_PART_ROUTE=0 every part's to every part) — or, with GS_PART_PUSH, on
    the push protocol — bit-identical to gs_run and the oracle; uneven part
    sizes, fragments, rows of 1024 lanes; 2-4, 5-8 and 9-16 parts take the
    routed pack's three destination widths (k_lpack_route<4 / 8 / 16>)."""
    push = mode == "push"
    if push:
        monkeypatch.setenv("GS_PART_PUSH", "1")
    if mode == "gather":
        monkeypatch.setenv("GS_PART_ROUTE", "0")
    if mode == "route_copy":
        monkeypatch.setenv("GS_PART_ROUTE", "1")
        monkeypatch.setenv("GS_PART_DIRECT", "0")
    N = 3001
    p = oracle.params(peers=N, seed=65, fragments=frags)
    sched = _sched(batch, N)
    ref, rst = _whole(p, 5, (50, 150, 40, 130), sched, batch)
    sims = _parts(p, 5, (50, 150, 40, 130), parts, batch)
    comm = gossipsim.Comm(local_parts=parts)
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ref["hops"])
    st = [s.stats() for s in sims]
    for k in ("deliveries", "frag_deliveries", "relaxations", "latency_sum_ms"):
        assert sum(x[k] for x in st) == rst[k], k
    assert all((x["list_pull_batches"] > 0) != push for x in st)
    if not push and batch <= 64:
        ora = oracle.simulate(p, 5, (50, 150, 40, 130), sched=sched)
        np.testing.assert_array_equal(ref["t_complete"], ora["t_complete"])
    comm.close()


def test_run_partitioned_more_parts_than_routes(monkeypatch):
    """17 loop-back parts: more than the routed pack's 16 destinations, so the
    list pass gathers every part's records (GS_PART_ROUTE=1 cannot force
    routing past PART_ROUTE_PMAX); bit-identical to gs_run."""
    monkeypatch.setenv("GS_PART_ROUTE", "1")
    N, parts, batch = 3001, 17, 32
    p = oracle.params(peers=N, seed=66)
    sched = _sched(batch, N)
    ref, rst = _whole(p, 5, (50, 150, 40, 130), sched, batch)
    sims = _parts(p, 5, (50, 150, 40, 130), parts, batch)
    comm = gossipsim.Comm(local_parts=parts)
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ref["hops"])
    st = [s.stats() for s in sims]
    assert sum(x["deliveries"] for x in st) == rst["deliveries"]
    assert all(x["list_pull_batches"] > 0 for x in st)
    comm.close()


def test_run_partitioned_list_overflow_falls_back_to_push(monkeypatch):
    """Candidate lists capped at 2 entries: some part overflows, every part
    restores its counters and the batch runs on the push protocol."""
    monkeypatch.setenv("GS_LPULL_CAP", "2")
    N = 2500
    p = oracle.params(peers=N, seed=66)
    sched = _sched(128, N)
    ref, rst = _whole(p, 5, (50, 150, 40, 130), sched, 128)
    sims = _parts(p, 5, (50, 150, 40, 130), 3, 128)
    comm = gossipsim.Comm(local_parts=3)
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ref["t_complete"])
    st = [s.stats() for s in sims]
    assert sum(x["relaxations"] for x in st) == rst["relaxations"]
    assert all(x["list_pull_batches"] == 0 for x in st)
    comm.close()


@pytest.mark.parametrize("route", [False, True])
@pytest.mark.parametrize("N,M", [(2000, 12), (100_000, 64)])
def test_run_partitioned_rccl_single_rank(monkeypatch, N, M, route):
    """gs_comm_init over RCCL with one rank on this GPU (the N = 1 case of the
    multi-GPU bench): the same protocol through RCCL's all-gather, grouped
    send/recv and MIN all-reduce (and the routed exchange's count matrix),
    bit-identical to gs_run."""
    if route:
        monkeypatch.setenv("GS_PART_ROUTE", "1")
    p = oracle.params(peers=N, seed=59)
    sched = _sched(M, N)
    ref, _ = _whole(p, 5, (50, 150, 40, 130), sched, M)
    (s,) = _parts(p, 5, (50, 150, 40, 130), 1, M)
    comm = gossipsim.Comm(nranks=1, rank=0, uid=gossipsim.Comm.get_id(), device=0)
    (r,) = comm.run_partitioned([s], sched)
    np.testing.assert_array_equal(r["t_complete"], ref["t_complete"])
    np.testing.assert_array_equal(r["hops"], ref["hops"])
    comm.close()


@pytest.mark.parametrize("piece", [1 << 20, (1 << 22) + 24 * 7])
def test_run_partitioned_rccl_many_pieces(monkeypatch, piece):
    """The RCCL record exchange cut into many ncclSend / ncclRecv pieces
    (GS_RCCL_PIECE_BYTES; 2^30 B by default): every bucket's
    transfer of a 100k-peer, 64-message batch spans several pieces, incl. a
    piece size that is not a multiple of the 24-B record; bit-identical to
    gs_run."""
    monkeypatch.setenv("GS_RCCL_PIECE_BYTES", str(piece))
    N, M = 100_000, 64
    p = oracle.params(peers=N, seed=61)
    sched = _sched(M, N)
    ref, rst = _whole(p, 5, (50, 150, 40, 130), sched, M)
    (s,) = _parts(p, 5, (50, 150, 40, 130), 1, M)
    comm = gossipsim.Comm(nranks=1, rank=0, uid=gossipsim.Comm.get_id(), device=0)
    (r,) = comm.run_partitioned([s], sched)
    np.testing.assert_array_equal(r["t_complete"], ref["t_complete"])
    np.testing.assert_array_equal(r["hops"], ref["hops"])
    assert s.stats()["relaxations"] == rst["relaxations"]
    comm.close()


def _ms_check(p, S, links, parts, sched, batch, rccl=False,
              summed=("deliveries", "frag_deliveries", "gossip_iwant", "latency_sum_ms")):
    """gs_run_partitioned against gs_run and the oracle on a batch the peer
    protocols hand to the message-sharded path; counters summed over parts."""
    ref, rst = _whole(p, S, links, sched, batch)
    ora = oracle.simulate(p, S, links, sched=sched)
    np.testing.assert_array_equal(ref["t_complete"], ora["t_complete"])
    np.testing.assert_array_equal(ref["hops"], ora["hops"])
    sims = _parts(p, S, links, 1 if rccl else parts, batch)
    comm = (gossipsim.Comm(nranks=1, rank=0, uid=gossipsim.Comm.get_id(), device=0) if rccl
            else gossipsim.Comm(local_parts=parts))
    res = comm.run_partitioned(sims, sched)
    np.testing.assert_array_equal(np.concatenate([r["t_complete"] for r in res], axis=1), ora["t_complete"])
    np.testing.assert_array_equal(np.concatenate([r["hops"] for r in res], axis=1), ora["hops"])
    st = [s.stats() for s in sims]
    for k in summed:
        assert sum(x[k] for x in st) == rst[k], k
    assert sum(x["deliveries"] for x in st) == ora["stats"]["deliveries"]
    assert all(x["messages"] == len(sched[0]) for x in st)
    comm.close()
    return st, rst


@pytest.mark.parametrize("parts,batch", [(3, 16), (8, 8), (3, 2)])
def test_run_partitioned_gossip_iwants_message_sharded(parts, batch):
    """A heartbeat at the publish instant: IHAVEs land before the last
    delivery, the peer protocols' eager result is discarded (counters restored)
    and the batch runs message-sharded with gossip; IWANTs taken, bit-exact
    against gs_run and the oracle (batch 2 < P = 3: parts with no messages)."""
    N = 3000
    p = oracle.params(peers=N, seed=60, lazy_gossip=1, hb_phase_ns=T0 % 1_000_000_000)
    st, rst = _ms_check(p, 5, (50, 150, 40, 130), parts, _sched(16, N), batch)
    assert rst["gossip_iwant"] > 0
    assert all(x["ms_batches"] == 16 // batch and x["gossip_fallback_batches"] >= 16 // batch for x in st)


@pytest.mark.parametrize("parts", [2, 8])
def test_run_partitioned_churn_message_sharded(parts):
    """Config #3's knobs (churn + lazy gossip, heterogeneous links) in
    partitioned mode: every batch message-sharded over the replicated graph
    (each part replays the churn epochs its messages need), loop-back P = 8,
    bit-exact against the oracle."""
    N = 4000
    p = oracle.params(peers=N, seed=62, churn_ppm=20000, hb_phase_ns=gossipsim.SHADOW_START_NS, lazy_gossip=1)
    st, rst = _ms_check(p, 5, (50, 150, 40, 130), parts, _sched(24, N), 8)
    assert rst["gossip_iwant"] > 0 and all(x["ms_batches"] == 3 for x in st)


def test_run_partitioned_idontwant_message_sharded():
    """The go preset (IDONTWANT above 1000 B, go-test-node/main.go:153-175)
    in partitioned mode, P = 4."""
    N = 3000
    p = oracle.params_for("go", peers=N, seed=63)
    st, _ = _ms_check(p, 5, (50, 150, 40, 130), 4, _sched(12, N), 12)
    assert all(x["ms_batches"] == 1 for x in st)


@pytest.mark.parametrize("piece", [0, 1 << 16])
def test_run_partitioned_rccl_message_sharded(monkeypatch, piece):
    """The message-sharded path over RCCL (one rank: pack, grouped send/recv
    of the result rows, in pieces with GS_RCCL_PIECE_BYTES) with churn and
    gossip."""
    if piece:
        monkeypatch.setenv("GS_RCCL_PIECE_BYTES", str(piece))
    N = 20_000
    p = oracle.params(peers=N, seed=64, churn_ppm=20000, hb_phase_ns=gossipsim.SHADOW_START_NS, lazy_gossip=1)
    st, _ = _ms_check(p, 5, (50, 150, 40, 130), 1, _sched(16, N), 16, rccl=True)
    assert st[0]["ms_batches"] == 1


def test_run_partitioned_refuses_traffic():
    """Per-peer traffic is the one knob partitioned mode refuses."""
    p = oracle.params(peers=600, seed=60)
    sims = _parts(p, 1, (50, 50, 50, 50), 2, 4)
    for s in sims:
        s.set_traffic(True)
    comm = gossipsim.Comm(local_parts=2)
    with pytest.raises(gossipsim.GossipSimError, match="GS_EUNSUPPORTED"):
        comm.run_partitioned(sims, _sched(4, 600))
    comm.close()
