#!/usr/bin/env python3
"""bench.py — simulated peer-message deliveries/s of the GossipSub dissemination
hot path on MI355X (BASELINE.json metric), plus the relaxation kernel's
roofline fraction and the CPU oracle's rate on a bounded sample.

One step = one batch of B messages disseminated over a frozen 1M-peer mesh
(publish -> flood -> mesh forwarding -> reassembly), inputs resident in HBM.
Multi-GPU: one process per GPU, each simulating its own message shard (weak
scaling; no data-path collective). Under torchrun the ranks come
from the environment; `python bench.py --gpus N` without it starts the N rank
processes itself (launch_ranks) before anything touches a GPU and relays rank
0's line. `--mode peer` instead partitions the peers across ranks and
exchanges each pass's records over RCCL (strong scaling of one batch, config
#4).

    python bench.py --gpus 1 --steps 20 --warmup 3
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dst-libp2p-test-node_amd"))

import numpy as np  # noqa: E402

import gossipsim  # noqa: E402

METRIC = "simulated peer-msg deliveries/sec at 100k & 1M peers; % of HBM BW"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def exchange_label(world, parts):
    """The partitioned list pass's record exchange (gs_comm.hip
    gs_run_partitioned): loop-back parts on one device route by default with
    direct stores; ranks gather by default; GS_PART_ROUTE / GS_PART_DIRECT
    override."""
    rte, dre = os.environ.get("GS_PART_ROUTE", ""), os.environ.get("GS_PART_DIRECT", "")
    local = world == 1 and parts > 1
    direct_ok = local and dre != "0"
    routed = ((rte != "0") if rte else direct_ok) and max(world, parts) <= 16  # PART_ROUTE_PMAX
    if not routed:
        return "gathered"
    return "routed, direct stores" if direct_ok else "routed, send segments"


def fp_lanes(f):
    p = 1
    while p < f:
        p <<= 1
    return p


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--peers", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--fragments", type=int, default=1)
    ap.add_argument("--msg-size", type=int, default=15000)
    ap.add_argument("--links", default="5,50,150,40,130", help="stages,bl,bh,ll,lh (topogen.py)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-heartbeats", type=int, default=400)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU oracle sample budget (0=off)")
    ap.add_argument("--cpu-gossip", type=int, default=0, help="also time the oracle with lazy gossip on (slow)")
    ap.add_argument("--output-steps", type=int, default=4,
                    help="with_output: steps timed with the results streamed to host memory (0=off)")
    ap.add_argument("--configs", type=int, default=1, help="also time BASELINE configs #1-#3 (1 GPU runs)")
    ap.add_argument("--mode", choices=("msg", "peer"), default="msg",
                    help="msg: message-sharded ranks (default); peer: peer-partitioned ranks")
    ap.add_argument("--parts", type=int, default=1,
                    help="--mode peer on one process: this many loop-back parts (1 = an RCCL rank of one)")
    ap.add_argument("--also-peers", type=int, default=100_000,
                    help="second graph size reported beside the headline (metric names 100k & 1M; 0=off)")
    ap.add_argument("--gossip-check", type=int, default=64,
                    help="messages of the 1M-peer gossip-on vs eager-only delivery comparison (0=off)")
    ap.add_argument("--config-traffic-json", default=os.path.join(ROOT, "profiles", "config_traffic_latest.json"),
                    help="per-config HBM bytes from rocprofv3 --pmc passes (scripts/config_pmc.sh + config_traffic.py)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of the relax kernel from a rocprofv3 --pmc pass")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, cmd=None, env=None, out=None):
    """`bench.py --gpus N` started without torchrun (no WORLD_SIZE): start N
    rank processes of this script with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set (rendezvous on 127.0.0.1), one per GPU. This
    process makes no GPU call (gossipsim is loaded lazily; nothing here touches
    HIP), so the ranks own their devices. Rank 0's stdout is collected and its
    JSON line relayed to `out`; the other ranks' stdout goes to stderr. If a
    rank fails, the others are terminated and its exit code is returned (a CPU
    box fails here, for want of a device, instead of timing one rank).
    `cmd` replaces the worker command (tests use a stub)."""
    out = out or sys.stdout
    cmd = cmd or [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      text=True))
    lines = []
    drain = threading.Thread(target=lambda: lines.extend(procs[0].stdout), daemon=True)
    drain.start()
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code
                print("bench.py: rank %d of %d exited with status %d; stopping the others" % (r, n, code),
                      file=sys.stderr, flush=True)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    drain.join(timeout=10)
    js = [ln for ln in lines if ln.lstrip().startswith("{")]
    for ln in lines:
        if ln not in js:
            sys.stderr.write(ln)
    if rc == 0 and not js:
        print("bench.py: rank 0 printed no result line", file=sys.stderr, flush=True)
        rc = 1
    if rc == 0:
        out.write(js[-1] if js[-1].endswith("\n") else js[-1] + "\n")
        out.flush()
    return rc


DIST = {}  # the torch.distributed backend of this run (dist_setup)


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch = dist = None
    try:
        import torch
        import torch.distributed as dist
    except ImportError:
        pass
    if world > 1:
        # one GPU per rank over RCCL; ranks sharing a GPU (a rehearsal of the
        # N-rank path on a box with fewer GPUs: RCCL refuses two ranks on one
        # device) reduce their few timing / counter scalars over gloo instead
        # (message sharding has no data-path collective either way)
        ndev = torch.cuda.device_count() if torch is not None else 0
        shared = ndev > 0 and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world))
        backend = os.environ.get("GS_BENCH_BACKEND") or ("nccl" if ndev and not shared else "gloo")
        if ndev:
            local = local % ndev
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
        DIST.update(backend=backend, ranks=world, ranks_share_gpus=bool(shared))
    return world, rank, local, torch, dist


def allreduce(torch, dist, world, vals, op):
    if world == 1:
        return vals
    dev = "cuda" if DIST.get("backend") == "nccl" else "cpu"
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return t.tolist()


def barrier_sync(torch, dist, world):
    if world > 1:
        dist.barrier()
    if torch is not None and torch.cuda.is_available():
        torch.cuda.synchronize()


def _pinned(core_set):
    """Context: this process pinned to `core_set` (restored afterwards)."""
    class _Pin:
        def __enter__(self):
            self.old = os.sched_getaffinity(0)
            os.sched_setaffinity(0, core_set)

        def __exit__(self, *a):
            os.sched_setaffinity(0, self.old)
    return _Pin()


def cpu_baseline(sim, args, S, links, budget_s):
    """The CPU oracle on the same graph + mesh, a bounded message sample
    (SURVEY §8d). The quoted value is like for like: the oracle's eager
    forwarding (lazy gossip off) single-threaded, pinned to one core — the
    GPU's timed batches compute exactly that and prove every IHAVE a no-op,
    so the same sample is re-checked bit-exact against the GPU's gossip-on
    run. Beside it: the same eager oracle message-parallel (OpenMP) on the
    host cores this process may use (capped at 16, the box's CPU share per
    GPU) and, with --cpu-gossip, the oracle with lazy gossip on (it simulates
    every IHAVE event: ~20 s per message at 1M peers)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / baseline only
    N = args.peers
    row, col, _ = sim.csr()
    mesh, cnt = sim.mesh()
    lat, bw = oracle.topogen_links(S, *links)
    stage = (np.arange(N) % S).astype(np.uint8)
    kw = {n: getattr(sim.cfg.c, n) for n, _ in oracle.OrParams._fields_}
    p = oracle.OrParams(**kw)
    t, pub, size = gossipsim.shard_messages(10_000, 0, 1, 256, N, args.msg_size)
    cores = sorted(os.sched_getaffinity(0))

    def timed(params, k_max, threads=0, budget=budget_s):
        deliv, elapsed, k, tcs, hps = 0, 0.0, 0, [], []
        step = max(1, threads)
        while k + step <= k_max and (elapsed < budget or k == 0):
            t0 = time.perf_counter()
            tc, hp, st = oracle.run(params, row, col, mesh, cnt, stage, lat, bw, bw, t[k:k + step], pub[k:k + step],
                                    size[k:k + step], threads=threads)
            elapsed += time.perf_counter() - t0
            deliv += st["deliveries"]
            tcs.append(tc)
            hps.append(hp)
            k += step
        return deliv / elapsed, k, elapsed, np.concatenate(tcs), np.concatenate(hps)

    pe = oracle.OrParams(**dict(kw, lazy_gossip=0))
    with _pinned({cores[0]}):
        ve, ke, ee, tcs, hps = timed(pe, 256)
        gossip_1core = None
        if args.cpu_gossip:
            vg, kg, eg, _, _ = timed(p, 64, budget=budget_s / 2)
            gossip_1core = {"value": vg, "sample": "lazy_gossip=1 (every IHAVE simulated), %d messages, %.1f s"
                            % (kg, eg)}
    nthr = min(16, len(cores))
    vm, km, em, _, _ = timed(pe, 1024, threads=nthr, budget=budget_s / 2)
    # parity of the single-core sample against the GPU's gossip-on run (outside every timed region)
    res = sim.run((t[:ke], pub[:ke], size[:ke]), collect=True)
    same = bool((res["t_complete"] == tcs).all() and (res["hops"] == hps).all())
    return {"value": ve, "unit": "deliveries/s", "cores": 1, "kind": "port",
            "sample": "oracle/gs_oracle.c or_run (binary-heap event simulation), eager forwarding (lazy gossip "
                      "off: the GPU proves every IHAVE of these batches a no-op), %d messages on the same %d-peer "
                      "graph+mesh, %.1f s, pinned to core %d" % (ke, N, ee, cores[0]),
            "all_cores": {"value": vm, "cores": nthr, "host_cpus_allowed": len(cores), "nproc": os.cpu_count(),
                          "sample": "or_run_mt (OpenMP, message-parallel), eager, %d messages, %.1f s" % (km, em)},
            "gossip_on_1core": gossip_1core if gossip_1core else "skipped (--cpu-gossip): the oracle simulates "
                               "every IHAVE event, ~20 s per 1M-peer message",
            "shadow": "not measured (no Shadow installation on the GPU box)",
            "parity_with_gpu_on_sample": same}


def gossip_check(args, S, links, local, msgs=64):
    """Does lazy gossip (on in rust-test-node, main.rs:230,235) change any
    delivery of the headline workload? Default phase (publish 3 ms after a
    heartbeat): the library's per-batch no-op proof. Heartbeats 370 ms after
    the publish (mid-dissemination): gossip on the push path vs eager-only on
    the pull path, on the same graph and mesh, counting the (peer, message)
    completions that differ."""
    out = {"default_phase": "publish 3 ms after a heartbeat (gossipsim.T0_NS): proven no-op per batch"}
    phase = (gossipsim.T0_NS + 370_000_000) % 1_000_000_000
    sched = gossipsim.shard_messages(0, 0, 1, msgs, args.peers, args.msg_size)
    res = {}
    for name, kw in (("gossip", dict(lazy_gossip=1, hb_phase_ns=phase)), ("eager", dict(lazy_gossip=0))):
        sim = gossipsim.Simulator(peers=args.peers, batch=msgs, fragments=args.fragments, seed=args.seed,
                                  device=local, **kw)
        sim.set_topogen_links(S, *links)
        sim.connect_gossipsub_peers()
        sim.mesh_converge(args.max_heartbeats)
        t0 = time.perf_counter()
        r = sim.run(sched, collect=True)
        r["s"] = time.perf_counter() - t0
        r["stats"] = sim.stats()
        res[name] = r
        sim.close()
    g, e = res["gossip"], res["eager"]
    diff = g["t_complete"] != e["t_complete"]
    earlier = g["t_complete"] < e["t_complete"]
    out["heartbeat_370ms"] = {
        "msgs": msgs, "peers": args.peers, "completions_differ": int(diff.sum()),
        "completions_earlier_via_iwant": int(earlier.sum()),
        "hops_differ": int((g["hops"] != e["hops"]).sum()),
        "gossip_iwant": int(g["stats"]["gossip_iwant"]), "fallback_batches": int(g["stats"]["gossip_fallback_batches"]),
        "max_latency_ms_gossip": int(g["stats"]["latency_max_ms"]), "max_latency_ms_eager": int(e["stats"]["latency_max_ms"]),
        "run_s_gossip_push": g["s"], "run_s_eager_pull": e["s"]}
    return out


def with_output(args, sim, rank, world):
    """The headline steps again with the reference's product leaving the
    device: the latency each peer logs for each message (main.rs:91-93, the
    value of its arrival-log line), streamed to host memory as u16 ms in
    message-major blocks of 64 messages (gs_result_sink.on_lat,
    GS_WANT_LAT_MS), timed like the headline."""
    blocks = [0]

    def on_lat(first, lat):
        blocks[0] += 1

    def steps(first, n):  # n batches' messages as one run (the batches' results stream beside the next passes)
        sh = [gossipsim.shard_messages(first + i, rank, world, args.batch, args.peers, args.msg_size) for i in range(n)]
        return tuple(np.concatenate([x[k] for x in sh]) for k in range(3))

    sim.run(steps(0, 2), on_lat=on_lat, block_msgs=64)  # warm-up: both pinned staging halves, transposes
    sim.reset_stats()
    blocks[0] = 0
    t0 = time.perf_counter()
    sim.run(steps(args.warmup, args.output_steps), on_lat=on_lat, block_msgs=64)
    dt = time.perf_counter() - t0
    st = sim.stats()
    return {"value": st["deliveries"] / dt, "unit": "deliveries/s", "steps": args.output_steps,
            "ms_per_step": dt * 1e3 / args.output_steps, "blocks": blocks[0],
            "bytes_to_host_per_step": args.batch * args.peers * 2,
            "sink": "on_lat: the logged latency (u16 ms, main.rs:93's value) of every (peer, message), 64-message "
                    "blocks; the steps as one gs_run of %d batches: completion from the final logs, device transpose, "
                    "each batch's D2H on a copy stream beside the next batch's passes" % args.output_steps}


def make_sim(args, peers, S, links, local):
    sim = gossipsim.Simulator(peers=peers, batch=args.batch, fragments=args.fragments,
                              seed=args.seed, device=local)
    t_setup = time.perf_counter()
    sim.set_topogen_links(S, *links)
    sim.connect_gossipsub_peers()
    epochs = sim.mesh_converge(args.max_heartbeats)
    sim._bench_links = (S, links)
    return sim, epochs, time.perf_counter() - t_setup


def measure(args, sim, peers, world, rank, torch, dist):
    """W untimed + K timed steps between barrier+synchronize; -> (max elapsed, stats, sums)."""
    sims = [sim]
    if args.mode == "peer":
        # gs_run_partitioned (C ABI): RCCL across ranks (rank 0's unique id
        # broadcast over torch.distributed), or loop-back parts in this process
        if world > 1 or args.parts == 1:
            uid = gossipsim.Comm.get_id() if rank == 0 else None
            if world > 1:
                box = [uid]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
            comm = gossipsim.Comm(nranks=world, rank=rank, uid=uid, device=sim.cfg.c.device)
        else:
            comm = gossipsim.Comm(local_parts=args.parts)
            sims += [make_sim(args, peers, *sim._bench_links, sim.cfg.c.device)[0] for _ in range(args.parts - 1)]
        sim._bench_comm = comm

        def step(i):  # every rank works on the same batch, each over its own peers
            comm.run_partitioned(sims, gossipsim.shard_messages(i, 0, 1, args.batch, peers, args.msg_size),
                                 collect=False)
    else:
        def step(i):
            sim.run(gossipsim.shard_messages(i, rank, world, args.batch, peers, args.msg_size),
                    collect=False)

    for i in range(args.warmup):
        step(i)
    for x in sims:
        x.reset_stats()
        x.set_timing(True)
    barrier_sync(torch, dist, world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    barrier_sync(torch, dist, world)
    elapsed = time.perf_counter() - t0
    st = sim.stats()
    if len(sims) > 1:  # loop-back parts: the job's counters are the parts' sum
        for x in sims[1:]:
            sx = x.stats()
            for k in ("deliveries", "frag_deliveries", "relaxations", "bytes_alg", "relax_bytes_alg", "relax_ms",
                      "scan_ms", "frontier_ms", "relax_launches"):
                st[k] += sx[k]
    for x in sims:
        x.set_timing(False)
    SUM = dist.ReduceOp.SUM if dist is not None else None
    MAX = dist.ReduceOp.MAX if dist is not None else None
    (max_elapsed,) = allreduce(torch, dist, world, [elapsed], MAX)
    tot = allreduce(torch, dist, world, [st["deliveries"], st["frag_deliveries"], st["relaxations"],
                                         st["bytes_alg"]], SUM)
    return max_elapsed, st, tot


# BASELINE.json configs #1-#3 on one GPU, timed like the headline (inputs in HBM,
# results left on the device): each is one Simulator with that config's knobs,
# a short untimed warm-up run, then `msgs` messages timed. The peer-partitioned
# config #4 is bench.py --mode peer.
CONFIGS = {
    "c1_1k_uniform_F1": dict(peers=1000, knobs={}, links=(1, 50, 50, 50, 50), fragments=1, batch=1024, msgs=1024,
                             reps=5),
    "c2_10k_F8": dict(peers=10_000, knobs={}, links=(5, 50, 150, 40, 130), fragments=8, batch=128, msgs=1024,
                      reps=3),
    # go-test-node flavour (gs_config_preset GS_NODE_GO: IDONTWANT >= 1000 B, main.go:165; Dout 2,
    # unsigned, own message logged) at 100k peers, the IDONTWANT list pass
    "go_100k_idontwant": dict(peers=100_000, knobs=dict(node="go"), links=(5, 50, 150, 40, 130), fragments=1,
                              batch=1024, msgs=1024, reps=2),
    # the go preset gossip-active: IDONTWANT and IHAVE / IWANT in the same list pass
    "go_100k_idontwant_gossip_370ms": dict(peers=100_000, links=(5, 50, 150, 40, 130), fragments=1, batch=1024,
                                           msgs=1024, reps=2, knobs=dict(
                                               node="go", hb_phase_ns=(gossipsim.T0_NS + 370_000_000) % 1_000_000_000)),
    # the headline graph with heartbeats 370 ms after every publish: IWANT answers overtake eager
    # forwards (0.7 % of completions change), the gossip runs inside the list pass
    "c4_1m_gossip_370ms": dict(peers=1_000_000, links=(5, 50, 150, 40, 130), fragments=1, batch=1024, msgs=1024,
                               reps=2, knobs=dict(hb_phase_ns=(gossipsim.T0_NS + 370_000_000) % 1_000_000_000)),
    # config #2's shape with heartbeats 370 ms after every publish: fragment rows with IHAVE/IWANT
    # inside the list pass (every fragment gossiped on its own)
    "c2_10k_F8_gossip_370ms": dict(peers=10_000, links=(5, 50, 150, 40, 130), fragments=8, batch=128, msgs=1024,
                                   reps=3, knobs=dict(hb_phase_ns=(gossipsim.T0_NS + 370_000_000) % 1_000_000_000)),
    "c3_100k_gossip_churn": dict(
        peers=100_000, links=(5, 50, 150, 40, 130), fragments=1, batch=1024, msgs=1024,
        knobs=dict(lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                   heartbeat_ns=1_000_000_000, hb_phase_ns=gossipsim.T0_NS - 20 * 1_000_000_000 + 370_000_000)),
    # config #3 over a longer schedule: 4096 publishes one per heartbeat = 4 batches of 1024, each
    # batch's epoch chain on XCD 0 beside the previous batch's passes; the
    # warm-up run covers the same number of epochs, so the timed run continues the chain
    "c3_100k_gossip_churn_4096": dict(
        peers=100_000, links=(5, 50, 150, 40, 130), fragments=1, batch=1024, msgs=4096, warm_msgs=4096,
        knobs=dict(lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                   heartbeat_ns=1_000_000_000, hb_phase_ns=gossipsim.T0_NS - 20 * 1_000_000_000 + 370_000_000)),
    # run.sh's free message_delay (run.sh:36) at 1500 ms under config #3: two offsets into the
    # heartbeat, each group of messages regrouped into one lockstep churn list-pass batch per
    # offset class
    "c3_100k_delay1500ms": dict(
        peers=100_000, links=(5, 50, 150, 40, 130), fragments=1, batch=1024, msgs=1024, delay_ns=1_500_000_000,
        knobs=dict(lazy_gossip=1, churn_ppm=10_000, churn_down=10, churn_horizon=16,
                   heartbeat_ns=1_000_000_000, hb_phase_ns=gossipsim.T0_NS - 20 * 1_000_000_000 + 370_000_000)),
}


def config_sched(step, msgs, peers, msg_size, delay_ns=None):
    """shard_messages(step, 0, 1, msgs, ...) with another publish spacing (run.sh's message_delay)"""
    t, pub, size = gossipsim.shard_messages(step, 0, 1, msgs, peers, msg_size)
    if delay_ns:
        idx = np.uint64(step) * np.uint64(msgs) + np.arange(msgs, dtype=np.uint64)
        t = np.uint64(gossipsim.T0_NS) + idx * np.uint64(delay_ns)
    return t, pub, size


def config_traffic(args):
    """{config: PMC entry} of --config-traffic-json (empty when absent or unreadable)"""
    try:
        return json.load(open(args.config_traffic_json)).get("configs", {})
    except (OSError, ValueError, AttributeError):
        return {}


def config_rates(args, local):
    out = {}
    ctraffic = config_traffic(args)
    mark = os.environ.get("GS_CFG_MARK") == "1"
    for name, c in CONFIGS.items():
        sim = gossipsim.Simulator(peers=c["peers"], batch=c["batch"], fragments=c["fragments"], seed=args.seed,
                                  device=local, **c["knobs"])
        sim.set_topogen_links(c["links"][0], *c["links"][1:])
        sim.connect_gossipsub_peers()
        sim.mesh_converge(args.max_heartbeats)
        sim.run(config_sched(0, c.get("warm_msgs", c["batch"]), c["peers"], args.msg_size, c.get("delay_ns")),
                collect=False)
        # repeats: the best of `reps` runs (config #1 runs ~1 ms, where one host hiccup doubles it);
        # every repeat simulates the same messages, so the counters are one run's
        dt = None
        for _ in range(c.get("reps", 1)):
            sim.reset_stats()
            sched = config_sched(1, c["msgs"], c["peers"], args.msg_size, c.get("delay_ns"))  # after the warm-up's
            t0, m0 = time.perf_counter(), time.monotonic_ns()
            sim.run(sched, collect=False)
            d = time.perf_counter() - t0
            if mark and dt is None:  # the first timed run's clock span (scripts/config_traffic.py)
                print(json.dumps({"mark": name, "t0_ns": m0, "t1_ns": time.monotonic_ns()}), file=sys.stderr)
            dt = d if dt is None else min(dt, d)
        st = sim.stats()
        # one more repeat with HIP events around every window pass / bucket: the
        # config's roofline on SURVEY 8(d)'s algorithmic bytes (kernel time only)
        sim.reset_stats()
        sim.set_timing(True)
        sim.run(sched, collect=False)
        sim.set_timing(False)
        tst = sim.stats()
        roof = None
        if tst["relax_ms"] > 0 and tst["relax_launches"]:
            ach = tst["relax_bytes_alg"] / (tst["relax_ms"] / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0,
                    "alg_bytes_per_launch": tst["relax_bytes_alg"] / tst["relax_launches"],
                    "avg_launch_us": tst["relax_ms"] * 1e3 / tst["relax_launches"],
                    "launches": int(tst["relax_launches"]), "pass_ms": tst["relax_ms"]}
        push = st["list_pull_batches"] < st["batches"] and (
            (st["gossip_fallback_batches"] and not st["gossip_list_batches"]) or
            (st["list_pull_batches"] == 0 and (sim.cfg.c.idontwant or c["knobs"].get("churn_ppm"))))
        out[name] = {"value": st["deliveries"] / dt, "unit": "deliveries/s", "msgs": c["msgs"], "best_of": c.get("reps", 1),
                     "ms": dt * 1e3, "deliveries": int(st["deliveries"]), "batches": int(st["batches"]),
                     "alg_bytes_per_batch": st["bytes_alg"] / max(1, st["batches"]),
                     "gossip_iwant": int(st["gossip_iwant"]), "gossip_noop_msgs": int(st["gossip_noop_msgs"]),
                     "gossip_list_batches": int(st["gossip_list_batches"]),
                     "gossip_fallback_batches": int(st["gossip_fallback_batches"]),
                     "list_pull_batches": int(st["list_pull_batches"]),
                     "kernel_path": "push (k_scan+k_frontier+k_gossip)" if push else
                     "pull (k_lpull churn: per-epoch meshes, IHAVE/IWANT inside the passes)"
                     if c["knobs"].get("churn_ppm") and st["list_pull_batches"] else
                     "pull (k_lpull, IHAVE/IWANT inside the passes)" if st["gossip_list_batches"] else
                     "pull (k_lpull)" if st["list_pull_batches"] else "pull (k_pull)",
                     "roofline": roof}
        pmc = ctraffic.get(name)
        # PMC bytes of the same window-pass kernel family as this run's path (k_lpull / k_pull)
        if roof and pmc and pmc.get("hbm_bytes_per_launch") and pmc.get("pass_kernels") and \
                all(k.split("<")[0] in out[name]["kernel_path"] for k in pmc["pass_kernels"]):
            roof["traffic"] = pmc["hbm_bytes_per_launch"]
            roof["traffic_ratio"] = pmc["hbm_bytes_per_launch"] / roof["alg_bytes_per_launch"]
            out[name]["hbm_bytes_per_batch_all_kernels"] = pmc.get("hbm_bytes_per_batch_all_kernels")
            out[name]["traffic_source"] = pmc.get("source")
        sim.close()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:  # no torchrun: be the launcher
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local, torch, dist = dist_setup()
    if args.gpus != world:  # under torchrun the launcher's WORLD_SIZE is the GPU count
        if rank == 0:
            print("bench.py: --gpus %d but WORLD_SIZE is %d: running on %d GPUs" % (args.gpus, world, world),
                  file=sys.stderr)
        args.gpus = world
    S, bl, bh, ll, lh = [int(x) for x in args.links.split(",")]
    links = (bl, bh, ll, lh)
    sim, epochs, t_setup = make_sim(args, args.peers, S, links, local)
    steps = measure(args, sim, args.peers, world, rank, torch, dist)
    max_elapsed, st, tot = steps
    deliveries = tot[0]
    extra = None
    if args.also_peers and args.also_peers != args.peers and args.mode == "msg":
        sim2, _, _ = make_sim(args, args.also_peers, S, links, local)
        e2, _, tot2 = measure(args, sim2, args.also_peers, world, rank, torch, dist)
        extra = {"peers": args.also_peers, "value": tot2[0] / e2, "ms_per_step": e2 * 1e3 / args.steps}
        sim2.close()

    # one launch = one Delta-window pass: k_lpull / k_pull (owner-computes paths, their
    # whole time is reported as frontier time) or k_scan + k_frontier (push path);
    # --mode peer: one bucket of the partitioned protocol (gs_comm.hip), timed by
    # HIP events around its scan and its export + exchange + relaxation
    launches = max(1, st["relax_launches"])
    fpl = fp_lanes(args.fragments)
    if args.mode == "peer" and st.get("list_pull_batches", 0) > 0:
        kernel = "k_lpull<%d> over each part's rows (partitioned list pass; records exchanged between " \
                 "passes, not timed here)" % fpl
    elif args.mode == "peer":
        kernel = "k_scan<%d,false,false> + k_pexport_dest<%d> + record exchange + k_precv<%d> " \
                 "(partitioned push path)" % (fpl, fpl, fpl)
    else:
        pull = st["relax_ms"] > 0 and st["scan_ms"] <= 0.01 * st["relax_ms"]
        lpull = pull and st.get("list_pull_batches", 0) > 0
        ch = 8 if args.batch * fpl <= 512 else 16  # 64-lane chunks per row (gs_lpull_kernel.h lpull_chunks)
        kernel = ("k_lpull<%d, %d>" % (fpl, ch)) if lpull else ("k_pull<%d>" % fpl) if pull else \
            "k_scan<%d,false,false> + k_frontier<%d,true,false>" % (fpl, fpl)
    achieved = st["relax_bytes_alg"] / (st["relax_ms"] / 1e3) / 1e9 if st["relax_ms"] > 0 else None
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            # PMC bytes only for the very kernel this line names (one kernel, same template)
            def targs(k):  # "k_lpull<1, 16u, false, false>" -> ("k_lpull", ["1", "16"])
                name, _, rest = k.partition("<")
                return name, [x.strip().rstrip("u") for x in rest.rstrip(">").split(",")]
            # the template id, without a descriptive suffix ("k_lpull<1> over each part's rows ...")
            kid = kernel[:kernel.find(">") + 1] if "<" in kernel else kernel.split(" ")[0]
            kn, ka = targs(kid if " + " not in kernel else "")
            same_kernel = bool(tj.get("kernels")) and " + " not in kernel and args.mode == tj.get("mode", "msg") \
                and all(targs(k)[0] == kn and targs(k)[1][:len(ka)] == ka for k in tj["kernels"])
            if tj.get("peers") == args.peers and tj.get("batch") == args.batch and same_kernel:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
            "kernel": "Delta-window relaxation = " + kernel,
            "alg_bytes_per_launch": st["relax_bytes_alg"] / launches,
            "avg_launch_us": st["relax_ms"] * 1e3 / launches,
            "avg_scan_us": st["scan_ms"] * 1e3 / launches,
            "avg_frontier_us": st["frontier_ms"] * 1e3 / launches,
            "launches": st["relax_launches"],
            "timing": "HIP events on the library stream around every window pass",
            "pushes_per_relaxation": st["pushes"] / max(1, st["relaxations"])}

    wout = None
    if args.output_steps and args.mode == "msg":
        wout = with_output(args, sim, rank, world)
        (wdt,) = allreduce(torch, dist, world, [wout["ms_per_step"]], dist.ReduceOp.MAX if dist else None)
        wout["value"] = wout["value"] * world * wout["ms_per_step"] / wdt  # job rate at the slowest rank
        wout["ms_per_step"] = wdt

    cfg_rates = None
    if world == 1 and args.configs and args.mode == "msg":
        cfg_rates = config_rates(args, local)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and args.mode == "msg":
        cpu = cpu_baseline(sim, args, S, links, args.cpu_seconds)
    gcheck = None
    if rank == 0 and world == 1 and args.gossip_check and args.mode == "msg":
        gcheck = gossip_check(args, S, links, local, args.gossip_check)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": deliveries / max_elapsed,
            "unit": "deliveries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "msg" else "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (random-ID dial graph + subscription/heartbeat-converged mesh, run.sh publish "
                    "schedule, rust preset incl. lazy gossip)",
            "config": {
                "workload": "%d peers, %d-stage topogen links (%d-%d Mbit, %d-%d ms), CONNECTTO=10, "
                            "D=6/4/8, F=%d, %d B msgs, %d msgs/step%s"
                            % (args.peers, S, bl, bh, ll, lh, args.fragments, args.msg_size, args.batch,
                               "/GPU, message-sharded" if args.mode == "msg" else ", peer-partitioned"),
                "peers": args.peers, "batch": args.batch, "fragments": args.fragments,
                "msg_size": args.msg_size, "links": args.links,
                "parallelism": "msg-shard%d" % world if args.mode == "msg" else
                ("peer-part%d (RCCL ranks)" % world if world > 1 or args.parts == 1 else
                 "peer-part%d (loop-back parts on one GPU)" % args.parts),
                "exchange": None if args.mode == "msg" else exchange_label(world, args.parts),
            },
            "deliveries": int(deliveries),
            "frag_deliveries": int(tot[1]),
            "relaxations": int(tot[2]),
            "bytes_alg": int(tot[3]),
            "dist": DIST or None,
            "setup_s": t_setup,
            "mesh_epochs": epochs,
            "buckets_per_step": st["buckets"] / max(1, args.steps),
            # verbose entries first: the driver keeps the last ~2000 characters of the
            # line, so the headline's companions (roofline, the 100k rate, the streamed
            # rate and every config's rate) come last
            "configs_1gpu": cfg_rates,
            "gossip": {"lazy_gossip": int(sim.cfg.c.lazy_gossip), "noop_msgs": int(st["gossip_noop_msgs"]),
                       "fallback_batches": int(st["gossip_fallback_batches"]), "iwant": int(st["gossip_iwant"]),
                       "check": gcheck},
            "cpu_baseline": cpu,
            "roofline": roof,
            "at_%dk_peers" % (args.also_peers // 1000) if extra else "at_second_size": extra,
            "with_output": wout,
            "configs_1gpu_rates": {k: {"value": v.get("value"), "ms": v.get("ms"),
                                       "frac": (v.get("roofline") or {}).get("frac"),
                                       "traffic_x": (v["hbm_bytes_per_batch_all_kernels"] / v["alg_bytes_per_batch"]
                                                     if v.get("hbm_bytes_per_batch_all_kernels")
                                                     and v.get("alg_bytes_per_batch") else None)}
                                   if isinstance(v, dict) else v
                                   for k, v in cfg_rates.items()} if isinstance(cfg_rates, dict) else None,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
