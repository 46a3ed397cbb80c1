"""Peer-partitioned dissemination driver.

The reference runs one OS process per peer inside Shadow (shadow/run.sh) and
the network between them is the exchange. Here partition p of P owns the key
rows of a contiguous peer range; every Delta-bucket runs in the HIP library as
a scan (own arrivals -> 24-B records) and a relax (gathered records -> pushes
into own peers), see include/gossipsim.h gs_part_*. This module only moves
records between partitions and reduces the next bucket key:

  * LoopbackExchange  P contexts in one process (tests, one GPU)
  * DistExchange      one partition per rank over a torch.distributed group:
                      RCCL (backend "nccl") on GPUs, gloo on CPUs

Records stay on the device: the library writes them into torch tensors by
pointer and reads the gathered tensor by pointer.
"""
import torch
import torch.distributed as dist

import gossipsim

REC_WORDS = 3  # gs_part_record = {u64 key, u64 start, u32 peer, u32 slot} = 3 x int64
KEY_NONE = gossipsim.KEY_NONE
_BIAS = 1 << 63


def key_to_i64(k):
    """Order-preserving u64 -> int64 (collectives reduce signed int64)."""
    return int(k) - _BIAS


def i64_to_key(s):
    return int(s) + _BIAS


class RecordBuffer:
    """Device buffer for one partition's bucket records; grows on GS_ERANGE."""

    def __init__(self, device, capacity=1 << 16):
        self.device = device
        self.t = torch.empty((capacity, REC_WORDS), dtype=torch.int64, device=device)

    def ensure(self, n):
        if n > self.t.shape[0]:
            self.t = torch.empty((max(n, 2 * self.t.shape[0]), REC_WORDS), dtype=torch.int64,
                                 device=self.device)

    def scan(self, sim, key):
        """gs_part_scan into this buffer -> (records [n, 3] view, scan's next pending key)."""
        ok, n, m1 = sim.part_scan(key, self.t.data_ptr(), self.t.shape[0])
        if not ok:  # state unchanged: grow and scan again
            self.ensure(n)
            ok, n, m1 = sim.part_scan(key, self.t.data_ptr(), self.t.shape[0])
            assert ok
        return self.t[:n], m1


class LoopbackExchange:
    """All partitions live in this process: the gather is a concatenation."""

    def gather(self, recs):
        return recs[0] if len(recs) == 1 else torch.cat(recs)

    def min_key(self, keys):
        return min(keys)


class DistExchange:
    """One partition per rank. Per bucket: all_gather of the record counts,
    all_gather of the (padded) records, all_reduce(MIN) of the next key."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cpu")

    def gather(self, recs):
        (r,) = recs
        n = torch.tensor([r.shape[0]], dtype=torch.int64, device=self.device)
        counts = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(counts, n, group=self.group)
        counts = [int(c.item()) for c in counts]
        mx = max(counts)
        if mx == 0:
            return r[:0]
        pad = torch.zeros((mx, REC_WORDS), dtype=torch.int64, device=self.device)
        pad[:r.shape[0]] = r
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(outs, pad, group=self.group)
        return torch.cat([o[:c] for o, c in zip(outs, counts)])

    def min_key(self, keys):
        (k,) = keys
        t = torch.tensor([key_to_i64(k)], dtype=torch.int64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return i64_to_key(t.item())


def _sync(device):
    if isinstance(device, torch.device) and device.type == "cuda":
        torch.cuda.synchronize(device)


def run_partitioned(sims, schedule, exchange, bufs=None, collect=True):
    """Drive one batch through the bucket protocol of include/gossipsim.h.

    `sims` are this process's partitions (Simulator with set_partition done).
    Returns (per-partition results, info) where results[i]["t_complete"] is
    [messages, own peers] and info counts buckets and exchanged records."""
    if bufs is None:
        dev = torch.device("cuda", sims[0].cfg.c.device) if torch.cuda.is_available() else torch.device("cpu")
        bufs = [RecordBuffer(dev) for _ in sims]
    k = exchange.min_key([s.part_begin(schedule) for s in sims])
    buckets = records = 0
    while k != KEY_NONE:
        scanned = [b.scan(s, k) for s, b in zip(sims, bufs)]
        allrec = exchange.gather([r for r, _ in scanned])
        _sync(allrec.device)  # the library reads the gathered records on its own stream
        m2 = [s.part_relax(k, allrec.data_ptr(), allrec.shape[0]) for s in sims]
        k = exchange.min_key([min(m1, x) for (_, m1), x in zip(scanned, m2)])
        buckets += 1
        records += int(allrec.shape[0])
    res = [s.part_finish(collect) for s in sims]
    return res, {"buckets": buckets, "records": records}
