// gs_part.h — peer-partitioned dissemination.
// Included by gs_relax.hip inside namespace gs (after the batch helpers).
//
// Partition `part` of P owns the keys rows of peers [u0, u0 + un); the CSR and
// the mesh are replicated (every partition builds them identically from the
// same seed). A Delta-bucket is split at the one place where data crosses
// partitions — the mesh edge u -> w with u and w owned by different parts:
//
//   scan    (owner of u)  k_scan (shared with gs_run) streams the own keys,
//                         compacts the bucket's arrivals and writes the final
//                         bitset; k_pexport folds each arrival's uplink FIFO
//                         (busy is owner-local: the FIFO is u's own uplink)
//                         and emits one 24-B record {key, start, u, slot} per
//                         arrival with at least one forward target.
//   exchange (caller)     all-gather of every part's records (RCCL / loopback).
//   relax   (owner of w)  k_precv re-walks u's mesh row from the record (same
//                         target order and position counter as relax_lane, so
//                         arrival = start + pos*ser + lat + max(0, dn - ser)),
//                         pushing only into own targets, with the same final
//                         bitset + read filter as the single-device frontier.
//
// The next bucket is min over parts of (scan's next pending key, relax's min
// pushed key): exactly the single-device ctrl word. Results are bit-identical
// to gs_run; the exchange volume per bucket is 24 B x (arrivals with targets).

namespace {

__global__ void k_pbucket(uint64_t* ctrl, uint64_t* pcnt, uint64_t key) {
  if (threadIdx.x == 0) {
    ctrl[0] = key;      // the bucket k_scan reads (launch 0)
    ctrl[1] = INF64;    // k_scan's next pending key
    ctrl[2] = INF64;
    pcnt[0] = 0;        // frontier groups
    pcnt[1] = 0;        // records emitted
  }
}

__global__ __launch_bounds__(TB) void k_pcount(const uint32_t* __restrict__ fr_cnt, uint32_t nwaves,
                                                uint64_t* pcnt) {
  uint64_t s = 0;
  for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < nwaves; i += gridDim.x * TB) s += fr_cnt[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd((unsigned long long*)&pcnt[0], (unsigned long long)s);
}

// Owner side of a bucket: the frontier segments written by k_scan -> records.
template <int FP>
__global__ __launch_bounds__(TB) void k_pexport(RelaxArgs a, gs_part_record* __restrict__ rec, uint64_t cap,
                                                uint64_t* pcnt) {
  __shared__ BucketLds L;
  load_tables(L, a);
  __syncthreads();
  const uint64_t cur = a.ctrl[0];
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t n = __builtin_amdgcn_readfirstlane(a.fr_cnt[wave]);
  const size_t seg = (size_t)wave * a.seg_cap;
  constexpr uint32_t GPW = 64 / FP;
  const uint64_t smask = (1ull << a.sb) - 1;
  uint64_t fd = 0, nr = 0;
  uint32_t err = 0;
  for (uint32_t base = 0; base < n; base += GPW) {
    const uint32_t gi = base + (uint32_t)lane / FP;
    const bool valid = gi < n;
    uint64_t gid, key;
    if constexpr (FP == 1) {
      gid = valid ? a.fr_idx[seg + gi] : 0;
      key = valid ? a.fr_key[seg + gi] : INF64;
    } else {
      gid = valid ? (uint64_t)a.fr_idx[seg + gi] * FP + (lane & (FP - 1)) : 0;
      key = valid ? a.keys[gid] : INF64;
    }
    const uint64_t t = key >> a.tshift;
    const uint32_t u = (uint32_t)(gid / LL);
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t ug = u + a.u0;
    const uint32_t pm = valid ? a.pub[slot / FP] : EMPTY;
    const bool active = valid && key != INF64 && t >= lo && t < hi && ug != pm;
    const uint32_t src = (uint32_t)(key & smask);
    uint32_t cnt = 0;
    if (active) {
      uint32_t row[MESH_W];
      load_mesh_row(a.mesh, ug, row);
#pragma unroll
      for (int j = 0; j < (int)MESH_W; j++) {
        const uint32_t w = row[j] & 0xFFFFFFu;
        cnt += (row[j] != EMPTY && w != src && w != pm) ? 1u : 0u;
      }
    }
    const uint32_t ser = L.su[a.stage[valid ? ug : a.u0]];
    const uint64_t start = uplink_start<FP>(a.busy, (size_t)u * a.B + slot / FP, active, key, cnt, ser, a.tshift);
    if (active) {
      fd++;
      nr += cnt;
      const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
      if (cnt && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
    }
    const bool want = active && cnt != 0;
    const uint64_t wm = __ballot(want);
    if (wm == 0) continue;
    uint64_t wbase = 0;
    if (lane == 0) wbase = atomicAdd((unsigned long long*)&pcnt[1], (unsigned long long)__popcll(wm));
    wbase = uniform64(wbase);
    if (want) {
      const uint64_t pos = wbase + (uint64_t)__popcll(wm & ((1ull << lane) - 1));
      if (pos < cap) {
        gs_part_record r;
        r.key = key;
        r.start = start;
        r.peer = ug;
        r.slot = slot;
        rec[pos] = r;
      }
    }
  }
  fd = wave_sum(fd);
  nr = wave_sum(nr);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if (lane == 0) {
    if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
    if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

// Target side: every gathered record pushes into this partition's own peers.
template <int FP>
__global__ __launch_bounds__(TB) void k_precv(RelaxArgs a, const gs_part_record* __restrict__ rec, uint64_t n,
                                              uint64_t* pcnt) {
  __shared__ BucketLds L;
  load_tables(L, a);
  __syncthreads();
  const uint32_t S = a.S, LL = a.L;
  const uint64_t smask = (1ull << a.sb) - 1;
  uint64_t nmin = INF64, np = 0;
  uint32_t err = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TB) {
    const gs_part_record r = rec[i];
    const uint32_t ug = r.peer, slot = r.slot;
    const uint32_t src = (uint32_t)(r.key & smask);
    const uint32_t hp = (uint32_t)((r.key >> a.sb) & ((1u << HOP_BITS) - 1));
    const uint32_t pm = a.pub[slot / FP];
    const uint32_t su = a.stage[ug];
    const uint32_t ser = L.su[su];
    const uint64_t hbits = ((uint64_t)(hp + 1) << a.sb) | ug;
    uint32_t row[MESH_W];
    load_mesh_row(a.mesh, ug, row);
    uint32_t pos = 0;
#pragma unroll
    for (int j = 0; j < (int)MESH_W; j++) {
      const uint32_t e = row[j];
      const uint32_t w = e & 0xFFFFFFu;
      if (e == EMPTY || w == src || w == pm) continue;
      pos++;
      if (w - a.u0 >= a.N) continue;  // another partition's peer
      const size_t dst = (size_t)(w - a.u0) * LL + slot;
      if ((a.fbits[dst >> 6] >> (dst & 63)) & 1) continue;  // final: cannot improve
      const uint32_t sw = e >> STAGE_SHIFT, sd = L.sd[sw];
      const uint64_t arr = r.start + (uint64_t)pos * ser + L.lat[su * S + sw] + (sd > ser ? sd - ser : 0);
      if (arr > a.tmax) err |= ERR_TIME;
      const uint64_t nk = (arr << a.tshift) | hbits;
      if (!(nk < a.keys[dst])) continue;
      atomicMin((unsigned long long*)&a.keys[dst], (unsigned long long)nk);
      np++;
      nmin = nk < nmin ? nk : nmin;
    }
  }
  nmin = wave_min(nmin);
  np = wave_sum(np);
  for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
  if ((threadIdx.x & 63) == 0) {
    if (nmin != INF64) atomicMin((unsigned long long*)&pcnt[2], (unsigned long long)nmin);
    if (np) atomicAdd((unsigned long long*)&a.counters[C_PUSH], (unsigned long long)np);
    if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
  }
}

// Owner of peer w among `parts` equal ranges [p*N/parts, (p+1)*N/parts).
__device__ __forceinline__ uint32_t part_of(uint32_t w, uint32_t N, uint32_t parts) {
  uint32_t p = (uint32_t)(((uint64_t)w * parts) / N);
  while (p + 1 < parts && (uint64_t)(p + 1) * N / parts <= w) p++;
  while (p > 0 && (uint64_t)p * N / parts > w) p--;
  return p;
}

// Routed export of a bucket's arrivals (gs_run_partitioned): a record goes
// only to the parts that own one of its forward targets (all-to-all-v instead
// of an all-gather). COUNT: records per destination part into dcnt (no state
// change); else the records themselves, destination d's at the offset
// sum(dcnt[< d]) of `rec`, with the FD / R counters and the uplink FIFO fold.
template <int FP, bool COUNT>
__global__ __launch_bounds__(TB) void k_pexport_dest(RelaxArgs a, gs_part_record* __restrict__ rec, uint64_t* dcnt,
                                                     uint64_t* dpos, uint32_t parts, uint32_t Nglob) {
  __shared__ BucketLds L;
  __shared__ uint64_t s_off[64];
  load_tables(L, a);
  if (!COUNT && threadIdx.x == 0) {
    uint64_t o = 0;
    for (uint32_t d = 0; d < parts; d++) { s_off[d] = o; o += dcnt[d]; }
  }
  __syncthreads();
  const uint64_t cur = a.ctrl[0];
  if (cur == INF64) return;  // block-uniform: no bucket left
  const uint64_t lo = ((cur >> a.tshift) / a.delta) * a.delta, hi = lo + a.delta;
  const uint32_t LL = a.L;
  const uint32_t wave = blockIdx.x * (TB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t n = __builtin_amdgcn_readfirstlane(a.fr_cnt[wave]);
  const size_t seg = (size_t)wave * a.seg_cap;
  constexpr uint32_t GPW = 64 / FP;
  const uint64_t smask = (1ull << a.sb) - 1;
  uint64_t fd = 0, nr = 0;
  uint32_t err = 0;
  for (uint32_t base = 0; base < n; base += GPW) {
    const uint32_t gi = base + (uint32_t)lane / FP;
    const bool valid = gi < n;
    uint64_t gid, key;
    if constexpr (FP == 1) {
      gid = valid ? a.fr_idx[seg + gi] : 0;
      key = valid ? a.fr_key[seg + gi] : INF64;
    } else {
      gid = valid ? (uint64_t)a.fr_idx[seg + gi] * FP + (lane & (FP - 1)) : 0;
      key = valid ? a.keys[gid] : INF64;
    }
    const uint64_t t = key >> a.tshift;
    const uint32_t u = (uint32_t)(gid / LL);
    const uint32_t slot = (uint32_t)(gid - (uint64_t)u * LL);
    const uint32_t ug = u + a.u0;
    const uint32_t pm = valid ? a.pub[slot / FP] : EMPTY;
    const bool active = valid && key != INF64 && t >= lo && t < hi && ug != pm;
    const uint32_t src = (uint32_t)(key & smask);
    uint32_t cnt = 0;
    uint64_t dmask = 0;  // destination parts of the record
    if (active) {
      uint32_t row[MESH_W];
      load_mesh_row(a.mesh, ug, row);
#pragma unroll
      for (int j = 0; j < (int)MESH_W; j++) {
        const uint32_t w = row[j] & 0xFFFFFFu;
        if (row[j] != EMPTY && w != src && w != pm) {
          cnt++;
          dmask |= 1ull << part_of(w, Nglob, parts);
        }
      }
    }
    uint64_t start = 0;
    if constexpr (!COUNT) {
      const uint32_t ser = L.su[a.stage[valid ? ug : a.u0]];
      start = uplink_start<FP>(a.busy, (size_t)u * a.B + slot / FP, active, key, cnt, ser, a.tshift);
      if (active) {
        fd++;
        nr += cnt;
        const uint32_t hp = (uint32_t)((key >> a.sb) & ((1u << HOP_BITS) - 1));
        if (cnt && hp + 1 >= (1u << HOP_BITS)) err |= ERR_HOPS;
      }
    }
    for (uint32_t d = 0; d < parts; d++) {  // wave-uniform
      const bool want = active && ((dmask >> d) & 1);
      const uint64_t wm = __ballot(want);
      if (wm == 0) continue;
      if constexpr (COUNT) {
        if (lane == 0) atomicAdd((unsigned long long*)&dcnt[d], (unsigned long long)__popcll(wm));
      } else {
        uint64_t wbase = 0;
        if (lane == 0) wbase = atomicAdd((unsigned long long*)&dpos[d], (unsigned long long)__popcll(wm));
        wbase = uniform64(wbase);
        if (want) {
          gs_part_record r;
          r.key = key;
          r.start = start;
          r.peer = ug;
          r.slot = slot;
          rec[s_off[d] + wbase + (uint64_t)__popcll(wm & ((1ull << lane) - 1))] = r;
        }
      }
    }
  }
  if constexpr (!COUNT) {
    fd = wave_sum(fd);
    nr = wave_sum(nr);
    for (int off = 32; off > 0; off >>= 1) err |= __shfl_xor(err, off);
    if (lane == 0) {
      if (fd) atomicAdd((unsigned long long*)&a.counters[C_FD], (unsigned long long)fd);
      if (nr) atomicAdd((unsigned long long*)&a.counters[C_R_FWD], (unsigned long long)nr);
      if (err) atomicOr((unsigned*)&a.counters[C_ERR], err);
    }
  }
}

// Bucket bookkeeping of the device-driven protocol: the bucket key is
// already in ctrl[0] (the MIN all-reduce wrote it); reset the rest.
__global__ void k_pbucket_dev(uint64_t* ctrl, uint64_t* pcnt, uint64_t* dcnt, uint64_t* dpos, uint32_t parts) {
  if (threadIdx.x == 0) {
    ctrl[1] = INF64;
    ctrl[2] = INF64;
    pcnt[0] = 0;
    pcnt[1] = 0;
    pcnt[2] = INF64;
  }
  if (threadIdx.x < parts) {
    dcnt[threadIdx.x] = 0;
    dpos[threadIdx.x] = 0;
  }
}

// This part's candidate for the next bucket: min(scan's next pending key,
// relax's min pushed key) into ctrl[0], ready for the MIN all-reduce.
__global__ void k_pnext(uint64_t* ctrl, const uint64_t* pcnt) {
  if (threadIdx.x == 0) ctrl[0] = ctrl[1] < pcnt[2] ? ctrl[1] : pcnt[2];
}

template <int FP>
void part_export_fp(const RelaxArgs& a, unsigned grid, hipStream_t s, gs_part_record* rec, uint64_t cap,
                    uint64_t* pcnt) {
  k_pexport<FP><<<grid, TB, 0, s>>>(a, rec, cap, pcnt);
}
template <int FP>
void part_recv_fp(const RelaxArgs& a, unsigned grid, hipStream_t s, const gs_part_record* rec, uint64_t n,
                  uint64_t* pcnt) {
  k_precv<FP><<<grid, TB, 0, s>>>(a, rec, n, pcnt);
}

RelaxArgs part_args(Ctx& c) {
  const Batch& b = c.part_b;
  RelaxArgs ra{};
  ra.keys = c.d_keys.p; ra.busy = c.d_busy.p; ra.mesh = c.d_mesh.p; ra.pub = c.d_pub.p;
  ra.fbits = c.d_fbits.p;
  ra.fr_idx = c.d_fr_idx.p; ra.fr_key = c.d_fr_key.p; ra.fr_cnt = c.d_fr_cnt.p;
  ra.stage = c.d_stage.p; ra.tables = c.d_tables.p; ra.ctrl = c.d_ctrl.p;
  ra.counters = c.d_counters.p;
  ra.total = (uint64_t)c.part_un * b.L;
  ra.delta = b.delta; ra.tmax = b.tmax; ra.seg_cap = c.part_seg_cap;
  ra.N = c.part_un; ra.B = b.B; ra.F = b.F; ra.L = b.L; ra.S = c.S; ra.sb = b.sb; ra.tshift = b.tshift;
  ra.launch = 0;
  ra.u0 = c.part_u0;
  return ra;
}

}  // namespace

void part_set(Ctx& c, uint32_t parts, uint32_t part) {
  const uint32_t N = c.cfg.peers;
  if (c.part_open) c.fail(GS_ESTATE, "a partitioned batch is in flight (gs_part_finish first)");
  if (parts < 1 || part >= parts || parts > N) c.fail(GS_EINVAL, "need 1 <= parts <= peers and part < parts");
  c.part_parts = parts;
  c.part_idx = part;
  const PartLayout lay{parts, N, 0};
  c.part_u0 = lay.u0(part);
  c.part_un = lay.un(part);
}

// The knobs a partitioned batch accepts (both protocols).
static uint32_t part_check(Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  if (c.part_un == 0) part_set(c, 1, 0);
  if (c.part_open) c.fail(GS_ESTATE, "a partitioned batch is in flight (gs_part_finish first)");
  if (n_msgs < 1 || n_msgs > c.cfg.batch) c.fail(GS_EINVAL, "partitioned batch needs 1..cfg.batch messages");
  check_schedule(c, sched, n_msgs);
  const uint32_t F = frags_of(c, sched[0]);
  for (uint64_t i = 1; i < n_msgs; i++)
    if (sched[i].msg_size != sched[0].msg_size || frags_of(c, sched[i]) != F)
      c.fail(GS_EINVAL, "partitioned batch needs equal msg_size and frags");
  if (c.cfg.churn_ppm) c.fail(GS_EUNSUPPORTED, "churn is not supported in partitioned mode");
  if (c.traffic) c.fail(GS_EUNSUPPORTED, "per-peer traffic is not supported in partitioned mode");
  if (c.cfg.idontwant && frag_payload(c.cfg.node, sched[0].msg_size, F) >= c.cfg.idontwant)
    c.fail(GS_EUNSUPPORTED, "IDONTWANT is not supported in partitioned mode");
  return F;
}

// gs_run_partitioned: a batch the peer protocols cannot take (churn's mesh per
// epoch, IDONTWANT) runs message-sharded over the replicated graph (gs_comm.hip).
bool part_needs_ms(Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  if (c.cfg.churn_ppm) return true;
  if (!c.cfg.idontwant || !n_msgs) return false;
  return frag_payload(c.cfg.node, sched[0].msg_size, frags_of(c, sched[0])) >= c.cfg.idontwant;
}

uint64_t part_begin(Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  const uint32_t F = part_check(c, sched, n_msgs);
  const uint32_t FP = pow2_at_least(F), Bmax = c.cfg.batch, un = c.part_un;
  if ((uint64_t)un * Bmax * FP >= (1ull << 32)) c.fail(GS_EUNSUPPORTED, "partition needs own peers*batch*FP < 2^32");
  hipStream_t s = c.stream;
  GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
  ensure_cus(c);
  const size_t lanes = (size_t)un * Bmax * FP, max_tiles = (lanes + 63) / 64;
  c.d_keys.alloc(lanes);
  c.d_fbits.alloc(max_tiles);
  if (FP > 1) c.d_busy.alloc((size_t)un * Bmax);
  c.d_tc.alloc((size_t)un * Bmax);
  c.d_hops.alloc((size_t)un * Bmax);
  c.d_pcnt.alloc(4);
  c.part_b = setup_batch(c, sched, 0, n_msgs);
  const Batch& b = c.part_b;
  const uint64_t total = (uint64_t)un * b.L;
  c.keys_log = false;  // dense rows from here on (gs_relax.hip list pull path leaves logs)
  GS_HIP(hipMemsetAsync(c.d_keys.p, 0xFF, total * 8, s));
  if (FP > 1) GS_HIP(hipMemsetAsync(c.d_busy.p, 0, (size_t)un * b.B * 8, s));
  GS_HIP(hipMemsetAsync(c.d_fbits.p, 0, (total + 63) / 64 * 8, s));
  GS_HIP(hipMemsetAsync(c.d_ctrl.p, 0xFF, 4 * 8, s));
  c.part_grid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>((total + TB - 1) / TB, (uint64_t)c.num_cus * split_blocks_per_cu(c)));
  const uint64_t nwaves = (uint64_t)c.part_grid * (TB / 64), ntiles = (total + 63) / 64;
  c.part_seg_cap = (uint32_t)(((ntiles + nwaves - 1) / nwaves) * (64 / FP));
  c.d_fr_idx.alloc(nwaves * c.part_seg_cap);
  if (FP == 1) c.d_fr_key.alloc(nwaves * c.part_seg_cap);
  c.d_fr_cnt.alloc(nwaves);
  launch_seed(c, b, c.part_u0, un);
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_ctrl.p, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  c.part_open = true;
  return c.h_pinned[0];
}

bool part_scan(Ctx& c, uint64_t bucket_key, gs_part_record* rec, uint64_t cap, uint64_t* n, uint64_t* m1) {
  if (!c.part_open) c.fail(GS_ESTATE, "gs_part_begin first");
  if (bucket_key == INF64) c.fail(GS_EINVAL, "bucket key is the empty marker");
  hipStream_t s = c.stream;
  const Batch& b = c.part_b;
  const RelaxArgs ra = part_args(c);
  const unsigned grid = c.part_grid;
  const uint32_t nwaves = grid * (TB / 64);
  k_pbucket<<<1, 64, 0, s>>>(c.d_ctrl.p, c.d_pcnt.p, bucket_key);
  switch (b.FP) {
    case 1: k_scan<1, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 2: k_scan<2, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 4: k_scan<4, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 8: k_scan<8, false, false><<<grid, TB, 0, s>>>(ra); break;
    default: k_scan<16, false, false><<<grid, TB, 0, s>>>(ra); break;
  }
  k_pcount<<<std::min<uint32_t>(64, (nwaves + TB - 1) / TB), TB, 0, s>>>(c.d_fr_cnt.p, nwaves, c.d_pcnt.p);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_ctrl.p + 1, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipMemcpyAsync(c.h_pinned + 1, c.d_pcnt.p, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  *m1 = c.h_pinned[0];
  const uint64_t need = c.h_pinned[1] * b.FP;  // lanes of the compacted groups bound the records
  c.stats.relax_launches++;
  if (need > cap) {
    *n = need;
    return false;
  }
  if (need) {
    if (!rec) c.fail(GS_EINVAL, "null record buffer");
    switch (b.FP) {
      case 1: part_export_fp<1>(ra, grid, s, rec, cap, c.d_pcnt.p); break;
      case 2: part_export_fp<2>(ra, grid, s, rec, cap, c.d_pcnt.p); break;
      case 4: part_export_fp<4>(ra, grid, s, rec, cap, c.d_pcnt.p); break;
      case 8: part_export_fp<8>(ra, grid, s, rec, cap, c.d_pcnt.p); break;
      default: part_export_fp<16>(ra, grid, s, rec, cap, c.d_pcnt.p); break;
    }
    GS_HIP(hipGetLastError());
  }
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pcnt.p + 1, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  *n = c.h_pinned[0];
  return true;
}

uint64_t part_relax(Ctx& c, uint64_t bucket_key, const gs_part_record* rec, uint64_t n) {
  if (!c.part_open) c.fail(GS_ESTATE, "gs_part_begin first");
  (void)bucket_key;  // records carry their own keys; the argument documents the protocol step
  if (n == 0) return INF64;
  if (!rec) c.fail(GS_EINVAL, "null record buffer");
  hipStream_t s = c.stream;
  const Batch& b = c.part_b;
  const RelaxArgs ra = part_args(c);
  GS_HIP(hipMemsetAsync(c.d_pcnt.p + 2, 0xFF, 8, s));
  const unsigned grid = (unsigned)std::min<uint64_t>((n + TB - 1) / TB, (uint64_t)c.num_cus * 16);
  switch (b.FP) {
    case 1: part_recv_fp<1>(ra, grid, s, rec, n, c.d_pcnt.p); break;
    case 2: part_recv_fp<2>(ra, grid, s, rec, n, c.d_pcnt.p); break;
    case 4: part_recv_fp<4>(ra, grid, s, rec, n, c.d_pcnt.p); break;
    case 8: part_recv_fp<8>(ra, grid, s, rec, n, c.d_pcnt.p); break;
    default: part_recv_fp<16>(ra, grid, s, rec, n, c.d_pcnt.p); break;
  }
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pcnt.p + 2, 8, hipMemcpyDeviceToHost, s));
  GS_HIP(hipStreamSynchronize(s));
  return c.h_pinned[0];
}

// Lazy gossip in partitioned mode: the eager result stands when gossip is a
// no-op (gossip_noop). Each part checks its own peers; the
// condition holds for the whole graph iff it holds in every part, so a part
// whose peers could take an IWANT fails the batch (GS_EUNSUPPORTED) rather
// than return a result without the gossip relaxations.
// ---- steps of the library-driven protocol (gs_comm.hip, gs_run_partitioned);
// every one is stream-ordered on the context's stream, no host synchronisation.

void part_dev_bucket(Ctx& c, uint32_t parts) {
  c.d_dcnt.alloc(64);
  c.d_dpos.alloc(64);
  k_pbucket_dev<<<1, 64, 0, c.stream>>>(c.d_ctrl.p, c.d_pcnt.p, c.d_dcnt.p, c.d_dpos.p, parts);
  GS_HIP(hipGetLastError());
}

// k_scan of the bucket in ctrl[0] + the per-destination record counts (d_dcnt).
void part_dev_scan_count(Ctx& c, uint32_t parts) {
  hipStream_t s = c.stream;
  const Batch& b = c.part_b;
  const RelaxArgs ra = part_args(c);
  const unsigned grid = c.part_grid;
  switch (b.FP) {
    case 1: k_scan<1, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 2: k_scan<2, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 4: k_scan<4, false, false><<<grid, TB, 0, s>>>(ra); break;
    case 8: k_scan<8, false, false><<<grid, TB, 0, s>>>(ra); break;
    default: k_scan<16, false, false><<<grid, TB, 0, s>>>(ra); break;
  }
#define GS_PCOUNT(F) k_pexport_dest<F, true><<<grid, TB, 0, s>>>(ra, nullptr, c.d_dcnt.p, c.d_dpos.p, parts, c.cfg.peers)
  switch (b.FP) {
    case 1: GS_PCOUNT(1); break;
    case 2: GS_PCOUNT(2); break;
    case 4: GS_PCOUNT(4); break;
    case 8: GS_PCOUNT(8); break;
    default: GS_PCOUNT(16); break;
  }
#undef GS_PCOUNT
  GS_HIP(hipGetLastError());
  c.stats.relax_launches++;
}

// The records, grouped by destination part (offsets = prefix of d_dcnt).
void part_dev_export(Ctx& c, uint32_t parts, gs_part_record* out) {
  hipStream_t s = c.stream;
  const Batch& b = c.part_b;
  const RelaxArgs ra = part_args(c);
  const unsigned grid = c.part_grid;
#define GS_PEXP(F) k_pexport_dest<F, false><<<grid, TB, 0, s>>>(ra, out, c.d_dcnt.p, c.d_dpos.p, parts, c.cfg.peers)
  switch (b.FP) {
    case 1: GS_PEXP(1); break;
    case 2: GS_PEXP(2); break;
    case 4: GS_PEXP(4); break;
    case 8: GS_PEXP(8); break;
    default: GS_PEXP(16); break;
  }
#undef GS_PEXP
  GS_HIP(hipGetLastError());
}

// Received records into own peers, then this part's next-bucket candidate in ctrl[0].
void part_dev_relax_next(Ctx& c, const gs_part_record* in, uint64_t n) {
  hipStream_t s = c.stream;
  const Batch& b = c.part_b;
  if (n) {
    const RelaxArgs ra = part_args(c);
    const unsigned grid = (unsigned)std::min<uint64_t>((n + TB - 1) / TB, (uint64_t)c.num_cus * 16);
    switch (b.FP) {
      case 1: part_recv_fp<1>(ra, grid, s, in, n, c.d_pcnt.p); break;
      case 2: part_recv_fp<2>(ra, grid, s, in, n, c.d_pcnt.p); break;
      case 4: part_recv_fp<4>(ra, grid, s, in, n, c.d_pcnt.p); break;
      case 8: part_recv_fp<8>(ra, grid, s, in, n, c.d_pcnt.p); break;
      default: part_recv_fp<16>(ra, grid, s, in, n, c.d_pcnt.p); break;
    }
  }
  k_pnext<<<1, 64, 0, s>>>(c.d_ctrl.p, c.d_pcnt.p);
  GS_HIP(hipGetLastError());
}

// Completion of this part's own peers (k_complete, with the 100 ms histograms
// when a summary is wanted) and, with lazy gossip, this part's half of the
// no-op proof (gossip_noop over its own peers; the batch stands iff every
// part's holds). Returns true without lazy gossip.
// Completion in two steps, so that several contexts' completions overlap:
// enqueue the reductions (and the message statistics' copy into pinned memory),
// then wait and check the gossip proof.
static void part_dev_complete_enqueue(Ctx& c, bool hist, bool store) {
  const Batch& b = c.part_b;
  run_complete(c, b, c.part_u0, c.part_un, true, hist, store);
  if (!c.cfg.lazy_gossip) return;
  const size_t msb = (size_t)b.B * MS_COLS * 8;
  if (c.h_slms_bytes < msb) {
    if (c.h_slms) GS_HIP(hipHostFree(c.h_slms));
    c.h_slms = nullptr;
    c.h_slms_bytes = 0;
    GS_HIP(hipHostMalloc((void**)&c.h_slms, msb, hipHostMallocDefault));
    c.h_slms_bytes = msb;
  }
  GS_HIP(hipMemcpyAsync(c.h_slms, c.d_mstat.p, msb, hipMemcpyDeviceToHost, c.stream));
}

static bool part_dev_complete_check(Ctx& c) {
  if (!c.cfg.lazy_gossip) return true;
  const Batch& b = c.part_b;
  GS_HIP(hipStreamSynchronize(c.stream));
  const uint64_t* ms = c.h_slms;
  std::vector<uint64_t> rel0(b.B);
  const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
  for (uint32_t q = 0; q < b.B; q++) {
    const uint64_t tp = b.tpub[q], h0 = tp <= ph ? 0 : (tp - ph + hb - 1) / hb;
    rel0[q] = ph + h0 * hb - tp;
  }
  const bool ok = gossip_noop(b, ms, rel0);
  if (!ok)
    for (uint32_t q = 0; q < b.B; q++) {
      const uint64_t und = ms[(size_t)q * MS_COLS + MS_UNDEL], tm = ms[(size_t)q * MS_COLS + MS_TMAX];
      if (und || tm >= rel0[q] + b.lat_min) {
        c.gossip_why = "part " + std::to_string(c.part_idx) + " message " + std::to_string(q) + ": " +
                       std::to_string(und) + " peers never complete, last completion " + std::to_string(tm) +
                       " ns >= first IHAVE " + std::to_string(rel0[q] + b.lat_min) + " ns";
        break;
      }
    }
  return ok;
}

bool part_dev_complete(Ctx& c, bool hist, bool store) {
  part_dev_complete_enqueue(c, hist, store);
  return part_dev_complete_check(c);
}

// Finish a completed batch whose gossip proof holds everywhere: delivery into
// sink rows [row0, row0 + B), counters.
void part_dev_finish(Ctx& c, const gs_result_sink* sink, uint64_t row0) {
  if (!c.part_open) c.fail(GS_ESTATE, "gs_part_begin first");
  c.part_open = false;
  const Batch& b = c.part_b;
  deliver(c, b, c.part_u0, c.part_un, sink, row0);
  if (c.cfg.lazy_gossip) c.stats.gossip_noop_msgs += b.B;
  c.stats.messages += b.B;
  c.stats.batches++;
  collect_stats(c);
}

void part_abort(Ctx& c) { c.part_open = false; }

void part_finish(Ctx& c, const gs_result_sink* sink) {
  if (!c.part_open) c.fail(GS_ESTATE, "gs_part_begin first");
  c.part_open = false;
  const Batch& b = c.part_b;
  const bool gossip = c.cfg.lazy_gossip != 0;
  run_complete(c, b, c.part_u0, c.part_un, gossip || (sink && sink->summary), sink && sink->summary);
  if (gossip) {
    std::vector<uint64_t> ms((size_t)b.B * MS_COLS), rel0(b.B);
    GS_HIP(hipMemcpyAsync(ms.data(), c.d_mstat.p, ms.size() * 8, hipMemcpyDeviceToHost, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
    const uint64_t hb = c.cfg.heartbeat_ns, ph = c.cfg.hb_phase_ns;
    for (uint32_t q = 0; q < b.B; q++) {
      const uint64_t tp = b.tpub[q], h0 = tp <= ph ? 0 : (tp - ph + hb - 1) / hb;
      rel0[q] = ph + h0 * hb - tp;
    }
    if (!gossip_noop(b, ms.data(), rel0))
      c.fail(GS_EUNSUPPORTED, "lazy gossip can change this batch (an IHAVE lands before the last delivery); "
                              "partitioned mode runs eager forwarding only: use gs_run");
    c.stats.gossip_noop_msgs += b.B;
  }
  deliver(c, b, c.part_u0, c.part_un, sink, 0);
  c.stats.messages += b.B;
  collect_stats(c);
}

// ---- the list pass over partitioned rows (gs_run_partitioned) ----
// Every part runs k_lpull<.., PART> over its own rows [u0, u0 + un) with the
// list path's per-row buffers sized for those rows; after each pass the host
// combines the parts' pass control (records emitted, min pending key, error
// word), every part packs its records (k_lpack) and the packed records, the
// per-peer counts and offsets are exchanged (gs_comm.hip), so that the next
// pass reads any neighbour's records exactly as gs_run's pass does.

static LPullArgs part_lp_args(Ctx& c) {
  const Batch& b = c.part_b;
  const uint32_t un = c.part_un, L = b.L;
  LPullArgs la{};
  la.keys = c.d_keys.p; la.flane = c.d_flane.p; la.busy = c.d_busy.p; la.blk = c.d_lblk.p;
  la.st = c.d_lst.p; la.fin = c.d_lfin.p; la.lrec = c.d_lrec.p; la.lcnt = c.d_lcnt.p;
  la.rpos = c.d_rpos.p; la.mesh = c.d_mesh.p; la.pub = c.d_pub.p; la.stage = c.d_stage.p;
  la.tables = c.d_tables.p; la.ctrl = c.d_pctrl.p; la.counters = c.d_counters.p;
  const uint64_t grain = pull_grain(b.tshift);
  la.delta = b.delta / grain * grain;
  la.tmax = b.tmax - grain;
  la.N = un; la.B = b.B; la.L = L; la.S = c.S; la.sb = b.sb; la.tshift = b.tshift;
  la.K = c.part_lpK; la.lb = c.part_lplb; la.dG = (uint32_t)(la.delta / grain);
  la.ls = lpull_stride(b);
  const char* cap = getenv("GS_LPULL_CAP");
  la.lcap = cap && *cap ? (uint32_t)std::min<long>(std::max(1, atoi(cap)), (long)la.ls) : la.ls;
  la.u0 = c.part_u0;
  la.rmax = lpull_rmax(b);
  la.rpk = c.d_rpk.p; la.roff = c.d_roffg.p; la.rcg = c.d_rcg.p;
  la.pass = c.part_lppass;
  return la;
}

bool part_lp_begin(Ctx& c, const gs_publish* sched, uint64_t n_msgs) {
  const uint32_t F = part_check(c, sched, n_msgs);
  (void)F;
  const char* ve = getenv("GS_RELAX_VARIANT");  // without bit 64 (or GS_PART_PUSH) the push protocol runs
  if ((ve && *ve && !(atoi(ve) & 64)) || getenv("GS_PART_PUSH")) return false;
  hipStream_t s = c.stream;
  GS_HIP(hipMemsetAsync(c.d_counters.p + C_ERR, 0, 8, s));
  ensure_cus(c);
  const uint32_t N = c.cfg.peers, un = c.part_un, Bmax = c.cfg.batch;
  c.part_b = setup_batch(c, sched, 0, n_msgs);
  const Batch& b = c.part_b;
  if (b.L > PULL_LMAX || b.delta < pull_grain(b.tshift)) return false;
  uint32_t lb = 0;
  const uint64_t grain = pull_grain(b.tshift);
  const uint32_t K = lpull_ring(c, b, b.delta / grain * grain, &lb);
  if (!K) return false;
  c.part_lpK = K;
  c.part_lplb = lb;
  c.part_lppass = 0;
  const size_t NL = (size_t)un * b.L;
  const uint32_t ls = lpull_stride(b);
  c.d_keys.alloc(NL);
  c.d_flane.alloc(NL);
  c.d_lrec.alloc(2 * NL);
  c.d_lcnt.alloc(2 * (size_t)un);
  c.d_lblk.alloc((size_t)K * un * ls);
  c.d_lst.alloc((size_t)un * LP_SW);
  c.d_lfin.alloc((size_t)un * LP_FW);
  c.d_pctrl.alloc(12);
  c.d_rcg.alloc(N);
  c.d_roffg.alloc(N);
  c.d_rpk.alloc(1);
  c.d_pkcur.alloc(1);
  if (b.FP > 1) c.d_busy.alloc((size_t)un * Bmax);
  c.d_tc.alloc((size_t)un * Bmax);
  c.d_hops.alloc((size_t)un * Bmax);
  if (!c.rpos_valid) {
    c.d_rpos.alloc((size_t)N * MESH_W);
    k_rpos<<<(unsigned)(((uint64_t)N * MESH_W + TB - 1) / TB), TB, 0, s>>>(c.d_mesh.p, c.d_rpos.p, N, c.d_counters.p);
    GS_HIP(hipGetLastError());
    if (read_counter(c, C_ERR) & ERR_MESH) c.fail(GS_ERANGE, "mesh is not symmetric");
    c.rpos_valid = true;
  }
  c.keys_log = false;
  if (b.FP > 1) GS_HIP(hipMemsetAsync(c.d_busy.p, 0, (size_t)un * b.B * 8, s));
  GS_HIP(hipMemsetAsync(c.d_lst.p, 0, (size_t)un * LP_SW * 4, s));
  GS_HIP(hipMemsetAsync(c.d_lfin.p, 0, (size_t)un * LP_FW * 4, s));
  GS_HIP(hipMemsetAsync(c.d_pctrl.p, 0, 12 * 8, s));
  for (int q = 0; q < 3; q++) GS_HIP(hipMemsetAsync(c.d_pctrl.p + q * 4 + 3, 0xFF, 8, s));
  c.d_lp_save.alloc(C_COUNT);
  GS_HIP(hipMemcpyAsync(c.d_lp_save.p, c.d_counters.p, C_COUNT * 8, hipMemcpyDeviceToDevice, s));
  const uint64_t scap = (uint64_t)b.B * b.Fe * std::max<uint64_t>(c.max_degree, MESH_W);
  c.d_skey.alloc(scap);
  c.d_slane.alloc(scap);
  c.d_scnt.alloc(1);
  GS_HIP(hipMemsetAsync(c.d_scnt.p, 0, 4, s));
  launch_seed(c, b, c.part_u0, un, c.d_pctrl.p + 2 * 4 + 3, nullptr, true);
  const LPullArgs la = part_lp_args(c);
  k_lseed<<<(unsigned)std::max<uint64_t>(1, std::min<uint64_t>((scap + TB - 1) / TB, (uint64_t)c.num_cus * 4)), TB, 0,
            s>>>(la, c.d_skey.p, c.d_slane.p, c.d_scnt.p);
  k_lpub<<<(b.B * b.Fe + 255) / 256, 256, 0, s>>>(la, b.Fe);
  GS_HIP(hipGetLastError());
  uint64_t auto_bpc = 4;  // as run_lpull_batch: whole blocks per CU by the rows this part owns
  while (auto_bpc < 16 && (uint64_t)un >= (uint64_t)c.num_cus * PULL_WAVES * 32 * auto_bpc * 2) auto_bpc *= 2;
  c.part_lpgrid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>(((uint64_t)un + PULL_WAVES - 1) / PULL_WAVES, (uint64_t)c.num_cus * auto_bpc));
  // the seeds' min key lands in pinned word 28; part_lp_seed_min waits for it
  // (the caller begins every part first, so that their setups overlap)
  GS_HIP(hipMemcpyAsync(c.h_pinned + 28, c.d_pctrl.p + 2 * 4 + 3, 8, hipMemcpyDeviceToHost, s));
  c.part_lp = true;
  c.part_open = true;
  return true;
}

uint64_t part_lp_seed_min(Ctx& c) {
  GS_HIP(hipStreamSynchronize(c.stream));
  return c.h_pinned[28];
}

// The combined pass control into the slot the next pass decides from (slot of the last pass).
void part_lp_set(Ctx& c, uint64_t records, uint64_t minp) {
  const uint32_t slot = (c.part_lppass + 2) % 3;  // the last pass's slot (seeds: slot 2 before pass 0)
  c.h_pinned[24] = records;
  c.h_pinned[25] = minp;
  // (no wait: the staging words are next written by the next part_lp_set,
  // after part_lp_read has drained this stream)
  GS_HIP(hipMemcpyAsync(c.d_pctrl.p + slot * 4 + 2, c.h_pinned + 24, 16, hipMemcpyHostToDevice, c.stream));
}

void part_lp_pass(Ctx& c) {
  const LPullArgs la = part_lp_args(c);
  lpull_dispatch_part(c.part_b.FP, la, c.part_lpgrid, c.stream);
  GS_HIP(hipGetLastError());
  c.part_lppass++;
  c.stats.relax_launches++;
}

// The last pass's control words into pinned memory (enqueued), then waited
// for: several parts' reads in flight together.
void part_lp_read_enqueue(Ctx& c) {
  const uint32_t slot = (c.part_lppass + 2) % 3;
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pctrl.p + slot * 4, 32, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipMemcpyAsync(c.h_pinned + 4, c.d_counters.p + C_ERR, 8, hipMemcpyDeviceToHost, c.stream));
}

void part_lp_read_wait(Ctx& c, uint64_t out[4]) {
  GS_HIP(hipStreamSynchronize(c.stream));
  out[0] = c.h_pinned[1];
  out[1] = c.h_pinned[2];
  out[2] = c.h_pinned[3];
  out[3] = c.h_pinned[4];
}

void part_lp_read(Ctx& c, uint64_t out[4]) {
  part_lp_read_enqueue(c);
  part_lp_read_wait(c, out);
}

void part_lp_pack(Ctx& c, uint64_t base, uint64_t mine) {
  const uint32_t un = c.part_un, L = c.part_b.L;
  (void)mine;  // the caller sized d_rpk for every part's records
  hipStream_t s = c.stream;
  GS_HIP(hipMemsetAsync(c.d_pkcur.p, 0, 8, s));
  const uint32_t nb = (c.part_lppass + 1) & 1;  // the last pass wrote lrec / lcnt [pass & 1]
  const unsigned grid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>(((uint64_t)un + 255) / 256, (uint64_t)c.num_cus * 8));
  k_lpack<<<grid, TB, 0, s>>>(c.d_lrec.p + (size_t)nb * un * L, c.d_lcnt.p + (size_t)nb * un, un, L, base,
                              c.d_rpk.p + base, c.d_roffg.p + c.part_u0, c.d_rcg.p + c.part_u0,
                              (unsigned long long*)c.d_pkcur.p);
  GS_HIP(hipGetLastError());
}

// Routed pack (k_lpack_route): this part's records of the last pass for each
// destination part, to the places `dst` names (part_lp_pack_route: send
// segments; the local exchange: the destination contexts' own buffers).
void part_lp_route_launch(Ctx& c, uint32_t P, uint32_t me, const RouteDst& dst) {
  const uint32_t un = c.part_un, L = c.part_b.L;
  hipStream_t s = c.stream;
  c.d_pkcur.alloc(P);
  GS_HIP(hipMemsetAsync(c.d_pkcur.p, 0, (size_t)P * 8, s));
  const uint32_t nb = (c.part_lppass + 1) & 1;  // the last pass wrote lrec / lcnt [pass & 1]
  const unsigned grid = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>(((uint64_t)un + 255) / 256, (uint64_t)c.num_cus * 8));
  RouteLo rl{};
  const PartLayout lay{P, c.cfg.peers, 0};
  for (uint32_t q = 0; q < P && q < LP_PMAX; q++) rl.lo[q] = lay.u0(q);
#define GS_LPR(PM)                                                                                             \
  k_lpack_route<PM><<<grid, TB, 0, s>>>(c.d_lrec.p + (size_t)nb * un * L, c.d_lcnt.p + (size_t)nb * un, c.d_mesh.p, \
                                        c.part_u0, un, L, P, me, (unsigned long long*)c.d_pkcur.p, rl, dst)
  if (P <= 4) GS_LPR(4);
  else if (P <= 8) GS_LPR(8);
  else GS_LPR(16);
#undef GS_LPR
  GS_HIP(hipGetLastError());
}

// The own part's records are read where the last pass wrote them (lrec half
// nb, rows of L): their offsets from d_rpk's base, as 64-bit element offsets
// modulo 2^64 (the pass adds them to the same base). d_rpk is sized before.
static void part_lp_own_inplace(Ctx& c, RouteDst& d) {
  const uint32_t un = c.part_un, L = c.part_b.L;
  const uint32_t nb = (c.part_lppass + 1) & 1;
  const uint64_t* rows = c.d_lrec.p + (size_t)nb * un * L;
  d.own_off = (uint64_t)(((intptr_t)rows - (intptr_t)c.d_rpk.p) / 8);  // (both 8-B aligned; may be negative)
  d.own_inplace = 1;
}

// Ranks: own records into d_rpk at base 0 with the global offset tables at its
// peers; other destinations into d_rsend[q * mine] with the tables
// d_rroff / d_rrcg[q * un] (offsets relative to the segment, k_roff_fix
// rebases them after the exchange).
void part_lp_pack_route(Ctx& c, uint32_t P, uint32_t me, uint64_t mine) {
  const uint32_t un = c.part_un;
  const uint64_t cap = std::max<uint64_t>(mine, 1);
  c.d_rsend.alloc((size_t)P * cap);
  c.d_rroff.alloc((size_t)P * un);
  c.d_rrcg.alloc((size_t)P * un);
  RouteDst d{};
  for (uint32_t q = 0; q < P; q++) {
    const bool own = q == me;
    d.out[q] = own ? c.d_rpk.p : c.d_rsend.p + (size_t)q * cap;
    d.roff[q] = own ? c.d_roffg.p + c.part_u0 : c.d_rroff.p + (size_t)q * un;
    d.rcg[q] = own ? c.d_rcg.p + c.part_u0 : c.d_rrcg.p + (size_t)q * un;
  }
  part_lp_own_inplace(c, d);
  part_lp_route_launch(c, P, me, d);
}

// Loop-back parts on one device: part `me`'s records straight into every
// destination context's gathered buffer at this part's gathered base (its
// capacity there is all its records), its tables at this part's peers; no copy,
// no rebasing. The destinations' buffers are sized before any part launches.
void part_lp_pack_route_direct(Ctx** cx, uint32_t P, uint32_t me, uint64_t base) {
  Ctx& c = *cx[me];
  const PartLayout lay{P, c.cfg.peers, 0};
  RouteDst d{};
  for (uint32_t q = 0; q < P; q++) {
    d.out[q] = cx[q]->d_rpk.p + base;
    d.roff[q] = cx[q]->d_roffg.p + lay.u0(me);
    d.rcg[q] = cx[q]->d_rcg.p + lay.u0(me);
    d.ob[q] = base;
  }
  part_lp_own_inplace(c, d);
  part_lp_route_launch(c, P, me, d);
}

// Loop-back parts on one device: every part's pass control combined on the
// device (k_part_combine on part 0's stream after every part's pass), read
// back once: st[p * 4 ..] = part p's {mode, records, min pending, error word},
// and every part's slot already holds the combined records and min pending
// key (no part_lp_set).
void part_lp_combine(Ctx** cx, uint32_t P, uint64_t* st) {
  Ctx& c0 = *cx[0];
  PartCtl pc{};
  for (uint32_t p = 0; p < P; p++) {
    Ctx& c = *cx[p];
    pc.ctrl[p] = c.d_pctrl.p;
    pc.err[p] = c.d_counters.p + C_ERR;
    if (p) {
      if (!c.part_pev) GS_HIP(hipEventCreateWithFlags(&c.part_pev, hipEventDisableTiming));
      GS_HIP(hipEventRecord(c.part_pev, c.stream));
      GS_HIP(hipStreamWaitEvent(c0.stream, c.part_pev, 0));
    }
  }
  c0.d_pstat.alloc((size_t)P * 4);
  if (!c0.h_pstat) GS_HIP(hipHostMalloc((void**)&c0.h_pstat, LP_PMAX * 4 * 8, hipHostMallocDefault));
  const uint32_t slot = (c0.part_lppass + 2) % 3;  // the last pass's slot (lockstep parts: the same in each)
  k_part_combine<<<1, 64, 0, c0.stream>>>(pc, P, slot, c0.d_pstat.p);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c0.h_pstat, c0.d_pstat.p, (size_t)P * 4 * 8, hipMemcpyDeviceToHost, c0.stream));
  GS_HIP(hipStreamSynchronize(c0.stream));
  memcpy(st, c0.h_pstat, (size_t)P * 4 * 8);
}

// The routed records per destination (counts[q]) of the last pack.
void part_lp_route_read(Ctx& c, uint32_t P, uint64_t* counts) {
  GS_HIP(hipMemcpyAsync(c.h_pinned, c.d_pkcur.p, (size_t)P * 8, hipMemcpyDeviceToHost, c.stream));
  GS_HIP(hipStreamSynchronize(c.stream));
  memcpy(counts, c.h_pinned, (size_t)P * 8);
}

// After the routed exchange: the foreign peers' offsets by their segment's base.
void part_lp_route_fix(Ctx& c, uint32_t P, uint32_t me, const uint64_t* base) {
  RouteBases rb{};
  for (uint32_t p = 0; p < P; p++) rb.b[p] = base[p];
  k_roff_fix<<<(unsigned)(((uint64_t)c.cfg.peers + TB - 1) / TB), TB, 0, c.stream>>>(c.d_roffg.p, c.cfg.peers, P, me,
                                                                                       rb);
  GS_HIP(hipGetLastError());
}

// As gs_run's list pass: completion reads the final logs (k_lcomplete) unless
// the sink takes rows or a summary, or the rows hold fragment groups (k_lfinal
// -> dense rows -> k_complete).
void part_lp_end_enqueue(Ctx& c, const gs_result_sink* sink) {
  const SinkWants w = sink_wants(sink);
  const bool dense = w.rows() || w.summary || c.part_b.FP > 1 || getenv("GS_LPULL_DENSE");
  if (dense) {
    const LPullArgs la = part_lp_args(c);
    k_lfinal<<<c.part_lpgrid, TB, 0, c.stream>>>(la);  // final logs -> dense rows of own peers
    GS_HIP(hipGetLastError());
  } else {
    c.keys_log = true;
  }
  c.stats.list_pull_batches++;
  c.part_lp = false;
  part_dev_complete_enqueue(c, w.summary, dense);
}

bool part_lp_end_check(Ctx& c) { return part_dev_complete_check(c); }

void part_lp_abort(Ctx& c) {  // the batch re-runs on the push protocol: counters as before the batch
  if (c.part_lp) {
    GS_HIP(hipMemcpyAsync(c.d_counters.p, c.d_lp_save.p, C_COUNT * 8, hipMemcpyDeviceToDevice, c.stream));
    GS_HIP(hipStreamSynchronize(c.stream));
  }
  c.part_lp = false;
  c.part_open = false;
}
