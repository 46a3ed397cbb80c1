/*
 * gs_oracle.c — single-threaded CPU restatement of the dissemination rules.
 *
 * TEST INFRASTRUCTURE ONLY (see gs_oracle.h). It is the parity checker for
 * libgossipsim.so and the `cpu_baseline` of bench.py; nothing in the product
 * links or calls it.
 *
 * Every function cites the reference file:line it follows. The gossipsub
 * router itself (libp2p-gossipsub 0.49.2) is not vendored: its rules are the
 * spec choices of DESIGN.md §2, written here with a binary-heap event
 * simulation (Dijkstra order) so that the GPU's Delta-stepping is checked by a
 * structurally different algorithm.
 */
#include "gs_oracle.h"
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define INF64 UINT64_MAX
#define HOP_BITS 6u
#define MESH_W 16u
#define BIT_OUT 1u
#define BIT_MESH 2u

enum { P_DIAL = 1, P_DIAL_ORDER = 2, P_GRAFT = 3, P_PRUNE = 4, P_OUT_GRAFT = 5 };

/* ---------------------------------------------------------------- RNG ---- */
/* Counter-based RNG keyed by (seed, purpose, a, b, c). The reference draws
 * from an unseeded thread RNG (rust-test-node/src/main.rs:308); go seeds it
 * with the node id (go-test-node/main.go:280-281). Here every draw is a pure
 * function of its coordinates so CPU and GPU agree bit for bit. */
static uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
    z ^= z >> 27; z *= 0x94D049BB133111EBULL;
    z ^= z >> 31; return z;
}
uint64_t or_rng(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b, uint32_t c) {
    uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ULL * (uint64_t)(purpose + 1u));
    h = mix64(h ^ ((uint64_t)a + 0x9E3779B97F4A7C15ULL));
    h = mix64(h ^ ((((uint64_t)b) << 32) | c) ^ 0xD6E8FEB86659FD93ULL);
    return h;
}
static uint64_t rand_below(uint64_t x, uint64_t n) {
    return (uint64_t)(((unsigned __int128)x * n) >> 64);
}

/* --------------------------------------------------------- wire bytes ---- */
static uint64_t varint_len(uint64_t x) { uint64_t n = 1; while (x >= 128) { x >>= 7; n++; } return n; }
static uint64_t pb_field(uint64_t len) { return 1 + varint_len(len) + len; }
static uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

/* Bytes on the wire for one fragment of `payload` bytes (model
 * constants). Signed gossipsub Message (main.rs:397): from
 * (38 B peer id), data, seqno (8 B), topic "test" (main.rs:443), signature
 * (64 B); unsigned (nim anonymize, gossipsub-queues/main.nim:447): data+topic.
 * RPC{publish} is length-prefixed on its stream. Then the MUXER stack of
 * main.rs:418-440: yamux 12 B per <=16 KiB frame, noise 18 B per <=65519 B,
 * TCP/IPv4 40 B per 1460 B segment; QUIC 65 B per 1415 B of stream data;
 * mplex 4 B per <=1 MiB frame. */
static uint64_t stack_bytes(uint64_t frame, uint32_t muxer);
uint64_t or_wire_bytes(uint64_t payload, uint32_t muxer, uint32_t signed_msgs) {
    uint64_t msg = pb_field(payload) + pb_field(4);
    if (signed_msgs) msg += pb_field(38) + pb_field(8) + pb_field(64);
    uint64_t rpc = pb_field(msg);
    return stack_bytes(varint_len(rpc) + rpc, muxer);
}

/* A length-delimited RPC frame through the muxer stack. */
static uint64_t stack_bytes(uint64_t frame, uint32_t muxer) {
    if (muxer == 1) /* quic */
        return frame + cdiv(frame, 1415) * 65;
    uint64_t a = (muxer == 2) ? frame + cdiv(frame, 1048576) * 4 : frame + cdiv(frame, 16384) * 12;
    uint64_t b = a + cdiv(a, 65519) * 18;
    return b + cdiv(b, 1460) * 40;
}

/* The packets of that last layer and their header bytes (the counters Shadow's
 * tracker keeps per host, shadow/summary_shadowlog.awk:21-63). */
void or_wire_packets(uint64_t payload, uint32_t muxer, uint32_t signed_msgs, uint64_t* packets,
                     uint64_t* header_bytes) {
    uint64_t w = or_wire_bytes(payload, muxer, signed_msgs), per = muxer == 1 ? 1415 + 65 : 1460 + 40;
    uint64_t n = cdiv(w, per); /* every packet but the last is full: ceil(wire / full packet) */
    *packets = n;
    *header_bytes = n * (muxer == 1 ? 65 : 40);
}

/* Lazy-gossip control RPCs, one message id each (model constants, DESIGN.md
 * §2.4): RPC{control: ControlMessage{ihave: ControlIHave{topic "test", id}}}
 * or RPC{control: {iwant: ControlIWant{id}}}. The id is the node's
 * message_id_fn output: rust DefaultHasher u64 as decimal (main.rs:73-77) and
 * nim $hash (gossipsub-queues/main.nim:123-124), up to 20 chars, modelled at
 * 20; go sha256 (go-test-node/main.go:26-29), 32 bytes. kind 2 = a pure ACK
 * packet (no payload): packets 1, bytes = header = one packet header. */
void or_ctrl_packets(uint32_t kind, uint32_t node, uint32_t muxer, uint64_t* bytes, uint64_t* packets,
                     uint64_t* header_bytes) {
    const uint64_t ph = muxer == 1 ? 65 : 40, per = muxer == 1 ? 1415 + 65 : 1460 + 40;
    if (kind == 2) { *bytes = ph; *packets = 1; *header_bytes = ph; return; }
    const uint64_t id = node == 1 ? 32 : 20;
    const uint64_t cm = kind == 0 ? pb_field(pb_field(4) + pb_field(id)) : pb_field(pb_field(id));
    const uint64_t rpc = pb_field(cm);
    const uint64_t w = stack_bytes(varint_len(rpc) + rpc, muxer);
    *bytes = w;
    *packets = cdiv(w, per);
    *header_bytes = *packets * ph;
}

/* ---------------------------------------------------------- link model ---- */
/* shadow/topogen.py:39-71: stage bandwidth ceil(i*bj + bl) Mbit (49-51),
 * self-loop max((S-i)*lj, ll) ms (55), edge i<j min(ceil((S-j)*lj+ll), lh) ms
 * (60), injector node S at 1 ms from everything (64-69). mode 0 = the direct
 * GML edge; mode 1 = shortest non-empty path over the GML graph incl. the
 * injector hub (Shadow's use_shortest_path; upstream, not vendored). */
int or_topogen_links(uint32_t S, uint32_t bl, uint32_t bh, uint32_t ll, uint32_t lh,
                     uint32_t mode, uint64_t* lat_ns, uint64_t* bw_bps) {
    if (S == 0 || S > 255 || bl > bh || ll > lh || mode > 1) return -1;
    uint64_t bj = (bh - bl) / S, lj = (lh - ll) / S;
    uint32_t V = S + 1;
    uint64_t* g = (uint64_t*)malloc(sizeof(uint64_t) * V * V);
    if (!g) return -2;
    for (uint32_t i = 0; i < S; i++) {
        bw_bps[i] = ((uint64_t)i * bj + bl) * 1000000ULL;
        uint64_t self = (uint64_t)(S - i) * lj; if (self < ll) self = ll;
        g[i * V + i] = self;
        for (uint32_t j = i + 1; j < S; j++) {
            uint64_t e = (uint64_t)(S - j) * lj + ll; if (e > lh) e = lh;
            g[i * V + j] = g[j * V + i] = e;
        }
    }
    for (uint32_t i = 0; i <= S; i++) g[i * V + S] = g[S * V + i] = 1;
    if (mode == 0) {
        for (uint32_t i = 0; i < S; i++)
            for (uint32_t j = 0; j < S; j++) lat_ns[i * S + j] = g[i * V + j] * 1000000ULL;
    } else {
        uint64_t* d = (uint64_t*)malloc(sizeof(uint64_t) * V * V);
        if (!d) { free(g); return -2; }
        for (uint32_t i = 0; i < V; i++)
            for (uint32_t j = 0; j < V; j++) d[i * V + j] = (i == j) ? 0 : g[i * V + j];
        for (uint32_t k = 0; k < V; k++)
            for (uint32_t i = 0; i < V; i++)
                for (uint32_t j = 0; j < V; j++)
                    if (d[i * V + k] + d[k * V + j] < d[i * V + j]) d[i * V + j] = d[i * V + k] + d[k * V + j];
        for (uint32_t i = 0; i < S; i++)
            for (uint32_t j = 0; j < S; j++) {
                uint64_t v = d[i * V + j];
                if (i == j) {
                    v = g[i * V + i];
                    for (uint32_t k = 0; k < V; k++)
                        if (k != i && d[i * V + k] + d[k * V + i] < v) v = d[i * V + k] + d[k * V + i];
                }
                lat_ns[i * S + j] = v * 1000000ULL;
            }
        free(d);
    }
    free(g);
    return 0;
}

/* ---------------------------------------------------------- topology ---- */
/* Dials per peer: rust takes min(2*CONNECTTO, N-1) shuffled candidates
 * (main.rs:311-320) and dials until connected > CONNECTTO (main.rs:336-354),
 * i.e. CONNECTTO+1 dials (defect D4); nim stops at CONNECTTO
 * (gossipsub-queues/main.nim:396). */
uint32_t or_dials_per_peer(const or_params* p) {
    uint64_t lim = 2ull * p->connect_to;
    if (lim > (uint64_t)p->peers - 1) lim = p->peers - 1;
    uint64_t k = (uint64_t)p->connect_to + p->dial_extra;
    return (uint32_t)(k < lim ? k : lim);
}

/* Peer v's dial list: a uniform k-subset of the other N-1 ids (Floyd's
 * sampling), put in dial order by a per-(v,id) random key. */
static void gen_dials(const or_params* p, uint32_t v, uint32_t k, uint32_t* out) {
    uint64_t n = p->peers - 1;
    uint32_t m = 0;
    for (uint32_t i = 0; i < k; i++) {
        uint64_t j = n - k + i;
        uint64_t r = rand_below(or_rng(p->seed, P_DIAL, v, i, 0), j + 1);
        int dup = 0;
        for (uint32_t q = 0; q < m; q++) if (out[q] == (uint32_t)r) { dup = 1; break; }
        out[m++] = dup ? (uint32_t)j : (uint32_t)r;
    }
    for (uint32_t i = 0; i < k; i++) out[i] = out[i] < v ? out[i] : out[i] + 1;
    /* insertion sort by (rng key, id) */
    for (uint32_t i = 1; i < k; i++) {
        uint32_t x = out[i]; uint64_t kx = or_rng(p->seed, P_DIAL_ORDER, v, x, 0);
        int32_t j = (int32_t)i - 1;
        while (j >= 0) {
            uint64_t kj = or_rng(p->seed, P_DIAL_ORDER, v, out[j], 0);
            if (kj < kx || (kj == kx && out[j] < x)) break;
            out[j + 1] = out[j]; j--;
        }
        out[j + 1] = x;
    }
}

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* Symmetric CSR of accepted dials. Entry (u,w) gets bit0 when u dialed w.
 * MAXCONNECTIONS (nim gossipsub-queues/main.nim:429): acceptor t takes its
 * non-mutual inbound dials in (dial index, dialer) order up to cap - k. */
int or_build_topology(const or_params* p, uint64_t* row_ptr, uint32_t* col, uint8_t* flags,
                      uint64_t* nnz_out) {
    uint32_t N = p->peers;
    if (N < 2) return -1;
    uint32_t k = or_dials_per_peer(p);
    if (k == 0) return -1; /* "Failed to connect any peers" (main.rs:381-382) */
    uint32_t* dial = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)N * k);
    uint8_t* acc = (uint8_t*)malloc((size_t)N * k);
    if (!dial || !acc) { free(dial); free(acc); return -2; }
    for (uint32_t v = 0; v < N; v++) gen_dials(p, v, k, dial + (size_t)v * k);
    memset(acc, 1, (size_t)N * k);
    if (p->max_connections) {
        uint32_t quota = p->max_connections > k ? p->max_connections - k : 0;
        /* inbound lists: key = (j << 32) | v, bucketed by acceptor */
        uint64_t* cnt = (uint64_t*)calloc((size_t)N + 1, sizeof(uint64_t));
        uint64_t* in = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N * k);
        uint64_t* fill = (uint64_t*)calloc((size_t)N, sizeof(uint64_t));
        if (!cnt || !in || !fill) { free(cnt); free(in); free(fill); free(dial); free(acc); return -2; }
        for (uint64_t e = 0; e < (uint64_t)N * k; e++) cnt[dial[e] + 1]++;
        for (uint32_t t = 0; t < N; t++) cnt[t + 1] += cnt[t];
        for (uint32_t v = 0; v < N; v++)
            for (uint32_t j = 0; j < k; j++) {
                uint32_t t = dial[(size_t)v * k + j];
                in[cnt[t] + fill[t]++] = ((uint64_t)j << 32) | v;
            }
        for (uint32_t t = 0; t < N; t++) {
            uint64_t b = cnt[t], e = cnt[t + 1];
            qsort(in + b, e - b, sizeof(uint64_t), cmp_u64);
            uint32_t taken = 0;
            for (uint64_t q = b; q < e; q++) {
                uint32_t v = (uint32_t)in[q], j = (uint32_t)(in[q] >> 32);
                int mutual = 0;
                for (uint32_t jj = 0; jj < k; jj++) if (dial[(size_t)t * k + jj] == v) { mutual = 1; break; }
                if (mutual) continue;
                if (taken < quota) taken++; else acc[(size_t)v * k + j] = 0;
            }
        }
        free(cnt); free(in); free(fill);
    }
    /* half-edges (row, col<<1 | out), then per-row sort + dedupe */
    uint64_t* deg = (uint64_t*)calloc((size_t)N + 1, sizeof(uint64_t));
    uint64_t* he = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)N * k * 2);
    uint64_t* fill = (uint64_t*)calloc((size_t)N, sizeof(uint64_t));
    if (!deg || !he || !fill) { free(deg); free(he); free(fill); free(dial); free(acc); return -2; }
    for (uint32_t v = 0; v < N; v++)
        for (uint32_t j = 0; j < k; j++)
            if (acc[(size_t)v * k + j]) { deg[v + 1]++; deg[dial[(size_t)v * k + j] + 1]++; }
    for (uint32_t v = 0; v < N; v++) deg[v + 1] += deg[v];
    for (uint32_t v = 0; v < N; v++)
        for (uint32_t j = 0; j < k; j++) {
            if (!acc[(size_t)v * k + j]) continue;
            uint32_t t = dial[(size_t)v * k + j];
            he[deg[v] + fill[v]++] = ((uint64_t)t << 1) | 1u;
            he[deg[t] + fill[t]++] = ((uint64_t)v << 1);
        }
    uint64_t nnz = 0;
    row_ptr[0] = 0;
    for (uint32_t v = 0; v < N; v++) {
        uint64_t b = deg[v], e = deg[v + 1];
        qsort(he + b, e - b, sizeof(uint64_t), cmp_u64);
        for (uint64_t q = b; q < e; q++) {
            uint32_t c = (uint32_t)(he[q] >> 1); uint8_t o = (uint8_t)(he[q] & 1u);
            if (nnz > row_ptr[v] && col[nnz - 1] == c) { flags[nnz - 1] |= o; continue; }
            col[nnz] = c; flags[nnz] = o; nnz++;
        }
        row_ptr[v + 1] = nnz;
    }
    *nnz_out = nnz;
    free(deg); free(he); free(fill); free(dial); free(acc);
    return 0;
}

/* -------------------------------------------------------------- mesh ---- */
/* Heartbeat GRAFT/PRUNE (libp2p-gossipsub heartbeat/handle_graft/handle_prune,
 * upstream, not vendored; parameters main.rs:228-236), synchronous epochs of
 * DESIGN.md §2.3 (mesh_epoch below). */
static uint64_t find_entry(const uint64_t* row_ptr, const uint32_t* col, uint32_t u, uint32_t w) {
    uint64_t lo = row_ptr[u], hi = row_ptr[u + 1];
    while (lo < hi) { uint64_t mid = (lo + hi) / 2; if (col[mid] < w) lo = mid + 1; else hi = mid; }
    return lo;
}

typedef struct { uint64_t key; uint64_t e; } sel_t;
static int cmp_sel(const void* a, const void* b) {
    const sel_t *x = (const sel_t*)a, *y = (const sel_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->e < y->e ? -1 : x->e > y->e;
}

/* Churn (config #3 of BASELINE.json, build-defined, parity
 * unpinned: the reference has no churn). Peer u is offline during heartbeat
 * epoch h >= 1 iff a departure was drawn at one of the epochs h-down+1..h:
 * rng(CHURN, u, h') below churn_ppm per million. Epoch 0 (before the first
 * heartbeat) has everyone online. */
enum { P_CHURN = 7 };
int or_offline(const or_params* p, uint32_t u, uint64_t h) {
    if (!p->churn_ppm || h == 0) return 0;
    for (uint64_t k = 0; k < p->churn_down && k < h; k++)
        if (rand_below(or_rng(p->seed, P_CHURN, u, (uint32_t)(h - k), 0), 1000000) < p->churn_ppm) return 1;
    return 0;
}

/* Mesh epoch workspace. nt > 1: the per-peer loops of mesh_epoch run on nt
 * OpenMP threads (every loop body writes only its own row's entries, and the
 * accept bits of phase B go to acc[], which only phase C reads), with one
 * selection buffer per thread; the result is the same as with nt = 1. */
typedef struct {
    uint32_t* until; uint8_t* prop; uint8_t* acc; uint64_t* rev; sel_t* sel; uint64_t bo; uint32_t nt, sel_n;
} mesh_ws;

static void mesh_ws_free(mesh_ws* w) { free(w->until); free(w->prop); free(w->acc); free(w->rev); free(w->sel); }

static int mesh_ws_init_nt(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, uint8_t* flags,
                           mesh_ws* w, uint32_t nt) {
    uint32_t N = p->peers;
    uint64_t nnz = row_ptr[N];
    w->nt = nt ? nt : 1;
    w->bo = (p->backoff_ns + p->heartbeat_ns - 1) / p->heartbeat_ns;
    w->until = (uint32_t*)calloc(nnz ? nnz : 1, sizeof(uint32_t));
    w->prop = (uint8_t*)calloc(nnz ? nnz : 1, 1); /* 1 graft, 2 prune */
    w->acc = (uint8_t*)calloc(nnz ? nnz : 1, 1);  /* 1 accepted (phase B -> C) */
    w->rev = (uint64_t*)malloc(sizeof(uint64_t) * (nnz ? nnz : 1));
    uint32_t maxdeg = 0;
    for (uint32_t u = 0; u < N; u++) {
        uint32_t dg = (uint32_t)(row_ptr[u + 1] - row_ptr[u]); if (dg > maxdeg) maxdeg = dg;
    }
    w->sel_n = maxdeg + 1;
    w->sel = (sel_t*)malloc(sizeof(sel_t) * w->sel_n * w->nt);
    if (!w->until || !w->prop || !w->acc || !w->rev || !w->sel) { mesh_ws_free(w); return -2; }
    for (uint32_t u = 0; u < N; u++)
        for (uint64_t e = row_ptr[u]; e < row_ptr[u + 1]; e++) w->rev[e] = find_entry(row_ptr, col, col[e], u);
    for (uint64_t e = 0; e < nnz; e++) flags[e] &= (uint8_t)~BIT_MESH;
    return 0;
}
static int mesh_ws_init(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, uint8_t* flags,
                        mesh_ws* w) {
    return mesh_ws_init_nt(p, row_ptr, col, flags, w, 1);
}

/* Handshake model of the subscription exchange: every peer
 * dials at the same instant (rust-test-node/src/main.rs:336-354 after the
 * common 60 s sleep, main.rs:457); a connection completes HS_RTTS round trips
 * later (TCP + multistream + Noise XX + yamux, a model constant) and each side
 * then sends its subscription, so w's subscription reaches u at
 * HS_RTTS*rtt(u,w) + lat(w->u), and u's GRAFT reaches w one lat(u->w) later. */
#define HS_RTTS_DEFAULT 3u
#define HS_RTTS (p->hs_rtts ? p->hs_rtts : HS_RTTS_DEFAULT)
static uint64_t rtt_of(const uint64_t* lat_ns, uint32_t S, uint32_t su, uint32_t sw) {
    return lat_ns[su * S + sw] + lat_ns[sw * S + su];
}

/* One synchronous heartbeat epoch: A) every peer decides
 * grafts/prunes from the start-of-epoch state; B) every receiver handles
 * incoming GRAFTs in (latency, id) order; C) PRUNEs and rejections are
 * applied, both ends back off. off = offline flags of the epoch (NULL: no
 * churn; §2.8). sub = the subscription epoch 0 (libp2p-gossipsub
 * handle_received_subscriptions, upstream, not vendored; reached through the
 * 20 s event pump of rust-test-node/src/main.rs:357-379): A grafts the first
 * min(D_lo, deg) connections in subscription-arrival order
 * (HS_RTTS*rtt + lat(w->u), id) and B takes GRAFTs in arrival order
 * ((HS_RTTS+1)*rtt, id). Returns the number of GRAFT/PRUNE changes. */
static uint64_t mesh_epoch(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                           uint8_t* flags, const uint8_t* stage, uint32_t S, const uint64_t* lat_ns,
                           mesh_ws* ws, uint32_t epoch, const uint8_t* off, int sub) {
    uint32_t N = p->peers;
    uint64_t nnz = row_ptr[N], changes = 0;
    uint32_t* until = ws->until; uint8_t* prop = ws->prop; uint8_t* acc = ws->acc; const uint64_t* rev = ws->rev;
    const uint32_t bo = (uint32_t)ws->bo;
    const int nt = (int)ws->nt;
    memset(prop, 0, nnz);
    memset(acc, 0, nnz);
    /* ---- 0: links to offline peers leave the mesh (disconnect: no back-off) ---- */
    if (off) {
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 1024)
        for (uint32_t u = 0; u < N; u++)
            for (uint64_t e = row_ptr[u]; e < row_ptr[u + 1]; e++)
                if (off[u] || off[col[e]]) flags[e] &= (uint8_t)~BIT_MESH;
    }
    /* ---- A0: subscription-time grafts (epoch 0 only) ---- */
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 1024)
    for (uint32_t u = 0; u < (sub ? N : 0); u++) {
        sel_t* sel = ws->sel + (size_t)omp_get_thread_num() * ws->sel_n;
        uint64_t b = row_ptr[u], en = row_ptr[u + 1];
        uint32_t nc = 0;
        for (uint64_t e = b; e < en; e++)
            if (!(flags[e] & BIT_MESH)) {
                const uint32_t su = stage[u], sw = stage[col[e]];
                sel[nc].key = HS_RTTS * rtt_of(lat_ns, S, su, sw) + lat_ns[sw * S + su];
                sel[nc].e = e; nc++;
            }
        qsort(sel, nc, sizeof(sel_t), cmp_sel);
        uint32_t want = p->d_lo < nc ? p->d_lo : nc;
        for (uint32_t q = 0; q < want; q++) prop[sel[q].e] |= 1;
    }
    /* ---- A: heartbeat decisions ---- */
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 1024)
    for (uint32_t u = 0; u < (sub ? 0 : N); u++) {
        sel_t* sel = ws->sel + (size_t)omp_get_thread_num() * ws->sel_n;
        if (off && off[u]) continue;
        uint64_t b = row_ptr[u], en = row_ptr[u + 1];
        uint32_t m = 0, o = 0;
        for (uint64_t e = b; e < en; e++) if (flags[e] & BIT_MESH) { m++; if (flags[e] & BIT_OUT) o++; }
        uint32_t mm = m, oo = o;
        if (m < p->d_lo) { /* graft mesh_n - len random eligible peers */
            uint32_t nc = 0;
            for (uint64_t e = b; e < en; e++)
                if (!(flags[e] & BIT_MESH) && epoch > until[e] && !(off && off[col[e]])) {
                    sel[nc].key = or_rng(p->seed, P_GRAFT, u, epoch, col[e]); sel[nc].e = e; nc++;
                }
            qsort(sel, nc, sizeof(sel_t), cmp_sel);
            uint32_t want = p->d - m; if (want > nc) want = nc;
            for (uint32_t q = 0; q < want; q++) {
                prop[sel[q].e] |= 1; mm++; if (flags[sel[q].e] & BIT_OUT) oo++;
            }
        }
        if (mm > p->d_hi) { /* prune down to mesh_n keeping mesh_outbound_min outbound */
            uint32_t nc = 0;
            for (uint64_t e = b; e < en; e++)
                if (flags[e] & BIT_MESH) { sel[nc].key = or_rng(p->seed, P_PRUNE, u, epoch, col[e]); sel[nc].e = e; nc++; }
            qsort(sel, nc, sizeof(sel_t), cmp_sel);
            uint32_t excess = mm - p->d, removed = 0;
            for (uint32_t q = 0; q < nc && removed < excess; q++) {
                uint64_t e = sel[q].e;
                if (flags[e] & BIT_OUT) { if (oo <= p->d_out) continue; oo--; }
                prop[e] |= 2; removed++; mm--;
            }
        }
        if (mm >= p->d_lo && oo < p->d_out) { /* graft outbound peers */
            uint32_t nc = 0;
            for (uint64_t e = b; e < en; e++)
                if ((flags[e] & BIT_OUT) && !(flags[e] & BIT_MESH) && !(prop[e] & 1) && epoch > until[e] &&
                    !(off && off[col[e]])) {
                    sel[nc].key = or_rng(p->seed, P_OUT_GRAFT, u, epoch, col[e]); sel[nc].e = e; nc++;
                }
            qsort(sel, nc, sizeof(sel_t), cmp_sel);
            uint32_t want = p->d_out - oo; if (want > nc) want = nc;
            for (uint32_t q = 0; q < want; q++) { prop[sel[q].e] |= 1; mm++; }
        }
    }
    /* ---- B: receivers handle GRAFTs ---- */
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 1024)
    for (uint32_t w = 0; w < N; w++) {
        sel_t* sel = ws->sel + (size_t)omp_get_thread_num() * ws->sel_n;
        uint64_t b = row_ptr[w], en = row_ptr[w + 1];
        uint32_t c = 0, nin = 0;
        for (uint64_t e = b; e < en; e++)
            if (((flags[e] & BIT_MESH) && !(prop[e] & 2)) || (prop[e] & 1)) c++;
        for (uint64_t e = b; e < en; e++)
            if (prop[rev[e]] & 1) {
                const uint32_t su = stage[col[e]], sw = stage[w];
                sel[nin].key = sub ? (HS_RTTS + 1) * rtt_of(lat_ns, S, su, sw) : lat_ns[su * S + sw];
                sel[nin].e = e; nin++;
            }
        /* order by (arrival, u): stable wrt ascending ids */
        for (uint32_t i = 1; i < nin; i++) {
            sel_t x = sel[i]; int32_t j = (int32_t)i - 1;
            while (j >= 0 && sel[j].key > x.key) { sel[j + 1] = sel[j]; j--; }
            sel[j + 1] = x;
        }
        for (uint32_t q = 0; q < nin; q++) {
            uint64_t e = sel[q].e;               /* entry (w -> u) */
            int in_mesh = ((flags[e] & BIT_MESH) && !(prop[e] & 2)) || (prop[e] & 1);
            if (in_mesh) { acc[rev[e]] = 1; continue; }
            if (epoch < until[e]) { until[e] = epoch + bo; continue; }
            if (c >= p->d_hi && !(flags[e] & BIT_OUT)) { until[e] = epoch + bo; continue; }
            acc[rev[e]] = 1; flags[e] |= BIT_MESH; c++;
        }
    }
    /* ---- C: apply prunes and rejections ---- */
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 1024) reduction(+ : changes)
    for (uint32_t u = 0; u < N; u++) {
        for (uint64_t e = row_ptr[u]; e < row_ptr[u + 1]; e++) {
            uint8_t pr = prop[e];
            if (pr & 1) {
                changes++;
                if (acc[e]) flags[e] |= BIT_MESH;
                else { flags[e] &= (uint8_t)~BIT_MESH; until[e] = epoch + bo; }
            }
            if (pr & 2) { changes++; flags[e] &= (uint8_t)~BIT_MESH; until[e] = epoch + bo; }
            if (prop[rev[e]] & 2) { flags[e] &= (uint8_t)~BIT_MESH; until[e] = epoch + bo; }
        }
    }
    return changes;
}

/* mesh ELL rows (ascending ids, UINT32_MAX padded) from the CSR flags */
static int mesh_extract(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const uint8_t* flags,
                        uint32_t* mesh, uint8_t* cnt) {
    for (uint32_t u = 0; u < p->peers; u++) {
        uint32_t c = 0;
        for (uint64_t e = row_ptr[u]; e < row_ptr[u + 1]; e++)
            if (flags[e] & BIT_MESH) {
                if (c >= MESH_W) return -5;
                mesh[(size_t)u * MESH_W + c++] = col[e];
            }
        cnt[u] = (uint8_t)c;
        for (uint32_t q = c; q < MESH_W; q++) mesh[(size_t)u * MESH_W + q] = UINT32_MAX;
    }
    return 0;
}

int or_mesh_converge(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                     uint8_t* flags, const uint8_t* stage, uint32_t S, const uint64_t* lat_ns,
                     uint32_t max_hb, uint32_t* mesh, uint8_t* cnt, uint32_t* epochs_out) {
    uint32_t N = p->peers;
    mesh_ws ws;
    if (mesh_ws_init(p, row_ptr, col, flags, &ws)) return -2;
    uint8_t* off = p->churn_ppm ? (uint8_t*)malloc(N ? N : 1) : NULL;
    if (p->churn_ppm && !off) { mesh_ws_free(&ws); return -2; }
    uint32_t epoch = 1, last = 0;
    if (p->sub_graft) mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, 0, NULL, 1);
    while (epoch <= max_hb) {
        if (off) { /* churn: no fixed point, every epoch runs */
            for (uint32_t u = 0; u < N; u++) off[u] = (uint8_t)or_offline(p, u, epoch);
            mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, epoch, off, 0);
            last = epoch++;
            continue;
        }
        uint64_t changes = mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, epoch, NULL, 0);
        last = epoch;
        if (changes) { epoch++; continue; }
        /* quiescent: next epoch at which a back-off expiry can wake a peer */
        uint64_t wake = UINT64_MAX;
        for (uint32_t u = 0; u < N; u++) {
            uint64_t b = row_ptr[u], en = row_ptr[u + 1];
            uint32_t m = 0, o = 0;
            for (uint64_t e = b; e < en; e++) if (flags[e] & BIT_MESH) { m++; if (flags[e] & BIT_OUT) o++; }
            int need_any = m < p->d_lo;
            int need_out = !need_any && m <= p->d_hi && o < p->d_out;
            if (!need_any && !need_out) continue;
            for (uint64_t e = b; e < en; e++) {
                if (flags[e] & BIT_MESH) continue;
                if (need_out && !(flags[e] & BIT_OUT)) continue;
                if (ws.until[e] >= epoch + 1 && (uint64_t)ws.until[e] + 1 < wake) wake = (uint64_t)ws.until[e] + 1;
            }
        }
        if (wake == UINT64_MAX || wake > max_hb) break;
        epoch = (uint32_t)wake;
    }
    int rc = mesh_extract(p, row_ptr, col, flags, mesh, cnt);
    *epochs_out = last;
    free(off);
    mesh_ws_free(&ws);
    return rc;
}

/* Mesh snapshots under churn: heartbeats 1..h_hi from the empty mesh; slot
 * h - h_lo holds the mesh after heartbeat h (h = 0: the initial mesh, after
 * the subscription epoch when sub_graft is on)
 * and the offline flags of epoch h, for h in [h_lo, h_hi]. */
int or_mesh_churn(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const uint8_t* flags_in,
                  const uint8_t* stage, uint32_t S, const uint64_t* lat_ns, uint32_t h_lo, uint32_t h_hi,
                  uint32_t* snap_mesh, uint8_t* snap_cnt, uint8_t* snap_off) {
    uint32_t N = p->peers;
    uint64_t nnz = row_ptr[N];
    if (h_hi < h_lo) return -1;
    uint8_t* flags = (uint8_t*)malloc(nnz ? nnz : 1);
    uint8_t* off = (uint8_t*)calloc(N ? N : 1, 1);
    if (!flags || !off) { free(flags); free(off); return -2; }
    memcpy(flags, flags_in, nnz);
    mesh_ws ws;
    if (mesh_ws_init(p, row_ptr, col, flags, &ws)) { free(flags); free(off); return -2; }
    int rc = 0;
    for (uint32_t h = 0; h <= h_hi && !rc; h++) {
        if (h > 0) {
            for (uint32_t u = 0; u < N; u++) off[u] = (uint8_t)or_offline(p, u, h);
            mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, h, off, 0);
        } else if (p->sub_graft) {  /* epoch 0: the subscription exchange, everyone online */
            mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, 0, NULL, 1);
        }
        if (h >= h_lo) {
            size_t o = (size_t)(h - h_lo);
            rc = mesh_extract(p, row_ptr, col, flags, snap_mesh + o * N * MESH_W, snap_cnt + o * N);
            memcpy(snap_off + o * N, off, N);
        }
    }
    mesh_ws_free(&ws);
    free(flags); free(off);
    return rc;
}

/* The same replay as or_mesh_churn, keeping only the epochs h <= h_hi with
 * keep[h] != 0 (in ascending order, slot = rank among the kept), on `threads`
 * OpenMP threads (0/1 = single-threaded; identical results). Test-side helper
 * for sampling messages spread over a long schedule (tests/test_gpu_configs.py). */
int or_mesh_churn_sel(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const uint8_t* flags_in,
                      const uint8_t* stage, uint32_t S, const uint64_t* lat_ns, uint32_t h_hi, const uint8_t* keep,
                      int threads, uint32_t* snap_mesh, uint8_t* snap_cnt, uint8_t* snap_off) {
    uint32_t N = p->peers;
    uint64_t nnz = row_ptr[N];
    const int nt = threads > 1 ? threads : 1;
    uint8_t* flags = (uint8_t*)malloc(nnz ? nnz : 1);
    uint8_t* off = (uint8_t*)calloc(N ? N : 1, 1);
    if (!flags || !off) { free(flags); free(off); return -2; }
    memcpy(flags, flags_in, nnz);
    mesh_ws ws;
    if (mesh_ws_init_nt(p, row_ptr, col, flags, &ws, (uint32_t)nt)) { free(flags); free(off); return -2; }
    int rc = 0;
    size_t o = 0;
    for (uint32_t h = 0; h <= h_hi && !rc; h++) {
        if (h > 0) {
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static, 4096)
            for (uint32_t u = 0; u < N; u++) off[u] = (uint8_t)or_offline(p, u, h);
            mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, h, off, 0);
        } else if (p->sub_graft) {
            mesh_epoch(p, row_ptr, col, flags, stage, S, lat_ns, &ws, 0, NULL, 1);
        }
        if (keep[h]) {
            rc = mesh_extract(p, row_ptr, col, flags, snap_mesh + o * N * MESH_W, snap_cnt + o * N);
            memcpy(snap_off + o * N, off, N);
            o++;
        }
    }
    mesh_ws_free(&ws);
    free(flags); free(off);
    return rc;
}

/* ------------------------------------------------------ dissemination ---- */
/* Events in time order; at equal time arrivals (type 0) precede IHAVE
 * arrivals (type 1), so "w has seen m by t" reads w's finality at the IHAVE. */
typedef struct { uint64_t t; uint64_t key; uint32_t dst; uint32_t frag; uint32_t type; } ev_t;
typedef struct { ev_t* a; size_t n, cap; } heap_t;

static int ev_less(const ev_t* x, const ev_t* y) {
    if (x->t != y->t) return x->t < y->t;
    if (x->type != y->type) return x->type < y->type;
    if (x->key != y->key) return x->key < y->key;
    if (x->dst != y->dst) return x->dst < y->dst;
    return x->frag < y->frag;
}
static int heap_push(heap_t* h, ev_t v) {
    if (h->n == h->cap) {
        size_t nc = h->cap ? h->cap * 2 : 1024;
        ev_t* na = (ev_t*)realloc(h->a, nc * sizeof(ev_t));
        if (!na) return -2;
        h->a = na; h->cap = nc;
    }
    size_t i = h->n++;
    while (i > 0) {
        size_t pa = (i - 1) / 2;
        if (!ev_less(&v, &h->a[pa])) break;
        h->a[i] = h->a[pa]; i = pa;
    }
    h->a[i] = v;
    return 0;
}
static ev_t heap_pop(heap_t* h) {
    ev_t top = h->a[0], last = h->a[--h->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, s = i;
        const ev_t* cur = &last;
        if (l < h->n && ev_less(&h->a[l], cur)) { s = l; cur = &h->a[l]; }
        if (r < h->n && ev_less(&h->a[r], cur)) { s = r; }
        if (s == i) break;
        h->a[i] = h->a[s]; i = s;
    }
    if (h->n) h->a[i] = last;
    return top;
}

static uint32_t bits_for(uint32_t n) { uint32_t b = 1; while ((1ull << b) < n) b++; return b; }

enum { P_GOSSIP = 6 };

/* Where a send reads the mesh: the frozen converged mesh, or under churn the
 * snapshot of the heartbeat epoch the send falls in. */
typedef struct {
    const uint32_t* mesh; const uint8_t* cnt;                               /* frozen */
    const uint32_t* snap_mesh; const uint8_t* snap_cnt; const uint8_t* snap_off; /* churn */
    uint64_t h_lo, n_snap;
    uint64_t h_cap;  /* last epoch the current message may use: epoch(t_pub) + churn_horizon */
} mesh_src;

/* heartbeat epoch containing absolute time tabs: heartbeats at hb_phase + h*hb */
static uint64_t epoch_at(const or_params* p, uint64_t tabs) {
    return tabs < p->hb_phase_ns ? 0 : (tabs - p->hb_phase_ns) / p->heartbeat_ns;
}
/* snapshot slot of epoch h; -1 past the message's lifetime h_cap (its event is
 * not made / not delivered) or outside the snapshots */
static int64_t slot_of(const mesh_src* ms, uint64_t h) {
    if (!ms->snap_mesh) return 0;
    return (h < ms->h_lo || h - ms->h_lo >= ms->n_snap || h > ms->h_cap) ? -1 : (int64_t)(h - ms->h_lo);
}
static const uint32_t* mesh_row(const mesh_src* ms, uint32_t N, int64_t slot, uint32_t u, uint32_t* cnt) {
    if (!ms->snap_mesh) { *cnt = ms->cnt[u]; return ms->mesh + (size_t)u * MESH_W; }
    *cnt = ms->snap_cnt[(size_t)slot * N + u];
    return ms->snap_mesh + ((size_t)slot * N + u) * MESH_W;
}
static int offline_at(const mesh_src* ms, uint32_t N, int64_t slot, uint32_t u) {
    return ms->snap_off ? ms->snap_off[(size_t)slot * N + u] : 0;
}

/* Lazy-gossip targets of peer v at heartbeat h (libp2p-gossipsub emit_gossip,
 * upstream, not vendored; gossip_lazy/gossip_factor at main.rs:230,235):
 * r = max(D_lazy, floor(factor*|non-mesh|)) non-mesh peers, capped at
 * |non-mesh|, the r smallest rng(GOSSIP, v, h, w) (ties by id). Under churn
 * the mesh is the epoch-h snapshot and offline peers are not candidates. */
static uint32_t gossip_targets(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                               const mesh_src* ms, int64_t slot, uint32_t v, uint64_t h,
                               sel_t* sel, uint32_t* out) {
    uint32_t N = p->peers, mc;
    const uint32_t* mr = mesh_row(ms, N, slot, v, &mc);
    uint32_t nc = 0;
    for (uint64_t e = row_ptr[v]; e < row_ptr[v + 1]; e++) {
        uint32_t w = col[e], in = 0;
        for (uint32_t q = 0; q < mc; q++) in |= mr[q] == w;
        if (in || offline_at(ms, N, slot, w)) continue;
        sel[nc].key = or_rng(p->seed, P_GOSSIP, v, (uint32_t)h, w);
        sel[nc].e = w;
        nc++;
    }
    qsort(sel, nc, sizeof(sel_t), cmp_sel);
    uint32_t r = (uint32_t)(((uint64_t)nc * p->gossip_factor_milli) / 1000);
    if (r < p->d_lazy) r = p->d_lazy;
    if (r > nc) r = nc;
    for (uint32_t q = 0; q < r; q++) out[q] = (uint32_t)sel[q].e;
    return r;
}

/* Per-peer traffic (gs_set_traffic; columns = the ABI's GS_TR_*): a send adds
 * its bytes / packets / header bytes to the sender's tx; a send that arrives
 * adds them to the receiver's rx, and the receiver answers every 2 packets
 * with a pure ACK (delayed ACK, one per <= 2 segments; a model constant), which
 * lands in its tx ctrl and the sender's rx ctrl columns. Lost sends (churn)
 * are not retransmitted: the connection is gone. */
typedef struct {
    uint64_t* tr;
    uint64_t w, pk, hd;          /* one data fragment send (or_wire_bytes / or_wire_packets) */
    uint64_t ihw, ihpk, ihhd;    /* one IHAVE RPC */
    uint64_t iww, iwpk, iwhd;    /* one IWANT RPC */
    uint64_t ack;                /* header bytes of one ACK packet */
} tr_t;
enum { TRC_TXB = 0, TRC_RXB = 1, TRC_TXP = 2, TRC_RXP = 3, TRC_TXH = 4, TRC_RXH = 5, TRC_RCV = 6, TRC_PUB = 7,
       TRC_TXCP = 8, TRC_RXCP = 9, TRC_TXCH = 10, TRC_RXCH = 11 };
static void tr_send(const tr_t* T, uint32_t x, uint64_t b, uint64_t pk, uint64_t hd) {
    uint64_t* r = T->tr + (size_t)x * OR_TR_COLS;
    r[TRC_TXB] += b; r[TRC_TXP] += pk; r[TRC_TXH] += hd;
}
static void tr_deliver(const tr_t* T, uint32_t s, uint32_t x, uint64_t b, uint64_t pk, uint64_t hd) {
    uint64_t* r = T->tr + (size_t)x * OR_TR_COLS;
    uint64_t* q = T->tr + (size_t)s * OR_TR_COLS;
    const uint64_t acks = (pk + 1) / 2;
    r[TRC_RXB] += b; r[TRC_RXP] += pk; r[TRC_RXH] += hd;
    r[TRC_TXCP] += acks; r[TRC_TXCH] += acks * T->ack;
    q[TRC_RXCP] += acks; q[TRC_RXCH] += acks * T->ack;
}

/* Events in time order; at equal time arrivals (type 0) precede IHAVE
 * arrivals (types 1, 2), so "w has seen m by t" reads w's finality at the
 * IHAVE. Type 2 = an IHAVE whose answer will be lost (churn; traffic only). */

/* Lazy gossip of (v, f) first received at t_v (relative to t_pub): IHAVE at
 * the history_gossip heartbeats T >= t_v to gossip_targets(v, h); the IHAVE
 * reaches w at T + lat(v,w); an IWANT comes back and v's answer lands at
 * T + 2 lat(v,w) + lat(w,v) + ser_up(v) + dn. Under churn v
 * gossips only while online, and an IHAVE or answer reaching an offline w is
 * lost (§2.8). With traffic (tm) the IHAVE sends are counted here. */
static int sched_gossip(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const mesh_src* ms,
                        const uint8_t* stage, uint32_t S, const uint64_t* lat_ns, const uint64_t* su,
                        const uint64_t* sd, uint64_t t_pub, uint32_t v, uint32_t f, uint64_t tv, uint64_t hp,
                        uint32_t tshift, uint32_t sb, uint64_t tmax, sel_t* gsel, uint32_t* gtg, heap_t* h,
                        const tr_t* tm) {
    const uint32_t N = p->peers;
    const uint64_t hmask = (1ull << HOP_BITS) - 1;
    const uint64_t tabs = t_pub + tv;
    uint64_t h0 = tabs <= p->hb_phase_ns ? 0 : (tabs - p->hb_phase_ns + p->heartbeat_ns - 1) / p->heartbeat_ns;
    const uint32_t sv = stage[v];
    for (uint32_t k = 0; k < p->history_gossip; k++) {
        const uint64_t hh = h0 + k;
        const uint64_t T = p->hb_phase_ns + hh * p->heartbeat_ns - t_pub;
        const int64_t sl = slot_of(ms, hh);
        if (sl < 0 || offline_at(ms, N, sl, v)) continue;  /* expired, or v is offline */
        const uint32_t r = gossip_targets(p, row_ptr, col, ms, sl, v, hh, gsel, gtg);
        if (r && hp + 1 > hmask) return -5;
        for (uint32_t q = 0; q < r; q++) {
            const uint32_t w = gtg[q], sw = stage[w];
            const uint64_t ti = T + lat_ns[sv * S + sw];
            const uint64_t dn = sd[sw] > su[sv] ? sd[sw] - su[sv] : 0;
            const uint64_t A = ti + lat_ns[sw * S + sv] + su[sv] + lat_ns[sv * S + sw] + dn;
            if (A > tmax) return -5;
            int lost_i = 0, lost_a = 0;
            if (ms->snap_off) {
                const int64_t si = slot_of(ms, epoch_at(p, t_pub + ti)), sa = slot_of(ms, epoch_at(p, t_pub + A));
                lost_i = si < 0 || offline_at(ms, N, si, w);
                lost_a = sa < 0 || offline_at(ms, N, sa, w);
            }
            if (tm) {
                tr_send(tm, v, tm->ihw, tm->ihpk, tm->ihhd);
                if (!lost_i) tr_deliver(tm, v, w, tm->ihw, tm->ihpk, tm->ihhd);
            }
            if (lost_i || (lost_a && !tm)) continue;
            ev_t ge = {ti, (A << tshift) | ((hp + 1) << sb) | v, w, f, lost_a ? 2u : 1u};
            if (heap_push(h, ge)) return -2;
        }
    }
    return 0;
}

/* Fragment layout per node flavour: the data field's size,
 * whether the node's own publish code fails (the run is rejected), and whether
 * all fragments are byte-identical (one msg-id, defect D8).
 *  rust publish_new_message (main.rs:109-121): msg_size/F bytes, i64 stamp in
 *    [0..8) (panics below 8 B), byte 10 = chunk only if the buffer is longer
 *    than 10 B;
 *  go publishNewMessage (go-test-node/main.go:63-74): 8-byte stamp + msg_size/F
 *    zero bytes, payload[10] = chunk (index out of range when msg_size/F <= 2);
 *  nim publishNewMessage (nim-test-node/gossipsub-queues/main.nim:158-175):
 *    16-byte header (stamp, random msgId) + msg_size div F - 16 bytes,
 *    nowBytes[16] = chunk (IndexDefect when msg_size div F <= 16). */
static uint64_t frag_payload(const or_params* p, uint64_t msg_size, uint32_t F) {
    return msg_size / F + (p->node == 1 ? 8 : 0);
}
static int frag_invalid(const or_params* p, uint64_t msg_size, uint32_t F) {
    uint64_t q = msg_size / F;
    return p->node == 1 ? q <= 2 : p->node == 2 ? q <= 16 : q < 8;
}
static int frag_collide(const or_params* p, uint64_t msg_size, uint32_t F) {
    return p->node == 0 && F > 1 && msg_size / F <= 10;
}
#define MAX_F 16u

/* One publish -> receive -> forward -> reassemble pass per message:
 *  publish_new_message (main.rs:101-143): F fragments (layout above),
 *    flood-published (main.rs:227) to every connection in ascending id,
 *    fragment after fragment, through the publisher's uplink FIFO.
 *  first receipt of (peer, fragment) wins by key (time, hops, src); it is
 *    forwarded to mesh \ {src, publisher} in ascending id through the peer's
 *    uplink FIFO (busy carried across that message's fragments).
 *  create_message_handler (main.rs:79-99): completion = arrival of the F-th
 *    distinct fragment; latency ms = (t_complete - tx_time)/1e6 truncated.
 *  churn: a publisher offline at t_pub publishes nothing;
 *    the flood goes to the connections online at t_pub; a forward uses the
 *    mesh snapshot of the epoch it is sent in; a delivery to a peer offline
 *    at its arrival is lost (the send still occupies the uplink); nothing
 *    happens past epoch(t_pub) + churn_horizon (the message's lifetime). */
static int run_impl(const or_params* p, const uint64_t* row_ptr, const uint32_t* col, const mesh_src* ms0,
                    const uint8_t* stage, uint32_t S, const uint64_t* lat_ns, const uint64_t* bw_up,
                    const uint64_t* bw_dn, const uint64_t* sched_t, const uint32_t* sched_pub,
                    const uint32_t* sched_size, const uint32_t* sched_frags, uint64_t n_msgs,
                    uint64_t* t_complete, uint8_t* hops, or_stats* st, uint64_t* tr) {
    uint32_t N = p->peers, F = p->fragments;  /* per message: its chunk count (rows of F slots) */
    if (p->fragments == 0 || p->fragments > MAX_F) return -6;
    uint32_t sb = bits_for(N), tshift = sb + HOP_BITS;
    uint64_t tmax = (tshift >= 64) ? 0 : (UINT64_MAX >> tshift);
    uint64_t hmask = (1ull << HOP_BITS) - 1, smask = (1ull << sb) - 1;
    size_t NF = (size_t)N * MAX_F;
    uint32_t maxdeg = 0;
    for (uint32_t u = 0; u < N; u++)
        if (row_ptr[u + 1] - row_ptr[u] > maxdeg) maxdeg = (uint32_t)(row_ptr[u + 1] - row_ptr[u]);
    uint64_t* best = (uint64_t*)malloc(sizeof(uint64_t) * NF);
    uint8_t* fin = (uint8_t*)malloc(NF);
    uint64_t* busy = (uint64_t*)malloc(sizeof(uint64_t) * N);
    uint64_t *su = (uint64_t*)malloc(8 * S), *sd = (uint64_t*)malloc(8 * S);
    sel_t* gsel = (sel_t*)malloc(sizeof(sel_t) * (maxdeg + 1));
    uint32_t* gtg = (uint32_t*)malloc(sizeof(uint32_t) * (maxdeg + 1));
    uint32_t* ftg = (uint32_t*)malloc(sizeof(uint32_t) * (maxdeg + 1));
    heap_t h = {0, 0, 0};
    int rc = 0;
    if (!best || !fin || !busy || !su || !sd || !gsel || !gtg || !ftg) { rc = -2; goto out; }
    for (uint64_t mi = 0; mi < n_msgs; mi++) {
        uint32_t pub = sched_pub[mi];
        /* chunks of this PublishCommand (main.rs:65-71,163-168); 0 = FRAGMENTS */
        const uint32_t Fm = (sched_frags && sched_frags[mi]) ? sched_frags[mi] : p->fragments;
        if (Fm > MAX_F) { rc = -1; goto out; }
        uint64_t payload = frag_payload(p, sched_size[mi], Fm);
        if (pub >= N || frag_invalid(p, sched_size[mi], Fm)) { rc = -1; goto out; } /* the node's publish fails */
        int collide = frag_collide(p, sched_size[mi], Fm);                      /* defect D8 */
        uint32_t Fe = collide ? 1 : Fm;
        F = Fm;
        NF = (size_t)N * F;
        uint64_t wire = or_wire_bytes(payload, p->muxer, p->signed_msgs);
        tr_t trm = {tr, wire, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        or_wire_packets(payload, p->muxer, p->signed_msgs, &trm.pk, &trm.hd);
        or_ctrl_packets(0, p->node, p->muxer, &trm.ihw, &trm.ihpk, &trm.ihhd);
        or_ctrl_packets(1, p->node, p->muxer, &trm.iww, &trm.iwpk, &trm.iwhd);
        { uint64_t x, y; or_ctrl_packets(2, p->node, p->muxer, &trm.ack, &x, &y); }
        const tr_t* T = tr ? &trm : NULL;
        const uint64_t tp = sched_t[mi];
        mesh_src msg_ms = *ms0;
        msg_ms.h_cap = epoch_at(p, tp) + p->churn_horizon;
        const mesh_src* ms = &msg_ms;
        for (uint32_t s = 0; s < S; s++) {
            su[s] = (wire * 8000000000ULL + bw_up[s] - 1) / bw_up[s];
            sd[s] = (wire * 8000000000ULL + bw_dn[s] - 1) / bw_dn[s];
        }
        for (size_t i = 0; i < NF; i++) { best[i] = INF64; fin[i] = 0; }
        for (uint32_t u = 0; u < N; u++) busy[u] = 0;
        h.n = 0;
        st->messages++;
        const int64_t sp0 = slot_of(ms, epoch_at(p, tp));
        if (sp0 < 0) { rc = -7; goto out; }
        if (offline_at(ms, N, sp0, pub)) { /* the injector's POST finds no node: nothing is published */
            for (uint32_t u = 0; u < N; u++) { t_complete[(size_t)mi * N + u] = INF64; hops[(size_t)mi * N + u] = 0xFF; }
            continue;
        }
        /* publisher: self key, flood through the uplink FIFO */
        if (tr) tr[(size_t)pub * OR_TR_COLS + TRC_PUB] += 1; /* published (main.rs:515) */
        uint32_t sp = stage[pub];
        for (uint32_t f = 0; f < Fe; f++) { best[(size_t)pub * F + f] = (uint64_t)pub; fin[(size_t)pub * F + f] = 1; }
        if (p->lazy_gossip)
            for (uint32_t f = 0; f < Fe; f++)
                if ((rc = sched_gossip(p, row_ptr, col, ms, stage, S, lat_ns, su, sd, tp, pub, f, 0, 0, tshift, sb,
                                       tmax, gsel, gtg, &h, T)))
                    goto out;
        uint32_t deg = 0;
        if (p->flood_publish) {
            for (uint64_t e = row_ptr[pub]; e < row_ptr[pub + 1]; e++)
                if (!offline_at(ms, N, sp0, col[e])) ftg[deg++] = col[e];
        } else {
            uint32_t mc;
            const uint32_t* mr = mesh_row(ms, N, sp0, pub, &mc);
            for (uint32_t q = 0; q < mc; q++) ftg[deg++] = mr[q];
        }
        for (uint32_t f = 0; f < Fe; f++)
            for (uint32_t j = 0; j < deg; j++) {
                uint32_t w = ftg[j], sw = stage[w];
                uint64_t dn = sd[sw] > su[sp] ? sd[sw] - su[sp] : 0;
                uint64_t arr = ((uint64_t)f * deg + j + 1) * su[sp] + lat_ns[sp * S + sw] + dn;
                if (arr > tmax) { rc = -5; goto out; }
                uint64_t key = (arr << tshift) | (1ull << sb) | pub;
                st->relaxations++;
                if (T) tr_send(T, pub, wire, T->pk, T->hd);
                if (ms->snap_off) {  /* lost: past the lifetime, or w offline at the arrival */
                    const int64_t sl = slot_of(ms, epoch_at(p, tp + arr));
                    if (sl < 0 || offline_at(ms, N, sl, w)) continue;
                }
                if (T) tr_deliver(T, pub, w, wire, T->pk, T->hd);
                if (key < best[(size_t)w * F + f]) best[(size_t)w * F + f] = key;
                ev_t ev = {arr, key, w, f, 0};
                if (heap_push(&h, ev)) { rc = -2; goto out; }
            }
        while (h.n) {
            ev_t ev = heap_pop(&h);
            size_t idx = (size_t)ev.dst * F + ev.frag;
            if (ev.type != 0) { /* IHAVE arrives at w: IWANT unless w already has it */
                if (fin[idx]) continue;
                const uint32_t v = (uint32_t)(ev.key & smask);
                if (T) { /* w's IWANT to v, v's answer to w (lost with type 2) */
                    tr_send(T, ev.dst, T->iww, T->iwpk, T->iwhd);
                    tr_deliver(T, ev.dst, v, T->iww, T->iwpk, T->iwhd);
                    tr_send(T, v, wire, T->pk, T->hd);
                    if (ev.type == 1) tr_deliver(T, v, ev.dst, wire, T->pk, T->hd);
                }
                if (ev.type == 2) continue;
                st->gossip_iwant++;
                st->relaxations++;
                if (ev.key < best[idx]) {
                    best[idx] = ev.key;
                    ev_t ne = {ev.key >> tshift, ev.key, ev.dst, ev.frag, 0};
                    if (heap_push(&h, ne)) { rc = -2; goto out; }
                }
                continue;
            }
            if (fin[idx]) continue;
            fin[idx] = 1;
            uint32_t u = ev.dst, su_ = stage[u];
            uint64_t t = ev.key >> tshift;
            uint64_t hp = (ev.key >> sb) & hmask;
            uint32_t src = (uint32_t)(ev.key & smask);
            st->frag_deliveries++;
            const int64_t sl = slot_of(ms, epoch_at(p, tp + t));
            if (sl < 0) continue;  /* received past the message's lifetime: delivered, not forwarded */
            uint32_t mc;
            const uint32_t* mr = mesh_row(ms, N, sl, u, &mc);
            uint32_t tg[MESH_W], n = 0;
            for (uint32_t q = 0; q < mc; q++) {
                uint32_t w = mr[q];
                if (w == src || w == pub) continue;
                if (p->idontwant && payload >= p->idontwant) {
                    uint64_t bw_ = best[(size_t)w * F + ev.frag];
                    if (bw_ != INF64 && (bw_ >> tshift) + lat_ns[stage[w] * S + su_] <= t) continue;
                }
                tg[n++] = w;
            }
            if (p->lazy_gossip &&
                (rc = sched_gossip(p, row_ptr, col, ms, stage, S, lat_ns, su, sd, tp, u, ev.frag, t, hp, tshift, sb,
                                   tmax, gsel, gtg, &h, T)))
                goto out;
            uint64_t start = (Fe > 1 && busy[u] > t) ? busy[u] : t;
            busy[u] = start + (uint64_t)n * su[su_];
            if (n && hp + 1 > hmask) { rc = -5; goto out; }
            for (uint32_t j = 0; j < n; j++) {
                uint32_t w = tg[j], sw = stage[w];
                uint64_t dn = sd[sw] > su[su_] ? sd[sw] - su[su_] : 0;
                uint64_t arr = start + (uint64_t)(j + 1) * su[su_] + lat_ns[su_ * S + sw] + dn;
                if (arr > tmax) { rc = -5; goto out; }
                uint64_t key = (arr << tshift) | ((hp + 1) << sb) | u;
                st->relaxations++;
                if (T) tr_send(T, u, wire, T->pk, T->hd);
                if (ms->snap_off) {
                    const int64_t sa = slot_of(ms, epoch_at(p, tp + arr));
                    if (sa < 0 || offline_at(ms, N, sa, w)) continue;
                }
                if (T) tr_deliver(T, u, w, wire, T->pk, T->hd);
                size_t wi = (size_t)w * F + ev.frag;
                if (key < best[wi]) {
                    best[wi] = key;
                    ev_t ne = {arr, key, w, ev.frag, 0};
                    if (heap_push(&h, ne)) { rc = -2; goto out; }
                }
            }
        }
        /* reassembly: F-th distinct fragment completes the message */
        for (uint32_t u = 0; u < N; u++) {
            size_t o = (size_t)mi * N + u;
            if (u == pub) { t_complete[o] = tp; hops[o] = 0; continue; }
            uint64_t mk = 0; int ok = !collide;
            for (uint32_t f = 0; f < Fm && ok; f++) {
                uint64_t k = best[(size_t)u * F + f];
                if (k == INF64) ok = 0; else if (k > mk) mk = k;
            }
            if (!ok) { t_complete[o] = INF64; hops[o] = 0xFF; continue; }
            uint64_t trel = mk >> tshift;
            t_complete[o] = tp + trel;
            hops[o] = (uint8_t)((mk >> sb) & hmask);
            uint64_t ms_ = trel / 1000000ULL;
            st->deliveries++;
            if (tr) tr[(size_t)u * OR_TR_COLS + TRC_RCV] += 1; /* received (main.rs:94) */
            st->latency_sum_ms += ms_;
            if (ms_ > st->latency_max_ms) st->latency_max_ms = ms_;
        }
    }
out:
    st->bytes_alg = 16 * st->frag_deliveries + 12 * st->relaxations + 8 * st->deliveries;
    free(best); free(fin); free(busy); free(su); free(sd); free(gsel); free(gtg); free(ftg); free(h.a);
    return rc;
}

int or_run(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
           const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
           const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
           const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
           const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, or_stats* st) {
    mesh_src ms = {mesh, cnt, NULL, NULL, NULL, 0, 0, 0};
    return run_impl(p, row_ptr, col, &ms, stage, S, lat_ns, bw_up, bw_dn, sched_t, sched_pub, sched_size,
                    sched_frags, n_msgs, t_complete, hops, st, NULL);
}

int or_run_churn(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                 const uint32_t* snap_mesh, const uint8_t* snap_cnt, const uint8_t* snap_off,
                 uint32_t h_lo, uint32_t n_snap, const uint8_t* stage, uint32_t S,
                 const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                 const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                 const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops,
                 or_stats* st) {
    mesh_src ms = {NULL, NULL, snap_mesh, snap_cnt, snap_off, h_lo, n_snap, 0};
    return run_impl(p, row_ptr, col, &ms, stage, S, lat_ns, bw_up, bw_dn, sched_t, sched_pub, sched_size,
                    sched_frags, n_msgs, t_complete, hops, st, NULL);
}

/* or_run plus per-peer traffic tr[N][OR_TR_COLS] (tx bytes, rx bytes, tx
 * packets, rx packets, tx header bytes, rx header bytes, completed messages,
 * published messages, tx / rx ACK packets, tx / rx ACK header bytes; see
 * tr_t), accumulated (caller zeroes). */
int or_run_traffic(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                   const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
                   const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                   const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                   const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops,
                   or_stats* st, uint64_t* tr) {
    mesh_src ms = {mesh, cnt, NULL, NULL, NULL, 0, 0, 0};
    return run_impl(p, row_ptr, col, &ms, stage, S, lat_ns, bw_up, bw_dn, sched_t, sched_pub, sched_size,
                    sched_frags, n_msgs, t_complete, hops, st, tr);
}

/* or_run_churn plus the per-peer traffic of or_run_traffic. */
int or_run_churn_traffic(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
                         const uint32_t* snap_mesh, const uint8_t* snap_cnt, const uint8_t* snap_off,
                         uint32_t h_lo, uint32_t n_snap, const uint8_t* stage, uint32_t S,
                         const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
                         const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
                         const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops,
                         or_stats* st, uint64_t* tr) {
    mesh_src ms = {NULL, NULL, snap_mesh, snap_cnt, snap_off, h_lo, n_snap, 0};
    return run_impl(p, row_ptr, col, &ms, stage, S, lat_ns, bw_up, bw_dn, sched_t, sched_pub, sched_size,
                    sched_frags, n_msgs, t_complete, hops, st, tr);
}

/* or_run message-parallel on `threads` host threads (OpenMP): messages are
 * independent given the frozen mesh, so each thread runs the
 * same single-message event simulation on its own messages. Used only as the
 * all-core CPU baseline of bench.py. */
int or_run_mt(const or_params* p, const uint64_t* row_ptr, const uint32_t* col,
              const uint32_t* mesh, const uint8_t* cnt, const uint8_t* stage, uint32_t S,
              const uint64_t* lat_ns, const uint64_t* bw_up, const uint64_t* bw_dn,
              const uint64_t* sched_t, const uint32_t* sched_pub, const uint32_t* sched_size,
              const uint32_t* sched_frags, uint64_t n_msgs, uint64_t* t_complete, uint8_t* hops, or_stats* st,
              int threads) {
    or_stats* ps = (or_stats*)calloc(n_msgs ? n_msgs : 1, sizeof(or_stats));
    if (!ps) return -2;
    const mesh_src ms = {mesh, cnt, NULL, NULL, NULL, 0, 0, 0};
    const size_t N = p->peers;
    int rc = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
    for (int64_t m = 0; m < (int64_t)n_msgs; m++) {
        int r = run_impl(p, row_ptr, col, &ms, stage, S, lat_ns, bw_up, bw_dn, sched_t + m, sched_pub + m,
                         sched_size + m, sched_frags ? sched_frags + m : NULL, 1, t_complete + (size_t)m * N,
                         hops + (size_t)m * N, &ps[m], NULL);
        if (r) {
#pragma omp critical
            rc = r;
        }
    }
    for (uint64_t m = 0; m < n_msgs; m++) {
        st->messages += ps[m].messages; st->deliveries += ps[m].deliveries;
        st->frag_deliveries += ps[m].frag_deliveries; st->relaxations += ps[m].relaxations;
        st->latency_sum_ms += ps[m].latency_sum_ms; st->gossip_iwant += ps[m].gossip_iwant;
        if (ps[m].latency_max_ms > st->latency_max_ms) st->latency_max_ms = ps[m].latency_max_ms;
    }
    st->bytes_alg = 16 * st->frag_deliveries + 12 * st->relaxations + 8 * st->deliveries;
    free(ps);
    return rc;
}
