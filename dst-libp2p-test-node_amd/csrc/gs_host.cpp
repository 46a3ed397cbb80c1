// gs_host.cpp — host-only entry points of the C ABI (no device work):
// config defaults and the env surface, wire-byte model, topogen link tables,
// run.sh publish schedule and the awk-compatible arrival-log writer.
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <new>
#include <string>
#include <vector>

#include "../../include/gossipsim.h"
#include "gs_common.h"

extern "C" void gs_config_default(gs_config* c) {
  memset(c, 0, sizeof(*c));
  c->abi_version = GS_ABI_VERSION;
  c->peers = 100;                 // env.rs:38-41
  c->connect_to = 10;             // env.rs:43-46
  c->dial_extra = 1;              // main.rs:337 (defect D4)
  c->max_connections = 0;         // rust has no cap
  c->fragments = 1;               // env.rs:64-67
  c->muxer = GS_MUX_YAMUX;        // env.rs:48-50
  c->signed_msgs = 1;             // main.rs:397
  c->d = 6; c->d_lo = 4; c->d_hi = 8;           // main.rs:36-38
  c->d_lazy = 6;                  // main.rs:235
  c->d_out = 3;                   // main.rs:234
  c->gossip_factor_milli = 250;   // main.rs:230
  c->heartbeat_ns = 1000000000ull;       // main.rs:228
  c->backoff_ns = 60000000000ull;        // main.rs:229
  c->flood_publish = 1;           // main.rs:227
  c->idontwant = 0;
  c->lazy_gossip = 1;             // gossip_lazy(6) + gossip_factor(0.25): rust always gossips (main.rs:230,235)
  c->self_log = 0;                // rust: no self delivery
  c->seed = 1;
  c->device = 0;
  c->batch = 1024;
  c->history_gossip = 3;          // libp2p-gossipsub default (not overridden, main.rs:223-241)
  c->hb_phase_ns = 0;
  c->churn_ppm = 0;               // frozen mesh (the reference has no churn)
  c->churn_down = 10;             // rejoin after 10 epochs
  c->churn_horizon = 16;
  c->node = GS_NODE_RUST;
  c->sub_graft = 1;               // handle_received_subscriptions grafts during the 20 s pump (main.rs:357-379)
  c->hs_rtts = gs::HS_RTTS;       // model constant (sensitivity table §3)
}

extern "C" gs_status gs_config_preset(gs_config* c, uint32_t node) {
  if (!c || node > GS_NODE_NIM) return GS_EINVAL;
  gs_config_default(c);
  c->node = node;
  if (node == GS_NODE_GO) {       // go-test-node/main.go:153-175,374-385
    c->d_out = 2;                 // gsParams.Dout = 2 (main.go:160)
    c->idontwant = 1000;          // IDontWantMessageThreshold = 1000 (main.go:165)
    c->signed_msgs = 0;           // WithMessageSignaturePolicy(StrictNoSign) (main.go:383)
    c->self_log = 1;              // the node's own subscription delivers its publish (readLoop, main.go:52-60)
    c->sub_graft = 0;             // go-libp2p-pubsub grafts from the heartbeat only (upstream, not vendored)
  } else if (node == GS_NODE_NIM) {  // nim-test-node/gossipsub-queues/main.nim
    c->dial_extra = 0;            // dials CONNECTTO peers (main.nim:396)
    c->max_connections = 250;     // withMaxConnections(MAXCONNECTIONS, default 250) (main.nim:429)
    c->d_out = c->d / 2;          // GOSSIPSUB_D_OUT default d div 2 (main.nim:258)
    c->d_lazy = c->d;             // GOSSIPSUB_D_LAZY default d (main.nim:259)
    c->signed_msgs = 0;           // initializeGossipsub(switch, anonymize = true) (main.nim:447)
    c->self_log = 1;              // triggerSelf = SELFTRIGGER, default true (main.nim:245)
    c->sub_graft = 0;             // nim-libp2p rebalances the mesh in its heartbeat (upstream, not vendored)
  }
  return GS_OK;
}

namespace {

bool env_u64(const char* name, uint64_t* out, char* err, size_t n, bool* bad) {
  const char* v = getenv(name);
  if (!v || !*v) return false;
  char* end = nullptr;
  errno = 0;
  unsigned long long x = strtoull(v, &end, 10);
  if (errno || *end) {  // rust's parse().unwrap_or(default) keeps the default
    (void)err; (void)n; (void)bad;
    return false;
  }
  *out = x;
  return true;
}

bool env_bool(const char* name, uint32_t* out) {
  const char* v = getenv(name);
  if (!v || !*v) return false;
  if (!strcasecmp(v, "true") || !strcmp(v, "1")) { *out = 1; return true; }
  if (!strcasecmp(v, "false") || !strcmp(v, "0")) { *out = 0; return true; }
  return false;
}

void set_err(char* err, size_t n, const std::string& s) {
  if (err && n) { snprintf(err, n, "%s", s.c_str()); }
}

}  // namespace

// Mirrors get_peer_details (rust-test-node/src/env.rs:27-87) plus the nim
// GOSSIPSUB_* names (nim-test-node/gossipsub-queues/main.nim:252-284).
extern "C" gs_status gs_config_from_env(gs_config* c, char* err, size_t err_len) {
  if (!c) return GS_EINVAL;
  bool bad = false;
  uint64_t x;
  const char* nd = getenv("GS_NODE");  // which test node's defaults (rust | go | nim)
  if (nd && *nd) {
    const uint32_t keep_dev = (uint32_t)c->device, keep_batch = c->batch;
    if (!strcasecmp(nd, "rust")) gs_config_preset(c, GS_NODE_RUST);
    else if (!strcasecmp(nd, "go")) gs_config_preset(c, GS_NODE_GO);
    else if (!strcasecmp(nd, "nim")) gs_config_preset(c, GS_NODE_NIM);
    else { set_err(err, err_len, std::string("Unknown node type: ") + nd); return GS_EINVAL; }
    c->device = (int32_t)keep_dev;
    c->batch = keep_batch;
  }
  if (env_u64("PEERS", &x, err, err_len, &bad)) c->peers = (uint32_t)x;
  if (env_u64("CONNECTTO", &x, err, err_len, &bad)) c->connect_to = (uint32_t)x;
  if (env_u64("FRAGMENTS", &x, err, err_len, &bad)) c->fragments = (uint32_t)x;
  if (env_u64("MAXCONNECTIONS", &x, err, err_len, &bad)) c->max_connections = (uint32_t)x;
  if (env_u64("GOSSIPSUB_D", &x, err, err_len, &bad)) c->d = (uint32_t)x;
  if (env_u64("GOSSIPSUB_D_LOW", &x, err, err_len, &bad)) c->d_lo = (uint32_t)x;
  if (env_u64("GOSSIPSUB_D_HIGH", &x, err, err_len, &bad)) c->d_hi = (uint32_t)x;
  if (env_u64("GOSSIPSUB_D_LAZY", &x, err, err_len, &bad)) c->d_lazy = (uint32_t)x;
  if (env_u64("GOSSIPSUB_D_OUT", &x, err, err_len, &bad)) c->d_out = (uint32_t)x;
  if (env_u64("GOSSIPSUB_HEARTBEAT_MS", &x, err, err_len, &bad)) c->heartbeat_ns = x * 1000000ull;
  if (env_u64("GOSSIPSUB_PRUNE_BACKOFF_SEC", &x, err, err_len, &bad)) c->backoff_ns = x * 1000000000ull;
  if (env_u64("GS_SEED", &x, err, err_len, &bad)) c->seed = x;
  if (env_u64("GS_BATCH", &x, err, err_len, &bad)) c->batch = (uint32_t)x;
  if (env_u64("GS_DEVICE", &x, err, err_len, &bad)) c->device = (int32_t)x;
  if (env_u64("GS_IDONTWANT", &x, err, err_len, &bad)) c->idontwant = (uint32_t)x;
  if (env_u64("GS_CHURN_PPM", &x, err, err_len, &bad)) c->churn_ppm = (uint32_t)x;
  if (env_u64("GS_CHURN_DOWN", &x, err, err_len, &bad)) c->churn_down = (uint32_t)x;
  if (env_u64("GS_CHURN_HORIZON", &x, err, err_len, &bad)) c->churn_horizon = (uint32_t)x;
  if (env_u64("GS_HB_PHASE_NS", &x, err, err_len, &bad)) c->hb_phase_ns = x;
  if (env_u64("GS_LAZY_GOSSIP", &x, err, err_len, &bad)) c->lazy_gossip = x ? 1 : 0;
  if (env_u64("GS_SUB_GRAFT", &x, err, err_len, &bad)) c->sub_graft = x ? 1 : 0;
  if (env_u64("GS_HS_RTTS", &x, err, err_len, &bad)) c->hs_rtts = (uint32_t)x;
  const char* gf = getenv("GOSSIPSUB_GOSSIP_FACTOR");
  if (gf && *gf) {
    char* end = nullptr;
    double f = strtod(gf, &end);
    if (!*end && f >= 0.0 && f <= 1.0) c->gossip_factor_milli = (uint32_t)(f * 1000.0 + 0.5);
  }
  env_bool("GOSSIPSUB_FLOOD_PUBLISH", &c->flood_publish);
  env_bool("SELFTRIGGER", &c->self_log);
  const char* mx = getenv("MUXER");
  if (mx && *mx) {
    std::string m(mx);
    for (auto& ch : m) ch = (char)tolower((unsigned char)ch);  // env.rs:50 to_lowercase
    if (m == "yamux") c->muxer = GS_MUX_YAMUX;
    else if (m == "quic") c->muxer = GS_MUX_QUIC;
    else if (m == "mplex") c->muxer = GS_MUX_MPLEX;  // nim only
    else { set_err(err, err_len, "Unknown muxer type: " + m); return GS_EINVAL; }  // env.rs:69-71
  }
  if (c->connect_to >= c->peers) {  // env.rs:73-75
    set_err(err, err_len, "Not enough peers to make target connections. Network size: " +
                              std::to_string(c->peers));
    return GS_EINVAL;
  }
  return GS_OK;
}

namespace {
uint64_t varint_len(uint64_t x) { uint64_t n = 1; while (x >= 128) { x >>= 7; n++; } return n; }
uint64_t pb_field(uint64_t len) { return 1 + varint_len(len) + len; }
uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
}  // namespace

// Per-hop wire bytes of one fragment:
// protobuf RPC{publish: Message{from, data, seqno, topic, signature}}
// length-prefixed, then the MUXER stack (rust-test-node/src/main.rs:418-440).
namespace {
// A length-delimited RPC frame through the MUXER stack -> wire bytes; *pkts /
// *hdr = packets of the last layer and their header bytes
uint64_t stack_model(uint64_t frame, uint32_t muxer, uint64_t* pkts, uint64_t* hdr) {
  if (muxer == GS_MUX_QUIC) {
    *pkts = cdiv(frame, 1415);
    *hdr = *pkts * 65;
    return frame + *hdr;
  }
  const uint64_t mux = (muxer == GS_MUX_MPLEX) ? frame + cdiv(frame, 1048576) * 4
                                               : frame + cdiv(frame, 16384) * 12;
  const uint64_t noise = mux + cdiv(mux, 65519) * 18;
  *pkts = cdiv(noise, 1460);
  *hdr = *pkts * 40;
  return noise + *hdr;
}
uint64_t wire_model(uint64_t payload, uint32_t muxer, uint32_t signed_msgs, uint64_t* pkts, uint64_t* hdr) {
  uint64_t body = pb_field(payload) + pb_field(4);               // data, topic "test"
  if (signed_msgs) body += pb_field(38) + pb_field(8) + pb_field(64);  // from, seqno, sig
  const uint64_t rpc = pb_field(body);
  return stack_model(varint_len(rpc) + rpc, muxer, pkts, hdr);
}
}  // namespace

// Lazy-gossip control RPCs with one message id:
// RPC{control: ControlMessage{ihave: ControlIHave{topic "test", ids}}} and
// RPC{control: {iwant: ControlIWant{ids}}}. The id is the node's
// message_id_fn: rust's DefaultHasher u64 in decimal (main.rs:73-77) and nim's
// $hash (gossipsub-queues/main.nim:123-124), up to 20 chars (modelled at 20);
// go's sha256 digest (go-test-node/main.go:26-29), 32 bytes. A pure ACK is
// one header-only packet.
extern "C" void gs_control_packets(uint32_t kind, uint32_t node, uint32_t muxer, uint64_t* bytes,
                                   uint64_t* packets, uint64_t* header_bytes) {
  uint64_t w, p = 1, h;
  if (kind == GS_CTRL_ACK) {
    w = h = muxer == GS_MUX_QUIC ? 65 : 40;
  } else {
    const uint64_t id = node == GS_NODE_GO ? 32 : 20;
    const uint64_t cm = kind == GS_CTRL_IHAVE ? pb_field(pb_field(4) + pb_field(id)) : pb_field(pb_field(id));
    const uint64_t rpc = pb_field(cm);
    w = stack_model(varint_len(rpc) + rpc, muxer, &p, &h);
  }
  if (bytes) *bytes = w;
  if (packets) *packets = p;
  if (header_bytes) *header_bytes = h;
}

extern "C" uint64_t gs_wire_bytes(uint64_t payload, uint32_t muxer, uint32_t signed_msgs) {
  uint64_t p, h;
  return wire_model(payload, muxer, signed_msgs, &p, &h);
}

extern "C" void gs_wire_packets(uint64_t payload, uint32_t muxer, uint32_t signed_msgs, uint64_t* packets,
                                uint64_t* header_bytes) {
  uint64_t p = 0, h = 0;
  wire_model(payload, muxer, signed_msgs, &p, &h);
  if (packets) *packets = p;
  if (header_bytes) *header_bytes = h;
}

// Shadow's tracker heartbeat line (Shadow v3.3.0, not vendored; the field
// positions are the ones shadow/summary_shadowlog.awk:12-64 reads): $5 the
// host, $9 "[node]", $10 "seconds,recv-bytes,send-bytes,cpu,delayed,avgdelay"
// then four ';'-separated groups of 12 counters (inbound / outbound localhost,
// inbound / outbound remote): packets, bytes, control packets, control header
// bytes, 2 control retransmit counters, data packets, data header bytes, data
// payload bytes, 3 data retransmit counters. Control packets are the modelled
// pure ACKs (header only); the simulator has no localhost traffic and no
// retransmissions: those stay 0.
extern "C" gs_status gs_write_shadow_heartbeat(const char* path, uint32_t peers, const uint64_t* tr,
                                               uint64_t sim_seconds) {
  if (!path || !tr) return GS_EINVAL;
  FILE* f = fopen(path, "w");
  if (!f) return GS_EINVAL;
  const unsigned long long hh = sim_seconds / 3600, mm = sim_seconds / 60 % 60, ss = sim_seconds % 60;
  typedef unsigned long long ull;
  for (uint32_t u = 0; u < peers; u++) {
    const uint64_t* r = tr + (size_t)u * GS_TRAFFIC_COLS;
    auto grp = [&](uint64_t pk, uint64_t by, uint64_t hd, uint64_t cpk, uint64_t chd) {
      char b[320];
      snprintf(b, sizeof b, "%llu,%llu,%llu,%llu,0,0,%llu,%llu,%llu,0,0,0", (ull)(pk + cpk), (ull)(by + chd),
               (ull)cpk, (ull)chd, (ull)pk, (ull)hd, (ull)(by - hd));
      return std::string(b);
    };
    const std::string zero = "0,0,0,0,0,0,0,0,0,0,0,0";
    fprintf(f, "00:00:00.000000 [thread-0] %02llu:%02llu:%02llu.000000000 [message] [pod-%u] [tracker] "
               "[_tracker_logNode] [shadow-heartbeat] [node] %llu,%llu,%llu,0,0,0;%s;%s;%s;%s\n",
            hh, mm, ss, u, (ull)sim_seconds, (ull)(r[GS_TR_RX_BYTES] + r[GS_TR_RX_CTRL_HDR]),
            (ull)(r[GS_TR_TX_BYTES] + r[GS_TR_TX_CTRL_HDR]), zero.c_str(), zero.c_str(),
            grp(r[GS_TR_RX_PKTS], r[GS_TR_RX_BYTES], r[GS_TR_RX_HDR], r[GS_TR_RX_CTRL_PKTS], r[GS_TR_RX_CTRL_HDR]).c_str(),
            grp(r[GS_TR_TX_PKTS], r[GS_TR_TX_BYTES], r[GS_TR_TX_HDR], r[GS_TR_TX_CTRL_PKTS], r[GS_TR_TX_CTRL_HDR]).c_str());
  }
  if (fclose(f)) return GS_EINVAL;
  return GS_OK;
}

namespace {
constexpr uint64_t NO_EDGE = ~0ull;

// Stage-to-stage latency table of the first S nodes of a V-node network graph
// g (ns, NO_EDGE = no edge). GS_LINKS_DIRECT: the edge itself (topogen's
// intent); GS_LINKS_SHORTEST: Shadow's use_shortest_path (upstream, not
// vendored) — the shortest non-empty path, so a self-loop may be beaten by a
// round trip through another node.
gs_status graph_latencies(uint32_t V, const std::vector<uint64_t>& g, uint32_t S, uint32_t mode, uint64_t* lat) {
  if (mode == GS_LINKS_DIRECT) {
    for (uint32_t i = 0; i < S; i++)
      for (uint32_t j = 0; j < S; j++) {
        if (g[(size_t)i * V + j] == NO_EDGE) return GS_EINVAL;  // direct mode needs every stage pair
        lat[(size_t)i * S + j] = g[(size_t)i * V + j];
      }
    return GS_OK;
  }
  std::vector<uint64_t> d((size_t)V * V);
  for (uint32_t i = 0; i < V; i++)
    for (uint32_t j = 0; j < V; j++) d[(size_t)i * V + j] = i == j ? 0 : g[(size_t)i * V + j];
  for (uint32_t k = 0; k < V; k++)
    for (uint32_t i = 0; i < V; i++)
      for (uint32_t j = 0; j < V; j++) {
        const uint64_t a = d[(size_t)i * V + k], b = d[(size_t)k * V + j];
        if (a != NO_EDGE && b != NO_EDGE && a + b < d[(size_t)i * V + j]) d[(size_t)i * V + j] = a + b;
      }
  for (uint32_t i = 0; i < S; i++)
    for (uint32_t j = 0; j < S; j++) {
      uint64_t v = d[(size_t)i * V + j];
      if (i == j) {
        v = g[(size_t)i * V + i];
        for (uint32_t k = 0; k < V; k++) {
          const uint64_t a = d[(size_t)i * V + k], b = d[(size_t)k * V + i];
          if (k != i && a != NO_EDGE && b != NO_EDGE && a + b < v) v = a + b;
        }
      }
      if (v == NO_EDGE) return GS_EINVAL;  // unreachable stage pair
      lat[(size_t)i * S + j] = v;
    }
  return GS_OK;
}
}  // namespace

// shadow/topogen.py:39-71 restated: stage i bandwidth ceil(i*bj + bl) Mbit
// (44,49-51); self-loop max((S-i)*lj, ll) ms (55); edge i<j
// min(ceil((S-j)*lj + ll), lh) ms (60); injector node S, 1 ms to all (64-69).
extern "C" gs_status gs_topogen_links(uint32_t S, uint32_t bl, uint32_t bh, uint32_t ll,
                                      uint32_t lh, uint32_t mode, uint64_t* lat_ns,
                                      uint64_t* bw_bps) {
  if (S == 0 || S > 255 || bl > bh || ll > lh || mode > GS_LINKS_SHORTEST || !lat_ns || !bw_bps)
    return GS_EINVAL;
  const uint64_t bj = (bh - bl) / S, lj = (lh - ll) / S;
  const uint32_t V = S + 1;
  std::vector<uint64_t> g((size_t)V * V, 0);
  for (uint32_t i = 0; i < S; i++) {
    bw_bps[i] = ((uint64_t)i * bj + bl) * 1000000ull;
    uint64_t self = (uint64_t)(S - i) * lj;
    g[(size_t)i * V + i] = self < ll ? ll : self;
    for (uint32_t j = i + 1; j < S; j++) {
      uint64_t e = (uint64_t)(S - j) * lj + ll;
      g[(size_t)i * V + j] = g[(size_t)j * V + i] = e > lh ? lh : e;
    }
  }
  for (uint32_t i = 0; i <= S; i++) g[(size_t)i * V + S] = g[(size_t)S * V + i] = 1;
  for (auto& x : g) x *= 1000000ull;  // ms -> ns
  return graph_latencies(V, g, S, mode, lat_ns);
}

namespace {
// "<number> <unit>" of Shadow's GML attributes -> value in base units (ns or bit/s).
bool parse_quantity(const std::string& s, bool time, uint64_t* out) {
  char* end = nullptr;
  const double x = strtod(s.c_str(), &end);
  if (end == s.c_str() || x < 0) return false;
  std::string u(end);
  u.erase(0, u.find_first_not_of(' '));
  double mul;
  if (time) {
    if (u == "ns") mul = 1;
    else if (u == "us" || u == "μs") mul = 1e3;
    else if (u == "ms") mul = 1e6;
    else if (u == "s" || u == "sec") mul = 1e9;
    else return false;
  } else {
    if (u == "bit") mul = 1;
    else if (u == "Kbit" || u == "kbit") mul = 1e3;
    else if (u == "Mbit") mul = 1e6;
    else if (u == "Gbit") mul = 1e9;
    else if (u == "Kibit") mul = 1024.0;
    else if (u == "Mibit") mul = 1048576.0;
    else if (u == "Gibit") mul = 1073741824.0;
    else return false;
  }
  *out = (uint64_t)(x * mul + 0.5);
  return true;
}
}  // namespace

// network_topology.gml as topogen.py:39-71 writes it (networkx write_gml):
// node [ id, host_bandwidth_up/down "<n> Mbit" ] and edge [ source, target,
// latency "<n> ms", packet_loss ] blocks, undirected. Every node becomes one
// link class (the injector node of topogen included; no peer maps to it).
extern "C" gs_status gs_links_from_gml(const char* path, uint32_t mode, uint32_t max_nodes, uint32_t* nodes,
                                       uint64_t* lat_ns, uint64_t* bw_up_bps, uint64_t* bw_down_bps) {
  if (!path || !nodes || mode > GS_LINKS_SHORTEST) return GS_EINVAL;
  FILE* f = fopen(path, "r");
  if (!f) return GS_EINVAL;
  std::string text;
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  // tokens: bare words, numbers, quoted strings, [ and ]
  std::vector<std::string> tok;
  for (size_t i = 0; i < text.size();) {
    const char ch = text[i];
    if (isspace((unsigned char)ch)) { i++; continue; }
    if (ch == '[' || ch == ']') { tok.emplace_back(1, ch); i++; continue; }
    if (ch == '"') {
      const size_t j = text.find('"', i + 1);
      if (j == std::string::npos) return GS_EINVAL;
      tok.push_back(text.substr(i, j - i + 1));
      i = j + 1;
      continue;
    }
    size_t j = i;
    while (j < text.size() && !isspace((unsigned char)text[j]) && text[j] != '[' && text[j] != ']') j++;
    tok.push_back(text.substr(i, j - i));
    i = j;
  }
  struct Node { int64_t id = -1; uint64_t up = 0, dn = 0; };
  struct Edge { int64_t s = -1, t = -1; uint64_t lat = 0; double loss = 0; };
  std::vector<Node> nv;
  std::vector<Edge> ev;
  auto unq = [](const std::string& s) { return s.size() >= 2 && s[0] == '"' ? s.substr(1, s.size() - 2) : s; };
  for (size_t i = 0; i + 1 < tok.size(); i++) {
    if ((tok[i] != "node" && tok[i] != "edge") || tok[i + 1] != "[") continue;
    const bool is_node = tok[i] == "node";
    Node nd;
    Edge ed;
    size_t j = i + 2;
    for (; j + 1 < tok.size() && tok[j] != "]"; j += 2) {
      const std::string& k = tok[j];
      const std::string v = unq(tok[j + 1]);
      if (tok[j + 1] == "[") return GS_EINVAL;  // no nested blocks in topogen's GML
      if (is_node && k == "id") nd.id = strtoll(v.c_str(), nullptr, 10);
      else if (is_node && k == "host_bandwidth_up") { if (!parse_quantity(v, false, &nd.up)) return GS_EINVAL; }
      else if (is_node && k == "host_bandwidth_down") { if (!parse_quantity(v, false, &nd.dn)) return GS_EINVAL; }
      else if (!is_node && k == "source") ed.s = strtoll(v.c_str(), nullptr, 10);
      else if (!is_node && k == "target") ed.t = strtoll(v.c_str(), nullptr, 10);
      else if (!is_node && k == "latency") { if (!parse_quantity(v, true, &ed.lat)) return GS_EINVAL; }
      else if (!is_node && k == "packet_loss") ed.loss = strtod(v.c_str(), nullptr);
    }
    if (is_node) nv.push_back(nd); else ev.push_back(ed);
    i = j;
  }
  const uint32_t V = (uint32_t)nv.size();
  *nodes = V;
  if (V == 0) return GS_EINVAL;
  if (V > max_nodes) return GS_ERANGE;  // *nodes tells the caller the size needed
  if (!lat_ns || !bw_up_bps || !bw_down_bps) return GS_EINVAL;
  std::vector<uint64_t> g((size_t)V * V, NO_EDGE);
  std::vector<bool> seen(V, false);
  for (const Node& nd : nv) {
    if (nd.id < 0 || nd.id >= (int64_t)V || seen[nd.id] || nd.up == 0 || nd.dn == 0) return GS_EINVAL;
    seen[nd.id] = true;
    bw_up_bps[nd.id] = nd.up;
    bw_down_bps[nd.id] = nd.dn;
  }
  for (const Edge& ed : ev) {
    if (ed.s < 0 || ed.t < 0 || ed.s >= (int64_t)V || ed.t >= (int64_t)V || ed.lat == 0) return GS_EINVAL;
    if (ed.loss != 0.0) return GS_EUNSUPPORTED;  // packet loss is not modelled (run.sh:33: "not yet tested")
    g[(size_t)ed.s * V + ed.t] = g[(size_t)ed.t * V + ed.s] = ed.lat;
  }
  return graph_latencies(V, g, V, mode, lat_ns);
}

// shadow.yaml as topogen.py:73-139 writes it (PyYAML): under "hosts:", blocks
// "  pod-<i>: &idN" with "    network_node_id: <k>", repeated hosts as
// aliases "  pod-<j>: *idN". The peer id is the number after the '-' of the
// host name (rust env.rs:34-36); hosts with ids >= peers (the injector) are
// skipped.
extern "C" gs_status gs_shadow_hosts(const char* path, uint32_t peers, uint8_t* stage_of_peer) {
  if (!path || !stage_of_peer) return GS_EINVAL;
  FILE* f = fopen(path, "r");
  if (!f) return GS_EINVAL;
  std::vector<int> stage(peers, -1);
  std::vector<std::pair<std::string, int>> anchors;
  auto anchor_get = [&](const std::string& a) {
    for (auto& kv : anchors) if (kv.first == a) return kv.second;
    return -1;
  };
  bool in_hosts = false;
  int64_t cur = -1;
  std::string cur_anchor;
  char line[4096];
  while (fgets(line, sizeof line, f)) {
    std::string s(line);
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    if (s.empty()) continue;
    const size_t ind = s.find_first_not_of(' ');
    if (ind == std::string::npos) continue;
    if (ind == 0) { in_hosts = s == "hosts:"; cur = -1; continue; }
    if (!in_hosts) continue;
    if (ind == 2) {  // a host
      const size_t colon = s.find(':');
      if (colon == std::string::npos) continue;
      const std::string name = s.substr(2, colon - 2);
      const size_t dash = name.find('-');
      char* end = nullptr;
      const int64_t id = dash == std::string::npos ? -1 : strtoll(name.c_str() + dash + 1, &end, 10);
      cur = (dash != std::string::npos && end && *end == '\0') ? id : -1;
      std::string rest = s.substr(colon + 1);
      rest.erase(0, rest.find_first_not_of(' '));
      cur_anchor.clear();
      if (!rest.empty() && rest[0] == '&') cur_anchor = rest.substr(1);
      else if (!rest.empty() && rest[0] == '*') {  // alias of an earlier host block
        const int st = anchor_get(rest.substr(1));
        if (st < 0) { fclose(f); return GS_EINVAL; }
        if (cur >= 0 && cur < (int64_t)peers) stage[cur] = st;
        cur = -1;
      }
      continue;
    }
    if (ind == 4 && s.compare(4, 16, "network_node_id:") == 0) {
      const long k = strtol(s.c_str() + 20, nullptr, 10);
      if (k < 0 || k > 255) { fclose(f); return GS_ERANGE; }
      if (!cur_anchor.empty()) anchors.emplace_back(cur_anchor, (int)k);
      if (cur >= 0 && cur < (int64_t)peers) stage[cur] = (int)k;
    }
  }
  fclose(f);
  for (uint32_t u = 0; u < peers; u++) {
    if (stage[u] < 0) return GS_EINVAL;  // every peer needs a host entry
    stage_of_peer[u] = (uint8_t)stage[u];
  }
  return GS_OK;
}

// The controller host of topogen's shadow.yaml (topogen.py:125-136):
//   pod-<N>:
//     processes:
//     - path: /usr/bin/python
//       args: ../../../traffic_sync.py -s 15000 -m 10 -d 1000.0 -n 100 --peer-selection
//         id                                      (PyYAML folds long scalars)
//       start_time: 500s
extern "C" gs_status gs_shadow_injector(const char* path, gs_injector* out) {
  if (!path || !out) return GS_EINVAL;
  FILE* f = fopen(path, "r");
  if (!f) return GS_EINVAL;
  std::string args, start;
  bool in_args = false;
  size_t args_ind = 0;
  char line[4096];
  while (fgets(line, sizeof line, f)) {
    std::string s(line);
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    const size_t ind = s.find_first_not_of(' ');
    if (ind == std::string::npos) continue;
    std::string body = s.substr(ind);
    if (body.compare(0, 2, "- ") == 0) body = body.substr(2);
    if (in_args && ind > args_ind && body.find(':') == std::string::npos) {  // folded continuation
      args += " " + body;
      continue;
    }
    in_args = false;
    if (body.compare(0, 5, "args:") == 0 && body.find("traffic_sync") != std::string::npos) {
      args = body.substr(5);
      in_args = true;
      args_ind = ind;
    } else if (body.compare(0, 11, "start_time:") == 0 && !args.empty() && start.empty()) {
      start = body.substr(11);
    }
  }
  fclose(f);
  if (args.empty()) return GS_EINVAL;  // no injector host in this config
  memset(out, 0, sizeof *out);
  out->start_ns = 500000000000ull;  // topogen.py:133
  if (!start.empty()) {
    char* end = nullptr;
    const double v = strtod(start.c_str(), &end);
    std::string u(end ? end : "");
    u.erase(0, u.find_first_not_of(" '\""));
    const double mul = (u.compare(0, 2, "ms") == 0) ? 1e6 : (u.compare(0, 3, "min") == 0) ? 6e10 : 1e9;
    out->start_ns = (uint64_t)(v * mul + 0.5);
  }
  // tokens after the script name
  std::vector<std::string> tok;
  for (size_t i = 0; i < args.size();) {
    while (i < args.size() && isspace((unsigned char)args[i])) i++;
    size_t j = i;
    while (j < args.size() && !isspace((unsigned char)args[j])) j++;
    if (j > i) tok.push_back(args.substr(i, j - i));
    i = j;
  }
  for (size_t i = 0; i + 1 < tok.size(); i++) {
    const std::string& k = tok[i];
    const char* v = tok[i + 1].c_str();
    if (k == "-s" || k == "--msg-size") out->msg_size = (uint32_t)strtoul(v, nullptr, 10);
    else if (k == "-m" || k == "--messages") out->messages = (uint32_t)strtoul(v, nullptr, 10);
    else if (k == "-n" || k == "--network-size") out->peers = (uint32_t)strtoul(v, nullptr, 10);
    else if (k == "-d" || k == "--delay") out->delay_ns = (uint64_t)(strtod(v, nullptr) * 1e6 + 0.5);  // ms (run.sh:36)
  }
  return (out->msg_size && out->messages) ? GS_OK : GS_EINVAL;
}

extern "C" gs_status gs_read_schedule(const char* path, gs_publish* out, uint64_t cap, uint64_t* n) {
  if (!path || !n) return GS_EINVAL;
  FILE* f = fopen(path, "r");
  if (!f) return GS_EINVAL;
  char line[1024];
  uint64_t rows = 0;
  gs_status st = GS_OK;
  while (fgets(line, sizeof line, f)) {
    char* h = strchr(line, '#');
    if (h) *h = 0;
    unsigned long long t = 0;
    unsigned pub = 0, size = 0, fr = 0;
    const int k = sscanf(line, "%llu %u %u %u", &t, &pub, &size, &fr);
    if (k <= 0) {
      char* q = line;
      while (*q && isspace((unsigned char)*q)) q++;
      if (*q) { st = GS_EINVAL; break; }  // not a number
      continue;                           // blank / comment
    }
    if (k < 3) { st = GS_EINVAL; break; }
    if (out && rows < cap) {
      out[rows].t_pub_ns = t;
      out[rows].publisher = pub;
      out[rows].msg_size = size;
      out[rows].frags = k == 4 ? fr : 0;
      out[rows].reserved = 0;
    }
    rows++;
  }
  fclose(f);
  *n = rows;
  if (st != GS_OK) return st;
  return rows > cap ? GS_ERANGE : GS_OK;
}

// The node's custom metrics (rust-test-node/src/metrics.rs:60-132, names shared
// with go metrics.go and nim gossipsub-queues/main.nim:25-78) for every peer,
// in prometheus-client's OpenMetrics text encoding (the format store_metrics
// dumps, env.rs:114-152): gauges as is, counters with the _total suffix,
// topic families labelled topic="test" (main.rs:248), "# EOF" at the end.
extern "C" gs_status gs_write_node_metrics(const gs_config* cfg, const char* path, const uint64_t* row_ptr,
                                           const uint8_t* mesh_count, const uint64_t* traffic) {
  if (!cfg || !path || !row_ptr || !mesh_count || !traffic) return GS_EINVAL;
  FILE* f = fopen(path, "w");
  if (!f) return GS_EINVAL;
  std::vector<char> buf(1 << 20);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  const uint32_t N = cfg->peers;
  auto deg = [&](uint32_t u) { return (unsigned long long)(row_ptr[u + 1] - row_ptr[u]); };
  auto family = [&](const char* name, const char* type, const char* help, bool topic, auto value) {
    fprintf(f, "# HELP %s %s.\n# TYPE %s %s\n", name, help, name, type);
    const char* suffix = strcmp(type, "counter") == 0 ? "_total" : "";
    for (uint32_t u = 0; u < N; u++)
      fprintf(f, "%s%s{%speer=\"pod-%u\"} %llu\n", name, suffix, topic ? "topic=\"test\"," : "", u,
              (unsigned long long)value(u));
  };
  const uint64_t* tr = traffic;
  auto mc = [&](uint32_t u) { return (uint64_t)mesh_count[u]; };
  family("libp2p_peers", "gauge", "total connected peers", false, deg);
  family("libp2p_pubsub_peers", "gauge", "pubsub peer instances", false, deg);
  family("libp2p_pubsub_topics", "gauge", "pubsub subscribed topics", false, [](uint32_t) { return 1ull; });
  family("libp2p_gossipsub_peers_per_topic_mesh", "gauge", "gossipsub peers per topic in mesh", true, mc);
  family("libp2p_gossipsub_peers_per_topic_gossipsub", "gauge", "gossipsub peers per topic in gossipsub", true, deg);
  // update_health (metrics.rs:158-176) over the one topic
  family("libp2p_gossipsub_no_peers_topics", "gauge", "number of topics in mesh with no peers", false,
         [&](uint32_t u) { return mc(u) == 0 ? 1ull : 0ull; });
  family("libp2p_gossipsub_low_peers_topics", "gauge",
         "number of topics in mesh with at least one but below dlow peers", false,
         [&](uint32_t u) { return mc(u) > 0 && mc(u) < cfg->d_lo ? 1ull : 0ull; });
  family("libp2p_gossipsub_healthy_peers_topics", "gauge", "number of topics in mesh with at least dlow peers",
         false, [&](uint32_t u) { return mc(u) >= cfg->d_lo ? 1ull : 0ull; });
  auto rcv = [&](uint32_t u) { return tr[(size_t)u * GS_TRAFFIC_COLS + GS_TR_RECEIVED]; };
  family("libp2p_gossipsub_received", "counter", "number of messages received (deduplicated)", false, rcv);
  family("libp2p_pubsub_messages_published", "counter", "published messages", true,
         [&](uint32_t u) { return tr[(size_t)u * GS_TRAFFIC_COLS + GS_TR_PUBLISHED]; });
  family("libp2p_pubsub_validation_success", "counter", "pubsub successfully validated messages", false, rcv);
  family("libp2p_pubsub_validation_failure", "counter", "pubsub failed validated messages", false,
         [](uint32_t) { return 0ull; });
  family("libp2p_pubsub_received_subscriptions", "counter", "pubsub received subscriptions", true, deg);
  family("libp2p_pubsub_received_unsubscriptions", "counter", "pubsub received unsubscriptions", true,
         [](uint32_t) { return 0ull; });
  fprintf(f, "# EOF\n");
  if (fclose(f)) return GS_EINVAL;
  return GS_OK;
}

// shadow/run.sh:34-36 + shadow/README.md:76-78: publisher_id, rotation 0/1,
// inter_message_delay. tx_time is the publish instant (main.rs:105-111).
extern "C" gs_status gs_schedule_runsh(uint32_t n_msgs, uint32_t peers, uint32_t publisher_id,
                                       uint32_t rotation, uint64_t t0_ns, uint64_t delay_ns,
                                       uint32_t msg_size, gs_publish* out) {
  if (!out || peers == 0) return GS_EINVAL;
  for (uint32_t i = 0; i < n_msgs; i++) {
    out[i].t_pub_ns = t0_ns + (uint64_t)i * delay_ns;
    out[i].publisher = (uint32_t)(((uint64_t)publisher_id + (uint64_t)i * rotation) % peers);
    out[i].msg_size = msg_size;
    out[i].frags = 0;  // cfg.fragments (FRAGMENTS of every node, env.rs:64-67)
    out[i].reserved = 0;
  }
  return GS_OK;
}

// The grep view of Shadow's per-host stdout (shadow/run.sh:61) for the line
// printed at rust-test-node/src/main.rs:93. Paths use `peer<id>` so that the
// split regex of shadow/summary_latency.awk:17 recovers the id (defect D3).
extern "C" gs_status gs_write_latency_log(const char* path, const gs_publish* sched,
                                          uint64_t n_msgs, uint32_t peers,
                                          const uint64_t* t_complete_ns, uint32_t self_log) {
  if (!path || !sched || !t_complete_ns) return GS_EINVAL;
  FILE* f = fopen(path, "w");
  if (!f) return GS_EINVAL;
  std::vector<char> buf(1 << 20);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  for (uint32_t u = 0; u < peers; u++) {
    uint64_t line = 0;
    for (uint64_t m = 0; m < n_msgs; m++) {
      const uint64_t t = t_complete_ns[m * peers + u];
      if (t == GS_UNDELIVERED) continue;
      if (u == sched[m].publisher && !self_log) continue;
      const uint64_t tx = sched[m].t_pub_ns;
      const int64_t ms = ((int64_t)t - (int64_t)tx) / 1000000;  // i64 division, main.rs:91-93
      fprintf(f, "shadow.data/hosts/peer%u/main.1000.stdout:%llu:%lld milliseconds: %lld\n", u,
              (unsigned long long)++line, (long long)tx, (long long)ms);
    }
  }
  if (fclose(f)) return GS_EINVAL;
  return GS_OK;
}

// One arrival line of a node flavour (rust main.rs:93 / go main.go:49: tx_time;
// nim main.nim:150: msgId) in grep's path:line:text form (shadow/run.sh:61).
namespace {
uint64_t nim_msg_id(const gs_config* cfg, const gs_publish& p) {  // msgId = rand(high(int64)) (main.nim:162)
  return gs::rng(cfg->seed, gs::P_MSGID, p.publisher, (uint32_t)(p.t_pub_ns >> 32), (uint32_t)p.t_pub_ns) >> 1;
}
void log_line_ms(FILE* f, const gs_config* cfg, uint32_t u, uint64_t line, const gs_publish& p, int64_t ms) {
  if (cfg->node == GS_NODE_NIM)
    fprintf(f, "shadow.data/hosts/peer%u/main.1000.stdout:%llu:%llu milliseconds: %lld\n", u,
            (unsigned long long)line, (unsigned long long)nim_msg_id(cfg, p), (long long)ms);
  else
    fprintf(f, "shadow.data/hosts/peer%u/main.1000.stdout:%llu:%lld milliseconds: %lld\n", u,
            (unsigned long long)line, (long long)p.t_pub_ns, (long long)ms);
}
void log_line(FILE* f, const gs_config* cfg, uint32_t u, uint64_t line, const gs_publish& p, uint64_t t) {
  log_line_ms(f, cfg, u, line, p, ((int64_t)t - (int64_t)p.t_pub_ns) / 1000000);  // i64 division, main.rs:91-93
}
}  // namespace

struct gs_log {
  gs_config cfg;
  FILE* f = nullptr;
  std::vector<uint64_t> line;  // per-peer line counter (grep -n numbers lines per host file)
  std::vector<char> buf;
};

extern "C" gs_status gs_log_open(const gs_config* cfg, const char* path, gs_log** out) {
  if (!cfg || !path || !out || cfg->node > GS_NODE_NIM) return GS_EINVAL;
  *out = nullptr;
  gs_log* L = new (std::nothrow) gs_log();
  if (!L) return GS_ENOMEM;
  L->cfg = *cfg;
  L->f = fopen(path, "w");
  if (!L->f) { delete L; return GS_EINVAL; }
  L->buf.resize(1 << 22);
  setvbuf(L->f, L->buf.data(), _IOFBF, L->buf.size());
  L->line.assign(cfg->peers, 0);
  *out = L;
  return GS_OK;
}

extern "C" gs_status gs_log_write(gs_log* L, const gs_publish* sched, uint32_t n_msgs, const uint64_t* tc) {
  if (!L || (!sched && n_msgs) || (!tc && n_msgs)) return GS_EINVAL;
  const uint32_t N = L->cfg.peers;
  for (uint32_t m = 0; m < n_msgs; m++)
    for (uint32_t u = 0; u < N; u++) {
      const uint64_t t = tc[(size_t)m * N + u];
      if (t == GS_UNDELIVERED || (u == sched[m].publisher && !L->cfg.self_log)) continue;
      log_line(L->f, &L->cfg, u, ++L->line[u], sched[m], t);
    }
  return ferror(L->f) ? GS_EINVAL : GS_OK;
}

// The same lines from the u16 latency stream (gs_result_sink.on_lat): the
// value is the log line's ms already, GS_LAT_NONE where nothing is logged.
extern "C" gs_status gs_log_write_lat(gs_log* L, const gs_publish* sched, uint32_t n_msgs, const uint16_t* lat_ms) {
  if (!L || (!sched && n_msgs) || (!lat_ms && n_msgs)) return GS_EINVAL;
  const uint32_t N = L->cfg.peers;
  for (uint32_t m = 0; m < n_msgs; m++)
    for (uint32_t u = 0; u < N; u++) {
      const uint16_t v = lat_ms[(size_t)m * N + u];
      if (v == GS_LAT_NONE) continue;
      log_line_ms(L->f, &L->cfg, u, ++L->line[u], sched[m], (int64_t)v);
    }
  return ferror(L->f) ? GS_EINVAL : GS_OK;
}

extern "C" gs_status gs_log_close(gs_log* L) {
  if (!L) return GS_EINVAL;
  const int rc = fclose(L->f);
  delete L;
  return rc ? GS_EINVAL : GS_OK;
}

extern "C" gs_status gs_write_node_log(const gs_config* cfg, const char* path, const gs_publish* sched,
                                       uint64_t n_msgs, const uint64_t* t_complete_ns) {
  if (!cfg || cfg->node > GS_NODE_NIM) return GS_EINVAL;
  if (cfg->node != GS_NODE_NIM)  // rust main.rs:93 and go main.go:49 print the same line
    return gs_write_latency_log(path, sched, n_msgs, cfg->peers, t_complete_ns, cfg->self_log);
  if (!path || !sched || !t_complete_ns) return GS_EINVAL;
  FILE* f = fopen(path, "w");
  if (!f) return GS_EINVAL;
  std::vector<char> buf(1 << 20);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  for (uint32_t u = 0; u < cfg->peers; u++) {
    uint64_t line = 0;
    for (uint64_t m = 0; m < n_msgs; m++) {
      const uint64_t t = t_complete_ns[m * cfg->peers + u];
      if (t == GS_UNDELIVERED) continue;
      if (u == sched[m].publisher && !cfg->self_log) continue;
      log_line(f, cfg, u, ++line, sched[m], t);  // delay.inMilliseconds() (nim) = the same truncation
    }
  }
  if (fclose(f)) return GS_EINVAL;
  return GS_OK;
}
