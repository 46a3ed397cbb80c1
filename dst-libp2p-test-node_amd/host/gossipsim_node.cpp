// gossipsim-node — C++ host CLI standing in for the reference experiment:
// the env surface of rust-test-node (src/env.rs:27-87), topogen.py's link
// graph parameters (shadow/topogen.py:13-36), run.sh's publish schedule
// (shadow/run.sh:23-36) in place of the HTTP injector, and the arrival log
// that shadow/summary_latency*.awk parse (main.rs:93, run.sh:61).
//
//   PEERS=1000 CONNECTTO=10 FRAGMENTS=1 MUXER=yamux \
//   ./gossipsim-node -bl 50 -bh 150 -ll 40 -lh 130 -st 5 -s 15000 -m 10 \
//       --publisher 6 --rotation 1 --delay-ms 1000 --latencies latencies1
//   awk -f summary_latency_large.awk latencies1
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/gossipsim.h"

namespace {

void usage() {
  fprintf(stderr,
          "usage: gossipsim-node [-bl MBIT] [-bh MBIT] [-ll MS] [-lh MS] [-st STAGES] [--shortest]\n"
          "         [-s MSG_BYTES] [-m MESSAGES] [--publisher ID] [--rotation 0|1]\n"
          "         [--delay-ms MS] [--t0-s SECONDS] [--http-us US] [--max-heartbeats H] [--latencies PATH]\n"
          "         [--gml network_topology.gml --yaml shadow.yaml] [--schedule FILE] [--shadowlog PATH] [--metrics PATH]\n"
          "  --yaml also supplies the injector's -s/-m/-d and start_time unless given on the command line\n"
          "env: PEERS CONNECTTO FRAGMENTS MUXER MAXCONNECTIONS GOSSIPSUB_* SELFTRIGGER GS_NODE GS_SEED GS_BATCH\n"
          "     GS_DEVICE\n");
}

// Results arrive as the logged latency, message-major blocks of u16 ms
// (gs_result_sink.on_lat, GS_WANT_LAT_MS: 2 bytes per (peer, message), the
// value main.rs:93 prints): the log is streamed through gs_log_write_lat and
// the latencies folded into a 1 ms histogram, so no [messages][peers] host
// array is held. A run with a latency of 65535 ms or more (which the u16
// stream cannot carry: gs_run fails with GS_ERANGE) is delivered again as
// completion times (on_block, gs_log_write), the log rewritten from the start.
struct Stream {
  gs_log* log = nullptr;
  const gs_publish* sched = nullptr;
  gs_status st = GS_OK;
  std::vector<uint64_t> hist_ms;
  bool self_log = false;
};

void on_lat(void* user, uint64_t first, uint32_t n, uint32_t peers, const uint16_t* lat) {
  Stream* S = (Stream*)user;
  if (S->log && S->st == GS_OK) S->st = gs_log_write_lat(S->log, S->sched + first, n, lat);
  for (size_t i = 0; i < (size_t)n * peers; i++) {
    const uint16_t ms = lat[i];
    if (ms == GS_LAT_NONE) continue;  // undelivered, or the publisher without SELFTRIGGER
    if (ms >= S->hist_ms.size()) S->hist_ms.resize((size_t)ms + 1, 0);
    S->hist_ms[ms]++;
  }
}

// The same from completion times (the u64 fallback): the lines main.rs:93
// prints, (t_complete - tx_time) / 1e6 truncated; the publisher logs only with
// SELFTRIGGER (cfg.self_log).
void on_block(void* user, uint64_t first, uint32_t n, uint32_t peers, const uint64_t* tc, const uint8_t*) {
  Stream* S = (Stream*)user;
  if (S->log && S->st == GS_OK) S->st = gs_log_write(S->log, S->sched + first, n, tc);
  for (uint32_t q = 0; q < n; q++) {
    const gs_publish& p = S->sched[first + q];
    for (uint32_t u = 0; u < peers; u++) {
      const uint64_t t = tc[(size_t)q * peers + u];
      if (t == GS_UNDELIVERED || (u == p.publisher && !S->self_log)) continue;
      const uint64_t ms = (t - p.t_pub_ns) / 1000000ull;
      if (ms >= S->hist_ms.size()) S->hist_ms.resize((size_t)ms + 1, 0);
      S->hist_ms[ms]++;
    }
  }
}

// nearest-rank percentile (rank ceil(q*n)) of the 1 ms histogram
uint64_t pct(const std::vector<uint64_t>& h, uint64_t n, uint32_t q100) {
  const uint64_t rank = (n * q100 + 99) / 100;
  uint64_t acc = 0;
  for (size_t i = 0; i < h.size(); i++)
    if ((acc += h[i]) >= rank && rank) return i;
  return 0;
}

int die(gs_ctx* ctx, gs_status st, const char* what) {
  fprintf(stderr, "%s failed (%d): %s\n", what, st, ctx ? gs_last_error(ctx) : "");
  if (ctx) gs_destroy(ctx);
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  // topogen.py defaults (topogen.py:15-26) and run.sh's fixed publisher knobs
  uint32_t bl = 50, bh = 50, ll = 100, lh = 100, stages = 1, mode = GS_LINKS_DIRECT;
  uint32_t msg_size = 1500, n_msgs = 10, publisher = 6, rotation = 1, max_hb = 400;
  uint64_t delay_ms = 1000, t0_s = 946684800ull + 500ull;  // Shadow epoch + injector start (topogen.py:130)
  // the POST reaches the node 1.5 round trips over the 1 ms injector-hub links
  // after the injector sends it (topogen.py:64-69); tx_time is stamped then
  uint64_t http_us = 3000;
  std::string latencies, gml, yaml, shadowlog, metrics, schedule;
  bool set_size = false, set_msgs = false, set_delay = false, set_t0 = false;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&](void) -> const char* {
      if (i + 1 >= argc) { usage(); exit(2); }
      return argv[++i];
    };
    if (a == "-bl") bl = (uint32_t)atoi(next());
    else if (a == "-bh") bh = (uint32_t)atoi(next());
    else if (a == "-ll") ll = (uint32_t)atoi(next());
    else if (a == "-lh") lh = (uint32_t)atoi(next());
    else if (a == "-st") stages = (uint32_t)atoi(next());
    else if (a == "--shortest") mode = GS_LINKS_SHORTEST;
    else if (a == "-s") { msg_size = (uint32_t)atoi(next()); set_size = true; }
    else if (a == "-m") { n_msgs = (uint32_t)atoi(next()); set_msgs = true; }
    else if (a == "--publisher") publisher = (uint32_t)atoi(next());
    else if (a == "--rotation") rotation = (uint32_t)atoi(next());
    else if (a == "--delay-ms") { delay_ms = strtoull(next(), nullptr, 10); set_delay = true; }
    else if (a == "--t0-s") { t0_s = strtoull(next(), nullptr, 10); set_t0 = true; }
    else if (a == "--http-us") http_us = strtoull(next(), nullptr, 10);
    else if (a == "--max-heartbeats") max_hb = (uint32_t)atoi(next());
    else if (a == "--latencies") latencies = next();
    else if (a == "--gml") gml = next();            // a Shadow experiment's network graph ...
    else if (a == "--yaml") yaml = next();          // ... and its host placement (topogen.py output)
    else if (a == "--shadowlog") shadowlog = next(); // tracker counters for summary_shadowlog.awk
    else if (a == "--metrics") metrics = next();    // the node metrics (rust-test-node/src/metrics.rs)
    else if (a == "--schedule") schedule = next();  // rows: t_pub_ns publisher msg_size [frags]
    else { usage(); return 2; }
  }
  gs_config cfg;
  gs_config_default(&cfg);
  char err[256] = {0};
  gs_status st = gs_config_from_env(&cfg, err, sizeof(err));
  if (st != GS_OK) { fprintf(stderr, "Error reading peer settings: %s\n", err); return 1; }

  std::vector<uint64_t> lat((size_t)stages * stages), bw(stages), bw_dn;
  std::vector<uint8_t> stage_of_peer;
  if (!gml.empty()) {  // links straight from the Shadow experiment files
    if (yaml.empty()) { fprintf(stderr, "--gml needs --yaml (host placement)\n"); return 2; }
    uint32_t V = 0;
    gs_links_from_gml(gml.c_str(), mode, 0, &V, nullptr, nullptr, nullptr);
    lat.assign((size_t)V * V, 0);
    bw.assign(V, 0);
    bw_dn.assign(V, 0);
    if ((st = gs_links_from_gml(gml.c_str(), mode, V, &V, lat.data(), bw.data(), bw_dn.data())) != GS_OK) {
      fprintf(stderr, "cannot read %s (%d)\n", gml.c_str(), st);
      return 1;
    }
    stages = V;
    stage_of_peer.assign(cfg.peers, 0);
    if ((st = gs_shadow_hosts(yaml.c_str(), cfg.peers, stage_of_peer.data())) != GS_OK) {
      fprintf(stderr, "cannot place the %u peers with %s (%d)\n", cfg.peers, yaml.c_str(), st);
      return 1;
    }
  } else {
    st = gs_topogen_links(stages, bl, bh, ll, lh, mode, lat.data(), bw.data());
    if (st != GS_OK) { fprintf(stderr, "invalid topogen parameters\n"); return 1; }
    bw_dn = bw;
  }

  gs_ctx* ctx = nullptr;
  if ((st = gs_create(&cfg, &ctx)) != GS_OK) return die(nullptr, st, "gs_create");
  if ((st = gs_set_links(ctx, stages, lat.data(), bw.data(), bw_dn.data(),
                         stage_of_peer.empty() ? nullptr : stage_of_peer.data())) != GS_OK)
    return die(ctx, st, "gs_set_links");
  const bool counters = !shadowlog.empty() || !metrics.empty();
  if (counters && (st = gs_set_traffic(ctx, 1)) != GS_OK) return die(ctx, st, "gs_set_traffic");
  if ((st = gs_build_topology(ctx)) != GS_OK) return die(ctx, st, "gs_build_topology");
  uint32_t epochs = 0;
  if ((st = gs_mesh_converge(ctx, max_hb, &epochs)) != GS_OK) return die(ctx, st, "gs_mesh_converge");

  std::vector<gs_publish> sched;
  if (!schedule.empty()) {  // an explicit publish schedule stands in for the HTTP injector
    uint64_t rows = 0;
    st = gs_read_schedule(schedule.c_str(), nullptr, 0, &rows);
    if (st != GS_OK && st != GS_ERANGE) { fprintf(stderr, "malformed schedule %s\n", schedule.c_str()); return die(ctx, st, "gs_read_schedule"); }
    sched.resize(rows);
    if ((st = gs_read_schedule(schedule.c_str(), sched.data(), rows, &rows)) != GS_OK) return die(ctx, st, "gs_read_schedule");
    n_msgs = (uint32_t)rows;
  } else {
    uint64_t t0_ns = t0_s * 1000000000ull;
    gs_injector inj;
    if (!yaml.empty() && gs_shadow_injector(yaml.c_str(), &inj) == GS_OK) {  // traffic_sync.py args (topogen.py:125-136)
      if (!set_size) msg_size = inj.msg_size;
      if (!set_msgs) n_msgs = inj.messages;
      if (!set_delay && inj.delay_ns) delay_ms = inj.delay_ns / 1000000ull;
      if (!set_t0) t0_ns = 946684800000000000ull + inj.start_ns;  // Shadow epoch + the controller's start_time
    }
    sched.resize(n_msgs);
    gs_schedule_runsh(n_msgs, cfg.peers, publisher, rotation, t0_ns + http_us * 1000ull, delay_ms * 1000000ull,
                      msg_size, sched.data());
  }
  Stream strm;
  strm.sched = sched.data();
  strm.self_log = cfg.self_log != 0;
  if (!latencies.empty() && (st = gs_log_open(&cfg, latencies.c_str(), &strm.log)) != GS_OK)
    return die(ctx, st, "gs_log_open");
  gs_result_sink sink{};
  sink.want = GS_WANT_LAT_MS;  // the logged latency, streamed through on_lat
  sink.on_lat = on_lat;
  sink.user = &strm;
  sink.block_msgs = 16;
  st = gs_run(ctx, sched.data(), n_msgs, &sink);
  if (st == GS_ERANGE && strstr(gs_last_error(ctx), "GS_WANT_LAT_MS")) {
    // a latency the u16 stream cannot carry: the same run again (it is
    // deterministic) through the u64 completion times, the log from the start
    if (strm.log) gs_log_close(strm.log);
    strm.log = nullptr;
    strm.st = GS_OK;
    strm.hist_ms.clear();
    if (!latencies.empty() && (st = gs_log_open(&cfg, latencies.c_str(), &strm.log)) != GS_OK)
      return die(ctx, st, "gs_log_open");
    gs_reset_stats(ctx);  // (also restarts the per-peer traffic counters)
    gs_result_sink wide{};
    wide.want = GS_WANT_T_COMPLETE;
    wide.on_block = on_block;
    wide.user = &strm;
    wide.block_msgs = 16;
    st = gs_run(ctx, sched.data(), n_msgs, &wide);
  }
  if (st != GS_OK) return die(ctx, st, "gs_run");
  if (strm.log && ((st = gs_log_close(strm.log)) != GS_OK || (st = strm.st) != GS_OK))
    return die(ctx, st, "gs_log_write");
  gs_stats s;
  gs_get_stats(ctx, &s);
  uint64_t n = 0;
  for (uint64_t c : strm.hist_ms) n += c;
  fprintf(stderr,
          "peers=%u mesh_epochs=%u messages=%llu deliveries=%llu frag_deliveries=%llu "
          "relaxations=%llu gossip_iwant=%llu latency_ms p50=%llu p95=%llu max=%llu\n",
          cfg.peers, epochs, (unsigned long long)s.messages, (unsigned long long)s.deliveries,
          (unsigned long long)s.frag_deliveries, (unsigned long long)s.relaxations,
          (unsigned long long)s.gossip_iwant, (unsigned long long)pct(strm.hist_ms, n, 50),
          (unsigned long long)pct(strm.hist_ms, n, 95), (unsigned long long)pct(strm.hist_ms, n, 100));
  if (counters) {
    std::vector<uint64_t> tr((size_t)cfg.peers * GS_TRAFFIC_COLS), row((size_t)cfg.peers + 1);
    std::vector<uint8_t> mc(cfg.peers);
    if ((st = gs_get_traffic(ctx, tr.data())) != GS_OK) return die(ctx, st, "gs_get_traffic");
    if ((st = gs_get_csr(ctx, row.data(), nullptr, nullptr)) != GS_OK) return die(ctx, st, "gs_get_csr");
    if ((st = gs_get_mesh(ctx, nullptr, mc.data())) != GS_OK) return die(ctx, st, "gs_get_mesh");
    const uint64_t end_s = sched.empty() ? 0 : (sched.back().t_pub_ns / 1000000000ull) - 946684800ull + 1;
    if (!shadowlog.empty() && (st = gs_write_shadow_heartbeat(shadowlog.c_str(), cfg.peers, tr.data(), end_s)) != GS_OK)
      return die(ctx, st, "gs_write_shadow_heartbeat");
    if (!metrics.empty() && (st = gs_write_node_metrics(&cfg, metrics.c_str(), row.data(), mc.data(), tr.data())) != GS_OK)
      return die(ctx, st, "gs_write_node_metrics");
  }
  gs_destroy(ctx);
  return 0;
}
