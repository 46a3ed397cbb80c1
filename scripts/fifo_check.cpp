// Host check of uplink_start's closed form (gs_relax_kernel.h): the prefix-sum FIFO
// equals the sequential (key, fragment) fold on random groups.  g++ -O2 scripts/fifo_check.cpp && ./a.out
#include <cstdint>
#include <cstdio>
#include <random>
const uint64_t INF = ~0ull;
int main() {
  std::mt19937_64 R(7);
  for (int it = 0; it < 2000000; it++) {
    const int FP = 1 << (1 + R() % 4);
    uint64_t kk[16]; uint32_t nn[16]; const uint32_t ser = R() % 5000; const int ts = 3;
    for (int g = 0; g < FP; g++) {
      kk[g] = (R() % 3 == 0) ? INF : ((R() % 40) << ts) | (R() & 7);
      if (R() % 5 == 0 && g) kk[g] = kk[g - 1];
      nn[g] = R() % 17;
    }
    const uint64_t cb0 = R() % 3 ? R() % 60 : 0;
    // sequential
    uint64_t st1[16] = {}, cb = cb0, pk = 0; int pg = -1; bool any = false;
    for (int g = 0; g < FP; g++) any |= kk[g] != INF;
    for (int i = 0; i < FP && any; i++) {
      uint64_t bk = INF; int bg = FP; uint32_t bn = 0;
      for (int g = 0; g < FP; g++) {
        bool after = kk[g] > pk || (kk[g] == pk && g > pg), better = kk[g] < bk || (kk[g] == bk && g < bg);
        if (kk[g] != INF && after && better) { bk = kk[g]; bg = g; bn = nn[g]; }
      }
      if (bg == FP) continue;
      uint64_t tb = bk >> ts, s = tb > cb ? tb : cb;
      st1[bg] = s; cb = s + (uint64_t)bn * ser; pk = bk; pg = bg;
    }
    // closed form
    uint64_t P[16], tot = 0;
    for (int i = 0; i < FP; i++) {
      P[i] = 0;
      if (kk[i] != INF) tot += (uint64_t)nn[i] * ser;
      for (int g = 0; g < FP; g++)
        if (kk[g] != INF && (kk[g] < kk[i] || (kk[g] == kk[i] && g < i))) P[i] += (uint64_t)nn[g] * ser;
    }
    for (int i = 0; i < FP; i++) {
      if (kk[i] == INF) continue;
      uint64_t s = cb0 + P[i];
      for (int g = 0; g < FP; g++)
        if (kk[g] != INF && (kk[g] < kk[i] || (kk[g] == kk[i] && g <= i))) {
          const uint64_t c = (kk[g] >> ts) + P[i] - P[g];
          s = c > s ? c : s;
        }
      if (s != st1[i]) { printf("start mismatch it %d\n", it); return 1; }
    }
    if (any) {
      uint64_t e = cb0 + tot;
      for (int g = 0; g < FP; g++)
        if (kk[g] != INF) { const uint64_t c = (kk[g] >> ts) + tot - P[g]; e = c > e ? c : e; }
      if (e != cb) { printf("end mismatch it %d\n", it); return 1; }
    }
  }
  puts("ok");
}
