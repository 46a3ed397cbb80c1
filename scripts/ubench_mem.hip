// ubench_mem.hip — random 8-byte access rates on gfx950, to size the relax
// kernels. Standalone: hipcc -O3 --offload-arch=gfx950.
//
// Every lane makes ITERS accesses at hashed indices into a u64 table of T
// bytes; a "cluster" of C consecutive lanes shares one 64-B sector (C = 1:
// every lane its own random sector). Ops: load, store, atomicMin (agent
// scope = default), atomicMin at workgroup scope, read + conditional
// atomicMin (the relax filter), returning atomicMin. Prints G accesses/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int ITERS = 64;

template <int OP>
__global__ __launch_bounds__(256) void k_rand(uint64_t* __restrict__ t, uint64_t mask_sectors, int cl_log,
                                              uint64_t salt, uint64_t* sink) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t grp = g >> cl_log, sub = g & ((1u << cl_log) - 1);
  uint64_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < ITERS; i++) {
    const uint64_t h = mix(grp * 0x100000001B3ull + i + salt);
    const uint64_t idx = ((h & mask_sectors) << 3) + sub;  // sector base + lane within it
    const uint64_t v = h | 1;
    if constexpr (OP == 0) acc += t[idx];
    else if constexpr (OP == 1) t[idx] = v;
    else if constexpr (OP == 2) atomicMin((unsigned long long*)&t[idx], (unsigned long long)v);
    else if constexpr (OP == 3)
      __hip_atomic_fetch_min((unsigned long long*)&t[idx], (unsigned long long)v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    else if constexpr (OP == 4) {
      if (v < t[idx]) atomicMin((unsigned long long*)&t[idx], (unsigned long long)v);
    } else if constexpr (OP == 5)
      acc += atomicMin((unsigned long long*)&t[idx], (unsigned long long)v);  // returning
  }
  if (acc == 0x1234567) sink[0] = acc;
}

static const char* NAMES[] = {"load", "store", "amin_agent", "amin_wg", "read_filter_amin", "amin_ret"};

template <int OP>
float run(uint64_t* t, uint64_t bytes, int cl_log, uint64_t* sink, unsigned grid) {
  const uint64_t sectors = bytes / 64;  // power of two
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_rand<OP><<<grid, 256>>>(t, sectors - 1, cl_log, 1, sink);  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int reps = 3;
  for (int r = 0; r < reps; r++) k_rand<OP><<<grid, 256>>>(t, sectors - 1, cl_log, 7 + r, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  const double acc = (double)grid * 256 * ITERS * reps;
  return (float)(acc / (ms * 1e-3) / 1e9);
}

int main() {
  const uint64_t maxb = 8ull << 30;
  uint64_t* t;
  uint64_t* sink;
  CK(hipMalloc(&t, maxb));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(t, 0xFF, maxb));
  const unsigned grid = 256 * 64;  // 4M lanes x 64 accesses = 268M per launch
  const uint64_t sizes[] = {64ull << 20, 256ull << 20, 1ull << 30, 8ull << 30};
  const int cls[] = {0, 2, 3};
  printf("{\"unit\": \"G accesses/s\", \"rows\": [\n");
  bool first = true;
  for (uint64_t sz : sizes)
    for (int cl : cls) {
      float r[6];
      r[0] = run<0>(t, sz, cl, sink, grid);
      r[1] = run<1>(t, sz, cl, sink, grid);
      CK(hipMemset(t, 0xFF, sz));
      r[2] = run<2>(t, sz, cl, sink, grid);
      CK(hipMemset(t, 0xFF, sz));
      r[3] = run<3>(t, sz, cl, sink, grid);
      CK(hipMemset(t, 0xFF, sz));
      r[4] = run<4>(t, sz, cl, sink, grid);
      CK(hipMemset(t, 0xFF, sz));
      r[5] = run<5>(t, sz, cl, sink, grid);
      for (int o = 0; o < 6; o++) {
        printf("%s{\"op\": \"%s\", \"table_MB\": %llu, \"lanes_per_sector\": %d, \"rate\": %.2f}", first ? "" : ",\n",
               NAMES[o], (unsigned long long)(sz >> 20), 1 << cl, r[o]);
        first = false;
      }
      fflush(stdout);
    }
  printf("\n]}\n");
  CK(hipFree(t));
  CK(hipFree(sink));
  return 0;
}
