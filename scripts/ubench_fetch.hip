// ubench_fetch.hip — calibrates rocprofv3 FETCH_SIZE against known bytes for the
// read shapes of the list pass and the churn pass ("calibrate the
// PMC read factor on a micro-kernel with the same short random-read shape").
// Standalone: hipcc -O3 --offload-arch=gfx950 -o ubench_fetch ubench_fetch.hip
//
// Each wave reads SEGS segments; a segment is a run of n records (8 B or 16 B
// per lane, lane i < n reads record i) at a hashed, row-aligned base in a 4 GiB
// table (past the 256 MiB Infinity Cache), as k_lpull reads a neighbour's 8-B
// records and the churn pass its 16-B records. One dispatch per (width, n);
// the program prints, in dispatch order, the bytes the lanes asked for and the
// 128-B lines they touch. FETCH_SIZE (KB) of the same dispatch divided into
// those gives the factor for that shape. The last two dispatches are the
// guide's reference shape (16 B per lane, fully coalesced stream) and the same
// stream at 8 B per lane.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));             \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr uint32_t SEGS = 64;       // segments per wave
constexpr uint64_t ROWB = 4096;     // row pitch in bytes (a row holds up to 256 16-B records)

template <int W>  // bytes per lane: 8 or 16
__global__ __launch_bounds__(256) void k_seg(const uint8_t* __restrict__ t, uint64_t rows, uint32_t n, uint64_t salt,
                                             uint64_t* sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  uint64_t acc = 0;
  for (uint32_t s = 0; s < SEGS; s++) {
    const uint64_t row = mix(wave * SEGS + s + salt) % rows;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      if (i < n) {
        const uint8_t* p = t + row * ROWB + (uint64_t)i * W;
        if constexpr (W == 16) {
          const uint4 v = *reinterpret_cast<const uint4*>(p);
          acc += v.x ^ v.y ^ v.z ^ v.w;
        } else {
          acc += *reinterpret_cast<const uint64_t*>(p);
        }
      }
    }
  }
  if (acc == 0x1234567) sink[0] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ t, uint64_t bytes, uint64_t* sink) {
  uint64_t acc = 0;
  const uint64_t n = bytes / W, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint8_t* p = t + i * W;
    if constexpr (W == 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    } else {
      acc += *reinterpret_cast<const uint64_t*>(p);
    }
  }
  if (acc == 0x1234567) sink[0] = acc;
}

int main() {
  const uint64_t TB = 4ull << 30, rows = TB / ROWB;
  uint8_t* t = nullptr;
  uint64_t* sink = nullptr;
  CK(hipMalloc(&t, TB));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(t, 1, TB));
  CK(hipDeviceSynchronize());
  const uint32_t waves = 256 * 64;  // 1M segments per dispatch
  const uint32_t blocks = waves / 4;
  printf("dispatch,width,n,segments,bytes_asked,lines128_touched,ms\n");
  int d = 0;
  const uint32_t ns[] = {1, 4, 8, 16, 24, 32, 64, 128};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int W : {8, 16})
    for (uint32_t n : ns) {
      CK(hipEventRecord(e0, 0));
      if (W == 8) k_seg<8><<<blocks, 256>>>(t, rows, n, 977 * d, sink);
      else k_seg<16><<<blocks, 256>>>(t, rows, n, 977 * d, sink);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const uint64_t segs = (uint64_t)waves * SEGS, asked = segs * n * W;
      const uint64_t lines = segs * ((n * W + 127) / 128);  // row bases are 4096-B aligned
      printf("%d,%d,%u,%llu,%llu,%llu,%.3f\n", d++, W, n, (unsigned long long)segs, (unsigned long long)asked,
             (unsigned long long)lines, ms);
    }
  for (int W : {16, 8}) {
    const uint64_t bytes = 2ull << 30;
    CK(hipEventRecord(e0, 0));
    if (W == 16) k_stream<16><<<4096, 256>>>(t, bytes, sink);
    else k_stream<8><<<4096, 256>>>(t, bytes, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%d,%d,stream,1,%llu,%llu,%.3f\n", d++, W, (unsigned long long)bytes, (unsigned long long)(bytes / 128), ms);
  }
  CK(hipFree(t));
  CK(hipFree(sink));
  return 0;
}
