// Launch floor of back-to-back small kernels on gfx950 (what bounds the churn
// epochs' 3 x 1024 k_ev_step launches per config #3 batch): per-launch time of
// an empty kernel, a kernel whose first wave reads 64 bytes per block and
// syncs (k_ev_step's row test), by grid size; 1000 launches each, HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 -o scripts/bin/ubench_launch scripts/ubench_launch.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_empty(uint32_t* out) {
  if (threadIdx.x == 999) out[0] = 1;  // never true: keeps the kernel non-trivial to the compiler
}

__global__ __launch_bounds__(256) void k_test_sync(const uint8_t* flags, uint32_t n, uint32_t* out) {
  __shared__ uint32_t nact;
  const uint32_t u = blockIdx.x * 64 + threadIdx.x;
  if (threadIdx.x < 64) {
    const bool on = u < n && flags[u];
    const uint64_t b = __ballot(on);
    if (threadIdx.x == 0) nact = (uint32_t)__popcll(b);
  }
  __syncthreads();
  if (nact > 1000) out[blockIdx.x] = nact;  // never
}

// grid-stride form: each wave tests its own 64-row chunks, no block sync
__global__ __launch_bounds__(256) void k_test_stride(const uint8_t* flags, uint32_t n, uint32_t* out) {
  const uint32_t nch = (n + 63) / 64;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (uint32_t ch = wave; ch < nch; ch += nw) {
    const uint32_t u = ch * 64 + (threadIdx.x & 63);
    const bool on = u < n && flags[u];
    const uint64_t b = __ballot(on);
    if (__popcll(b) > 1000) out[ch] = 1;  // never
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const uint32_t N = 100000;
  uint8_t* flags;
  uint32_t* out;
  CK(hipMalloc(&flags, N));
  CK(hipMalloc(&out, 4 * N));
  CK(hipMemset(flags, 0, N));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int R = 1000;
  auto run = [&](const char* name, unsigned grid, auto fn) {
    for (int i = 0; i < 50; i++) fn(grid);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < R; i++) fn(grid);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-14s grid %6u: %7.2f us per launch\n", name, grid, ms * 1e3 / R);
    return 0;
  };
  for (unsigned g : {64u, 256u, 512u, 1024u, 1563u, 4096u}) {
    run("empty", g, [&](unsigned gr) { k_empty<<<gr, 256>>>(out); });
    run("test+sync", g, [&](unsigned gr) { k_test_sync<<<gr, 256>>>(flags, gr * 64 < N ? gr * 64 : N, out); });
    run("test-stride", g, [&](unsigned gr) { k_test_stride<<<gr, 256>>>(flags, N, out); });
  }
  return 0;
}
