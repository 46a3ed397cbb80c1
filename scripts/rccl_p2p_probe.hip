// rccl_p2p_probe.hip — does RCCL's point-to-point path (ncclSend/ncclRecv to
// self on a one-rank communicator, the transfer gs_run_partitioned makes with
// one rank) deliver single transfers past 2^31 bytes intact? (VERDICT r02
// item 1c) Each case fills the send buffer with a position
// hash, zeroes the receive buffer, runs one grouped send/recv of `count`
// elements of `type` and counts the 8-byte words that differ.
//
//   hipcc --offload-arch=gfx950 -O2 -o rccl_p2p_probe rccl_p2p_probe.hip -lrccl
//   ./rccl_p2p_probe            # prints one JSON line per case
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)
#define NC(x)                                                                  \
  do {                                                                         \
    ncclResult_t r_ = (x);                                                     \
    if (r_ != ncclSuccess) { fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r_)); exit(1); } \
  } while (0)

__device__ __forceinline__ uint64_t mixw(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = mixw(i);
}

// mismatches[0] = words that differ, [1] = first differing word index, [2] = last
__global__ void k_check(const uint64_t* p, uint64_t n, unsigned long long* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (p[i] != mixw(i)) {
      atomicAdd(&out[0], 1ull);
      atomicMin(&out[1], (unsigned long long)i);
      atomicMax(&out[2], (unsigned long long)i);
    }
}

int main() {
  CK(hipSetDevice(0));
  ncclUniqueId id;
  NC(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NC(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const uint64_t maxb = (5ull << 30);  // 5 GiB buffers
  uint64_t *snd = nullptr, *rcv = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc((void**)&snd, maxb));
  CK(hipMalloc((void**)&rcv, maxb));
  CK(hipMalloc((void**)&out, 24));
  k_fill<<<4096, 256, 0, s>>>(snd, maxb / 8);
  struct Case { uint64_t bytes; ncclDataType_t t; int esz; const char* tn; };
  const Case cases[] = {
      {(1ull << 31) - 4096, ncclUint8, 1, "uint8"},
      {(1ull << 31), ncclUint8, 1, "uint8"},
      {(1ull << 31) + 4096, ncclUint8, 1, "uint8"},
      {3ull << 30, ncclUint8, 1, "uint8"},
      {(1ull << 32) + (1ull << 29), ncclUint8, 1, "uint8"},
      {(1ull << 31) + 4096, ncclUint64, 8, "uint64"},
      {3ull << 30, ncclUint64, 8, "uint64"},
      {(1ull << 32) + (1ull << 29), ncclUint64, 8, "uint64"},
      {(1ull << 30), ncclUint8, 1, "uint8"},
  };
  for (const Case& c : cases) {
    const uint64_t words = c.bytes / 8, count = c.bytes / c.esz;
    CK(hipMemsetAsync(rcv, 0, maxb, s));
    unsigned long long init[3] = {0, ~0ull, 0};
    CK(hipMemcpyAsync(out, init, 24, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    NC(ncclGroupStart());
    NC(ncclSend(snd, count, c.t, 0, comm, s));
    NC(ncclRecv(rcv, count, c.t, 0, comm, s));
    NC(ncclGroupEnd());
    k_check<<<4096, 256, 0, s>>>(rcv, words, out);
    unsigned long long h[3];
    CK(hipMemcpyAsync(h, out, 24, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    // words past the transfer must still be zero (no write beyond count)
    printf("{\"bytes\": %llu, \"type\": \"%s\", \"count\": %llu, \"count_gt_int32\": %s, \"bad_words\": %llu, "
           "\"first_bad_byte\": %lld, \"last_bad_byte\": %lld}\n",
           (unsigned long long)c.bytes, c.tn, (unsigned long long)count, count > 0x7FFFFFFFull ? "true" : "false",
           h[0], h[0] ? (long long)(h[1] * 8) : -1LL, h[0] ? (long long)(h[2] * 8 + 7) : -1LL);
    fflush(stdout);
  }
  NC(ncclCommDestroy(comm));
  return 0;
}
