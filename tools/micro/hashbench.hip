// Throughput of candidate dropout hashes (pairs/s): lowbias32 (2 x v_mul_lo_u32) vs 24-bit-multiply
// variants. Each thread hashes a stream of counters; results folded so nothing is eliminated.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return __umul24(a, b); }
__device__ __forceinline__ uint32_t h24(uint32_t x) {
  x ^= x >> 17; x = mul24(x, 0xed5ad5u) + (x >> 24);
  x ^= x >> 11; x = mul24(x, 0xac4c1bu) + (x >> 24);
  x ^= x >> 15; x = mul24(x, 0x31848bu) + (x >> 24);
  x ^= x >> 14; return x;
}
template <int K>
__global__ void bench(uint32_t* out, uint32_t seed, int iters) {
  uint32_t acc = 0, base = (blockIdx.x * blockDim.x + threadIdx.x) * 4096u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t x = (base + i * 8 + j) ^ seed;
      acc += K == 0 ? lowbias32(x) : (K == 1 ? h24(x) : x * 3u);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  uint32_t* d; hipMalloc(&d, 1 << 24);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int blocks = 256 * 16, threads = 256, iters = 256;
  const double n = (double)blocks * threads * iters * 8;
  for (int rep = 0; rep < 2; ++rep) {
    float ms[3];
#define RUN(K) hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(threads), 0, 0, d, 12345u, iters); hipEventRecord(a); \
    hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(threads), 0, 0, d, 12345u, iters); hipEventRecord(b); \
    hipEventSynchronize(b); hipEventElapsedTime(&ms[K], a, b);
    RUN(0) RUN(1) RUN(2)
    printf("lowbias32 %.1f Ghash/s   mul24x3 %.1f Ghash/s   baseline(add/mul3) %.1f G/s\n", n / ms[0] / 1e6,
           n / ms[1] / 1e6, n / ms[2] / 1e6);
  }
  return 0;
}
