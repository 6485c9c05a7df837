// Issue-rate micro-benchmark of dropout-hash candidates on gfx950: each lane runs 8 independent
// hash chains for ITERS rounds; one wave per SIMD (4 waves per workgroup, one workgroup per CU).
// Reports cycles per wave-instruction-equivalent per hash (s_memtime around the loop).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 4096
__device__ __forceinline__ uint32_t h_lowbias(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t h_wang(uint32_t x) {
  x = (x ^ 61u) ^ (x >> 16); x *= 9u; x ^= x >> 4; x *= 0x27d4eb2du; x ^= x >> 15; return x;
}
__device__ __forceinline__ uint32_t h_mul24(uint32_t x) {
  x ^= x >> 16; x = __umul24(x, 0x2C1B3Cu) + (x >> 24) ; x ^= x >> 13;
  x = __umul24(x, 0x94D049u) + (x >> 24); x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t h_mullo_only(uint32_t x) { return x * 0x7FEB352Du; }
__device__ __forceinline__ uint32_t h_xor_only(uint32_t x) { return (x ^ 0x7FEB352Du) + 3u; }
template <int V>
__global__ void bench(uint32_t* out, long long* cyc) {
  uint32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 8 + j + blockIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (V == 0) a[j] = h_lowbias(a[j]);
      if (V == 1) a[j] = h_wang(a[j]);
      if (V == 2) a[j] = h_mul24(a[j]);
      if (V == 3) a[j] = h_mullo_only(a[j]);
      if (V == 4) a[j] = h_xor_only(a[j]);
    }
  }
  long long t1 = clock64();
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  uint32_t* o; long long* c; hipMalloc(&o, 256 * 256 * 4); hipMalloc(&c, 8);
  const char* names[] = {"lowbias32 (2 mul_lo)", "wang (1 mul_lo)", "mul24 x2", "mul_lo alone", "xor+add alone"};
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) bench<0><<<256, 256>>>(o, c);
      if (v == 1) bench<1><<<256, 256>>>(o, c);
      if (v == 2) bench<2><<<256, 256>>>(o, c);
      if (v == 3) bench<3><<<256, 256>>>(o, c);
      if (v == 4) bench<4><<<256, 256>>>(o, c);
      hipDeviceSynchronize();
    }
    long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    printf("%-24s %.2f cycles per wave-hash (one wave per SIMD)\n", names[v], (double)cy / (ITERS * 8.0));
  }
  return 0;
}
