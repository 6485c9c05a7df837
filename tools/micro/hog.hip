// Interference probe (tools/hog_bench.py): NB workgroups that each hold a CU's worth of
// resources (64 KB LDS, 256 threads) and spin for `cycles` shader clocks on a side stream, the way
// RCCL's all-reduce workgroups hold CUs while the compute stream runs the backward GEMMs.
#include <hip/hip_runtime.h>
__global__ __launch_bounds__(256) void hog_kernel(long long cycles, int* sink) {
  __shared__ int pad[16384];
  pad[threadIdx.x] = threadIdx.x;
  const long long t0 = clock64();
  int acc = 0;
  while (clock64() - t0 < cycles) acc += pad[(threadIdx.x + acc) & 255];
  if (acc == 0x7fffffff) sink[0] = acc;
}
extern "C" int hog_launch(int nblk, long long cycles, void* sink, void* stream) {
  hipLaunchKernelGGL(hog_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, cycles, (int*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
