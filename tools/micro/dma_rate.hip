// L2/HBM -> LDS fetch rate per CU with the 8-phase GEMM's load pattern and no MFMA work.
// Question (round-5 counters, profiles/r05ap_gemm_mfma_counters.txt): the 256^2 x 64 GEMM moves 64 KB
// into LDS per K-tile per CU; at the measured 4,480 cycles per K-tile that is 14.6 B/cycle/CU. Is the
// main loop at the chip's LDS-DMA fetch rate (then fewer barriers cannot help), or well under it?
// Persistent grid, one 512-thread workgroup per CU, 2 x 64 KB LDS stages, each wave issuing the
// 4 A + 4 B pieces of 1 KB (8 rows x 128 B) per K-tile exactly as the GEMM's units do, waiting for the
// previous K-tile's pieces (vmcnt(8)) and crossing one barrier per K-tile.
//   mode 0: fc1 shape (A [50432, 768] bf16, B [3072, 768]), tiles t -> (t / 12, t % 12), K 768
//   mode 1: every workgroup fetches tile (0, 0): L2-resident source
//   mode 2: as mode 0 with no prefetch (vmcnt(0) right after issue): latency-bound reference
//   mode 3: fc2 shape (A [50432, 3072], B [768, 3072]), tiles t -> (t / 3, t % 3), K 3072
//   modes 4 / 5: fc1 / fc2 shape with each row block's tiles on one XCD
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/dma_rate tools/micro/dma_rate.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__device__ u32x4 rsrc4(const void* base) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, 0x7FFFFFF0u, 0x00020000u};
}
__device__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ void dma16(const void* lds, const u32x4& rs, uint32_t voff) {
  uint32_t t;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(t)
      : "s"(lds_addr(lds)), "v"(voff), "s"(rs)
      : "memory");
}

template <int MODE>
__global__ __launch_bounds__(512) void dma_kernel(const char* A, const char* B, int K, int tiles_n, int tiles,
                                                  unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const u32x4 ra = rsrc4(A), rb = rsrc4(B);
  const int ktiles = K / 64;
  const uint32_t row_b = (uint32_t)K * 2;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // modes 4, 5: the tiles of row block tm all on XCD tm % 8 (a round-robin dispatch puts workgroup b
  // on XCD b % 8), so an A row block is fetched into one L2 only
  const bool xg = MODE >= 4;
  const int xcd = blockIdx.x & 7, tms = tiles / tiles_n;
  const int first = xg ? blockIdx.x >> 3 : blockIdx.x, stride = xg ? gridDim.x >> 3 : gridDim.x;
  const int items = xg ? ((tms - xcd + 7) / 8) * tiles_n : tiles;
  for (int t = first; t < items; t += stride) {
    const int tm = MODE == 1 ? 0 : xg ? xcd + 8 * (t / tiles_n) : t / tiles_n;
    const int tn = MODE == 1 ? 0 : t % tiles_n;
    for (int kt = 0; kt < ktiles; ++kt) {
      char* st = smem + (kt & 1) * 65536;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int piece = wave * 4 + p;  // 32 pieces of 8 rows = 256 rows
        const uint32_t row = piece * 8 + (lane >> 3);
        const uint32_t col = kt * 128 + (lane & 7) * 16;
        dma16(st + piece * 1024, ra, (tm * 256 + row) * row_b + col);
        dma16(st + 32768 + piece * 1024, rb, (tn * 256 + row) * row_b + col);
      }
      if (MODE == 2)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    unsigned long long* o = cyc + blockIdx.x;
    *o = t1 - t0;  // vector store
  }
}

template <int MODE>
int run(const char* name, const char* A, const char* B, int K, int tiles_n, int tiles, int grid,
        unsigned long long* dcyc) {
  CK(hipFuncSetAttribute((const void*)dma_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(dma_kernel<MODE>, dim3(grid), dim3(512), 131072, 0, A, B, K, tiles_n, tiles, dcyc);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(dma_kernel<MODE>, dim3(grid), dim3(512), 131072, 0, A, B, K, tiles_n, tiles, dcyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  std::vector<unsigned long long> c(grid);
  CK(hipMemcpy(c.data(), dcyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double mc = 0, xc = 0;
  for (auto v : c) {
    mc += v;
    xc = v > xc ? v : xc;
  }
  mc /= grid;
  const double bytes = (double)tiles * (K / 64) * 65536.0;
  const double per_cu = bytes / grid;
  printf("%-34s %8.1f us  %6.2f TB/s  cycles/WG mean %9.0f max %9.0f  %5.2f B/cycle/CU (mean)  "
         "%6.0f cycles per 64 KB K-tile  clock %.2f GHz\n",
         name, ms * 1e3, bytes / (ms * 1e-3) / 1e12, mc, xc, per_cu / mc,
         mc / ((double)tiles * (K / 64) / grid), xc / (ms * 1e6));
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  const int M = 50432;
  char *A, *B;
  CK(hipMalloc(&A, (size_t)M * 3072 * 2));
  CK(hipMalloc(&B, (size_t)3072 * 768 * 2));
  CK(hipMemset(A, 0x3c, (size_t)M * 3072 * 2));
  CK(hipMemset(B, 0x3c, (size_t)3072 * 768 * 2));
  unsigned long long* dcyc;
  CK(hipMalloc(&dcyc, grid * sizeof(unsigned long long)));
  printf("CUs %d\n", grid);
  if (run<0>("fc1 shape, prefetch depth 1", A, B, 768, 12, 197 * 12, grid, dcyc)) return 1;
  if (run<1>("tile (0,0) only, L2-resident", A, B, 768, 12, 197 * 12, grid, dcyc)) return 1;
  if (run<2>("fc1 shape, no prefetch", A, B, 768, 12, 197 * 12, grid, dcyc)) return 1;
  if (run<3>("fc2 shape, prefetch depth 1", A, B, 3072, 3, 197 * 3, grid, dcyc)) return 1;
  if (run<4>("fc1 shape, XCD-grouped rows", A, B, 768, 12, 197 * 12, grid, dcyc)) return 1;
  if (run<5>("fc2 shape, XCD-grouped rows", A, B, 3072, 3, 197 * 3, grid, dcyc)) return 1;
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(dcyc));
  return 0;
}
