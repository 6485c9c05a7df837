// VALU issue-rate micro-benchmark on gfx950: cycles per wave-instruction of common epilogue / softmax /
// dropout instructions, at 1 and 2 waves per SIMD (256- or 512-thread workgroups, one per CU).
// Each lane runs 8 independent chains of the instruction (inline asm: nothing is folded), ITERS times.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 2048
#define CHAIN8(INS)                                                                                  \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
               INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"      \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
               : "v"(k))
#define CHAIN8U(INS)                                                                                 \
  asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS " %4, %4\n\t" \
               INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"                                      \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]))
#define CHAIN8P(INS)                                                                                 \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
               INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"      \
               : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7]) \
               : "v"(kp))
#define CHAIN8F(INS)                                                                                 \
  asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" INS " %3, %3, %8, %8\n\t" \
               INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t" INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"      \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
               : "v"(k))
typedef __attribute__((ext_vector_type(2))) float f2;
template <int V>
__global__ void bench(uint32_t* out, long long* cyc) {
  uint32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 8 + j + blockIdx.x + 0x3f800000u;
  uint32_t k = threadIdx.x | 0x3f000000u;
  f2 p[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = f2{(float)j, 1.f};
  f2 kp = f2{0.5f, 0.25f};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if (V == 0) CHAIN8("v_add_u32");
    if (V == 1) CHAIN8("v_mul_lo_u32");
    if (V == 2) CHAIN8U("v_exp_f32");
    if (V == 3) CHAIN8("v_mul_f32");
    if (V == 4) CHAIN8U("v_rcp_f32");
    if (V == 5) CHAIN8("v_xor_b32");
    if (V == 6) CHAIN8("v_mul_u32_u24");
    if (V == 7) CHAIN8("v_mul_hi_u32");
    if (V == 8) CHAIN8("v_cvt_pk_bf16_f32");
    if (V == 9) CHAIN8("v_min_f32");
    if (V == 10) CHAIN8("v_lshrrev_b32");
    if (V == 11) CHAIN8P("v_pk_mul_f32");
    if (V == 12) CHAIN8P("v_pk_add_f32");
    if (V == 13) CHAIN8F("v_fma_f32");
    if (V == 14) CHAIN8F("v_bfe_u32");
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= a[j] ^ __float_as_uint(p[j][0] + p[j][1]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
template <int V>
static double run(int threads, uint32_t* o, long long* c) {
  hipLaunchKernelGGL(bench<V>, dim3(256), dim3(threads), 0, 0, o, c);
  hipLaunchKernelGGL(bench<V>, dim3(256), dim3(threads), 0, 0, o, c);
  hipDeviceSynchronize();
  long long cy;
  hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  return (double)cy / (ITERS * 8.0);
}
int main() {
  uint32_t* o;
  long long* c;
  hipMalloc(&o, 256 * 1024 * 4);
  hipMalloc(&c, 8);
  const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_exp_f32", "v_mul_f32", "v_rcp_f32", "v_xor_b32",
                         "v_mul_u32_u24", "v_mul_hi_u32", "v_cvt_pk_bf16_f32", "v_min_f32", "v_lshrrev_b32", "v_pk_mul_f32", "v_pk_add_f32", "v_fma_f32", "v_bfe_u32"};
  for (int t : {256, 512, 1024, 2048}) {
    double r[15] = {run<0>(t, o, c), run<1>(t, o, c), run<2>(t, o, c), run<3>(t, o, c), run<4>(t, o, c), run<5>(t, o, c),
                    run<6>(t, o, c), run<7>(t, o, c), run<8>(t, o, c), run<9>(t, o, c), run<10>(t, o, c),
                    run<11>(t, o, c), run<12>(t, o, c), run<13>(t, o, c), run<14>(t, o, c)};
    for (int v = 0; v < 15; ++v)
      printf("%d waves/SIMD  %-20s %6.2f cycles per wave-instruction per wave (SIMD: %.2f)\n", t / 256, names[v], r[v],
             r[v] / (t / 256));
  }
  return 0;
}
