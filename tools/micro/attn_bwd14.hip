// Performance prototype (not a product kernel, numerics unchecked): the attention backward of one
// (batch, head) unit at 4 waves per SIMD -- 14 waves of 16-key blocks, v_mfma_f32_16x16x32_bf16, <= 128
// VGPRs -- against the shipped attn_bwd_pers<7> (7 waves of 32-key blocks, 256 VGPRs). Same per-step
// structure: S = Q K^T and dP = dO V^T for (32 queries, the wave's 16 keys), softmax / dropout / dS on
// the VALU, dV^T += dO^T P and dK^T += Q^T dS (the permuted query order of the accumulator layout on both
// operands: no cross-lane moves), dS tile to LDS, barrier, dQ += dS K for the wave pair's query block
// and half of d, barrier. Non-persistent (one workgroup per unit), Dq precomputed, no bias-gradient
// partials. ViT-B/16 shape: B 256, N 197, H 12, dh 64.   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
#define DEV __device__ __forceinline__

constexpr int NB = 7, NQ = 32 * NB, IMG = NQ * 128, NW = 14;

DEV int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
DEV int img_off(int r, int c) { return r * 128 + ((c ^ swz(r)) << 4); }
DEV bf16x8 rd_row(const char* img, int r, int c) { return *(const bf16x8*)(img + img_off(r, c)); }
DEV bf16x8 cat8(short4_t a, short4_t b) {
  const u32x2 x = __builtin_bit_cast(u32x2, a), y = __builtin_bit_cast(u32x2, b);
  return __builtin_bit_cast(bf16x8, u32x4{x[0], x[1], y[0], y[1]});
}
// 4 x 16 block (rows row0 + {0..3}, columns c16 .. c16 + 15) of an image, transposed: lane j of its
// 16-lane group gets column c16 + j, rows row0 + {0..3}
DEV short4_t tr4(const char* img, int row0, int c16, int lane) {
  const int i = lane & 15;
  const int r = row0 + (i >> 2), col = c16 + 4 * (i & 3);
  const char* a = img + r * 128 + (((col >> 3) ^ swz(r)) << 4) + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a);
}
DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd14(
    const bf16* __restrict__ qkv, long ldq, const bf16* __restrict__ dout, long lddo, const float* __restrict__ lse,
    const float* __restrict__ dqv, const uint32_t* __restrict__ mask, bf16* __restrict__ dqkv, int N, int H,
    float scale, float sl2, float dscale) {
  __shared__ __attribute__((aligned(1024))) char lds[3 * IMG + NW * 1024 + 2 * NQ * 4];
  char* Qi = lds;
  char* Oi = lds + IMG;
  char* Ki = lds + 2 * IMG;
  char* Sall = lds + 3 * IMG;
  float* L = (float*)(Sall + NW * 1024);
  float* Dq = L + NQ;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, j16 = lane & 15;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, dh = 64, D = H * dh;
  // images: Q, dO, K rows [0, 224) (zero padded)
  for (int idx = threadIdx.x; idx < NQ * 8; idx += 64 * NW) {
    const int r = idx >> 3, c = idx & 7;
    bf16x8 q = {}, o = {}, k = {};
    if (r < N) {
      const long row = (long)b * N + r;
      q = *(const bf16x8*)(qkv + row * ldq + h * dh + c * 8);
      k = *(const bf16x8*)(qkv + row * ldq + D + h * dh + c * 8);
      o = *(const bf16x8*)(dout + row * lddo + h * dh + c * 8);
    }
    *(bf16x8*)(Qi + img_off(r, c)) = q;
    *(bf16x8*)(Oi + img_off(r, c)) = o;
    *(bf16x8*)(Ki + img_off(r, c)) = k;
  }
  for (int r = threadIdx.x; r < NQ; r += 64 * NW) {
    L[r] = r < N ? -lse[(long)bh * N + r] / scale : -INFINITY;
    Dq[r] = r < N ? dqv[(long)bh * N + r] : 0.f;
  }
  // this wave's keys: K / V as the B operand of S = Q K^T, dP = dO V^T (column = key, 8 d per lane group)
  const int key = 16 * w + j16;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    bf16x8 kk = {}, vv = {};
    if (key < N) {
      const long row = (long)b * N + key;
      kk = *(const bf16x8*)(qkv + row * ldq + D + h * dh + 32 * ks + 8 * g);
      vv = *(const bf16x8*)(qkv + row * ldq + 2 * D + h * dh + 32 * ks + 8 * g);
    }
    kf[ks] = kk;
    vf[ks] = vv;
  }
  __syncthreads();
  f32x4 dk[4] = {}, dv[4] = {}, dq[2][2] = {};
  const int jq = w >> 1, dhalf = w & 1;
#pragma unroll 1
  for (int i = 0; i < NB; ++i) {
    int qb = jq + i;
    if (qb >= NB) qb -= NB;
    {  // phase A
      f32x4 st[2], dp[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 l4 = *(const f32x4*)(L + qb * 32 + 16 * mt + 4 * g);
        st[mt] = l4;
        dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int row = qb * 32 + 16 * mt + j16;
          st[mt] = mfma16(rd_row(Qi, row, 4 * ks + g), kf[ks], st[mt]);
          dp[mt] = mfma16(rd_row(Oi, row, 4 * ks + g), vf[ks], dp[mt]);
        }
      }
      const uint32_t mw = mask ? mask[(((long)bh * NW + w) * NB + qb) * 64 + lane] : 0xFFFFFFFFu;
      f32x4 pd[2], ds[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 d4 = *(const f32x4*)(Dq + qb * 32 + 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = ex2(st[mt][r] * sl2);
          const uint32_t km = (uint32_t)((int32_t)(mw << (31 - (4 * mt + r))) >> 31);
          pd[mt][r] = __uint_as_float(__float_as_uint(p) & km);
          ds[mt][r] = p * fmaf(__uint_as_float(__float_as_uint(dp[mt][r]) & km), dscale, -d4[r]);
        }
      }
      // the dS tile of this wave, [32 queries][16 keys] bf16 row-major (32 B rows)
      char* Si = Sall + w * 1024;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) *(bf16*)(Si + (16 * mt + 4 * g + r) * 32 + j16 * 2) = (bf16)ds[mt][r];
      const bf16x8 pB = {(bf16)pd[0][0], (bf16)pd[0][1], (bf16)pd[0][2], (bf16)pd[0][3],
                         (bf16)pd[1][0], (bf16)pd[1][1], (bf16)pd[1][2], (bf16)pd[1][3]};
      const bf16x8 sB = {(bf16)ds[0][0], (bf16)ds[0][1], (bf16)ds[0][2], (bf16)ds[0][3],
                         (bf16)ds[1][0], (bf16)ds[1][1], (bf16)ds[1][2], (bf16)ds[1][3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 aO = cat8(tr4(Oi, qb * 32 + 4 * g, 16 * dt, lane), tr4(Oi, qb * 32 + 16 + 4 * g, 16 * dt, lane));
        const bf16x8 aQ = cat8(tr4(Qi, qb * 32 + 4 * g, 16 * dt, lane), tr4(Qi, qb * 32 + 16 + 4 * g, 16 * dt, lane));
        dv[dt] = mfma16(aO, pB, dv[dt]);
        dk[dt] = mfma16(aQ, sB, dk[dt]);
      }
    }
    __syncthreads();
    {  // phase B: dQ[query block jq][d half] += dS[jq][keys of pair s] K[keys of pair s][d half]
      int s = jq - i;
      if (s < 0) s += NB;
      const char* Sa = Sall + (2 * s + (lane >> 5)) * 1024;
      bf16x8 aS[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) aS[mt] = *(const bf16x8*)(Sa + (16 * mt + j16) * 32 + ((lane >> 4) & 1) * 16);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int c16 = 32 * dhalf + 16 * nt;
        const bf16x8 bK = cat8(tr4(Ki, 32 * s + 8 * g, c16, lane), tr4(Ki, 32 * s + 8 * g + 4, c16, lane));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) dq[mt][nt] = mfma16(aS[mt], bK, dq[mt][nt]);
      }
    }
    __syncthreads();
  }
  // outputs: dK, dV rows of this wave's keys (4 consecutive d per lane), dQ (scattered)
  bf16* out = dqkv;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    if (key < N) {
      const long row = (long)b * N + key;
      *(bf16x4*)(out + row * ldq + D + h * dh + 16 * dt + 4 * g) =
          bf16x4{(bf16)(dk[dt][0] * scale), (bf16)(dk[dt][1] * scale), (bf16)(dk[dt][2] * scale), (bf16)(dk[dt][3] * scale)};
      *(bf16x4*)(out + row * ldq + 2 * D + h * dh + 16 * dt + 4 * g) =
          bf16x4{(bf16)(dv[dt][0] * dscale), (bf16)(dv[dt][1] * dscale), (bf16)(dv[dt][2] * dscale), (bf16)(dv[dt][3] * dscale)};
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = jq * 32 + 16 * mt + 4 * g + r;
        if (q < N) out[((long)b * N + q) * ldq + h * dh + 32 * dhalf + 16 * nt + j16] = (bf16)(dq[mt][nt][r] * scale);
      }
}

int main() {
  const int B = 256, N = 197, H = 12, dh = 64, D = H * dh, BH = B * H;
  const long M = (long)B * N;
  bf16 *qkv, *dout, *dqkv;
  float *lse, *dqv;
  uint32_t* mask;
  hipMalloc(&qkv, M * 3 * D * 2);
  hipMalloc(&dout, M * D * 2);
  hipMalloc(&dqkv, M * 3 * D * 2);
  hipMalloc(&lse, (long)BH * N * 4);
  hipMalloc(&dqv, (long)BH * N * 4);
  hipMalloc(&mask, (long)BH * NW * NB * 64 * 4);
  hipMemset(qkv, 0, M * 3 * D * 2);
  hipMemset(dout, 0, M * D * 2);
  hipMemset(lse, 0, (long)BH * N * 4);
  hipMemset(dqv, 0, (long)BH * N * 4);
  hipMemset(mask, 0xFF, (long)BH * NW * NB * 64 * 4);
  const float scale = 0.125f, sl2 = scale * 1.4426950408889634f, dscale = 1.f / 0.9f;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int p = 0; p < 2; ++p) {
    const uint32_t* mk = p ? mask : nullptr;
    for (int it = 0; it < 3; ++it)
      hipLaunchKernelGGL(attn_bwd14, dim3(BH), dim3(64 * NW), 0, 0, qkv, (long)3 * D, dout, (long)D, lse, dqv, mk, dqkv,
                         N, H, scale, sl2, dscale);
    hipEventRecord(e0);
    const int R = 20;
    for (int it = 0; it < R; ++it)
      hipLaunchKernelGGL(attn_bwd14, dim3(BH), dim3(64 * NW), 0, 0, qkv, (long)3 * D, dout, (long)D, lse, dqv, mk, dqkv,
                         N, H, scale, sl2, dscale);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("attn_bwd14 prototype (%s mask): %.1f us per launch (B %d N %d H %d dh %d)\n", p ? "with" : "no",
           ms * 1000.f / R, B, N, H, dh);
  }
  const hipError_t err = hipDeviceSynchronize();
  printf("status: %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
