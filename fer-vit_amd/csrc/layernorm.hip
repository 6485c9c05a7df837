// LayerNorm forward / backward (HBM-bound, one wave per row, vectorised 4-wide).
//
// Post-norm nn.TransformerEncoderLayer (norm1/norm2, eps 1e-5) and timm pre-norm
// Block (eps 1e-6). Forward saves (mean, rstd) per row. Backward fuses: the
// residual-gradient add, the dropout-mask application for the branch that fed
// the norm (post-norm `LN(x + Drop(h))` -> d h = Drop'(d(x+Drop h))), and the
// per-column partial sums for dgamma, dbeta and the branch bias gradient, reduced
// afterwards in fixed block order (deterministic).
#include <stdlib.h>

#include "common.h"
#include "fervit_internal.h"

namespace fer {

constexpr int LN_VPL = 4;  // vectors (of 4) per lane: D <= 1024

template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, long ldx, const float* __restrict__ g,
                                                     const float* __restrict__ b, int grows, int rdiv,
                                                     T* __restrict__ y, long ldy, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = D >> 2;
  f32x4 v[LN_VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_VPL; ++i) {
    const int c = (lane + i * 64);
    v[i] = c < nv ? load4<T>(x + row * ldx + c * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_VPL; ++i) {
    const int c = (lane + i * 64);
    if (c < nv) {
      f32x4 d = v[i] - mu;
      q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
  }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
  const long gr = grows > 1 ? ((row / rdiv) % grows) * D : 0;
#pragma unroll
  for (int i = 0; i < LN_VPL; ++i) {
    const int c = (lane + i * 64);
    if (c < nv) {
      f32x4 gg = *(const f32x4*)(g + gr + c * 4), bb = *(const f32x4*)(b + gr + c * 4);
      store4<T>(y + row * ldy + c * 4, (v[i] - mu) * rs * gg + bb);
    }
  }
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = rs;
  }
}

// partial layout: ws[blk][3][D]
// VPL = vectors of 4 per lane = ceil(D / 256): sized per D so that D = 768 keeps the register
// sets (two rows in flight + the column partials) at 3 waves per SIMD instead of 2.
template <typename T, int VPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, long lddy, const T* __restrict__ x,
                                                     long ldx, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ g,
                                                     int grows, int rdiv, const T* __restrict__ res, long ldr,
                                                     T* __restrict__ dx, long lddx, T* __restrict__ dxd,
                                                     uint32_t thr, float dscale, uint64_t seed,
                                                     float* __restrict__ part, int want_part, int M, int D) {
  seed = step_seed(seed);
  __shared__ float red[4][VPL * 256];  // one partial at a time
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv = D >> 2;
  f32x4 pg[VPL], pb[VPL], pd[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) pg[i] = pb[i] = pd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Rows are processed in pairs with two register sets: the loads of the next row are issued
  // before the stores of the current one. (vmcnt retires loads and stores in issue order: a
  // load issued after a store would make every use wait for that store to drain.)
  typedef typename Raw4<T>::type R4;
  R4 dyA[VPL], xA[VPL], rA[VPL], dyB[VPL], xB[VPL], rB[VPL];
  auto load_row = [&](long row, R4(&dyr)[VPL], R4(&xr)[VPL], R4(&rr)[VPL]) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        dyr[i] = *(const R4*)(dy + row * lddy + c * 4);
        xr[i] = *(const R4*)(x + row * ldx + c * 4);
        if (res) rr[i] = *(const R4*)(res + row * ldr + c * 4);
      }
    }
  };
  auto proc_row = [&](long row, const R4(&dyr)[VPL], const R4(&xr)[VPL], const R4(&rr)[VPL]) {
    const float mu = mean[row], rs = rstd[row];
    const long gr = grows > 1 ? ((row / rdiv) % grows) * D : 0;
    f32x4 xh[VPL], gy[VPL], dyv[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        dyv[i] = raw4_to_f(dyr[i]);
        xh[i] = (raw4_to_f(xr[i]) - mu) * rs;
        gy[i] = dyv[i] * *(const f32x4*)(g + gr + c * 4);
        s1 += gy[i][0] + gy[i][1] + gy[i][2] + gy[i][3];
        f32x4 t = gy[i] * xh[i];
        s2 += t[0] + t[1] + t[2] + t[3];
      } else {
        dyv[i] = xh[i] = gy[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        f32x4 d = (gy[i] - s1 - xh[i] * s2) * rs;
        if (res) d += raw4_to_f(rr[i]);
        store4<T>(dx + row * lddx + c * 4, d);
        if (dxd) {
          drop4(seed, (uint32_t)row * (uint32_t)D + (uint32_t)(c * 4), thr, dscale, d);
          store4<T>(dxd + row * lddx + c * 4, d);
        }
        pg[i] += dyv[i] * xh[i];
        pb[i] += dyv[i];
        pd[i] += d;
      }
    }
  };
  const long stride = (long)gridDim.x * 4;
  long row = (long)blockIdx.x * 4 + w;
  if (row < M) load_row(row, dyA, xA, rA);
  for (; row < M; row += 2 * stride) {
    const long r2 = row + stride;
    if (r2 < M) load_row(r2, dyB, xB, rB);
    proc_row(row, dyA, xA, rA);
    if (r2 >= M) break;
    if (r2 + stride < M) load_row(r2 + stride, dyA, xA, rA);
    proc_row(r2, dyB, xB, rB);
  }
  if (!want_part) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k) __syncthreads();
#pragma unroll
    for (int i = 0; i < VPL; ++i) *(f32x4*)&red[w][(lane + i * 64) * 4] = k == 0 ? pg[i] : (k == 1 ? pb[i] : pd[i]);
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256)
      part[((long)blockIdx.x * 3 + k) * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// ---------------------------------------------------------------- bf16, 16-byte rows
// Half-wave (32 lanes) per row, 8 consecutive columns (one 16-byte piece) per lane and chunk,
// CPL = ceil(D / 256) chunks: half the memory instructions of the 4-wide kernels above; the forward
// keeps two rows in flight per half-wave (the next row's loads issued before the current row's
// stores).
FER_DEV f32x4 lo4b(bf16x8 x) { return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]}; }
FER_DEV f32x4 hi4b(bf16x8 x) { return f32x4{(float)x[4], (float)x[5], (float)x[6], (float)x[7]}; }
FER_DEV bf16x8 pk8(f32x4 a, f32x4 b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}
FER_DEV float half_sum(float v) {  // sum over the 32 lanes of this half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int CPL>
__global__ __launch_bounds__(256) void ln_fwd8_kernel(const bf16* __restrict__ x, long ldx, const float* __restrict__ g,
                                                      const float* __restrict__ b, int grows, int rdiv,
                                                      bf16* __restrict__ y, long ldy, float* __restrict__ mean,
                                                      float* __restrict__ rstd, int M, int D, float eps) {
  const int l32 = threadIdx.x & 31;
  const long hw = (long)blockIdx.x * 8 + (threadIdx.x >> 5);  // this half-wave's first row
  const long stride = (long)gridDim.x * 8;
  const int nc = D >> 3;
  bf16x8 va[CPL], vb[CPL];
  auto load = [&](long row, bf16x8(&v)[CPL]) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      v[i] = (row < M && c < nc) ? *(const bf16x8*)(x + row * ldx + c * 8) : bf16x8{};
    }
  };
  auto proc = [&](long row, const bf16x8(&v)[CPL]) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const f32x4 a = lo4b(v[i]), c = hi4b(v[i]);
      s += (a[0] + a[1]) + (a[2] + a[3]) + (c[0] + c[1]) + (c[2] + c[3]);
    }
    const float mu = half_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      if (l32 + 32 * i < nc) {
        const f32x4 a = lo4b(v[i]) - mu, c = hi4b(v[i]) - mu;
        q += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3] + c[0] * c[0] + c[1] * c[1] + c[2] * c[2] +
             c[3] * c[3];
      }
    }
    const float rs = rsqrtf(half_sum(q) / D + eps);
    const long gr = grows > 1 ? ((row / rdiv) % grows) * D : 0;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      if (c < nc) {
        const float* gp = g + gr + c * 8;
        const float* bp = b + gr + c * 8;
        const f32x4 o0 = (lo4b(v[i]) - mu) * rs * *(const f32x4*)gp + *(const f32x4*)bp;
        const f32x4 o1 = (hi4b(v[i]) - mu) * rs * *(const f32x4*)(gp + 4) + *(const f32x4*)(bp + 4);
        *(bf16x8*)(y + row * ldy + c * 8) = pk8(o0, o1);
      }
    }
    if (l32 == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
  };
  long row = hw;
  load(row, va);
  for (; row < M; row += 2 * stride) {
    const long r2 = row + stride;
    load(r2, vb);
    proc(row, va);
    if (r2 >= M) break;
    load(r2 + stride, va);
    proc(r2, vb);
  }
}

// partial layout as ln_bwd_kernel: ws[blk][3][D]
// G1: one gamma row (no LayerWiseNorm row groups): gamma is loaded into registers once per thread
// instead of twice per row (12 of the 18 16-byte loads a row cost): 91 -> 72 us at ViT-B. (Loading
// the next row's dy / x ahead of this row's math on top of that measured 82 us: not kept.)
template <int CPL, bool G1 = false>
__global__ __launch_bounds__(256) void ln_bwd8_kernel(const bf16* __restrict__ dy, long lddy, const bf16* __restrict__ x,
                                                      long ldx, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, const float* __restrict__ g,
                                                      int grows, int rdiv, const bf16* __restrict__ res, long ldr,
                                                      bf16* __restrict__ dx, long lddx, bf16* __restrict__ dxd,
                                                      uint32_t thr, float dscale, uint64_t seed,
                                                      float* __restrict__ part, int want_part, int M, int D) {
  seed = step_seed(seed);
  const int l32 = threadIdx.x & 31, hwi = threadIdx.x >> 5;
  const long stride = (long)gridDim.x * 8;
  const int nc = D >> 3;
  f32x4 pg[CPL][2], pb[CPL][2], pd[CPL][2];
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) pg[i][h] = pb[i][h] = pd[i][h] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 dyA[CPL], xA[CPL], rA[CPL];
  auto load = [&](long row, bf16x8(&dyr)[CPL], bf16x8(&xr)[CPL], bf16x8(&rr)[CPL]) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      const bool ok = row < M && c < nc;
      dyr[i] = ok ? *(const bf16x8*)(dy + row * lddy + c * 8) : bf16x8{};
      xr[i] = ok ? *(const bf16x8*)(x + row * ldx + c * 8) : bf16x8{};
      if (res) rr[i] = ok ? *(const bf16x8*)(res + row * ldr + c * 8) : bf16x8{};
    }
  };
  f32x4 gh[CPL][2];  // G1: this lane's gamma
  if constexpr (G1) {
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = l32 + 32 * i;
        gh[i][h] = c < nc ? *(const f32x4*)(g + c * 8 + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
  }
  auto gam = [&](long gr, int i, int h) -> f32x4 {
    if constexpr (G1) return gh[i][h];
    else return *(const f32x4*)(g + gr + (l32 + 32 * i) * 8 + 4 * h);
  };
  auto proc = [&](long row, const bf16x8(&dyr)[CPL], const bf16x8(&xr)[CPL], const bf16x8(&rr)[CPL]) {
    const float mu = mean[row], rs = rstd[row];
    const long gr = (!G1 && grows > 1) ? ((row / rdiv) % grows) * D : 0;
    // pass 1: the two row sums (xhat and dy*gamma are recomputed in pass 2: registers, not VALU,
    // bound this kernel's occupancy)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      if (c < nc) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 dv = h ? hi4b(dyr[i]) : lo4b(dyr[i]);
          const f32x4 xh = ((h ? hi4b(xr[i]) : lo4b(xr[i])) - mu) * rs;
          const f32x4 gy = dv * gam(gr, i, h);
          const f32x4 t = gy * xh;
          s1 += (gy[0] + gy[1]) + (gy[2] + gy[3]);
          s2 += (t[0] + t[1]) + (t[2] + t[3]);
          pg[i][h] += dv * xh;
          pb[i][h] += dv;
        }
      }
    }
    s1 = half_sum(s1) / D;
    s2 = half_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      if (c < nc) {
        f32x4 d[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 xh = ((h ? hi4b(xr[i]) : lo4b(xr[i])) - mu) * rs;
          const f32x4 gy = (h ? hi4b(dyr[i]) : lo4b(dyr[i])) * gam(gr, i, h);
          d[h] = (gy - s1 - xh * s2) * rs;
          if (res) d[h] += h ? hi4b(rr[i]) : lo4b(rr[i]);
        }
        *(bf16x8*)(dx + row * lddx + c * 8) = pk8(d[0], d[1]);
        if (dxd) {
          const uint32_t idx = (uint32_t)row * (uint32_t)D + (uint32_t)(c * 8);
          const uint32_t k = thr ? (keep4(seed, idx, thr) | (keep4(seed, idx + 4, thr) << 4)) : 0xFFu;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            d[0][r] = (k >> r) & 1 ? d[0][r] * dscale : 0.f;
            d[1][r] = (k >> (4 + r)) & 1 ? d[1][r] * dscale : 0.f;
          }
          *(bf16x8*)(dxd + row * lddx + c * 8) = pk8(d[0], d[1]);
        }
        pd[i][0] += d[0];
        pd[i][1] += d[1];
      }
    }
  };
  // one row at a time per half-wave (the column partials take the registers a second row set would
  // need; occupancy hides the load latency)
  for (long row = (long)blockIdx.x * 8 + hwi; row < M; row += stride) {
    load(row, dyA, xA, rA);
    proc(row, dyA, xA, rA);
  }
  if (!want_part) return;
  // column partials: 8 half-waves of the block (same columns), fixed order through LDS
  __shared__ float red[8][CPL * 256];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k) __syncthreads();
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        *(f32x4*)&red[hwi][(l32 + 32 * i) * 8 + 4 * h] = k == 0 ? pg[i][h] : (k == 1 ? pb[i][h] : pd[i][h]);
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) t += red[j][c];
      part[((long)blockIdx.x * 3 + k) * D + c] = t;
    }
  }
}

// out_k[col] (+)= sum_blk part[blk][k][col] for k in {0,1,2}
__global__ __launch_bounds__(256) void ln_part_reduce_kernel(const float* __restrict__ part, int nblk, int D,
                                                             float* o0, float* o1, float* o2, int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= 3 * D) return;
  const int k = c / D, col = c - k * D;
  float* o = k == 0 ? o0 : (k == 1 ? o1 : o2);
  if (!o) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(long)b * 3 * D + c];
  o[col] = accumulate ? o[col] + s : s;
}

// One round of workgroups: two per CU (the kernel runs two waves per SIMD), each walking its rows
// with the grid stride. 1024 blocks (two rounds) measured 71.5 us at ViT-B vs 63.5 us: the second
// round's tail and twice the column partials for part_reduce.
static int ln_bwd_blocks(int M) {
  static const int cap = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return 2 * n;
  }();
  return std::max(1, std::min(ceil_div(M, 16), cap));
}

}  // namespace fer

using namespace fer;

int fer::set_step_ptr_layernorm(const uint64_t* p) { return set_step_ptr_here(p) == hipSuccess ? 0 : -1; }

extern "C" int fer_layernorm_fwd(int dtype, const void* x, int64_t ldx, const float* gamma, const float* beta,
                                 int gamma_rows, int row_div, void* y, int64_t ldy, float* mean, float* rstd, int M,
                                 int D, float eps, fer_stream_t stream) {
  if (M <= 0) return 0;
  if (D % 4 || D > 1024 || ldx % 4 || ldy % 4) return set_error("layernorm_fwd: D must be a multiple of 4 and <= 1024");
  if (gamma_rows < 1) gamma_rows = 1;
  if (row_div < 1) row_div = 1;
  dim3 grid(ceil_div(M, 4));
  if (dtype == FER_BF16 && D % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0) {
    // one round of workgroups (four per CU at this kernel's 4 waves per SIMD): 25.8 us at ViT-B vs
    // 27.7 us with 2048 (two rounds)
    static const int fcap = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return 4 * n;
    }();
    const dim3 g8(std::max(1, std::min(ceil_div(M, 16), fcap)));  // two rows per half-wave in flight
#define FER_LN_FWD8(C)                                                                                          \
  hipLaunchKernelGGL(ln_fwd8_kernel<C>, g8, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (long)ldx, gamma, \
                     beta, gamma_rows, row_div, (bf16*)y, (long)ldy, mean, rstd, M, D, eps);
    switch ((D + 255) / 256) {
      case 1: FER_LN_FWD8(1) break;
      case 2: FER_LN_FWD8(2) break;
      case 3: FER_LN_FWD8(3) break;
      default: FER_LN_FWD8(4) break;
    }
#undef FER_LN_FWD8
  } else if (dtype == FER_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (long)ldx, gamma,
                       beta, gamma_rows, row_div, (bf16*)y, (long)ldy, mean, rstd, M, D, eps);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (const float*)x, (long)ldx,
                       gamma, beta, gamma_rows, row_div, (float*)y, (long)ldy, mean, rstd, M, D, eps);
  return hip_check("layernorm_fwd");
}

extern "C" int64_t fer_layernorm_bwd_ws(int M, int D) { return (int64_t)ln_bwd_blocks(M) * 3 * D * 4; }

extern "C" int fer_layernorm_bwd(int dtype, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                                 const float* mean, const float* rstd, const float* gamma, int gamma_rows,
                                 int row_div, const void* res, int64_t ldr, void* dx, int64_t lddx, void* dx_drop,
                                 uint32_t drop_thresh, float drop_scale, uint64_t seed, float* dgamma, float* dbeta,
                                 float* dbias, int accumulate, float* ws, int64_t ws_bytes, int M, int D,
                                 fer_stream_t stream) {
  if (M <= 0) return 0;
  if (D % 4 || D > 1024) return set_error("layernorm_bwd: D must be a multiple of 4 and <= 1024");
  if (dx_drop && check_drop_range(drop_thresh, (long)M * D, "layernorm_bwd: dropout over >= 2^32 elements"))
    return -1;
  if (gamma_rows < 1) gamma_rows = 1;
  if (row_div < 1) row_div = 1;
  const bool want = dgamma || dbeta || dbias;
  if (want && gamma_rows != 1) return set_error("layernorm_bwd: parameter grads need shared gamma");
  const int nblk = ln_bwd_blocks(M);
  if (want && (!ws || ws_bytes < fer_layernorm_bwd_ws(M, D))) return set_error("layernorm_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (want) ws = reduction_ws(ws, (size_t)fer_layernorm_bwd_ws(M, D), 3 * D, st);
  if (dtype == FER_BF16 && D % 8 == 0 && lddy % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 && (!res || ldr % 8 == 0)) {
    const bool g1 = gamma_rows <= 1;  // gamma held in registers for the whole row loop
#define FER_LN_BWD8(C)                                                                                          \
  if (g1) FER_LN_BWD8K((ln_bwd8_kernel<C, true>))                                                               \
  else FER_LN_BWD8K((ln_bwd8_kernel<C, false>))
#define FER_LN_BWD8K(K)                                                                                         \
  hipLaunchKernelGGL(K, dim3(nblk), dim3(256), 0, st, (const bf16*)dy, (long)lddy, (const bf16*)x, \
                     (long)ldx, mean, rstd, gamma, gamma_rows, row_div, (const bf16*)res, (long)ldr, (bf16*)dx,   \
                     (long)lddx, (bf16*)dx_drop, drop_thresh, drop_scale, seed, ws, (int)want, M, D);
    switch ((D + 255) / 256) {
      case 1: FER_LN_BWD8(1) break;
      case 2: FER_LN_BWD8(2) break;
      case 3: FER_LN_BWD8(3) break;
      default: FER_LN_BWD8(4) break;
    }
#undef FER_LN_BWD8
#undef FER_LN_BWD8K
    int rc = hip_check("layernorm_bwd8");
    if (rc || !want) return rc;
    part_reduce(ws, nblk, 3L * D, 3 * D, D, dgamma, dbeta, dbias, accumulate, nullptr, st);
    return hip_check("layernorm_bwd_reduce");
  }
#define FER_LN_BWD(VP)                                                                                       \
  if (dtype == FER_BF16)                                                                                     \
    hipLaunchKernelGGL((ln_bwd_kernel<bf16, VP>), dim3(nblk), dim3(256), 0, st, (const bf16*)dy, (long)lddy,  \
                       (const bf16*)x, (long)ldx, mean, rstd, gamma, gamma_rows, row_div, (const bf16*)res,   \
                       (long)ldr, (bf16*)dx, (long)lddx, (bf16*)dx_drop, drop_thresh, drop_scale, seed, ws,   \
                       (int)want, M, D);                                                                     \
  else                                                                                                       \
    hipLaunchKernelGGL((ln_bwd_kernel<float, VP>), dim3(nblk), dim3(256), 0, st, (const float*)dy,           \
                       (long)lddy, (const float*)x, (long)ldx, mean, rstd, gamma, gamma_rows, row_div,       \
                       (const float*)res, (long)ldr, (float*)dx, (long)lddx, (float*)dx_drop, drop_thresh,   \
                       drop_scale, seed, ws, (int)want, M, D);
  switch ((D + 255) / 256) {
    case 1: FER_LN_BWD(1) break;
    case 2: FER_LN_BWD(2) break;
    case 3: FER_LN_BWD(3) break;
    default: FER_LN_BWD(4) break;
  }
#undef FER_LN_BWD
  int rc = hip_check("layernorm_bwd");
  if (rc || !want) return rc;
  part_reduce(ws, nblk, 3L * D, 3 * D, D, dgamma, dbeta, dbias, accumulate, nullptr, st);
  return hip_check("layernorm_bwd_reduce");
}
