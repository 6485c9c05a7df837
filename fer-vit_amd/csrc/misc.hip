// HBM-bound kernels around the transformer trunk: bias-gradient column sums, patch
// im2col, token assembly (CLS + pos), classification head (LN + Linear on CLS rows),
// softmax cross-entropy, the w+ prologue (SemanticPE / LayerWiseNorm / LEAM), the
// LatentDecomposer projection, casts, dropout and the fused AdamW optimizer.
// All cross-row reductions are two-pass (per-block partials, then a fixed-order sum),
// so every result is bitwise reproducible run to run.
#include <mutex>

#include "common.h"
#include "fervit_internal.h"

namespace fer {

// ------------------------------------------------------------------ reductions
// Deterministic second pass: out_k[c % seg] (+)= scale * sum_{b<nb} part[b*ld + c],
// k = c / seg selects one of three outputs.
// CB columns per block x (256 / CB) row phases, 8 independent accumulators per thread (8 loads in
// flight; the partial slabs are read once and the sum is latency-bound otherwise). CB is picked so
// that the grid covers the CUs (ViT-B: 2304 columns -> 288 blocks of 8 columns instead of 72 of
// 32). Fixed association order for a given shape -> deterministic.
template <int CB>
__device__ __forceinline__ void part_reduce_body(const float* __restrict__ part, int nb, long ld, int ncols, int seg,
                                                 float* o0, float* o1, float* o2, int accumulate,
                                                 const float* __restrict__ scale, int bx) {
  constexpr int RP = 256 / CB;
  __shared__ float red[RP][CB + 1];
  const int cx = threadIdx.x % CB, j = threadIdx.x / CB;
  const int c = bx * CB + cx;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < ncols) {
    int b = j;
    for (; b + 7 * RP < nb; b += 8 * RP) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += part[(long)(b + RP * u) * ld + c];
    }
    for (int u = 0; b < nb; b += RP, ++u) s[u] += part[(long)b * ld + c];
  }
  red[j][cx] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (j == 0 && c < ncols) {
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < RP; ++i) t += red[i][cx];
    if (scale) t *= *scale;
    const int k = c / seg, col = c - k * seg;
    float* o = k == 0 ? o0 : (k == 1 ? o1 : o2);
    if (o) o[col] = accumulate ? o[col] + t : t;
  }
}
template <int CB>
__global__ __launch_bounds__(256) void part_reduce_kernel(const float* __restrict__ part, int nb, long ld, int ncols,
                                                          int seg, float* o0, float* o1, float* o2, int accumulate,
                                                          const float* __restrict__ scale) {
  part_reduce_body<CB>(part, nb, ld, ncols, seg, o0, o1, o2, accumulate, scale, blockIdx.x);
}

// Deferred reductions (fer_reduce_defer): inside a backward pass the column partials of the bias /
// LayerNorm / attention-bias gradients are written into an arena instead of the shared scratch and
// their part_reduce launches are queued; fer_reduce_flush (the end of the backward, or before a
// gradient-ready hook such as the DDP bucket all-reduce reads them) runs them all as ONE launch.
// Same per-column arithmetic as part_reduce_kernel<8> (the batch only takes shapes that would use
// the 8-column kernel), so bit-identical results; only their time on the compute stream moves.
struct RedDesc {
  const float* part;
  long ld;
  float* o[3];
  int nb, ncols, seg, accumulate, blk0;
};
constexpr int kRedMax = 56;  // kernel-argument budget (64 bytes each)
struct RedBatch {
  RedDesc d[kRedMax];
  int n;
};
// The batch kernel: 64 columns per block (a wave reads 256 contiguous bytes of a partial row,
// where part_reduce_kernel<8>'s 8-column blocks read 32-byte pieces -- it needs narrow blocks to
// spread one small reduction over the CUs; a batch has blocks enough). Lane = column, wave w owns
// the row phases j = 8w .. 8w+7 of part_reduce_kernel<8> (RP = 32) and runs each with the same
// eight accumulators in the same order, then the phases are summed in order j = 0..31: the same
// float operations per column as the immediate kernel, so bit-identical.
__global__ __launch_bounds__(256) void part_reduce_multi_kernel(const RedBatch b) {
  constexpr int RP = 32;
  __shared__ float red[RP][65];
  int i = 0;
  while (i + 1 < b.n && (int)blockIdx.x >= b.d[i + 1].blk0) ++i;
  const RedDesc& d = b.d[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x - d.blk0) * 64 + lane;
  const float* __restrict__ part = d.part;
  const int nb = d.nb;
  const long ld = d.ld;
  for (int jj = 0; jj < 8; ++jj) {
    const int j = w * 8 + jj;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c < d.ncols) {
      int bb = j;
      for (; bb + 7 * RP < nb; bb += 8 * RP) {
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += part[(long)(bb + RP * u) * ld + c];
      }
      for (int u = 0; bb < nb; bb += RP, ++u) s[u] += part[(long)bb * ld + c];
    }
    red[j][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  }
  __syncthreads();
  if (w == 0 && c < d.ncols) {
    float t = 0.f;
#pragma unroll 8
    for (int k = 0; k < RP; ++k) t += red[k][lane];
    const int k = c / d.seg, col = c - k * d.seg;
    float* o = k == 0 ? d.o[0] : (k == 1 ? d.o[1] : d.o[2]);
    if (o) o[col] = d.accumulate ? o[col] + t : t;
  }
}
// One window per process, on one device (fer_reduce_defer rejects a second device while open); the
// state is guarded by g_red_mu (part_reduce / reduction_ws are reached from every host entry point).
static std::mutex g_red_mu;
static struct {
  bool on = false, take = false;  // window open (queue valid) / taking new reductions
  int dev = -1;
  char* arena = nullptr;
  size_t cap = 0, used = 0;
  hipStream_t st = nullptr;
  RedBatch b;
  int blocks = 0;
} g_red;
static bool red_batchable(int ncols) { return ceil_div(ncols, 16) < 256; }
static int red_flush() {
  if (g_red.b.n) {
    hipLaunchKernelGGL(part_reduce_multi_kernel, dim3(g_red.blocks), dim3(256), 0, g_red.st, g_red.b);
    g_red.b.n = 0;
    g_red.blocks = 0;
  }
  g_red.used = 0;
  return hip_check("reduce_flush");
}
// Only partial sets up to 2 MB are deferred: the small-token
// configurations' (latent w+ 1.5-1.9 MB per LayerNorm / attention bias) gain one launch each
// (latent ViT 2.22 -> 2.16 ms), while ViT-B's (4.7-16.5 MB, 52 per step) measured 35.62 -> 35.75
// ms deferred (their sums then re-read from HBM at the end of the backward instead of from the
// last-level cache right after the producer; profiles/r03am_reduce_defer_ab.txt).
float* reduction_ws(float* ws, size_t bytes, int ncols, hipStream_t st) {
  constexpr size_t max_b = 2048 * 1024L;
  std::lock_guard<std::mutex> lk(g_red_mu);
  if (!g_red.take || st != g_red.st || !red_batchable(ncols) || bytes > g_red.cap || bytes > max_b) return ws;
  bytes = (bytes + 255) & ~(size_t)255;
  if (g_red.used + bytes > g_red.cap || g_red.b.n == kRedMax) red_flush();
  float* p = (float*)(g_red.arena + g_red.used);
  g_red.used += bytes;
  return p;
}

void part_reduce(const float* part, int nb, long ld, int ncols, int seg, float* o0, float* o1, float* o2,
                 int accumulate, const float* scale, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_red_mu);
  const bool in_arena = g_red.take && st == g_red.st && (const char*)part >= g_red.arena &&
                        (const char*)part < g_red.arena + g_red.cap;
  // an output range overlapping a queued one (any base pointer: segmented o0/o1/o2 outputs vs a
  // whole-buffer output): run the queue first, keeping the two updates in stream order
  auto span = [](float* const (&o)[3], int k, int ncols, int seg) -> std::pair<const float*, const float*> {
    const int n = std::min(seg, ncols - k * seg);
    return o[k] && n > 0 ? std::make_pair((const float*)o[k], (const float*)o[k] + n)
                         : std::make_pair((const float*)nullptr, (const float*)nullptr);
  };
  float* const mine[3] = {o0, o1, o2};
  bool dup = false;
  for (int i = 0; i < g_red.b.n && !dup; ++i)
    for (int k = 0; k < 3 && !dup; ++k) {
      const auto q = span(g_red.b.d[i].o, k, g_red.b.d[i].ncols, g_red.b.d[i].seg);
      if (!q.first) continue;
      for (int j = 0; j < 3 && !dup; ++j) {
        const auto m = span(mine, j, ncols, seg);
        dup = m.first && m.first < q.second && q.first < m.second;
      }
    }
  if (in_arena && !scale && red_batchable(ncols) && g_red.b.n < kRedMax && !dup) {
    g_red.b.d[g_red.b.n++] = RedDesc{part, ld, {o0, o1, o2}, nb, ncols, seg, accumulate, g_red.blocks};
    g_red.blocks += ceil_div(ncols, 64);
    return;
  }
  if (g_red.b.n && (in_arena || dup)) {  // run the queue first; this call's partials stay valid
    const size_t keep = g_red.used;
    red_flush();
    g_red.used = keep;
  }
  if (ceil_div(ncols, 16) >= 256)
    hipLaunchKernelGGL(part_reduce_kernel<16>, dim3(ceil_div(ncols, 16)), dim3(256), 0, st, part, nb, ld, ncols, seg,
                       o0, o1, o2, accumulate, scale);
  else
    hipLaunchKernelGGL(part_reduce_kernel<8>, dim3(ceil_div(ncols, 8)), dim3(256), 0, st, part, nb, ld, ncols, seg,
                       o0, o1, o2, accumulate, scale);
  if (in_arena && !g_red.b.n) g_red.used = 0;
}

// ------------------------------------------------------------------ colsum
// part[rb][n] = sum over row chunk rb of x[m][n]; block = 64 vec4 columns x 4 row phases.
constexpr int CS_ROWBLK = 256;
template <typename T>
__global__ __launch_bounds__(256) void colsum_part_kernel(const T* __restrict__ x, long ldx, int M, int N,
                                                          float* __restrict__ part, int rows_per_blk) {
  __shared__ f32x4 red[4][64];
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(M, r0 + rows_per_blk);
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (c4 * 4 < N) {
    int r = r0 + j;
    for (; r + 4 < r1; r += 8) {
      s0 += load4<T>(x + (long)r * ldx + c4 * 4);
      s1 += load4<T>(x + (long)(r + 4) * ldx + c4 * 4);
    }
    if (r < r1) s0 += load4<T>(x + (long)r * ldx + c4 * 4);
  }
  red[j][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (j == 0 && c4 * 4 < N) {
    const int t = threadIdx.x & 63;
    *(f32x4*)(part + (long)blockIdx.y * N + c4 * 4) = red[0][t] + red[1][t] + red[2][t] + red[3][t];
  }
}
// row blocks of 32 rows (up to 256): a 4,864-row colsum (hybrid adapters' bias gradients) was
// 38 x 3 = 114 workgroups of 128 rows, 7.6 us for 7.5 MB
static int colsum_nblk(int M) { return std::max(1, std::min(ceil_div(M, 32), CS_ROWBLK)); }

// ------------------------------------------------------------------ im2col
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int B, int C, int Hh, int Ww, int P,
                                                     T* __restrict__ cols, long ldc) {
  const int gh = Hh / P, gw = Ww / P, K = C * P * P;
  const long total = (long)B * gh * gw * K;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const int k = i % K;
    const long tok = i / K;
    const int gx = tok % gw, gy = (tok / gw) % gh, b = tok / ((long)gw * gh);
    const int c = k / (P * P), kh = (k / P) % P, kw = k % P;
    cols[tok * ldc + k] = from_f<T>(x[(((long)b * C + c) * Hh + gy * P + kh) * Ww + gx * P + kw]);
  }
}

// 4 consecutive kw per thread (P % 4 == 0, Ww % 4 == 0, ldc % 4 == 0): one 16-byte input load
// and one 4-element store, 32-bit index arithmetic (total / 4 < 2^31, checked by the host).
template <typename T>
__global__ __launch_bounds__(256) void im2col4_kernel(const float* __restrict__ x, int B, int C, int Hh, int Ww,
                                                      int P, T* __restrict__ cols, long ldc) {
  const int gh = Hh / P, gw = Ww / P, K = C * P * P, K4 = K >> 2, PP = P * P;
  const int total = B * gh * gw * K4;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int k = (i % K4) * 4;
    const int tok = i / K4;
    const int gx = tok % gw, gy = (tok / gw) % gh, b = tok / (gw * gh);
    const int c = k / PP, kh = (k / P) % P, kw = k % P;
    const f32x4 v = *(const f32x4*)(x + (((long)b * C + c) * Hh + gy * P + kh) * Ww + gx * P + kw);
    store4<T>(cols + (long)tok * ldc + k, v);
  }
}

// ------------------------------------------------------------------ tokens
// 4 consecutive d per thread (D % 4 == 0); dropout keep bits identical to the scalar form.
template <typename T>
__global__ __launch_bounds__(256) void tokens_fwd4_kernel(const T* __restrict__ emb, const float* __restrict__ cls,
                                                          const float* __restrict__ pos, T* __restrict__ t, int B,
                                                          int n, int D, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  const int N = n + 1, D4 = D >> 2;
  const long total = (long)B * N * D4;
  for (long i4 = blockIdx.x * 256L + threadIdx.x; i4 < total; i4 += (long)gridDim.x * 256L) {
    const int d = (int)(i4 % D4) * 4;
    const long row = i4 / D4;
    const int tk = (int)(row % N), b = (int)(row / N);
    f32x4 v = tk == 0 ? *(const f32x4*)(cls + d) : load4<T>(emb + ((long)b * n + tk - 1) * D + d);
    v += *(const f32x4*)(pos + (long)tk * D + d);
    if (thr) drop4(seed, (uint32_t)(row * D + d), thr, dscale, v);
    store4<T>(t + row * D + d, v);
  }
}

// bf16 with D % 8 == 0 (ViT-B: 256 x 197 x 768): 8 consecutive d per thread (16-byte loads and stores) and
// 32-bit index arithmetic (the 4-wide form's 64-bit divisions per element group were most of its time); the
// same per-element values and keep bits (two keep4 per 8 elements).
__global__ __launch_bounds__(256) void tokens_fwd8_kernel(const bf16* __restrict__ emb, const float* __restrict__ cls,
                                                          const float* __restrict__ pos, bf16* __restrict__ t, int B,
                                                          int n, int D, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  const uint32_t N = n + 1, D8 = D >> 3;
  const uint32_t total = (uint32_t)B * N * D8;  // (host: < 2^31)
  for (uint32_t i8 = blockIdx.x * 256u + threadIdx.x; i8 < total; i8 += gridDim.x * 256u) {
    const uint32_t row = i8 / D8, d = (i8 - row * D8) * 8;
    const uint32_t b = row / N, tk = row - b * N;
    f32x4 v0, v1;
    if (tk == 0) {
      v0 = *(const f32x4*)(cls + d);
      v1 = *(const f32x4*)(cls + d + 4);
    } else {
      const bf16x8 e = *(const bf16x8*)(emb + ((long)b * n + tk - 1) * D + d);
      v0 = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
      v1 = f32x4{(float)e[4], (float)e[5], (float)e[6], (float)e[7]};
    }
    v0 += *(const f32x4*)(pos + (long)tk * D + d);
    v1 += *(const f32x4*)(pos + (long)tk * D + d + 4);
    if (thr) {
      const uint32_t idx = row * (uint32_t)D + d;
      drop4(seed, idx, thr, dscale, v0);
      drop4(seed, idx + 4, thr, dscale, v1);
    }
    *(bf16x8*)(t + (long)row * D + d) =
        bf16x8{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3], (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
  }
}

template <typename T>
__global__ __launch_bounds__(256) void tokens_fwd_kernel(const T* __restrict__ emb, const float* __restrict__ cls,
                                                         const float* __restrict__ pos, T* __restrict__ t, int B,
                                                         int n, int D, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  const int N = n + 1;
  const long total = (long)B * N * D;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const int d = i % D;
    const long row = i / D;
    const int tk = row % N, b = row / N;
    float v = tk == 0 ? cls[d] : to_f<T>(emb[((long)b * n + tk - 1) * D + d]);
    v += pos[(long)tk * D + d];
    if (thr) v = drop_keep(seed, (uint32_t)i, thr) ? v * dscale : 0.f;
    t[i] = from_f<T>(v);
  }
}
// dpos partial per b-chunk; demb written directly
template <typename T>
__global__ __launch_bounds__(256) void tokens_bwd_kernel(const T* __restrict__ dt, T* __restrict__ demb, int B, int n,
                                                         int D, uint32_t thr, float dscale, uint64_t seed,
                                                         float* __restrict__ part, int bchunk) {
  seed = step_seed(seed);
  const int N = n + 1;
  const long cols = (long)N * D;
  const long j = blockIdx.x * 256L + threadIdx.x;  // (token, d)
  if (j >= cols) return;
  const int tk = j / D;
  const int b0 = blockIdx.y * bchunk, b1 = min(B, b0 + bchunk);
  float s = 0.f;
  for (int b = b0; b < b1; ++b) {
    const long i = (long)b * cols + j;
    float g = to_f<T>(dt[i]);
    if (thr) g = drop_keep(seed, (uint32_t)i, thr) ? g * dscale : 0.f;
    s += g;
    if (tk > 0 && demb) demb[((long)b * n + tk - 1) * D + (j % D)] = from_f<T>(g);
  }
  part[(long)blockIdx.y * cols + j] = s;
}
// 4 consecutive (token, d) columns per thread (D % 4 == 0: one token): 8/16-byte loads and
// stores and one keep4 per 4 elements instead of a hash per element; same per-element values
// and the same summation order over b as tokens_bwd_kernel (bit-identical partials).
template <typename T>
__global__ __launch_bounds__(256) void tokens_bwd4_kernel(const T* __restrict__ dt, T* __restrict__ demb, int B, int n,
                                                          int D, uint32_t thr, float dscale, uint64_t seed,
                                                          float* __restrict__ part, int bchunk) {
  seed = step_seed(seed);
  const int N = n + 1;
  const long cols = (long)N * D;
  const long j = (blockIdx.x * 256L + threadIdx.x) * 4;  // (token, d), d % 4 == 0
  if (j >= cols) return;
  const int tk = j / D, d = j - (long)tk * D;
  const int b0 = blockIdx.y * bchunk, b1 = min(B, b0 + bchunk);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (int b = b0; b < b1; ++b) {
    const long i = (long)b * cols + j;
    f32x4 g = load4<T>(dt + i);
    if (thr) {
      const uint32_t k = keep4(seed, (uint32_t)i, thr);
#pragma unroll
      for (int r = 0; r < 4; ++r) g[r] = (k >> r) & 1 ? g[r] * dscale : 0.f;
    }
    s += g;
    if (tk > 0 && demb) store4<T>(demb + ((long)b * n + tk - 1) * D + d, g);
  }
  *(f32x4*)(part + (long)blockIdx.y * cols + j) = s;
}
// bf16 with D % 8 == 0 (ViT-B's token gradient, 50,432 x 768): 8 consecutive columns per thread (16-byte
// loads and stores), four batch rows in flight per iteration, and 16 batch chunks instead of 64 (a quarter
// of the fp32 partial slabs the reduction reads: 9.7 instead of 38.7 MB at ViT-B). Per column the batch
// rows of a chunk are summed in ascending order, as in tokens_bwd4_kernel.
__global__ __launch_bounds__(256) void tokens_bwd8_kernel(const bf16* __restrict__ dt, bf16* __restrict__ demb, int B,
                                                          int n, int D, uint32_t thr, float dscale, uint64_t seed,
                                                          float* __restrict__ part, int bchunk) {
  seed = step_seed(seed);
  const int N = n + 1;
  const long cols = (long)N * D;
  const long j = (blockIdx.x * 256L + threadIdx.x) * 8;  // (token, d), d % 8 == 0
  if (j >= cols) return;
  const int tk = j / D, d = j - (long)tk * D;
  const int b0 = blockIdx.y * bchunk, b1 = min(B, b0 + bchunk);
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  auto one = [&](int b, bf16x8 v) {
    f32x4 g0 = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    f32x4 g1 = f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
    if (thr) {
      const uint32_t i = (uint32_t)((long)b * cols + j);
      const uint32_t k = keep4(seed, i, thr) | (keep4(seed, i + 4, thr) << 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        g0[r] = (k >> r) & 1 ? g0[r] * dscale : 0.f;
        g1[r] = (k >> (4 + r)) & 1 ? g1[r] * dscale : 0.f;
      }
    }
    s0 += g0;
    s1 += g1;
    if (tk > 0 && demb)
      *(bf16x8*)(demb + ((long)b * n + tk - 1) * D + d) =
          bf16x8{(bf16)g0[0], (bf16)g0[1], (bf16)g0[2], (bf16)g0[3], (bf16)g1[0], (bf16)g1[1], (bf16)g1[2], (bf16)g1[3]};
  };
  int b = b0;
  for (; b + 4 <= b1; b += 4) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(dt + (long)(b + u) * cols + j);
#pragma unroll
    for (int u = 0; u < 4; ++u) one(b + u, v[u]);
  }
  for (; b < b1; ++b) one(b, *(const bf16x8*)(dt + (long)b * cols + j));
  *(f32x4*)(part + (long)blockIdx.y * cols + j) = s0;
  *(f32x4*)(part + (long)blockIdx.y * cols + j + 4) = s1;
}
__global__ void tokens_bwd_final(const float* __restrict__ part, int nchunk, int N, int D, float* dcls, float* dpos,
                                 int accumulate) {
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= (long)N * D) return;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += part[(long)c * N * D + j];
  if (dpos) dpos[j] = accumulate ? dpos[j] + s : s;
  if (j < D && dcls) dcls[j] = accumulate ? dcls[j] + s : s;
}

// ------------------------------------------------------------------ head
// One block (256 threads) per sample. stats[b] = {mean, rstd}.
template <typename T>
__global__ __launch_bounds__(256) void head_fwd_kernel(const T* __restrict__ t, long rs, const float* __restrict__ lw,
                                                       const float* __restrict__ lb, float eps,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       float* __restrict__ logits, float* __restrict__ stats, int D,
                                                       int C, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  __shared__ float h[1024];
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* x = t + (long)b * rs;
  float s = 0.f;
  for (int d = tid; d < D; d += 256) {
    const float v = to_f<T>(x[d]);
    h[d] = v;
    s += v;
  }
  s = wave_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  const float mu = (red[0] + red[1] + red[2] + red[3]) / D;
  float q = 0.f;
  for (int d = tid; d < D; d += 256) q += (h[d] - mu) * (h[d] - mu);
  q = wave_sum(q);
  __syncthreads();
  if (lane == 0) red[4 + w] = q;
  __syncthreads();
  const float rsd = rsqrtf((red[4] + red[5] + red[6] + red[7]) / D + eps);
  for (int d = tid; d < D; d += 256) {
    float v = (h[d] - mu) * rsd * lw[d] + lb[d];
    if (thr) v = drop_keep(seed, (uint32_t)b * (uint32_t)D + (uint32_t)d, thr) ? v * dscale : 0.f;
    h[d] = v;
  }
  __syncthreads();
  for (int c = w; c < C; c += 4) {
    float a = 0.f;
    for (int d = lane; d < D; d += 64) a += h[d] * W[(long)c * D + d];
    a = wave_sum(a);
    if (lane == 0) logits[(long)b * C + c] = a + bias[c];
  }
  if (tid == 0) {
    stats[2 * b] = mu;
    stats[2 * b + 1] = rsd;
  }
}
// part[b] = [dW (C*D) | dbias (C) | dln_w (D) | dln_b (D)]
template <typename T>
__global__ __launch_bounds__(256) void head_bwd_kernel(const T* __restrict__ t, long rs, const float* __restrict__ lw,
                                                       const float* __restrict__ lb, const float* __restrict__ W,
                                                       const float* __restrict__ stats,
                                                       const float* __restrict__ dlogits, T* __restrict__ dt, int D,
                                                       int C, uint32_t thr, float dscale, uint64_t seed,
                                                       float* __restrict__ part) {
  seed = step_seed(seed);
  __shared__ float xh[1024], gh[1024];
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* x = t + (long)b * rs;
  const float mu = stats[2 * b], rsd = stats[2 * b + 1];
  const long pstride = (long)C * D + C + 2 * D;
  float* pp = part + (long)b * pstride;
  float s1 = 0.f, s2 = 0.f;
  for (int d = tid; d < D; d += 256) {
    const float xhat = (to_f<T>(x[d]) - mu) * rsd;
    float hv = xhat * lw[d] + lb[d];
    bool keep = true;
    if (thr) keep = drop_keep(seed, (uint32_t)b * (uint32_t)D + (uint32_t)d, thr);
    const float hd = thr ? (keep ? hv * dscale : 0.f) : hv;
    float g = 0.f;
    for (int c = 0; c < C; ++c) {
      const float dl = dlogits[(long)b * C + c];
      g += dl * W[(long)c * D + d];
      pp[(long)c * D + d] = dl * hd;
    }
    if (thr) g = keep ? g * dscale : 0.f;
    pp[(long)C * D + C + d] = g * xhat;  // dln_w
    pp[(long)C * D + C + D + d] = g;     // dln_b
    const float gg = g * lw[d];
    xh[d] = xhat;
    gh[d] = gg;
    s1 += gg;
    s2 += gg * xhat;
  }
  if (tid < C) pp[(long)C * D + tid] = dlogits[(long)b * C + tid];
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    red[w] = s1;
    red[4 + w] = s2;
  }
  __syncthreads();
  const float m1 = (red[0] + red[1] + red[2] + red[3]) / D, m2 = (red[4] + red[5] + red[6] + red[7]) / D;
  for (int d = tid; d < D; d += 256) dt[(long)b * rs + d] = from_f<T>((gh[d] - m1 - xh[d] * m2) * rsd);
}
__global__ void head_bwd_final(const float* __restrict__ part, int B, int C, int D, float* dW, float* dbias,
                               float* dlw, float* dlb, int accumulate) {
  const long pstride = (long)C * D + C + 2 * D;
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= pstride) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += part[(long)b * pstride + j];
  float* o;
  long k;
  if (j < (long)C * D) { o = dW; k = j; }
  else if (j < (long)C * D + C) { o = dbias; k = j - (long)C * D; }
  else if (j < (long)C * D + C + D) { o = dlw; k = j - (long)C * D - C; }
  else { o = dlb; k = j - (long)C * D - C - D; }
  if (!o) return;
  o[k] = accumulate ? o[k] + s : s;
}
template <typename T>
__global__ void zero_rows4_kernel(T* __restrict__ dt, long rows, int D_ld, int D, long stride_keep) {
  const int D4 = D >> 2;
  const long total = rows * (long)D4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const long r = i / D4;
    if (r % stride_keep) store4<T>(dt + r * D_ld + (i % D4) * 4, f32x4{0.f, 0.f, 0.f, 0.f});
  }
}
template <typename T>
__global__ void zero_rows_kernel(T* __restrict__ dt, long rows, int D_ld, int D, long stride_keep) {
  const long total = rows * (long)D;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const long r = i / D;
    if (r % stride_keep) dt[r * D_ld + (i % D)] = from_f<T>(0.f);
  }
}

// ------------------------------------------------------------------ cross entropy
__global__ __launch_bounds__(256) void ce_kernel(const float* __restrict__ logits, const int64_t* __restrict__ y,
                                                 const float* __restrict__ wt, int B, int C, float ls, float gscale,
                                                 float* loss, float* dlogits) {
  // single block; pass 1: per-sample terms; pass 2: normalise
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float num = 0.f, den = 0.f;
  for (int b = tid; b < B; b += 256) {
    const float* z = logits + (long)b * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, z[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(z[c] - m);
    const float lse = m + logf(se);
    const int yb = (int)y[b];
    const float wy = wt ? wt[yb] : 1.f;
    float sm = 0.f;
    for (int c = 0; c < C; ++c) sm += (wt ? wt[c] : 1.f) * (lse - z[c]);
    num += (1.f - ls) * wy * (lse - z[yb]) + ls / C * sm;
    den += wy;
  }
  num = wave_sum(num);
  den = wave_sum(den);
  if (lane == 0) {
    red[0][w] = num;
    red[1][w] = den;
  }
  __syncthreads();
  const float N = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const float Dn = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  if (tid == 0 && loss) *loss = N / Dn;
  if (!dlogits) return;
  for (int b = tid; b < B; b += 256) {
    const float* z = logits + (long)b * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, z[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(z[c] - m);
    const int yb = (int)y[b];
    const float wy = wt ? wt[yb] : 1.f;
    float wsum = 0.f;
    for (int c = 0; c < C; ++c) wsum += wt ? wt[c] : 1.f;
    for (int c = 0; c < C; ++c) {
      const float p = expf(z[c] - m) / se;
      // d/dz_c of (1-ls) wy (lse - z_y) + ls/C sum_k w_k (lse - z_k)
      float g = (1.f - ls) * wy * (p - (c == yb ? 1.f : 0.f)) + ls / C * (wsum * p - (wt ? wt[c] : 1.f));
      dlogits[(long)b * C + c] = g * gscale / Dn;
    }
  }
}

// ------------------------------------------------------------------ w+ prologue
// Block per (row r = b*L + l); 256 threads; D <= 1024. saved[r] = {mean, rstd}.
__global__ __launch_bounds__(256) void wplus_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int L,
                                                        int D, const float* sg, const float* sl, const int64_t* grp,
                                                        const float* lw, const float* lb, const float* gate,
                                                        const float* lm, float eps, float* saved) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  const int l = r % L, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = tid + i * 256;
    float a = 0.f;
    if (d < D) {
      a = x[r * D + d];
      if (sg) a += sg[grp[l] * D + d] + sl[(long)l * D + d];
    }
    v[i] = a;
    s += a;
  }
  float mu = 0.f, rs = 0.f;
  if (lw) {
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
    __syncthreads();
    mu = (red[0] + red[1] + red[2] + red[3]) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (tid + i * 256 < D) q += (v[i] - mu) * (v[i] - mu);
    q = wave_sum(q);
    if (lane == 0) red[4 + w] = q;
    __syncthreads();
    rs = rsqrtf((red[4] + red[5] + red[6] + red[7]) / D + eps);
  }
  const float sgate = gate ? 1.f / (1.f + __expf(-gate[l])) : 0.f;
  const float slm = lm ? 1.f / (1.f + __expf(-lm[l])) : 1.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = tid + i * 256;
    if (d >= D) continue;
    float u = v[i];
    if (lw) {
      const float n = (v[i] - mu) * rs * lw[(long)l * D + d] + lb[(long)l * D + d];
      u = gate ? v[i] + sgate * (n - v[i]) : n;
    }
    y[r * D + d] = u * slm;
  }
  if (tid == 0 && saved) {
    saved[2 * r] = mu;
    saved[2 * r + 1] = rs;
  }
}
// Block per (l, b-chunk). part layout per (chunk, l): [dlw D | dlb D | dsl D | dgate 1 | dleam 1]
__global__ __launch_bounds__(256) void wplus_bwd_kernel(const float* __restrict__ x, const float* __restrict__ saved,
                                                        const float* __restrict__ dy, float* __restrict__ dx, int B,
                                                        int L, int D, int bchunk, const float* sg, const float* sl,
                                                        const int64_t* grp, const float* lw, const float* lb,
                                                        const float* gate, const float* lm,
                                                        float* __restrict__ part) {
  __shared__ float red[3][4];
  const int l = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b0 = ch * bchunk, b1 = min(B, b0 + bchunk);
  const float sgate = gate ? 1.f / (1.f + __expf(-gate[l])) : 0.f;
  const float slm = lm ? 1.f / (1.f + __expf(-lm[l])) : 1.f;
  float plw[4] = {}, plb[4] = {}, psl[4] = {};
  float pgate = 0.f, pleam = 0.f;
  for (int b = b0; b < b1; ++b) {
    const long r = (long)b * L + l;
    const float mu = saved ? saved[2 * r] : 0.f, rs = saved ? saved[2 * r + 1] : 0.f;
    float v[4], xh[4], n[4], du[4];
    float a1 = 0.f, a2 = 0.f, ag = 0.f, al = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = tid + i * 256;
      v[i] = xh[i] = n[i] = du[i] = 0.f;
      if (d >= D) continue;
      float a = x[r * D + d];
      if (sg) a += sg[grp[l] * D + d] + sl[(long)l * D + d];
      v[i] = a;
      float u = a;
      if (lw) {
        xh[i] = (a - mu) * rs;
        n[i] = xh[i] * lw[(long)l * D + d] + lb[(long)l * D + d];
        u = gate ? a + sgate * (n[i] - a) : n[i];
      }
      const float g = dy[r * D + d];
      al += g * u;
      du[i] = g * slm;
    }
    // through LWN
    float dv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = tid + i * 256;
      dv[i] = du[i];
      if (d >= D || !lw) continue;
      const float dn = gate ? du[i] * sgate : du[i];
      if (gate) {
        ag += du[i] * (n[i] - v[i]);
        dv[i] = du[i] * (1.f - sgate);
      } else {
        dv[i] = 0.f;
      }
      plw[i] += dn * xh[i];
      plb[i] += dn;
      const float gg = dn * lw[(long)l * D + d];
      n[i] = gg;  // reuse: g*gamma
      a1 += gg;
      a2 += gg * xh[i];
    }
    if (lw) {
      a1 = wave_sum(a1);
      a2 = wave_sum(a2);
      ag = wave_sum(ag);
      __syncthreads();
      if (lane == 0) {
        red[0][w] = a1;
        red[1][w] = a2;
        red[2][w] = ag;
      }
      __syncthreads();
      const float m1 = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / D;
      const float m2 = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / D;
      if (tid == 0) pgate += red[2][0] + red[2][1] + red[2][2] + red[2][3];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (tid + i * 256 < D) dv[i] += (n[i] - m1 - xh[i] * m2) * rs;
    }
    al = wave_sum(al);
    __syncthreads();
    if (lane == 0) red[0][w] = al;
    __syncthreads();
    if (tid == 0) pleam += red[0][0] + red[0][1] + red[0][2] + red[0][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = tid + i * 256;
      if (d >= D) continue;
      dx[r * D + d] = dv[i];
      psl[i] += dv[i];
    }
  }
  const long ps = 3L * D + 2;
  float* pp = part + ((long)ch * L + l) * ps;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = tid + i * 256;
    if (d >= D) continue;
    pp[d] = plw[i];
    pp[D + d] = plb[i];
    pp[2 * D + d] = psl[i];
  }
  if (tid == 0) {
    pp[3 * D] = pgate * sgate * (1.f - sgate);
    pp[3 * D + 1] = pleam * slm * (1.f - slm);
  }
}
// reduce chunks; group embedding grad = sum of layer-embedding grads over its layers
__global__ void wplus_bwd_final(const float* __restrict__ part, int nch, int L, int D, const int64_t* grp, float* dsg,
                                float* dsl, float* dlw, float* dlb, float* dgate, float* dleam, int accumulate) {
  const long ps = 3L * D + 2;
  const long j = blockIdx.x * 256L + threadIdx.x;
  if (j >= (long)L * ps) return;
  const int l = j / ps;
  const long k = j - (long)l * ps;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[((long)c * L + l) * ps + k];
  float* o = nullptr;
  long oi = 0;
  if (k < D) { o = dlw; oi = (long)l * D + k; }
  else if (k < 2 * D) { o = dlb; oi = (long)l * D + k - D; }
  else if (k < 3 * D) { o = dsl; oi = (long)l * D + k - 2 * D; }
  else if (k == 3 * D) { o = dgate; oi = l; }
  else { o = dleam; oi = l; }
  if (o) o[oi] = accumulate ? o[oi] + s : s;
  if (k >= 2 * D && k < 3 * D && dsg && l == 0) {
    // group sums computed by the l == 0 thread of each column: fixed order over layers
    const int d = k - 2 * D;
    float gsum[3] = {0.f, 0.f, 0.f};
    for (int ll = 0; ll < L; ++ll) {
      float t = 0.f;
      for (int c = 0; c < nch; ++c) t += part[((long)c * L + ll) * ps + 2 * D + d];
      gsum[grp[ll]] += t;
    }
    for (int g = 0; g < 3; ++g) dsg[(long)g * D + d] = accumulate ? dsg[(long)g * D + d] + gsum[g] : gsum[g];
  }
}

// ------------------------------------------------------------------ decomposer
__global__ __launch_bounds__(256) void decomp_scores_kernel(const float* __restrict__ w, const float* __restrict__ dirs,
                                                            int C, int LD, float* __restrict__ scores) {
  __shared__ float red[16][4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float acc[16] = {};
  for (int i = tid; i < LD; i += 256) {
    const float x = w[(long)b * LD + i];
    for (int c = 0; c < C; ++c) acc[c] += x * dirs[(long)c * LD + i];
  }
  for (int c = 0; c < C; ++c) {
    const float s = wave_sum(acc[c]);
    if (lane == 0) red[c][wv] = s;
  }
  __syncthreads();
  if (tid < C) scores[(long)b * C + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}
__global__ __launch_bounds__(256) void decomp_out_kernel(const float* __restrict__ w, const float* __restrict__ dirs,
                                                         const float* __restrict__ scores, int C, int LD, int omode,
                                                         float alpha, int dmode, float* __restrict__ y) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= LD) return;
  const float* sc = scores + (long)b * C;
  float e = 0.f;
  if (dmode == 0) {
    for (int c = 0; c < C; ++c) e += sc[c] * dirs[(long)c * LD + i];
  } else {
    int best = 0;
    float bv = fabsf(sc[0]);
    for (int c = 1; c < C; ++c)
      if (fabsf(sc[c]) > bv) { bv = fabsf(sc[c]); best = c; }
    e = sc[best] * dirs[(long)best * LD + i];
  }
  const float x = w[(long)b * LD + i];
  const float idv = x - e;
  if (omode == 3) {
    y[(long)b * 2 * LD + i] = e;
    y[(long)b * 2 * LD + LD + i] = idv;
  } else {
    y[(long)b * LD + i] = omode == 0 ? e : (omode == 1 ? idv : idv + alpha * e);
  }
}

// ------------------------------------------------------------------ elementwise
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) y[i] = (bf16)x[i];
}
__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) y[i] = (float)x[i];
}
template <typename T>
__global__ void axpy_kernel(const T* __restrict__ x, const T* __restrict__ t, const float* __restrict__ s,
                            T* __restrict__ y, long n) {
  const float a = *s;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L)
    y[i] = from_f<T>(to_f<T>(x[i]) + a * to_f<T>(t[i]));
}
template <typename T>
__global__ __launch_bounds__(256) void dot_part_kernel(const T* __restrict__ a, const T* __restrict__ b, long n,
                                                       float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L)
    s += to_f<T>(a[i]) * (b ? to_f<T>(b[i]) : to_f<T>(a[i]));
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// Fixed-order (deterministic) sum of the partials: thread t adds partials t, t+256, ... in order,
// then a butterfly per wave and the four wave sums in order. (One thread walking up to 1024 partials
// was a chain of dependent L2 loads: 46 us per call, the hybrid adapters' alpha gradients 0.5 ms
// per step.)
__global__ __launch_bounds__(256) void sum_final_kernel(const float* __restrict__ part, int n, float* out,
                                                        int accumulate) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (red[0] + red[1]) + (red[2] + red[3]);
    *out = accumulate ? *out + t : t;
  }
}
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, uint32_t thr, float sc,
                               uint64_t seed) {
  seed = step_seed(seed);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L)
    y[i] = from_f<T>(drop_keep(seed, (uint32_t)i, thr) ? to_f<T>(x[i]) * sc : 0.f);
}
__global__ void clip_coef_kernel(const float* sumsq, float sq_scale, float max_norm, float* coef) {
  if (threadIdx.x) return;
  const float nrm = sqrtf(*sumsq * sq_scale);
  *coef = fminf(1.f, max_norm / (nrm + 1e-6f));
}

// ------------------------------------------------------------------ AdamW
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, bf16* __restrict__ pb,
                                                    const fer_adamw_segment* __restrict__ segs, float gscale,
                                                    const float* __restrict__ clip,
                                                    const uint64_t* __restrict__ step_add) {
  const fer_adamw_segment sg = segs[blockIdx.y];
  const float sc = gscale * (clip ? *clip : 1.f);
  const float t = (float)(sg.step + (step_add ? (long)*step_add : 0L));  // + graph replays
  const float bc1 = 1.f - powf(sg.beta1, t);
  const float bc2 = 1.f - powf(sg.beta2, t);
  const float step_size = sg.lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.f - sg.lr * sg.weight_decay;
  // 16-byte accesses over the segment's multiple-of-4 head (segment offsets are 64-element aligned
  // in FlatParams; checked per segment), then the per-element loop over the tail -- the same
  // arithmetic per element either way
  long j0 = 0;
  if ((sg.offset & 3) == 0) {
    j0 = sg.numel & ~3L;
    for (long j = (blockIdx.x * 256L + threadIdx.x) * 4; j < j0; j += (long)gridDim.x * 1024L) {
      const long i = sg.offset + j;
      const f32x4 g4 = *(const f32x4*)(g + i);
      f32x4 p4 = *(const f32x4*)(p + i), m4 = *(const f32x4*)(m + i), v4 = *(const f32x4*)(v + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gr = g4[e] * sc;
        float pv = p4[e] * decay;
        const float mv = sg.beta1 * m4[e] + (1.f - sg.beta1) * gr;
        const float vv = sg.beta2 * v4[e] + (1.f - sg.beta2) * gr * gr;
        m4[e] = mv;
        v4[e] = vv;
        pv -= step_size * mv / (sqrtf(vv) / bc2s + sg.eps);
        p4[e] = pv;
      }
      *(f32x4*)(m + i) = m4;
      *(f32x4*)(v + i) = v4;
      *(f32x4*)(p + i) = p4;
      if (pb) *(bf16x4*)(pb + i) = bf16x4{(bf16)p4[0], (bf16)p4[1], (bf16)p4[2], (bf16)p4[3]};
    }
  }
  for (long j = j0 + blockIdx.x * 256L + threadIdx.x; j < sg.numel; j += (long)gridDim.x * 256L) {
    const long i = sg.offset + j;
    const float gr = g[i] * sc;
    float pv = p[i] * decay;
    const float mv = sg.beta1 * m[i] + (1.f - sg.beta1) * gr;
    const float vv = sg.beta2 * v[i] + (1.f - sg.beta2) * gr * gr;
    m[i] = mv;
    v[i] = vv;
    pv -= step_size * mv / (sqrtf(vv) / bc2s + sg.eps);
    p[i] = pv;
    if (pb) pb[i] = (bf16)pv;
  }
}

static int grid_for(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

// Transposed bf16 weight shadow: for each 2-D segment {off, rows, cols, first_tile} of a flat
// buffer, dst[off + c*rows + r] = src[off + r*cols + c]. One launch over all segments (64x64
// tiles through LDS, block -> segment by binary search on first_tile). The dgrad GEMMs read the
// result as a K-contiguous operand (dX = dY W = dY (W^T)^T), which streams through the
// 16-byte-row DMA path instead of the transposed-LDS-read path of an MN operand.
__global__ __launch_bounds__(256) void transpose_segs_kernel(const uint16_t* __restrict__ src,
                                                             uint16_t* __restrict__ dst,
                                                             const int64_t* __restrict__ segs, int nseg) {
  __shared__ uint32_t tile[64][33];  // 64 rows x 64 bf16 (as 32 pairs), +1 word pad
  __shared__ __attribute__((aligned(16))) uint16_t t16x[64 * 72];  // fast path: rows padded by 16 B
  const long t = blockIdx.x;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid * 4 + 3] <= t) lo = mid;
    else hi = mid - 1;
  }
  const long off = segs[lo * 4], rows = segs[lo * 4 + 1], cols = segs[lo * 4 + 2];
  const long lt = t - segs[lo * 4 + 3], tc = (cols + 63) / 64;
  const long r0 = (lt / tc) * 64, c0 = (lt % tc) * 64;
  const uint16_t* s = src + off;
  uint16_t* d = dst + off;
  const int tid = threadIdx.x;
  if (r0 + 64 <= rows && c0 + 64 <= cols && rows % 8 == 0 && cols % 8 == 0 && off % 8 == 0) {
    // full, 16-byte aligned tile: 16-byte loads along input rows, 16-byte stores along output rows
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + k * 256, r = i >> 3, ch = i & 7;
      const uint4 v = *(const uint4*)(s + (r0 + r) * cols + c0 + ch * 8);
      *(uint4*)(t16x + r * 72 + ch * 8) = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + k * 256, c = i >> 3, rc = i & 7;  // output row c, 8 input rows from rc*8
      uint16_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = t16x[(rc * 8 + j) * 72 + c];
      uint4 o;
      o.x = e[0] | ((uint32_t)e[1] << 16);
      o.y = e[2] | ((uint32_t)e[3] << 16);
      o.z = e[4] | ((uint32_t)e[5] << 16);
      o.w = e[6] | ((uint32_t)e[7] << 16);
      *(uint4*)(d + (c0 + c) * rows + r0 + rc * 8) = o;
    }
    return;
  }
  // load: row r, column pair cp (2 bf16); 64 x 32 pairs = 2048 / 256 threads
  for (int i = tid; i < 64 * 32; i += 256) {
    const int r = i >> 5, cp = i & 31;
    const long gr = r0 + r, gc = c0 + cp * 2;
    uint32_t v = 0;
    if (gr < rows) {
      const uint16_t lo16 = gc < cols ? s[gr * cols + gc] : 0;
      const uint16_t hi16 = gc + 1 < cols ? s[gr * cols + gc + 1] : 0;
      v = lo16 | ((uint32_t)hi16 << 16);
    }
    tile[r][cp] = v;
  }
  __syncthreads();
  // store: output row c (= input column), pair of input rows rp
  for (int i = tid; i < 64 * 32; i += 256) {
    const int c = i >> 5, rp = i & 31;
    const long gc = c0 + c, gr = r0 + rp * 2;
    if (gc >= cols) continue;
    const uint32_t a = tile[rp * 2][c >> 1], b = tile[rp * 2 + 1][c >> 1];
    const uint16_t x0 = (c & 1) ? (uint16_t)(a >> 16) : (uint16_t)a;
    const uint16_t x1 = (c & 1) ? (uint16_t)(b >> 16) : (uint16_t)b;
    if (gr + 1 < rows && ((off + gc * rows + gr) & 1) == 0) {
      *(uint32_t*)(d + gc * rows + gr) = x0 | ((uint32_t)x1 << 16);
    } else {
      if (gr < rows) d[gc * rows + gr] = x0;
      if (gr + 1 < rows) d[gc * rows + gr + 1] = x1;
    }
  }
}

}  // namespace fer

using namespace fer;

int fer::set_step_ptr_misc(const uint64_t* p) { return set_step_ptr_here(p) == hipSuccess ? 0 : -1; }

extern "C" int64_t fer_colsum_ws(int M, int N) { return (int64_t)colsum_nblk(M) * N * 4; }

extern "C" int fer_reduce_defer(int mode, void* arena, int64_t arena_bytes, fer_stream_t stream) {
  std::lock_guard<std::mutex> lk(g_red_mu);
  if (mode == 2) {  // pause: keep the queue, stop taking new reductions
    g_red.take = false;
    return 0;
  }
  if (mode != 0 && mode != 1) return set_error("reduce_defer: mode must be 0, 1 or 2");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return set_error("reduce_defer: hipGetDevice failed");
  if (mode == 1 && g_red.on && dev != g_red.dev)
    return set_error("reduce_defer: a window is open on another device (one window per process)");
  const bool same = g_red.on && g_red.arena == (char*)arena && g_red.cap == (size_t)arena_bytes &&
                    g_red.st == (hipStream_t)stream;
  if (g_red.on && (mode == 0 || !same)) {
    const int rc = red_flush();
    g_red.on = g_red.take = false;
    if (rc) return rc;
  }
  if (mode == 0) return 0;
  if (!arena || arena_bytes < 65536) return set_error("reduce_defer: arena too small");
  if (!same) {
    g_red.arena = (char*)arena;
    g_red.cap = (size_t)arena_bytes;
    g_red.st = (hipStream_t)stream;
    g_red.used = 0;
  }
  g_red.dev = dev;
  g_red.on = g_red.take = true;
  return 0;
}

extern "C" int fer_reduce_flush(void) {
  std::lock_guard<std::mutex> lk(g_red_mu);
  return g_red.on ? red_flush() : 0;
}

extern "C" int fer_colsum(int dtype, const void* x, int64_t ldx, int M, int N, float* out, int accumulate,
                          const float* scale_ptr, float* ws, int64_t ws_bytes, fer_stream_t stream) {
  if (N <= 0) return 0;
  if (N % 4 || ldx % 4) return set_error("colsum: N and ld must be multiples of 4");
  const int nblk = colsum_nblk(M);
  if (!ws || ws_bytes < fer_colsum_ws(M, N)) return set_error("colsum: workspace too small");
  const int rpb = ceil_div(std::max(M, 1), nblk);
  hipStream_t st = (hipStream_t)stream;
  ws = reduction_ws(ws, (size_t)fer_colsum_ws(M, N), N, st);
  dim3 grid(ceil_div(N / 4, 64), nblk);
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(colsum_part_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)x, (long)ldx, M, N, ws, rpb);
  else
    hipLaunchKernelGGL(colsum_part_kernel<float>, grid, dim3(256), 0, st, (const float*)x, (long)ldx, M, N, ws, rpb);
  part_reduce(ws, nblk, N, N, N, out, nullptr, nullptr, accumulate, scale_ptr, st);
  return hip_check("colsum");
}

extern "C" int fer_im2col_patch(int dtype, const float* x, int B, int C, int Hh, int Ww, int P, void* cols,
                                int64_t ldc, fer_stream_t stream) {
  const long total = (long)B * (Hh / P) * (Ww / P) * C * P * P;
  if (total <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (P % 4 == 0 && Ww % 4 == 0 && ldc % 4 == 0 && total / 4 < 0x7FFFFFFFL && (uintptr_t)x % 16 == 0) {
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(im2col4_kernel<bf16>, dim3(grid_for(total / 4)), dim3(256), 0, st, x, B, C, Hh, Ww, P,
                         (bf16*)cols, (long)ldc);
    else
      hipLaunchKernelGGL(im2col4_kernel<float>, dim3(grid_for(total / 4)), dim3(256), 0, st, x, B, C, Hh, Ww, P,
                         (float*)cols, (long)ldc);
    return hip_check("im2col_patch");
  }
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, x, B, C, Hh, Ww, P, (bf16*)cols,
                       (long)ldc);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x, B, C, Hh, Ww, P,
                       (float*)cols, (long)ldc);
  return hip_check("im2col_patch");
}

extern "C" int fer_tokens_fwd(int dtype, const void* emb, const float* cls, const float* pos, void* t, int B, int n,
                              int D, uint32_t drop_thresh, float drop_scale, uint64_t seed, fer_stream_t stream) {
  const long total = (long)B * (n + 1) * D;
  if (total <= 0) return 0;
  if (check_drop_range(drop_thresh, total, "tokens_fwd: dropout over >= 2^32 elements")) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16 && D % 8 == 0 && total < (1L << 31)) {
    hipLaunchKernelGGL(tokens_fwd8_kernel, dim3(grid_for(total / 8)), dim3(256), 0, st, (const bf16*)emb, cls, pos,
                       (bf16*)t, B, n, D, drop_thresh, drop_scale, seed);
    return hip_check("tokens_fwd8");
  }
  if (D % 4 == 0) {
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(tokens_fwd4_kernel<bf16>, dim3(grid_for(total / 4)), dim3(256), 0, st, (const bf16*)emb, cls,
                         pos, (bf16*)t, B, n, D, drop_thresh, drop_scale, seed);
    else
      hipLaunchKernelGGL(tokens_fwd4_kernel<float>, dim3(grid_for(total / 4)), dim3(256), 0, st, (const float*)emb,
                         cls, pos, (float*)t, B, n, D, drop_thresh, drop_scale, seed);
    return hip_check("tokens_fwd");
  }
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(tokens_fwd_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)emb, cls, pos,
                       (bf16*)t, B, n, D, drop_thresh, drop_scale, seed);
  else
    hipLaunchKernelGGL(tokens_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)emb, cls,
                       pos, (float*)t, B, n, D, drop_thresh, drop_scale, seed);
  return hip_check("tokens_fwd");
}

static int tokens_chunks(int B) { return std::max(1, std::min(B, 64)); }
extern "C" int64_t fer_tokens_bwd_ws(int B, int N, int D) { return (int64_t)tokens_chunks(B) * N * D * 4; }

extern "C" int fer_tokens_bwd(int dtype, const void* dt, void* demb, float* dcls, float* dpos, int accumulate, int B,
                              int n, int D, uint32_t drop_thresh, float drop_scale, uint64_t seed, float* ws,
                              int64_t ws_bytes, fer_stream_t stream) {
  const int N = n + 1;
  if (B <= 0) return 0;
  const int nch = tokens_chunks(B);
  if (!ws || ws_bytes < fer_tokens_bwd_ws(B, N, D)) return set_error("tokens_bwd: workspace too small");
  if (check_drop_range(drop_thresh, (long)B * N * D, "tokens_bwd: dropout over >= 2^32 elements")) return -1;
  int bchunk = ceil_div(B, nch);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16 && D % 8 == 0) {
    const int nch8 = std::min(nch, 16);  // (the workspace is sized for tokens_chunks(B) >= nch8 slabs)
    bchunk = ceil_div(B, nch8);
    dim3 grid8(ceil_div((long)N * D / 8, 256), nch8);
    hipLaunchKernelGGL(tokens_bwd8_kernel, grid8, dim3(256), 0, st, (const bf16*)dt, (bf16*)demb, B, n, D, drop_thresh,
                       drop_scale, seed, ws, bchunk);
    if (dpos) part_reduce(ws, nch8, (long)N * D, N * D, N * D, dpos, nullptr, nullptr, accumulate, nullptr, st);
    if (dcls) part_reduce(ws, nch8, (long)N * D, D, D, dcls, nullptr, nullptr, accumulate, nullptr, st);
    return hip_check("tokens_bwd8");
  }
  if (D % 4 == 0) {
    dim3 grid4(ceil_div((long)N * D / 4, 256), nch);
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(tokens_bwd4_kernel<bf16>, grid4, dim3(256), 0, st, (const bf16*)dt, (bf16*)demb, B, n, D,
                         drop_thresh, drop_scale, seed, ws, bchunk);
    else
      hipLaunchKernelGGL(tokens_bwd4_kernel<float>, grid4, dim3(256), 0, st, (const float*)dt, (float*)demb, B, n,
                         D, drop_thresh, drop_scale, seed, ws, bchunk);
  } else {
    dim3 grid(ceil_div((long)N * D, 256), nch);
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(tokens_bwd_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)dt, (bf16*)demb, B, n, D,
                         drop_thresh, drop_scale, seed, ws, bchunk);
    else
      hipLaunchKernelGGL(tokens_bwd_kernel<float>, grid, dim3(256), 0, st, (const float*)dt, (float*)demb, B, n, D,
                         drop_thresh, drop_scale, seed, ws, bchunk);
  }
  if (dpos) part_reduce(ws, nch, (long)N * D, N * D, N * D, dpos, nullptr, nullptr, accumulate, nullptr, st);
  if (dcls) part_reduce(ws, nch, (long)N * D, D, D, dcls, nullptr, nullptr, accumulate, nullptr, st);
  return hip_check("tokens_bwd");
}

extern "C" int fer_head_fwd(int dtype, const void* t, int64_t row_stride, const float* ln_w, const float* ln_b,
                            float eps, const float* W, const float* bias, float* logits, float* stats, int B, int D,
                            int C, uint32_t drop_thresh, float drop_scale, uint64_t seed, fer_stream_t stream) {
  if (B <= 0) return 0;
  if (D > 1024) return set_error("head_fwd: D <= 1024");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16>, dim3(B), dim3(256), 0, st, (const bf16*)t, (long)row_stride, ln_w, ln_b,
                       eps, W, bias, logits, stats, D, C, drop_thresh, drop_scale, seed);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(B), dim3(256), 0, st, (const float*)t, (long)row_stride, ln_w,
                       ln_b, eps, W, bias, logits, stats, D, C, drop_thresh, drop_scale, seed);
  return hip_check("head_fwd");
}

extern "C" int64_t fer_head_bwd_ws(int B, int D, int C) { return (int64_t)B * ((int64_t)C * D + C + 2 * D) * 4; }

extern "C" int fer_head_bwd(int dtype, const void* t, int64_t row_stride, const float* ln_w, const float* ln_b,
                            const float* W, const float* stats, const float* dlogits, void* dt, int zero_rest,
                            int rows_total, int D_ld, float* dln_w, float* dln_b, float* dW, float* dbias,
                            int accumulate, int B, int D, int C, uint32_t drop_thresh, float drop_scale,
                            uint64_t seed, float* ws, int64_t ws_bytes, fer_stream_t stream) {
  if (B <= 0) return 0;
  if (D > 1024) return set_error("head_bwd: D <= 1024");
  if (!ws || ws_bytes < fer_head_bwd_ws(B, D, C)) return set_error("head_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (zero_rest && D % 4 == 0 && D_ld % 4 == 0) {
    const long total = (long)rows_total * D / 4;
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(zero_rows4_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (bf16*)dt, (long)rows_total,
                         D_ld, D, (long)(row_stride / D_ld));
    else
      hipLaunchKernelGGL(zero_rows4_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (float*)dt,
                         (long)rows_total, D_ld, D, (long)(row_stride / D_ld));
  } else if (zero_rest) {
    const long total = (long)rows_total * D;
    if (dtype == FER_BF16)
      hipLaunchKernelGGL(zero_rows_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (bf16*)dt, (long)rows_total,
                         D_ld, D, (long)(row_stride / D_ld));
    else
      hipLaunchKernelGGL(zero_rows_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (float*)dt,
                         (long)rows_total, D_ld, D, (long)(row_stride / D_ld));
  }
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(head_bwd_kernel<bf16>, dim3(B), dim3(256), 0, st, (const bf16*)t, (long)row_stride, ln_w, ln_b,
                       W, stats, dlogits, (bf16*)dt, D, C, drop_thresh, drop_scale, seed, ws);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(B), dim3(256), 0, st, (const float*)t, (long)row_stride, ln_w,
                       ln_b, W, stats, dlogits, (float*)dt, D, C, drop_thresh, drop_scale, seed, ws);
  const long ps = (long)C * D + C + 2 * D;
  if (dW) part_reduce(ws, B, ps, C * D, C * D, dW, nullptr, nullptr, accumulate, nullptr, st);
  if (dbias) part_reduce(ws + (long)C * D, B, ps, C, C, dbias, nullptr, nullptr, accumulate, nullptr, st);
  if (dln_w || dln_b) part_reduce(ws + (long)C * D + C, B, ps, 2 * D, D, dln_w, dln_b, nullptr, accumulate, nullptr, st);
  return hip_check("head_bwd");
}

extern "C" int fer_cross_entropy(const float* logits, const int64_t* labels, const float* weight, int B, int C,
                                 float label_smoothing, float grad_scale, float* loss, float* dlogits,
                                 fer_stream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, labels, weight, B, C,
                     label_smoothing, grad_scale, loss, dlogits);
  return hip_check("cross_entropy");
}

static int wplus_chunks(int B) { return std::max(1, std::min(B, 32)); }
extern "C" int64_t fer_wplus_ws(int B, int L, int D) { return (int64_t)wplus_chunks(B) * L * (3L * D + 2) * 4; }

extern "C" int fer_wplus_fwd(const float* x, float* y, int B, int L, int D, const float* spe_group,
                             const float* spe_layer, const int64_t* groups, const float* lwn_w, const float* lwn_b,
                             const float* lwn_gate, const float* leam_w, float eps, float* saved,
                             fer_stream_t stream) {
  if (B <= 0) return 0;
  if (D > 1024) return set_error("wplus_fwd: D <= 1024");
  hipLaunchKernelGGL(wplus_fwd_kernel, dim3(B * L), dim3(256), 0, (hipStream_t)stream, x, y, L, D, spe_group,
                     spe_layer, groups, lwn_w, lwn_b, lwn_gate, leam_w, eps, saved);
  return hip_check("wplus_fwd");
}

extern "C" int fer_wplus_bwd(const float* x, const float* saved, const float* dy, float* dx, int B, int L, int D,
                             const float* spe_group, const float* spe_layer, const int64_t* groups,
                             const float* lwn_w, const float* lwn_b, const float* lwn_gate, const float* leam_w,
                             float eps, float* d_spe_group, float* d_spe_layer, float* d_lwn_w, float* d_lwn_b,
                             float* d_lwn_gate, float* d_leam_w, int accumulate, float* ws, int64_t ws_bytes,
                             fer_stream_t stream) {
  (void)eps;
  if (B <= 0) return 0;
  if (!ws || ws_bytes < fer_wplus_ws(B, L, D)) return set_error("wplus_bwd: workspace too small");
  const int nch = wplus_chunks(B);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wplus_bwd_kernel, dim3(L, nch), dim3(256), 0, st, x, saved, dy, dx, B, L, D, ceil_div(B, nch),
                     spe_group, spe_layer, groups, lwn_w, lwn_b, lwn_gate, leam_w, ws);
  const long tot = (long)L * (3L * D + 2);
  hipLaunchKernelGGL(wplus_bwd_final, dim3(ceil_div(tot, 256)), dim3(256), 0, st, ws, nch, L, D, groups, d_spe_group,
                     d_spe_layer, d_lwn_w, d_lwn_b, d_lwn_gate, d_leam_w, accumulate);
  return hip_check("wplus_bwd");
}

extern "C" int fer_decompose(const float* w, const float* dirs, int B, int C, int LD, int output_mode, float alpha,
                             int decompose_mode, float* y, float* scores, fer_stream_t stream) {
  if (B <= 0) return 0;
  if (C > 16) return set_error("decompose: at most 16 directions");
  if (!scores) return set_error("decompose: scores buffer required");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(decomp_scores_kernel, dim3(B), dim3(256), 0, st, w, dirs, C, LD, scores);
  if (y)
    hipLaunchKernelGGL(decomp_out_kernel, dim3(ceil_div(LD, 256), B), dim3(256), 0, st, w, dirs, (const float*)scores,
                       C, LD, output_mode, alpha, decompose_mode, y);
  return hip_check("decompose");
}

extern "C" int fer_cast_f32_bf16(const float* x, void* y, int64_t n, fer_stream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, (long)n);
  return hip_check("cast_f32_bf16");
}
extern "C" int fer_cast_bf16_f32(const void* x, float* y, int64_t n, fer_stream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, y,
                     (long)n);
  return hip_check("cast_bf16_f32");
}
extern "C" int fer_axpy(int dtype, const void* x, const void* t, const float* scale_ptr, void* y, int64_t n,
                        fer_stream_t stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(axpy_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)x, (const bf16*)t,
                       scale_ptr, (bf16*)y, (long)n);
  else
    hipLaunchKernelGGL(axpy_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)x, (const float*)t,
                       scale_ptr, (float*)y, (long)n);
  return hip_check("axpy");
}
static int dot_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 1023) / 1024, 1024)); }
extern "C" int fer_dot(int dtype, const void* a, const void* b, int64_t n, float* out, int accumulate, float* ws,
                       int64_t ws_bytes, fer_stream_t stream) {
  const int nb = dot_blocks(n);
  if (!ws || ws_bytes < nb * 4) return set_error("dot: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(dot_part_kernel<bf16>, dim3(nb), dim3(256), 0, st, (const bf16*)a, (const bf16*)b, (long)n, ws);
  else
    hipLaunchKernelGGL(dot_part_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)a, (const float*)b, (long)n,
                       ws);
  hipLaunchKernelGGL(sum_final_kernel, dim3(1), dim3(256), 0, st, ws, nb, out, accumulate);
  return hip_check("dot");
}
extern "C" int fer_sumsq(const float* x, int64_t n, float* out, float* ws, int64_t ws_bytes, fer_stream_t stream) {
  return fer_dot(FER_F32, x, nullptr, n, out, 0, ws, ws_bytes, stream);
}
extern "C" int fer_clip_coef(const float* sumsq, float sq_scale, float max_norm, float* coef, fer_stream_t stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, sumsq, sq_scale, max_norm, coef);
  return hip_check("clip_coef");
}
extern "C" int fer_dropout(int dtype, const void* x, void* y, int64_t n, uint32_t drop_thresh, float drop_scale,
                           uint64_t seed, fer_stream_t stream) {
  if (n <= 0) return 0;
  if (check_drop_range(drop_thresh, n, "dropout: >= 2^32 elements")) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FER_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, (long)n,
                       drop_thresh, drop_scale, seed);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)x, (float*)y,
                       (long)n, drop_thresh, drop_scale, seed);
  return hip_check("dropout");
}
// ------------------------------------------------------------------ latent augmentation
// LatentAugment (`data/latent_dataset.py:6-49`) on device, in the reference's order:
// x += N(0, noise_std) (Box-Muller on two 32-bit hashes), x *= U(scale_lo, scale_hi) drawn once
// per sample, x *= (U(0,1) > mask_prob). Same distributions as the reference's torch RNG calls
// (not the same stream). Counter-based like the dropout masks: element i of the batch.
FER_DEV float u01(uint32_t h) { return ((float)(h >> 8) + 0.5f) * (1.f / 16777216.f); }
__global__ void latent_augment_kernel(float* __restrict__ x, long n, int LD, float noise_std, float scale_lo,
                                      float scale_hi, float mask_prob, uint64_t seed) {
  seed = step_seed(seed);
  const uint64_t s_noise = seed, s_scale = seed ^ 0x5851F42D4C957F2Dull, s_mask = seed ^ 0x14057B7EF767814Full;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
    float v = x[i];
    if (noise_std > 0.f) {
      const uint32_t e = (uint32_t)i;
      const float u1 = u01(fer_hash(s_noise, 2u * e)), u2 = u01(fer_hash(s_noise, 2u * e + 1u));
      v += noise_std * sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958648f * u2);
    }
    if (scale_hi > scale_lo || scale_lo != 1.f) {
      const uint32_t b = (uint32_t)(i / LD);
      v *= scale_lo + (scale_hi - scale_lo) * u01(fer_hash(s_scale, b));
    }
    if (mask_prob > 0.f && !(u01(fer_hash(s_mask, (uint32_t)i)) > mask_prob)) v = 0.f;
    x[i] = v;
  }
}

extern "C" int fer_transpose_bf16_segments(const void* src, void* dst, const int64_t* segs, int nseg,
                                          int64_t total_tiles, fer_stream_t stream) {
  if (nseg <= 0 || total_tiles <= 0) return 0;
  if (!src || !dst || !segs || src == dst) return set_error("transpose_bf16_segments: bad pointers (in-place is not supported)");
  hipLaunchKernelGGL(transpose_segs_kernel, dim3((unsigned)total_tiles), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)src, (uint16_t*)dst, segs, nseg);
  return hip_check("transpose_bf16_segments");
}

extern "C" int fer_latent_augment(float* x, int64_t B, int LD, float noise_std, float scale_lo, float scale_hi,
                                  float mask_prob, uint64_t seed, fer_stream_t stream) {
  const long n = (long)B * LD;
  if (n <= 0) return 0;
  if (n > 0x7FFFFFFFL) return set_error("latent_augment: more than 2^31 elements per call");
  hipLaunchKernelGGL(latent_augment_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, LD,
                     noise_std, scale_lo, scale_hi, mask_prob, seed);
  return hip_check("latent_augment");
}

__global__ void step_advance_kernel(uint64_t* counter) {
  if (threadIdx.x == 0) *counter += 1;
}

extern "C" int fer_step_advance(uint64_t* counter, fer_stream_t stream) {
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter);
  return hip_check("step_advance");
}

extern "C" int fer_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_bf16,
                         const fer_adamw_segment* segs_device, int nsegs, int64_t max_seg_numel, float grad_scale,
                         const float* clip_coef, const uint64_t* step_add, fer_stream_t stream) {
  if (nsegs <= 0) return 0;
  // blocks per segment: enough for the largest one to stream at full rate (the grid-stride loop
  // covers the rest); every block of a smaller segment past its end exits at once, and with one
  // block per 1024 elements of the largest segment those empty blocks (~80 % of a latent-ViT
  // launch's 82 k blocks) cost more than the update itself
  const long per_seg = std::max<long>(8, std::min<long>(256, 32768 / std::max(1, nsegs)));
  dim3 grid((unsigned)std::max<long>(1, std::min<long>((max_seg_numel + 1023) / 1024, per_seg)), nsegs);
  hipLaunchKernelGGL(adamw_kernel, grid, dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq,
                     (bf16*)param_bf16, segs_device, grad_scale, clip_coef, step_add);
  return hip_check("adamw");
}
