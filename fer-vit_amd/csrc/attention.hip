// Multi-head self-attention core for short token sequences (N <= 256):
// N = 10 (48 px ImageViT), 19 (w+ latents + CLS), 37 (concat decomposer), 197 (ViT-B/16).
// Replaces F.multi_head_attention_forward -> scaled_dot_product_attention inside
// nn.TransformerEncoderLayer (`image_vit.py:101`, `latent_vit.py:24`) and timm's Attention
// (hybrid). Dropout on the probabilities is regenerated from (seed, (bh*N+q)*N+k).
//
// bf16 path: one workgroup per (batch, head); the whole key/value set of the head lives in
// LDS ([Npad][64] bf16 images, Npad = 32*NB), one wave per 32-row block.
//   forward : S^T = K Q^T  (v_mfma_f32_32x32x16_bf16, K from LDS by ds_read_b128, Q in VGPRs)
//             softmax along the key axis = along the 16 accumulator registers + one lane-32 swap
//             O^T = V^T P^T (P^T taken straight from the accumulators as the B operand;
//             V^T fragments by ds_read_b64_tr_b16)
//   backward: phase 1 (wave = query block): S^T, dP^T -> dS^T -> dQ^T = K^T dS^T
//             phase 2 (wave = key block)  : S, dP -> dS -> dV = P_drop^T dO, dK = dS^T Q
//             (P and dS recomputed in each orientation: no atomics, deterministic)
// Every LDS image uses one swizzle that is bank-conflict free for both the b128 row reads
// and the transposed reads:  chunk' = chunk ^ f(row),  f(r) = ((r>>1)&1)<<2 | ((r>>2)&3).
//
// fp32 path (parity mode): straightforward kernels over a global [B*H][N][N] workspace.
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "fervit_internal.h"

namespace fer {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

FER_DEV int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
FER_DEV int img_off(int r, int c) { return r * 128 + ((c ^ swz(r)) << 4); }

// rows [0, 32*NB) of a [N][dh] column block (row stride ld) -> LDS image (zero padded)
template <int NB>
FER_DEV void load_image(char* img, const bf16* src, long ld, int N, int dh) {
  for (int idx = threadIdx.x; idx < NB * 32 * 8; idx += blockDim.x) {
    const int r = idx >> 3, c = idx & 7;
    bf16x8 v = {};
    if (r < N && c * 8 < dh) v = *(const bf16x8*)(src + (long)r * ld + c * 8);
    *(bf16x8*)(img + img_off(r, c)) = v;
  }
}

FER_DEV bf16x8 rd_row(const char* img, int r, int c) { return *(const bf16x8*)(img + img_off(r, c)); }
// == rd_row(img, R + (lane & 31), 2s + (lane >> 5)) for img + R * 128 passed as `img`
FER_DEV int row_base(int lane) { return (lane & 31) * 128 + (((lane >> 5) ^ swz(lane & 31)) << 4); }
FER_DEV bf16x8 rd_rowb(const char* img, int rb, int s) { return *(const bf16x8*)(img + (rb ^ (s << 5))); }

// B/A operand of the 32x32x16 MFMA built from 8 rows (k) of an image, columns cb..cb+31:
// lane l gets column cb + (l&31), rows R+{0..3} (elements 0..3) and R+8+{0..3} (4..7),
// R = rbase + 4*(l>>5).
FER_DEV bf16x8 rd_tr(const char* img, int rbase, int cb, int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int R = rbase + 4 * (gg >> 1);
  const int col = cb + 16 * (gg & 1) + 4 * p;
  const int c = col >> 3, half = (p & 1) * 8;
  const int r1 = R + q, r2 = R + 8 + q;
  const char* a1 = img + r1 * 128 + ((c ^ swz(r1)) << 4) + half;
  const char* a2 = img + r2 * 128 + ((c ^ swz(r2)) << 4) + half;
  short4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a1);
  short4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a2);
  return cat8(t1, t2);
}

FER_DEV bf16x8 pack8(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

FER_DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }

// accumulator register -> row within the 32-row tile
FER_DEV int acc_row(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

// Dropout element index of P[bh][q][k]: (bh*N + q)*NP + k with NP = N rounded up to even, so
// keys 2j, 2j+1 of one query share one 32-bit hash (one 16-bit half each).
FER_DEV uint32_t drop_row(int bh, int N, int q) { return ((uint32_t)bh * N + q) * (uint32_t)(N + (N & 1)); }

// v_exp_f32 without the denormal range fix-up of exp2f: arguments here are <= 0 (scores minus
// the running max / the logsumexp), results below 2^-126 flush to 0 and -inf gives 0.
FER_DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// Dropout of the 16 accumulator registers when registers hold KEYS (S^T orientation): registers
// 2i, 2i+1 are consecutive keys (the first even) = the two halves of one hash. v[r] *= keep ?
// dscale : 0 for every register.
FER_DEV void drop16_keys(uint64_t seed, uint32_t row, int kb, int hh, uint32_t thr, float dscale, f32x16& v) {
  const uint32_t p0 = (row >> 1) + kb * 16 + 2 * hh;  // pair of register 0
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const uint32_t h = fer_hash(seed, p0 + (uint32_t)(acc_row(r, 0) >> 1));
    v[r] = (h & 0xFFFFu) >= thr ? v[r] * dscale : 0.f;
    v[r + 1] = (h >> 16) >= thr ? v[r + 1] * dscale : 0.f;
  }
}

// rows [0, 32*NB) of a [N][dh] column block -> swizzled LDS image by LDS-DMA (16 B per lane,
// lane-linear destination, swizzle applied on the source address). Wave w of NB issues the
// four 1 KB pieces [4w, 4w+4). Rows >= N and chunks >= dh/8 are zero-filled (range check).
template <int NB>
FER_DEV void img_dma(char* img, __amdgpu_buffer_rsrc_t rs, long row0, long ld, int col0, int N, int dh, int w,
                     int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = 4 * w + i;
    const int r = pc * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ swz(r);
    const bool ok = r < N && ch * 8 < dh;
    const uint32_t voff = ok ? (uint32_t)(((row0 + r) * ld + col0 + ch * 8) * 2) : FER_OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + pc * 1024), 16, voff, 0, 0, 0);
  }
}

// img_dma through the inline-asm LDS-DMA (common.h dma16_asm): for kernels that wait explicitly
template <int NB>
FER_DEV void img_dma_asm(char* img, const u32x4& rs, long row0, long ld, int col0, int N, int dh, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = 4 * w + i;
    const int r = pc * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ swz(r);
    const bool ok = r < N && ch * 8 < dh;
    dma16_asm(img + pc * 1024, rs, ok ? (uint32_t)(((row0 + r) * ld + col0 + ch * 8) * 2) : FER_OOB);
  }
}

FER_DEV void store_rows_q(bf16* o, const f32x16& a0, const f32x16& a1, float mul, int hh, int dh) {
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x16& a = db ? a1 : a0;
      const int d = db * 32 + 8 * g4 + 4 * hh;
      if (d < dh)
        *(bf16x4*)(o + d) = bf16x4{(bf16)(a[4 * g4] * mul), (bf16)(a[4 * g4 + 1] * mul),
                                   (bf16)(a[4 * g4 + 2] * mul), (bf16)(a[4 * g4 + 3] * mul)};
    }
}

// ---------------------------------------------------------------- forward
// One workgroup per (batch, head), wave w = query block w. K and V images arrive by LDS-DMA;
// S^T = K Q^T per 32-key block with an online (running max) softmax, O^T += V^T P^T.
template <int NB>
__global__ __launch_bounds__(64 * NB) __attribute__((amdgpu_waves_per_eu(4))) void attn_fwd_bf16(const bf16* __restrict__ qkv, long ldq, bf16* __restrict__ out,
                                                          long ldo, float* __restrict__ lse, int N, int H, int dh,
                                                          float sl2, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  __shared__ __attribute__((aligned(1024))) char lds[2 * NB * 32 * 128];
  char* Ki = lds;
  char* Vi = lds + NB * 32 * 128;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(qkv);
  img_dma<NB>(Ki, rs, (long)b * N, ldq, D + h * dh, N, dh, w, lane);
  img_dma<NB>(Vi, rs, (long)b * N, ldq, 2 * D + h * dh, N, dh, w, lane);

  const int q = w * 32 + (lane & 31);
  const bf16* base = qkv + (long)b * N * ldq;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int d0 = 16 * s + 8 * hh;
    qf[s] = (q < N && d0 < dh) ? *(const bf16x8*)(base + (long)q * ldq + h * dh + d0) : bf16x8{};
  }
  __syncthreads();  // vmcnt(0) + barrier: every wave's DMA pieces have landed

  const uint32_t row = drop_row(bh, N, q);
  float m = -INFINITY, l = 0.f;
  f32x16 ot[2] = {f32x16{}, f32x16{}};
#pragma unroll 1
  for (int kb = 0; kb < NB; ++kb) {
    f32x16 st = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) st = mfma32(rd_row(Ki, kb * 32 + (lane & 31), 2 * s + hh), qf[s], st);
    if (kb * 32 + 32 > N) {  // only the last key block has padding keys (wave-uniform)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb * 32 + acc_row(r, hh) >= N) st[r] = -INFINITY;
    }
    float bm = st[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) bm = fmaxf(bm, st[r]);
    bm = xhalf_max(bm) * sl2;
    const float mn = fmaxf(m, bm);
    const float al = ex2(m - mn);
    m = mn;
    l *= al;
#pragma unroll
    for (int db = 0; db < 2; ++db) ot[db] *= al;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      st[r] = ex2(fmaf(st[r], sl2, -mn));
      l += st[r];
    }
    if (thr) drop16_keys(seed, row, kb, hh, thr, dscale, st);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = pack8(st, s2);
#pragma unroll
      for (int db = 0; db < 2; ++db) ot[db] = mfma32(rd_tr(Vi, kb * 32 + 16 * s2, db * 32, lane), pf, ot[db]);
    }
  }
  l = xhalf_sum(l);
  if (q < N) {
    store_rows_q(out + ((long)b * N + q) * ldo + h * dh, ot[0], ot[1], 1.f / l, hh, dh);
    if (hh == 0) lse[(long)bh * N + q] = (m + log2f(l)) * LN2;
  }
}

// ---------------------------------------------------------------- forward, persistent
// One workgroup per CU walks the (batch, head) units u = blockIdx.x, + gridDim.x, ...: NB compute
// waves (wave w = query block w) and one producer wave that DMAs the NEXT unit's K and V images
// into the other half of a double buffer while the compute waves work on the current unit, so the
// load phase hides behind the compute phase (one barrier per unit). Compute waves load their next
// Q fragments at the start of the current unit.
// Softmax with lazy rescaling: a row's running max m (log2 units) only moves -- and O, l are
// rescaled -- when a key block's max exceeds it by more than 8 (wave-uniform branch), so
// P = 2^(s*scale*log2e - m) <= 2^8 and the result is the exact softmax (l uses the same m).
// Dropout: keep bits hashed as in the other kernels; dscale is applied once per output row instead
// of once per probability. With `mask` the keep bits are also stored for the backward:
// mask[((bh*NB + kb)*NB + qb)*32 + j] = bits over the 32 queries of block qb for key kb*32 + j
// (the ballot of the keep compare of one accumulator register IS such a word for two keys; a
// wave stores / loads the 32 words of one (kb, qb) tile as one 128-byte row).

// Ballots of the keep compares of accumulator registers R..R+7 (register r: keys acc_row(r, 0)
// (lanes 0-31) and acc_row(r, 0) + 4 (lanes 32-63)) -> lane k of w takes the 32 query bits of key k
// (v_writelane_b32). The s_nop: a v_writelane reading an SGPR that a VALU compare wrote in the
// previous instruction reads the stale value (measured: those keys came back all-zero) and the
// compiler does not pad inline asm; one nop ahead of 16 writelanes covers all 8 ballots.
template <int R>
FER_DEV uint32_t wl_keys8(uint32_t w, const uint64_t* b) {
  constexpr int k0 = 8 * (R >> 2), k2 = k0 + 2, k4 = k0 + 8, k6 = k0 + 10;
  asm volatile(
      "s_nop 4\n\t"
      "v_writelane_b32 %0, %1, %17\n\tv_writelane_b32 %0, %2, %18\n\t"
      "v_writelane_b32 %0, %3, %19\n\tv_writelane_b32 %0, %4, %20\n\t"
      "v_writelane_b32 %0, %5, %21\n\tv_writelane_b32 %0, %6, %22\n\t"
      "v_writelane_b32 %0, %7, %23\n\tv_writelane_b32 %0, %8, %24\n\t"
      "v_writelane_b32 %0, %9, %25\n\tv_writelane_b32 %0, %10, %26\n\t"
      "v_writelane_b32 %0, %11, %27\n\tv_writelane_b32 %0, %12, %28\n\t"
      "v_writelane_b32 %0, %13, %29\n\tv_writelane_b32 %0, %14, %30\n\t"
      "v_writelane_b32 %0, %15, %31\n\tv_writelane_b32 %0, %16, %32"
      : "+v"(w)
      : "s"((uint32_t)b[0]), "s"((uint32_t)(b[0] >> 32)), "s"((uint32_t)b[1]), "s"((uint32_t)(b[1] >> 32)),
        "s"((uint32_t)b[2]), "s"((uint32_t)(b[2] >> 32)), "s"((uint32_t)b[3]), "s"((uint32_t)(b[3] >> 32)),
        "s"((uint32_t)b[4]), "s"((uint32_t)(b[4] >> 32)), "s"((uint32_t)b[5]), "s"((uint32_t)(b[5] >> 32)),
        "s"((uint32_t)b[6]), "s"((uint32_t)(b[6] >> 32)), "s"((uint32_t)b[7]), "s"((uint32_t)(b[7] >> 32)),
        "n"(k0), "n"(k0 + 4), "n"(k0 + 1), "n"(k0 + 5), "n"(k2), "n"(k2 + 4), "n"(k2 + 1), "n"(k2 + 5),
        "n"(k4), "n"(k4 + 4), "n"(k4 + 1), "n"(k4 + 5), "n"(k6), "n"(k6 + 4), "n"(k6 + 1), "n"(k6 + 5));
  return w;
}

// wl_keys8<0> for accumulator registers 0-3 only (keys 0-7 of the block; lanes 8-31 of w unchanged)
FER_DEV uint32_t wl_keys4(uint32_t w, const uint64_t* b) {
  asm volatile(
      "s_nop 4\n\t"
      "v_writelane_b32 %0, %1, 0\n\tv_writelane_b32 %0, %2, 4\n\t"
      "v_writelane_b32 %0, %3, 1\n\tv_writelane_b32 %0, %4, 5\n\t"
      "v_writelane_b32 %0, %5, 2\n\tv_writelane_b32 %0, %6, 6\n\t"
      "v_writelane_b32 %0, %7, 3\n\tv_writelane_b32 %0, %8, 7"
      : "+v"(w)
      : "s"((uint32_t)b[0]), "s"((uint32_t)(b[0] >> 32)), "s"((uint32_t)b[1]), "s"((uint32_t)(b[1] >> 32)),
        "s"((uint32_t)b[2]), "s"((uint32_t)(b[2] >> 32)), "s"((uint32_t)b[3]), "s"((uint32_t)(b[3] >> 32)));
  return w;
}

template <int NB>
FER_DEV void fwd_dma_unit(char* buf, const u32x4& rs, int unit, long ldq, int N, int H, int dh, int lane) {
  const int b = unit / H, h = unit - b * H, D = H * dh;
#pragma unroll 1
  for (int ww = 0; ww < NB; ++ww) {
    img_dma_asm<NB>(buf, rs, (long)b * N, ldq, D + h * dh, N, dh, ww, lane);
    img_dma_asm<NB>(buf + NB * 32 * 128, rs, (long)b * N, ldq, 2 * D + h * dh, N, dh, ww, lane);
  }
}

FER_DEV void fwd_load_q(bf16x8 (&qf)[4], const bf16* qkv, long ldq, int unit, int N, int H, int dh, int q, int hh) {
  const int b = unit / H, h = unit - b * H;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int d0 = 16 * s + 8 * hh;
    qf[s] = (q < N && d0 < dh) ? *(const bf16x8*)(qkv + ((long)b * N + q) * ldq + h * dh + d0) : bf16x8{};
  }
}

#ifdef FER_ATTN_STAMPS
// Diagnostic build only: s_memtime stamps of workgroup 0, units 2..3, every wave (lane 0).
__device__ unsigned long long g_ast[9][64];
__device__ unsigned long long g_bst[8][128];
#define BST(i)                                                                        \
  do {                                                                                \
    if (bst_on) {                                                                     \
      unsigned long long t_;                                                          \
      __builtin_amdgcn_sched_barrier(0);                                              \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      __builtin_amdgcn_sched_barrier(0);                                              \
      if ((threadIdx.x & 63) == 0) g_bst[w][(i)] = t_;                                \
    }                                                                                 \
  } while (0)
#define AST(i)                                                                        \
  do {                                                                                \
    if (st_on) {                                                                      \
      unsigned long long t_;                                                          \
      __builtin_amdgcn_sched_barrier(0);                                              \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
      __builtin_amdgcn_sched_barrier(0);                                              \
      if (lane == 0) g_ast[w][(i)] = t_;                                              \
    }                                                                                 \
  } while (0)
#else
#define AST(i) do {} while (0)
#define BST(i) do {} while (0)
#endif

template <int NB>
__global__ __launch_bounds__(64 * (NB + 1)) void attn_fwd_pers(const bf16* __restrict__ qkv, long ldq,
                                                               bf16* __restrict__ out, long ldo,
                                                               float* __restrict__ lse, uint32_t* __restrict__ mask,
                                                               int BH, int N, int H, int dh, float sl2, uint32_t thr,
                                                               float dscale, uint64_t seed, WqArgs wq) {
  seed = step_seed(seed);
  constexpr int IMG = NB * 32 * 128;
  __shared__ __attribute__((aligned(1024))) char lds[4 * IMG + 16];  // 2 x (K image, V image), unit hand-off
  lds_vint* hand = FER_LDS_INT(lds + 4 * IMG);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const u32x4 rs = rsrc4(qkv);
  const int q = w * 32 + (lane & 31);
  // Every global access of the consumers is a buffer op with the out-of-range lanes at FER_OOB (dropped
  // / zero-filled by the range check) instead of an exec-masked one: the compiler's vmcnt counts stay
  // exact (with masked loads it flushed vmcnt(0) at the key-block loop's entry, i.e. waited for the
  // next unit's Q prefetch before starting this unit). Per-lane offsets once; the unit part is the
  // scalar offset.
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv), ro = make_rsrc(out), rl = make_rsrc(lse),
                               rmk = make_rsrc(mask ? (const void*)mask : (const void*)lse);
  // per-lane Q / O offsets recomputed where they are used (not 12 VGPRs held through the key blocks)
  // (32-bit offsets: the host keeps qkv / out under 2 GiB; selects, not branches)
  // (arithmetic, not a select: hipcc turned the select into two exec-masked copies of the load)
  auto q_off = [&](int s, int ln) -> uint32_t {
    const int qq = w * 32 + (ln & 31), d0 = 16 * s + 8 * (ln >> 5);
    const uint32_t off = ((uint32_t)qq * (uint32_t)ldq + (uint32_t)d0) * 2u;
    return off | ((uint32_t)(qq >= N || d0 >= dh) << 31);  // bit 31 set: past the range (FER_OOB)
  };
  auto o_off = [&](int i, int ln) -> uint32_t {
    const int qq = w * 32 + (ln & 31), d = (i >> 2) * 32 + 8 * (i & 3) + 4 * (ln >> 5);
    const uint32_t off = ((uint32_t)qq * (uint32_t)ldo + (uint32_t)d) * 2u;
    return off | ((uint32_t)(qq >= N || d >= dh) << 31);
  };
  const uint32_t lse_off = (q < N && hh == 0) ? (uint32_t)(q * 4) : FER_OOB;
  const uint32_t mk_off = (mask && lane < 32) ? (uint32_t)(lane * 4) : FER_OOB;
  auto load_q = [&](bf16x8 (&qv)[4], int unit) {
    const int b = unit / H, h = unit - b * H;
    const int so = __builtin_amdgcn_readfirstlane((int)((((long)b * N) * ldq + h * dh) * 2));
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qv[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, q_off(s, lane), so, 0));
  };
  // units: fixed stride, or the work queue `wq` (common.h): the first unit is blockIdx.x, the next
  // one is claimed at the start, then the producer's lane 0 claims the unit after next while this
  // one runs and hands it on through hand[k & 1] at the unit's last barrier
  const bool claimer = threadIdx.x == 64 * NB;
  int u, un;
  if (wq.q) {
    u = wq_first(BH);
    if (u < 0) return;
  } else {
    u = blockIdx.x;
    un = u + (int)gridDim.x < BH ? u + (int)gridDim.x : -1;
  }
  // producer and compute waves run separate unit loops with the same barriers (prologue + one per
  // unit) and hand-off reads: a loop shared by both roles merged their register states at its latch
  if (w == NB) {
    uint32_t c0 = 0;
    if (wq.q && claimer) c0 = wq_claim_issue(wq.q);  // its round trip overlaps the DMA wait
    fwd_dma_unit<NB>(lds, rs, u, ldq, N, H, dh, lane);
    wait_vm<0>();
    asm volatile("" : "+v"(c0));
    if (wq.q && claimer) hand[2] = wq_claim_finish(c0, wq.base, BH);
    bar_lds();
    if (wq.q) un = __builtin_amdgcn_readfirstlane(hand[2]);
#pragma unroll 1
    for (int k = 0;; ++k) {
#ifdef FER_ATTN_STAMPS
      const bool st_on = blockIdx.x == 0 && (k == 2 || k == 3);
      const int sb = (k - 2) * 32;
#endif
      AST(sb + 0);
      int unn = -1;
      uint32_t craw = 0;
      if (wq.q) {
        if (claimer && un >= 0) craw = wq_claim_issue(wq.q);
      } else if (un >= 0 && un + (int)gridDim.x < BH) {
        unn = un + gridDim.x;
      }
      if (un >= 0) fwd_dma_unit<NB>(lds + ((k + 1) & 1) * 2 * IMG, rs, un, ldq, N, H, dh, lane);
      AST(sb + 1);
      wait_vm<0>();
      AST(sb + 2);
      asm volatile("" : "+v"(craw));
      if (wq.q && claimer && un >= 0) unn = wq_claim_finish(craw, wq.base, BH);
      if (claimer) hand[k & 1] = unn;
      bar_lds();  // the DMA of unit un has landed (wait_vm above); every wave is done with unit u
      AST(sb + 21);
      u = un;
      un = __builtin_amdgcn_readfirstlane(hand[k & 1]);
      if (u < 0) break;
    }
    return;
  }
  bf16x8 qf[4];
  load_q(qf, u);
  // consumed here: the first unit's loads complete before the loop, so the loop header's wait state
  // (merged over this entry and the back edge) keeps the back edge's count -- Q issued before the
  // previous unit's 9 output stores -- instead of waiting for those stores too
  asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]));
  bar_lds();
  if (wq.q) un = __builtin_amdgcn_readfirstlane(hand[2]);
#pragma unroll 1
  for (int k = 0;; ++k) {
#ifdef FER_ATTN_STAMPS
    const bool st_on = blockIdx.x == 0 && (k == 2 || k == 3);
    const int sb = (k - 2) * 32;
#endif
    AST(sb + 0);
    {
      const char* Ki = lds + (k & 1) * 2 * IMG;
      const char* Vi = Ki + IMG;
      const int bh = u, b = u / H, h = u - b * H;
      const uint32_t row = drop_row(bh, N, q);
      float m = -INFINITY, l = 0.f;
      f32x16 ot[2] = {f32x16{}, f32x16{}};
      bf16x8 kfr[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kfr[s] = rd_row(Ki, lane & 31, 2 * s + hh);
      // softmax + dropout + P.V of key block kb, whose S^T is in st
      auto block = [&](int kb, f32x16& st, const bf16x8 (&vfr)[2][2]) {
        if (kb == NB - 1 && NB * 32 > N) {  // only the last key block has padding keys
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kb * 32 + acc_row(r, hh) >= N) st[r] = -INFINITY;
        }
        float bm = fmaxf(fmaxf(st[0], st[1]), st[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) bm = fmaxf(fmaxf(bm, st[r]), st[r + 1]);
        bm = fmaxf(bm, st[15]);
        bm = xhalf_max(bm) * sl2;
        if (__builtin_amdgcn_ballot_w64(bm > m + 8.f)) {  // wave-uniform
          const float mn = fmaxf(m, bm);
          const float al = ex2(m - mn);
          m = mn;
          l *= al;
          ot[0] *= al;
          ot[1] *= al;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) st[r] = ex2(fmaf(st[r], sl2, -m));
        // the block's row sum as a tree (four independent chains), not a 16-long dependent chain
        float ls[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) ls[c] = (st[c] + st[c + 4]) + (st[c + 8] + st[c + 12]);
        l += (ls[0] + ls[1]) + (ls[2] + ls[3]);
        if (thr) {
          const uint32_t p0 = (row >> 1) + kb * 16 + 2 * hh;  // hash pair of register 0
          uint64_t bal[16];
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const uint32_t hv = fer_hash(seed, p0 + (uint32_t)(acc_row(r, 0) >> 1));
            const bool k0 = (hv & 0xFFFFu) >= thr, k1 = (hv >> 16) >= thr;
            st[r] = k0 ? st[r] : 0.f;
            st[r + 1] = k1 ? st[r + 1] : 0.f;
            bal[r] = __builtin_amdgcn_ballot_w64(k0);
            bal[r + 1] = __builtin_amdgcn_ballot_w64(k1);
          }
          if (mask) {  // two independent writelane chains (lanes 0-15, 16-31)
            const uint32_t word = wl_keys8<0>(0u, bal) | wl_keys8<8>(0u, bal + 8);
            __builtin_amdgcn_raw_buffer_store_b32(
                word, rmk, mk_off, __builtin_amdgcn_readfirstlane((int)((((long)bh * NB + kb) * NB + w) * 128)), 0);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pf = pack8(st, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db) ot[db] = mfma32(vfr[s2][db], pf, ot[db]);
        }
      };
#pragma unroll 1
      for (int kb = 0; kb < NB; ++kb) {
        bf16x8 vfr[2][2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int db = 0; db < 2; ++db) vfr[s2][db] = rd_tr(Vi, kb * 32 + 16 * s2, db * 32, lane);
        f32x16 st = {};
#pragma unroll
        for (int s = 0; s < 4; ++s) st = mfma32(kfr[s], qf[s], st);
        if (kb + 1 < NB) {
#pragma unroll
          for (int s = 0; s < 4; ++s) kfr[s] = rd_row(Ki, (kb + 1) * 32 + (lane & 31), 2 * s + hh);
        }
        AST(sb + 1 + 2 * kb);
        block(kb, st, vfr);
        AST(sb + 2 + 2 * kb);
      }
      // the next unit's Q straight into qf (dead after the last key block): issued ahead of the output
      // stores, so its wait at the next unit's first key block skips them; unconditional (un < 0: this
      // unit's again), so the loop carries one version of qf
      load_q(qf, un >= 0 ? un : u);
      l = xhalf_sum(l);
      {
        const float mul = dscale / l;
        const int so = __builtin_amdgcn_readfirstlane((int)((((long)b * N) * ldo + h * dh) * 2));
        // 16-byte stores of chunk pairs through permlane32 swaps, as attn_fwd_occ
        auto pack4 = [&](int i) {
          const f32x16& a = ot[i >> 2];
          const int g4 = i & 3;
          const bf16x4 v = {(bf16)(a[4 * g4] * mul), (bf16)(a[4 * g4 + 1] * mul), (bf16)(a[4 * g4 + 2] * mul),
                            (bf16)(a[4 * g4 + 3] * mul)};
          return __builtin_bit_cast(u32x2, v);
        };
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          const u32x2 pk[2] = {pack4(i), pack4(i + 1)};
          const auto x = __builtin_amdgcn_permlane32_swap(pk[0][0], pk[1][0], false, false);
          const auto y = __builtin_amdgcn_permlane32_swap(pk[0][1], pk[1][1], false, false);
          // o_off(i + hh, lane & 31): chunk i + hh of the row = d 8 (i + hh)
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{x[0], y[0], x[1], y[1]}, ro, o_off(i + hh, lane & 31), so, 0);
        }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((m + log2f(l)) * LN2), rl, lse_off,
                                              __builtin_amdgcn_readfirstlane(bh * N * 4), 0);
      }
      AST(sb + 20);
    }
    bar_lds();  // the producer's DMA of unit un has landed (its wait_vm); every wave is done with unit u
    AST(sb + 21);
    u = un;
    un = __builtin_amdgcn_readfirstlane(hand[k & 1]);
    if (u < 0) break;
  }
}

// ---------------------------------------------------------------- forward, occupancy form
// The persistent forward's per-block arithmetic (lazy rescale, tree row sums, keep bits stored for
// the backward) in one workgroup per (batch, head) of NB compute waves and no producer: <= 128
// VGPRs and one K + V image (NB x 8 KB) per workgroup, so two workgroups share a CU (14 waves for
// NB = 7: 3-4 per SIMD instead of the persistent kernel's 2). The persistent kernel hides the K / V
// load behind the previous unit with a producer wave and a double buffer; here the other
// workgroup's compute covers it, and the extra waves per SIMD hide the softmax / hashing VALU
// latency (2 waves per SIMD issue at ~2.5 cycles per VALU instruction, 4 at ~1.2:
// tools/micro/issue_rate.hip).
template <int NB>
__global__ __launch_bounds__(64 * NB) __attribute__((amdgpu_waves_per_eu(4))) void attn_fwd_occ(
    const bf16* __restrict__ qkv, long ldq, bf16* __restrict__ out, long ldo, float* __restrict__ lse,
    uint32_t* __restrict__ mask, int N, int H, int dh, float sl2, uint32_t thr, float dscale, uint64_t seed) {
  constexpr int IMG = NB * 32 * 128;
  __shared__ __attribute__((aligned(1024))) char lds[2 * IMG];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int q = w * 32 + (lane & 31);
  seed = step_seed(seed);  // (its load and wait ahead of the DMA: a wait after it would cover the DMA)
  const u32x4 rs = rsrc4(qkv);
  img_dma_asm<NB>(lds, rs, (long)b * N, ldq, D + h * dh, N, dh, w, lane);
  img_dma_asm<NB>(lds + IMG, rs, (long)b * N, ldq, 2 * D + h * dh, N, dh, w, lane);
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv), ro = make_rsrc(out), rl = make_rsrc(lse),
                               rmk = make_rsrc(mask ? (const void*)mask : (const void*)lse);
  bf16x8 qf[4];
  {
    const int so = __builtin_amdgcn_readfirstlane((int)((((long)b * N) * ldq + h * dh) * 2));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d0 = 16 * s + 8 * hh;
      const uint32_t off = (((uint32_t)q * (uint32_t)ldq + (uint32_t)d0) * 2u) | ((uint32_t)(q >= N || d0 >= dh) << 31);
      qf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, off, so, 0));
    }
  }
  wait_vm<0>();  // this wave's K / V pieces and its Q rows
  asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]));
  bar_lds();  // every wave's pieces landed
  const char* Ki = lds;
  const char* Vi = lds + IMG;
  const uint32_t row = drop_row(bh, N, q);
  float m = -INFINITY, l = 0.f;
  f32x16 ot[2] = {f32x16{}, f32x16{}};
  // K row reads through one lane offset (chunk 2s + hh = chunk hh XOR 2s: rd_rowb), re-derived per key block
  // through an opaque copy: held as four loop-invariant offsets plus the mask-store offset, the 128-VGPR
  // budget of this form spilled them to scratch, and each block's reload waited (vmcnt(0)) for the previous
  // block's mask store
  const int krb = row_base(lane);
  bf16x8 kfr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) kfr[s] = rd_rowb(Ki, krb, s);
  // key block kb; TAIL: the last block with at most 8 real keys (TAIL4 below), where only accumulator
  // registers 0-3 (keys 0-7 of the block) can hold one: the softmax, hashing and keep-bit packing of
  // registers 4-15 are skipped (their P is 0, as the full form computes it from -inf scores). Same
  // results bit for bit, except the stored keep bits of padding keys: 0 here (no backward reads them).
  auto kblock = [&](int kb, auto tail) {
    constexpr bool TAIL = decltype(tail)::value;
    constexpr int NR = TAIL ? 4 : 16;  // live accumulator registers
    int kr = krb;
    asm volatile("" : "+v"(kr));
    // the tail's V offsets from a re-derived lane: from `lane` they were hoisted and spilled
    const int lv = TAIL ? (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) : lane;
    bf16x8 vfr[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < 2; ++db) vfr[s2][db] = rd_tr(Vi, kb * 32 + 16 * s2, db * 32, lv);
    f32x16 st = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) st = mfma32(kfr[s], qf[s], st);
    if (!TAIL && kb + 1 < NB) {
#pragma unroll
      for (int s = 0; s < 4; ++s) kfr[s] = rd_rowb(Ki + (kb + 1) * 4096, kr, s);
    }
    if (TAIL || (kb == NB - 1 && NB * 32 > N)) {  // only the last key block has padding keys
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (kb * 32 + acc_row(r, hh) >= N) st[r] = -INFINITY;
    }
    float bm = fmaxf(fmaxf(st[0], st[1]), st[2]);
#pragma unroll
    for (int r = 3; r < NR - 1; r += 2) bm = fmaxf(fmaxf(bm, st[r]), st[r + 1]);
    bm = fmaxf(bm, st[NR - 1]);
    bm = xhalf_max(bm) * sl2;
    if (__builtin_amdgcn_ballot_w64(bm > m + 8.f)) {  // lazy rescale (wave-uniform), as attn_fwd_pers
      const float mn = fmaxf(m, bm);
      const float al = ex2(m - mn);
      m = mn;
      l *= al;
      ot[0] *= al;
      ot[1] *= al;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = r < NR ? ex2(fmaf(st[r], sl2, -m)) : 0.f;
    if (TAIL) {
      l += (st[0] + st[1]) + (st[2] + st[3]);  // = the tree below with registers 4-15 at 0, bit for bit
    } else {
      float ls[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) ls[c] = (st[c] + st[c + 4]) + (st[c + 8] + st[c + 12]);
      l += (ls[0] + ls[1]) + (ls[2] + ls[3]);
    }
    if (thr) {
      const uint32_t rw = TAIL ? drop_row(bh, N, w * 32 + (lv & 31)) : row;  // (re-derived: as lv)
      const uint32_t p0 = (rw >> 1) + kb * 16 + 2 * hh;
      // the key's low word in a VGPR: with both key words in SGPRs the hash's counter step (pair ^ lo) + hi
      // cannot be one v_xad_u32 (one scalar operand per VOP3), and costs an xor and an add per hash
      uint32_t klo = (uint32_t)seed;
      asm volatile("" : "+v"(klo));
      // two rounds of 8 ballots (16 SGPRs live instead of 32: the 16-ballot form spilled at 128 VGPRs)
      uint32_t word = 0u;
#pragma unroll
      for (int half = 0; half < (TAIL ? 1 : 2); ++half) {
        uint64_t bal[8];
#pragma unroll
        for (int r = 0; r < 8; r += 2) {
          const int rr = 8 * half + r;
          if (rr >= NR) {
            bal[r] = bal[r + 1] = 0;
            continue;
          }
          uint32_t hlo;  // fer_hash's halves
          const uint32_t hx = fer_mix_pre(((p0 + (uint32_t)(acc_row(rr, 0) >> 1)) ^ klo) + (uint32_t)(seed >> 32), hlo);
          const bool k0 = hlo >= thr, k1 = (hx >> 16) >= thr;
          st[rr] = k0 ? st[rr] : 0.f;
          st[rr + 1] = k1 ? st[rr + 1] : 0.f;
          bal[r] = __builtin_amdgcn_ballot_w64(k0);
          bal[r + 1] = __builtin_amdgcn_ballot_w64(k1);
        }
        if (mask) word |= TAIL ? wl_keys4(0u, bal) : half ? wl_keys8<8>(0u, bal) : wl_keys8<0>(0u, bal);
      }
      if (mask) {
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));  // lane, re-derived
        const uint32_t mk_off = ln < 32 ? (uint32_t)(ln * 4) : FER_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(word, rmk, mk_off,
                                              __builtin_amdgcn_readfirstlane((int)((((long)bh * NB + kb) * NB + w) * 128)), 0);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = pack8(st, s2);
#pragma unroll
      for (int db = 0; db < 2; ++db) ot[db] = mfma32(vfr[s2][db], pf, ot[db]);
    }
  };
  const bool tail4 = NB * 32 - N >= 24;  // (ViT-B/16: N = 197, 5 keys in block 6)
#pragma unroll 1
  for (int kb = 0; kb < NB - (tail4 ? 1 : 0); ++kb) kblock(kb, std::false_type{});
  if (tail4) {
    int kbt = NB - 1;  // opaque: a constant block index let the compiler hoist the tail's LDS offsets
    asm volatile("" : "+s"(kbt));  // into the prologue, and they spilled across the loop
    kblock(kbt, std::true_type{});
  }
  l = xhalf_sum(l);
  const float mul = dscale / l;
  const int so = __builtin_amdgcn_readfirstlane((int)((((long)b * N) * ldo + h * dh) * 2));
  // 16-byte stores: lane half hh holds d = 8i + 4hh + {0..3} of its query row (i = 0..7); a permlane32
  // swap per dword pairs the halves so that each lane stores whole 16-byte chunks i + hh of chunk pairs
  // (i, i + 1) -- 4 dwordx4 stores per lane instead of 8 dwordx2 (the store tail is issue-bound)
  auto pack4 = [&](int i) {
    const f32x16& a = ot[i >> 2];
    const int g4 = i & 3;
    const bf16x4 v = {(bf16)(a[4 * g4] * mul), (bf16)(a[4 * g4 + 1] * mul), (bf16)(a[4 * g4 + 2] * mul),
                      (bf16)(a[4 * g4 + 3] * mul)};
    return __builtin_bit_cast(u32x2, v);
  };
  // lane terms re-derived here: computed in the prologue, the compiler kept them across the key loop (spilled)
  const int le = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int qe = w * 32 + (le & 31), he = le >> 5;
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const u32x2 pk[2] = {pack4(i), pack4(i + 1)};
    const auto x = __builtin_amdgcn_permlane32_swap(pk[0][0], pk[1][0], false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(pk[0][1], pk[1][1], false, false);
    // lanes 0-31: {own chunk i lo, partner's chunk i hi}; lanes 32-63: {partner's chunk i+1 lo, own hi}
    const u32x4 c = {x[0], y[0], x[1], y[1]};
    const int d = 8 * (i + he);
    const uint32_t off = (((uint32_t)qe * (uint32_t)ldo + (uint32_t)d) * 2u) | ((uint32_t)(qe >= N || d >= dh) << 31);
    __builtin_amdgcn_raw_buffer_store_b128(c, ro, off, so, 0);
  }
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((m + log2f(l)) * LN2), rl,
                                        (qe < N && he == 0) ? (uint32_t)(qe * 4) : FER_OOB,
                                        __builtin_amdgcn_readfirstlane(bh * N * 4), 0);
}

// ---------------------------------------------------------------- backward, fused
// One workgroup per (batch, head), NB waves, wave w owns key block w (K, V fragments in
// registers, dK / dV accumulators). At step i wave w visits query block qb = (w + i) % NB, so
// the NB waves always work on NB different query blocks:
//   S = Q K^T, dP = dO V^T (registers hold queries, lanes hold keys; once per block pair),
//   P, dS = P o (dropout'(dP) - Dq);  dV += P_drop^T dO;  dK += dS^T Q;
//   dQ: wave w also owns query block w's dQ^T accumulator in registers. After the step barrier
//   it adds K_src^T dS(w, src)^T from the dS tile (LDS, [key][query], double-buffered by step)
//   and K image of the wave src that visited block w in this step, both read by
//   ds_read_b64_tr_b16; the key blocks arrive in a fixed order (deterministic, no atomics).
// S, dP, P and the dropout mask are computed once per (query block, key block) instead of once
// in each of the dQ and dK/dV orientations of the two-kernel path.
// LDS (NB = 7): Q + dO images 2 x 28 KB, K images 28 KB, dS tiles 2 x 14 KB, lse / Dq 1.75 KB =
// 113.75 KB (NB = 8, N <= 256: 130 KB); 256 VGPRs -> one workgroup per CU.
template <int NB>
constexpr int fused_lds_bytes() {
  return 3 * NB * 32 * 128 + 2 * NB * 2048 + 2 * NB * 32 * 4;
}

// [32][32] bf16 tile with 64-byte rows (keys x queries): B operand of the 32x32x16 MFMA with
// lanes = columns (queries) and k = rows rbase + {0..3, 8..11} + 4*(lane>>5) (same k order as
// rd_tr and the accumulator registers). Four consecutive 64-byte rows per 32-lane half: no
// bank conflicts without a swizzle.
// dS tile [32 keys][32 queries] bf16, 64-byte rows: 8-byte piece c of row r at piece c ^ ((r >> 1) & 7).
// The writer's ds_write_b64 lane groups (16 consecutive rows, one piece) then cover 16 distinct bank
// pairs (unswizzled: 8-way conflict, every row on banks {0,16} mod 32); the transposed reads (rows
// R..R+3, all 8 pieces per 32-lane group) stay conflict-free.
FER_DEV int ds_off(int r, int c8) { return r * 64 + ((c8 ^ ((r >> 1) & 7)) << 3); }
FER_DEV bf16x8 rd_tr64(const char* img, int rbase, int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int R = rbase + 4 * (gg >> 1);
  const int c8 = 4 * (gg & 1) + p;
  const char* a1 = img + ds_off(R + q, c8);
  const char* a2 = img + ds_off(R + 8 + q, c8);
  short4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a1);
  short4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a2);
  return cat8(t1, t2);
}

// Lane offsets of the LDS reads above, computed once per step instead of per read. The swizzles
// depend on row bits 1-3 only, so a read at row base R (a multiple of 16) is the R = 0 offset + the
// row term; rd_tr's second 32-column half (cb = 32) flips chunk bit 2 of a chunk index below 4,
// i.e. byte bit 6 (XOR 64); rd_row's chunk 2s + hh is the s = 0 chunk XOR 2s (byte XOR 32s).
struct TrB {
  int a1, a2;  // rd_tr(img, 0, 0) byte offsets of the two row groups (cb = 32: XOR 64)
};
FER_DEV TrB tr_base(int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int R = 4 * (gg >> 1);
  const int c = (16 * (gg & 1) + 4 * p) >> 3, half = (p & 1) * 8;
  const int r1 = R + q, r2 = R + 8 + q;
  TrB b;
  b.a1 = r1 * 128 + ((c ^ swz(r1)) << 4) + half;
  b.a2 = r2 * 128 + ((c ^ swz(r2)) << 4) + half;
  return b;
}
// == rd_tr(img, R, 32 * hi, lane) for img + R * 128 passed as `img`
FER_DEV bf16x8 rd_trb(const char* img, const TrB& b, bool hi) {
  short4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(img + (hi ? (b.a1 ^ 64) : b.a1)));
  short4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(img + (hi ? (b.a2 ^ 64) : b.a2)));
  return cat8(t1, t2);
}
// == rd_tr64(img, R, lane) for img + R * 64 passed as `img`
FER_DEV int2 tr64_base(int lane) {
  const int gg = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int R = 4 * (gg >> 1), c8 = 4 * (gg & 1) + p;
  return int2{ds_off(R + q, c8), ds_off(R + 8 + q, c8)};
}
// attn_bwd_pers' per-lane offset table entry: {row_base | tr_base.a1 << 16, tr_base.a2 | dS-write base
// ds_off(lane & 31, lane >> 5) << 16, tr64_base.x | .y << 16, 0} (every offset < 4096)
FER_DEV u32x4 lane_table(int lane) {
  const TrB b = tr_base(lane);
  const int2 t = tr64_base(lane);
  return u32x4{(uint32_t)row_base(lane) | ((uint32_t)b.a1 << 16), (uint32_t)b.a2 | ((uint32_t)ds_off(lane & 31, lane >> 5) << 16),
               (uint32_t)t.x | ((uint32_t)t.y << 16), 0u};
}
FER_DEV bf16x8 rd_tr64b(const char* img, int2 b) {
  short4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(img + b.x));
  short4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(img + b.y));
  return cat8(t1, t2);
}

// dQacc: [NB*32 queries][64 d] fp32, 16-byte chunk index XOR (row & 15)
FER_DEV int dq_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

template <int NB>
__global__ __launch_bounds__(64 * NB) void attn_bwd_fused_bf16(const bf16* __restrict__ qkv, long ldq,
                                                               const bf16* __restrict__ out, long ldo,
                                                               const bf16* __restrict__ dout, long lddo,
                                                               const float* __restrict__ lse,
                                                               bf16* __restrict__ dqkv, long lddq, int N, int H,
                                                               int dh, float scale, float sl2, uint32_t thr,
                                                               float dscale, uint64_t seed, float* __restrict__ cs_part) {
  seed = step_seed(seed);
  constexpr int IMG = NB * 32 * 128;
  __shared__ __attribute__((aligned(1024))) char lds[fused_lds_bytes<NB>()];
  char* Qi = lds;
  char* Oi = lds + IMG;                       // dO image
  char* Kimg = lds + 2 * IMG;                 // NB x [32 keys][64 d] images
  char* Sall = lds + 3 * IMG;                 // 2 x NB x [32 keys][32 queries] bf16 dS tiles
  char* dqa = lds;                            // after the steps: dQ rows, fp32, over the Q / dO images
  float* lse_s = (float*)(Sall + 2 * NB * 2048);
  float* dd_s = lse_s + NB * 32;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  img_dma<NB>(Qi, make_rsrc(qkv), (long)b * N, ldq, h * dh, N, dh, w, lane);
  img_dma<NB>(Oi, make_rsrc(dout), (long)b * N, lddo, h * dh, N, dh, w, lane);
  // Dq = rowsum(dO o O): two threads per query row
  for (int t = threadIdx.x; t < NB * 64; t += 64 * NB) {
    const int qr = t >> 1, half = t & 1;
    float dsum = 0.f;
    if (qr < N) {
      const bf16* po = out + ((long)b * N + qr) * ldo + h * dh;
      const bf16* pd = dout + ((long)b * N + qr) * lddo + h * dh;
      for (int d = half * 8; d < dh; d += 16) {
        const bf16x8 a = *(const bf16x8*)(po + d), c = *(const bf16x8*)(pd + d);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)a[j] * (float)c[j];
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    if (!half) {
      dd_s[qr] = dsum;
      lse_s[qr] = qr < N ? lse[(long)bh * N + qr] * LOG2E : INFINITY;
    }
  }
  const int key = w * 32 + (lane & 31);
  const bool kval = key < N;
  bf16x8 kf[4], vf[4];
  char* Ki = Kimg + w * 4096;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int d0 = 16 * s + 8 * hh;
    const bool ok = kval && d0 < dh;
    kf[s] = ok ? *(const bf16x8*)(qkv + ((long)b * N + key) * ldq + D + h * dh + d0) : bf16x8{};
    vf[s] = ok ? *(const bf16x8*)(qkv + ((long)b * N + key) * ldq + 2 * D + h * dh + d0) : bf16x8{};
    // this wave's K block as an LDS image (A operand of dQ^T = K^T dS^T, transposed reads)
    *(bf16x8*)(Ki + img_off(lane & 31, 2 * s + hh)) = kf[s];
  }
  __syncthreads();  // images (DMA: vmcnt(0) + barrier), dQacc zero, lse / Dq visible

  const int NP = N + (N & 1);
  const bool odd = lane & 1;
  f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
  f32x16 dq[2] = {f32x16{}, f32x16{}};  // dQ^T of query block w (this wave owns it), registers
  const int nsteps = NB;
#pragma unroll 1
  for (int i = 0; i < nsteps; ++i) {
    int qb = w + i;
    if (qb >= NB) qb -= NB;
    char* Si = Sall + (i & 1) * NB * 2048 + w * 2048;
    f32x16 st = {}, dp = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      st = mfma32(rd_row(Qi, qb * 32 + (lane & 31), 2 * s + hh), kf[s], st);
      dp = mfma32(rd_row(Oi, qb * 32 + (lane & 31), 2 * s + hh), vf[s], dp);
    }
    uint32_t keep = 0xFFFFu;
    if (thr) {
      // this lane hashes rows [8*odd, 8*odd + 8) for the key pair (key & ~1, key | 1)
      uint32_t hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qr = qb * 32 + acc_row(8 * odd + j, hh);
        hv[j] = fer_hash(seed, (((uint32_t)bh * N + qr) * (uint32_t)NP + (uint32_t)(key & ~1)) >> 1);
      }
      keep = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t other = (uint32_t)__shfl_xor((int)hv[j], 1, 64);
        const uint32_t h_lo = odd ? other : hv[j];  // rows j (even lane's own)
        const uint32_t h_hi = odd ? hv[j] : other;  // rows 8 + j
        const uint32_t u_lo = odd ? (h_lo >> 16) : (h_lo & 0xFFFFu);
        const uint32_t u_hi = odd ? (h_hi >> 16) : (h_hi & 0xFFFFu);
        keep |= (uint32_t)(u_lo >= thr) << j;
        keep |= (uint32_t)(u_hi >= thr) << (8 + j);
      }
    }
    // lse / Dq of the 16 query rows of this lane: 4 groups of 4 consecutive rows (one b128 each)
    f32x4 lq4[4], dq4[4];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      lq4[g4] = *(const f32x4*)(lse_s + qb * 32 + 8 * g4 + 4 * hh);
      dq4[g4] = *(const f32x4*)(dd_s + qb * 32 + 8 * g4 + 4 * hh);
    }
    f32x16 pd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = ex2(fmaf(st[r], sl2, -lq4[r >> 2][r & 3]));
      p = kval ? p : 0.f;
      const bool kp = (keep >> r) & 1;
      const float g = thr ? (kp ? dp[r] * dscale : 0.f) : dp[r];
      pd[r] = thr ? (kp ? p * dscale : 0.f) : p;
      st[r] = p * (g - dq4[r >> 2][r & 3]);  // dS
    }
    // dS tile -> LDS as [key][query] (bf16), read back below as the B operand of dQ^T
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
      *(bf16x4*)(Si + ds_off(lane & 31, 2 * g4 + hh)) =
          bf16x4{(bf16)st[4 * g4], (bf16)st[4 * g4 + 1], (bf16)st[4 * g4 + 2], (bf16)st[4 * g4 + 3]};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = pack8(pd, s2), df = pack8(st, s2);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dv[db] = mfma32(pf, rd_tr(Oi, qb * 32 + 16 * s2, db * 32, lane), dv[db]);
        dk[db] = mfma32(df, rd_tr(Qi, qb * 32 + 16 * s2, db * 32, lane), dk[db]);
      }
    }
    // step barrier: every wave's dS tile of this step is in Sall[i & 1] (double-buffered: the
    // tiles of step i-1 may still be read by slow owners until they pass this barrier)
    __syncthreads();
    // dQ^T(w) += K_src^T dS(w, src)^T from the wave src that visited query block w this step;
    // the key blocks arrive in a fixed order (w, w-1, ...): deterministic, no atomics
    {
      int src = w - i;
      if (src < 0) src += NB;
      const char* So = Sall + (i & 1) * NB * 2048 + src * 2048;
      const char* Ko = Kimg + src * 4096;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 sf = rd_tr64(So, 16 * s2, lane);
#pragma unroll
        for (int db = 0; db < 2; ++db) dq[db] = mfma32(rd_tr(Ko, 16 * s2, db * 32, lane), sf, dq[db]);
      }
    }
  }
  __syncthreads();  // Q / dO images no longer read: they take the dQ rows
  {
    const int qrow = w * 32 + (lane & 31);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *(f32x4*)(dqa + dq_off(qrow, 8 * db + 2 * g4 + hh)) =
            f32x4{dq[db][4 * g4], dq[db][4 * g4 + 1], dq[db][4 * g4 + 2], dq[db][4 * g4 + 3]};
  }
  __syncthreads();
  // dQ: 16-byte row pieces, scaled
  for (int t = threadIdx.x; t < NB * 32 * 8; t += 64 * NB) {
    const int qr = t >> 3, c8 = t & 7;  // 8 d per piece
    if (qr < N && c8 * 8 < dh) {
      const f32x4 lo = *(const f32x4*)(dqa + dq_off(qr, 2 * c8)), hi = *(const f32x4*)(dqa + dq_off(qr, 2 * c8 + 1));
      *(bf16x8*)(dqkv + ((long)b * N + qr) * lddq + h * dh + c8 * 8) =
          bf16x8{(bf16)(lo[0] * scale), (bf16)(lo[1] * scale), (bf16)(lo[2] * scale), (bf16)(lo[3] * scale),
                 (bf16)(hi[0] * scale), (bf16)(hi[1] * scale), (bf16)(hi[2] * scale), (bf16)(hi[3] * scale)};
    }
  }
  if (cs_part) {
    // in_proj.bias gradient partials of batch b: column sums of dq (from dQacc), dk, dv (from
    // the accumulators) over this head's rows, in a fixed order. Scratch: the K-image area.
    float* red = (float*)Kimg;  // [NB][3][64]
    {  // dQ: wave w sums rows w, w+NB, ... of column d = lane
      float t = 0.f;
      for (int r = w; r < NB * 32; r += NB) t += ((const float*)(dqa + dq_off(r, lane >> 2)))[lane & 3];
      red[w * 192 + lane] = t * scale;
    }
#pragma unroll
    for (int db = 0; db < 2; ++db) {  // dK / dV: 16 key rows per lane, + the other half-wave
      float tk = 0.f, tv = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        tk += dk[db][r];
        tv += dv[db][r];
      }
      tk = xhalf_sum(tk);
      tv = xhalf_sum(tv);
      if (hh == 0) {
        red[w * 192 + 64 + db * 32 + lane] = tk * scale;
        red[w * 192 + 128 + db * 32 + lane] = tv;
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 192; c += 64 * NB) {
      float t = 0.f;
      for (int j = 0; j < NB; ++j) t += red[j * 192 + c];
      const int mat = c >> 6, d = c & 63;
      if (d < dh) cs_part[(long)b * 3 * D + mat * D + h * dh + d] = t;
    }
  }
  // dK / dV: stage each wave's 32 x 64 tiles through LDS (reusing the image area) for 16-byte
  // row stores. dk/dv[db][r]: key row = w*32 + acc_row(r, hh), d = db*32 + (lane&31).
  __syncthreads();  // the dQ rows (same area) have been read
  bf16* stg = (bf16*)(lds + w * 8192);  // [2][32][64], inside the (now unused) Q / dO images
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = acc_row(r, hh), d = db * 32 + (lane & 31);
      stg[kr * 64 + d] = (bf16)(dk[db][r] * scale);
      stg[2048 + kr * 64 + d] = (bf16)dv[db][r];
    }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int t = i * 64 + lane;  // 512 chunks of 16 B: [2 mats][32 rows][8 chunks]
    const int mat = t >> 8, kr = (t >> 3) & 31, c = t & 7;
    const int gk = w * 32 + kr;
    if (gk < N && c * 8 < dh)
      *(bf16x8*)(dqkv + ((long)b * N + gk) * lddq + (1 + mat) * D + h * dh + c * 8) =
          *(const bf16x8*)(stg + mat * 2048 + kr * 64 + c * 8);
  }
}

// ---------------------------------------------------------------- backward, persistent
// attn_bwd_fused_bf16's block-pair schedule (wave w = key block w and owner of query block w's
// dQ; at step i it visits query block (w + i) % NB) in a persistent workgroup per CU that walks
// the (batch, head) units. While the waves work on unit u, each wave also prepares ITS 32 rows of
// unit u+1 in the other half of a double buffer, by LDS-DMA only: at step 0 the next dO rows, the
// next O rows (into the Q slot) and lse; a few steps later (the DMA has landed) Dq = rowsum(dO o O)
// of those rows from the images, then the next Q rows over the consumed O rows. In the last step
// the K / V fragments (registers) are reloaded with the next unit's right after their last use.
// So nothing at a unit boundary waits on HBM latency.
// Dropout keep bits come from the forward's mask (attn_fwd_pers): one coalesced 128-byte row per
// (key block, query block) tile. The row's lse enters as the initial accumulator of S
// (st = S - lse/scale, p = 2^(st * scale * log2e)), so no register holds it.
// dS tiles are single-buffered (LDS budget), so a step has two barriers: dS written | dQ read.
// Epilogue (one barrier): dQ^T accumulators stored straight from registers (4 consecutive d per
// lane = 8-byte pieces), dK / dV staged through the unit's (now free) Q/dO half for 16-byte row
// stores; in_proj bias-gradient partials per (batch, wave) go straight to `cs_part`
// ([B][NB][3*D], reduced by part_reduce): dK / dV column sums from the accumulators,
// colsum(dQ) = K_w^T cs_w with cs_w[k] = sum_q dS[q][k] accumulated over the steps (two MFMAs per
// 32-column block instead of a cross-lane reduction of the transposed dQ accumulators).
// LDS (NB = 7): Q/dO images 2 x 56 KB, K images 28 KB, dS tiles 14 KB, lse/Dq 2 x 1.75 KB,
// cs 0.9 KB = 158.4 KB.
// From 6 key blocks up an extra (NB+1)-th wave prepares the next unit for every compute wave (LDS-DMA of
// its dO / O rows and lse, Dq, the Q rows): it lands on the one SIMD that holds a single compute wave
// (a workgroup's waves k and k+4 share a SIMD), so that work leaves the SIMDs of the critical waves.
template <int NB> constexpr bool bwd_helper() { return NB >= 6; }
template <int NB> constexpr int bwd_threads() { return 64 * (NB + (bwd_helper<NB>() ? 1 : 0)); }

template <int NB>
constexpr int pers_bwd_lds_bytes() {
  return 5 * NB * 4096 + NB * 2048 + 2 * 2 * NB * 32 * 4 + NB * 32 * 4;
}

template <int NB>
__global__ __launch_bounds__(bwd_threads<NB>()) void attn_bwd_pers(
    const bf16* __restrict__ qkv, long ldq, const bf16* __restrict__ out, long ldo, const bf16* __restrict__ dout,
    long lddo, const float* __restrict__ lse, const uint32_t* __restrict__ mask, bf16* __restrict__ dqkv, long lddq,
    int BH, int N, int H, int dh, float scale, float sl2, float dscale, float* __restrict__ cs_part, WqArgs wq) {
  constexpr int IMG = NB * 32 * 128;
  constexpr int PREP = NB >= 4 ? 3 : NB - 1;  // step whose dQ phase computes the next unit's Dq
  __shared__ __attribute__((aligned(1024))) char lds[pers_bwd_lds_bytes<NB>() + 16 + 1024];
  lds_vint* hand = FER_LDS_INT(lds + pers_bwd_lds_bytes<NB>());  // unit hand-off (work queue)
  // per-lane LDS offsets of the step's fragment reads and dS writes, 16-bit packed (lane_table):
  // one ds_read_b128 per step phase instead of ~40 VALU re-deriving them from the lane id
  const char* ltab = lds + pers_bwd_lds_bytes<NB>() + 16;
  char* Kimg = lds + 4 * IMG;               // NB x [32 keys][64 d] images
  char* Sall = lds + 5 * IMG;               // NB x [32 keys][32 queries] bf16 dS tiles
  float* lsd = (float*)(Sall + NB * 2048);  // 2 x {L[NB*32] = -lse/scale, -Dq[NB*32]}
  float* csl = lsd + 4 * NB * 32;           // NB x 32: sum_q dS[q][k] of each wave's keys
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int D = H * dh;
  const int key = w * 32 + (lane & 31);
  const float inv_scale = 1.f / scale;

  // this wave's 32 rows of `unit`: dO, O (-> Q slot) images and raw lse, by DMA (no wait)
  auto prep_issue = [&](int unit, int hb) {
    const int b = unit / H, h = unit - b * H;
    char* Qi = lds + hb * 2 * IMG;
    img_dma_asm<NB>(Qi + IMG, rsrc4(dout), (long)b * N, lddo, h * dh, N, dh, w, lane);
    img_dma_asm<NB>(Qi, rsrc4(out), (long)b * N, ldo, h * dh, N, dh, w, lane);
    int ln = threadIdx.x & 63;  // recomputed here (laundered): a kept offset was spilled, and the scratch
    asm volatile("" : "+v"(ln));  // reload's vmcnt(0) then waited for the previous unit's epilogue stores
    const int r = w * 32 + ln;  // lanes 32..63 would land in the next wave's words: masked off
    if (ln < 32) dma4_asm(lsd + hb * 2 * NB * 32 + w * 32, rsrc4(lse + (long)unit * N), r < N ? r * 4 : FER_OOB);
  };
  // after the DMA landed: L and Dq of this wave's rows, then its Q rows over the consumed O rows
  auto prep_finish = [&](int unit, int hb) {
    const int b = unit / H, h = unit - b * H;
    char* Qi = lds + hb * 2 * IMG;
    float* L = lsd + hb * 2 * NB * 32;
    wait_vm<0>();
    const int r = w * 32 + (lane >> 1), half = lane & 1;  // two lanes per row, 4 chunks each
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 o = rd_row(Qi, r, 4 * half + c), g = rd_row(Qi + IMG, r, 4 * half + c);
#pragma unroll
      for (int e = 0; e < 8; e += 2)  // v_dot2c_f32_bf16: one instruction per element pair (no unpacking)
        a = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{o[e], o[e + 1]}, bf16x2{g[e], g[e + 1]}, a, false);
    }
    a += __shfl_xor(a, 1, 64);
    if (!half) {
      L[NB * 32 + r] = -a;  // -Dq: the step's dS = P o (dP' - Dq) adds it as is
      L[r] = r < N ? -L[r] * inv_scale : -INFINITY;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // O rows read: Q may land on them
    img_dma_asm<NB>(Qi, rsrc4(qkv), (long)b * N, ldq, h * dh, N, dh, w, lane);
  };
  // K (col0 = D) / V (2D) row fragments and keep words by buffer loads, out-of-range lanes through the
  // range check (FER_OOB): no per-lane branches, so the compiler's wait counts stay exact (with
  // exec-masked loads it fell back to vmcnt(0) and the last step waited for the next unit's loads)
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv);
  const __amdgpu_buffer_rsrc_t rmk = make_rsrc(mask ? (const void*)mask : (const void*)qkv);
  // per-lane byte offsets (computed once; the unit / column part goes into the scalar offset)
  uint32_t kv_off[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int d0 = 16 * s + 8 * hh;
    kv_off[s] = (key < N && d0 < dh) ? (uint32_t)(((long)key * ldq + d0) * 2) : FER_OOB;
  }
  const uint32_t mk_off = mask ? (uint32_t)((lane & 31) * 4) : FER_OOB;
  auto load_frag = [&](bf16x8 (&vq)[4], int unit, int col0) {
    const int b = unit / H, h = unit - b * H;
    const int so = __builtin_amdgcn_readfirstlane((int)((((long)b * N) * ldq + col0 + h * dh) * 2));
#pragma unroll
    for (int s = 0; s < 4; ++s)
      vq[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, kv_off[s], so, 0));
  };
  auto write_kimg = [&](const bf16x8 (&kq)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) *(bf16x8*)(Kimg + w * 4096 + img_off(lane & 31, 2 * s + hh)) = kq[s];
  };
  auto mask_word = [&](int unit, int i) -> uint32_t {  // keep word of (key block w, query block (w+i)%NB)
    int qb = w + i;
    if (qb >= NB) qb -= NB;
    const int so = __builtin_amdgcn_readfirstlane((int)((((long)unit * NB + w) * NB + qb) * 128));
    return __builtin_amdgcn_raw_buffer_load_b32(rmk, mk_off, so, 0);  // (p = 0: 0, read as all-keep below)
  };

  // units: fixed stride, or the work queue `wq` (common.h): the first unit is blockIdx.x, the next
  // one is claimed at the start (overlapping the first unit's loads), then thread 0 claims the
  // unit after next in each unit's epilogue and hands it on through hand[k & 1]
  int u, un = -1;
  if (wq.q) {
    u = wq_first(BH);
    if (u < 0) return;
  } else {
    u = blockIdx.x;
    un = u + (int)gridDim.x < BH ? u + (int)gridDim.x : -1;
  }
  constexpr bool HELPER = bwd_helper<NB>();
  if (HELPER && w == NB) {
    // The helper wave: same barriers as the compute waves (prologue, two per step, one per unit), its
    // own work in the first phase of steps 0-5 of every unit that has a next one (buffer cur ^ 1,
    // free since the previous unit's last barrier): dO rows + lse | O rows | wait, Dq of rows 0-111 |
    // Dq of rows 112-223 | Q rows of waves 0-3 over the O rows | Q rows of waves 4..NB-1.
    bar_lds();
    if (wq.q) un = __builtin_amdgcn_readfirstlane(hand[2]);
#pragma unroll 1
    for (int k = 0;; ++k) {
      const int cur = k & 1, hb = cur ^ 1;
      const bool has_next = un >= 0;
#pragma unroll 1
      for (int i = 0; i < NB; ++i) {
        if (has_next && i < 6) {
          const int b = un / H, h = un - b * H;
          char* Qi = lds + hb * 2 * IMG;
          float* L = lsd + hb * 2 * NB * 32;
          if (i == 0) {
#pragma unroll 1
            for (int ww = 0; ww < NB; ++ww) {
              img_dma_asm<NB>(Qi + IMG, rsrc4(dout), (long)b * N, lddo, h * dh, N, dh, ww, lane);
              int ln = threadIdx.x & 63;
              asm volatile("" : "+v"(ln));
              const int r = ww * 32 + ln;
              if (ln < 32) dma4_asm(L + ww * 32, rsrc4(lse + (long)un * N), r < N ? r * 4 : FER_OOB);
            }
          } else if (i == 1) {
#pragma unroll 1
            for (int ww = 0; ww < NB; ++ww) img_dma_asm<NB>(Qi, rsrc4(out), (long)b * N, ldo, h * dh, N, dh, ww, lane);
          } else if (i == 2 || i == 3) {
            if (i == 2) wait_vm<0>();
#pragma unroll 1
            for (int p = (i == 2 ? 0 : NB / 2); p < (i == 2 ? NB / 2 : NB); ++p) {
              const int r = p * 32 + (lane >> 1), half = lane & 1;  // two lanes per row, 4 chunks each
              float a = 0.f;
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                const bf16x8 o = rd_row(Qi, r, 4 * half + c), g = rd_row(Qi + IMG, r, 4 * half + c);
#pragma unroll
                for (int e = 0; e < 8; e += 2)
                  a = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{o[e], o[e + 1]}, bf16x2{g[e], g[e + 1]}, a, false);
              }
              a += __shfl_xor(a, 1, 64);
              if (!half) {
                L[NB * 32 + r] = -a;
                L[r] = r < N ? -L[r] * inv_scale : -INFINITY;
              }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // O rows read: Q may land on them
          } else {
#pragma unroll 1
            for (int ww = (i == 4 ? 0 : 4); ww < (i == 4 ? 4 : NB); ++ww)
              img_dma_asm<NB>(Qi, rsrc4(qkv), (long)b * N, ldq, h * dh, N, dh, ww, lane);
          }
        }
        bar_lds();  // dS tiles written
        bar_lds();  // dS tiles and K images read
      }
      if (has_next) wait_vm<0>();  // the next unit's rows landed before the unit barrier
      bar_lds();
      u = un;
      un = __builtin_amdgcn_readfirstlane(hand[cur]);
      if (u < 0) break;
    }
    return;
  }
  bf16x8 kf[4], vf[4];
  prep_issue(u, 0);
  load_frag(kf, u, D);
  load_frag(vf, u, 2 * D);
  uint32_t mwn = mask_word(u, 0);
  int c0 = -1;
  if (wq.q && threadIdx.x == 0) c0 = wq_claim(wq.q, wq.base, BH);  // overlaps the loads' wait
  prep_finish(u, 0);
  write_kimg(kf);
  wait_vm<0>();
  mwn = mask ? mwn : 0xFFFFFFFFu;
  asm volatile("" : "+v"(mwn));  // resolved after the wait: the first step's use waits for nothing
  if (wq.q && threadIdx.x == 0) hand[2] = c0;
  if (w == 0) *(u32x4*)(lds + pers_bwd_lds_bytes<NB>() + 16 + lane * 16) = lane_table(lane);
  bar_lds();
  if (wq.q) un = __builtin_amdgcn_readfirstlane(hand[2]);

#pragma unroll 1
  for (int k = 0;; ++k) {
    const int cur = k & 1;
    const bool has_next = un >= 0;
    int unn = -1;  // the unit after next (work queue: claimed by thread 0 in the epilogue below)
    if (!wq.q && has_next && un + (int)gridDim.x < BH) unn = un + gridDim.x;
    const char* Qi = lds + cur * 2 * IMG;
    const char* Oi = Qi + IMG;
    const float* L = lsd + cur * 2 * NB * 32;
    const float* Dq = L + NB * 32;
    f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
    f32x16 dq[2] = {f32x16{}, f32x16{}};  // dQ^T of query block w
    float cs = 0.f;                       // sum over this lane's query rows of dS[q][key]
    uint32_t mw0 = 0;                     // keep word of the next unit's first step
    uint32_t claim_raw = 0;               // work queue: the claim issued in the last step
    // one step; the last is a separate instantiation (LAST) so that its extra work -- reloading
    // kf / vf with the next unit's fragments, the bias-gradient sums -- does not turn every
    // register it touches into a loop-carried copy
#ifdef FER_ATTN_STAMPS
    const bool bst_on = blockIdx.x == 0 && (k == 2 || k == 3);
    const int sb = (k - 2) * 64;
#endif
    BST(sb + 0);
    // FIRST / LAST: the first step (its keep word resolved before the unit, so its use waits for no
    // memory op -- in the loop it would wait for the previous unit's epilogue stores) and the last one
    // (reloads kf / vf, bias-gradient sums) are separate instantiations
    auto step = [&](int i, auto last_tag, auto first_tag) {
      constexpr bool LAST = decltype(last_tag)::value;
      constexpr bool FIRST = decltype(first_tag)::value;
      BST(sb + 1 + 7 * i);
      {
        int lane = threadIdx.x & 63;  // laundered per step: lane-derived LDS addresses are not
        asm volatile("" : "+v"(lane));  // hoisted out of the step loop (they would pin ~40 VGPRs)
        const int hh = lane >> 5;
        // the keep word (loaded at the end of the previous step) is taken before any DMA of this step is
        // issued: the DMA is inline asm, invisible to the compiler's wait counts, so its vmcnt(0) for
        // the word would otherwise wait for the DMA as well
        // bit acc_row(r, 0) = keep of query row r
        uint32_t mws = (FIRST ? mwn : (mask ? mwn : 0xFFFFFFFFu)) >> (4 * hh);
        // pinned here: left to the compiler, the select sank below the LAST step's loads of the next
        // unit (and its exec-masked claim atomic) and waited vmcnt(0) for all of them (~4k cycles/unit)
        asm volatile("" : "+v"(mws)::"memory");
        if (!HELPER && i == 0 && has_next) prep_issue(un, cur ^ 1);
        // the next step's keep word, a whole step ahead of its use (issued in the dQ phase, its latency
        // was exposed at the next step's start: ~500 cycles per step); after this step's DMA, so the
        // next step's wait covers nothing issued later
        if (i + 1 < NB) mwn = mask_word(u, i + 1);
        int qb = w + i;
        if (qb >= NB) qb -= NB;
        const u32x4 lt = *(const u32x4*)(ltab + lane * 16);
        const TrB tb{(int)(lt[0] >> 16), (int)(lt[1] & 0xFFFFu)};
        const int rb = (int)(lt[0] & 0xFFFFu), dsb = (int)(lt[1] >> 16);
        const char* Qq = Qi + qb * 4096;
        const char* Oq = Oi + qb * 4096;
        f32x16 st, dp = {};
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {  // S starts at -lse/scale of its 16 query rows
          const f32x4 l4 = *(const f32x4*)(L + qb * 32 + 8 * g4 + 4 * hh);
          st[4 * g4] = l4[0];
          st[4 * g4 + 1] = l4[1];
          st[4 * g4 + 2] = l4[2];
          st[4 * g4 + 3] = l4[3];
        }
        // LDS operands of each phase grouped ahead of its MFMAs (one exposed LDS latency per phase
        // instead of one per MFMA)
        bf16x8 qr[4], orr[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          qr[s] = rd_rowb(Qq, rb, s);
          orr[s] = rd_rowb(Oq, rb, s);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(qr[s], kf[s], st);
          dp = mfma32(orr[s], vf[s], dp);
        }
        if (LAST && has_next) {  // kf / vf are dead from here on: the next unit's go straight in
          load_frag(kf, un, D);
          load_frag(vf, un, 2 * D);
          mw0 = mask_word(un, 0);
          // the claim of the unit after next: its round trip overlaps the rest of this step (the
          // result is read in the epilogue, after its wait)
          if (wq.q && threadIdx.x == 0) claim_raw = wq_claim_issue(wq.q);
        }
        if (LAST) BST(sb + 54);
        f32x16 pd;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 d4 = *(const f32x4*)(Dq + qb * 32 + 8 * g4 + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g4 + j;
            const float p = ex2(st[r] * sl2);
            // keep bit as an all-ones / zero mask (one v_bfe_i32): AND selects p / dp or +0.0,
            // bit-identical to kp ? x : 0.f without a compare and two selects per element
            const uint32_t km = (uint32_t)((int32_t)(mws << (31 - acc_row(r, 0))) >> 31);
            pd[r] = __uint_as_float(__float_as_uint(p) & km);
            st[r] = p * fmaf(__uint_as_float(__float_as_uint(dp[r]) & km), dscale, d4[j]);  // dS (d4 = -Dq)
            cs += st[r];
          }
        }
        BST(sb + 6 + 7 * i);
        char* Si = Sall + w * 2048;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)  // ds_off(lane & 31, 2 * g4 + hh) = dsb ^ (g4 << 4)
          *(bf16x4*)(Si + (dsb ^ (g4 << 4))) =
              bf16x4{(bf16)st[4 * g4], (bf16)st[4 * g4 + 1], (bf16)st[4 * g4 + 2], (bf16)st[4 * g4 + 3]};
        bf16x8 ot_[2][2], qt_[2][2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            ot_[s2][db] = rd_trb(Oq + s2 * 2048, tb, db);
            qt_[s2][db] = rd_trb(Qq + s2 * 2048, tb, db);
          }
        BST(sb + 7 + 7 * i);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pf = pack8(pd, s2), df = pack8(st, s2);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dv[db] = mfma32(pf, ot_[s2][db], dv[db]);
            dk[db] = mfma32(df, qt_[s2][db], dk[db]);
          }
        }
        if (LAST && cs_part) {  // this wave's keys: sum over all queries of dS
          cs = xhalf_sum(cs);
          if (hh == 0) csl[w * 32 + lane] = cs;
        }
      }
      BST(sb + 2 + 7 * i);
      bar_lds();  // every dS tile of this step is in Sall
      BST(sb + 3 + 7 * i);
      {
        int lane = threadIdx.x & 63;
        asm volatile("" : "+v"(lane));
        const int hh = lane >> 5;
        int src = w - i;
        if (src < 0) src += NB;
        const char* So = Sall + src * 2048;
        const char* Ko = Kimg + src * 4096;
        const u32x4 lt = *(const u32x4*)(ltab + lane * 16);
        const TrB tb{(int)(lt[0] >> 16), (int)(lt[1] & 0xFFFFu)};
        const int2 t64{(int)(lt[2] & 0xFFFFu), (int)(lt[2] >> 16)};
        bf16x8 sf[2], kt[2][2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          sf[s2] = rd_tr64b(So + s2 * 1024, t64);
#pragma unroll
          for (int db = 0; db < 2; ++db) kt[s2][db] = rd_trb(Ko + s2 * 2048, tb, db);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int db = 0; db < 2; ++db) dq[db] = mfma32(kt[s2][db], sf[s2], dq[db]);
        if (!HELPER && i == PREP && has_next) prep_finish(un, cur ^ 1);
        if (LAST && cs_part) {
          // colsum(dQ)[d] over this unit = sum_w K_w^T cs_w: B operand = cs of the wave's keys (k)
          // in every column (wave-private LDS read-back), A = K_w^T from its image.
          const int b = u / H, h = u - b * H;
          const char* Kw = Kimg + w * 4096;
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            f32x16 acc = {};
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const f32x4 c0 = *(const f32x4*)(csl + w * 32 + 16 * s2 + 4 * hh);
              const f32x4 c1 = *(const f32x4*)(csl + w * 32 + 16 * s2 + 8 + 4 * hh);
              const bf16x8 cf = {(bf16)c0[0], (bf16)c0[1], (bf16)c0[2], (bf16)c0[3],
                                 (bf16)c1[0], (bf16)c1[1], (bf16)c1[2], (bf16)c1[3]};
              acc = mfma32(rd_tr(Kw, 16 * s2, db * 32, lane), cf, acc);
            }
            if ((lane & 31) == 0) {  // every column holds the same sums: rows d = db*32 + acc_row(r, hh)
              float* o = cs_part + ((long)b * NB + w) * 3 * D + h * dh + db * 32;
#pragma unroll
              for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 8 * g4 + 4 * hh;
                if (db * 32 + d < dh)
                  *(f32x4*)(o + d) = f32x4{acc[4 * g4] * scale, acc[4 * g4 + 1] * scale, acc[4 * g4 + 2] * scale,
                                           acc[4 * g4 + 3] * scale};
              }
            }
          }
        }
      }
      BST(sb + 4 + 7 * i);
      bar_lds();  // dS tiles and K images read: the next step may overwrite them
      BST(sb + 5 + 7 * i);
        };
    if constexpr (NB > 1) step(0, std::false_type{}, std::true_type{});
#pragma unroll 1
    for (int i = 1; i + 1 < NB; ++i) step(i, std::false_type{}, std::false_type{});
    step(NB - 1, std::true_type{}, std::bool_constant<NB == 1>{});
    // ---- epilogue of unit u (one barrier)
    if (has_next) {
      wait_vm<0>();  // this wave's DMA rows of the next unit, its K / V fragments, its mask word, the claim
      asm volatile("" : "+v"(claim_raw));  // read only after the wait above
      if (wq.q && threadIdx.x == 0) unn = wq_claim_finish(claim_raw, wq.base, BH);
      write_kimg(kf);  // the last step's dQ phase (barrier above) was the last reader of the K images
      // the next unit's first keep word, consumed here (after the wait above, so the compiler's wait for
      // it costs nothing) instead of in that unit's first step, where it would also wait for the stores
      // this epilogue issues below
      mw0 = mask ? mw0 : 0xFFFFFFFFu;
      asm volatile("" : "+v"(mw0));
    }
    BST(sb + 50);
    {
      const int b = u / H, h = u - b * H;
      // dQ^T (lane = query, registers = 4 consecutive d per group) through a wave-private [32][64] bf16
      // tile (16-byte chunk c of row r at c ^ (r & 7)), stored as whole 128-byte rows: the per-lane
      // 8-byte stores at the row stride were store-issue bound (2k cycles per unit)
      char* dqs = lds + cur * 2 * IMG + w * 8192;  // this unit's Q/dO half, wave-private
      // every store below is a buffer store with out-of-range lanes at FER_OOB (dropped by the range
      // check) instead of an exec-masked store: no divergent branches, so the compiler's vmcnt counts
      // stay exact and later waits (the next unit's keep word) do not wait for these stores
      const __amdgpu_buffer_rsrc_t rdq = make_rsrc(dqkv);
      {
        const int qr = lane & 31;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int d = db * 32 + 8 * g4 + 4 * hh;
            *(bf16x4*)(dqs + qr * 128 + ((((d >> 3) ^ (qr & 7))) << 4) + (d & 4) * 2) =
                bf16x4{(bf16)(dq[db][4 * g4] * scale), (bf16)(dq[db][4 * g4 + 1] * scale),
                       (bf16)(dq[db][4 * g4 + 2] * scale), (bf16)(dq[db][4 * g4 + 3] * scale)};
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private: no barrier
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = i * 64 + lane, r = t >> 3, c = t & 7;
          const int q = w * 32 + r;
          const bf16x8 v = *(const bf16x8*)(dqs + r * 128 + ((c ^ (r & 7)) << 4));
          const uint32_t off = (q < N && c * 8 < dh) ? (uint32_t)((((long)b * N + q) * lddq + h * dh + c * 8) * 2)
                                                     : FER_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rdq, off, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the dK / dV staging reuses it
      }
      BST(sb + 51);
      if (cs_part) {
#pragma unroll
        for (int db = 0; db < 2; ++db) {  // dK / dV column sums over this wave's valid key rows
          float tk = 0.f, tv = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool ok = w * 32 + acc_row(r, hh) < N;
            tk += ok ? dk[db][r] : 0.f;
            tv += ok ? dv[db][r] : 0.f;
          }
          tk = xhalf_sum(tk);
          tv = xhalf_sum(tv);
          const int d = db * 32 + (lane & 31);
          const uint32_t o = (hh == 0 && d < dh) ? (uint32_t)((((long)b * NB + w) * 3 * D + h * dh + d) * 4) : FER_OOB;
          const __amdgpu_buffer_rsrc_t rcs = make_rsrc(cs_part);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(tk * scale), rcs, o, D * 4, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(tv * dscale), rcs, o, 2 * D * 4, 0);
        }
      }
      BST(sb + 52);
      bf16* stg = (bf16*)(lds + cur * 2 * IMG + w * 8192);  // [2][32][64], wave-private (this unit's Q/dO half)
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = acc_row(r, hh), d = db * 32 + (lane & 31);
          stg[kr * 64 + d] = (bf16)(dk[db][r] * scale);
          stg[2048 + kr * 64 + d] = (bf16)(dv[db][r] * dscale);
        }
      BST(sb + 53);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = i * 64 + lane;  // 512 chunks of 16 B: [2 mats][32 rows][8 chunks]
        const int mat = t >> 8, kr = (t >> 3) & 31, c = t & 7;
        const int gk = w * 32 + kr;
        const uint32_t off = (gk < N && c * 8 < dh)
                                 ? (uint32_t)((((long)b * N + gk) * lddq + (1 + mat) * D + h * dh + c * 8) * 2)
                                 : FER_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *(const bf16x8*)(stg + mat * 2048 + kr * 64 + c * 8)),
                                               rdq, off, 0, 0);
      }
    }
    if (has_next) mwn = mw0;
    if (threadIdx.x == 0) hand[cur] = unn;
    BST(sb + 60);
    bar_lds();  // next unit: K / Q / dO images (each wave waited for its DMA), L / Dq; staging read
    BST(sb + 61);
    u = un;
    un = __builtin_amdgcn_readfirstlane(hand[cur]);
    if (!has_next) break;
  }
}

// ---------------------------------------------------------------- general path
// Any N, dh <= 128 (dh % 8 == 0): the head dimension in DH2 halves of 64 columns (each half is
// one swizzled [rows][128 B] image, so every address helper above is reused unchanged), keys /
// queries streamed through LDS in chunks of 128 rows. Workgroup = 4 waves = 128 queries (forward,
// dQ) or 128 keys (dK/dV) of one (batch, head); grid.y walks the chunks of the sequence. Used
// where the single-workgroup-per-head kernels do not fit (N > 256 or dh > 64): e.g. LatentViTv2
// with heads=4 (dh = 128, `latent_vit.py:24-31` accepts any head count).
constexpr int GEN_ROWS = 128;
constexpr int GEN_IMG = GEN_ROWS * 128;  // one 64-column half of a 128-row chunk

// chunk rows [row0, row0 + 128) of the column block col0 (DH2 halves) -> DH2 images
template <int DH2>
FER_DEV void gen_dma(char* img, __amdgpu_buffer_rsrc_t rs, long row0, long ld, int col0, int nrows, int dh, int w,
                     int lane) {
#pragma unroll
  for (int hf = 0; hf < DH2; ++hf)
    img_dma<4>(img + hf * GEN_IMG, rs, row0, ld, col0 + 64 * hf, nrows, dh - 64 * hf, w, lane);
}

template <int DH2>
__global__ __launch_bounds__(256) void attn_fwd_gen(const bf16* __restrict__ qkv, long ldq, bf16* __restrict__ out,
                                                    long ldo, float* __restrict__ lse, int N, int H, int dh,
                                                    float sl2, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  __shared__ __attribute__((aligned(1024))) char lds[2 * DH2 * GEN_IMG];
  char* Ki = lds;
  char* Vi = lds + DH2 * GEN_IMG;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int q = blockIdx.y * GEN_ROWS + w * 32 + (lane & 31);
  const bool qv = q < N;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(qkv);
  bf16x8 qf[4 * DH2];
#pragma unroll
  for (int s = 0; s < 4 * DH2; ++s) {
    const int d0 = 16 * s + 8 * hh;
    qf[s] = (qv && d0 < dh) ? *(const bf16x8*)(qkv + ((long)b * N + q) * ldq + h * dh + d0) : bf16x8{};
  }
  const uint32_t row = drop_row(bh, N, q);
  float m = -INFINITY, l = 0.f;
  f32x16 ot[2 * DH2];
#pragma unroll
  for (int j = 0; j < 2 * DH2; ++j) ot[j] = f32x16{};
#pragma unroll 1
  for (int c0 = 0; c0 < N; c0 += GEN_ROWS) {
    if (c0) __syncthreads();  // every wave is done with the previous chunk's images
    gen_dma<DH2>(Ki, rs, (long)b * N + c0, ldq, D + h * dh, N - c0, dh, w, lane);
    gen_dma<DH2>(Vi, rs, (long)b * N + c0, ldq, 2 * D + h * dh, N - c0, dh, w, lane);
    wait_vm<0>();
    __syncthreads();
    const int nkb = min(GEN_ROWS / 32, (N - c0 + 31) / 32);
#pragma unroll 1
    for (int kb = 0; kb < nkb; ++kb) {
      const int kg = c0 / 32 + kb;  // global key block
      f32x16 st = {};
#pragma unroll
      for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          st = mfma32(rd_row(Ki + hf * GEN_IMG, kb * 32 + (lane & 31), 2 * s + hh), qf[4 * hf + s], st);
      if (kg * 32 + 32 > N) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kg * 32 + acc_row(r, hh) >= N) st[r] = -INFINITY;
      }
      float bm = st[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) bm = fmaxf(bm, st[r]);
      bm = xhalf_max(bm) * sl2;
      const float mn = fmaxf(m, bm);
      const float al = ex2(m - mn);
      m = mn;
      l *= al;
#pragma unroll
      for (int j = 0; j < 2 * DH2; ++j) ot[j] *= al;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        st[r] = ex2(fmaf(st[r], sl2, -mn));
        l += st[r];
      }
      if (thr) drop16_keys(seed, row, kg, hh, thr, dscale, st);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(st, s2);
#pragma unroll
        for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
          for (int db = 0; db < 2; ++db)
            ot[2 * hf + db] = mfma32(rd_tr(Vi + hf * GEN_IMG, kb * 32 + 16 * s2, db * 32, lane), pf, ot[2 * hf + db]);
      }
    }
  }
  l = xhalf_sum(l);
  if (qv) {
#pragma unroll
    for (int hf = 0; hf < DH2; ++hf)
      store_rows_q(out + ((long)b * N + q) * ldo + h * dh + 64 * hf, ot[2 * hf], ot[2 * hf + 1], 1.f / l, hh,
                   dh - 64 * hf);
    if (hh == 0) lse[(long)bh * N + q] = (m + log2f(l)) * LN2;
  }
}

// dQ: wave = query block; K, V streamed. Per key block: S^T, dP^T = V dO^T,
// dS^T = P^T o (dropout'(dP^T) - Dq), dQ^T += K^T dS^T.   Dq = rowsum(dO o O).
template <int DH2>
__global__ __launch_bounds__(256) void attn_dq_gen(const bf16* __restrict__ qkv, long ldq,
                                                   const bf16* __restrict__ out, long ldo,
                                                   const bf16* __restrict__ dout, long lddo,
                                                   const float* __restrict__ lse, bf16* __restrict__ dqkv, long lddq,
                                                   int N, int H, int dh, float scale, float sl2, uint32_t thr,
                                                   float dscale, uint64_t seed) {
  seed = step_seed(seed);
  __shared__ __attribute__((aligned(1024))) char lds[2 * DH2 * GEN_IMG];
  char* Ki = lds;
  char* Vi = lds + DH2 * GEN_IMG;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int q = blockIdx.y * GEN_ROWS + w * 32 + (lane & 31);
  const bool qv = q < N;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(qkv);
  bf16x8 qf[4 * DH2], of[4 * DH2];
  float dsum = 0.f;
#pragma unroll
  for (int s = 0; s < 4 * DH2; ++s) {
    const int d0 = 16 * s + 8 * hh;
    const bool ok = qv && d0 < dh;
    qf[s] = ok ? *(const bf16x8*)(qkv + ((long)b * N + q) * ldq + h * dh + d0) : bf16x8{};
    of[s] = ok ? *(const bf16x8*)(dout + ((long)b * N + q) * lddo + h * dh + d0) : bf16x8{};
    const bf16x8 ov = ok ? *(const bf16x8*)(out + ((long)b * N + q) * ldo + h * dh + d0) : bf16x8{};
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += (float)ov[j] * (float)of[s][j];
  }
  dsum = xhalf_sum(dsum);
  const float lq = qv ? lse[(long)bh * N + q] * LOG2E : INFINITY;
  const uint32_t row = drop_row(bh, N, q);
  f32x16 dqt[2 * DH2];
#pragma unroll
  for (int j = 0; j < 2 * DH2; ++j) dqt[j] = f32x16{};
#pragma unroll 1
  for (int c0 = 0; c0 < N; c0 += GEN_ROWS) {
    if (c0) __syncthreads();
    gen_dma<DH2>(Ki, rs, (long)b * N + c0, ldq, D + h * dh, N - c0, dh, w, lane);
    gen_dma<DH2>(Vi, rs, (long)b * N + c0, ldq, 2 * D + h * dh, N - c0, dh, w, lane);
    wait_vm<0>();
    __syncthreads();
    const int nkb = min(GEN_ROWS / 32, (N - c0 + 31) / 32);
#pragma unroll 1
    for (int kb = 0; kb < nkb; ++kb) {
      const int kg = c0 / 32 + kb;
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(rd_row(Ki + hf * GEN_IMG, kb * 32 + (lane & 31), 2 * s + hh), qf[4 * hf + s], st);
          dp = mfma32(rd_row(Vi + hf * GEN_IMG, kb * 32 + (lane & 31), 2 * s + hh), of[4 * hf + s], dp);
        }
      if (thr) drop16_keys(seed, row, kg, hh, thr, dscale, dp);
      const bool tail = kg * 32 + 32 > N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = ex2(fmaf(st[r], sl2, -lq));
        if (tail && kg * 32 + acc_row(r, hh) >= N) p = 0.f;
        st[r] = p * (dp[r] - dsum);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 df = pack8(st, s2);
#pragma unroll
        for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
          for (int db = 0; db < 2; ++db)
            dqt[2 * hf + db] = mfma32(rd_tr(Ki + hf * GEN_IMG, kb * 32 + 16 * s2, db * 32, lane), df, dqt[2 * hf + db]);
      }
    }
  }
  if (qv) {
#pragma unroll
    for (int hf = 0; hf < DH2; ++hf)
      store_rows_q(dqkv + ((long)b * N + q) * lddq + h * dh + 64 * hf, dqt[2 * hf], dqt[2 * hf + 1], scale, hh,
                   dh - 64 * hf);
  }
}

// dK, dV: wave = key block; Q and dO streamed (with lse and Dq of the chunk's queries in LDS).
// S = Q K^T, dP = dO V^T (registers hold queries), dV += P_drop^T dO, dK += dS^T Q. The dropout
// hash pairs are consecutive KEYS = neighbouring lanes: each lane of a pair hashes 8 of the 16
// query rows and swaps them with its neighbour.
template <int DH2>
__global__ __launch_bounds__(256) void attn_dkv_gen(const bf16* __restrict__ qkv, long ldq,
                                                    const bf16* __restrict__ out, long ldo,
                                                    const bf16* __restrict__ dout, long lddo,
                                                    const float* __restrict__ lse, bf16* __restrict__ dqkv, long lddq,
                                                    int N, int H, int dh, float scale, float sl2, uint32_t thr,
                                                    float dscale, uint64_t seed) {
  seed = step_seed(seed);
  __shared__ __attribute__((aligned(1024))) char lds[2 * DH2 * GEN_IMG + 2 * GEN_ROWS * 4];
  char* Qi = lds;
  char* Oi = lds + DH2 * GEN_IMG;  // dO images
  float* lse_s = (float*)(lds + 2 * DH2 * GEN_IMG);
  float* dd_s = lse_s + GEN_ROWS;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int key = blockIdx.y * GEN_ROWS + w * 32 + (lane & 31);
  const bool kval = key < N;
  bf16x8 kf[4 * DH2], vf[4 * DH2];
#pragma unroll
  for (int s = 0; s < 4 * DH2; ++s) {
    const int d0 = 16 * s + 8 * hh;
    const bool ok = kval && d0 < dh;
    kf[s] = ok ? *(const bf16x8*)(qkv + ((long)b * N + key) * ldq + D + h * dh + d0) : bf16x8{};
    vf[s] = ok ? *(const bf16x8*)(qkv + ((long)b * N + key) * ldq + 2 * D + h * dh + d0) : bf16x8{};
  }
  const int NP = N + (N & 1);
  const bool odd = lane & 1;
  f32x16 dk[2 * DH2], dv[2 * DH2];
#pragma unroll
  for (int j = 0; j < 2 * DH2; ++j) dk[j] = dv[j] = f32x16{};
#pragma unroll 1
  for (int c0 = 0; c0 < N; c0 += GEN_ROWS) {
    if (c0) __syncthreads();
    gen_dma<DH2>(Qi, make_rsrc(qkv), (long)b * N + c0, ldq, h * dh, N - c0, dh, w, lane);
    gen_dma<DH2>(Oi, make_rsrc(dout), (long)b * N + c0, lddo, h * dh, N - c0, dh, w, lane);
    {  // lse and Dq = rowsum(dO o O) of the chunk's queries: two threads per row
      const int qr = threadIdx.x >> 1, half = threadIdx.x & 1, qg = c0 + qr;
      float dsum = 0.f;
      if (qg < N) {
        const bf16* po = out + ((long)b * N + qg) * ldo + h * dh;
        const bf16* pd = dout + ((long)b * N + qg) * lddo + h * dh;
        for (int d = half * 8; d < dh; d += 16) {
          const bf16x8 a = *(const bf16x8*)(po + d), c = *(const bf16x8*)(pd + d);
#pragma unroll
          for (int j = 0; j < 8; ++j) dsum += (float)a[j] * (float)c[j];
        }
      }
      dsum += __shfl_xor(dsum, 1, 64);
      if (!half) {
        dd_s[qr] = dsum;
        lse_s[qr] = qg < N ? lse[(long)bh * N + qg] * LOG2E : INFINITY;
      }
    }
    wait_vm<0>();
    __syncthreads();
    const int nqb = min(GEN_ROWS / 32, (N - c0 + 31) / 32);
#pragma unroll 1
    for (int qb = 0; qb < nqb; ++qb) {
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(rd_row(Qi + hf * GEN_IMG, qb * 32 + (lane & 31), 2 * s + hh), kf[4 * hf + s], st);
          dp = mfma32(rd_row(Oi + hf * GEN_IMG, qb * 32 + (lane & 31), 2 * s + hh), vf[4 * hf + s], dp);
        }
      uint32_t keep = 0xFFFFu;
      if (thr) {
        uint32_t hv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int qg = c0 + qb * 32 + acc_row(8 * odd + i, hh);
          hv[i] = fer_hash(seed, (((uint32_t)bh * N + qg) * (uint32_t)NP + (uint32_t)(key & ~1)) >> 1);
        }
        keep = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t other = (uint32_t)__shfl_xor((int)hv[i], 1, 64);
          const uint32_t h_lo = odd ? other : hv[i];
          const uint32_t h_hi = odd ? hv[i] : other;
          const uint32_t u_lo = odd ? (h_lo >> 16) : (h_lo & 0xFFFFu);
          const uint32_t u_hi = odd ? (h_hi >> 16) : (h_hi & 0xFFFFu);
          keep |= (uint32_t)(u_lo >= thr) << i;
          keep |= (uint32_t)(u_hi >= thr) << (8 + i);
        }
      }
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = qb * 32 + acc_row(r, hh);
        const float p = kval ? ex2(fmaf(st[r], sl2, -lse_s[qr])) : 0.f;
        const bool kp = (keep >> r) & 1;
        const float g = thr ? (kp ? dp[r] * dscale : 0.f) : dp[r];
        pd[r] = thr ? (kp ? p * dscale : 0.f) : p;
        st[r] = p * (g - dd_s[qr]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(pd, s2), df = pack8(st, s2);
#pragma unroll
        for (int hf = 0; hf < DH2; ++hf)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dv[2 * hf + db] = mfma32(pf, rd_tr(Oi + hf * GEN_IMG, qb * 32 + 16 * s2, db * 32, lane), dv[2 * hf + db]);
            dk[2 * hf + db] = mfma32(df, rd_tr(Qi + hf * GEN_IMG, qb * 32 + 16 * s2, db * 32, lane), dk[2 * hf + db]);
          }
      }
    }
  }
  // dk/dv[2*hf+db][r]: key row = w*32 + acc_row(r, hh), d = 64*hf + db*32 + (lane&31). Stage each
  // wave's [2 mats][32 rows][64*DH2] tile through LDS (wave-private region, inside the images) for
  // 16-byte row stores.
  __syncthreads();
  constexpr int W = 64 * DH2;
  bf16* stg = (bf16*)(lds + w * (2 * 32 * W * 2));
#pragma unroll
  for (int j = 0; j < 2 * DH2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = acc_row(r, hh), d = j * 32 + (lane & 31);
      stg[kr * W + d] = (bf16)(dk[j][r] * scale);
      stg[32 * W + kr * W + d] = (bf16)dv[j][r];
    }
#pragma unroll
  for (int i = 0; i < 8 * DH2; ++i) {
    const int t = i * 64 + lane;  // [2 mats][32 rows][W/8 chunks]
    constexpr int CPR = W / 8;
    const int mat = t / (32 * CPR), kr = (t / CPR) & 31, c = t % CPR;
    const int gk = blockIdx.y * GEN_ROWS + w * 32 + kr;
    if (gk < N && c * 8 < dh)
      *(bf16x8*)(dqkv + ((long)b * N + gk) * lddq + (1 + mat) * D + h * dh + c * 8) =
          *(const bf16x8*)(stg + mat * 32 * W + kr * W + c * 8);
  }
}

// ------------------------------------------------------------------ fp32 path
// ws layout: P [BH][N][N] (softmax probs, undropped), then G [BH][N][N]
__global__ void attn_f32_scores(const float* qkv, long ldq, float* P, int B, int N, int H, int dh, float scale) {
  const long idx = blockIdx.x * 256L + threadIdx.x;
  const long total = (long)B * H * N * N;
  if (idx >= total) return;
  const int k = idx % N, q = (idx / N) % N, bh = idx / ((long)N * N), b = bh / H, h = bh % H, D = H * dh;
  const float* qr = qkv + ((long)b * N + q) * ldq + h * dh;
  const float* kr = qkv + ((long)b * N + k) * ldq + D + h * dh;
  float s = 0.f;
  for (int d = 0; d < dh; ++d) s = fmaf(qr[d], kr[d], s);
  P[idx] = s * scale;
}
__global__ void attn_f32_softmax(float* P, float* lse, long rows, int N) {
  const long r = blockIdx.x * 256L + threadIdx.x;
  if (r >= rows) return;
  float* p = P + r * N;
  float m = -INFINITY;
  for (int k = 0; k < N; ++k) m = fmaxf(m, p[k]);
  float l = 0.f;
  for (int k = 0; k < N; ++k) l += expf(p[k] - m);
  for (int k = 0; k < N; ++k) p[k] = expf(p[k] - m) / l;
  if (lse) lse[r] = m + logf(l);
}
__global__ void attn_f32_pv(const float* P, const float* qkv, long ldq, float* out, long ldo, int B, int N, int H,
                            int dh, uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  const long idx = blockIdx.x * 256L + threadIdx.x;
  const long total = (long)B * H * N * dh;
  if (idx >= total) return;
  const int d = idx % dh, q = (idx / dh) % N, bh = idx / ((long)dh * N), b = bh / H, h = bh % H, D = H * dh;
  const float* pr = P + ((long)bh * N + q) * N;
  const uint32_t rowidx = drop_row(bh, N, q);
  float s = 0.f;
  for (int k = 0; k < N; ++k) {
    float p = pr[k];
    if (thr) p = drop_keep(seed, rowidx + k, thr) ? p * dscale : 0.f;
    s = fmaf(p, qkv[((long)b * N + k) * ldq + 2 * D + h * dh + d], s);
  }
  out[((long)b * N + q) * ldo + h * dh + d] = s;
}
// G = dS (into the second ws slab); dd = rowsum(dO * O)
__global__ void attn_f32_ds(const float* P, float* G, const float* qkv, long ldq, const float* out, long ldo,
                            const float* dout, long lddo, int B, int N, int H, int dh, uint32_t thr, float dscale,
                            uint64_t seed) {
  seed = step_seed(seed);
  const long r = blockIdx.x * 256L + threadIdx.x;
  const long rows = (long)B * H * N;
  if (r >= rows) return;
  const int q = r % N, bh = r / N, b = bh / H, h = bh % H, D = H * dh;
  const float* o = out + ((long)b * N + q) * ldo + h * dh;
  const float* g = dout + ((long)b * N + q) * lddo + h * dh;
  float dd = 0.f;
  for (int d = 0; d < dh; ++d) dd = fmaf(o[d], g[d], dd);
  for (int k = 0; k < N; ++k) {
    const float* v = qkv + ((long)b * N + k) * ldq + 2 * D + h * dh;
    float dp = 0.f;
    for (int d = 0; d < dh; ++d) dp = fmaf(g[d], v[d], dp);
    if (thr) dp = drop_keep(seed, drop_row(bh, N, q) + k, thr) ? dp * dscale : 0.f;
    G[r * N + k] = P[r * N + k] * (dp - dd);
  }
}
__global__ void attn_f32_grads(const float* P, const float* G, const float* qkv, long ldq, const float* dout,
                               long lddo, float* dqkv, long lddq, int B, int N, int H, int dh, float scale,
                               uint32_t thr, float dscale, uint64_t seed) {
  seed = step_seed(seed);
  const long idx = blockIdx.x * 256L + threadIdx.x;
  const long total = (long)B * H * N * dh;
  if (idx >= total) return;
  const int d = idx % dh, t = (idx / dh) % N, bh = idx / ((long)dh * N), b = bh / H, h = bh % H, D = H * dh;
  const long rb = (long)bh * N;
  float dq = 0.f, dk = 0.f, dv = 0.f;
  for (int j = 0; j < N; ++j) {
    dq = fmaf(G[(rb + t) * N + j], qkv[((long)b * N + j) * ldq + D + h * dh + d], dq);
    dk = fmaf(G[(rb + j) * N + t], qkv[((long)b * N + j) * ldq + h * dh + d], dk);
    float p = P[(rb + j) * N + t];
    if (thr) p = drop_keep(seed, drop_row(bh, N, j) + t, thr) ? p * dscale : 0.f;
    dv = fmaf(p, dout[((long)b * N + j) * lddo + h * dh + d], dv);
  }
  float* o = dqkv + ((long)b * N + t) * lddq + h * dh + d;
  o[0] = dq * scale;
  o[D] = dk * scale;
  o[2 * D] = dv;
}

#define FER_NB_SWITCH(NB, ...)     \
  switch (NB) {                    \
    case 1: { constexpr int NB_ = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int NB_ = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int NB_ = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int NB_ = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int NB_ = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int NB_ = 6; __VA_ARGS__; } break; \
    case 7: { constexpr int NB_ = 7; __VA_ARGS__; } break; \
    default: { constexpr int NB_ = 8; __VA_ARGS__; } break; \
  }

}  // namespace fer

using namespace fer;

int fer::set_step_ptr_attention(const uint64_t* p) { return set_step_ptr_here(p) == hipSuccess ? 0 : -1; }

#ifdef FER_ATTN_STAMPS
extern "C" int fer_debug_attn_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ast), sizeof(unsigned long long) * 9 * 64) == hipSuccess ? 0 : 1;
}
extern "C" int fer_debug_attn_bwd_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bst), sizeof(unsigned long long) * 8 * 128) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int64_t fer_attention_ws(int dtype, int B, int N, int H) {
  // fp32 path: P and dS slabs, then the stand-alone colsum pass's partials; bf16: the fused
  // bias-gradient partials [B][3*H*64]
  const int64_t cs = std::max<int64_t>(fer_colsum_ws(B * N, 3 * H * 128), (int64_t)B * 7 * 3 * H * 64 * 4);
  return (dtype == FER_F32 ? (int64_t)2 * B * H * N * N * 4 : 0) + cs;
}

static bool pers_path(int dtype, int N, int dh) { return dtype == FER_BF16 && N <= 224 && dh <= 64; }
// forward kernel for N <= 224, dh <= 64 (fer_attention_set_fwd_kernel): 0 automatic (the occupancy form
// from 4 query blocks up with dropout on -- ViT-B/16's N = 197: 36.57 vs 36.87 ms per step on one box,
// profiles/r05d_*; alone 116 vs 125-139 us at p = 0.1 -- the persistent kernel without dropout (82 vs
// 90 us at p = 0, profiles/r06e_attn_fwd_spill_ab.txt: its producer wave hides the K / V loads and no
// hashing VALU is left for the occupancy form's extra waves to hide) and below 4 query blocks, where
// its occupancy-sized grids were tuned for the w+ / 48 px token counts), 1 persistent, 2 occupancy form
static int g_fwd_kernel = 0;
static int64_t lse_floats(int B, int N, int H) { return ((int64_t)B * H * N + 63) / 64 * 64; }
// persistent kernels walk a fixed blockIdx stride instead of the work queue (fer_set_persistent_mode)
static bool fixed_stride() { return fixed_stride_mode(); }
static int n_cus() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 256;
    return c > 0 ? c : 256;
  }();
  return n;
}

// Workgroups per CU a persistent attention kernel can hold (registers / LDS; the occupancy API,
// queried once per instantiation): the small-N instantiations (w+ latents: N = 19, one key block)
// are one or two waves and fit several to a CU, so their persistent grid is CUs x this, not CUs --
// one wave per CU left the latent-ViT attention latency-bound.
template <typename Kern>
static int pers_occ(Kern k, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, threads, 0) != hipSuccess || n < 1) n = 1;
  return std::min(n, 8);
}

extern "C" int64_t fer_attention_saved_floats(int dtype, int B, int N, int H, int dh, uint32_t drop_thresh) {
  const int64_t nb = (N + 31) / 32;
  const int64_t mask_words = (drop_thresh && pers_path(dtype, N, dh)) ? (int64_t)B * H * nb * nb * 32 : 0;
  return lse_floats(B, N, H) + mask_words;
}

extern "C" int fer_attention_fwd(int dtype, const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse,
                                 int64_t saved_floats, int B, int N, int H, int dh, float scale, uint32_t drop_thresh,
                                 float drop_scale, uint64_t seed, float* ws, int64_t ws_bytes, fer_stream_t stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (saved_floats < fer_attention_saved_floats(dtype, B, N, H, dh, drop_thresh))
    return set_error("attention_fwd: saved-state buffer smaller than fer_attention_saved_floats()");
  if (dtype == FER_F32) {
    if (!ws || ws_bytes < fer_attention_ws(dtype, B, N, H)) return set_error("attention_fwd: fp32 workspace too small");
    const long pe = (long)B * H * N * N, rows = (long)B * H * N, oe = rows * dh;
    hipLaunchKernelGGL(attn_f32_scores, dim3(ceil_div(pe, 256)), dim3(256), 0, st, (const float*)qkv, (long)ld_qkv, ws,
                       B, N, H, dh, scale);
    hipLaunchKernelGGL(attn_f32_softmax, dim3(ceil_div(rows, 256)), dim3(256), 0, st, ws, lse, rows, N);
    hipLaunchKernelGGL(attn_f32_pv, dim3(ceil_div(oe, 256)), dim3(256), 0, st, (const float*)ws, (const float*)qkv,
                       (long)ld_qkv, (float*)out, (long)ld_out, B, N, H, dh, drop_thresh, drop_scale, seed);
    return hip_check("attention_fwd_f32");
  }
  if (dh > 128 || dh % 8) return set_error("attention_fwd(bf16): needs dh <= 128, dh % 8 == 0");
  if (check_drop_range(drop_thresh, (long)B * H * N * (N + (N & 1)), "attention_fwd: dropout over >= 2^32 probabilities"))
    return -1;
  if (ld_qkv % 8 || ld_out % 4) return set_error("attention_fwd(bf16): misaligned leading dimension");
  // (the persistent kernel addresses qkv and out through 32-bit buffer offsets, bit 31 = out of range)
  if ((long)B * N * ld_qkv * 2 >= 0x7FFFFFF0L || (long)B * N * ld_out * 2 >= 0x7FFFFFF0L)
    return set_error("attention_fwd(bf16): qkv or out exceeds 2 GiB");
  const float sl2 = scale * LOG2E;
  if (N <= 256 && dh <= 64 && N > 224) {  // NB = 8: 9 waves would not fit 2/SIMD
    const int nb = (N + 31) / 32;
    FER_NB_SWITCH(nb, hipLaunchKernelGGL(attn_fwd_bf16<NB_>, dim3(B * H), dim3(64 * NB_), 0, st, (const bf16*)qkv,
                                         (long)ld_qkv, (bf16*)out, (long)ld_out, lse, N, H, dh, sl2, drop_thresh,
                                         drop_scale, seed));
  } else if (N <= 224 && dh <= 64 && (g_fwd_kernel == 2 || (g_fwd_kernel == 0 && drop_thresh && (N + 31) / 32 >= 4))) {
    const int nb = (N + 31) / 32;
    uint32_t* mask = (drop_thresh && pers_path(dtype, N, dh)) ? (uint32_t*)(lse + lse_floats(B, N, H)) : nullptr;
#define FER_FOCC2(NBV)                                                                                     \
  case NBV:                                                                                                \
    hipLaunchKernelGGL((attn_fwd_occ<NBV>), dim3(B * H), dim3(64 * NBV), 0, st, (const bf16*)qkv,          \
                       (long)ld_qkv, (bf16*)out, (long)ld_out, lse, mask, N, H, dh, sl2, drop_thresh,       \
                       drop_scale, seed);                                                                  \
    break;
    switch (nb) {
      FER_FOCC2(1) FER_FOCC2(2) FER_FOCC2(3) FER_FOCC2(4) FER_FOCC2(5) FER_FOCC2(6) FER_FOCC2(7)
    }
#undef FER_FOCC2
  } else if (N <= 224 && dh <= 64) {
    const int nb = (N + 31) / 32;
    uint32_t* mask = (drop_thresh && pers_path(dtype, N, dh)) ? (uint32_t*)(lse + lse_floats(B, N, H)) : nullptr;
    int occ = 1;
#define FER_FOCC(NBV)                                                               \
  case NBV: {                                                                       \
    static const int o = pers_occ(attn_fwd_pers<NBV>, 64 * (NBV + 1));             \
    occ = o;                                                                        \
  } break;
    switch (nb) { FER_FOCC(1) FER_FOCC(2) FER_FOCC(3) FER_FOCC(4) FER_FOCC(5) FER_FOCC(6) FER_FOCC(7) }
#undef FER_FOCC
    const int grid = std::min(B * H, n_cus() * occ);
    const WqArgs wq = fixed_stride() ? WqArgs{} : wq_prepare_here(st, grid, B * H);
#define FER_FPERS(NBV)                                                                                     \
  case NBV:                                                                                                \
    hipLaunchKernelGGL((attn_fwd_pers<NBV>), dim3(grid), dim3(64 * (NBV + 1)), 0, st, (const bf16*)qkv,    \
                       (long)ld_qkv, (bf16*)out, (long)ld_out, lse, mask, B * H, N, H, dh, sl2, drop_thresh, \
                       drop_scale, seed, wq);                                                             \
    break;
    switch (nb) {
      FER_FPERS(1) FER_FPERS(2) FER_FPERS(3) FER_FPERS(4) FER_FPERS(5) FER_FPERS(6) FER_FPERS(7)
    }
#undef FER_FPERS
    wq_check_launch(st, wq);
  } else {
    const dim3 grid(B * H, (N + GEN_ROWS - 1) / GEN_ROWS);
    if (dh <= 64)
      hipLaunchKernelGGL(attn_fwd_gen<1>, grid, dim3(256), 0, st, (const bf16*)qkv, (long)ld_qkv, (bf16*)out,
                         (long)ld_out, lse, N, H, dh, sl2, drop_thresh, drop_scale, seed);
    else
      hipLaunchKernelGGL(attn_fwd_gen<2>, grid, dim3(256), 0, st, (const bf16*)qkv, (long)ld_qkv, (bf16*)out,
                         (long)ld_out, lse, N, H, dh, sl2, drop_thresh, drop_scale, seed);
  }
  return hip_check("attention_fwd_bf16");
}

extern "C" int fer_attention_bwd(int dtype, const void* qkv, int64_t ld_qkv, const void* out, int64_t ld_out,
                                 const void* dout, int64_t ld_dout, const float* lse, int64_t saved_floats, void* dqkv,
                                 int64_t ld_dqkv, float* ws, int64_t ws_bytes, int B, int N, int H, int dh,
                                 float scale, uint32_t drop_thresh, float drop_scale, uint64_t seed, float* colsum,
                                 int colsum_accumulate, fer_stream_t stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (saved_floats < fer_attention_saved_floats(dtype, B, N, H, dh, drop_thresh))
    return set_error("attention_bwd: saved-state buffer smaller than fer_attention_saved_floats()");
  const int D3 = 3 * H * dh;
  if (colsum && (!ws || ws_bytes < fer_attention_ws(dtype, B, N, H)))
    return set_error("attention_bwd: colsum needs the workspace (fer_attention_ws bytes)");
  // column sums of dqkv by a separate pass (fp32 path, two-kernel bf16 path)
  auto colsum_pass = [&](float* cws, int64_t cbytes) -> int {
    return fer_colsum(dtype, dqkv, ld_dqkv, B * N, D3, colsum, colsum_accumulate, nullptr, cws, cbytes, stream);
  };
  if (dtype == FER_F32) {
    if (!ws || ws_bytes < fer_attention_ws(dtype, B, N, H)) return set_error("attention_bwd: fp32 workspace too small");
    const long pe = (long)B * H * N * N, rows = (long)B * H * N, oe = rows * dh;
    float* P = ws;
    float* G = ws + pe;
    hipLaunchKernelGGL(attn_f32_scores, dim3(ceil_div(pe, 256)), dim3(256), 0, st, (const float*)qkv, (long)ld_qkv, P,
                       B, N, H, dh, scale);
    hipLaunchKernelGGL(attn_f32_softmax, dim3(ceil_div(rows, 256)), dim3(256), 0, st, P, (float*)nullptr, rows, N);
    hipLaunchKernelGGL(attn_f32_ds, dim3(ceil_div(rows, 256)), dim3(256), 0, st, (const float*)P, G,
                       (const float*)qkv, (long)ld_qkv, (const float*)out, (long)ld_out, (const float*)dout,
                       (long)ld_dout, B, N, H, dh, drop_thresh, drop_scale, seed);
    hipLaunchKernelGGL(attn_f32_grads, dim3(ceil_div(oe, 256)), dim3(256), 0, st, (const float*)P, (const float*)G,
                       (const float*)qkv, (long)ld_qkv, (const float*)dout, (long)ld_dout, (float*)dqkv,
                       (long)ld_dqkv, B, N, H, dh, scale, drop_thresh, drop_scale, seed);
    int rc = hip_check("attention_bwd_f32");
    if (rc || !colsum) return rc;
    return colsum_pass(ws + 2 * pe, ws_bytes - 2 * pe * 4);
  }
  if (dh > 128 || dh % 8) return set_error("attention_bwd(bf16): needs dh <= 128, dh % 8 == 0");
  if (check_drop_range(drop_thresh, (long)B * H * N * (N + (N & 1)), "attention_bwd: dropout over >= 2^32 probabilities"))
    return -1;
  if (ld_qkv % 8 || ld_out % 8 || ld_dout % 8 || ld_dqkv % 8) return set_error("attention_bwd(bf16): misaligned ld");
  if ((long)B * N * ld_qkv * 2 >= 0x7FFFFFF0L || (long)B * N * ld_dout * 2 >= 0x7FFFFFF0L ||
      (long)B * N * ld_dqkv * 2 >= 0x7FFFFFF0L || (long)B * N * ld_out * 2 >= 0x7FFFFFF0L)
    return set_error("attention_bwd(bf16): operand exceeds 2 GiB (buffer-resource range)");
  const int nb = (N + 31) / 32;
  const float sl2 = scale * LOG2E;
  if (pers_path(dtype, N, dh)) {
    const uint32_t* mask = drop_thresh ? (const uint32_t*)(lse + lse_floats(B, N, H)) : nullptr;
    if (colsum) ws = reduction_ws(ws, (size_t)B * nb * D3 * 4, D3, st);
    int occ = 1;
#define FER_BOCC(NBV)                                                               \
  case NBV: {                                                                       \
    static const int o = pers_occ(attn_bwd_pers<NBV>, bwd_threads<NBV>());                   \
    occ = o;                                                                        \
  } break;
    switch (nb) { FER_BOCC(1) FER_BOCC(2) FER_BOCC(3) FER_BOCC(4) FER_BOCC(5) FER_BOCC(6) FER_BOCC(7) }
#undef FER_BOCC
    const int grid = std::min(B * H, n_cus() * occ);
    const WqArgs wq = fixed_stride() ? WqArgs{} : wq_prepare_here(st, grid, B * H);
#define FER_PERS(NBV)                                                                                          \
  case NBV:                                                                                                    \
    hipLaunchKernelGGL(attn_bwd_pers<NBV>, dim3(grid), dim3(bwd_threads<NBV>()), 0, st, (const bf16*)qkv,                \
                       (long)ld_qkv, (const bf16*)out, (long)ld_out, (const bf16*)dout, (long)ld_dout, lse, mask, \
                       (bf16*)dqkv, (long)ld_dqkv, B * H, N, H, dh, scale, sl2, drop_scale, colsum ? ws : nullptr, \
                       wq);                                                                                      \
    break;
    switch (nb) {
      FER_PERS(1) FER_PERS(2) FER_PERS(3) FER_PERS(4) FER_PERS(5) FER_PERS(6) FER_PERS(7)
    }
#undef FER_PERS
    wq_check_launch(st, wq);
    int rc = hip_check("attention_bwd_bf16_pers");
    if (rc || !colsum) return rc;
    part_reduce(ws, B * nb, D3, D3, D3, colsum, nullptr, nullptr, colsum_accumulate, nullptr, st);
    return hip_check("attention_bwd_colsum");
  }
  if (nb <= 8 && dh <= 64) {
    if (colsum) ws = reduction_ws(ws, (size_t)B * D3 * 4, D3, st);
#define FER_FUSED(NBV)                                                                                       \
  case NBV:                                                                                                  \
    hipLaunchKernelGGL(attn_bwd_fused_bf16<NBV>, dim3(B * H), dim3(64 * NBV), 0, st, (const bf16*)qkv,       \
                       (long)ld_qkv, (const bf16*)out, (long)ld_out, (const bf16*)dout, (long)ld_dout, lse,   \
                       (bf16*)dqkv, (long)ld_dqkv, N, H, dh, scale, sl2, drop_thresh, drop_scale, seed,      \
                       colsum ? ws : nullptr);                                                              \
    break;
    switch (nb) {  // every N <= 256
      FER_FUSED(1) FER_FUSED(2) FER_FUSED(3) FER_FUSED(4) FER_FUSED(5) FER_FUSED(6) FER_FUSED(7)
      FER_FUSED(8)
    }
#undef FER_FUSED
    int rc = hip_check("attention_bwd_bf16_fused");
    if (rc || !colsum) return rc;
    part_reduce(ws, B, D3, D3, D3, colsum, nullptr, nullptr, colsum_accumulate, nullptr, st);
    return hip_check("attention_bwd_colsum");
  }
  const dim3 grid(B * H, (N + GEN_ROWS - 1) / GEN_ROWS);
#define FER_GEN(DH2)                                                                                           \
  hipLaunchKernelGGL(attn_dq_gen<DH2>, grid, dim3(256), 0, st, (const bf16*)qkv, (long)ld_qkv, (const bf16*)out, \
                     (long)ld_out, (const bf16*)dout, (long)ld_dout, lse, (bf16*)dqkv, (long)ld_dqkv, N, H, dh,    \
                     scale, sl2, drop_thresh, drop_scale, seed);                                                \
  hipLaunchKernelGGL(attn_dkv_gen<DH2>, grid, dim3(256), 0, st, (const bf16*)qkv, (long)ld_qkv, (const bf16*)out, \
                     (long)ld_out, (const bf16*)dout, (long)ld_dout, lse, (bf16*)dqkv, (long)ld_dqkv, N, H, dh,     \
                     scale, sl2, drop_thresh, drop_scale, seed);
  if (dh <= 64) {
    FER_GEN(1)
  } else {
    FER_GEN(2)
  }
#undef FER_GEN
  int rc = hip_check("attention_bwd_bf16");
  if (rc || !colsum) return rc;
  return colsum_pass(ws, ws_bytes);
}

extern "C" int fer_attention_set_fwd_kernel(int k) {
  if (k < 0 || k > 2) return fer::set_error("attention_set_fwd_kernel: 0 (default), 1 (persistent) or 2 (occupancy form)");
  g_fwd_kernel = k;
  return 0;
}
