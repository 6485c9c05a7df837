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
  bf16x4 b1 = __builtin_bit_cast(bf16x4, t1), b2 = __builtin_bit_cast(bf16x4, t2);
  return bf16x8{b1[0], b1[1], b1[2], b1[3], b2[0], b2[1], b2[2], b2[3]};
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

template <int NB>
__global__ __launch_bounds__(64 * NB) void attn_fwd_bf16(const bf16* __restrict__ qkv, long ldq, bf16* __restrict__ out,
                                                       long ldo, float* __restrict__ lse, int N, int H, int dh,
                                                       float sl2, uint32_t thr, float dscale, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char lds[2 * NB * 32 * 128];
  char* Ki = lds;
  char* Vi = lds + NB * 32 * 128;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const bf16* base = qkv + (long)b * N * ldq;
  load_image<NB>(Ki, base + D + h * dh, ldq, N, dh);
  load_image<NB>(Vi, base + 2 * D + h * dh, ldq, N, dh);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5;
  const int q = w * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int d0 = 16 * s + 8 * hh;
    qf[s] = (q < N && d0 < dh) ? *(const bf16x8*)(base + (long)q * ldq + h * dh + d0) : bf16x8{};
  }
  __syncthreads();

  f32x16 st[NB];
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    st[kb] = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) st[kb] = mfma32(rd_row(Ki, kb * 32 + (lane & 31), 2 * s + hh), qf[s], st[kb]);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kb * 32 + acc_row(r, hh);
      const float v = key < N ? st[kb][r] * sl2 : -INFINITY;
      st[kb][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float l = 0.f;
  const uint64_t rowidx = ((uint64_t)bh * N + q) * (uint64_t)N;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = exp2f(st[kb][r] - mx);
      l += e;
      float pv = e;
      if (thr) {
        const int key = kb * 32 + acc_row(r, hh);
        pv = drop_keep(seed, rowidx + key, thr) ? e * dscale : 0.f;
      }
      st[kb][r] = pv;
    }
  l += __shfl_xor(l, 32, 64);

  f32x16 ot[2] = {f32x16{}, f32x16{}};
#pragma unroll
  for (int kb = 0; kb < NB; ++kb)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = pack8(st[kb], s2);
#pragma unroll
      for (int db = 0; db < 2; ++db) ot[db] = mfma32(rd_tr(Vi, kb * 32 + 16 * s2, db * 32, lane), pf, ot[db]);
    }
  if (q < N) {
    const float inv = 1.f / l;
    bf16* o = out + ((long)b * N + q) * ldo + h * dh;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = db * 32 + 8 * g4 + 4 * hh;
        if (d < dh)
          *(bf16x4*)(o + d) = bf16x4{(bf16)(ot[db][4 * g4] * inv), (bf16)(ot[db][4 * g4 + 1] * inv),
                                     (bf16)(ot[db][4 * g4 + 2] * inv), (bf16)(ot[db][4 * g4 + 3] * inv)};
      }
    if (hh == 0) lse[(long)bh * N + q] = (mx + log2f(l)) * LN2;
  }
}

template <int NB>
__global__ __launch_bounds__(64 * NB) void attn_bwd_bf16(const bf16* __restrict__ qkv, long ldq,
                                                       const bf16* __restrict__ out, long ldo,
                                                       const bf16* __restrict__ dout, long lddo,
                                                       const float* __restrict__ lse, bf16* __restrict__ dqkv,
                                                       long lddq, int N, int H, int dh, float scale, float sl2,
                                                       uint32_t thr, float dscale, uint64_t seed) {
  constexpr int IMG = NB * 32 * 128;
  __shared__ __attribute__((aligned(16))) char lds[4 * IMG + 2 * NB * 32 * 4];
  char* Qi = lds;
  char* Ki = lds + IMG;
  char* Vi = lds + 2 * IMG;
  char* Oi = lds + 3 * IMG;  // dO image
  float* lse_s = (float*)(lds + 4 * IMG);
  float* dd_s = lse_s + NB * 32;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H, D = H * dh;
  const bf16* base = qkv + (long)b * N * ldq;
  load_image<NB>(Qi, base + h * dh, ldq, N, dh);
  load_image<NB>(Ki, base + D + h * dh, ldq, N, dh);
  load_image<NB>(Vi, base + 2 * D + h * dh, ldq, N, dh);
  load_image<NB>(Oi, dout + (long)b * N * lddo + h * dh, lddo, N, dh);
  for (int q = threadIdx.x; q < NB * 32; q += blockDim.x) {
    float dsum = 0.f, lv = INFINITY;
    if (q < N) {
      const bf16* po = out + ((long)b * N + q) * ldo + h * dh;
      const bf16* pd = dout + ((long)b * N + q) * lddo + h * dh;
      for (int d = 0; d < dh; d += 8) {
        bf16x8 a = *(const bf16x8*)(po + d), c = *(const bf16x8*)(pd + d);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)a[j] * (float)c[j];
      }
      lv = lse[(long)bh * N + q] * LOG2E;
    }
    lse_s[q] = lv;
    dd_s[q] = dsum;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5;
  // ---------------- phase 1: wave w owns query block w -> dQ
  {
    const int q = w * 32 + (lane & 31);
    bf16x8 qf[4], of[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = rd_row(Qi, q, 2 * s + hh);
      of[s] = rd_row(Oi, q, 2 * s + hh);
    }
    const float lq = lse_s[q], dq = dd_s[q];
    const uint64_t rowidx = ((uint64_t)bh * N + q) * (uint64_t)N;
    f32x16 dqt[2] = {f32x16{}, f32x16{}};
    for (int kb = 0; kb < NB; ++kb) {
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(rd_row(Ki, kb * 32 + (lane & 31), 2 * s + hh), qf[s], st);
        dp = mfma32(rd_row(Vi, kb * 32 + (lane & 31), 2 * s + hh), of[s], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * 32 + acc_row(r, hh);
        const float p = key < N ? exp2f(st[r] * sl2 - lq) : 0.f;
        float g = dp[r];
        if (thr) g = drop_keep(seed, rowidx + key, thr) ? g * dscale : 0.f;
        st[r] = p * (g - dq);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 df = pack8(st, s2);
#pragma unroll
        for (int db = 0; db < 2; ++db) dqt[db] = mfma32(rd_tr(Ki, kb * 32 + 16 * s2, db * 32, lane), df, dqt[db]);
      }
    }
    if (q < N) {
      bf16* o = dqkv + ((long)b * N + q) * lddq + h * dh;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = db * 32 + 8 * g4 + 4 * hh;
          if (d < dh)
            *(bf16x4*)(o + d) = bf16x4{(bf16)(dqt[db][4 * g4] * scale), (bf16)(dqt[db][4 * g4 + 1] * scale),
                                       (bf16)(dqt[db][4 * g4 + 2] * scale), (bf16)(dqt[db][4 * g4 + 3] * scale)};
        }
    }
  }
  // ---------------- phase 2: wave w owns key block w -> dK, dV
  {
    const int key = w * 32 + (lane & 31);
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = rd_row(Ki, key, 2 * s + hh);
      vf[s] = rd_row(Vi, key, 2 * s + hh);
    }
    f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
    const bool kval = key < N;
    for (int qb = 0; qb < NB; ++qb) {
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(rd_row(Qi, qb * 32 + (lane & 31), 2 * s + hh), kf[s], st);
        dp = mfma32(rd_row(Oi, qb * 32 + (lane & 31), 2 * s + hh), vf[s], dp);
      }
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qb * 32 + acc_row(r, hh);
        const float p = kval ? exp2f(st[r] * sl2 - lse_s[q]) : 0.f;
        float g = dp[r], pdv = p;
        if (thr) {
          const bool keep = drop_keep(seed, ((uint64_t)bh * N + q) * (uint64_t)N + key, thr);
          g = keep ? g * dscale : 0.f;
          pdv = keep ? p * dscale : 0.f;
        }
        pd[r] = pdv;
        st[r] = p * (g - dd_s[q]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(pd, s2), df = pack8(st, s2);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          dv[db] = mfma32(pf, rd_tr(Oi, qb * 32 + 16 * s2, db * 32, lane), dv[db]);
          dk[db] = mfma32(df, rd_tr(Qi, qb * 32 + 16 * s2, db * 32, lane), dk[db]);
        }
      }
    }
    // dk/dv[db][r]: key row = w*32 + acc_row(r), d = db*32 + (lane&31)
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int d = db * 32 + (lane & 31);
      if (d >= dh) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = w * 32 + acc_row(r, hh);
        if (kr < N) {
          bf16* o = dqkv + ((long)b * N + kr) * lddq;
          o[D + h * dh + d] = (bf16)(dk[db][r] * scale);
          o[2 * D + h * dh + d] = (bf16)dv[db][r];
        }
      }
    }
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
  const long idx = blockIdx.x * 256L + threadIdx.x;
  const long total = (long)B * H * N * dh;
  if (idx >= total) return;
  const int d = idx % dh, q = (idx / dh) % N, bh = idx / ((long)dh * N), b = bh / H, h = bh % H, D = H * dh;
  const float* pr = P + ((long)bh * N + q) * N;
  const uint64_t rowidx = ((uint64_t)bh * N + q) * (uint64_t)N;
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
    if (thr) dp = drop_keep(seed, (uint64_t)r * N + k, thr) ? dp * dscale : 0.f;
    G[r * N + k] = P[r * N + k] * (dp - dd);
  }
}
__global__ void attn_f32_grads(const float* P, const float* G, const float* qkv, long ldq, const float* dout,
                               long lddo, float* dqkv, long lddq, int B, int N, int H, int dh, float scale,
                               uint32_t thr, float dscale, uint64_t seed) {
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
    if (thr) p = drop_keep(seed, (uint64_t)(rb + j) * N + t, thr) ? p * dscale : 0.f;
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

extern "C" int64_t fer_attention_ws(int dtype, int B, int N, int H) {
  return dtype == FER_F32 ? (int64_t)2 * B * H * N * N * 4 : 0;
}

extern "C" int fer_attention_fwd(int dtype, const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse,
                                 int B, int N, int H, int dh, float scale, uint32_t drop_thresh, float drop_scale,
                                 uint64_t seed, float* ws, int64_t ws_bytes, fer_stream_t stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
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
  if (N > 256 || dh > 64 || dh % 8) return set_error("attention_fwd(bf16): needs N <= 256, dh <= 64, dh % 8 == 0");
  if (ld_qkv % 8 || ld_out % 4) return set_error("attention_fwd(bf16): misaligned leading dimension");
  const int nb = (N + 31) / 32;
  const float sl2 = scale * LOG2E;
  FER_NB_SWITCH(nb, hipLaunchKernelGGL(attn_fwd_bf16<NB_>, dim3(B * H), dim3(64 * NB_), 0, st, (const bf16*)qkv,
                                       (long)ld_qkv, (bf16*)out, (long)ld_out, lse, N, H, dh, sl2, drop_thresh,
                                       drop_scale, seed));
  return hip_check("attention_fwd_bf16");
}

extern "C" int fer_attention_bwd(int dtype, const void* qkv, int64_t ld_qkv, const void* out, int64_t ld_out,
                                 const void* dout, int64_t ld_dout, const float* lse, void* dqkv, int64_t ld_dqkv,
                                 float* ws, int64_t ws_bytes, int B, int N, int H, int dh, float scale,
                                 uint32_t drop_thresh, float drop_scale, uint64_t seed, fer_stream_t stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
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
    return hip_check("attention_bwd_f32");
  }
  if (N > 256 || dh > 64 || dh % 8) return set_error("attention_bwd(bf16): needs N <= 256, dh <= 64, dh % 8 == 0");
  if (ld_qkv % 8 || ld_out % 8 || ld_dout % 8 || ld_dqkv % 4) return set_error("attention_bwd(bf16): misaligned ld");
  const int nb = (N + 31) / 32;
  const float sl2 = scale * LOG2E;
  FER_NB_SWITCH(nb, hipLaunchKernelGGL(attn_bwd_bf16<NB_>, dim3(B * H), dim3(64 * NB_), 0, st, (const bf16*)qkv,
                                       (long)ld_qkv, (const bf16*)out, (long)ld_out, (const bf16*)dout, (long)ld_dout,
                                       lse, (bf16*)dqkv, (long)ld_dqkv, N, H, dh, scale, sl2, drop_thresh, drop_scale,
                                       seed));
  return hip_check("attention_bwd_bf16");
}
