// GEMM family for every Linear / Conv-as-GEMM on the FER-ViT hot path.
//
//   C[m][n] = epilogue( sum_k A(m,k) * B(n,k) )
//   A(m,k) = A[m*lda + k]  (A_KC, "K-contiguous")  or  A[k*lda + m]  (MN-contiguous)
//   B(n,k) = B[n*ldb + k]  (B_KC)                  or  B[k*ldb + n]
//
// The three nn.Linear passes map onto it without any transposed copies:
//   forward  Y  = X W^T      : A=X  (KC), B=W (KC)            (nn.Linear, `image_vit.py:101-113`)
//   dgrad    dX = dY W       : A=dY (KC), B=W (MN)
//   wgrad    dW = dY^T X     : A=dY (MN), B=X (MN), K = rows = B*N tokens (split-K)
//
// bf16 path: v_mfma_f32_16x16x32_bf16 (fp32 accumulate), 256x256x64 tiles on 4 waves (one
// per SIMD, 128x128 accumulators each), double-buffered LDS stages filled by LDS-DMA
// (buffer_load ... lds, 16 B/lane) one K-step ahead, fragment reads software-pipelined.
// The swizzle is applied on the per-lane SOURCE address (the DMA image is lane-linear):
//   KC image  [rows][64 k]  (128 B rows):  chunk' = chunk ^ ((row>>1)&7)
//   MN image  [64 k][rows]  (2*R B rows):  chunk' = chunk ^ (rho(k)<<1),
//                                          rho(k) = (k&3) | ((k>>3)&1)<<2
// KC fragments are read with ds_read_b128, MN fragments with two ds_read_b64_tr_b16
// (hardware transpose); both images are bank-conflict free for their reads.
// Out-of-range rows/cols/k (tails) are zero-filled by the buffer range check.
// The MFMA is issued with the B fragment as the instruction's A operand, so each
// lane ends with 4 consecutive n of one m (8/16-byte epilogue accesses).
//
// fp32 path (parity mode): a plain LDS-tiled VALU kernel with the same epilogue.
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "fervit_internal.h"

namespace fer {

// ------------------------------------------------------------------- epilogue
// bf16 tile epilogue on 8 consecutive columns (one 16-byte store per output row piece; the
// store issue rate, not bandwidth, bounds a tile's store tail). x = res[m][n..n+7] when e.res
// is set, else aux[m][n..n+7] (only when both are set is aux loaded here, a path no caller of
// the hot path takes). b0/b1 = bias of the 8 columns, ps = *post_scale, both loaded once.
FER_DEV f32x4 lo4(bf16x8 x) { return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]}; }
FER_DEV f32x4 hi4(bf16x8 x) { return f32x4{(float)x[4], (float)x[5], (float)x[6], (float)x[7]}; }
FER_DEV bf16x8 pack8(f32x4 a, f32x4 b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}
FER_DEV void epi8_bf16(const EpiArgs& e, long m, long n, f32x4& v0, f32x4& v1, f32x4 b0, f32x4 b1, bf16x8 x,
                       float ps, uint64_t seed) {
  const int act = e.act & 15;
  const bool gate = (e.act & FER_PRE_GATE) && e.pre;
  v0 = v0 * e.alpha + b0;
  v1 = v1 * e.alpha + b1;
  if (e.pre && !gate) *(bf16x8*)((bf16*)e.pre + m * e.ldp + n) = pack8(v0, v1);
  f32x4 g0 = f32x4{1.f, 1.f, 1.f, 1.f}, g1 = g0;  // gate act'(pre), when `pre` receives it
  if (act == FER_ACT_GELU) {
    if (gate) {
      f32x2 t;
      v0.xy = gelu_and_grad2(v0.xy, t); g0.xy = t;
      v0.zw = gelu_and_grad2(v0.zw, t); g0.zw = t;
      v1.xy = gelu_and_grad2(v1.xy, t); g1.xy = t;
      v1.zw = gelu_and_grad2(v1.zw, t); g1.zw = t;
    } else {
      v0.xy = gelu_erf_fast2(v0.xy);
      v0.zw = gelu_erf_fast2(v0.zw);
      v1.xy = gelu_erf_fast2(v1.xy);
      v1.zw = gelu_erf_fast2(v1.zw);
    }
  } else if (act == FER_ACT_RELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      g0[r] = v0[r] > 0.f ? 1.f : 0.f;
      g1[r] = v1[r] > 0.f ? 1.f : 0.f;
      v0[r] = fmaxf(v0[r], 0.f);
      v1[r] = fmaxf(v1[r], 0.f);
    }
  }
  if (e.drop_thresh) {
    const uint32_t idx = (uint32_t)m * (uint32_t)e.drop_ld + (uint32_t)n;
    const uint32_t k = keep4(seed, idx, e.drop_thresh) | (keep4(seed, idx + 4, e.drop_thresh) << 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v0[r] = (k >> r) & 1 ? v0[r] * e.drop_scale : 0.f;
      v1[r] = (k >> (4 + r)) & 1 ? v1[r] * e.drop_scale : 0.f;
      g0[r] = (k >> r) & 1 ? g0[r] * e.drop_scale : 0.f;
      g1[r] = (k >> (4 + r)) & 1 ? g1[r] * e.drop_scale : 0.f;
    }
  }
  if (gate) *(bf16x8*)((bf16*)e.pre + m * e.ldp + n) = pack8(g0, g1);
  if (e.post_scale) {
    v0 *= ps;
    v1 *= ps;
  }
  if (e.aux) {
    const bf16x8 a = e.res ? *(const bf16x8*)((const bf16*)e.aux + m * e.ldx + n) : x;
    const f32x4 a0 = lo4(a), a1 = hi4(a);
    if (e.aux_act == FER_ACT_MUL) {
      v0 *= a0;
      v1 *= a1;
    } else if (e.aux_act == FER_ACT_GELU) {
      v0.xy *= gelu_erf_grad2(a0.xy);
      v0.zw *= gelu_erf_grad2(a0.zw);
      v1.xy *= gelu_erf_grad2(a1.xy);
      v1.zw *= gelu_erf_grad2(a1.zw);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v0[r] *= act_grad(e.aux_act, a0[r]);
        v1[r] *= act_grad(e.aux_act, a1[r]);
      }
    }
  }
  if (e.res) {
    v0 += lo4(x);
    v1 += hi4(x);
  }
  if (e.c_f32) {
    float* c = (float*)e.c + m * e.ldc + n;
    if (e.accumulate) {
      v0 += *(const f32x4*)c;
      v1 += *(const f32x4*)(c + 4);
    }
    *(f32x4*)c = v0;
    *(f32x4*)(c + 4) = v1;
  } else {
    bf16* c = (bf16*)e.c + m * e.ldc + n;
    if (e.accumulate) {
      const bf16x8 o = *(const bf16x8*)c;
      v0 += lo4(o);
      v1 += hi4(o);
    }
    *(bf16x8*)c = pack8(v0, v1);
  }
}

// Epilogue kinds with the flags fixed at compile time (the 8-phase kernel's hot shapes): the
// generic epi8_bf16 tests every flag per row piece, and its branches and the register shuffles
// between them cost more issue slots than the arithmetic of the plain and residual epilogues.
// Same operations in the same order as epi8_bf16, so the results are bit-identical.
enum { EPI_GEN = 0, EPI_STORE = 1, EPI_GATE = 2, EPI_RES = 3, EPI_MUL = 4, EPI_RES2 = 5, EPI_MUL2 = 6, EPI_GATER = 7 };
//   EPI_STORE: c = alpha*acc + bias                                   (qkv fwd, out-proj dgrad)
//   EPI_GATE : c = drop(gelu(v)), pre = drop(gelu'(v)), v = alpha*acc + bias      (fc1 fwd)
//   EPI_GATER: c = drop(relu(v)), pre = drop(v > 0)              (fc1 fwd of the ReLU encoders)
//   EPI_RES  : c = drop(alpha*acc + bias) + res                (out-proj / fc2 fwd, dgrad + res)
//   EPI_MUL  : c = (alpha*acc + bias) * aux                      (fc2 dgrad through the gate)
// (bf16 c without accumulate, no post_scale; dropout is a run-time choice in GATE and RES)
// EPI_RES2 / EPI_MUL2: the same arithmetic as RES / MUL; the tile epilogue loads the row operand
// straight into registers instead of LDS, which frees the LDS for two staging areas.
constexpr int epi_base(int S) { return S == EPI_RES2 ? EPI_RES : (S == EPI_MUL2 ? EPI_MUL : S); }
// Keep bits of 8 consecutive elements from an even index (4 hashes), as compares: the same
// decisions as keep4 (u16 >= thr; the high half as h >= thr << 16) without packing them into an
// integer and testing its bits again per element.
FER_DEV void keep8(uint64_t seed, uint32_t idx, uint32_t thr, bool (&kp)[8]) {
  const uint32_t thr_hi = thr << 16;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t h = fer_hash(seed, (idx >> 1) + q);
    kp[2 * q] = (h & 0xFFFFu) >= thr;
    kp[2 * q + 1] = h >= thr_hi;
  }
}

// keep8 for idx % 8 == 0 (the fixed kinds: 8-column pieces at n % 8 == 0, drop_ld % 8 == 0 checked by
// epi_kind): the pair index p = idx / 2 is then a multiple of 4, so hash q's counter (p + q) ^ lo equals
// (p ^ lo) ^ q -- one xor-add per hash instead of an add, a xor and an add. Same decisions as keep8.
FER_DEV void keep8a(uint64_t seed, uint32_t idx, uint32_t thr, bool (&kp)[8]) {
  const uint32_t thr_hi = thr << 16, a = (idx >> 1) ^ (uint32_t)seed, hi = (uint32_t)(seed >> 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t lo;
    const uint32_t x = fer_mix_pre((a ^ (uint32_t)q) + hi, lo);
    kp[2 * q] = lo >= thr;
    kp[2 * q + 1] = x >= thr_hi;
  }
}

template <int S0>
FER_DEV void epi8_t(const EpiArgs& e, long m, long n, f32x4& v0, f32x4& v1, f32x4 b0, f32x4 b1, bf16x8 x,
                    float ps, uint64_t seed) {
  constexpr int S = epi_base(S0);
  if constexpr (S == EPI_GEN) {
    epi8_bf16(e, m, n, v0, v1, b0, b1, x, ps, seed);
  } else {
    v0 = v0 * e.alpha + b0;
    v1 = v1 * e.alpha + b1;
    if constexpr (S == EPI_GATE) {
      f32x4 g0, g1;
      f32x2 t;
      f32x2 xs[4] = {v0.xy, v0.zw, v1.xy, v1.zw}, gs[4];
      gelu_and_grad8(xs, gs);
      v0.xy = xs[0]; v0.zw = xs[1]; v1.xy = xs[2]; v1.zw = xs[3];
      g0.xy = gs[0]; g0.zw = gs[1]; g1.xy = gs[2]; g1.zw = gs[3];
      (void)t;
      if (e.drop_thresh) {
        bool kp[8];
        keep8(seed, (uint32_t)m * (uint32_t)e.drop_ld + (uint32_t)n, e.drop_thresh, kp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v0[r] = kp[r] ? v0[r] * e.drop_scale : 0.f;
          v1[r] = kp[4 + r] ? v1[r] * e.drop_scale : 0.f;
          g0[r] = kp[r] ? g0[r] * e.drop_scale : 0.f;
          g1[r] = kp[4 + r] ? g1[r] * e.drop_scale : 0.f;
        }
      }
      *(bf16x8*)((bf16*)e.pre + m * e.ldp + n) = pack8(g0, g1);
    }
    if constexpr (S == EPI_RES) {
      if (e.drop_thresh) {
        bool kp[8];
        keep8(seed, (uint32_t)m * (uint32_t)e.drop_ld + (uint32_t)n, e.drop_thresh, kp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v0[r] = kp[r] ? v0[r] * e.drop_scale : 0.f;
          v1[r] = kp[4 + r] ? v1[r] * e.drop_scale : 0.f;
        }
      }
      v0 += lo4(x);
      v1 += hi4(x);
    }
    if constexpr (S == EPI_MUL) {
      v0 *= lo4(x);
      v1 *= hi4(x);
    }
    *(bf16x8*)((bf16*)e.c + m * e.ldc + n) = pack8(v0, v1);
  }
}

// The fixed kinds with the row addressing done by the caller (element offsets oc / op into c / pre
// and the dropout index di, advanced by adds per row instead of a 64-bit multiply per store) and
// the dropout scale folded into constants: GATE takes it in the GELU constants (gelu_and_grad8s),
// RES as acc * (alpha*s) + b*s (ab = alpha*s, b0 / b1 pre-scaled by the caller), so a dropped
// element costs a select only.
// Returns the output row piece; GATE / GATER also the pre-activation gate piece (`gp`). The caller
// stores them (pointer stores behind the row check in the shared staged loop -- buffer stores there
// made the 128^2 kernel's STORE / MUL kinds 50-80 % slower on the latent shapes, profiles/r04z_* --
// buffer stores with FER_OOB rows in the 8-phase kernel's register-fed and wave-private paths).
template <int S0, typename E>
FER_DEV bf16x8 epi8_k(const E& e, uint32_t di, f32x4& v0, f32x4& v1, f32x4 b0, f32x4 b1, bf16x8 x,
                      uint64_t seed, float ab, f32x2 ghs, f32x2 gps, float dsr, bf16x8& gp) {
  constexpr int S = epi_base(S0);
  static_assert(S != EPI_GEN, "generic epilogue goes through epi8_t");
  v0 = v0 * ab + b0;
  v1 = v1 * ab + b1;
  if constexpr (S == EPI_GATER) {  // scale folded into ab / b (relu(x) * s = relu(x * s), s > 0)
    f32x4 g0, g1;
    bool kp[8];
    if (e.drop_thresh) keep8a(seed, di, e.drop_thresh, kp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool k0 = e.drop_thresh ? kp[r] : true, k1 = e.drop_thresh ? kp[4 + r] : true;
      g0[r] = (k0 && v0[r] > 0.f) ? dsr : 0.f;
      g1[r] = (k1 && v1[r] > 0.f) ? dsr : 0.f;
      v0[r] = k0 ? fmaxf(v0[r], 0.f) : 0.f;
      v1[r] = k1 ? fmaxf(v1[r], 0.f) : 0.f;
    }
    gp = pack8(g0, g1);
  }
  if constexpr (S == EPI_GATE) {
    f32x4 g0, g1;
    f32x2 xs[4] = {v0.xy, v0.zw, v1.xy, v1.zw}, gs[4];
    gelu_and_grad8s(xs, gs, ghs, gps);
    v0.xy = xs[0]; v0.zw = xs[1]; v1.xy = xs[2]; v1.zw = xs[3];
    g0.xy = gs[0]; g0.zw = gs[1]; g1.xy = gs[2]; g1.zw = gs[3];
    if (e.drop_thresh) {
      bool kp[8];
      keep8a(seed, di, e.drop_thresh, kp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v0[r] = kp[r] ? v0[r] : 0.f;
        v1[r] = kp[4 + r] ? v1[r] : 0.f;
        g0[r] = kp[r] ? g0[r] : 0.f;
        g1[r] = kp[4 + r] ? g1[r] : 0.f;
      }
    }
    gp = pack8(g0, g1);
  }
  if constexpr (S == EPI_RES) {
    if (e.drop_thresh) {
      bool kp[8];
      keep8a(seed, di, e.drop_thresh, kp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v0[r] = kp[r] ? v0[r] : 0.f;
        v1[r] = kp[4 + r] ? v1[r] : 0.f;
      }
    }
    v0 += lo4(x);
    v1 += hi4(x);
  }
  if constexpr (S == EPI_MUL) {
    v0 *= lo4(x);
    v1 *= hi4(x);
  }
  return pack8(v0, v1);
}
// epi8_k + buffer stores at byte offsets ocb / opb (FER_OOB for a row out of range: dropped without a
// branch, so the compiler's wait counts around them stay exact)
template <int S0, typename E>
FER_DEV void epi8_kb(const E& e, uint32_t ocb, uint32_t opb, uint32_t di, f32x4& v0, f32x4& v1, f32x4 b0,
                     f32x4 b1, bf16x8 x, uint64_t seed, float ab, f32x2 ghs, f32x2 gps, float dsr,
                     const __amdgpu_buffer_rsrc_t& rc, const __amdgpu_buffer_rsrc_t& rp) {
  constexpr int S = epi_base(S0);
  bf16x8 gp;
  const bf16x8 o = epi8_k<S0>(e, di, v0, v1, b0, b1, x, seed, ab, ghs, gps, dsr, gp);
  if constexpr (S == EPI_GATE || S == EPI_GATER)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, gp), rp, opb, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rc, ocb, 0, 0);
}

// kind for a launch (EPI_GEN unless every flag matches one of the fixed kinds)
// The fixed kinds address c / pre / res / aux through 32-bit buffer offsets (out-of-range rows at
// FER_OOB): each operand must span less than 2 GiB, else the generic epilogue runs.
static inline bool epi_span_ok(const void* p, long ld, long M, long N) {
  return !p || ((M - 1) * ld + N) * 2 < 0x7FFFFFF0L;
}
static inline int epi_kind(const EpiArgs& e, long M, long N) {
  if (e.c_f32 || e.accumulate || e.post_scale) return EPI_GEN;
  if (e.drop_thresh && (e.drop_ld & 7)) return EPI_GEN;  // keep8a's index alignment
  if (!epi_span_ok(e.c, e.ldc, M, N) || !epi_span_ok(e.pre, e.ldp, M, N) || !epi_span_ok(e.res, e.ldr, M, N) ||
      !epi_span_ok(e.aux, e.ldx, M, N))
    return EPI_GEN;
  const int act = e.act & 15;
  const bool gate = (e.act & FER_PRE_GATE) && e.pre;
  if (gate) {
    if (e.aux || e.res || e.colsum) return EPI_GEN;
    return act == FER_ACT_GELU ? EPI_GATE : (act == FER_ACT_RELU ? EPI_GATER : EPI_GEN);
  }
  if (e.pre || act) return EPI_GEN;
  if (e.aux) return (e.aux_act == FER_ACT_MUL && !e.res && !e.drop_thresh) ? EPI_MUL2 : EPI_GEN;
  if (e.colsum) return EPI_GEN;
  if (e.res) return EPI_RES2;
  return e.drop_thresh ? EPI_GEN : EPI_STORE;
}

template <typename T>
FER_DEV void epi4(const EpiArgs& e, long m, long n, f32x4 v, uint64_t seed) {
  const int act = e.act & 15;
  const bool gate = (e.act & FER_PRE_GATE) && e.pre;
  v *= e.alpha;
  if (e.bias) v += *(const f32x4*)(e.bias + n);
  if (e.pre && !gate) store4<T>((T*)e.pre + m * e.ldp + n, v);
  f32x4 gt = f32x4{1.f, 1.f, 1.f, 1.f};
  if (act) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (gate) gt[r] = act_grad(act, v[r]);
      v[r] = act_fwd(act, v[r]);
    }
  }
  if (e.drop_thresh) {
    const uint32_t k = keep4(seed, (uint32_t)m * (uint32_t)e.drop_ld + (uint32_t)n, e.drop_thresh);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = (k >> r) & 1 ? v[r] * e.drop_scale : 0.f;
      gt[r] = (k >> r) & 1 ? gt[r] * e.drop_scale : 0.f;
    }
  }
  if (gate) store4<T>((T*)e.pre + m * e.ldp + n, gt);
  if (e.post_scale) v *= *e.post_scale;
  if (e.aux) {
    f32x4 a = load4<T>((const T*)e.aux + m * e.ldx + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= act_grad(e.aux_act, a[r]);
  }
  if (e.res) v += load4<T>((const T*)e.res + m * e.ldr + n);
  if (e.c_f32) {
    float* c = (float*)e.c + m * e.ldc + n;
    if (e.accumulate) v += *(const f32x4*)c;
    *(f32x4*)c = v;
  } else {
    T* c = (T*)e.c + m * e.ldc + n;
    if (e.accumulate) v += load4<T>(c);
    store4<T>(c, v);
  }
}

// ------------------------------------------------------------ tile scheduling
// XCD-aware, bijective remap (blocks b and b+8 share an XCD under round-robin
// dispatch) followed by GROUP_M-row grouping for L2 reuse of both panels.
FER_DEV void tile_of(int bid, int tiles_m, int tiles_n, int& tm, int& tn, int group = 8) {
  const int nwg = tiles_m * tiles_n;
  int wgid = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int GROUP = group;
  const int per_group = GROUP * tiles_n;
  const int g = wgid / per_group;
  const int first = g * GROUP;
  const int gsize = min(tiles_m - first, GROUP);
  const int w = wgid - g * per_group;
  tm = first + w % gsize;
  tn = w / gsize;
}

// Split-K launches (grid = tiles x splits): XCD-aware (split, tile) assignment. Blocks are dealt to
// the XCDs round-robin by linear id (ids l and l + 8 share an XCD), so each XCD is given a
// contiguous chunk of the split-major item list (split ks, tile t): the tiles of one split, which
// read the same K rows of both operands in lockstep -- served by that XCD's L2 instead of once per
// tile from the fabric (a weight gradient's A rows are shared by its tiles_n tiles, its B rows by
// its tiles_m tiles). With the plain blockIdx.y = split order every XCD held tiles of every split.
FER_DEV void split_tile_of(int tiles_m, int tiles_n, int& tm, int& tn, int& ks) {
  const int T = tiles_m * tiles_n;
  const int items = T * (int)gridDim.y;
  const int lin = (int)blockIdx.y * (int)gridDim.x + (int)blockIdx.x;
  const int xcd = lin & 7, q = items >> 3, r = items & 7;
  const int item = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
  ks = item / T;
  const int t = item - ks * T;
  tm = t % tiles_m;
  tn = t / tiles_m;
}

// ------------------------------------------------------------- LDS-DMA stage
constexpr int BK = 64;
// KC image [rows][BKT k] (2*BKT-byte rows). BKT=64: chunk ^= (row>>1)&7. BKT=32 (4 rows per
// 256 B): chunk ^= s(row>>2) with s = 0,0,2,2,1,1,3,3 — conflict-free for the ds_read_b128
// lane groups of both the 32x32 (16 rows, one chunk) and 16x16 (rows x 2 chunks) reads.
template <int BKT> FER_DEV int kc_swz(int row) {
  if constexpr (BKT == 64) return (row >> 1) & 7;
  else return (((row >> 3) & 1) << 1) | ((row >> 4) & 1);
}

// Per-lane DMA source offsets of this wave's pieces, computed once per tile; an
// out-of-range row/column gets base FER_OOB so voffset = base + k-advance stays out of range
// (one add per piece per K-step). For KC the K-step adds k0*2 bytes, for MN the wave-uniform
// k0*ld*2. `kof` (the lane's K inside the stage) is checked only on a partial last K-step.
// MN tr-read image swizzle (16-byte chunk XOR by K row), see read_frag.
template <int MT> FER_DEV int mn_swz_t(int k) {
  if constexpr (MT == 32) return (k & 3) << 2;               // 4 rows x 64 B per 32-lane half
  else return ((k & 3) | (((k >> 3) & 1) << 2)) << 1;       // 8 rows x 32 B per 32-lane half
}

template <int R, bool KC, int NW, int MT, int BKT = BK>
struct DmaPlan {
  static constexpr int NI = R * BKT * 2 / 1024 / NW;
  static_assert(NI * NW * 1024 == R * BKT * 2, "tile/wave mismatch");
  uint32_t base[NI];
  int kof[NI];
  FER_DEV void init(int wave, int lane, long ld, int r0, int rmax) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int gi = wave * NI + i;
      bool ok;
      uint32_t off;
      if constexpr (KC) {
        constexpr int CPR = BKT / 8;  // 16-byte chunks per row
        const int row = gi * (64 / CPR) + lane / CPR;
        const int c = (lane % CPR) ^ kc_swz<BKT>(row);
        const int gr = r0 + row;
        ok = gr < rmax;
        kof[i] = c * 8;
        off = (uint32_t)(((long)gr * ld + c * 8) * 2);
      } else {
        constexpr int RB = R * 2;
        const int byte = gi * 1024 + lane * 16;
        const int k = byte / RB;
        const int c = ((byte % RB) >> 4) ^ mn_swz_t<MT>(k);
        const int gc = r0 + c * 8;
        ok = gc < rmax;
        kof[i] = k;
        off = (uint32_t)(((long)k * ld + gc) * 2);
      }
      base[i] = ok ? off : FER_OOB;
    }
  }
  // Inline-asm DMA (common.h dma16_asm): with the builtin, the compiler's wait-count pass put an
  // s_waitcnt vmcnt(0) in front of the fragment reads of every K-step of the MN-operand kernels (it
  // cannot tell a ds_read_b64_tr_b16 from the DMA's target), i.e. waited for the stages still in
  // flight. The issuing waves' counted waits (wait_vm) stay as they are. Measured neutral (fc1 weight
  // gradient alone 275.7 vs 274.1 us, the step 35.97-36.11 vs 36.01-36.08 ms on one box:
  // profiles/r04aj_asm_dma_gemm_ab.txt, r04ak_asm_dma_step_ab.txt): two stages in flight already
  // covered the DMA latency; kept so the prefetch depth is the one the code states.
  FER_DEV void issue(const u32x4& rs, char* lds_tile, int wave, long ld, int k0, int kmax, bool tail) const {
    const uint32_t kadd = KC ? (uint32_t)(k0 * 2) : (uint32_t)(k0 * ld * 2);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t voff = (!tail || k0 + kof[i] < kmax) ? base[i] + kadd : FER_OOB;
      dma16_asm(lds_tile + (wave * NI + i) * 1024, rs, voff);
    }
  }
};

// MFMA operand fragments. MT = 32: v_mfma_f32_32x32x16_bf16, lane l holds index i0 + (l&31),
// k = 16kk + 8(l>>5) + j. MT = 16: v_mfma_f32_16x16x32_bf16, lane l holds index i0 + (l&15),
// k = 32kk + 8(l>>4) + j (j = 0..7). KC images are read with ds_read_b128, MN images with two
// ds_read_b64_tr_b16 (rows k..k+3 and k+4..k+7 of 16 consecutive indices).

template <int MT, int R, bool KC, int BKT = BK>
FER_DEV bf16x8 read_frag(const char* lds_tile, int i0, int kk, int lane) {
  if constexpr (KC) {
    const int row = i0 + (MT == 32 ? (lane & 31) : (lane & 15));
    const int ch = MT == 32 ? 2 * kk + (lane >> 5) : 4 * kk + (lane >> 4);
    return *(const bf16x8*)(lds_tile + row * (BKT * 2) + ((ch ^ kc_swz<BKT>(row)) << 4));
  } else {
    constexpr int RB = R * 2;
    const int gg = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    int k1, c;
    if constexpr (MT == 32) {
      k1 = 16 * kk + 8 * (gg >> 1) + q;
      c = ((i0 + 16 * (gg & 1)) >> 3) + (p >> 1);
    } else {
      k1 = 32 * kk + 8 * gg + q;
      c = (i0 >> 3) + (p >> 1);
    }
    const int k2 = k1 + 4;
    const char* a1 = lds_tile + k1 * RB + ((c ^ mn_swz_t<MT>(k1)) << 4) + (p & 1) * 8;
    const char* a2 = lds_tile + k2 * RB + ((c ^ mn_swz_t<MT>(k2)) << 4) + (p & 1) * 8;
    short4_t t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a1);
    short4_t t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)a2);
    return cat8(t1, t2);
  }
}

template <int MT> struct Acc;
template <> struct Acc<32> { typedef f32x16 T; };
template <> struct Acc<16> { typedef f32x4 T; };

template <int MT>
FER_DEV typename Acc<MT>::T mfma(bf16x8 a, bf16x8 b, typename Acc<MT>::T c) {
  if constexpr (MT == 32) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

#ifdef FER_GEMM_STAMPS
// diagnostic build only: s_memtime at the epilogue's stage boundaries (lane 0 of waves 0 and 4 of
// workgroup 0; the last tile's values remain)
__device__ unsigned long long g_epst[2][16];
#define EP_STAMP(i)                                                          \
  do {                                                                       \
    if (ep_on) {                                                             \
      unsigned long long t_;                                                 \
      __builtin_amdgcn_sched_barrier(0);                                     \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                     \
      if (lane == 0) g_epst[(tid_ >> 6) >> 2][i] = t_;                       \
    }                                                                        \
  } while (0)
#else
#define EP_STAMP(i) do {} while (0)
#endif

// ---- epilogue. Every workgroup barrier in the epilogue (and between the tiles of a persistent
// workgroup) is bar_lds (lgkmcnt(0) + s_barrier): the barriers order LDS staging only. (With no
// LDS-DMA in flight hipcc lowers __syncthreads to the same two instructions; bar_lds makes sure no
// vmcnt(0) -- a wait for every earlier output store -- can appear there.)
// Accumulator element (i, j, q, r) -> tile row/col. Split-K partials go to
// the fp32 slab; otherwise each wave-row half of the tile (in EPC row chunks) is staged
// through LDS as fp32 with padded rows and every thread applies the epilogue on 4 consecutive
// columns of one row: all global traffic of the epilogue is row-contiguous.
template <int BM, int BN, int WM, int WN, int MT, int EPC, int SMEMB, int EK = EPI_GEN, typename AccT, int FN, int FM>
FER_DEV void tile_epilogue(const GemmArgs& g, const EpiArgs& e, AccT (&acc)[FN][FM], char* smem, int m0, int n0,
                           int ks, int wm, int wn, int lane, uint64_t seed) {
  int tid_ = threadIdx.x;  // laundered: not hoisted out of a persistent tile loop
  asm volatile("" : "+v"(tid_));
#ifdef FER_GEMM_STAMPS
  const bool ep_on = blockIdx.x == 0 && ks == 0 && ((tid_ >> 6) & 3) == 0;
#endif
  EP_STAMP(0);
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int NQ = MT == 32 ? 4 : 1;
  const int lr = MT == 32 ? (lane & 31) : (lane & 15);
  const int lc = MT == 32 ? 4 * (lane >> 5) : 4 * (lane >> 4);
  if (g.partial) {  // split-K partial slab, fp32 [split][M][N] (reduced by splitk_reduce_kernel)
    float* ws = g.ws + (long)ks * g.M * g.N;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const long m = m0 + wm * TM + j * MT + lr, n = n0 + wn * TN + i * MT + 8 * q + lc;
          if (m < g.M && n < g.N)
            *(f32x4*)(ws + m * g.N + n) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        }
    return;
  }
  static_assert(WM == 2, "epilogue staging splits the tile by the wave-row halves");
  static_assert(EPC == 1 || EPC == 2, "chunk pairing assumes 1 or 2 chunks per wave-row half");
  constexpr int EROWS = TM / EPC, FJ = FM / EPC;  // rows per chunk; MFMA row blocks per chunk
  static_assert(FJ * EPC == FM, "row chunks must split the MFMA blocks evenly");
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int C8 = BN / 8;                     // 8-column groups per row
  static_assert(NT % C8 == 0, "each thread keeps one column group for the whole tile");
  constexpr int RPI = NT / C8, IT = EROWS / RPI;  // rows per pass, passes per chunk
  static_assert(IT * RPI == EROWS, "chunk rows must split evenly over the passes");
  // LDS: [staging: EROWS x BN fp32, 16-byte chunks XOR-swizzled by (row & 7)]
  //      [X0 | X1: EROWS x BN bf16 each, the chunk's residual / aux rows]
  constexpr int SROW = BN * 4, XBYTES = EROWS * BN * 2;
  constexpr int NP = XBYTES / 1024, PPW = NP / NW;     // 1 KB DMA pieces per chunk / per wave
  constexpr int RPP = 1024 / (BN * 2), LPR = BN / 8;   // rows per piece, lanes per row
  static_assert(PPW * NW == NP && RPP * LPR == 64, "X tile must split into whole 1 KB pieces per wave");
  static_assert(EROWS * SROW + 2 * XBYTES <= SMEMB, "epilogue staging + X buffers exceed the kernel's LDS");
  char* const stg = smem;
  char* const xb = smem + EROWS * SROW;
  auto swz = [](int row, int col) { return row * SROW + ((((col >> 2) ^ (row & 7))) << 4); };

  // Each thread owns 4 consecutive columns for the whole tile (bias loaded once) and rows
  // tr + RPI*it of every chunk. The residual / aux rows ("x") of chunk h+1 are brought into
  // LDS by LDS-DMA while chunk h is processed. vmcnt retires loads, stores and DMA in issue
  // order, so each DMA is issued BEFORE the previous chunk's stores... and waited for with a
  // count that skips exactly those stores; the item loop itself never waits on memory.
  const int tc = (tid_ % C8) * 8, tr = tid_ / C8;
  const int wave = tid_ >> 6;
  const long n = n0 + tc;
  const bool nok = n < g.N;  // N % 8 == 0 on this path (checked by the host)
  f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (e.bias && nok) {
    b0 = ldg_f32x4(e.bias + n);
    b1 = ldg_f32x4(e.bias + n + 4);
  }
  const float ps = e.post_scale ? *e.post_scale : 1.f;
  // fixed kinds (epi8_k): dropout scale folded into the bias / alpha (RES) or the GELU constants (GATE)
  constexpr bool KIND = EK != EPI_GEN;
  constexpr bool CS = !KIND || epi_base(EK) == EPI_MUL;  // only these kinds carry fused column sums
  const float dsc = e.drop_thresh ? e.drop_scale : 1.f;
  const float ab = (epi_base(EK) == EPI_RES || EK == EPI_GATER) ? e.alpha * dsc : e.alpha;
  if constexpr (epi_base(EK) == EPI_RES || EK == EPI_GATER) {
    b0 *= dsc;
    b1 *= dsc;
  }
  const f32x2 ghs = f32x2(0.5f * dsc), gps = f32x2(0.39894228040143268f * dsc);  // GATE: gelu_and_grad8s
  const void* xs = e.res ? e.res : e.aux;  // the row operand brought in by DMA
  const long ldxs = e.res ? e.ldr : e.ldx;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(xs), rc = make_rsrc(e.c), rp = make_rsrc(e.pre ? e.pre : e.c);
  (void)rp;
  // this lane's DMA source for piece k of chunk 0 (rows advance by EROWS per chunk)
  const int xrow = lane / LPR, xcol = (lane % LPR) * 8;
  const bool xcol_ok = n0 + xcol + 8 <= g.N;
  auto issue_x = [&](int h) {
    char* dst = xb + (h & 1) * XBYTES;
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const int piece = wave * PPW + k;
      const long m = m0 + h * EROWS + piece * RPP + xrow;
      const uint32_t voff = (xcol_ok && m < g.M) ? (uint32_t)((m * ldxs + n0 + xcol) * 2) : FER_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)(dst + piece * 1024), 16, voff, 0, 0, 0);
    }
  };
  // Stores per wave per chunk when every row of the tile is in range (else a full drain).
  const bool full = m0 + BM <= g.M && !e.accumulate && !(e.res && e.aux);
  const int spc = full ? IT * (e.pre ? 2 : 1) : -1;
  auto wait_x = [&](int pending) {  // wait until the DMA of the current chunk has landed
    switch (pending) {
      case 0: wait_vm<0>(); break;
      case 4: wait_vm<4>(); break;
      case 8: wait_vm<8>(); break;
      case 12: wait_vm<12>(); break;
      case 16: wait_vm<16>(); break;
      case 20: wait_vm<20>(); break;
      default: wait_vm<0>(); break;
    }
  };
  auto stage = [&](int h, int half, int sub) {
    bar_lds();  // every wave is done with the staging area and with X[(h+1)&1]
    const bool more = h + 1 < 2 * EPC;
    if (xs && more) issue_x(h + 1);
    if (wm == half) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int jj = 0; jj < FJ; ++jj)
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int j = sub * FJ + jj;
            *(f32x4*)(stg + swz(jj * MT + lr, wn * TN + i * MT + 8 * q + lc)) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          }
    }
    if (xs) {
      const int after = (more ? PPW : 0) + (h > 0 ? spc : 0);
      wait_x(spc < 0 ? 0 : after);
    }
    bar_lds();  // staging and X[h&1] (all waves' DMA) visible
  };
  f32x4 cs0 = f32x4{0.f, 0.f, 0.f, 0.f}, cs1 = cs0;  // fused column sums of this thread's rows
  auto finish = [&](int h, const char* stg) {
    const char* xh = xb + (h & 1) * XBYTES;
    const long mr = m0 + h * EROWS + tr;  // this thread's first row of the chunk
    long oc = mr * e.ldc + n, op = mr * e.ldp + n;
    uint32_t di = (uint32_t)mr * (uint32_t)e.drop_ld + (uint32_t)n;
#pragma unroll 1
    for (int it = 0; it < IT; ++it) {
      const int r = tr + it * RPI;
      const long m = m0 + h * EROWS + r;
      f32x4 v0 = *(const f32x4*)(stg + swz(r, tc)), v1 = *(const f32x4*)(stg + swz(r, tc + 4));
      const bf16x8 x = xs ? *(const bf16x8*)(xh + (r * BN + tc) * 2) : bf16x8{};
      if (nok && m < g.M) {
        if constexpr (KIND) {
          bf16x8 gp;
          const bf16x8 o = epi8_k<EK>(e, di, v0, v1, b0, b1, x, seed, ab, ghs, gps, dsc, gp);
          if constexpr (epi_base(EK) == EPI_GATE || EK == EPI_GATER) *(bf16x8*)((bf16*)e.pre + op) = gp;
          *(bf16x8*)((bf16*)e.c + oc) = o;
        } else {
          epi8_t<EK>(e, m, n, v0, v1, b0, b1, x, ps, seed);
        }
        if constexpr (CS) {
          cs0 += v0;
          cs1 += v1;
        }
      }
      oc += RPI * e.ldc;
      op += RPI * e.ldp;
      di += (uint32_t)RPI * (uint32_t)e.drop_ld;
    }
  };
  if constexpr ((EK == EPI_RES2 || EK == EPI_MUL2) && EPC == 2 && 2 * EROWS * SROW <= SMEMB) {
    // row operand in registers: this thread's 2 x IT rows of a round are loaded before the round's
    // staging (round 0's at entry, round 1's once round 0's accumulators are in LDS), so they fly
    // during the staging and the other round; loads issued before the stores retire first (vmcnt)
    const bf16* xg = (const bf16*)xs;
    // branch-free: out-of-range rows load zeros / drop their stores through FER_OOB offsets, so the
    // compiler counts the round's loads exactly instead of draining every store before their use
    const uint32_t ldxb = (uint32_t)ldxs * 2, ldcb = (uint32_t)e.ldc * 2;
    auto load_x = [&](int p, bf16x8 (&xr)[2 * IT]) {
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        const long m = m0 + ((k / IT) * EPC + p) * EROWS + tr + (k % IT) * RPI;
        const uint32_t off = (nok && m < g.M) ? (uint32_t)m * ldxb + (uint32_t)n * 2 : FER_OOB;
        xr[k] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
      }
    };
    auto finish_x = [&](int h, const char* stg, const bf16x8* xr) {
      f32x4 v0 = *(const f32x4*)(stg + swz(tr, tc)), v1 = *(const f32x4*)(stg + swz(tr, tc + 4));
      const long mr = m0 + h * EROWS + tr;
      const uint32_t di0 = (uint32_t)mr * (uint32_t)e.drop_ld + (uint32_t)n;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int r = tr + it * RPI;
        const long m = m0 + h * EROWS + r;
        f32x4 n0 = v0, n1 = v1;
        if (it + 1 < IT) {
          n0 = *(const f32x4*)(stg + swz(r + RPI, tc));
          n1 = *(const f32x4*)(stg + swz(r + RPI, tc + 4));
        }
        const bool ok = nok && m < g.M;
        epi8_kb<EK>(e, ok ? (uint32_t)m * ldcb + (uint32_t)n * 2 : FER_OOB, FER_OOB,
                   di0 + (uint32_t)(it * RPI) * (uint32_t)e.drop_ld, v0, v1, b0, b1, xr[it], seed, ab, ghs, gps, dsc,
                   rc, rp);
        if constexpr (CS) {  // no select: out-of-range rows multiply by zeros (x through FER_OOB), as in tile_epilogue_wp
          cs0 += v0;
          cs1 += v1;
        }
        v0 = n0;
        v1 = n1;
      }
    };
    auto put = [&](auto sub) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int jj = 0; jj < FJ; ++jj)
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int j = decltype(sub)::value * FJ + jj;
            *(f32x4*)(stg + wm * (EROWS * SROW) + swz(jj * MT + lr, wn * TN + i * MT + 8 * q + lc)) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          }
    };
    // both rounds' rows are issued up front (round 1's before round 0's stores: vmcnt retires in
    // issue order, so a load issued after the stores would wait for them)
    bf16x8 xr[2 * IT], xr1[2 * IT];
    load_x(0, xr);
    load_x(1, xr1);
    bar_lds();
    put(std::integral_constant<int, 0>{});
    bar_lds();
    EP_STAMP(1);
    finish_x(0, stg, xr);
    EP_STAMP(2);
    finish_x(EPC, stg + EROWS * SROW, xr + IT);
    EP_STAMP(3);
    bar_lds();
    put(std::integral_constant<int, 1>{});
    bar_lds();
    EP_STAMP(5);
    finish_x(1, stg, xr1);
    EP_STAMP(6);
    finish_x(EPC + 1, stg + EROWS * SROW, xr1 + IT);
    EP_STAMP(7);
    EP_STAMP(4);
    EP_STAMP(8);
  } else if constexpr ((EK == EPI_STORE || EK == EPI_GATE || EK == EPI_GATER) && EPC == 2 &&
                       2 * EROWS * SROW <= SMEMB) {
    // no row operand: the X buffers' LDS holds a second staging area, so both wave-row halves
    // stage a chunk at once (all waves write, two barrier rounds instead of four); chunk sub p of
    // half w is tile chunk h = 2w + p (rows 64h..64h+63)
#pragma unroll 1
    for (int p = 0; p < EPC; ++p) {
      bar_lds();  // every wave is done with both staging areas
      // accumulator indices must be compile-time constants (a run-time p would index the
      // accumulator array dynamically: scratch)
      auto put = [&](auto sub) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int jj = 0; jj < FJ; ++jj)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              const int j = decltype(sub)::value * FJ + jj;
              *(f32x4*)(stg + wm * (EROWS * SROW) + swz(jj * MT + lr, wn * TN + i * MT + 8 * q + lc)) =
                  f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
            }
      };
      if (p == 0) put(std::integral_constant<int, 0>{});
      else put(std::integral_constant<int, 1>{});
      bar_lds();
      EP_STAMP(1 + 4 * p);
      finish(p, stg);
      EP_STAMP(2 + 4 * p);
      finish(EPC + p, stg + EROWS * SROW);
      EP_STAMP(3 + 4 * p);
      EP_STAMP(4 + 4 * p);
    }
  } else {
    // The X buffers overlap the main loop's last operand stage: every wave must be done reading its
    // fragments before the first row-operand DMA lands there. (Without this barrier a fast wave's DMA
    // overwrote 8 A rows a slower wave was still reading: one 8-row band of a tile wrong, about 1 in 40
    // launches of the 128^2 residual GEMM, profiles/r05_store_war_gemm128_stress_before.txt.)
    if (xs) {
      bar_lds();
      issue_x(0);
    }
#pragma unroll 1
    for (int p = 0; p < EPC; ++p) {
      const int h0 = 2 * p, h1 = 2 * p + 1;
      stage(h0, h0 / EPC, 0);
      EP_STAMP(1 + 4 * p);
      finish(h0, stg);
      EP_STAMP(2 + 4 * p);
      stage(h1, h1 / EPC, EPC == 2 ? 1 : 0);
      EP_STAMP(3 + 4 * p);
      finish(h1, stg);
      EP_STAMP(4 + 4 * p);
    }
  }
  if (g.cs_part) {  // column partial sums of this tile -> cs_part[tile row][n], fixed order
    bar_lds();  // staging area free
    float* red = (float*)smem;  // [RPI][BN]
    *(f32x4*)(red + tr * BN + tc) = cs0;
    *(f32x4*)(red + tr * BN + tc + 4) = cs1;
    bar_lds();
    for (int c = tid_; c < BN; c += NT) {
      float t = 0.f;
      for (int r = 0; r < RPI; ++r) t += red[r * BN + c];
      if (n0 + c < g.N) g.cs_part[(long)(m0 / BM) * g.N + n0 + c] = t;
    }
  }
}

// Wave grid WM x WN over a BM x BN tile; each wave owns (BM/WM) x (BN/WN) as MT x MT MFMA
// blocks. The MFMA is issued with the B fragment as the instruction's A operand, so the
// accumulator's column index is m: for MT=32, lane l holds m = l&31 and n = 8q + 4(l>>5) + r
// (q, r = 0..3); for MT=16, m = l&15 and n = 4(l>>4) + r.
// Double-buffered BK=64 stages. Per K-step t: all LDS-DMA pieces of stage t+1, then SS
// substeps of  ds_read(t, kk+1) | MFMAs(t, kk); then vmcnt(0) + s_barrier hands t+1 over.
template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT, int EK = EPI_GEN>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_bf16_kernel(GemmArgs g, EpiArgs e) {
  typedef typename Acc<MT>::T AccT;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / MT, FN = TN / MT;
  constexpr int SS = MT == 32 ? 4 : 2;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EROWS = BM / 2, ELD = BN + 4;                         // epilogue staging: half tile fp32
  constexpr int SMEM = (2 * STAGE > EROWS * ELD * 4) ? 2 * STAGE : EROWS * ELD * 4;
  static_assert(WM == 2, "epilogue staging splits the tile by the wave-row halves");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;

  int tm, tn, ks = 0;
  if (gridDim.y > 1) split_tile_of(g.tiles_m, g.tiles_n, tm, tn, ks);
  else {
    tile_of(blockIdx.x, g.tiles_m, g.tiles_n, tm, tn);
    ks = blockIdx.y;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const u32x4 ra = rsrc4(g.A);
  const u32x4 rb = rsrc4(g.B);
  DmaPlan<BM, AKC, NW, MT> pa;
  DmaPlan<BN, BKC, NW, MT> pb;
  pa.init(wave, lane, g.lda, m0, g.M);
  pb.init(wave, lane, g.ldb, n0, g.N);
  const int ktail = kbeg + (nk - 1) * BK;  // first K of the last step (only step that can be partial)

  AccT acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = AccT{};

  bf16x8 af[FM], bfr[FN];
  if (nk > 0) {
    pa.issue(ra, smem, wave, g.lda, kbeg, kend, kbeg == ktail);
    pb.issue(rb, smem + A_BYTES, wave, g.ldb, kbeg, kend, kbeg == ktail);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < FN; ++i) bfr[i] = read_frag<MT, BN, BKC>(smem + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
    for (int j = 0; j < FM; ++j) af[j] = read_frag<MT, BM, AKC>(smem, wm * TM + j * MT, 0, lane);
  }
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * STAGE;
    char* nxt = smem + ((t + 1) & 1) * STAGE;
    const bool more = t + 1 < nk;
    const int k1 = kbeg + (t + 1) * BK;
    // the whole of stage t+1 goes out first: it has the full K-step to land
    if (more) {
      pa.issue(ra, nxt, wave, g.lda, k1, kend, k1 == ktail);
      pb.issue(rb, nxt + A_BYTES, wave, g.ldb, k1, kend, k1 == ktail);
    }
#pragma unroll
    for (int kk = 0; kk < SS; ++kk) {
      bf16x8 an[FM], bn[FN];
      if (kk < SS - 1) {
#pragma unroll
        for (int i = 0; i < FN; ++i) bn[i] = read_frag<MT, BN, BKC>(cur + A_BYTES, wn * TN + i * MT, kk + 1, lane);
#pragma unroll
        for (int j = 0; j < FM; ++j) an[j] = read_frag<MT, BM, AKC>(cur, wm * TM + j * MT, kk + 1, lane);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) acc[i][j] = mfma<MT>(bfr[i], af[j], acc[i][j]);
      if (kk < SS - 1) {
#pragma unroll
        for (int i = 0; i < FN; ++i) bfr[i] = bn[i];
#pragma unroll
        for (int j = 0; j < FM; ++j) af[j] = an[j];
      }
    }
    if (more) {
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < FN; ++i) bfr[i] = read_frag<MT, BN, BKC>(nxt + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
      for (int j = 0; j < FM; ++j) af[j] = read_frag<MT, BM, AKC>(nxt, wm * TM + j * MT, 0, lane);
    }
  }

  tile_epilogue<BM, BN, WM, WN, MT, (BM >= 256 ? 2 : 1), SMEM, EK>(g, e, acc, smem, m0, n0, ks, wm, wn, lane,
                                                                     e.drop_thresh ? step_seed(e.seed) : 0);
}

// Ring variant: BK=32 stages in an NST-slot LDS ring, LDS-DMA issued NST-1 K-steps ahead and
// spread over the substeps (so no wave blocks on a burst of DMA issue and each stage has
// ~NST-2 K-steps to land). Per K-step t, in its last substep: counted vmcnt for stage t+1,
// s_barrier, fragment reads of (t+1, 0) — behind the MFMAs of (t, last). The slot refilled in
// step t is the one read in step t-1, released by the barrier of step t-1... which every wave
// passed after issuing (and before consuming) those reads.
template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT, int NST>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_ring_kernel(GemmArgs g, EpiArgs e) {
  typedef typename Acc<MT>::T AccT;
  constexpr int RBK = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / MT, FN = TN / MT;
  constexpr int SS = MT == 32 ? 2 : 1;
  constexpr int PD = NST - 1;  // prefetch distance in K-steps
  constexpr int A_BYTES = BM * RBK * 2, B_BYTES = BN * RBK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EPC = (TM * (BN + 4) * 4 <= NST * STAGE) ? 1 : 2;
  static_assert(TM / EPC * (BN + 4) * 4 <= NST * STAGE, "epilogue staging does not fit");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;

  int tm, tn, ks = 0;
  if (gridDim.y > 1) split_tile_of(g.tiles_m, g.tiles_n, tm, tn, ks);
  else {
    tile_of(blockIdx.x, g.tiles_m, g.tiles_n, tm, tn);
    ks = blockIdx.y;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + RBK - 1) / RBK;

  const u32x4 ra = rsrc4(g.A);
  const u32x4 rb = rsrc4(g.B);
  typedef DmaPlan<BM, AKC, NW, MT, RBK> PA;
  typedef DmaPlan<BN, BKC, NW, MT, RBK> PB;
  PA pa;
  PB pb;
  pa.init(wave, lane, g.lda, m0, g.M);
  pb.init(wave, lane, g.ldb, n0, g.N);
  const int ktail = kbeg + (nk - 1) * RBK;
  constexpr int PER = PA::NI + PB::NI;      // DMA instructions per stage per wave
  constexpr int EARLY = SS > 1 ? PA::NI : 0;  // of those, issued before the last substep

  AccT acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = AccT{};

  auto slot = [&](int st) -> char* { return smem + (st % NST) * STAGE; };
  auto issue_a = [&](int st) {
    const int k0 = kbeg + st * RBK;
    pa.issue(ra, slot(st), wave, g.lda, k0, kend, k0 == ktail);
  };
  auto issue_b = [&](int st) {
    const int k0 = kbeg + st * RBK;
    pb.issue(rb, slot(st) + A_BYTES, wave, g.ldb, k0, kend, k0 == ktail);
  };

  bf16x8 af[FM], bfr[FN];
  if (nk > 0) {
#pragma unroll
    for (int st = 0; st < PD; ++st)
      if (st < nk) {
        issue_a(st);
        issue_b(st);
      }
    // stage 0 landed: the stages after it may still be in flight
    if (nk >= 3) wait_vm<2 * PER>();
    else if (nk == 2) wait_vm<PER>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < FN; ++i) bfr[i] = read_frag<MT, BN, BKC, RBK>(smem + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
    for (int j = 0; j < FM; ++j) af[j] = read_frag<MT, BM, AKC, RBK>(smem, wm * TM + j * MT, 0, lane);
  }
  static_assert(NST == 4, "vmcnt bookkeeping below assumes a 4-slot ring (PD = 3)");
  // One MFMA substep (t, kk) on fragments (ca, cb), the next substep's fragments read into (na, nb).
  // The two fragment sets alternate by substep (SS = 2: within a K-step; SS = 1: the K loop unrolled by
  // two): with one set copied forward at every substep's end, those copies were 48 v_mov per K-step
  // (the loads into the next set are in flight while the MFMAs read the current one).
  bf16x8 af1[FM], bf1[FN];
  auto sub = [&](int t, int kk, const bf16x8 (&ca)[FM], const bf16x8 (&cb)[FN], bf16x8 (&na)[FM], bf16x8 (&nb)[FN]) {
    const char* cur = slot(t);
    const bool pf = t + PD < nk;
    if (kk < SS - 1) {
#pragma unroll
      for (int i = 0; i < FN; ++i) nb[i] = read_frag<MT, BN, BKC, RBK>(cur + A_BYTES, wn * TN + i * MT, kk + 1, lane);
#pragma unroll
      for (int j = 0; j < FM; ++j) na[j] = read_frag<MT, BM, AKC, RBK>(cur, wm * TM + j * MT, kk + 1, lane);
      if (pf) issue_a(t + PD);
    } else {
      if (t + 1 < nk) {
        // stage t+1 landed; stage t+2 and (SS>1) the A pieces of stage t+3 may be in flight
        if (pf) wait_vm<PER + EARLY>();
        else if (t + 2 < nk) wait_vm<PER>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* nx = slot(t + 1);
#pragma unroll
        for (int i = 0; i < FN; ++i) nb[i] = read_frag<MT, BN, BKC, RBK>(nx + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
        for (int j = 0; j < FM; ++j) na[j] = read_frag<MT, BM, AKC, RBK>(nx, wm * TM + j * MT, 0, lane);
      }
      if (pf) {
        if (SS == 1) issue_a(t + PD);
        issue_b(t + PD);
      }
    }
#pragma unroll
    for (int j = 0; j < FM; ++j)
#pragma unroll
      for (int i = 0; i < FN; ++i) acc[i][j] = mfma<MT>(cb[i], ca[j], acc[i][j]);
  };
  if constexpr (SS == 2) {
    for (int t = 0; t < nk; ++t) {
      sub(t, 0, af, bfr, af1, bf1);
      sub(t, 1, af1, bf1, af, bfr);
    }
  } else {
    for (int t = 0; t < nk; t += 2) {
      sub(t, 0, af, bfr, af1, bf1);
      if (t + 1 < nk) sub(t + 1, 0, af1, bf1, af, bfr);
    }
  }
  tile_epilogue<BM, BN, WM, WN, MT, EPC, NST * STAGE>(g, e, acc, smem, m0, n0, ks, wm, wn, lane,
                                                      e.drop_thresh ? step_seed(e.seed) : 0);
}

// ===================================================================== ping-pong kernel
// 256x128 tile on 4 waves (2 x 2, each a 128x64 accumulator tile of 16x16 blocks), BK=32 stages in
// a 3-slot LDS ring (72 KB): small enough for TWO workgroups per CU, so one workgroup's epilogue
// (VALU: bias, GELU, dropout hashing; LDS staging; stores) runs beside the other's MFMA main loop
// instead of idling the matrix pipe. One barrier per K-step: it publishes stage t (every wave
// waited for its own DMA pieces of it) and releases slot (t-1)%3, which is refilled with stage
// t+2 right after it (two K-steps of DMA slack). Fragments of a K-step are read after the
// barrier; the partner workgroup's waves fill the SIMD while they land.
template <bool AKC, bool BKC, int EK = EPI_GEN>
__global__ __launch_bounds__(256, 2) void gemm_pp_kernel(GemmArgs g, EpiArgs e) {
  typedef f32x4 AccT;
  constexpr int BM = 256, BN = 128, WM = 2, WN = 2, MT = 16, RBK = 32, NST = 3, NW = 4;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / MT, FN = TN / MT;
  constexpr int A_BYTES = BM * RBK * 2, B_BYTES = BN * RBK * 2, STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;
  int tm, tn, ks = 0;
  if (gridDim.y > 1) split_tile_of(g.tiles_m, g.tiles_n, tm, tn, ks);
  else {
    tile_of(blockIdx.x, g.tiles_m, g.tiles_n, tm, tn);
    ks = blockIdx.y;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + RBK - 1) / RBK;
  const int ktail = kbeg + (nk - 1) * RBK;
  const u32x4 ra = rsrc4(g.A);
  const u32x4 rb = rsrc4(g.B);
  typedef DmaPlan<BM, AKC, NW, MT, RBK> PA;
  typedef DmaPlan<BN, BKC, NW, MT, RBK> PB;
  PA pa;
  PB pb;
  pa.init(wave, lane, g.lda, m0, g.M);
  pb.init(wave, lane, g.ldb, n0, g.N);
  constexpr int PER = PA::NI + PB::NI;  // DMA instructions per stage per wave
  auto slot = [&](int st) -> char* { return smem + (st % NST) * STAGE; };
  auto issue = [&](int st) {
    const int k0 = kbeg + st * RBK;
    pa.issue(ra, slot(st), wave, g.lda, k0, kend, k0 == ktail);
    pb.issue(rb, slot(st) + A_BYTES, wave, g.ldb, k0, kend, k0 == ktail);
  };
  AccT acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = AccT{};
  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) wait_vm<PER>();  // stage t landed (own pieces); stage t+1 may fly
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();   // stage t published; slot (t-1)%3 free
    asm volatile("" ::: "memory");
    if (t + 2 < nk) issue(t + 2);
    const char* cur = slot(t);
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) bfr[i] = read_frag<MT, BN, BKC, RBK>(cur + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
    for (int j = 0; j < FM; ++j) af[j] = read_frag<MT, BM, AKC, RBK>(cur, wm * TM + j * MT, 0, lane);
#pragma unroll
    for (int j = 0; j < FM; ++j)
#pragma unroll
      for (int i = 0; i < FN; ++i) acc[i][j] = mfma<MT>(bfr[i], af[j], acc[i][j]);
  }
  bar_lds();  // every wave's fragment reads are done: the ring becomes epilogue staging
  tile_epilogue<BM, BN, WM, WN, MT, 2, NST * STAGE, EK>(g, e, acc, smem, m0, n0, ks, wm, wn, lane,
                                                         e.drop_thresh ? step_seed(e.seed) : 0);
}

template <bool AKC, bool BKC>
static int launch_pp(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  g.tiles_m = (g.M + 255) / 256;
  g.tiles_n = (g.N + 127) / 128;
  const dim3 grid(g.tiles_m * g.tiles_n, g.splits);
  // fixed-flag epilogue kinds as in the 8-phase kernel (K-contiguous operands, no split-K)
  const int ek = (AKC && BKC && !g.partial) ? epi_kind(e, g.M, g.N) : EPI_GEN;
#define FER_PPK(K) hipLaunchKernelGGL((gemm_pp_kernel<AKC, BKC, K>), grid, dim3(256), 0, st, g, e)
  if constexpr (AKC && BKC) {
    switch (ek) {
      case EPI_STORE: FER_PPK(EPI_STORE); break;
      case EPI_GATE: FER_PPK(EPI_GATE); break;
      case EPI_GATER: FER_PPK(EPI_GATER); break;
      case EPI_RES2: FER_PPK(EPI_RES2); break;
      case EPI_MUL2: FER_PPK(EPI_MUL2); break;
      default: FER_PPK(EPI_GEN); break;
    }
  } else {
    FER_PPK(EPI_GEN);
  }
#undef FER_PPK
  return 0;
}

// ===================================================================== 8-phase kernel
// 256x256x64 tile, 8 waves as 2 (row halves, wr = wave>>2) x 4 (column quarters, wc = wave&3),
// each wave a 128x64 accumulator tile cut into four 64x32 quadrants. A K-tile runs as four
// PHASES; each phase is  [load segment: fragment ds_reads + one 16 KB LDS-DMA unit + counted
// vmcnt] s_barrier [MFMA segment, s_setprio 1: one quadrant x K=64] s_barrier.  Waves 4-7 run
// one barrier behind waves 0-3, so on every SIMD one wave's MFMA segment overlaps its
// partner's load segment and the matrix pipe never waits on LDS/DMA issue.
//
// LDS: 2 buffers x {A unit qm=0, A unit qm=1, B unit qn=0, B unit qn=1}, 16 KB each. A unit qm
// holds the 128 A rows {wr*128 + qm*64 + i}; B unit qn the 128 B columns {wc*64 + qn*32 + i}:
// exactly what quadrant row/column qm/qn of all waves reads, so a unit is refilled as soon as
// its readers are done. Quadrant order (0,0) (1,1) (0,1) (1,0): phases 0 and 1 read all
// fragments (8 A + 4 B each), phases 2 and 3 reuse them. Unit issue per phase q of K-tile T:
//   q=0: B0(T+1)  q=1: A1(T+1)  q=2: B1(T+1)  q=3: A0(T+2)
// (each >= 3 phases after its last read in the same buffer). Waits: q=3 retires A0/B0(T+1)
// (vmcnt 6: A1, B1(T+1), A0(T+2) may fly), q=0 retires A1/B1(T) (vmcnt 4); a unit is read one
// phase after the wait that retires it (the barrier between publishes other waves' DMA).
template <bool KC, int MT, bool ISA>
struct UnitPlan {
  uint32_t base[2];
  int kof[2];
  // local index (0..127) -> index inside the 256-wide tile
  FER_DEV static int map(int l, int q) {
    return ISA ? (l >> 6) * 128 + q * 64 + (l & 63) : (l >> 5) * 64 + q * 32 + (l & 31);
  }
  FER_DEV void init(int wave, int lane, long ld, int r0, int rmax, int q) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int gi = wave * 2 + i;
      bool ok;
      uint32_t off;
      if constexpr (KC) {
        const int row = gi * 8 + (lane >> 3);
        const int c = (lane & 7) ^ kc_swz<64>(row);
        const int gr = r0 + map(row, q);
        ok = gr < rmax;
        kof[i] = c * 8;
        off = (uint32_t)(((long)gr * ld + c * 8) * 2);
      } else {
        const int byte = gi * 1024 + lane * 16;
        const int k = byte >> 8;
        const int c = ((byte & 255) >> 4) ^ mn_swz_t<MT>(k);
        const int gc = r0 + map(c * 8, q);
        ok = gc < rmax;
        kof[i] = k;
        off = (uint32_t)(((long)k * ld + gc) * 2);
      }
      base[i] = ok ? off : FER_OOB;
    }
  }
  FER_DEV void issue(__amdgpu_buffer_rsrc_t rs, char* unit, int wave, long ld, int k0, int kmax, bool tail) const {
    const uint32_t kadd = KC ? (uint32_t)(k0 * 2) : (uint32_t)(k0 * ld * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t voff = (!tail || k0 + kof[i] < kmax) ? base[i] + kadd : FER_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(unit + (wave * 2 + i) * 1024), 16, voff, 0, 0, 0);
    }
  }
};

#ifdef FER_GEMM_STAMPS
// Diagnostic build only (cdna_hip_programming.md §7 in-kernel stamps): wave 0 and wave 4 of
// workgroup 0 record s_memtime at the phase boundaries of their second tile into LDS, dumped to
// g_stamps after the main loop. Never built into libfervit.so.
__device__ unsigned long long g_stamps[2][4 + 16 * 4 * 4];
FER_DEV unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define FER_STAMP(i)                                              \
  do {                                                            \
    if (st_on) {                                                  \
      const unsigned long long t_ = stamp_now();                  \
      if (lane == 0) st_l[st_w * (4 + 256) + (i)] = t_;           \
    }                                                             \
  } while (0)
#else
#define FER_STAMP(i) do {} while (0)
#endif

// Wave-private epilogue of the 8-phase kernel (fixed kinds, MFMA 16x16). Each wave stages its own
// 128 x 64 accumulator region through its own 16 KB of LDS (the main loop's operand buffers) in
// 32-row chunks of fp32, XOR-swizzled by row, and reads it back row-contiguous: lane = (row
// lane >> 3 of an 8-row pass, 8 columns 8 (lane & 7)), so the kind's arithmetic (epi8_k), the
// row operand's loads (RES / MUL, 16 B per lane, one chunk ahead) and the output stores (16 B per
// lane, whole 128-byte rows per 8 lanes) are row-contiguous. No workgroup barrier between chunks:
// the workgroup-wide staging (all waves through two shared areas, four stage / finish rounds with
// barriers) spent 28-34 k cycles per GELU-gate tile mostly waiting at those barriers for the slower
// wave-row half. (Storing straight from the accumulator layout -- 8 bytes per lane, 16 rows per
// instruction -- measured 10-25 % slower kernels: profiles/r04k_gemm_ab.txt.)
// MUL's fused column sums (cs_part): per lane over its rows, over the 8 row lanes of a column group,
// then the two wave-row halves through LDS.
template <int EK>
FER_DEV void tile_epilogue_wp(const GemmArgs& g, const EpiArgs& e, f32x4 (&acc)[4][8], char* smem, int m0, int n0,
                              int wr, int wc, int lane, uint64_t seed) {
  constexpr int S = epi_base(EK);
  constexpr bool X = S == EPI_RES || S == EPI_MUL;
  constexpr bool CS = S == EPI_MUL;
  const int wave = wr * 4 + wc;
  char* const ws = smem + wave * 16384;  // two 8 KB chunk buffers
  // staging write: block (i, j) of the chunk -> local row 16 (j & 1) + (lane & 15), column 16 i + 4 (lane >> 4)
  auto swz = [](int row, int c16) { return row * 256 + ((c16 ^ (row & 15)) << 4); };
  const int prow = lane >> 3, pc = 8 * (lane & 7);  // read-back: row of the pass, first column
  const int n = n0 + wc * 64 + pc;
  const bool nok = n < g.N;  // N % 8 == 0 on this path (checked by the host)
  const float dsc = e.drop_thresh ? e.drop_scale : 1.f;
  const float ab = (S == EPI_RES || EK == EPI_GATER) ? e.alpha * dsc : e.alpha;
  const f32x2 ghs = f32x2(0.5f * dsc), gps = f32x2(0.39894228040143268f * dsc);
  f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (e.bias && nok) {
    b0 = ldg_f32x4(e.bias + n);
    b1 = ldg_f32x4(e.bias + n + 4);
  }
  if (S == EPI_RES || EK == EPI_GATER) {
    b0 *= dsc;
    b1 *= dsc;
  }
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(e.c), rp = make_rsrc(e.pre ? e.pre : e.c);
  const void* xs = e.res ? e.res : e.aux;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(X && xs ? xs : e.c);
  const uint32_t ldcb = (uint32_t)e.ldc * 2, ldpb = (uint32_t)e.ldp * 2;
  const uint32_t ldxb = X ? (uint32_t)(e.res ? e.ldr : e.ldx) * 2 : 0u;
  const int rw0 = m0 + wr * 128 + prow;  // this lane's row in pass 0 of chunk 0
  auto load_x = [&](int c, bf16x8 (&xc)[4]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = rw0 + c * 32 + p * 8;
      const uint32_t off = (nok && row < g.M) ? (uint32_t)row * ldxb + (uint32_t)n * 2 : FER_OOB;
      xc[p] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    }
  };
  f32x4 cs0 = f32x4{0.f, 0.f, 0.f, 0.f}, cs1 = cs0;
  bf16x8 xr[2][4];
  if constexpr (X) load_x(0, xr[0]);
  bar_lds();  // every wave is done with the main loop's operand buffers
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    char* const buf = ws + (c & 1) * 8192;
    if constexpr (X) {
      if (c + 1 < 4) load_x(c + 1, xr[(c + 1) & 1]);
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(f32x4*)(buf + swz(16 * jj + (lane & 15), 4 * i + (lane >> 4))) = acc[i][2 * c + jj];
    // (a wave's own LDS writes are complete for its later reads: in-order LDS, no barrier)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int lrow = p * 8 + prow;
      f32x4 v0 = *(const f32x4*)(buf + swz(lrow, pc >> 2)), v1 = *(const f32x4*)(buf + swz(lrow, (pc >> 2) + 1));
      const int row = rw0 + c * 32 + p * 8;
      const bool ok = nok && row < g.M;
      const uint32_t di = (uint32_t)row * (uint32_t)e.drop_ld + (uint32_t)n;
      epi8_kb<EK>(e, ok ? (uint32_t)row * ldcb + (uint32_t)n * 2 : FER_OOB,
                  ok ? (uint32_t)row * ldpb + (uint32_t)n * 2 : FER_OOB, di, v0, v1, b0, b1,
                  X ? xr[c & 1][p] : bf16x8{}, seed, ab, ghs, gps, dsc, rc, rp);
      // no row / column select: an out-of-range row or column multiplies by its row operand x, loaded
      // through FER_OOB as zeros, so it adds exactly 0 (its accumulators are 0 as well: zero-filled A rows)
      if constexpr (CS) {
        cs0 += v0;
        cs1 += v1;
      }
    }
  }
  if constexpr (CS) {
    if (g.cs_part) {
      // over the 8 row lanes of the column group (lanes 8 apart), fixed order
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int d = 8; d < 64; d <<= 1) {
          cs0[r] += __shfl_xor(cs0[r], d);
          cs1[r] += __shfl_xor(cs1[r], d);
        }
      }
      float* red = (float*)smem;  // [2 wave-row halves][256 columns]
      bar_lds();                  // every wave is done with its staging
      if (prow == 0) {
        *(f32x4*)(red + wr * 256 + wc * 64 + pc) = cs0;
        *(f32x4*)(red + wr * 256 + wc * 64 + pc + 4) = cs1;
      }
      bar_lds();
      const int t = threadIdx.x;
      if (t < 256 && n0 + t < g.N) g.cs_part[(long)(m0 / 256) * g.N + n0 + t] = red[t] + red[256 + t];
    }
  }
}

// claim_slot (work-queue mode): thread 0 claims a tile at the start of this one, before the
// prologue's operand DMA, and parks the id in that LDS word after the prologue's wait (which
// retires the atomic together with the previous tile's epilogue stores and the first K-tile)
template <bool AKC, bool BKC, int MT, int EK>
FER_DEV void tile_8ph(const GemmArgs& g, const EpiArgs& e, int bid, char* smem, lds_vint* claim_slot, uint64_t seed) {
  typedef typename Acc<MT>::T AccT;
  constexpr int UNIT = 16384, BUF = 4 * UNIT;  // A0 A1 B0 B1
  constexpr int FM = 128 / MT, FN = 64 / MT;   // MFMA blocks per wave (rows, cols)
  constexpr int QJ = FM / 2, QI = FN / 2;      // per quadrant
  constexpr int KS = 64 / (MT == 32 ? 16 : 32);  // MFMA K-steps per K-tile
  // launder the thread index: lane-derived addressing is recomputed per tile instead of being
  // hoisted out of the persistent loop (hoisting pushed the kernel past 256 VGPRs)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
#ifdef FER_GEMM_STAMPS
  __shared__ unsigned long long st_l[2 * (4 + 256)];
  const bool st_on = blockIdx.x == 0 && blockIdx.y == 0 && bid == (int)gridDim.x && (wave & 3) == 0;
  const int st_w = wave >> 2;
#endif
  FER_STAMP(0);

  int tm, tn;
  // GELU-gate fc1 forward: row groups of 4 tiles (377 -> 367-370 us alone, profiles/r03w_tile_group_ab.txt;
  // the other kinds gain nothing from it)
  tile_of(bid, g.tiles_m, g.tiles_n, tm, tn, EK == EPI_GATE ? 4 : 8);
  const int m0 = tm * 256, n0 = tn * 256;
  const int ks = blockIdx.y;
  const int kbeg = ks * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + 63) / 64;
  const int ktail = kbeg + (nk - 1) * 64;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.B);
  UnitPlan<AKC, MT, true> pa0, pa1;
  UnitPlan<BKC, MT, false> pb0, pb1;
  pa0.init(wave, lane, g.lda, m0, g.M, 0);
  pa1.init(wave, lane, g.lda, m0, g.M, 1);
  pb0.init(wave, lane, g.ldb, n0, g.N, 0);
  pb1.init(wave, lane, g.ldb, n0, g.N, 1);
  auto unit = [&](int T, int u) -> char* { return smem + (T & 1) * BUF + u * UNIT; };
  auto kt = [&](int T) { return kbeg + T * 64; };
  auto iA0 = [&](int T) { pa0.issue(ra, unit(T, 0), wave, g.lda, kt(T), kend, kt(T) == ktail); };
  auto iA1 = [&](int T) { pa1.issue(ra, unit(T, 1), wave, g.lda, kt(T), kend, kt(T) == ktail); };
  auto iB0 = [&](int T) { pb0.issue(rb, unit(T, 2), wave, g.ldb, kt(T), kend, kt(T) == ktail); };
  auto iB1 = [&](int T) { pb1.issue(rb, unit(T, 3), wave, g.ldb, kt(T), kend, kt(T) == ktail); };

  AccT acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = AccT{};
  bf16x8 fa[2][KS][QJ], fb[2][KS][QI];

  int claimed = -1;
  if (claim_slot && tid == 0) claimed = wq_claim(g.tq, g.tq_base, g.tiles_m * g.tiles_n);
  if (nk > 0) {
    iA0(0); iB0(0); iA1(0); iB1(0);
    if (nk > 1) {
      iA0(1);
      wait_vm<6>();
    } else {
      wait_vm<4>();
    }
    __builtin_amdgcn_s_barrier();
    if (wr) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
    asm volatile("" ::: "memory");
  }
  if (claim_slot && tid == 0) *claim_slot = claimed;
  FER_STAMP(1);

  for (int T = 0; T < nk; ++T) {
    const bool n1 = T + 1 < nk, n2 = T + 2 < nk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int st_i = 4 + (T * 4 + q) * 4;
      if (T < 16) FER_STAMP(st_i);
      // ---- load segment
      // Fragment reads spread over the four phases (quadrants in the order (0,0) (0,1) (1,1) (1,0)):
      // B0 in phase 0 (with A0 in the first K-tile), B1 in phase 1, A1 in phase 2 and the next K-tile's
      // A0 in phase 3, 4-8 reads per load segment instead of 12, 12, 0, 0 (profiles/r05bf_*).
      if (q < 2) {
        const char* ub = unit(T, 2 + q);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int i = 0; i < QI; ++i) fb[q][kk][i] = read_frag<MT, 128, BKC, 64>(ub, wc * 32 + i * MT, kk, lane);
      }
      if ((q == 0 && T == 0) || q == 2 || (q == 3 && n1)) {
        const int qa = q == 2 ? 1 : 0;
        const char* ua = unit(q == 3 ? T + 1 : T, qa);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int j = 0; j < QJ; ++j) fa[qa][kk][j] = read_frag<MT, 128, AKC, 64>(ua, wr * 64 + j * MT, kk, lane);
      }
      if (q == 0) {
        if (n1) { iB0(T + 1); wait_vm<4>(); } else { wait_vm<0>(); }
      } else if (q == 1) {
        if (n1) iA1(T + 1);
      } else if (q == 2) {
        if (n1) { iB1(T + 1); wait_vm<6>(); }  // the next K-tile's A0 (phase 3 reads it)
      } else {
        if (n2) { iA0(T + 2); wait_vm<6>(); } else if (n1) { wait_vm<4>(); }
      }
      if (T < 16) FER_STAMP(st_i + 1);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (T < 16) FER_STAMP(st_i + 2);
      // ---- MFMA segment: quadrant (qm, qn) for q = 0..3 -> (0,0) (0,1) (1,1) (1,0)
      constexpr int dummy = 0;
      (void)dummy;
      const int qm = q >= 2 ? 1 : 0;
      const int qn = (q == 1 || q == 2) ? 1 : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int j = 0; j < QJ; ++j)
#pragma unroll
          for (int i = 0; i < QI; ++i)
            acc[qn * QI + i][qm * QJ + j] = mfma<MT>(fb[qn][kk][i], fa[qm][kk][j], acc[qn * QI + i][qm * QJ + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (T < 16) FER_STAMP(st_i + 3);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if (nk > 0 && !wr) __builtin_amdgcn_s_barrier();  // waves 0-3 catch up with the stagger
  FER_STAMP(2);
  static_assert(64 * (256 + 4) * 4 <= 2 * BUF, "epilogue staging (2 chunks per half) must fit");
  if constexpr (EK != EPI_GEN && MT == 16)
    tile_epilogue_wp<EK>(g, e, acc, smem, m0, n0, wr, wc, lane, seed);
  else
    tile_epilogue<256, 256, 2, 4, MT, 2, 2 * BUF, EK>(g, e, acc, smem, m0, n0, ks, wr, wc, lane, seed);
  FER_STAMP(3);
#ifdef FER_GEMM_STAMPS
  if (st_on) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int i = lane; i < 4 + 256; i += 64) g_stamps[st_w][i] = st_l[st_w * (4 + 256) + i];
  }
#endif
}

// ---- Pipelined schedule for the plain kind (EPI_STORE, MT 16): a tile's epilogue overlaps the next
// tile's first operand loads and its own store drain overlaps the next tile's first K-tile.
// vmcnt retires in issue order, so in the plain schedule (epilogue stores, then the next tile's
// prologue DMA and its wait) every tile start waits for the previous tile's stores to reach memory
// and then for a full DMA round trip. Here the workgroup issues the next tile's prologue (pro_8ph:
// A0 B0 A1 B1 of K-tile 0 and A0 of K-tile 1, ten instructions per wave) right after its main loop,
// BEFORE the epilogue; the epilogue stages through stage 1's B units (free until K-tile 1's B0
// issue, which comes after the epilogue's closing barrier), and the next tile's first two waits
// skip the epilogue's PP_SV vector-memory instructions (its 16 buffer stores per wave, issued
// unconditionally at FER_OOB offsets; anything the compiler adds only makes those waits stricter),
// which are younger than the operands they wait for. The first wait covering them is K-tile 1's.
// Measured (profiles/r04ah_gemm_pipelined_store_ab.txt, same box, against the plain schedule):
// fc1-shape fwd 237.4 -> 224.7 us (+bias 231.9 -> 221.2), qkv fwd 167.0 -> 163.7, the transposed-
// copy fc2 dgrad 229.3 -> 226.1; K = 3072 (fc2 fwd) unchanged. (A first version lost most of it:
// alpha / bias read through the EpiArgs reference were kept in a per-thread copy the compiler
// promoted to LDS, and that read waited vmcnt(0) for the LDS DMA -- r04ag.) The row-operand and
// gate kinds stay on tile_8ph: this schedule for them (gpurun_out/patches/
// gemm_pipelined_all_kinds.patch) faulted the GPU (r04af, r05w): cause found in r05y -- in the second
// tile on, a spilled SGPR pair reloaded by v_readlane right before the inline-asm claim atomic that
// takes it as its address, without the 5 wait states "VALU writes SGPR -> VMEM reads it" needs (LLVM
// does not look inside inline asm); the build pass (store_hazard_pad.py) now pads every such site.
// The gate and row-operand kinds on this schedule (round 5, epilogue fields by value) passed the kernel
// tests but measured slower (profiles/r05y_*, r05ad_*: gate-mul +16 us, fc2 fwd +2-5 us, the step
// +0.3 ms) and were removed in round 6: only the plain kind is pipelined.
// PP_SV: the vector-memory instructions every wave's epilogue issues after pro_8ph, all of them
// unconditional (FER_OOB offsets): its 16 output stores. Anything the compiler adds only makes the next
// tile's first waits stricter; the epilogue's compiler barriers keep its memory operations on their
// side of pro_8ph.
template <int EK>
constexpr int pp_sv() {
  return 16;
}
template <int EK>
constexpr bool pp_kind() {
  return EK == EPI_STORE;
}

// Always exactly ten instructions per wave, without a branch (the epilogue's compiler-placed waits
// for its bias loads would otherwise merge the issue and no-issue paths into a
// vmcnt(0), i.e. wait for this DMA): bid < 0 (no next tile) or units beyond K go to FER_OOB, whose
// LDS writes land in stage 0 and stage 1's A0 unit, which the epilogue does not use.
template <bool AKC, bool BKC, int MT, int EK>
FER_DEV void pro_8ph(const GemmArgs& g, int bid, char* smem, int wave, int lane) {
  constexpr int UNIT = 16384, BUF = 4 * UNIT;
  int tm, tn;
  tile_of(bid < 0 ? 0 : bid, g.tiles_m, g.tiles_n, tm, tn, EK == EPI_GATE ? 4 : 8);
  const int kbeg = blockIdx.y * g.k_chunk, kend = bid < 0 ? kbeg : min(g.K, kbeg + g.k_chunk);
  const int ktail = kbeg + ((kend - kbeg + 63) / 64 - 1) * 64;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A), rb = make_rsrc(g.B);
  UnitPlan<AKC, MT, true> a0, a1;
  UnitPlan<BKC, MT, false> b0, b1;
  a0.init(wave, lane, g.lda, tm * 256, g.M, 0);
  a1.init(wave, lane, g.lda, tm * 256, g.M, 1);
  b0.init(wave, lane, g.ldb, tn * 256, g.N, 0);
  b1.init(wave, lane, g.ldb, tn * 256, g.N, 1);
  // (tail: every unit at or past the last K-tile checks its columns against kend)
  a0.issue(ra, smem, wave, g.lda, kbeg, kend, kbeg >= ktail);
  b0.issue(rb, smem + 2 * UNIT, wave, g.ldb, kbeg, kend, kbeg >= ktail);
  a1.issue(ra, smem + UNIT, wave, g.lda, kbeg, kend, kbeg >= ktail);
  b1.issue(rb, smem + 3 * UNIT, wave, g.ldb, kbeg, kend, kbeg >= ktail);
  a0.issue(ra, smem + BUF, wave, g.lda, kbeg + 64, kend, kbeg + 64 >= ktail);
}

// The pipelined schedule's epilogue (EPI_STORE: c = alpha acc + bias), with the next tile's prologue
// issued after the bias loads. Each wave stages its 128 x 64 region through its own 4 KB of stage
// 1's B units, eight 16-row chunks of fp32 XOR-swizzled by row, read back row-contiguous (lane =
// row lane >> 3 of an 8-row pass, columns 8 (lane & 7)): 16-byte buffer stores, whole 128-byte
// rows per 8 lanes, FER_OOB for rows past M.
// (the epilogue fields arrive as values, PpEpi: reading them through the EpiArgs reference left
// alpha and bias in a per-thread copy that the compiler promoted to LDS, whose read then waited
// vmcnt(0) for the in-flight LDS DMA)
struct PpEpi {
  void* c;
  const float* bias;
  long ldc;
  float alpha;
};
template <bool AKC, bool BKC, int MT>
FER_DEV void epi_8ph_pp(const GemmArgs& g, const PpEpi& e, f32x4 (&acc)[4][8], char* smem, int m0, int n0, int wave,
                        int lane, int next) {
  constexpr int UNIT = 16384, BUF = 4 * UNIT;
  const int wr = wave >> 2, wc = wave & 3;
  const int prow = lane >> 3, pc = 8 * (lane & 7);
  const int n = n0 + wc * 64 + pc;
  const bool nok = n < g.N;  // N % 8 == 0 on this path (checked by the host)
  const __amdgpu_buffer_rsrc_t rbias = make_rsrc(e.bias ? (const void*)e.bias : e.c);
  const uint32_t boff = (e.bias && nok) ? (uint32_t)n * 4 : FER_OOB;
  const f32x4 b0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rbias, boff, 0, 0));
  const f32x4 b1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rbias, boff + 16, 0, 0));
  pro_8ph<AKC, BKC, MT, EPI_STORE>(g, next, smem, wave, lane);
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(e.c);
  const uint32_t ldcb = (uint32_t)e.ldc * 2;
  const float alpha = e.alpha;
  const int rw0 = m0 + wr * 128 + prow;  // this lane's row in pass 0 of chunk 0
  char* const ws = smem + BUF + 2 * UNIT + wave * 4096;
  auto swz = [](int row, int c16) { return row * 256 + ((c16 ^ row) << 4); };
#pragma unroll
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *(f32x4*)(ws + swz(lane & 15, 4 * i + (lane >> 4))) = acc[i][c];
    // (a wave's own LDS accesses complete in order: no barrier)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lrow = p * 8 + prow;
      const f32x4 v0 = *(const f32x4*)(ws + swz(lrow, pc >> 2)) * alpha + b0;
      const f32x4 v1 = *(const f32x4*)(ws + swz(lrow, (pc >> 2) + 1)) * alpha + b1;
      const int row = rw0 + c * 16 + p * 8;
      const uint32_t oc = (nok && row < g.M) ? (uint32_t)row * ldcb + (uint32_t)n * 2 : FER_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pack8(v0, v1)), rc, oc, 0, 0);
    }
  }
  bar_lds();  // the staging area is K-tile 1's B units
}

// One tile of the pipelined schedule; returns the workgroup's next tile (-1: none). PEND: the
// previous tile's epilogue sits between this tile's prologue DMA and its first wait (every tile
// but a workgroup's first; a template flag: as a loop-carried bool it took a VGPR that spilled).
template <bool AKC, bool BKC, int MT, int EK, bool PEND, typename EP>
FER_DEV int tile_8ph_pp(const GemmArgs& g, const EP& e, int bid, char* smem, lds_vint* slot) {
  static_assert(MT == 16 && pp_kind<EK>(), "pipelined schedule: MT 16 fragments, the pipelined kinds");
  constexpr int UNIT = 16384, BUF = 4 * UNIT;
  constexpr int FM = 8, FN = 4, QJ = 4, QI = 2, KS = 2;
  constexpr int SV = pp_sv<EK>();
  static_assert(6 + SV <= 63, "vmcnt range");
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  int tm, tn;
  tile_of(bid, g.tiles_m, g.tiles_n, tm, tn, EK == EPI_GATE ? 4 : 8);
  const int m0 = tm * 256, n0 = tn * 256;
  const int kbeg = blockIdx.y * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + 63) / 64;
  const int ktail = kbeg + (nk - 1) * 64;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.B);
  UnitPlan<AKC, MT, true> pa0, pa1;
  UnitPlan<BKC, MT, false> pb0, pb1;
  pa0.init(wave, lane, g.lda, m0, g.M, 0);
  pa1.init(wave, lane, g.lda, m0, g.M, 1);
  pb0.init(wave, lane, g.ldb, n0, g.N, 0);
  pb1.init(wave, lane, g.ldb, n0, g.N, 1);
  auto unit = [&](int T, int u) -> char* { return smem + (T & 1) * BUF + u * UNIT; };
  auto kt = [&](int T) { return kbeg + T * 64; };
  auto iA0 = [&](int T) { pa0.issue(ra, unit(T, 0), wave, g.lda, kt(T), kend, kt(T) == ktail); };
  auto iA1 = [&](int T) { pa1.issue(ra, unit(T, 1), wave, g.lda, kt(T), kend, kt(T) == ktail); };
  auto iB0 = [&](int T) { pb0.issue(rb, unit(T, 2), wave, g.ldb, kt(T), kend, kt(T) == ktail); };
  auto iB1 = [&](int T) { pb1.issue(rb, unit(T, 3), wave, g.ldb, kt(T), kend, kt(T) == ktail); };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][KS][QJ], fb[2][KS][QI];

  // The next tile's claim, read after the main loop (whose last K-tile waits for vmcnt(0)). Inline
  // asm (wq_claim_issue): the builtin atomic's result is consumed at once, a vmcnt(0) that would
  // wait for the previous epilogue's stores. In wave 0 it adds one younger instruction to the
  // first two waits, which then also wait for one more DMA instruction.
  uint32_t claim_raw = 0;
  if (slot && tid == 0) {
    // (the queue word's address in SGPRs: a VGPR pair kept across the main loop spilled)
    const int* qp = g.tq + (blockIdx.x & 7) * FER_WQ_PAD;
    asm volatile("global_atomic_add %0, %1, %2, %3 sc0" : "=v"(claim_raw) : "v"(0u), "v"(1), "s"(qp) : "memory");
  }
  if (nk > 0) {
    // A0, B0 of K-tile 0 (pro_8ph always issues five units)
    if constexpr (PEND) wait_vm<6 + SV>(); else wait_vm<6>();
    __builtin_amdgcn_s_barrier();
    if (wr) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
    asm volatile("" ::: "memory");
  }

  for (int T = 0; T < nk; ++T) {
    const bool n1 = T + 1 < nk, n2 = T + 2 < nk;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // Fragment reads spread over the four phases (quadrants in the order (0,0) (0,1) (1,1) (1,0)):
      // B0 in phase 0 (with A0 in the first K-tile), B1 in phase 1, A1 in phase 2 and the next K-tile's
      // A0 in phase 3, 4-8 reads per load segment instead of 12, 12, 0, 0 (profiles/r05bf_*).
      if (q < 2) {
        const char* ub = unit(T, 2 + q);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int i = 0; i < QI; ++i) fb[q][kk][i] = read_frag<MT, 128, BKC, 64>(ub, wc * 32 + i * MT, kk, lane);
      }
      if ((q == 0 && T == 0) || q == 2 || (q == 3 && n1)) {
        const int qa = q == 2 ? 1 : 0;
        const char* ua = unit(q == 3 ? T + 1 : T, qa);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int j = 0; j < QJ; ++j) fa[qa][kk][j] = read_frag<MT, 128, AKC, 64>(ua, wr * 64 + j * MT, kk, lane);
      }
      if (q == 0) {
        if (n1) {
          iB0(T + 1);
          if (PEND && T == 0) wait_vm<4 + SV>(); else wait_vm<4>();
        } else {
          wait_vm<0>();
        }
      } else if (q == 1) {
        if (n1) iA1(T + 1);
      } else if (q == 2) {
        if (n1) {  // the next K-tile's A0 (phase 3 reads it)
          iB1(T + 1);
          if (PEND && T == 0) wait_vm<6 + SV>(); else wait_vm<6>();
        }
      } else {
        if (n2) { iA0(T + 2); wait_vm<6>(); } else if (n1) { wait_vm<4>(); }
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const int qm = q >= 2 ? 1 : 0;
      const int qn = (q == 1 || q == 2) ? 1 : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int j = 0; j < QJ; ++j)
#pragma unroll
          for (int i = 0; i < QI; ++i)
            acc[qn * QI + i][qm * QJ + j] = mfma<MT>(fb[qn][kk][i], fa[qm][kk][j], acc[qn * QI + i][qm * QJ + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if (slot && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (already retired by the last K-tile's wait)
    asm volatile("" : "+v"(claim_raw));
    *slot = claim_raw;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (nk > 0 && !wr) __builtin_amdgcn_s_barrier();  // waves 0-3 catch up with the stagger
  int next;
  if (slot) {
    next = wq_claim_finish((uint32_t)__builtin_amdgcn_readfirstlane(*slot), g.tq_base, g.tiles_m * g.tiles_n);
  } else {
    next = bid + (int)gridDim.x;
    if (next >= g.tiles_m * g.tiles_n) next = -1;
  }

  epi_8ph_pp<AKC, BKC, MT>(g, e, acc, smem, m0, n0, wave, lane, next);
  return next;
}

// Persistent launch (one workgroup per CU, tiles bid, bid + grid, ...: the XCD-aware tile order
// is kept since grid % 8 == 0). A workgroup goes from one tile's epilogue stores straight into
// the next tile's operand DMA, so the store drain overlaps the next tile's first loads instead
// of sitting between a workgroup's exit and its successor's launch.
// DYN: tiles from the per-stream work queue (common.h wq_*; the class of tile bid is bid & 7, the
// XCD tile_of's remap gives it): the first tile is blockIdx.x, each tile claims the next one at
// its start (tile_8ph claim_slot) and hands it on through LDS at its end. !DYN: fixed stride
// (split-K launches, stream capture, fer_set_persistent_mode).
template <bool AKC, bool BKC, int MT, bool DYN, int EK>
__global__ __launch_bounds__(512, 1) void gemm_8ph_kernel(GemmArgs g, EpiArgs e) {
  __shared__ __attribute__((aligned(1024))) char smem[8 * 16384 + 16];
  const int ntiles = g.tiles_m * g.tiles_n;
  if constexpr (MT == 16 && pp_kind<EK>()) {
    lds_vint* slot = DYN ? FER_LDS_INT(smem + 8 * 16384) : nullptr;
    int bid = DYN ? wq_first(ntiles) : ((int)blockIdx.x < ntiles ? (int)blockIdx.x : -1);
    if (bid < 0) return;
    {
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      pro_8ph<AKC, BKC, MT, EK>(g, bid, smem, __builtin_amdgcn_readfirstlane(tid >> 6), tid & 63);
    }
    auto run = [&](const auto& pe) {
      bid = tile_8ph_pp<AKC, BKC, MT, EK, false>(g, pe, bid, smem, slot);
#pragma unroll 1
      while (bid >= 0) bid = tile_8ph_pp<AKC, BKC, MT, EK, true>(g, pe, bid, smem, slot);
    };
    run(PpEpi{e.c, e.bias, (long)e.ldc, e.alpha});
  } else if constexpr (!DYN) {
    // the dropout seed mixed with the step counter once per launch, not in every tile's epilogue
    // (its global load and vmcnt(0) wait sat at the start of each epilogue)
    const uint64_t seed = e.drop_thresh ? step_seed(e.seed) : 0;
#pragma unroll 1
    for (int bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
      tile_8ph<AKC, BKC, MT, EK>(g, e, bid, smem, nullptr, seed);
      bar_lds();  // every wave is done with the epilogue's LDS before the next tile's DMA
    }
  } else {
    lds_vint* slot = FER_LDS_INT(smem + 8 * 16384);
    const uint64_t seed = e.drop_thresh ? step_seed(e.seed) : 0;
    int bid = wq_first(ntiles), par = 0;
#pragma unroll 1
    while (bid >= 0) {
      tile_8ph<AKC, BKC, MT, EK>(g, e, bid, smem, slot + par, seed);
      bar_lds();  // every wave is done with the epilogue's LDS before the next tile's DMA
      bid = __builtin_amdgcn_readfirstlane(slot[par]);
      par ^= 1;
    }
  }
}

// Ordered (deterministic) split-K reduction + epilogue.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long M, long N,
                                                           EpiArgs e) {
  const long n4 = N >> 2;
  const long total = M * n4;
  const uint64_t seed = e.drop_thresh ? step_seed(e.seed) : 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const long m = i / n4, n = (i - m * n4) * 4;
    f32x4 v = *(const f32x4*)(ws + m * N + n);
    for (int s = 1; s < splits; ++s) v += *(const f32x4*)(ws + (long)s * M * N + m * N + n);
    epi4<T>(e, m, n, v, seed);
  }
}

// fp32 parity path: 64x64 tile, BK 16, 256 threads x (4x4) outputs, exact fp32 FMA.
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g, EpiArgs e, int akc, int bkc) {
  __shared__ float As[16][68];
  __shared__ float Bs[16][68];
  const int t = threadIdx.x;
  const int tm = blockIdx.x / g.tiles_n, tn = blockIdx.x % g.tiles_n;
  const long m0 = tm * 64L, n0 = tn * 64L;
  const float* A = (const float*)g.A;
  const float* B = (const float*)g.B;
  float acc[4][4] = {};
  const int ty = t >> 4, tx = t & 15;
  const uint64_t seed = e.drop_thresh ? step_seed(e.seed) : 0;
  for (int k0 = 0; k0 < g.K; k0 += 16) {
    for (int i = t; i < 16 * 64; i += 256) {
      int kk, mm;
      if (akc) { mm = i >> 4; kk = i & 15; } else { kk = i >> 6; mm = i & 63; }
      const long m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < g.M && k < g.K) ? (akc ? A[m * g.lda + k] : A[k * g.lda + m]) : 0.f;
      int nn;
      if (bkc) { nn = i >> 4; kk = i & 15; } else { kk = i >> 6; nn = i & 63; }
      const long n = n0 + nn, k2 = k0 + kk;
      Bs[kk][nn] = (n < g.N && k2 < g.K) ? (bkc ? B[n * g.ldb + k2] : B[k2 * g.ldb + n]) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { a[r] = As[kk][ty * 4 + r]; b[r] = Bs[kk][tx * 4 + r]; }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(a[r], b[c], acc[r][c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long m = m0 + ty * 4 + r, n = n0 + tx * 4;
    if (m < g.M && n < g.N) epi4<float>(e, m, n, f32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]}, seed);
  }
}

// ============================================================ grouped weight gradients
// dW_i (+)= dY_i^T X_i for the weight gradients of one encoder layer in ONE launch (fer_wgrad_group):
// the small-token configurations (w+ latents: 4,864 rows, 48 px images: 640) have 16-64 output tiles
// per weight, so each weight gradient alone needed split-K (fp32 slabs + a separate ordered
// reduction launch) and still ran latency-bound (a 10 GF GEMM in ~40 us). Grouped, the layer's
// 100-200 128x128 tiles fill the chip with little or no K split. Both operands are MN-contiguous
// (token rows), read by LDS-DMA into an NST-slot ring of BK=64 stages, ds_read_b64_tr_b16
// fragments, v_mfma_f32_16x16x32_bf16, 2 x WN waves. Output written straight from the accumulators
// (fp32 rows of 4, accumulate optional).
// K split (splits > 1): every split writes its partial tile to a tile-local fp32 slab with
// write-through (sc1) stores, drains them, and takes a ticket from the tile's counter (agent-scope
// atomic, zeroed by the host per launch); the split that draws the last ticket sums the tile's
// slabs in split order -- its own partial from registers at its own position, the others by sc1
// loads -- and writes dW (MI355X_MICROARCH.md, Workgroup dispatch: the sc1-store / counter /
// sc1-load hand-off, one workgroup per CU). Deterministic for any arrival order.
constexpr int WG_MAX = 8;
struct WgItem {
  const bf16* A;  // dY [K tokens][M], row stride lda
  const bf16* B;  // X  [K tokens][N], row stride ldb
  float* C;       // dW [M][N], row stride ldc
  long lda, ldb, ldc;
  int M, N, tiles_m, tile0, acc;
};
struct WgGroup {
  WgItem it[WG_MAX];
  int n, K, splits, k_chunk;
  unsigned* cnt;  // [tiles] tickets (zeroed by the host before the launch)
  float* slab;    // [tiles][splits][128*128]
};

template <int NST, int WN>
__global__ __launch_bounds__(128 * WN, 1) void gemm_wgrad_group_kernel(WgGroup grp) {
  constexpr int BM = 128, BN = 128, NW = 2 * WN, MT = 16, TM = 64, TN = 128 / WN, FM = TM / MT, FN = TN / MT;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE + 16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;  // 2 x WN waves of 64 x TN
  const int tl = blockIdx.x, ks = blockIdx.y;
  int ii = 0;
#pragma unroll
  for (int i = 1; i < WG_MAX; ++i)
    if (i < grp.n && tl >= grp.it[i].tile0) ii = i;
  const WgItem& it = grp.it[ii];
  const int t = tl - it.tile0;
  const int tm = t % it.tiles_m, tn = t / it.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks * grp.k_chunk;
  const int kend = min(grp.K, kbeg + grp.k_chunk);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int ktail = kbeg + (nk - 1) * BK;

  const u32x4 ra = rsrc4(it.A);
  const u32x4 rb = rsrc4(it.B);
  typedef DmaPlan<BM, false, NW, MT> PA;
  typedef DmaPlan<BN, false, NW, MT> PB;
  PA pa;
  PB pb;
  pa.init(wave, lane, it.lda, m0, it.M);
  pb.init(wave, lane, it.ldb, n0, it.N);
  constexpr int PER = PA::NI + PB::NI;  // DMA instructions per stage per wave
  auto slot = [&](int st) -> char* { return smem + (st % NST) * STAGE; };
  auto issue = [&](int st) {
    const int k0 = kbeg + st * BK;
    pa.issue(ra, slot(st), wave, it.lda, k0, kend, k0 == ktail);
    pb.issue(rb, slot(st) + A_BYTES, wave, it.ldb, k0, kend, k0 == ktail);
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) issue(st);
  for (int k = 0; k < nk; ++k) {
    // stage k landed (this wave's pieces); up to NST-2 later stages stay in flight
    const int ahead = min(NST - 2, nk - 1 - k);
    if constexpr (NST >= 4) {
      if (ahead >= 2) wait_vm<2 * PER>();
      else if (ahead == 1) wait_vm<PER>();
      else wait_vm<0>();
    } else if constexpr (NST == 3) {
      if (ahead >= 1) wait_vm<PER>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    // every wave's pieces of stage k are in LDS, and every wave is done with stage k-1's slot
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (k + NST - 1 < nk) issue(k + NST - 1);
    const char* cur = slot(k);
    bf16x8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < FN; ++i) bfr[kk][i] = read_frag<MT, BN, false>(cur + A_BYTES, wn * TN + i * MT, kk, lane);
#pragma unroll
      for (int j = 0; j < FM; ++j) af[kk][j] = read_frag<MT, BM, false>(cur, wm * TM + j * MT, kk, lane);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) acc[i][j] = mfma<MT>(bfr[kk][i], af[kk][j], acc[i][j]);
  }

  // accumulator (i, j): rows m0 + wm*64 + 16j + (lane & 15), columns n0 + wn*64 + 16i + 4(lane >> 4) + 0..3
  const int lr = lane & 15, lc = 4 * (lane >> 4);
  if (grp.splits > 1) {
    const int S = grp.splits;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(grp.slab + (long)tl * S * (BM * BN));
    auto soff = [&](int sp, int i, int j) -> uint32_t {
      return (uint32_t)(((sp * BM + wm * TM + j * MT + lr) * BN + wn * TN + i * MT + lc) * 4);
    };
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, acc[i][j]), rs, soff(ks, i, j), 0, 16 /* sc1: write-through */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drained
    __syncthreads();
    lds_vuint* flag = FER_LDS_UINT(smem + NST * STAGE);
    if (threadIdx.x == 0) {
      // the sc1 stores are write-through and drained: no release needed (MI355X_MICROARCH.md). The
      // last split also takes an agent-scope acquire before its sc1 loads: the sc1-only hand-off
      // is measured at one workgroup per CU, this kernel runs two (a release on every producer
      // measured +5 us per launch and is not needed for write-through stores).
      const unsigned tk = __hip_atomic_fetch_add(grp.cnt + tl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tk == (unsigned)(S - 1)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = tk;
    }
    __syncthreads();
    if (*flag != (unsigned)(S - 1)) return;  // not the last split of this tile
    // last split: slabs in split order (sc1 loads: every load of the handed-off bytes)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int sp = 0; sp < S; ++sp) {
          const f32x4 v = sp == ks ? acc[i][j]
                                   : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, soff(sp, i, j), 0, 16));
          sum = sp == 0 ? v : sum + v;
        }
        acc[i][j] = sum;
      }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const long m = m0 + wm * TM + j * MT + lr, n = n0 + wn * TN + i * MT + lc;
      if (m < it.M && n < it.N) {
        f32x4* c = (f32x4*)(it.C + m * it.ldc + n);
        *c = it.acc ? *c + acc[i][j] : acc[i][j];
      }
    }
}

// -------------------------------------------------------------------- launch
template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT>
static int launch_bf16(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  dim3 grid(g.tiles_m * g.tiles_n, g.splits);
#define FER_BF16K(K) \
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, AKC, BKC, MT, K>), grid, dim3(64 * WM * WN), 0, st, g, e)
  // the 128^2 K-contiguous MT16 kernel (the small-grid configs: w+ latents, 48 px) also gets the
  // fixed-flag epilogues (row operands through its LDS-DMA staging: the LDS-DMA kinds)
  if constexpr (BM == 128 && (BN == 128 || BN == 64) && AKC && BKC && MT == 16) {
    int ek = g.partial ? EPI_GEN : epi_kind(e, g.M, g.N);
    if (ek == EPI_RES2) ek = EPI_RES;
    if (ek == EPI_MUL2) ek = EPI_MUL;
    switch (ek) {
      case EPI_STORE: FER_BF16K(EPI_STORE); break;
      case EPI_GATE: FER_BF16K(EPI_GATE); break;
      case EPI_GATER: FER_BF16K(EPI_GATER); break;
      case EPI_RES: FER_BF16K(EPI_RES); break;
      case EPI_MUL: FER_BF16K(EPI_MUL); break;
      default: FER_BF16K(EPI_GEN); break;
    }
  } else {
    FER_BF16K(EPI_GEN);
  }
#undef FER_BF16K
  return 0;
}

template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT>
static int launch_ring(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  dim3 grid(g.tiles_m * g.tiles_n, g.splits);
  hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, WM, WN, AKC, BKC, MT, 4>), grid, dim3(64 * WM * WN), 0, st, g, e);
  return 0;
}



template <bool AKC, bool BKC, int MT>
static int launch_8ph(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  // fixed-flag epilogues for the K-contiguous MT16 kernel (the forward and transposed-shadow dgrad path)
  const int ek = (AKC && BKC && MT == 16 && !g.partial) ? epi_kind(e, g.M, g.N) : EPI_GEN;
  g.tiles_m = (g.M + 255) / 256;
  g.tiles_n = (g.N + 255) / 256;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  // persistent grid: one workgroup per CU (a multiple of 8: the XCD-aware tile order)
  const int ntiles = g.tiles_m * g.tiles_n;
  const int gx = std::min(ntiles, std::max(8, ncu / 8 * 8));
  g.tq = nullptr;
  WqArgs w{};
  if (!fixed_stride_mode() && g.splits == 1) {
    w = wq_prepare_here(st, gx, ntiles);
    g.tq = w.q;
    for (int c = 0; c < 8; ++c) g.tq_base[c] = w.base[c];
  }
  dim3 grid(gx, g.splits);
#define FER_8PH(DY, K) hipLaunchKernelGGL((gemm_8ph_kernel<AKC, BKC, MT, DY, K>), grid, dim3(512), 0, st, g, e)
#define FER_8PH_K(DY)                                  \
  if constexpr (AKC && BKC && MT == 16) {              \
    switch (ek) {                                      \
      case EPI_STORE: FER_8PH(DY, EPI_STORE); break;   \
      case EPI_GATE: FER_8PH(DY, EPI_GATE); break;     \
      case EPI_GATER: FER_8PH(DY, EPI_GATER); break;   \
      case EPI_RES2: FER_8PH(DY, EPI_RES2); break;     \
      case EPI_MUL2: FER_8PH(DY, EPI_MUL2); break;     \
      default: FER_8PH(DY, EPI_GEN); break;            \
    }                                                  \
  } else {                                             \
    FER_8PH(DY, EPI_GEN);                              \
  }
  if (g.tq) {
    FER_8PH_K(true)
  } else {
    FER_8PH_K(false)
  }
#undef FER_8PH_K
#undef FER_8PH
  wq_check_launch(st, w);
  return 0;
}

#ifdef FER_GEMM_STAMPS
extern "C" int fer_debug_gemm_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
extern "C" int fer_debug_gemm_ep_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_epst), sizeof(unsigned long long) * 32) == hipSuccess ? 0 : 1;
}
#endif

// Round fill of a grid: tiles / (rounds x slots), slots = CUs x workgroups per CU (128^2: 2 by LDS,
// 128x64: 3). The 128x64 tiles win where they fill the rounds clearly better (by 0.15 at short K,
// where their extra per-tile prologue / epilogue weighs more).
static bool use_128x64(long t128, long t64, int K) {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  auto fill = [](long t, long slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
  return fill(t64, 3L * ncu) > fill(t128, 2L * ncu) + (K < 1024 ? 0.15 : 0.0);
}

static int g_forced_cfg = -1;  // fer_gemm_set_config; -1: automatic

static int forced_cfg() { return g_forced_cfg; }

// Tile configuration: 0..3 double-buffered (256^2 MT32, 256^2 MT16, 128^2 MT32, 128^2 MT16),
// 4..7 BK=32 ring (same order), 8/9 the 8-phase 256^2 kernel (MT16 / MT32), 10 the ping-pong
// 256x128 kernel (two workgroups per CU), 11 double-buffered 128x64 MT16.
static bool cfg_is_256(int c) { return c == 0 || c == 1 || c == 4 || c == 5 || c == 8 || c == 9 || c == 10; }

template <bool AKC, bool BKC>
static int dispatch_tile(int cfg, GemmArgs g, const EpiArgs& e, hipStream_t st) {
  switch (cfg) {
    case 0: return launch_bf16<256, 256, 2, 4, AKC, BKC, 32>(g, e, st);
    case 1: return launch_bf16<256, 256, 2, 4, AKC, BKC, 16>(g, e, st);
    case 2: return launch_bf16<128, 128, 2, 2, AKC, BKC, 32>(g, e, st);
    case 3: return launch_bf16<128, 128, 2, 2, AKC, BKC, 16>(g, e, st);
    case 4: return launch_ring<256, 256, 2, 4, AKC, BKC, 32>(g, e, st);
    case 5: return launch_ring<256, 256, 2, 4, AKC, BKC, 16>(g, e, st);
    case 6: return launch_ring<128, 128, 2, 2, AKC, BKC, 32>(g, e, st);
    case 7: return launch_ring<128, 128, 2, 2, AKC, BKC, 16>(g, e, st);
    case 9: return launch_8ph<AKC, BKC, 32>(g, e, st);
    case 10: return launch_pp<AKC, BKC>(g, e, st);
    case 11:  // (the MN-contiguous image swizzle needs >= 128-wide tiles: an MN B operand keeps 128^2)
      if constexpr (BKC) return launch_bf16<128, 64, 2, 2, AKC, BKC, 16>(g, e, st);
      else return launch_bf16<128, 128, 2, 2, AKC, BKC, 16>(g, e, st);
    default: return launch_8ph<AKC, BKC, 16>(g, e, st);
  }
}

int gemm_launch(const GemmDesc& d, const EpiArgs& e_in, hipStream_t st) {
  EpiArgs e = e_in;
  GemmArgs g{};
  g.A = d.A; g.B = d.B; g.lda = d.lda; g.ldb = d.ldb;
  g.M = d.M; g.N = d.N; g.K = d.K;
  if (d.M <= 0 || d.N <= 0) return 0;
  if (d.N % 4) return set_error("gemm: N must be a multiple of 4");
  if (e.colsum && (!d.ws || d.ws_bytes < fer_gemm_colsum_ws(d.M, d.N)))
    return set_error("gemm: fused column sums need the desc workspace (fer_gemm_colsum_ws bytes)");
  // column sums of the output by a separate pass (fp32 parity path)
  auto colsum_pass = [&]() -> int {
    return fer_colsum(e.c_f32 ? FER_F32 : d.dtype, e.c, e.ldc, d.M, d.N, e.colsum, e.colsum_accumulate, nullptr,
                      d.ws, d.ws_bytes, (fer_stream_t)st);
  };
  if (d.dtype == FER_F32) {
    g.tiles_m = (d.M + 63) / 64;
    g.tiles_n = (d.N + 63) / 64;
    g.splits = 1;
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(g.tiles_m * g.tiles_n), dim3(256), 0, st, g, e, d.a_kc, d.b_kc);
    int rc = hip_check("gemm_f32");
    return (rc || !e.colsum) ? rc : colsum_pass();
  }
  // bf16: alignment contract of the DMA staging (16-byte chunks)
  if ((d.a_kc && (d.K % 8 || d.lda % 8)) || (!d.a_kc && (d.M % 8 || d.lda % 8)))
    return set_error("gemm: A layout needs 8-element aligned rows");
  if ((d.b_kc && (d.K % 8 || d.ldb % 8)) || (!d.b_kc && (d.N % 8 || d.ldb % 8)))
    return set_error("gemm: B layout needs 8-element aligned rows");
  // epilogue row operand (res / aux) is fetched by 16-byte LDS-DMA pieces
  if (check_drop_range(e.drop_thresh, (long)d.M * e.drop_ld, "gemm: dropout over >= 2^32 elements")) return -1;
  // The tile epilogue works on 16-byte row pieces (8 bf16): output, pre-activation and the
  // res / aux operand (fetched by LDS-DMA) need 8-element aligned rows.
  auto al8 = [](const void* p, long ld) { return !p || (ld % 8 == 0 && (uintptr_t)p % 16 == 0); };
  if (d.N % 8 || !al8(e.c, e.ldc) || !al8(e.pre, e.ldp) || !al8(e.res, e.ldr) || !al8(e.aux, e.ldx))
    return set_error("gemm: bf16 path needs N and every epilogue row stride multiples of 8 (16-byte aligned rows)");
  const long a_bytes = (d.a_kc ? (long)(d.M - 1) * d.lda + d.K : (long)(d.K - 1) * d.lda + d.M) * 2;
  const long b_bytes = (d.b_kc ? (long)(d.N - 1) * d.ldb + d.K : (long)(d.K - 1) * d.ldb + d.N) * 2;
  if (a_bytes >= 0x7FFFFFF0L || b_bytes >= 0x7FFFFFF0L) return set_error("gemm: operand exceeds 2 GiB");

  // Configuration (measured on MI355X, tools/gemm_bench.py, tools/gemm_small_bench.py): the
  // 8-phase 256^2 kernel for grids of >= 256 such tiles or K >= 8192 (the BK=32 ring for the
  // MN x MN weight gradient: 261 vs 283 us on fc1); grids smaller than the CU count (the latent
  // w+ and 48 px configs) run 128^2 tiles at two blocks per CU (latent fc2 fwd 37 vs 45 us).
  // Split-K (weight gradients, K = tokens) targets one 256^2 workgroup per CU.
  const long t256 = (long)((d.M + 255) / 256) * ((d.N + 255) / 256);
  const long t128 = (long)((d.M + 127) / 128) * ((d.N + 127) / 128);
  // (fused column sums use the workspace for their tile partials: no split-K then)
  const int max_splits = (d.ws && !e.colsum) ? (int)std::min<long>(64, d.ws_bytes / ((long)d.M * d.N * 4)) : 1;
  auto splits_for = [&](long tiles, long target) -> int {
    if (max_splits < 2 || d.K < 1024 || tiles >= target) return 1;
    return (int)std::max<long>(1, std::min<long>({target / tiles, d.K / 256, (long)max_splits}));
  };
  // split targets (workgroups per launch) of the 256^2 / 128^2 tile configs
  // (MN x MN weight gradients: 224 workgroups, not one per CU -- they run beside the compute stream,
  // and leaving it CUs took the ViT-B step 36.06-36.33 -> 35.81-36.02 ms at 192; 128 is 39 ms: the last
  // layers' weight gradients then form a long tail; profiles/r03aa_wgrad_split_target_ab.txt. With the
  // round-4 compute-stream kernels 224 is 35.91 / 35.92 vs 192 35.98 / 36.04 and 160 36.04 / 36.07 ms,
  // profiles/r04ac_wgrad_split_target_ab.txt)
  constexpr long tgt256 = 256, tgt256_mn = 224;
  // (128^2, K-contiguous: split only below half a round; the ordered slab reduction costs more than the
  // idle CUs of an unsplit 152-228 tile grid -- latent fc2 fwd 50.7 -> 29.4 us, qkv dgrad 46.4 -> 22.9 us)
  const long tgt128k = (d.a_kc && d.b_kc) ? 256 : 512;
  int cfg = forced_cfg();
  if (cfg < 0) {
    if (d.K >= 8192 || t256 >= 256)  // big grids, and token-long weight gradients (split-K fills the GPU)
      // (MN x MN weight gradients split >= 16 ways -- out_proj / patch embed, 9 tiles x 28 splits --
      // run 97.7 -> 74.1 us alone on the MT32 ring, but the ViT-B step got 0.1-0.3 ms SLOWER with
      // it on the weight-gradient stream (profiles/r03x_*, r03z_*): the MT16 ring stays)
      cfg = t256 * splits_for(t256, tgt256) >= 128 ? (!d.a_kc && !d.b_kc ? 5 : 8) : 3;
    else if (d.a_kc && d.b_kc && t128 >= 128 && use_128x64(t128, (long)((d.M + 127) / 128) * ((d.N + 63) / 64), d.K))
      // 128x64 tiles (three workgroups per CU) where they fill the rounds better: latent fc2 fwd /
      // fc1 dgrad (152 tiles of 128^2, K 2048) 28.5 / 27.4 -> 25.4 / 24.3 us, fc1 fwd (608 tiles)
      // 27.4 -> 24.4 us; qkv fwd (456 tiles, 0.89 of a 128^2 round) stays (15.0 vs 17.6 us)
      cfg = 11;
    else  // fewer 256^2 tiles than CUs (latent / 48 px configs): 128^2 tiles, two workgroups per CU
      cfg = 3;
  }
  int splits = cfg_is_256(cfg) ? splits_for(t256, (!d.a_kc && !d.b_kc) ? tgt256_mn : tgt256) : splits_for(t128, tgt128k);
  g.splits = splits;
  g.k_chunk = splits > 1 ? (((d.K + splits - 1) / splits + BK - 1) / BK) * BK : d.K;
  if (splits > 1) g.splits = (d.K + g.k_chunk - 1) / g.k_chunk;
  g.partial = g.splits > 1;
  g.ws = d.ws;
  g.cs_part = e.colsum ? reduction_ws(d.ws, (size_t)((d.M + (cfg_is_256(cfg) ? 255 : 127)) / (cfg_is_256(cfg) ? 256 : 128)) * d.N * 4,
                                      d.N, st)
                       : nullptr;
  if (d.a_kc && d.b_kc) dispatch_tile<true, true>(cfg, g, e, st);
  else if (d.a_kc && !d.b_kc) dispatch_tile<true, false>(cfg, g, e, st);
  else if (!d.a_kc && !d.b_kc) dispatch_tile<false, false>(cfg, g, e, st);
  else dispatch_tile<false, true>(cfg, g, e, st);
  int rc = hip_check("gemm_bf16");
  if (!rc && e.colsum) {  // fixed-order reduction of the per-tile column partials
    const int bm = cfg_is_256(cfg) ? 256 : 128;
    part_reduce(g.cs_part, (d.M + bm - 1) / bm, d.N, d.N, d.N, e.colsum, nullptr, nullptr, e.colsum_accumulate,
                nullptr, st);
    rc = hip_check("gemm_colsum_reduce");
  }
  if (rc || !g.partial) return rc;
  const long work = (long)d.M * (d.N / 4);
  const int blocks = (int)std::min<long>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel<bf16>, dim3(blocks), dim3(256), 0, st, d.ws, g.splits, (long)d.M,
                     (long)d.N, e);
  return hip_check("splitk_reduce");
}

// ---- grouped weight gradients (fer_wgrad_group)
namespace {
int wg_splits(int tiles, int K, int req) {
  if (req > 0) return std::min(req, 8);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  // two 64 KB-ring workgroups per CU: split K while the grid stays within one round of those
  return std::max(1, std::min({2 * ncu / std::max(1, tiles), K / 1024, 8}));
}
long wg_tiles(const fer_wgrad_item* it, int n) {
  long t = 0;
  for (int i = 0; i < n; ++i) t += (long)((it[i].N + 127) / 128) * ((it[i].K + 127) / 128);
  return t;
}
}  // namespace
}  // namespace fer

extern "C" int64_t fer_wgrad_group_ws(const fer_wgrad_item* items, int n, int splits) {
  if (!items || n <= 0) return 0;
  const long tiles = fer::wg_tiles(items, n);
  const int S = fer::wg_splits((int)tiles, items[0].M, splits);
  return S > 1 ? tiles * S * 128 * 128 * 4 + tiles * 4 + 64 : 0;
}

extern "C" int fer_wgrad_group(const fer_wgrad_item* items, int n, int splits, float* ws, int64_t ws_bytes,
                               fer_stream_t stream) {
  using namespace fer;
  if (n <= 0) return 0;
  if (!items || n > WG_MAX) return set_error("wgrad_group: 1..8 items");
  hipStream_t st = (hipStream_t)stream;
  WgGroup g{};
  g.n = n;
  g.K = items[0].M;
  int tile0 = 0;
  for (int i = 0; i < n; ++i) {
    const fer_wgrad_item& x = items[i];
    if (x.M != g.K) return set_error("wgrad_group: every item needs the same token count M");
    if (x.M <= 0 || x.N <= 0 || x.K <= 0) return set_error("wgrad_group: empty item");
    if (x.N % 8 || x.K % 8 || x.ld_dy % 8 || x.ld_x % 8 || x.ld_dw % 4 || x.ld_dy < x.N || x.ld_x < x.K ||
        x.ld_dw < x.K || (uintptr_t)x.dy % 16 || (uintptr_t)x.x % 16 || (uintptr_t)x.dw % 16)
      return set_error("wgrad_group: N, K and the row strides need 8-element (16-byte) alignment");
    if ((long)(x.M - 1) * x.ld_dy * 2 + 2L * x.N >= 0x7FFFFFF0L || (long)(x.M - 1) * x.ld_x * 2 + 2L * x.K >= 0x7FFFFFF0L)
      return set_error("wgrad_group: operand exceeds 2 GiB");
    WgItem& w = g.it[i];
    w.A = (const bf16*)x.dy; w.lda = x.ld_dy;
    w.B = (const bf16*)x.x; w.ldb = x.ld_x;
    w.C = x.dw; w.ldc = x.ld_dw;
    w.M = x.N; w.N = x.K;
    w.tiles_m = (x.N + 127) / 128;
    w.tile0 = tile0;
    w.acc = x.accumulate;
    tile0 += w.tiles_m * ((x.K + 127) / 128);
  }
  int S = wg_splits(tile0, g.K, splits);
  g.splits = S;
  g.k_chunk = S > 1 ? ((g.K + S - 1) / S + BK - 1) / BK * BK : g.K;
  if (S > 1) {
    g.splits = S = (g.K + g.k_chunk - 1) / g.k_chunk;
    const long need = (long)tile0 * S * 128 * 128 * 4 + (long)tile0 * 4;
    if (!ws || ws_bytes < need) return set_error("wgrad_group: workspace smaller than fer_wgrad_group_ws()");
    g.slab = ws;
    g.cnt = (unsigned*)((char*)ws + (long)tile0 * S * 128 * 128 * 4);
    if (hipMemsetAsync(g.cnt, 0, (size_t)tile0 * 4, st) != hipSuccess) return set_error("wgrad_group: memset failed");
  }
  // Shipped: 4 waves of 64x64, 2-slot ring (64 KB: two workgroups per CU, whose stage latencies
  // interleave), K split to ~2 workgroups per CU. Latent-ViT layer (4 weights, 192 tiles, K 4864):
  // 57 us vs 74-77 us for the 4-slot ring (one workgroup per CU) with 4 or 8 waves at any split,
  // and 189 us as four split-K launches (profiles/r03o_wgrad_group_variants.txt).
  hipLaunchKernelGGL((gemm_wgrad_group_kernel<2, 2>), dim3(tile0, S), dim3(256), 0, st, g);
  return hip_check("wgrad_group");
}

namespace fer {

}  // namespace fer

int fer::set_step_ptr_gemm(const uint64_t* p) { return set_step_ptr_here(p) == hipSuccess ? 0 : -1; }

extern "C" int64_t fer_gemm_colsum_ws(int M, int N) {
  // tile partials (128-row tiles at most) or the stand-alone colsum pass's partials
  return (int64_t)std::max(fer::ceil_div(std::max(M, 1), 128), 256) * N * 4;
}



extern "C" int fer_gemm_set_config(int cfg) {
  if (cfg < -1 || cfg > 11) return fer::set_error("gemm_set_config: cfg must be -1 (automatic) or 0..11");
  fer::g_forced_cfg = cfg;
  return 0;
}
