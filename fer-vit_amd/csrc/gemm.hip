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

#include "common.h"
#include "fervit_internal.h"

namespace fer {

// ------------------------------------------------------------------- epilogue
template <typename T>
FER_DEV void epi4(const EpiArgs& e, long m, long n, f32x4 v) {
  v *= e.alpha;
  if (e.bias) v += *(const f32x4*)(e.bias + n);
  if (e.pre) store4<T>((T*)e.pre + m * e.ldp + n, v);
  if (e.act) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_fwd(e.act, v[r]);
  }
  if (e.drop_thresh) drop4(e.seed, (uint64_t)m * (uint64_t)e.drop_ld + (uint64_t)n, e.drop_thresh, e.drop_scale, v);
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
FER_DEV void tile_of(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  int wgid = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int g = wgid / per_group;
  const int first = g * GROUP;
  const int gsize = min(tiles_m - first, GROUP);
  const int w = wgid - g * per_group;
  tm = first + w % gsize;
  tn = w / gsize;
}

// ------------------------------------------------------------- LDS-DMA stage
constexpr int BK = 64;
FER_DEV int kc_swz(int row) { return (row >> 1) & 7; }

// Per-lane DMA source offsets of this wave's pieces, computed once per tile; an
// out-of-range row/column gets base FER_OOB so voffset = base + k-advance stays out of range
// (one add per piece per K-step). For KC the K-step adds k0*2 bytes, for MN the wave-uniform
// k0*ld*2. `kof` (the lane's K inside the stage) is checked only on a partial last K-step.
// MN tr-read image swizzle (16-byte chunk XOR by K row), see read_frag.
template <int MT> FER_DEV int mn_swz_t(int k) {
  if constexpr (MT == 32) return (k & 3) << 2;               // 4 rows x 64 B per 32-lane half
  else return ((k & 3) | (((k >> 3) & 1) << 2)) << 1;       // 8 rows x 32 B per 32-lane half
}

template <int R, bool KC, int NW, int MT>
struct DmaPlan {
  static constexpr int NI = R * BK * 2 / 1024 / NW;
  static_assert(NI * NW * 1024 == R * BK * 2, "tile/wave mismatch");
  uint32_t base[NI];
  int kof[NI];
  FER_DEV void init(int wave, int lane, long ld, int r0, int rmax) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int gi = wave * NI + i;
      bool ok;
      uint32_t off;
      if constexpr (KC) {
        const int row = gi * 8 + (lane >> 3);
        const int c = (lane & 7) ^ kc_swz(row);
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
  FER_DEV void issue(__amdgpu_buffer_rsrc_t rs, char* lds_tile, int wave, long ld, int k0, int kmax,
                     bool tail) const {
    const uint32_t kadd = KC ? (uint32_t)(k0 * 2) : (uint32_t)(k0 * ld * 2);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t voff = (!tail || k0 + kof[i] < kmax) ? base[i] + kadd : FER_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds_tile + (wave * NI + i) * 1024), 16, voff, 0, 0,
                                               0);
    }
  }
};

// MFMA operand fragments. MT = 32: v_mfma_f32_32x32x16_bf16, lane l holds index i0 + (l&31),
// k = 16kk + 8(l>>5) + j. MT = 16: v_mfma_f32_16x16x32_bf16, lane l holds index i0 + (l&15),
// k = 32kk + 8(l>>4) + j (j = 0..7). KC images are read with ds_read_b128, MN images with two
// ds_read_b64_tr_b16 (rows k..k+3 and k+4..k+7 of 16 consecutive indices).

template <int MT, int R, bool KC>
FER_DEV bf16x8 read_frag(const char* lds_tile, int i0, int kk, int lane) {
  if constexpr (KC) {
    const int row = i0 + (MT == 32 ? (lane & 31) : (lane & 15));
    const int ch = MT == 32 ? 2 * kk + (lane >> 5) : 4 * kk + (lane >> 4);
    return *(const bf16x8*)(lds_tile + row * 128 + ((ch ^ kc_swz(row)) << 4));
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
    bf16x4 b1 = __builtin_bit_cast(bf16x4, t1), b2 = __builtin_bit_cast(bf16x4, t2);
    return bf16x8{b1[0], b1[1], b1[2], b1[3], b2[0], b2[1], b2[2], b2[3]};
  }
}

template <int N>
FER_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MT> struct Acc;
template <> struct Acc<32> { typedef f32x16 T; };
template <> struct Acc<16> { typedef f32x4 T; };

template <int MT>
FER_DEV typename Acc<MT>::T mfma(bf16x8 a, bf16x8 b, typename Acc<MT>::T c) {
  if constexpr (MT == 32) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Wave grid WM x WN over a BM x BN tile; each wave owns (BM/WM) x (BN/WN) as MT x MT MFMA
// blocks. The MFMA is issued with the B fragment as the instruction's A operand, so the
// accumulator's column index is m: for MT=32, lane l holds m = l&31 and n = 8q + 4(l>>5) + r
// (q, r = 0..3); for MT=16, m = l&15 and n = 4(l>>4) + r.
// Double-buffered BK=64 stages. Per K-step t: all LDS-DMA pieces of stage t+1, then SS
// substeps of  ds_read(t, kk+1) | MFMAs(t, kk); then vmcnt(0) + s_barrier hands t+1 over.
template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT>
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

  int tm, tn;
  tile_of(blockIdx.x, g.tiles_m, g.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ks = blockIdx.y;
  const int kbeg = ks * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.B);
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
    if (more && !(g.dbg & 1)) {
      pa.issue(ra, nxt, wave, g.lda, k1, kend, k1 == ktail);
      pb.issue(rb, nxt + A_BYTES, wave, g.ldb, k1, kend, k1 == ktail);
    }
#pragma unroll
    for (int kk = 0; kk < SS; ++kk) {
      bf16x8 an[FM], bn[FN];
      if (kk < SS - 1 && !(g.dbg & 8)) {
#pragma unroll
        for (int i = 0; i < FN; ++i) bn[i] = read_frag<MT, BN, BKC>(cur + A_BYTES, wn * TN + i * MT, kk + 1, lane);
#pragma unroll
        for (int j = 0; j < FM; ++j) an[j] = read_frag<MT, BM, AKC>(cur, wm * TM + j * MT, kk + 1, lane);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) acc[i][j] = mfma<MT>(bfr[i], af[j], acc[i][j]);
      if (kk < SS - 1 && !(g.dbg & 8)) {
#pragma unroll
        for (int i = 0; i < FN; ++i) bfr[i] = bn[i];
#pragma unroll
        for (int j = 0; j < FM; ++j) af[j] = an[j];
      }
    }
    if (more && !(g.dbg & 2)) {
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < FN; ++i) bfr[i] = read_frag<MT, BN, BKC>(nxt + A_BYTES, wn * TN + i * MT, 0, lane);
#pragma unroll
      for (int j = 0; j < FM; ++j) af[j] = read_frag<MT, BM, AKC>(nxt, wm * TM + j * MT, 0, lane);
    }
  }

  if (g.dbg & 4) {
    if (acc[0][0][0] == 12345.f) g.ws[0] = 1.f;  // keep the MFMAs alive
    return;
  }
  // ---- epilogue. Accumulator element (i, j, q, r) -> tile row/col:
  constexpr int NQ = MT == 32 ? 4 : 1;
  const int lr = MT == 32 ? (lane & 31) : (lane & 15);
  const int lc = MT == 32 ? 4 * (lane >> 5) : 4 * (lane >> 4);
  if (g.partial) {  // split-K partial slab, fp32 [split][M][N]
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
  // Stage each half of the tile (the rows of wave-row wm == h) through LDS as fp32 with padded
  // rows, then every thread applies the epilogue on 4 consecutive columns of one row: all
  // global traffic of the epilogue (bias, pre, residual, aux, output) is row-contiguous.
  float* ep = (float*)smem;
  constexpr int NT = 64 * NW;
  constexpr int C4 = BN / 4;  // float4 groups per row
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int r = j * MT + lr;
            const int c = wn * TN + i * MT + 8 * q + lc;
            *(f32x4*)(ep + r * ELD + c) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < EROWS * C4; idx += NT) {
      const int r = idx / C4, c = (idx - r * C4) * 4;
      const long m = m0 + h * EROWS + r, n = n0 + c;
      if (m < g.M && n < g.N) epi4<bf16>(e, m, n, *(const f32x4*)(ep + r * ELD + c));
    }
  }
}

// Ordered (deterministic) split-K reduction + epilogue.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long M, long N,
                                                           EpiArgs e) {
  const long n4 = N >> 2;
  const long total = M * n4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
    const long m = i / n4, n = (i - m * n4) * 4;
    f32x4 v = *(const f32x4*)(ws + m * N + n);
    for (int s = 1; s < splits; ++s) v += *(const f32x4*)(ws + (long)s * M * N + m * N + n);
    epi4<T>(e, m, n, v);
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
    if (m < g.M && n < g.N) epi4<float>(e, m, n, f32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
  }
}

// -------------------------------------------------------------------- launch
template <int BM, int BN, int WM, int WN, bool AKC, bool BKC, int MT>
static int launch_bf16(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  dim3 grid(g.tiles_m * g.tiles_n, g.splits);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, AKC, BKC, MT>), grid, dim3(64 * WM * WN), 0, st, g, e);
  return 0;
}

static int forced_cfg() {
  static int v = -2;
  if (v == -2) {
    const char* s = getenv("FERVIT_GEMM_CFG");
    v = s ? atoi(s) : -1;
  }
  return v;
}

template <bool AKC, bool BKC>
static int dispatch_tile(GemmArgs g, const EpiArgs& e, hipStream_t st) {
  switch (forced_cfg()) {
    case 0: return launch_bf16<256, 256, 2, 4, AKC, BKC, 32>(g, e, st);
    case 1: return launch_bf16<256, 256, 2, 4, AKC, BKC, 16>(g, e, st);
    case 2: return launch_bf16<128, 128, 2, 2, AKC, BKC, 32>(g, e, st);
    case 3: return launch_bf16<128, 128, 2, 2, AKC, BKC, 16>(g, e, st);
    default: break;
  }
  // measured on MI355X (tools/gemm_bench.py): 256^2 / 8 waves / 32x32x16 for the forward and
  // dgrad layouts when the grid fills the chip; 128^2 / 4 waves / 16x16x32 (2 blocks per CU)
  // for split-K weight gradients and small problems.
  const long t256 = ((g.M + 255) / 256) * ((g.N + 255) / 256) * (long)g.splits;
  if (AKC && t256 >= 200) return launch_bf16<256, 256, 2, 4, AKC, BKC, 32>(g, e, st);
  return launch_bf16<128, 128, 2, 2, AKC, BKC, 16>(g, e, st);
}

int gemm_launch(const GemmDesc& d, const EpiArgs& e_in, hipStream_t st) {
  EpiArgs e = e_in;
  GemmArgs g{};
  g.A = d.A; g.B = d.B; g.lda = d.lda; g.ldb = d.ldb;
  g.M = d.M; g.N = d.N; g.K = d.K;
  static const int dbg = getenv("FERVIT_GEMM_DBG") ? atoi(getenv("FERVIT_GEMM_DBG")) : 0;
  g.dbg = dbg;
  if (d.M <= 0 || d.N <= 0) return 0;
  if (d.N % 4) return set_error("gemm: N must be a multiple of 4");
  if (d.dtype == FER_F32) {
    g.tiles_m = (d.M + 63) / 64;
    g.tiles_n = (d.N + 63) / 64;
    g.splits = 1;
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(g.tiles_m * g.tiles_n), dim3(256), 0, st, g, e, d.a_kc, d.b_kc);
    return hip_check("gemm_f32");
  }
  // bf16: alignment contract of the DMA staging (16-byte chunks)
  if ((d.a_kc && (d.K % 8 || d.lda % 8)) || (!d.a_kc && (d.M % 8 || d.lda % 8)))
    return set_error("gemm: A layout needs 8-element aligned rows");
  if ((d.b_kc && (d.K % 8 || d.ldb % 8)) || (!d.b_kc && (d.N % 8 || d.ldb % 8)))
    return set_error("gemm: B layout needs 8-element aligned rows");
  const long a_bytes = (d.a_kc ? (long)(d.M - 1) * d.lda + d.K : (long)(d.K - 1) * d.lda + d.M) * 2;
  const long b_bytes = (d.b_kc ? (long)(d.N - 1) * d.ldb + d.K : (long)(d.K - 1) * d.ldb + d.N) * 2;
  if (a_bytes >= 0x7FFFFFF0L || b_bytes >= 0x7FFFFFF0L) return set_error("gemm: operand exceeds 2 GiB");

  // split-K when the output tiles alone cannot fill 256 CUs
  int splits = 1;
  const long tiles = ((d.M + 255) / 256) * ((d.N + 255) / 256);
  const long tiles128 = ((d.M + 127) / 128) * ((d.N + 127) / 128);
  if (d.ws && tiles < 200 && tiles128 < 256 && d.K >= 1024) {
    const long t = tiles128;
    splits = (int)std::min<long>((512 + t - 1) / t, d.K / 256);
    splits = std::max(1, std::min<int>(splits, (int)(d.ws_bytes / ((long)d.M * d.N * 4))));
  }
  g.splits = splits;
  g.k_chunk = splits > 1 ? (((d.K + splits - 1) / splits + BK - 1) / BK) * BK : d.K;
  if (splits > 1) g.splits = (d.K + g.k_chunk - 1) / g.k_chunk;
  g.partial = g.splits > 1;
  g.ws = d.ws;

  if (d.a_kc && d.b_kc) dispatch_tile<true, true>(g, e, st);
  else if (d.a_kc && !d.b_kc) dispatch_tile<true, false>(g, e, st);
  else if (!d.a_kc && !d.b_kc) dispatch_tile<false, false>(g, e, st);
  else dispatch_tile<false, true>(g, e, st);
  int rc = hip_check("gemm_bf16");
  if (rc || !g.partial) return rc;
  const long work = (long)d.M * (d.N / 4);
  const int blocks = (int)std::min<long>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel<bf16>, dim3(blocks), dim3(256), 0, st, d.ws, g.splits, (long)d.M,
                     (long)d.N, e);
  return hip_check("splitk_reduce");
}

}  // namespace fer
