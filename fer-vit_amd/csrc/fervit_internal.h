// Internal host/device declarations shared by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include "../../include/fervit.h"

namespace fer {

typedef fer_epilogue EpiArgs;
typedef fer_gemm_desc GemmDesc;

struct GemmArgs {
  const void* A;
  const void* B;
  long lda, ldb;
  int M, N, K;
  int tiles_m, tiles_n;
  int splits, k_chunk, partial;
  float* ws;
  float* cs_part;  // fused column sums: per-tile partials [tiles_m][N] (or null)
  int* tq;               // persistent 8-phase kernel: work-queue counters (common.h wq_*), null = fixed stride
  unsigned tq_base[8];   // their values at launch
};

int set_error(const char* msg);
// per-code-object setters of the device step-counter pointer (common.h step_seed)
int set_step_ptr_gemm(const uint64_t* p);
int set_step_ptr_attention(const uint64_t* p);
int set_step_ptr_layernorm(const uint64_t* p);
int set_step_ptr_misc(const uint64_t* p);
int hip_check(const char* what);
// persistent GEMM / attention kernels: walk a fixed blockIdx stride instead of the work queue
// (fer_set_persistent_mode(1))
bool fixed_stride_mode();
int gemm_launch(const GemmDesc& d, const EpiArgs& e, hipStream_t st);
inline int ceil_div(long a, long b);
// out_k[c % seg] (+)= scale * sum_b part[b*ld + c]  (deterministic, misc.hip)
void part_reduce(const float* part, int nb, long ld, int ncols, int seg, float* o0, float* o1, float* o2,
                 int accumulate, const float* scale, hipStream_t st);
// Workspace for column partials that part_reduce will sum: inside fer_reduce_defer's window (same
// stream, a shape the batched reduction takes) a slice of the deferral arena, else ws itself (misc.hip)
float* reduction_ws(float* ws, size_t bytes, int ncols, hipStream_t st);

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Dropout element indices are 32-bit (common.h fer_hash): a dropout site covers < 2^32 elements.
inline int check_drop_range(uint32_t thresh, long elements, const char* what) {
  if (thresh && elements > 0xFFFFFFFFL) return set_error(what);
  return 0;
}

}  // namespace fer
