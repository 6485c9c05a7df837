// C ABI glue: error state and the GEMM entry point.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fervit_internal.h"

namespace fer {

static thread_local char g_err[512] = "";

int set_error(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}

int hip_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -2;
  }
  return 0;
}

static int g_fixed_stride = [] {  // fer_set_persistent_mode; FERVIT_FIXED_STRIDE=1 at start-up (fervit.h)
  const char* v = getenv("FERVIT_FIXED_STRIDE");
  return v && v[0] == '1' ? 1 : 0;
}();

bool fixed_stride_mode() { return g_fixed_stride == 1; }

}  // namespace fer

extern "C" int fer_set_persistent_mode(int mode) {
  if (mode < 0 || mode > 1) return fer::set_error("set_persistent_mode: mode must be 0 (work queue) or 1 (fixed stride)");
  fer::g_fixed_stride = mode;
  return 0;
}

extern "C" const char* fer_last_error(void) { return fer::g_err; }
extern "C" const char* fer_version(void) { return "fervit-mi355x 0.1 (gfx950)"; }

extern "C" int fer_gemm(const fer_gemm_desc* d, const fer_epilogue* e, fer_stream_t stream) {
  if (!d || !e) return fer::set_error("gemm: null descriptor");
  return fer::gemm_launch(*d, *e, (hipStream_t)stream);
}

extern "C" int fer_set_step_counter(const uint64_t* counter) {
  // every code object that has dropout kernels keeps its own copy of the pointer
  if (fer::set_step_ptr_gemm(counter) || fer::set_step_ptr_attention(counter) ||
      fer::set_step_ptr_layernorm(counter) || fer::set_step_ptr_misc(counter))
    return fer::set_error("set_step_counter: hipMemcpyToSymbol failed");
  return 0;
}

extern "C" int fer_stream_create_cu_mask(const uint32_t* mask, int nwords, int priority, fer_stream_t* out) {
  if (!out || nwords < 0 || (nwords > 0 && !mask)) return fer::set_error("stream_create_cu_mask: bad arguments");
  // hipExtStreamCreateWithCUMask has neither a priority nor a flags argument: refuse a priority it
  // would silently drop (the masked stream is created blocking, at the default priority)
  if (nwords > 0 && priority != 0) return fer::set_error("stream_create_cu_mask: priority must be 0 with a CU mask");
  hipStream_t s = nullptr;
  hipError_t e = nwords == 0 ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority)
                             : hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask);
  if (e != hipSuccess) {
    char msg[160];
    snprintf(msg, sizeof(msg), "stream_create_cu_mask: %s", hipGetErrorString(e));
    return fer::set_error(msg);
  }
  *out = (fer_stream_t)s;
  return 0;
}

extern "C" int fer_stream_destroy(fer_stream_t s) {
  if (s && hipStreamDestroy((hipStream_t)s) != hipSuccess) return fer::set_error("stream_destroy failed");
  return 0;
}
