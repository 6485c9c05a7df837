// Packed w+ latent shards: the input side of the latent trainers.
//
// The reference reads one torch-pickled .pt file per sample (`data/latent_dataset.py:93-116`,
// written by `data/generate_latents.py:87-91` as {"latent": fp32 [L][D], "label": int,
// "img_path": str}): one unpickle per 36 KB sample, four DataLoader worker processes. A packed
// shard holds the same samples in ONE memory-mapped file:
//   [0, 64)      header: "FWPS0001", u64 count, u32 L, u32 D, u32 dtype (0 = fp32), u32 0,
//                u64 labels_off, u64 latents_off, u64 paths_off, u64 paths_bytes
//   labels_off : int32 [count]
//   latents_off: fp32 [count][L][D], 4096-byte aligned
//   paths_off  : '\0'-separated UTF-8 image paths (may be empty)
// fio_gather copies a batch of samples, in any index order, into a caller buffer (pinned host
// memory, the source of the H2D copy) with several threads. Host C++ only: no GPU here.
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../../include/fervit_io.h"

namespace {

thread_local char g_err[256] = "";

int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}

struct Header {
  char magic[8];
  uint64_t count;
  uint32_t L, D, dtype, reserved;
  uint64_t labels_off, latents_off, paths_off, paths_bytes;
};
static_assert(sizeof(Header) == 64, "shard header is 64 bytes");

struct Shard {
  int fd = -1;
  size_t size = 0;
  const char* base = nullptr;
  Header h{};
  size_t sample_bytes() const { return (size_t)h.L * h.D * sizeof(float); }
};

}  // namespace

extern "C" {

const char* fio_last_error(void) { return g_err; }

void* fio_open(const char* path) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    fail("fio_open: cannot open the shard file");
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(Header)) {
    close(fd);
    fail("fio_open: not a packed latent shard (shorter than its header)");
    return nullptr;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    fail("fio_open: mmap failed");
    return nullptr;
  }
  Shard* s = new Shard;
  s->fd = fd;
  s->size = (size_t)st.st_size;
  s->base = (const char*)p;
  memcpy(&s->h, p, sizeof(Header));
  const Header& h = s->h;
  const uint64_t sb = s->sample_bytes();
  const bool ok = memcmp(h.magic, "FWPS0001", 8) == 0 && h.dtype == 0 && h.L > 0 && h.D > 0 &&
                  h.labels_off >= sizeof(Header) && h.labels_off + h.count * 4 <= s->size &&
                  h.latents_off % 4096 == 0 && h.latents_off + h.count * sb <= s->size &&
                  h.paths_off + h.paths_bytes <= s->size;
  if (!ok) {
    fio_close(s);
    fail("fio_open: bad shard header (magic, dtype or section bounds)");
    return nullptr;
  }
  // shuffled training reads touch samples in random order
  madvise(p, s->size, MADV_RANDOM);
  return s;
}

int fio_info(void* handle, int64_t* count, int* L, int* D) {
  const Shard* s = (const Shard*)handle;
  if (!s) return fail("fio_info: null handle");
  if (count) *count = (int64_t)s->h.count;
  if (L) *L = (int)s->h.L;
  if (D) *D = (int)s->h.D;
  return 0;
}

const int32_t* fio_labels(void* handle) {
  const Shard* s = (const Shard*)handle;
  return s ? (const int32_t*)(s->base + s->h.labels_off) : nullptr;
}

int fio_paths(void* handle, const char** blob, int64_t* bytes) {
  const Shard* s = (const Shard*)handle;
  if (!s) return fail("fio_paths: null handle");
  *blob = s->base + s->h.paths_off;
  *bytes = (int64_t)s->h.paths_bytes;
  return 0;
}

int fio_gather(void* handle, const int64_t* idx, int64_t n, float* dst, int32_t* labels, int nthreads) {
  const Shard* s = (const Shard*)handle;
  if (!s) return fail("fio_gather: null handle");
  if (n <= 0) return 0;
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || (uint64_t)idx[i] >= s->h.count) return fail("fio_gather: sample index out of range");
  const size_t sb = s->sample_bytes();
  const char* lat = s->base + s->h.latents_off;
  const int32_t* lab = (const int32_t*)(s->base + s->h.labels_off);
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      memcpy((char*)dst + (size_t)i * sb, lat + (size_t)idx[i] * sb, sb);
      if (labels) labels[i] = lab[idx[i]];
    }
  };
  // one thread per >= 16 samples (a 36 KB sample is a few us of memcpy / page faults)
  const int64_t t = std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(nthreads, 1), (n + 15) / 16, 64}));
  if (t == 1) {
    work(0, n);
    return 0;
  }
  std::vector<std::thread> pool;
  pool.reserve((size_t)t);
  const int64_t per = (n + t - 1) / t;
  for (int64_t k = 0; k < t; ++k) {
    const int64_t lo = k * per, hi = std::min(n, lo + per);
    if (lo < hi) pool.emplace_back(work, lo, hi);
  }
  for (auto& th : pool) th.join();
  return 0;
}

void fio_close(void* handle) {
  Shard* s = (Shard*)handle;
  if (!s) return;
  if (s->base) munmap((void*)s->base, s->size);
  if (s->fd >= 0) close(s->fd);
  delete s;
}

}  // extern "C"
