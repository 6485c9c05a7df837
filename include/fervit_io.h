/* fervit_io.h — C ABI of libfervit_io.so: host-side reader of packed w+ latent shards.
 *
 * Replaces the reference's one-torch.load-per-sample dataset (`data/latent_dataset.py:52-116`,
 * LatentFERDataset.__getitem__) for the latent trainers (`train/train_latent_vit_v2.py:205-219`),
 * SURVEY §8(f) row 1. A shard is one memory-mapped file holding every sample of a latent
 * directory (format in csrc/io/latent_shard.cpp; written by fervit.data.pack_latent_dir).
 * Host memory only (no GPU): fio_gather fills a caller buffer, typically pinned memory that a
 * stream-ordered H2D copy then moves to HBM (fervit.data.PackedLatentLoader).
 * Errors: NULL / negative return, message in fio_last_error() (thread-local).
 */
#ifndef FERVIT_IO_H
#define FERVIT_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Open (mmap) a shard; NULL on error. */
void* fio_open(const char* path);
/* Sample count and the [L][D] shape of one latent. */
int fio_info(void* shard, int64_t* count, int* L, int* D);
/* int32 [count] labels (inside the mapping; valid until fio_close). */
const int32_t* fio_labels(void* shard);
/* '\0'-separated image paths (`data/generate_latents.py:87-91` "img_path"); bytes may be 0. */
int fio_paths(void* shard, const char** blob, int64_t* bytes);
/* dst[i] = latent[idx[i]] (fp32 [L][D] each), labels[i] = label[idx[i]] (labels may be NULL),
 * for i < n, with up to nthreads threads. Indices are checked. */
int fio_gather(void* shard, const int64_t* idx, int64_t n, float* dst, int32_t* labels, int nthreads);
void fio_close(void* shard);
const char* fio_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
