/*
 * snappy_mi355x.h -- C ABI of the MI355X (gfx950) snappy codec (libsnappy_mi355x.so).
 *
 * Drop-in boundary for krm01/Snappy.jl's hot path.  Every entry point names the reference
 * interface it replaces (paths relative to the reference repo root).  The shape follows
 * snappy-c.h, the C ABI the reference already ccalls in test/libsnappy.jl:5-30: caller
 * allocates the output, sizes travel as size_t in/out.  INTEGRATION.md shows the Julia
 * ccall binding a maintainer adds to src/Snappy.jl.
 *
 * Error model: the reference throws ErrorException(msg) (src/Snappy.jl:21,50,
 * src/varint.jl:36, src/internal.jl:499,505,518).  Here each message has its own status
 * code (16..21), sm_status_message() returns the reference's exact text, and codes 1/2 keep
 * libsnappy's meaning (INVALID_INPUT, BUFFER_TOO_SMALL).
 *
 * Three compress modes:
 *   SM_MODE_REFERENCE  -- output byte-identical to Snappy.jl compress() (incl. its quirks);
 *   SM_MODE_FAST       -- wave-parallel parse; any output decodes bit-exactly under
 *                         Snappy.jl uncompress() and libsnappy, bytes differ from the reference;
 *   SM_MODE_FAST_DENSE -- SM_MODE_FAST verifying two hash-chain candidates per position:
 *                         smaller output, about 10% slower.
 * Decompression has one mode, with the reference's accept/reject behaviour.
 *
 * Threading: an sm_ctx owns one HIP device, one stream and its scratch.  The host-buffer
 * entry points lock the ctx (concurrent callers on one ctx are serialised); the *_device entry
 * points only launch on the caller's stream and take no lock.  Distinct ctxs are independent.
 */
#ifndef SNAPPY_MI355X_H_
#define SNAPPY_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t sm_status;
enum {
  SM_OK = 0,
  SM_INVALID_INPUT = 1,        /* snappy-c.h SNAPPY_INVALID_INPUT (generic) */
  SM_BUFFER_TOO_SMALL = 2,     /* snappy-c.h SNAPPY_BUFFER_TOO_SMALL */
  SM_ERR_INPUT_TOO_LARGE = 16, /* "Input too large."                   src/Snappy.jl:21 */
  SM_ERR_INVALID = 17,         /* "Invalid input."                     src/Snappy.jl:50 */
  SM_ERR_VARINT = 18,          /* "Could not decode varint32."         src/varint.jl:36 */
  SM_ERR_COPY_OFFSET = 19,     /* "Invalid input: corrupt copy offset" src/internal.jl:499 */
  SM_ERR_COPY_LENGTH = 20,     /* "Invalid input: corrupt copy length" src/internal.jl:505 */
  SM_ERR_LITERAL = 21,         /* "Invalid input: corrupt literal"     src/internal.jl:518 */
  SM_ERR_DEVICE = 32,          /* HIP runtime failure / no device */
  SM_ERR_ARGUMENT = 33         /* bad argument (NULL, block > 64 KiB in a batch, ...) */
};

enum { SM_MODE_REFERENCE = 0, SM_MODE_FAST = 1, SM_MODE_FAST_DENSE = 2 };

#define SM_BLOCK_SIZE 65536u /* src/internal.jl:31 K_BLOCK_SIZE */
/* d_out_len[b] >= SM_OUT_LEN_ERROR: block b failed (see sm_compress_batch_device).  The
 * reference raises instead of returning a length (src/Snappy.jl:21). */
#define SM_OUT_LEN_ERROR 0xfff00000u

typedef struct sm_ctx sm_ctx;

/* Reference text for a status code (the ErrorException message), or a description. */
const char* sm_status_message(sm_status st);

/* ---- format helpers (host, no device needed) ------------------------------------ */
/* replaces maxlength_compressed, src/Snappy.jl:80-82 (= snappy_max_compressed_length) */
size_t sm_max_compressed_length(size_t source_length);
/* replaces length_uncompressed, src/Snappy.jl:90-92 (= snappy_uncompressed_length) */
sm_status sm_uncompressed_length(const char* compressed, size_t compressed_length, size_t* result);
/* replaces parse32, src/varint.jl:12-37.  off is 0-based; *next is 0-based. */
sm_status sm_parse32(const uint8_t* buf, size_t len, size_t off, uint32_t* value, size_t* next);
/* replaces encode32!, src/varint.jl:46-69.  Writes 1..5 bytes, returns the count. */
size_t sm_encode32(uint8_t* buf, uint32_t value);
/* replaces find_match_length, src/internal.jl:343-387 (host; the reference's tests call it,
 * test/runtests.jl:168-267).  0-based i1 < i2, limit INCLUSIVE: the length of the common run
 * of buf[i1..] and buf[i2..] with i2 + n - 1 <= limit.  SM_ERR_ARGUMENT where the reference
 * would read past buf (its @test_broken case). */
sm_status sm_find_match_length(const uint8_t* buf, size_t len, size_t i1, size_t i2, size_t limit,
                               size_t* matched);

/* ---- device context -------------------------------------------------------------- */
sm_ctx* sm_ctx_create(int device);
void sm_ctx_destroy(sm_ctx* ctx);
/* the HIP stream the ctx launches on (hipStream_t) */
void* sm_ctx_stream(sm_ctx* ctx);
/* diagnostic: how the ctx's last sm_uncompress decoded -- 0 in stream order (one wave),
 * 1 as parallel 64 KiB fragments (a large block-structured stream), 2 in parallel by origin
 * pointers (a large stream whose copies cross 64 KiB blocks), 3 a large stream's first error
 * found in parallel (per-tag checks over its tag path), 4 a small stream (<= 1 MiB compressed)
 * decoded in parallel by origin pointers entirely on the device (one synchronisation), 5 a stream
 * of literal tags only (at most 16, e.g. an incompressible input's) copied by one kernel from the
 * pinned input staging to the pinned output staging (one synchronisation), -1 none yet */
int sm_ctx_last_path(sm_ctx* ctx);
/* diagnostic: enable (1, the default) or disable (0) paths 4 and 5 for the ctx's sm_uncompress
 * calls (the tests run the other paths on small streams with them off) */
sm_status sm_ctx_set_small_decode(sm_ctx* ctx, int enable);
/* diagnostic: enable (1, the default) or disable (0) parsing the fragments of a small fast-mode
 * sm_compress input (<= 4 MiB) in parts on their own workgroups -- the same bytes as the
 * whole-fragment parse, at a fraction of its latency; sm_ctx_last_compress_split: 1 when the
 * ctx's last sm_compress did so, 0 when not, -1 for a null ctx */
sm_status sm_ctx_set_split_compress(sm_ctx* ctx, int enable);
int sm_ctx_last_compress_split(sm_ctx* ctx);

/* ---- single buffer, host memory (the reference's exported API) -------------------- */
/* replaces compress(::Vector{UInt8}), src/Snappy.jl:20-36 (and compress(::String), :38).
 * *compressed_length: in = capacity (>= sm_max_compressed_length(n)), out = bytes written. */
sm_status sm_compress(sm_ctx* ctx, const char* input, size_t input_length, char* compressed,
                      size_t* compressed_length, int mode);
/* replaces uncompress(::Vector{UInt8}), src/Snappy.jl:46-52.
 * *uncompressed_length: in = capacity, out = bytes written. */
sm_status sm_uncompress(sm_ctx* ctx, const char* compressed, size_t compressed_length, char* uncompressed,
                        size_t* uncompressed_length);

/* ---- batched, device memory (the GPU hot path; asynchronous on `stream`) ----------------
 * Block b: input d_in[d_in_off[b] .. +d_in_len[b]), d_in_len[b] <= 65536; each block becomes
 * an independent snappy stream (varint header + one compress_fragment!, i.e. exactly
 * compress(block) of src/Snappy.jl:20-36) written at d_out + d_out_off[b], which must have
 * room for sm_max_compressed_length(d_in_len[b]) bytes.  d_out_len[b] receives its size, or
 * an error mark >= SM_OUT_LEN_ERROR (no stream was written for that block):
 *   0xffffffff            the block was longer than 64 KiB;
 *   SM_OUT_LEN_ERROR | k  the device parse failed internally (k != 0: a bounded wait between
 *                         the kernel's waves gave up; never expected -- report it as a device
 *                         error, SM_ERR_DEVICE).
 * Every mark is larger than any real size (<= sm_max_compressed_length(65536) = 76,490); the
 * host-buffer entry points check the lengths and return SM_ERR_DEVICE / SM_ERR_ARGUMENT instead
 * of a mark.  stream: the hipStream_t to launch on (NULL = the default stream, as everywhere in
 * HIP); nothing is synchronised. */
sm_status sm_compress_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                   const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                   const uint64_t* d_out_off, uint32_t* d_out_len, int mode, void* stream);
/* Fragments of ONE stream (the block loop of src/Snappy.jl:29-33): like
 * sm_compress_batch_device but no per-fragment varint header, and every fragment uses the
 * hash-table size the reference derives from the stream's total length total_len
 * (src/Snappy.jl:27, quirk Q2).  The caller writes varint(total_len) and concatenates the
 * fragments in order (e.g. after a size all-gather across GPUs, snappy.jl_amd/dist.py). */
sm_status sm_compress_fragments_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                       const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                       const uint64_t* d_out_off, uint32_t* d_out_len, uint64_t total_len,
                                       int mode, void* stream);
/* Places fragments of ONE stream at their offsets in it -- the concatenation of src/Snappy.jl:29-35
 * (fragment i's bytes follow fragment i-1's behind varint(total)) for a stream whose fragments were
 * compressed in shards, e.g. one contiguous shard per GPU (snappy.jl_amd/dist.py).
 * Fragment b, d_len[b] bytes at d_src + d_src_off[b] (sm_compress_fragments_device's output), is
 * copied to d_dst + (d_dst_off[b] - base), where d_dst_off[b] is its offset in the whole stream
 * (the exclusive scan of all fragments' sizes behind the header) and
 *   write_header != 0: base = 0 -- d_dst is the stream from its first byte, and varint(total_len)
 *                      is written at d_dst[0..] (the shard holding fragment 0);
 *   write_header == 0: base = d_dst_off[0] -- d_dst is this caller's byte range of the stream,
 *                      starting at its first fragment.
 * d_dst has room for dst_capacity bytes.  d_local_off (optional, nfrag u64) receives
 * d_dst_off[b] - base (the fragments' offsets in d_dst, for sm_uncompress_fragments_device).
 * A length that is an error mark (>= SM_OUT_LEN_ERROR), or a fragment that would end past
 * dst_capacity, copies nothing and sets *d_status = SM_ERR_DEVICE (optional; never cleared: zero
 * it first).  Asynchronous on `stream`. */
sm_status sm_place_fragments_device(sm_ctx* ctx, const uint8_t* d_src, const uint64_t* d_src_off,
                                    const uint32_t* d_len, uint32_t nfrag, const uint64_t* d_dst_off,
                                    uint64_t total_len, int write_header, uint8_t* d_dst, uint64_t dst_capacity,
                                    uint64_t* d_local_off, int32_t* d_status, void* stream);
/* Fragments of ONE stream, decoded (the inverse of sm_compress_fragments_device; the block loop
 * of src/Snappy.jl:46-52 over src/internal.jl:411-466 without the varint header): fragment b is
 * d_in[d_in_off[b] .. +d_in_len[b]) and must decode to exactly d_frag_len[b] (<= 65536) bytes at
 * d_out + d_out_off[b].  d_status[b] / d_out_len[b] as in sm_uncompress_batch_device. */
sm_status sm_uncompress_fragments_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                         const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                         const uint64_t* d_out_off, const uint32_t* d_frag_len, uint32_t* d_out_len,
                                         int32_t* d_status, void* stream);

/* Block b: compressed stream d_in[d_in_off[b] .. +d_in_len[b]) -> d_out + d_out_off[b] with
 * capacity d_out_cap[b].  d_status[b] = SM_OK or the reference's error code (first error in
 * stream order); d_out_len[b] = decoded bytes (0 on error).  Each block decodes as
 * uncompress(block), src/Snappy.jl:46-52. */
sm_status sm_uncompress_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                     const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                     const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                     uint32_t* d_out_len, int32_t* d_status, void* stream);

/* Block b: d_status[b] = exactly the status uncompress(block) would return
 * (src/Snappy.jl:46-52 with the checks of src/internal.jl:411-527) given enough output room,
 * found by the decoder's tag walk and checks alone -- no output is written.  Batched
 * snappy_validate_compressed_buffer (snappy-c.h), SURVEY §8(f) row 4. */
sm_status sm_validate_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                   const uint32_t* d_in_len, uint32_t nblk, int32_t* d_status, void* stream);
/* Block b: d_len[b] = its declared uncompressed length (the varint header) and d_status[b] =
 * SM_OK, or SM_ERR_VARINT with d_len[b] = 0.  Batched length_uncompressed, src/Snappy.jl:90-92. */
sm_status sm_uncompressed_length_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                              const uint32_t* d_in_len, uint32_t nblk, uint32_t* d_len,
                                              int32_t* d_status, void* stream);

/* ---- batched, host memory (H2D + kernel + D2H, synchronous) ------------------------ */
sm_status sm_compress_batch(sm_ctx* ctx, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                            uint32_t nblk, uint8_t* out, const uint64_t* out_off, uint32_t* out_len, int mode);
sm_status sm_uncompress_batch(sm_ctx* ctx, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                              uint32_t nblk, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                              uint32_t* out_len, int32_t* status);

/* Multi-GPU, one process: the blocks are cut into nctx contiguous shards of (nearly) equal
 * block count, shard i runs sm_compress_batch / sm_uncompress_batch on ctxs[i] (one context per
 * GPU) from its own host thread, all shards concurrently.  Same arguments and per-block results
 * as the single-context calls; the first failing shard's status is returned.  The
 * one-process-per-GPU path (torch.distributed, snappy.jl_amd/dist.py) is the alternative. */
sm_status sm_compress_batch_sharded(sm_ctx* const* ctxs, int nctx, const uint8_t* in, const uint64_t* in_off,
                                    const uint32_t* in_len, uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                                    uint32_t* out_len, int mode);
sm_status sm_uncompress_batch_sharded(sm_ctx* const* ctxs, int nctx, const uint8_t* in, const uint64_t* in_off,
                                      const uint32_t* in_len, uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                                      const uint32_t* out_cap, uint32_t* out_len, int32_t* status);

/* snappy_validate_compressed_buffer (snappy-c.h) for one host buffer, on the device: the status
 * sm_uncompress would return with enough output room, without decoding into memory. */
sm_status sm_validate_compressed_buffer(sm_ctx* ctx, const char* compressed, size_t compressed_length);

/* ---- snappy-c.h-shaped entry points, no ctx (a process-wide default context) ---------
 * Same argument shapes and statuses as libsnappy's snappy-c.h: 0 OK, 1 INVALID_INPUT (every
 * error, device and argument failures included), 2 BUFFER_TOO_SMALL -- the detailed codes
 * (the reference's messages, SM_ERR_*) come from the ctx API.  That is exactly the ccall
 * signature the reference's helper binds (test/libsnappy.jl:5-30:
 * (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}) -> Cint), so a Julia binding switches from
 * libsnappy by library and symbol name alone.  The default context is created on first use on
 * device $SNAPPY_MI355X_DEVICE (default 0); calls are serialised on it.
 * sm_snappy_compress uses SM_MODE_FAST_DENSE (sizes within 1.01x of Snappy.jl's) unless
 * sm_snappy_set_mode() selects another mode (SM_MODE_REFERENCE for Snappy.jl's exact bytes,
 * SM_MODE_FAST for the highest rate). */
sm_status sm_snappy_compress(const char* input, size_t input_length, char* compressed, size_t* compressed_length);
sm_status sm_snappy_uncompress(const char* compressed, size_t compressed_length, char* uncompressed,
                               size_t* uncompressed_length);
size_t sm_snappy_max_compressed_length(size_t source_length);
sm_status sm_snappy_uncompressed_length(const char* compressed, size_t compressed_length, size_t* result);
sm_status sm_snappy_validate_compressed_buffer(const char* compressed, size_t compressed_length);
sm_status sm_snappy_set_mode(int mode);

/* library build identification ("snappy_mi355x gfx950 <git-describe>") */
const char* sm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SNAPPY_MI355X_H_ */
