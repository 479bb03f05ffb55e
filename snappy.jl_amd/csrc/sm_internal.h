// sm_internal.h -- launcher interfaces between the C-ABI layer (sm_api.hip) and the
// kernels (sm_compress.hip, sm_decompress.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

// Batch descriptor: block b is in[in_off[b] .. +in_len[b]) -> out[out_off[b] ..).
// All pointers are device pointers.
struct CompressArgs {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint32_t* in_len;
  uint8_t* out;
  const uint64_t* out_off;
  uint32_t* out_len;
  uint32_t nblk;
  uint32_t table_size;  // 0: per block from its length (internal.jl:107-113); else fixed (Q2)
  int header;           // 1: prefix each block with varint(len) (independent snappy stream)
  int screened;         // set by launch_compress_fast: out_len holds k_literal_screen's verdicts
  // plan_n != 0 (sm_compress, fast modes): the blocks are the 64 KiB fragments of one input of
  // plan_n bytes at slot pitch plan_slot, and k_literal_screen writes in_off / in_len / out_off
  // (instead of a k_frag_plan launch) before the kernels after it read them
  uint64_t plan_n = 0;
  uint64_t plan_slot = 0;
  // in_host != null (sm_compress, fast modes): the input in device-mapped pinned host memory; the
  // screen reads its block there and writes the device copy at `in`, which the parse reads
  const uint8_t* in_host = nullptr;
};

struct DecompressArgs {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint32_t* in_len;
  uint8_t* out;
  const uint64_t* out_off;
  const uint32_t* out_cap;
  uint32_t* out_len;
  int32_t* status;
  uint32_t nblk;
  int raw;  // 1: no varint header -- a fragment of one stream, declared length = out_cap[b]
  // one_n != 0 (sm_uncompress's in-order path): ONE stream of one_n bytes at in, output capacity
  // one_cap at out -- in_off / in_len / out_off / out_cap are not read (no upload for them)
  uint32_t one_n = 0;
  uint32_t one_cap = 0;
};

// mode 0 = reference (byte-identical to Snappy.jl), 1 = fast (wave-parallel parse), 2 = fast, denser
hipError_t launch_compress(const CompressArgs& a, int mode, hipStream_t s);
hipError_t launch_compress_fast(const CompressArgs& a, int mode, hipStream_t s);
hipError_t launch_compress_sc(const CompressArgs& a, int mode, hipStream_t s);  // sm_compress_sc.hip (after the screen)
hipError_t launch_decompress(const DecompressArgs& a, int large, hipStream_t s);

// One large stream decoded in parallel (sm_uncompress): an index pass over 4 KiB chunks of the
// compressed body, then one wave per 64 KiB output fragment (see sm_decompress.hip).
constexpr uint32_t kIdxChunk = 4096;  // compressed bytes per index chunk
constexpr uint32_t kIdxEntries = 64;  // entry offsets 0..63 covered per chunk
// path 4 (a small stream on the device): bytes per index chunk -- kSmallChunkFine for bodies of
// mostly copies (shorter index and fill latency per chunk), kSmallChunk when literals are long or
// the body large (fewer chain elements).  sm_api.hip small_chunk() picks.
constexpr uint32_t kSmallChunk = 1024;
constexpr uint32_t kSmallChunkFine = 512;
constexpr uint32_t kSmallChunkTiny = 128;  // small bodies of mostly copies (sm_api.hip small_chunk)
#ifndef SM_SMALL_HOPS
#define SM_SMALL_HOPS 1024
#endif
constexpr uint32_t kSmallHops = SM_SMALL_HOPS;  // path 4: chain steps per pointer per resolve launch
constexpr uint32_t kOneLaunchHops = 256u << 10;  // path 4: outputs up to this size resolve in one launch of size hops
constexpr uint32_t kDeepLevels = 4;     // path 4: deep-entry records per chain (consecutive long literals)
constexpr uint32_t kDeepChains = 4;     // path 4: deep-record chains per chunk (distinct entry-lane exits)
constexpr uint32_t kIdxPad = 288;     // staged bytes past a chunk: +16 entry slack, a 256-byte walk window + 16
struct StreamFrag {
  uint32_t y;    // a true tag start at or before the fragment's first tag (chunk entry)
  uint32_t O;    // output position of the tag at y
  uint32_t F;    // the fragment's first output position (a multiple of 65536)
  uint32_t lim;  // output limit (0xffffffff for the last fragment: parse to the end)
};
hipError_t launch_validate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk,
                           int32_t* status, hipStream_t s);
hipError_t launch_uncompressed_length(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                      uint32_t nblk, uint32_t* out_len, int32_t* status, hipStream_t s);
// rec: nchunks * kIdxEntries (exit, output) u32 pairs
hipError_t launch_stream_index(const uint8_t* in, uint32_t N, uint32_t ip0, uint32_t nchunks, uint32_t* rec,
                               hipStream_t s);
hipError_t launch_decompress_frags(const uint8_t* in, uint32_t N, uint32_t size, uint8_t* out,
                                   const StreamFrag* frags, uint32_t nfrag, int32_t* status, hipStream_t s);
// Any large stream (copies may reach into earlier blocks): origin pointers per output byte,
// resolved by pointer jumping (sm_decompress.hip).  Path element = the tags starting in [y, ex),
// whose out bytes of output start at O.
struct OriginPath {
  uint32_t y, ex, O, out;
};
hipError_t launch_origin_fill(const uint8_t* in, uint32_t N, uint32_t size, const OriginPath* path, uint32_t npath,
                              uint32_t* P, int32_t* status, hipStream_t s);
// The same walk without the pointers: per path element, the reference's exact status of its first
// failing tag (kErrCross: the element's tags do not tile it).
hipError_t launch_path_check(const uint8_t* in, uint32_t N, uint32_t size, const OriginPath* path, uint32_t npath,
                             int32_t* status, hipStream_t s);
hipError_t launch_origin_resolve(uint32_t* P, uint32_t size, uint32_t* pending, hipStream_t s);
// A small stream entirely on the device (index, chain, fill, `rounds` resolve launches, gather; no
// host synchronisation).  rec: nchunks * kIdxEntries u32 pairs, then nchunks * kDeepChains *
// kDeepLevels 16-byte deep-entry records; path: nchunks elements; ctl: 4 +
// rounds u32 (zeroed by the chain kernel) -- ctl[0] path elements, ctl[1] != 0: the chain found no exact path (fall
// back), ctl[2] != 0: an element failed its checks (fall back), ctl[4 + r] != 0: pointers still
// unresolved after round r.  P: size u32.  The resolve launches write the output (each quad of
// bytes in the launch that resolves it) and words[0..1] = ctl[1], ctl[2]; the last launch sets
// words[2] = 1 when a pointer is still unresolved after it (the caller zeroes words[2] first).  Any
// nonzero word: fall back.  out and words may be device-mapped pinned host memory.
// in_host (nullable): the input in device-mapped pinned host memory -- the index launch reads it
// there and writes the device copy at in, which the later launches read (no separate upload).
hipError_t launch_small_decode(const uint8_t* in, const uint8_t* in_host, uint32_t N, uint32_t ip0, uint32_t size, uint32_t chunk,
                               uint32_t nchunks, uint32_t* rec, OriginPath* path, uint32_t* ctl, uint32_t* P,
                               uint32_t rounds, uint32_t hops, uint8_t* out, uint32_t* words, hipStream_t s);
// src[0, n) to dst and wsrc[0, nw) to words by a kernel (dst, words: device-mapped pinned host
// memory; no copy engine behind the kernels -- or, for uploads, src mapped host memory and dst
// the device's).  src, dst 16-byte aligned; nw <= 256.
hipError_t launch_to_host(const uint8_t* src, uint32_t n, uint8_t* dst, const uint32_t* wsrc, uint32_t nw,
                          uint32_t* words, hipStream_t s);
// sm_uncompress path 5: a stream of at most kLitSpans literal tags.  Literal s's bytes are at
// in + src[s] (any alignment) and go to out + dst[s], dst[s + 1] = dst[s] + its length, dst[n] the
// stream's length (the declared one, which the literals cover exactly); words[0..1] = (length,
// SM_OK) behind the bytes.  in and out may be device-mapped host memory.
constexpr uint32_t kLitSpans = 16;
struct LitSpans {
  uint32_t src[kLitSpans];
  uint32_t dst[kLitSpans + 1];
  uint32_t n;
};
hipError_t launch_literal_spans(const uint8_t* in, const LitSpans& sp, uint8_t* out, uint32_t* words, hipStream_t s);
hipError_t launch_origin_gather(const uint8_t* in, const uint32_t* P, uint32_t size, uint8_t* out, hipStream_t s);
// sm_compress, small inputs (at most 64 fragments), without host round trips: the fragments'
// offsets and lengths (fragment f = input [64 KiB f, +64 KiB), output slot f at pitch `slot`);
// then, after the compress launch, the fragments gathered behind one another into dst (tot[0] =
// their total length, tot[1] = 1 on a bad length, when nothing is copied).
hipError_t launch_frag_plan(uint64_t n, uint32_t nfrag, uint64_t slot, uint64_t* in_off, uint32_t* in_len,
                            uint64_t* out_off, hipStream_t s);
// Fast modes, small inputs, for latency: each block parsed in `parts` parts of `span` 1 KiB
// super-chunks on their own workgroups (k_compress_sc_span; with launch_parts_gather, the same
// bytes as the whole-block parse).  Part j of block b writes at out + out_off[b] + j pitch (pitch >=
// span kSpanSlot) and its length to part_len[b parts + j]; parts * span >= 64.  Runs the screen
// first.
constexpr uint32_t kSpanSlot = 1088;  // a super-chunk's output bound (k_compress_sc's staging slot)
struct ScSpan {
  uint32_t parts, span;
  uint64_t pitch;
  uint32_t* part_len;
};
hipError_t launch_compress_span(const CompressArgs& a, int mode, const ScSpan& sp, hipStream_t s);
hipError_t launch_compress_sc_span(const CompressArgs& a, int mode, const ScSpan& sp, hipStream_t s);  // (no screen)
// The parts of nblk (<= 256 / parts) blocks behind one another into dst (a block whose parts sum to
// more than one literal of the block -- the whole-block parse's fallback -- as that literal, from
// in): tot[0] = the total, tot[1] = 1 on an error mark or an over-long part (nothing copied).
hipError_t launch_parts_gather(const uint8_t* src, const uint64_t* out_off, const ScSpan& sp, const uint8_t* in,
                               const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk, uint64_t* tot,
                               uint8_t* dst, hipStream_t s);
hipError_t launch_frag_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* out_len,
                              const uint32_t* in_len, uint32_t nfrag, uint64_t* tot, uint8_t* dst, hipStream_t s);
// a sharded stream's fragments at their global offsets (sm_place_fragments_device, k_place)
hipError_t launch_place(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, const uint64_t* dst_off,
                        uint32_t nfrag, uint64_t total, int header, uint64_t cap, uint8_t* dst, uint64_t* loc_off,
                        int32_t* status, hipStream_t s);
// concatenate per-fragment outputs into one stream after a varint header (single-buffer API)
hipError_t launch_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                         const uint64_t* dst_off, uint8_t* dst, uint32_t nblk, hipStream_t s);

}  // namespace sm
