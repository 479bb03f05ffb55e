// sm_api.hip -- C ABI (include/snappy_mi355x.h) over the gfx950 kernels.
// Host framing follows src/Snappy.jl:20-52: varint header, 64 KiB fragments sharing one
// table size derived from the total length (quirk Q2), final produced==declared check (the
// latter lives in the decode kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/snappy_mi355x.h"
#include "sm_device.h"
#include "sm_internal.h"

#ifndef SM_VERSION_STR
#define SM_VERSION_STR "dev"
#endif

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n < 4096 ? 4096 : n;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Host staging: page-aligned ordinary memory registered for DMA (hipHostRegister), so the CPU
// reads it through its caches -- the host walks the index records and scatters batch outputs
// from it.  (hipHostMalloc'd staging was read ~2x slower by those CPU loops.)  It is also mapped
// into the device (dp): the single-buffer calls' last kernel writes its result there directly,
// because a copy-engine transfer queued behind kernels waited up to ~120 us on this box
// (tools/probes/latency_probe.hip, profiles/r04_latency_probe.txt).
// Visibility: kernels store results into this memory and the host reads them only after
// hipStreamSynchronize on the launching stream; HIP makes a kernel's writes to host memory visible
// to the host at that synchronisation (the completion signal is a system-scope release), so the
// writers issue no fence of their own.  A __threadfence_system() in each writer
// was measured in round 5: every wave writes back the L2 (buffer_wbl2), and single calls took
// 20-45 us longer (alice29.txt compress 60 -> 104 us, urls.10K uncompress 296 -> 527 us, same box).
struct HostBuf {
  void* p = nullptr;
  void* dp = nullptr;  // the device's address of p (nullptr: not mapped)
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    const size_t want = ((n < (1u << 20) ? (1u << 20) : n) + 4095) & ~(size_t)4095;
    void* q = nullptr;
    if (posix_memalign(&q, 4096, want) != 0) return hipErrorOutOfMemory;
    const hipError_t e = hipHostRegister(q, want, hipHostRegisterMapped);
    if (e != hipSuccess) {
      free(q);
      return e;
    }
    p = q;
    cap = want;
    if (hipHostGetDevicePointer(&dp, q, 0) != hipSuccess) dp = nullptr;
    return hipSuccess;
  }
  void release() {
    if (p) {
      (void)hipHostUnregister(p);
      free(p);
    }
    p = nullptr;
    dp = nullptr;
    cap = 0;
  }
};

struct sm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy = nullptr;     // host->device copies that overlap the kernels (sm_compress)
  std::vector<hipEvent_t> ev;     // their completion events
  DevBuf in, out, out2, meta, idx, gat, org;  // org: origin pointers of the general parallel decode
  HostBuf stage;
  HostBuf stage_in;              // small host inputs on their way up (upload_input)
  hipEvent_t in_ev = nullptr;    // recorded behind the last upload from stage_in
  int last_path = -1;  // sm_ctx_last_path
  bool small = true;   // sm_ctx_set_small_decode
  bool split = true;   // sm_ctx_set_split_compress
  bool last_split = false;  // the last sm_compress parsed its fragments in parts
  std::mutex mu;       // serialises the host-buffer entry points (they share the scratch above)
};

#ifndef SM_SMALL_BODY8  // path 4 when the body is at most SM_SMALL_BODY8/8 of the output
#define SM_SMALL_BODY8 8
#endif

namespace {

bool valid_mode(int m) { return m == SM_MODE_REFERENCE || m == SM_MODE_FAST || m == SM_MODE_FAST_DENSE; }

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};


inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

#ifdef SM_HOST_TRACE  // diagnostic builds: phase times of the single-buffer entry points on stderr
#include <chrono>
#include <cstdio>
struct HostTrace {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what, hipStream_t s) {
    (void)hipStreamSynchronize(s);
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "  %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};
#define HT_DECL HostTrace ht_;
#define HT(what) ht_.mark(what, s);
#else
#define HT_DECL
#define HT(what)
#endif

constexpr uint32_t kParallelMinOutput = 4 * 65536;  // smaller streams: one wave is as fast
constexpr size_t kOrgKeep = 256u << 20;  // origin-pointer scratch a context keeps after a decode
constexpr size_t kPipeMinInput = 32u << 20;  // sm_compress: inputs this large upload in pieces
constexpr size_t kSmallCompressMax = 4u << 20;  // sm_compress: inputs up to this size (64 fragments) synchronise once
constexpr uint32_t kPieceFrags = 256;        // 16 MiB per piece
#ifndef SM_OUT_PIECE
#define SM_OUT_PIECE 2048
#endif
constexpr uint32_t kOutPieceFrags = SM_OUT_PIECE;  // sm_uncompress: output pieces (128 MiB)

constexpr size_t kPinnedInMin = 32u << 10;  // host inputs from this size up go through stage_in
constexpr size_t kPinnedInMax = 16u << 20;  // ... up to this size

// A host input of a single-buffer call into ctx->in.  Inputs of 32 KiB to 16 MiB are copied on
// the host into the context's pinned, device-mapped staging and moved to the device by a copy
// kernel (k_to_host reading the mapped pages): fireworks.jpeg's uncompress 60 -> 50 us, html's
// 70 -> 67, 64 KiB compress 52 -> 48 (profiles/r06_upload_ab.txt).  Smaller inputs stay with the
// runtime's pageable copy, which is 2-4 us faster there than the staging (its event and the
// extra launch), and so does an upload through the copy engine from the staging at every size.
// The staging is reused by the next call only after the previous upload's event.
// the pinned input staging for n bytes, once the device is done with its previous contents (the
// event recorded behind the last launch that read it); false: no staging
bool stage_in_acquire(sm_ctx* ctx, size_t n) {
  if (ctx->stage_in.ensure(n + 16) != hipSuccess || !ctx->stage_in.dp) return false;
  return !ctx->in_ev || hipEventSynchronize(ctx->in_ev) == hipSuccess;
}
// after the launches that read the staging: their completion event
hipError_t stage_in_release(sm_ctx* ctx, hipStream_t s) {
  if (!ctx->in_ev) {
    const hipError_t e = hipEventCreateWithFlags(&ctx->in_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      ctx->in_ev = nullptr;
      return e;
    }
  }
  return hipEventRecord(ctx->in_ev, s);
}

hipError_t upload_input(sm_ctx* ctx, const void* src, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n >= kPinnedInMin && n <= kPinnedInMax && stage_in_acquire(ctx, n)) {
    memcpy(ctx->stage_in.p, src, n);
    const hipError_t e = sm::launch_to_host((const uint8_t*)ctx->stage_in.dp, (uint32_t)n, (uint8_t*)ctx->in.p,
                                            nullptr, 0, nullptr, s);
    if (e != hipSuccess) return e;
    return stage_in_release(ctx, s);
  }
  return hipMemcpyAsync(ctx->in.p, src, n, hipMemcpyHostToDevice, s);
}

// sm_uncompress path 5: are the stream's tags literals only?  At most kLitSpans of them (an
// incompressible input's stream has one literal per 64 KiB block), each with at most 3 length
// bytes, inside the input and the declared length, together covering both exactly.  Then the
// reference's decode (internal.jl:411-527: every tag starts before the input's last byte, and
// copy_literal!'s checks pass) is those literals' bytes in order, and Snappy.jl:50's length check
// holds.  Anything else -- a copy tag, a 4-byte length, more tags, a stream that ends early or
// late -- is not path 5, and the other paths reproduce the reference's accept/reject.  Reads the
// tag headers only (at most 4 bytes a tag); the bytes move on the device.
bool literal_only(const uint8_t* c, size_t n, size_t hdr, uint32_t size, sm::LitSpans& sp) {
  size_t p = hdr;
  uint64_t o = 0;
  sp.n = 0;
  while (p < n) {
    if (sp.n == sm::kLitSpans) return false;
    const uint32_t t = c[p];
    if (t & 3) return false;  // a copy
    uint64_t len = (t >> 2) + 1;
    size_t q = p + 1;
    if ((t >> 2) >= 60) {
      const uint32_t nb = (t >> 2) - 59;
      if (nb > 3 || q + nb > n) return false;
      uint32_t v = 0;
      for (uint32_t k = 0; k < nb; ++k) v |= (uint32_t)c[q + k] << (8 * k);
      len = (uint64_t)v + 1;
      q += nb;
    }
    if (q + len > n || o + len > size) return false;
    sp.src[sp.n] = (uint32_t)q;
    sp.dst[sp.n] = (uint32_t)o;
    ++sp.n;
    o += len;
    p = q + len;
  }
  sp.dst[sp.n] = (uint32_t)o;
  return sp.n > 0 && o == size;
}

// path 5: the input into the pinned staging on the host, the literals to the pinned output by
// k_literal_spans reading and writing the mapped pages, then the bytes to the caller.  1: done,
// 0: not taken (no mapped staging), -1: a device error.
int literal_uncompress(sm_ctx* ctx, const uint8_t* comp, size_t n, uint32_t size, const sm::LitSpans& ls,
                       uint8_t* host_out) {
  hipStream_t s = ctx->stream;
  const size_t w_off = align_up(size, 256);
  if (ctx->stage.ensure(w_off + 64) != hipSuccess || !ctx->stage.dp) return 0;
  if (!stage_in_acquire(ctx, n)) return 0;
  memcpy(ctx->stage_in.p, comp, n);
  uint8_t* const sdp = (uint8_t*)ctx->stage.dp;
  volatile uint32_t* const w = (volatile uint32_t*)((uint8_t*)ctx->stage.p + w_off);
  w[1] = 0xffffffffu;  // (the kernel writes SM_OK)
  if (sm::launch_literal_spans((const uint8_t*)ctx->stage_in.dp, ls, sdp, (uint32_t*)(sdp + w_off), s) != hipSuccess)
    return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  if (w[1] != 0 || w[0] != size) return -1;
  memcpy(host_out, ctx->stage.p, size);
  return 1;
}

// the context's copy stream and at least n events (created on first use)
hipError_t ensure_copy_stream(sm_ctx* ctx, size_t n) {
  if (!ctx->copy) {
    const hipError_t e = hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking);
    if (e != hipSuccess) {
      ctx->copy = nullptr;
      return e;
    }
  }
  while (ctx->ev.size() < n) {
    hipEvent_t e;
    const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return r;
    ctx->ev.push_back(e);
  }
  return hipSuccess;
}

// Host tag walk over [p, lim) of a stream (zero-padded lookahead, internal.jl:426-462): where it
// leaves the range and how much output the tags make.  Used when a chunk is entered deeper than
// the entry offsets the index kernel covers.
void host_walk(const uint8_t* comp, uint32_t n, uint64_t p, uint64_t lim, uint64_t* exit_pos, uint64_t* produced) {
  uint64_t o = 0;
  while (p < lim) {
    const uint32_t c = comp[p];
    const uint32_t entry = sm::char_entry(c);
    const uint32_t taglen = entry >> 11;
    uint32_t tr = 0;
    for (uint32_t k = 0; k < 4; ++k) tr |= (p + 1 + k < n ? (uint32_t)comp[p + 1 + k] : 0u) << (8 * k);
    const uint32_t trailer = taglen >= 4 ? tr : (tr & ((1u << (8 * taglen)) - 1u));
    if (c & 3) {
      p += 1 + taglen;
      o += entry & 0xff;
    } else {
      const uint32_t lit = (entry & 0xff) + trailer;
      p += 1ull + taglen + lit;
      o += lit;
    }
  }
  *exit_pos = p;
  *produced = o;
}

// The first error of a stream whose tag path is known: one wave per path element checks its tags
// (k_path_check), and the first failing element in path order holds the reference's status.  With
// no failing tag the stream is short of its declared length (Snappy.jl:50).  Returns 3 with *err
// set, 0 to fall back to the in-order decode, -1 on a device error.
struct PathChunk {
  uint64_t y, O, out, ex;
};
int path_first_error(sm_ctx* ctx, uint32_t n, uint32_t size, const std::vector<PathChunk>& path, int32_t* err) {
  if (n >= 0x80000000u || path.empty()) return 0;
  hipStream_t s = ctx->stream;
  const size_t npath = path.size();
  std::vector<sm::OriginPath> op(npath);
  for (size_t e = 0; e < npath; ++e) {
    // an element past 2^32 of output is past any declared size: its O saturates (it fails its checks)
    const uint64_t O = std::min<uint64_t>(path[e].O, 0xffffffffull), out = std::min<uint64_t>(path[e].out, 0xffffffffull - O);
    op[e] = {(uint32_t)path[e].y, (uint32_t)std::min<uint64_t>(path[e].ex, 0xffffffffull), (uint32_t)O, (uint32_t)out};
  }
  const size_t st_off = align_up(npath * sizeof(sm::OriginPath), 256);
  if (ctx->org.ensure(st_off + npath * 4) != hipSuccess) return 0;
  sm::OriginPath* d_path = (sm::OriginPath*)ctx->org.p;
  int32_t* d_st = (int32_t*)((uint8_t*)ctx->org.p + st_off);
  if (hipMemcpyAsync(d_path, op.data(), npath * sizeof(sm::OriginPath), hipMemcpyHostToDevice, s) != hipSuccess)
    return -1;
  if (sm::launch_path_check((const uint8_t*)ctx->in.p, n, size, d_path, (uint32_t)npath, d_st, s) != hipSuccess)
    return -1;
  std::vector<int32_t> st(npath);
  if (hipMemcpyAsync(st.data(), d_st, npath * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  for (int32_t v : st) {
    if (v == sm::kOk) continue;
    if (v == sm::kErrCross) return 0;  // the tags do not tile an element: let the in-order decode decide
    *err = v;
    return 3;
  }
  const PathChunk& last = path.back();
  if (last.O + last.out == size) return 0;  // no failing tag and the right length: not an error after all
  *err = sm::kErrInvalid;  // Snappy.jl:50
  return 3;
}

// One large stream in parallel (sm_decompress.hip, "one large stream"): index pass, true path
// on the host, one wave per 64 KiB fragment.  The compressed bytes are in ctx->in.  Returns
// 1 (or 2, origin pointers) with the output in ctx->out, 3 with *err when the stream has an
// error (its first one in stream order), 0 to fall back to the in-order decode, -1 on a device
// error.  With host_out, a large output goes down in pieces on the copy stream as the fragment
// decode finishes them (*copied = true: host_out holds the result when 1 is returned).
int parallel_uncompress(sm_ctx* ctx, const uint8_t* comp, uint32_t n, uint32_t ip0, uint32_t size,
                        uint8_t* host_out, bool* copied, int32_t* err) {
  *copied = false;
  using sm::kIdxChunk;
  using sm::kIdxEntries;
  const uint32_t nchunks = (n - ip0 + kIdxChunk - 1) / kIdxChunk;
  const uint32_t nfrag = (uint32_t)(((uint64_t)size + 65535) / 65536);
  const size_t rec_n = (size_t)nchunks * kIdxEntries;
  const size_t frag_off = align_up(2 * rec_n * 4, 16);
  const size_t st_off = frag_off + (size_t)nfrag * sizeof(sm::StreamFrag);
  if (ctx->idx.ensure(st_off + (size_t)nfrag * 4) != hipSuccess) return 0;  // (the in-order decode needs no scratch)
  hipStream_t s = ctx->stream;
  HT_DECL
  uint32_t* d_rec = (uint32_t*)ctx->idx.p;
  const uint8_t* d_in = (const uint8_t*)ctx->in.p;
  if (sm::launch_stream_index(d_in, n, ip0, nchunks, d_rec, s) != hipSuccess) return -1;
  HT("index kernel")
  // the index records (8 B per entry, ~9 MB per 64 MiB of stream) come back through the
  // context's pinned staging: one DMA, no page faults, no zero fill
  if (ctx->stage.ensure(2 * rec_n * 4) != hipSuccess) return 0;
  const uint32_t* rec = (const uint32_t*)ctx->stage.p;
  if (hipMemcpyAsync(ctx->stage.p, d_rec, 2 * rec_n * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  HT("index records D2H")
  // true path: chunk entries y, output before them O, output of their tags
  std::vector<PathChunk> path;
  path.reserve(nchunks + 16);
  uint64_t y = ip0, O = 0;
  while (y < (uint64_t)n - 1) {  // internal.jl:416
    const uint64_t c = (y - ip0) / kIdxChunk, base = ip0 + c * kIdxChunk, l = y - base;
    // the walk enters a chunk a few bytes in: the head of a record a few chunks ahead
    if (c + 8 < nchunks) __builtin_prefetch(&rec[2 * (c + 8) * kIdxEntries]);
    uint64_t ex, ot;
    if (l < kIdxEntries) {
      ex = rec[2 * (c * kIdxEntries + l)];
      ot = rec[2 * (c * kIdxEntries + l) + 1];
    } else {
      host_walk(comp, n, y, std::min<uint64_t>(base + kIdxChunk, (uint64_t)n - 1), &ex, &ot);
    }
    path.push_back({y, O, ot, ex});
    O += ot;
    if (ex <= y) return 0;
    y = ex;
    if (O > size) break;  // a tag of this element (or an earlier one) fails: find the first
  }
  if (O != size) return path_first_error(ctx, n, size, path, err);
  std::vector<sm::StreamFrag> frags(nfrag);
  size_t k = 0;
  for (uint32_t f = 0; f < nfrag; ++f) {
    const uint64_t F = (uint64_t)f * 65536;
    while (k + 1 < path.size() && path[k].O + path[k].out <= F) ++k;
    frags[f] = {(uint32_t)path[k].y, (uint32_t)path[k].O, (uint32_t)F,
                f + 1 == nfrag ? 0xffffffffu : (uint32_t)(F + 65536)};
  }
  HT("host path + fragments")
  sm::StreamFrag* d_frags = (sm::StreamFrag*)((uint8_t*)ctx->idx.p + frag_off);
  int32_t* d_st = (int32_t*)((uint8_t*)ctx->idx.p + st_off);
  if (hipMemcpyAsync(d_frags, frags.data(), frags.size() * sizeof(sm::StreamFrag), hipMemcpyHostToDevice, s) !=
      hipSuccess)
    return -1;
  const uint32_t nfp = (nfrag + kOutPieceFrags - 1) / kOutPieceFrags;
  const uint32_t npiece = (host_out && nfp > 1 && ensure_copy_stream(ctx, nfp) == hipSuccess) ? nfp : 1;
  uint8_t* out = (uint8_t*)ctx->out.p;
  for (uint32_t pc = 0; pc < npiece; ++pc) {
    const uint32_t f0 = pc * kOutPieceFrags, f1 = npiece == 1 ? nfrag : std::min(nfrag, f0 + kOutPieceFrags);
    if (sm::launch_decompress_frags(d_in, n, size, out, d_frags + f0, f1 - f0, d_st + f0, s) != hipSuccess) return -1;
    if (npiece > 1 && hipEventRecord(ctx->ev[pc], s) != hipSuccess) return -1;
  }
  if (npiece > 1) {  // each piece's output goes down while the later pieces decode
    for (uint32_t pc = 0; pc < npiece; ++pc) {
      const size_t b0 = (size_t)pc * kOutPieceFrags * 65536;
      const size_t b1 = std::min((size_t)size, b0 + (size_t)kOutPieceFrags * 65536);
      if (hipStreamWaitEvent(ctx->copy, ctx->ev[pc], 0) != hipSuccess) return -1;
      if (hipMemcpyAsync(host_out + b0, out + b0, b1 - b0, hipMemcpyDeviceToHost, ctx->copy) != hipSuccess) return -1;
    }
    if (hipStreamSynchronize(ctx->copy) != hipSuccess) return -1;
  }
  std::vector<int32_t> st(nfrag);
  if (hipMemcpyAsync(st.data(), d_st, nfrag * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  HT("fragment decode")
  bool cross = false;
  for (int32_t v : st) {
    if (v == sm::kErrCross) cross = true;
    else if (v != sm::kOk) return path_first_error(ctx, n, size, path, err);  // the first error, in parallel
  }
  if (!cross) {
    *copied = npiece > 1;
    return 1;
  }
  // Not block-structured (a copy reaches into an earlier block): origin pointers per output
  // byte, resolved by pointer jumping (sm_decompress.hip, "any large stream").
  if (n >= 0x80000000u || size >= 0x80000000u) return 0;  // 31-bit positions
  const size_t npath = path.size();
  std::vector<sm::OriginPath> op(npath);
  for (size_t e = 0; e < npath; ++e)
    op[e] = {(uint32_t)path[e].y, (uint32_t)path[e].ex, (uint32_t)path[e].O, (uint32_t)path[e].out};
  const size_t p_off = 0, path_off = align_up((size_t)size * 4, 256), st2_off = align_up(path_off + npath * 16, 256);
  const size_t pend_off = align_up(st2_off + npath * 4, 256);
  if (ctx->org.ensure(pend_off + 16) != hipSuccess) return 0;  // (4 B per output byte: the in-order decode needs none)
  uint8_t* ob = (uint8_t*)ctx->org.p;
  uint32_t* d_P = (uint32_t*)(ob + p_off);
  sm::OriginPath* d_path = (sm::OriginPath*)(ob + path_off);
  int32_t* d_st2 = (int32_t*)(ob + st2_off);
  uint32_t* d_pend = (uint32_t*)(ob + pend_off);
  if (hipMemcpyAsync(d_path, op.data(), npath * sizeof(sm::OriginPath), hipMemcpyHostToDevice, s) != hipSuccess)
    return -1;
  if (sm::launch_origin_fill(d_in, n, size, d_path, (uint32_t)npath, d_P, d_st2, s) != hipSuccess) return -1;
  std::vector<int32_t> st2(npath);
  if (hipMemcpyAsync(st2.data(), d_st2, npath * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  for (int32_t v : st2)
    if (v != sm::kOk) return path_first_error(ctx, n, size, path, err);
  // round k moves every unresolved pointer >= 2^k chain steps: 32 rounds cover any size
  bool done = false;
  for (int round = 0; round < 32 && !done; ++round) {
    uint32_t pend = 0;
    if (hipMemsetAsync(d_pend, 0, 4, s) != hipSuccess) return -1;
    if (sm::launch_origin_resolve(d_P, size, d_pend, s) != hipSuccess) return -1;
    if (hipMemcpyAsync(&pend, d_pend, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    done = pend == 0;
  }
  if (!done) return 0;
  if (sm::launch_origin_gather(d_in, d_P, size, (uint8_t*)ctx->out.p, s) != hipSuccess) return -1;
  if (ctx->org.cap > kOrgKeep) {  // 4 B per output byte: do not keep gigabytes in the context
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    ctx->org.release();
  }
  return 2;
}

// A small stream entirely on the device (sm_decompress.hip, "a small stream"): index, chain,
// origin pointers, resolve, gather, then one synchronisation with the output's download.
// Returns 4 with the output in host_out, 0 to fall back (an error or anything unexpected: the
// old paths find the reference's first error), -1 on a device error.
#ifndef SM_SMALL_MIN
#define SM_SMALL_MIN 4096
#endif
constexpr uint32_t kSmallMinOutput = SM_SMALL_MIN;  // smaller streams: the one-wave decode
constexpr uint32_t kSmallMaxChunks = (1u << 20) / sm::kSmallChunk;  // compressed bodies up to 1 MiB
// Index chunk size for path 4: 512-byte chunks halve the index and fill kernels' per-chunk walk
// (both latency chains of 256-byte windows) but double the chain's elements and split more long
// literals into deep entries.  Measured single calls (fast streams, r05): html (body 0.22 of the
// output) 83 -> 70 us, alice29.txt (0.56) 82 -> 74, paper-100k.pdf (0.82, long literals) 145 ->
// 184, urls.10K (0.48, 336 KB body) 150 -> 156.  So: fine chunks for bodies up to 0.6 of the
// output and 256 KiB.
#ifndef SM_SMALL_FINE_BODY10
#define SM_SMALL_FINE_BODY10 6
#endif
#ifndef SM_SMALL_TINY_BODY
#define SM_SMALL_TINY_BODY 16384  // bodies up to this size ...
#endif
#ifndef SM_SMALL_TINY_BODY10
#define SM_SMALL_TINY_BODY10 9    // ... and at most this many tenths of the output: 128-byte chunks
#endif
// path 4's index chunk: 128 bytes for small bodies with copies (sample-tweet.json 52 -> 45 us, 4-16
// KiB of text 51-56 -> 45-48 us), 512 for bodies of mostly copies, else 1024 (literal-rich
// streams, where finer chunks lengthen the chain: paper-100k.pdf 137 -> 168 us at 512)
uint32_t small_chunk(uint32_t body, uint32_t size) {
  if (body <= SM_SMALL_TINY_BODY && (uint64_t)body * 10 <= (uint64_t)size * SM_SMALL_TINY_BODY10)
    return sm::kSmallChunkTiny;
  if ((uint64_t)body * 10 > (uint64_t)size * SM_SMALL_FINE_BODY10 || body > (256u << 10)) return sm::kSmallChunk;
  return sm::kSmallChunkFine;
}
constexpr uint32_t kSmallMaxOutput = 64u << 20;    // 4 B of origin pointer per output byte
constexpr uint32_t kPinnedOutMax = 16u << 20;      // outputs the last kernel writes into the pinned staging

// comp: the call's input on the host.  It goes to the device through the index launch (the pinned
// staging read there, the device copy written there); 0 returns before any launch leave
// ctx->in without it.
int small_uncompress(sm_ctx* ctx, const uint8_t* comp, uint32_t n, uint32_t ip0, uint32_t size, uint8_t* host_out) {
  using sm::kIdxEntries;
  const uint32_t chunk = small_chunk(n - ip0, size);
  const uint32_t nchunks = (n - ip0 + chunk - 1) / chunk;
  uint32_t rounds = 1;  // kSmallHops^rounds >= size: every chain (at most size steps) resolves
  uint32_t hops = sm::kSmallHops;
  if (size <= sm::kOneLaunchHops)
    hops = std::max(hops, size);  // one launch of size hops (up to 256 KiB of output: one dispatch fewer)
  else
    for (uint64_t reach = sm::kSmallHops; reach < size; reach *= sm::kSmallHops) ++rounds;
  const size_t path_off = align_up((size_t)nchunks * kIdxEntries * 8 + (size_t)nchunks * sm::kDeepChains * sm::kDeepLevels * 16, 256);  // records, deep records
  const size_t ctl_off = align_up(path_off + (size_t)nchunks * sizeof(sm::OriginPath), 256);
  const size_t ctl_n = 4 + rounds;
  if (ctx->idx.ensure(ctl_off + ctl_n * 4) != hipSuccess) return 0;
  if (ctx->org.ensure((size_t)size * 4) != hipSuccess) return 0;
  // the output and the verdict words straight into the pinned staging (a large output: the words
  // only, the output by a copy into host_out)
  const bool pin_out = size <= kPinnedOutMax;
  const size_t w_off = pin_out ? align_up(size, 256) : 0;
  if (ctx->stage.ensure(w_off + 64) != hipSuccess || !ctx->stage.dp) return 0;
  hipStream_t s = ctx->stream;
  uint8_t* ib = (uint8_t*)ctx->idx.p;
  uint32_t* d_ctl = (uint32_t*)(ib + ctl_off);
  uint8_t* const sdp = (uint8_t*)ctx->stage.dp;
  if (!stage_in_acquire(ctx, n)) return 0;
  memcpy(ctx->stage_in.p, comp, n);
  // the third verdict word is written by the device only when a pointer stays unresolved
  ((volatile uint32_t*)((uint8_t*)ctx->stage.p + w_off))[2] = 0;
  const hipError_t le = sm::launch_small_decode((const uint8_t*)ctx->in.p, (const uint8_t*)ctx->stage_in.dp, n, ip0,
                                                size, chunk, nchunks, (uint32_t*)ib, (sm::OriginPath*)(ib + path_off),
                                                d_ctl, (uint32_t*)ctx->org.p, rounds, hops,
                                                pin_out ? sdp : (uint8_t*)ctx->out.p, (uint32_t*)(sdp + w_off), s);
  if (le != hipSuccess || stage_in_release(ctx, s) != hipSuccess) {
    (void)hipStreamSynchronize(s);  // (no launch may still read the staging when the call returns)
    return -1;
  }
  if (!pin_out && hipMemcpyAsync(host_out, ctx->out.p, size, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  const volatile uint32_t* w = (const volatile uint32_t*)((uint8_t*)ctx->stage.p + w_off);
  if (w[0] || w[1] || w[2]) return 0;  // (w[2]: never, by the round count -- checked, not assumed)
  if (pin_out) memcpy(host_out, ctx->stage.p, size);
  return 4;
}

}  // namespace

#define SM_CHECK(x)                 \
  do {                              \
    if ((x) != hipSuccess) return SM_ERR_DEVICE; \
  } while (0)

namespace {
// Shard [b0, b1) of a host batch, rebased so the single-context call copies only the shard's
// bytes: offsets relative to the shard's lowest input / output offset.
struct Shard {
  uint32_t b0 = 0, n = 0;
  uint64_t in_base = 0, out_base = 0;
  std::vector<uint64_t> in_off, out_off;
};

std::vector<Shard> make_shards(int nctx, uint32_t nblk, const uint64_t* in_off, const uint64_t* out_off) {
  std::vector<Shard> sh((size_t)nctx);
  for (int i = 0; i < nctx; ++i) {
    Shard& s = sh[(size_t)i];
    s.b0 = (uint32_t)((uint64_t)nblk * (uint64_t)i / (uint64_t)nctx);
    s.n = (uint32_t)((uint64_t)nblk * (uint64_t)(i + 1) / (uint64_t)nctx) - s.b0;
    if (s.n == 0) continue;
    s.in_base = *std::min_element(in_off + s.b0, in_off + s.b0 + s.n);
    s.out_base = *std::min_element(out_off + s.b0, out_off + s.b0 + s.n);
    s.in_off.resize(s.n);
    s.out_off.resize(s.n);
    for (uint32_t k = 0; k < s.n; ++k) {
      s.in_off[k] = in_off[s.b0 + k] - s.in_base;
      s.out_off[k] = out_off[s.b0 + k] - s.out_base;
    }
  }
  return sh;
}

template <typename F>
sm_status run_shards(int nctx, F&& shard_fn) {
  std::vector<sm_status> st((size_t)nctx, SM_OK);
  std::vector<std::thread> th;
  th.reserve((size_t)nctx);
  for (int i = 0; i < nctx; ++i) th.emplace_back([&, i] { st[(size_t)i] = shard_fn(i); });
  for (auto& t : th) t.join();
  for (sm_status x : st)
    if (x != SM_OK) return x;
  return SM_OK;
}

// The blocks [d_src + src_off[b], +len[b]) of a device batch back to host + out_off[b]: one
// gather launch packs them back to back in ctx->out2, one D2H transfer brings them into the
// pinned staging buffer, and the host scatters them (instead of one small copy per block).
// len: host copy of the lengths (0 = nothing to copy); d_len: the same on the device.
sm_status gather_to_host(sm_ctx* ctx, const uint8_t* d_src, const uint64_t* d_src_off, const uint32_t* d_len,
                         const uint32_t* len, uint32_t nblk, const uint64_t* out_off, uint8_t* host) {
  hipStream_t s = ctx->stream;
  std::vector<uint64_t> dst(nblk);
  uint64_t total = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    dst[b] = total;
    total += len[b];
  }
  if (total == 0) return SM_OK;
  if (ctx->gat.ensure(8 * (size_t)nblk) != hipSuccess || ctx->out2.ensure(total + 16) != hipSuccess ||
      ctx->stage.ensure(total) != hipSuccess)
    return SM_ERR_DEVICE;
  uint64_t* d_dst = (uint64_t*)ctx->gat.p;
  if (hipMemcpyAsync(d_dst, dst.data(), 8 * (size_t)nblk, hipMemcpyHostToDevice, s) != hipSuccess) return SM_ERR_DEVICE;
  if (sm::launch_gather(d_src, d_src_off, d_len, d_dst, (uint8_t*)ctx->out2.p, nblk, s) != hipSuccess)
    return SM_ERR_DEVICE;
  if (hipMemcpyAsync(ctx->stage.p, ctx->out2.p, total, hipMemcpyDeviceToHost, s) != hipSuccess) return SM_ERR_DEVICE;
  if (hipStreamSynchronize(s) != hipSuccess) return SM_ERR_DEVICE;
  const uint8_t* st = (const uint8_t*)ctx->stage.p;
  for (uint32_t b = 0; b < nblk; ++b)
    if (len[b]) memcpy(host + out_off[b], st + dst[b], len[b]);
  return SM_OK;
}

// The compressor's lengths as the host receives them: a length above the block's bound is an
// error mark (SM_OUT_LEN_ERROR | k: a bounded wait inside the kernel gave up; 0xffffffff: a block
// over 64 KiB, rejected before the launch here).  Checked before any length is summed, allocated
// or gathered, so a mark never becomes a copy size.
sm_status check_compressed_lengths(const uint32_t* out_len, const uint32_t* in_len, uint32_t nblk) {
  for (uint32_t b = 0; b < nblk; ++b)
    if (out_len[b] > sm::max_compressed_length(in_len[b])) return out_len[b] >= SM_OUT_LEN_ERROR ? SM_ERR_DEVICE : SM_ERR_ARGUMENT;
  return SM_OK;
}

bool valid_ctxs(sm_ctx* const* ctxs, int nctx) {
  if (!ctxs || nctx <= 0) return false;
  for (int i = 0; i < nctx; ++i) {
    if (!ctxs[i]) return false;
    for (int j = 0; j < i; ++j)
      if (ctxs[j] == ctxs[i]) return false;  // two shards on one ctx would race on its scratch
  }
  return true;
}
}  // namespace

extern "C" {

int sm_ctx_last_path(sm_ctx* ctx) { return ctx ? ctx->last_path : -1; }

sm_status sm_ctx_set_small_decode(sm_ctx* ctx, int enable) {
  if (!ctx) return SM_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->small = enable != 0;
  return SM_OK;
}

sm_status sm_ctx_set_split_compress(sm_ctx* ctx, int enable) {
  if (!ctx) return SM_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->split = enable != 0;
  return SM_OK;
}

int sm_ctx_last_compress_split(sm_ctx* ctx) { return ctx ? (ctx->last_split ? 1 : 0) : -1; }

const char* sm_status_message(sm_status st) {
  switch (st) {
    case SM_OK: return "OK";
    case SM_INVALID_INPUT: return "Invalid input.";
    case SM_BUFFER_TOO_SMALL: return "Buffer too small.";
    case SM_ERR_INPUT_TOO_LARGE: return "Input too large.";
    case SM_ERR_INVALID: return "Invalid input.";
    case SM_ERR_VARINT: return "Could not decode varint32.";
    case SM_ERR_COPY_OFFSET: return "Invalid input: corrupt copy offset";
    case SM_ERR_COPY_LENGTH: return "Invalid input: corrupt copy length";
    case SM_ERR_LITERAL: return "Invalid input: corrupt literal";
    case SM_ERR_DEVICE: return "HIP device error.";
    case SM_ERR_ARGUMENT: return "Invalid argument.";
    default: return "Unknown status.";
  }
}

const char* sm_version(void) { return "snappy_mi355x gfx950 " SM_VERSION_STR; }

size_t sm_max_compressed_length(size_t n) { return 32 + n + n / 6; }

sm_status sm_parse32(const uint8_t* buf, size_t len, size_t off, uint32_t* value, size_t* next) {
  uint32_t result = 0;
  for (int i = 0; i < 5; ++i) {
    if (off + i >= len) return SM_ERR_VARINT;
    uint32_t b = buf[off + i];
    if (i < 4) {
      result |= (b & 0x7f) << (7 * i);
      if (b < 0x80) {
        if (value) *value = result;
        if (next) *next = off + i + 1;
        return SM_OK;
      }
    } else {
      result |= (b & 0x7f) << 28;
      if (b < 0x10) {
        if (value) *value = result;
        if (next) *next = off + 5;
        return SM_OK;
      }
    }
  }
  return SM_ERR_VARINT;
}

size_t sm_encode32(uint8_t* buf, uint32_t v) {
  size_t i = 0;
  while (v >= 0x80) {
    buf[i++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  buf[i++] = (uint8_t)v;
  return i;
}

sm_status sm_find_match_length(const uint8_t* buf, size_t len, size_t i1, size_t i2, size_t limit,
                               size_t* matched) {
  if (!matched || (len && !buf)) return SM_ERR_ARGUMENT;
  // 8 bytes at a time while i2 + 7 <= limit, then bytes (internal.jl:356-386); every read
  // the reference makes must lie inside buf
  auto ld64 = [&](size_t i, uint64_t* v) {
    if (i + 8 > len) return false;
    memcpy(v, buf + i, 8);
    return true;
  };
  size_t m = 0;
  while (i2 + 7 <= limit) {
    uint64_t a, b;
    if (!ld64(i1 + m, &a) || !ld64(i2, &b)) return SM_ERR_ARGUMENT;
    if (a != b) {
      *matched = m + (__builtin_ctzll(a ^ b) >> 3);
      return SM_OK;
    }
    i2 += 8;
    m += 8;
  }
  while (i2 <= limit) {
    if (i2 >= len || i1 + m >= len) return SM_ERR_ARGUMENT;
    if (buf[i1 + m] != buf[i2]) break;
    ++i2;
    ++m;
  }
  *matched = m;
  return SM_OK;
}

sm_status sm_uncompressed_length(const char* compressed, size_t n, size_t* result) {
  uint32_t v = 0;
  sm_status st = sm_parse32((const uint8_t*)compressed, n, 0, &v, nullptr);
  if (st == SM_OK && result) *result = v;
  return st;
}

sm_ctx* sm_ctx_create(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count) return nullptr;
  sm_ctx* ctx = new (std::nothrow) sm_ctx();
  if (!ctx) return nullptr;
  ctx->device = device;
  DeviceGuard g(device);
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void sm_ctx_destroy(sm_ctx* ctx) {
  if (!ctx) return;
  {
    DeviceGuard g(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->in.release();
    ctx->out.release();
    ctx->out2.release();
    ctx->meta.release();
    ctx->idx.release();
    ctx->gat.release();
    ctx->org.release();
    ctx->stage.release();
    ctx->stage_in.release();
    if (ctx->in_ev) (void)hipEventDestroy(ctx->in_ev);
    if (ctx->copy) {
      (void)hipStreamSynchronize(ctx->copy);
      (void)hipStreamDestroy(ctx->copy);
    }
    for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
}

void* sm_ctx_stream(sm_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

sm_status sm_compress_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                   const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                   const uint64_t* d_out_off, uint32_t* d_out_len, int mode, void* stream) {
  if (!ctx || !valid_mode(mode)) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  sm::CompressArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, nblk, 0, 1};
  SM_CHECK(sm::launch_compress(a, mode, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_compress_fragments_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                       const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                       const uint64_t* d_out_off, uint32_t* d_out_len, uint64_t total_len,
                                       int mode, void* stream) {
  if (!ctx || !valid_mode(mode)) return SM_ERR_ARGUMENT;
  if (total_len > 0xffffffffull) return SM_ERR_INPUT_TOO_LARGE;        // src/Snappy.jl:21
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  sm::CompressArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, nblk, sm::hashtable_size(total_len), 0};
  SM_CHECK(sm::launch_compress(a, mode, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_place_fragments_device(sm_ctx* ctx, const uint8_t* d_src, const uint64_t* d_src_off,
                                    const uint32_t* d_len, uint32_t nfrag, const uint64_t* d_dst_off,
                                    uint64_t total_len, int write_header, uint8_t* d_dst, uint64_t dst_capacity,
                                    uint64_t* d_local_off, int32_t* d_status, void* stream) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (total_len > 0xffffffffull) return SM_ERR_INPUT_TOO_LARGE;  // src/Snappy.jl:21
  if (nfrag == 0 && !write_header) return SM_OK;
  if (!d_dst || (nfrag && (!d_src || !d_src_off || !d_len || !d_dst_off))) return SM_ERR_ARGUMENT;
  if (write_header && dst_capacity < sm::varint_len((uint32_t)total_len)) return SM_BUFFER_TOO_SMALL;
  DeviceGuard g(ctx->device);
  SM_CHECK(sm::launch_place(d_src, d_src_off, d_len, d_dst_off, nfrag, total_len, write_header ? 1 : 0, dst_capacity,
                            d_dst, d_local_off, d_status, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_uncompress_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                     const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                     const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                     uint32_t* d_out_len, int32_t* d_status, void* stream) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_cap || !d_out_len || !d_status)
    return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  sm::DecompressArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_cap, d_out_len, d_status, nblk};
  SM_CHECK(sm::launch_decompress(a, 0, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_compress_batch(sm_ctx* ctx, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                            uint32_t nblk, uint8_t* out, const uint64_t* out_off, uint32_t* out_len, int mode) {
  if (!ctx || !valid_mode(mode)) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_len) return SM_ERR_ARGUMENT;
  size_t in_total = 0, out_total = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    if (in_len[b] > SM_BLOCK_SIZE) return SM_ERR_ARGUMENT;
    size_t ie = in_off[b] + in_len[b];
    size_t oe = out_off[b] + sm_max_compressed_length(in_len[b]);
    if (ie > in_total) in_total = ie;
    if (oe > out_total) out_total = oe;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  size_t meta_bytes = (size_t)nblk * (8 + 4 + 8 + 4);
  SM_CHECK(ctx->in.ensure(in_total + 16));
  SM_CHECK(ctx->out.ensure(out_total + 16));
  SM_CHECK(ctx->meta.ensure(meta_bytes + 64));
  uint8_t* m = (uint8_t*)ctx->meta.p;
  uint64_t* d_in_off = (uint64_t*)m;
  uint64_t* d_out_off = (uint64_t*)(m + 8 * (size_t)nblk);
  uint32_t* d_in_len = (uint32_t*)(m + 16 * (size_t)nblk);
  uint32_t* d_out_len = (uint32_t*)(m + 20 * (size_t)nblk);
  SM_CHECK(hipMemcpyAsync(ctx->in.p, in, in_total, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_in_off, in_off, 8 * (size_t)nblk, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_out_off, out_off, 8 * (size_t)nblk, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_in_len, in_len, 4 * (size_t)nblk, hipMemcpyHostToDevice, s));
  sm::CompressArgs a{(const uint8_t*)ctx->in.p, d_in_off, d_in_len, (uint8_t*)ctx->out.p, d_out_off, d_out_len,
                     nblk, 0, 1};
  SM_CHECK(sm::launch_compress(a, mode, s));
  SM_CHECK(hipMemcpyAsync(out_len, d_out_len, 4 * (size_t)nblk, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  const sm_status lst = check_compressed_lengths(out_len, in_len, nblk);
  if (lst != SM_OK) return lst;
  // copy back only each block's bytes
  return gather_to_host(ctx, (const uint8_t*)ctx->out.p, d_out_off, d_out_len, out_len, nblk, out_off, out);
}

sm_status sm_uncompress_batch(sm_ctx* ctx, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                              uint32_t nblk, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                              uint32_t* out_len, int32_t* status) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len || !status) return SM_ERR_ARGUMENT;
  size_t in_total = 0, out_total = 0;
  for (uint32_t b = 0; b < nblk; ++b) {
    size_t ie = in_off[b] + in_len[b];
    size_t oe = out_off[b] + out_cap[b];
    if (ie > in_total) in_total = ie;
    if (oe > out_total) out_total = oe;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  size_t meta_bytes = (size_t)nblk * (8 + 8 + 4 + 4 + 4 + 4);
  SM_CHECK(ctx->in.ensure(in_total + 16));
  SM_CHECK(ctx->out.ensure(out_total + 16));
  SM_CHECK(ctx->meta.ensure(meta_bytes + 64));
  uint8_t* m = (uint8_t*)ctx->meta.p;
  uint64_t* d_in_off = (uint64_t*)m;
  uint64_t* d_out_off = (uint64_t*)(m + 8 * (size_t)nblk);
  uint32_t* d_in_len = (uint32_t*)(m + 16 * (size_t)nblk);
  uint32_t* d_out_cap = (uint32_t*)(m + 20 * (size_t)nblk);
  uint32_t* d_out_len = (uint32_t*)(m + 24 * (size_t)nblk);
  int32_t* d_status = (int32_t*)(m + 28 * (size_t)nblk);
  SM_CHECK(hipMemcpyAsync(ctx->in.p, in, in_total, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_in_off, in_off, 8 * (size_t)nblk, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_out_off, out_off, 8 * (size_t)nblk, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_in_len, in_len, 4 * (size_t)nblk, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_out_cap, out_cap, 4 * (size_t)nblk, hipMemcpyHostToDevice, s));
  sm::DecompressArgs a{(const uint8_t*)ctx->in.p, d_in_off, d_in_len, (uint8_t*)ctx->out.p, d_out_off,
                       d_out_cap, d_out_len, d_status, nblk};
  SM_CHECK(sm::launch_decompress(a, 0, s));
  SM_CHECK(hipMemcpyAsync(out_len, d_out_len, 4 * (size_t)nblk, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipMemcpyAsync(status, d_status, 4 * (size_t)nblk, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  for (uint32_t b = 0; b < nblk; ++b)
    if (status[b] != SM_OK) out_len[b] = 0;  // (the kernel already reports 0 for failed blocks)
  return gather_to_host(ctx, (const uint8_t*)ctx->out.p, d_out_off, d_out_len, out_len, nblk, out_off, out);
}

sm_status sm_validate_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                   const uint32_t* d_in_len, uint32_t nblk, int32_t* d_status, void* stream) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_status) return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  SM_CHECK(sm::launch_validate(d_in, d_in_off, d_in_len, nblk, d_status, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_uncompressed_length_batch_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                              const uint32_t* d_in_len, uint32_t nblk, uint32_t* d_len,
                                              int32_t* d_status, void* stream) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_len || !d_status) return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  SM_CHECK(sm::launch_uncompressed_length(d_in, d_in_off, d_in_len, nblk, d_len, d_status, (hipStream_t)stream));
  return SM_OK;
}

sm_status sm_compress_batch_sharded(sm_ctx* const* ctxs, int nctx, const uint8_t* in, const uint64_t* in_off,
                                    const uint32_t* in_len, uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                                    uint32_t* out_len, int mode) {
  if (!valid_ctxs(ctxs, nctx) || !valid_mode(mode)) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_len) return SM_ERR_ARGUMENT;
  for (uint32_t b = 0; b < nblk; ++b)
    if (in_len[b] > SM_BLOCK_SIZE) return SM_ERR_ARGUMENT;
  const std::vector<Shard> sh = make_shards(nctx, nblk, in_off, out_off);
  return run_shards(nctx, [&](int i) -> sm_status {
    const Shard& s = sh[(size_t)i];
    if (s.n == 0) return SM_OK;
    return sm_compress_batch(ctxs[i], in + s.in_base, s.in_off.data(), in_len + s.b0, s.n, out + s.out_base,
                             s.out_off.data(), out_len + s.b0, mode);
  });
}

sm_status sm_uncompress_batch_sharded(sm_ctx* const* ctxs, int nctx, const uint8_t* in, const uint64_t* in_off,
                                      const uint32_t* in_len, uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                                      const uint32_t* out_cap, uint32_t* out_len, int32_t* status) {
  if (!valid_ctxs(ctxs, nctx)) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !out_len || !status) return SM_ERR_ARGUMENT;
  const std::vector<Shard> sh = make_shards(nctx, nblk, in_off, out_off);
  return run_shards(nctx, [&](int i) -> sm_status {
    const Shard& s = sh[(size_t)i];
    if (s.n == 0) return SM_OK;
    return sm_uncompress_batch(ctxs[i], in + s.in_base, s.in_off.data(), in_len + s.b0, s.n, out + s.out_base,
                               s.out_off.data(), out_cap + s.b0, out_len + s.b0, status + s.b0);
  });
}

sm_status sm_validate_compressed_buffer(sm_ctx* ctx, const char* compressed, size_t n) {
  if (!ctx || (n && !compressed)) return SM_ERR_ARGUMENT;
  if (n > 0xffffffffull) return SM_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  SM_CHECK(ctx->in.ensure(n + 16));
  SM_CHECK(ctx->meta.ensure(64));
  uint8_t* m = (uint8_t*)ctx->meta.p;
  uint64_t* d_off = (uint64_t*)m;
  uint32_t* d_len = (uint32_t*)(m + 8);
  int32_t* d_status = (int32_t*)(m + 12);
  const uint64_t zero = 0;
  const uint32_t len32 = (uint32_t)n;
  int32_t st = SM_ERR_DEVICE;
  SM_CHECK(upload_input(ctx, compressed, n, s));
  SM_CHECK(hipMemcpyAsync(d_off, &zero, 8, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_len, &len32, 4, hipMemcpyHostToDevice, s));
  SM_CHECK(sm::launch_validate((const uint8_t*)ctx->in.p, d_off, d_len, 1, d_status, s));
  SM_CHECK(hipMemcpyAsync(&st, d_status, 4, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  return st;
}

// src/Snappy.jl:20-36 on the device: every 64 KiB fragment is one wave; fragments use the
// table size of the WHOLE input (Q2) and no per-fragment header; a gather kernel then
// concatenates them behind the varint header.
sm_status sm_compress(sm_ctx* ctx, const char* input, size_t n, char* compressed, size_t* compressed_length,
                      int mode) {
  if (!ctx || !compressed_length || (n && !input) || !compressed) return SM_ERR_ARGUMENT;
  if (!valid_mode(mode)) return SM_ERR_ARGUMENT;
  if (n > 0xffffffffull) return SM_ERR_INPUT_TOO_LARGE;                  // Snappy.jl:21
  if (*compressed_length < sm_max_compressed_length(n)) return SM_BUFFER_TOO_SMALL;
  uint8_t hdr[5];
  size_t hl = sm_encode32(hdr, (uint32_t)n);                                // Snappy.jl:26
  memcpy(compressed, hdr, hl);
  if (n == 0) {
    *compressed_length = hl;
    return SM_OK;
  }
  const uint32_t nfrag = (uint32_t)((n + SM_BLOCK_SIZE - 1) / SM_BLOCK_SIZE);
  const size_t slot = align_up(sm_max_compressed_length(SM_BLOCK_SIZE) + 8, 256);
  std::vector<uint64_t> in_off(nfrag), out_off(nfrag), dst_off(nfrag);
  std::vector<uint32_t> in_len(nfrag), out_len(nfrag);
  for (uint32_t i = 0; i < nfrag; ++i) {
    in_off[i] = (uint64_t)i * SM_BLOCK_SIZE;
    size_t e = in_off[i] + SM_BLOCK_SIZE;
    in_len[i] = (uint32_t)((e < n ? e : n) - in_off[i]);
    out_off[i] = (uint64_t)i * slot;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  ctx->last_split = false;
  SM_CHECK(ctx->in.ensure(n + 16));
  SM_CHECK(ctx->out.ensure((size_t)nfrag * slot));
  SM_CHECK(ctx->out2.ensure(sm_max_compressed_length(n) + 16));
  SM_CHECK(ctx->meta.ensure((size_t)nfrag * 32 + 64 + 4 * 256));
  uint8_t* m = (uint8_t*)ctx->meta.p;
  uint64_t* d_in_off = (uint64_t*)m;
  uint64_t* d_out_off = (uint64_t*)(m + 8 * (size_t)nfrag);
  uint64_t* d_dst_off = (uint64_t*)(m + 16 * (size_t)nfrag);
  uint32_t* d_in_len = (uint32_t*)(m + 24 * (size_t)nfrag);
  uint32_t* d_out_len = (uint32_t*)(m + 28 * (size_t)nfrag);
  uint32_t* d_part_len = (uint32_t*)(m + 32 * (size_t)nfrag + 64);
  HT_DECL
  // Small inputs: one synchronisation -- the fragment table and the gather (with the lengths'
  // prefix sums) on the device; the gather kernel writes the stream body into the context's
  // pinned staging (device-mapped: no copy engine behind the kernels), copied out on the host.
  // The fast modes parse each fragment in parts on their own workgroups (k_compress_sc_span: the
  // same bytes, a fraction of one block's latency; up to 256 parts in all, one per CU).
  const size_t t_off = align_up(sm_max_compressed_length(n) + 16, 256);
  if (n <= kSmallCompressMax && ctx->stage.ensure(t_off + 16) == hipSuccess && ctx->stage.dp) {
    uint32_t parts = 1;
    if (mode != SM_MODE_REFERENCE && ctx->split) {
      uint32_t p2 = 1;
      while (p2 < nfrag) p2 <<= 1;
      parts = std::min<uint32_t>(sm::kWave, 256 / p2);  // nfrag * parts <= 256 gather units
    }
    const uint32_t span = (uint32_t)((SM_BLOCK_SIZE / 1024 + parts - 1) / parts);
    const size_t sl = parts > 1 ? std::max<size_t>(slot, (size_t)parts * span * sm::kSpanSlot) : slot;
    SM_CHECK(ctx->out.ensure((size_t)nfrag * sl));
    sm::CompressArgs a{(const uint8_t*)ctx->in.p, d_in_off, d_in_len, (uint8_t*)ctx->out.p, d_out_off, d_out_len,
                       nfrag, sm::hashtable_size(n), 0};
    // fast modes: the screen (the first kernel) reads the input from the pinned staging and leaves
    // the device copy the parse reads -- no separate upload
    const bool staged = mode != SM_MODE_REFERENCE && stage_in_acquire(ctx, n);
    if (staged) {
      memcpy(ctx->stage_in.p, input, n);
      a.in_host = (const uint8_t*)ctx->stage_in.dp;
    } else {
      SM_CHECK(upload_input(ctx, input, n, s));
    }
    if (mode == SM_MODE_REFERENCE) {
      SM_CHECK(sm::launch_frag_plan(n, nfrag, sl, d_in_off, d_in_len, d_out_off, s));
    } else {  // (the screen, the fast modes' first kernel, writes the fragment table)
      a.plan_n = n;
      a.plan_slot = sl;
    }
    // the gather writes the body and its (length, error) pair straight into the pinned staging
    uint8_t* const sdp = (uint8_t*)ctx->stage.dp;
    const sm::ScSpan sp{parts, span, (uint64_t)span * sm::kSpanSlot, d_part_len};
    hipError_t le = parts > 1 ? sm::launch_compress_span(a, mode, sp, s) : sm::launch_compress(a, mode, s);
    if (le == hipSuccess)
      le = parts > 1 ? sm::launch_parts_gather((const uint8_t*)ctx->out.p, d_out_off, sp, (const uint8_t*)ctx->in.p,
                                               d_in_off, d_in_len, nfrag, (uint64_t*)(sdp + t_off), sdp, s)
                     : sm::launch_frag_gather((const uint8_t*)ctx->out.p, d_out_off, d_out_len, d_in_len, nfrag,
                                              (uint64_t*)(sdp + t_off), sdp, s);
    // the staging's release after the last launch (an event between the launches costs each call
    // ~4 us), and recorded even when a launch failed: the screen, its only reader, may be queued
    if (staged) {
      const hipError_t re = stage_in_release(ctx, s);
      if (le == hipSuccess) le = re;
    }
    if (le != hipSuccess) {
      (void)hipStreamSynchronize(s);
      return SM_ERR_DEVICE;
    }
    SM_CHECK(hipStreamSynchronize(s));
    HT("compress (small): all")
    const volatile uint64_t* tot = (const volatile uint64_t*)((uint8_t*)ctx->stage.p + t_off);
    const uint64_t len = tot[0];
    if (tot[1]) return SM_ERR_DEVICE;  // a block's error mark (SM_OUT_LEN_ERROR), never expected
    if (hl + len > *compressed_length) return SM_BUFFER_TOO_SMALL;
    memcpy(compressed + hl, ctx->stage.p, len);
    *compressed_length = hl + len;
    ctx->last_split = parts > 1;
    return SM_OK;
  }
  SM_CHECK(hipMemcpyAsync(d_in_off, in_off.data(), 8 * (size_t)nfrag, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_out_off, out_off.data(), 8 * (size_t)nfrag, hipMemcpyHostToDevice, s));
  SM_CHECK(hipMemcpyAsync(d_in_len, in_len.data(), 4 * (size_t)nfrag, hipMemcpyHostToDevice, s));
  // Large inputs go up in pieces on the copy stream, and each piece's fragments compress as
  // soon as it lands, so the kernels run under the rest of the upload.
  uint32_t npiece = n >= kPipeMinInput ? (nfrag + kPieceFrags - 1) / kPieceFrags : 1;
  if (npiece > 1 && ensure_copy_stream(ctx, npiece) != hipSuccess) npiece = 1;  // one upload then
  for (uint32_t pc = 0; pc < npiece; ++pc) {
    const uint32_t f0 = pc * kPieceFrags, f1 = npiece == 1 ? nfrag : std::min(nfrag, f0 + kPieceFrags);
    const size_t b0 = (size_t)f0 * SM_BLOCK_SIZE, b1 = std::min(n, (size_t)f1 * SM_BLOCK_SIZE);
    if (npiece == 1) {
      SM_CHECK(hipMemcpyAsync(ctx->in.p, input, n, hipMemcpyHostToDevice, s));
    } else {
      SM_CHECK(hipMemcpyAsync((uint8_t*)ctx->in.p + b0, input + b0, b1 - b0, hipMemcpyHostToDevice, ctx->copy));
      SM_CHECK(hipEventRecord(ctx->ev[pc], ctx->copy));
      SM_CHECK(hipStreamWaitEvent(s, ctx->ev[pc], 0));
    }
    sm::CompressArgs a{(const uint8_t*)ctx->in.p, d_in_off + f0, d_in_len + f0, (uint8_t*)ctx->out.p,
                       d_out_off + f0, d_out_len + f0, f1 - f0, sm::hashtable_size(n), 0};
    SM_CHECK(sm::launch_compress(a, mode, s));
  }
  HT("compress: H2D input + kernels")
  SM_CHECK(hipMemcpyAsync(out_len.data(), d_out_len, 4 * (size_t)nfrag, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  HT("compress: kernels + lengths")
  {
    const sm_status lst = check_compressed_lengths(out_len.data(), in_len.data(), nfrag);
    if (lst != SM_OK) return lst;
  }
  size_t total = 0;
  for (uint32_t i = 0; i < nfrag; ++i) {
    dst_off[i] = total;
    total += out_len[i];
  }
  if (hl + total > *compressed_length) return SM_BUFFER_TOO_SMALL;
  SM_CHECK(hipMemcpyAsync(d_dst_off, dst_off.data(), 8 * (size_t)nfrag, hipMemcpyHostToDevice, s));
  SM_CHECK(sm::launch_gather((const uint8_t*)ctx->out.p, d_out_off, d_out_len, d_dst_off, (uint8_t*)ctx->out2.p,
                             nfrag, s));
  HT("compress: gather")
  SM_CHECK(hipMemcpyAsync(compressed + hl, ctx->out2.p, total, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  HT("compress: D2H output")
  *compressed_length = hl + total;
  return SM_OK;
}

// src/Snappy.jl:46-52: header parsed on the host (to size the output), the stream decoded by
// one wave (foreign streams carry no fragment index).
sm_status sm_uncompress(sm_ctx* ctx, const char* compressed, size_t n, char* uncompressed,
                        size_t* uncompressed_length) {
  if (!ctx || !uncompressed_length || (n && !compressed)) return SM_ERR_ARGUMENT;
  uint32_t size = 0;
  sm_status st = sm_parse32((const uint8_t*)compressed, n, 0, &size, nullptr);
  if (st != SM_OK) return st;
  if (n > 0xffffffffull) return SM_ERR_ARGUMENT;
  if (*uncompressed_length < size) return SM_BUFFER_TOO_SMALL;
  if (size && !uncompressed) return SM_ERR_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  SM_CHECK(ctx->in.ensure(n + 16));
  SM_CHECK(ctx->out.ensure((size_t)size + 16));
  SM_CHECK(ctx->meta.ensure(64));
  uint8_t* m = (uint8_t*)ctx->meta.p;
  uint64_t* d_off = (uint64_t*)m;           // in_off = out_off = 0
  uint32_t* d_in_len = (uint32_t*)(m + 8);
  uint32_t* d_cap = (uint32_t*)(m + 12);
  uint32_t* d_out_len = (uint32_t*)(m + 16);
  int32_t* d_status = (int32_t*)(m + 20);
  uint32_t hv[2] = {(uint32_t)n, size};
  HT_DECL
  size_t hdr = 0;
  (void)sm_parse32((const uint8_t*)compressed, n, 0, &size, &hdr);
  // path 5: literal tags only (an incompressible input) -- one copy kernel from the pinned input
  // staging to the pinned output staging, one synchronisation
  {
    sm::LitSpans ls;
    if (ctx->small && size <= kPinnedOutMax && n <= kPinnedInMax && literal_only((const uint8_t*)compressed, n, hdr, size, ls)) {
      const int r = literal_uncompress(ctx, (const uint8_t*)compressed, n, size, ls, (uint8_t*)uncompressed);
      if (r < 0) return SM_ERR_DEVICE;
      if (r == 1) {
        ctx->last_path = 5;
        *uncompressed_length = size;
        return SM_OK;
      }
    }
  }
  // a large stream: fragments in parallel when it is block-structured (Snappy.jl, libsnappy
  // and this library all write such streams); otherwise, or on any error, the in-order decode
  // (a body longer than its output is all literals, which the in-order engine copies HBM to HBM at
  // bandwidth: path 0 is faster there -- fireworks.jpeg 59 us against ~100; a body just under
  // its output is random data with short copies sprinkled in, which path 0 walks in small batches
  // of one wave: alice29.snappy's fast stream 573 us there, 114 us in path 4, so path 4 takes
  // everything up to body == output; round 4's bound was 7/8)
  if (ctx->small && size >= kSmallMinOutput && size <= kSmallMaxOutput && n > hdr &&
      (uint64_t)(n - hdr) * 8 <= (uint64_t)size * SM_SMALL_BODY8 &&
      (n - hdr + sm::kSmallChunk - 1) / sm::kSmallChunk <= kSmallMaxChunks) {
    const int r = small_uncompress(ctx, (const uint8_t*)compressed, (uint32_t)n, (uint32_t)hdr, size,
                                   (uint8_t*)uncompressed);
    if (r < 0) return SM_ERR_DEVICE;
    if (r == 4) {
      ctx->last_path = 4;
      *uncompressed_length = size;
      return SM_OK;
    }
  }
  // (path 4 uploads through its index launch; every other path from here)
  SM_CHECK(upload_input(ctx, compressed, n, s));
  HT("uncompress: H2D input")
  if (size >= kParallelMinOutput && n - hdr >= 2 * sm::kIdxChunk) {
    bool copied = false;
    int32_t err = SM_OK;
    const int r = parallel_uncompress(ctx, (const uint8_t*)compressed, (uint32_t)n, (uint32_t)hdr, size,
                                      (uint8_t*)uncompressed, &copied, &err);
    if (r < 0) return SM_ERR_DEVICE;
    if (r == 3) {  // the stream's first error, found in parallel (the reference throws: no output)
      ctx->last_path = 3;
      return err;
    }
    if (r >= 1) {
      ctx->last_path = r;
      if (!copied) {
        SM_CHECK(hipMemcpyAsync(uncompressed, ctx->out.p, size, hipMemcpyDeviceToHost, s));
        SM_CHECK(hipStreamSynchronize(s));
      }
      HT("uncompress: D2H output")
      *uncompressed_length = size;
      return SM_OK;
    }
  }
  ctx->last_path = 0;
  sm::DecompressArgs a{(const uint8_t*)ctx->in.p, d_off, d_in_len, (uint8_t*)ctx->out.p, d_off, d_cap, d_out_len,
                       d_status, 1};
  a.one_n = hv[0];  // (n >= 1 here: the header parsed) -- the stream's length and capacity as arguments
  a.one_cap = hv[1];
  SM_CHECK(sm::launch_decompress(a, size > SM_BLOCK_SIZE, s));
  // the output (whatever the status) and (out_len, status) into the pinned staging by a kernel
  const size_t w_off = align_up(size, 256);
  if (size <= kPinnedOutMax && ctx->stage.ensure(w_off + 64) == hipSuccess && ctx->stage.dp) {
    uint8_t* const sdp = (uint8_t*)ctx->stage.dp;
    SM_CHECK(sm::launch_to_host((const uint8_t*)ctx->out.p, size, sdp, d_out_len, 2, (uint32_t*)(sdp + w_off), s));
    SM_CHECK(hipStreamSynchronize(s));
    const volatile uint32_t* w = (const volatile uint32_t*)((uint8_t*)ctx->stage.p + w_off);
    const uint32_t dlen = w[0];
    const int32_t dst = (int32_t)w[1];
    if (dst != SM_OK) return dst;
    if (dlen > size) return SM_ERR_DEVICE;  // (never: the kernel's bound)
    if (dlen) memcpy(uncompressed, ctx->stage.p, dlen);  // (uncompressed may be NULL when dlen == 0)
    *uncompressed_length = dlen;
    return SM_OK;
  }
  int32_t dst = 0;
  uint32_t dlen = 0;
  SM_CHECK(hipMemcpyAsync(&dst, d_status, 4, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipMemcpyAsync(&dlen, d_out_len, 4, hipMemcpyDeviceToHost, s));
  SM_CHECK(hipStreamSynchronize(s));
  if (dst != SM_OK) return dst;
  if (dlen) {
    SM_CHECK(hipMemcpyAsync(uncompressed, ctx->out.p, dlen, hipMemcpyDeviceToHost, s));
    SM_CHECK(hipStreamSynchronize(s));
  }
  *uncompressed_length = dlen;
  return SM_OK;
}

sm_status sm_uncompress_fragments_device(sm_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off,
                                         const uint32_t* d_in_len, uint32_t nblk, uint8_t* d_out,
                                         const uint64_t* d_out_off, const uint32_t* d_frag_len, uint32_t* d_out_len,
                                         int32_t* d_status, void* stream) {
  if (!ctx) return SM_ERR_ARGUMENT;
  if (nblk == 0) return SM_OK;
  if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_frag_len || !d_out_len || !d_status)
    return SM_ERR_ARGUMENT;
  DeviceGuard g(ctx->device);
  sm::DecompressArgs a{d_in, d_in_off, d_in_len, d_out, d_out_off, d_frag_len, d_out_len, d_status, nblk, 1};
  SM_CHECK(sm::launch_decompress(a, 0, (hipStream_t)stream));
  return SM_OK;
}

// ---- snappy-c.h-shaped entry points on a process-wide default context --------------------
// The exact ccall shape of the reference's libsnappy helper (test/libsnappy.jl:5-30):
// (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}) -> Cint, so a binding rebinds by symbol name
// alone.  The default context lives on device SNAPPY_MI355X_DEVICE (default 0); its mutex
// serialises callers.

namespace {
std::mutex g_default_mu;
sm_ctx* g_default_ctx = nullptr;
// Dense by default: a drop-in caller gets stream sizes within 1.01x of Snappy.jl's on every
// corpus file, and a single call's fixed costs (PCIe, launches) hide dense's extra kernel time.
std::atomic<int> g_default_mode{SM_MODE_FAST_DENSE};  // set and read from any thread

sm_ctx* default_ctx() {
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (!g_default_ctx) {
    const char* e = getenv("SNAPPY_MI355X_DEVICE");
    g_default_ctx = sm_ctx_create(e ? atoi(e) : 0);
  }
  return g_default_ctx;
}
}  // namespace

namespace {
// snappy-c.h knows three statuses: 0 OK, 1 INVALID_INPUT, 2 BUFFER_TOO_SMALL.  The detailed codes
// (the reference's messages 16-21, device and argument failures) stay on the ctx API.
sm_status snappy_c_status(sm_status st) {
  return st == SM_OK ? SM_OK : (st == SM_BUFFER_TOO_SMALL ? SM_BUFFER_TOO_SMALL : SM_INVALID_INPUT);
}
}  // namespace

sm_status sm_snappy_set_mode(int mode) {
  if (!valid_mode(mode)) return SM_ERR_ARGUMENT;
  g_default_mode.store(mode, std::memory_order_relaxed);
  return SM_OK;
}

sm_status sm_snappy_compress(const char* input, size_t input_length, char* compressed, size_t* compressed_length) {
  sm_ctx* ctx = default_ctx();
  if (!ctx) return SM_INVALID_INPUT;
  return snappy_c_status(sm_compress(ctx, input, input_length, compressed, compressed_length,
                                     g_default_mode.load(std::memory_order_relaxed)));
}

sm_status sm_snappy_uncompress(const char* compressed, size_t compressed_length, char* uncompressed,
                               size_t* uncompressed_length) {
  sm_ctx* ctx = default_ctx();
  if (!ctx) return SM_INVALID_INPUT;
  return snappy_c_status(sm_uncompress(ctx, compressed, compressed_length, uncompressed, uncompressed_length));
}

size_t sm_snappy_max_compressed_length(size_t source_length) { return sm_max_compressed_length(source_length); }

sm_status sm_snappy_uncompressed_length(const char* compressed, size_t compressed_length, size_t* result) {
  return snappy_c_status(sm_uncompressed_length(compressed, compressed_length, result));
}

sm_status sm_snappy_validate_compressed_buffer(const char* compressed, size_t compressed_length) {
  sm_ctx* ctx = default_ctx();
  if (!ctx) return SM_INVALID_INPUT;
  return snappy_c_status(sm_validate_compressed_buffer(ctx, compressed, compressed_length));
}

}  // extern "C"
