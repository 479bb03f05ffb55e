// sm_decompress.hip -- batched snappy decompression for gfx950 (MI355X).
//
// One wavefront per compressed stream.  Accept/reject semantics are Snappy.jl's
// (src/internal.jl:411-527, src/Snappy.jl:46-52), including its leniencies:
//   * `while ip < endof(input)` (internal.jl:416): a tag on the last byte is never parsed;
//   * the 4-byte lookahead is zero-padded past the end (internal.jl:426-430);
//   * literal length is len + trailer in UInt32 arithmetic (wraps);
//   * copy offset check `op-1 <= offset-1` with unsigned wrap (internal.jl:499);
//   * the copy-length check is skipped on the 2x8-byte fast path (internal.jl:500-505).
// The first error in stream order wins, as the reference throws at the first one.
//
// Batched tag engine (declared length <= 64 KiB -- every block the compressor produces):
//  * the compressed stream flows through a 1 KiB LDS ring (4 x 256-B slots + mirror), one
//    slot prefetched into registers a batch ahead;
//  * every lane computes, for its 4 positions of the current slot, the size a tag starting
//    there would have (packed u8, 255 = literal too long for a batch); a pointer-doubling walk
//    gives lane t the t-th tag directly;
//  * up to 64 tags per batch decode one per lane, output offsets from a wave scan, the
//    reference's error checks per tag -- the lowest failing lane decides the status;
//  * tags execute lane-parallel in 16-byte pieces into a linear LDS output window (sources in
//    the window or, older, in HBM), the few copies whose source overlaps the batch's own
//    output (or offset < 16) in stream order after them; whole 16-byte blocks go to HBM when
//    a batch ends.
// Literals longer than 64 bytes are copied by the whole wave.
// Streams declaring > 64 KiB use a simple per-tag engine (also straight into HBM).
#include "sm_device.h"
#include "sm_internal.h"




namespace sm {


typedef uint16_t __attribute__((aligned(1))) du16u;
typedef uint32_t __attribute__((aligned(1))) du32u;
typedef uint64_t __attribute__((aligned(1))) du64u;

constexpr uint32_t kRing = 1024;
constexpr uint32_t kRingMirror = 96;  // the ring's first bytes again past its end: a literal's
                                      // 16-byte pieces (<= 64 B) read at ring offset + 48 + 20
constexpr uint32_t kMaxBatchLit = 200;  // longer literals stop a window walk (size 255)
constexpr int kWalkLevels = 5;  // tables J0..J4 in LDS; J5 (bit 5 of a lane's chain index) = J4 o J4
constexpr int kJtRow = 256;             // a jump-table row (u8): positions 0..254, 255 = beyond the window
constexpr int kJt = kWalkLevels * kJtRow / 2;  // u16 words of a walk's jump tables (1.25 KB)
__device__ inline uint32_t load_word(const uint8_t* __restrict__ in, uint32_t N, uint32_t p) {
  if (p + 3 < N && (((uintptr_t)(in + p)) & 3) == 0) return *reinterpret_cast<const uint32_t*>(in + p);
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v |= (p + k < N ? (uint32_t)in[p + k] : 0u) << (8 * k);
  return v;
}

// ---------------------------------------------------------------------------------------
// batched tag engine

// Speculative size of a tag starting at a window position (u8; 255 = a literal the batch walk
// leaves to the general path, which decodes any tag): a copy 1 + taglen; a literal without
// length bytes (hi < 60) 1 + len; one length byte b (tag byte 0xf0) 2 + (b + 1) when that
// literal is <= kMaxBatchLit bytes, else 255; two to four length bytes (hi >= 61: longer than
// 256 bytes in a minimal encoding) always 255.  In SWAR: copy sizes by a v_perm_b32 byte
// lookup on the kind bits, short literals as hi + 2 per byte; a word holding a literal tag byte
// with length bytes (63% of the text windows: a copy's offset byte 0xf0/f4/f8/fc somewhere in
// the 256 bytes) fixes those bytes in SWAR too (no per-byte path).  tools/check_tag_sizes.c
// restates the per-byte definition and checks this form against it (tests/test_host_logic.py).
__device__ inline uint32_t pack_sizes(uint32_t cur, uint32_t nxt) {
  const uint32_t K = cur & 0x03030303u, H = (cur >> 2) & 0x3f3f3f3fu;
  const uint32_t csz = __builtin_amdgcn_perm(0u, 0x05030200u, K);       // kind 1/2/3 -> 2/3/5
  const uint32_t ml = __builtin_amdgcn_perm(0u, 0x000000ffu, K);        // 0xff per literal byte (kind 0)
  uint32_t sz = (csz & ~ml) | ((H + 0x02020202u) & ml);
  const uint32_t h60 = (H + 0x44444444u) & 0x80808080u & ml;           // 0x80: a literal with length bytes
  if (h60) {
    const uint32_t hm = h60 | (h60 - (h60 >> 7));                       // 0xff there
    const uint32_t b = __builtin_amdgcn_alignbyte(nxt, cur, 1);         // the byte after each position
    const uint32_t e = cur ^ 0xf0f0f0f0u;                               // 0 at a one-length-byte tag
    const uint32_t ne = (((e & 0x7f7f7f7fu) + 0x7f7f7f7fu) | e) & 0x80808080u;  // 0x80: not 0xf0
    const uint32_t bb = (((b >> 1) & 0x7f7f7f7fu) + 0x1c1c1c1cu) & 0x80808080u;  // 0x80: b >= 200
    const uint32_t st = ne | bb;                                        // 0x80: size 255
    const uint32_t sm = st | (st - (st >> 7));
    const uint32_t v = (b | sm) + (0x03030303u & ~sm);                  // b + 3 (<= 202) or 0xff: no carry
    sz = (sz & ~hm) | (v & hm);
  }
  return sz;
}

// the literals the batch walk stops at (size 255 above), for a scalar walk's step over them
__device__ inline bool walk_stop_literal(uint32_t c, uint64_t lit) {
  return (c & 3) == 0 && ((c >> 2) >= 61 || lit > kMaxBatchLit);
}

// ring slot write: stream bytes [base, base+256) (word per lane) at ring[(base & 1023)]
__device__ inline void ring_put(uint8_t* ring, uint32_t base, uint32_t word, uint32_t lane) {
  uint32_t r = base & (kRing - 1);
  reinterpret_cast<uint32_t*>(ring + r)[lane] = word;
  if (r == 0 && lane < kRingMirror / 4) reinterpret_cast<uint32_t*>(ring + kRing)[lane] = word;  // mirror
}

// 8 stream bytes at pos (aligned dword reads: the mirror covers the 12 bytes past kRing)
__device__ inline uint64_t ring_get8(const uint8_t* ring, uint32_t pos) { return lds_ld64(ring, pos & (kRing - 1)); }

// ring refill at wb: slots [wb, wb+768) and the two prefetch words, all five loads in flight
__device__ inline void ring_fill(const uint8_t* __restrict__ in, uint32_t N, uint32_t wb, uint8_t* ring, uint32_t& pre1,
                                 uint32_t& pre2, uint32_t lane) {
  uint32_t w[5];
  if ((((uintptr_t)(in + wb)) & 3) == 0 && wb + 1280 <= N) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(in + wb) + lane;
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = s[64 * i];
  } else {
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = load_word(in, N, wb + 256 * i + 4 * lane);
  }
  ring_put(ring, wb, w[0], lane);
  ring_put(ring, wb + 256, w[1], lane);
  ring_put(ring, wb + 512, w[2], lane);
  pre1 = w[3];
  pre2 = w[4];
}

// ---- LDS output window --------------------------------------------------------------------
// The recent output of the stream lives in a per-wave linear LDS window besides going to HBM:
// output position x at byte x - wbase (wbase a multiple of 16).  Every byte at or past the
// current output position op is zero when a batch starts, so tags write by or-ing whole 16-byte
// pieces (five aligned ds_or_b32, the bytes past the tag trimmed to 0) with no read-modify-write
// races between lanes.  When a batch would write past the window's end, the last kKeep+ bytes
// move to its start and the rest is zeroed (win_shift: a few 16-byte LDS ops per lane every
// couple of batches), so a copy source at distance <= op - wbase (>= kKeep right after a shift,
// growing until the next) is in LDS; older sources are read from HBM, which holds every byte
// before the window (only the last partial 16-byte block of a batch waits for the next flush,
// and it is inside the window).  No position ever wraps: reads and writes are plain offsets.
#ifndef SM_DEC_WIN
#define SM_DEC_WIN 2560
#endif
constexpr uint32_t kWin = SM_DEC_WIN;  // window bytes (a multiple of 16)
#ifndef SM_DEC_BOUT
#define SM_DEC_BOUT 512
#endif
constexpr uint32_t kBatchOut = SM_DEC_BOUT;  // most output bytes of one batch
#ifndef SM_DEC_KEEP
#define SM_DEC_KEEP 480
#endif
constexpr uint32_t kKeep = SM_DEC_KEEP;  // bytes a shift keeps (the least LDS source reach)
constexpr uint32_t kWinPad = 16;         // bytes before the window (the dword below a piece)
static_assert(kKeep + 15 + kBatchOut + 32 <= kWin && kKeep >= 80 && kWin % 16 == 0, "window bounds");
static_assert(kKeep + 15 <= 16 * kWave, "win_shift moves at most one 16-byte unit per lane");

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// 16 bytes at LDS byte address a + k (k a compile-time multiple of 4): five aligned dword reads,
// four funnel shifts (v_alignbyte_b32 reads only the low 2 bits of the shift operand)
__device__ inline uint4 lds_get16(uint32_t a, uint32_t k) {
  const lds_u32* w = (const lds_u32*)(size_t)((a & ~3u) + k);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, a), __builtin_amdgcn_alignbyte(w2, w1, a),
                    __builtin_amdgcn_alignbyte(w3, w2, a), __builtin_amdgcn_alignbyte(w4, w3, a));
}

// v with the bytes from len (1..16) on cleared: two 64-bit right shifts of all-ones (amounts in
// 0..56 for len >= 1) and a select for the high half
__device__ inline uint4 trim16(uint4 v, uint32_t len) {
  uint32_t l8 = len << 3;
  asm("" : "+v"(l8));  // (else 128 - 8 len folds into a quarter-rate multiply)
  uint64_t mlo, mhi;   // (v_lshrrev_b64 of the inline constant -1: two shifts, not four)
  asm("v_lshrrev_b64 %0, %1, -1" : "=v"(mlo) : "v"(64 - min(l8, 64u)));
  asm("v_lshrrev_b64 %0, %1, -1" : "=v"(mhi) : "v"(128 - l8));
  const bool hi = len > 8;
  return make_uint4(v.x & (uint32_t)mlo, v.y & (uint32_t)(mlo >> 32), hi ? v.z & (uint32_t)mhi : 0u,
                    hi ? v.w & (uint32_t)(mhi >> 32) : 0u);
}

// or the 16 bytes v (zero past the piece) into the zeroed window at LDS byte address a + k (k a
// compile-time multiple of 4): the five dwords from (a - 1) & ~3 with t = -a, alignbyte(hi, lo,
// t) = (hi:lo) >> 8 (t & 3) -- an aligned a shifts the piece one dword up and ors a zero below
// it (the window's front pad), no selects
__device__ inline void lds_or16(uint32_t a, uint32_t k, uint4 v) {
  const uint32_t wa = ((a - 1u) & ~3u) + k, t = 0u - a;
  const uint32_t u0 = __builtin_amdgcn_alignbyte(v.x, 0u, t);
  const uint32_t u1 = __builtin_amdgcn_alignbyte(v.y, v.x, t);
  const uint32_t u2 = __builtin_amdgcn_alignbyte(v.z, v.y, t);
  const uint32_t u3 = __builtin_amdgcn_alignbyte(v.w, v.z, t);
  const uint32_t u4 = __builtin_amdgcn_alignbyte(0u, v.w, t);
  asm volatile("ds_or_b32 %0, %1\nds_or_b32 %0, %2 offset:4\nds_or_b32 %0, %3 offset:8\nds_or_b32 %0, %4 offset:12\n"
               "ds_or_b32 %0, %5 offset:16"
               : : "v"(wa), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(u4) : "memory");
}

// the window's first byte at output position wbase = op0 & ~15, all of it zero
__device__ inline void win_init(uint8_t* win, uint32_t lane) {
  for (uint32_t u = lane; u < kWin / 16; u += kWave) reinterpret_cast<uint4*>(win)[u] = make_uint4(0, 0, 0, 0);
}

// move the window so that it starts at nb = (op - kKeep) & ~15: bytes [nb, op) (rounded up to a
// 16-byte unit -- the bytes past op are zero) to its start, zeros after
__device__ inline void win_shift(uint8_t* win, uint32_t& wbase, uint32_t op, uint32_t lane) {
  const uint32_t nb = (op - kKeep) & ~15u;
  const uint32_t d = nb - wbase, n = (op - nb + 15) >> 4;
  uint4* w = reinterpret_cast<uint4*>(win);
  uint4 v = make_uint4(0, 0, 0, 0);
  if (lane < n) v = w[(d >> 4) + lane];  // (every read is issued before the first write)
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  for (uint32_t u = lane; u < kWin / 16; u += kWave) w[u] = u < n ? v : make_uint4(0, 0, 0, 0);
  wbase = nb;
}

// HBM gets the window bytes of output positions [from, to): head bytes up to a 16-byte
// position boundary, 16-byte blocks, tail bytes
__device__ inline void win_flush(uint8_t* out, const uint8_t* win, uint32_t wbase, uint32_t from, uint32_t to,
                                 uint32_t lane) {
  if (to <= from) return;
  const uint32_t h = min((16u - (from & 15u)) & 15u, to - from);
  if (lane < h) out[from + lane] = win[from + lane - wbase];
  from += h;
  const uint32_t nb = (to - from) >> 4;
  for (uint32_t k = lane; k < nb; k += kWave) {
    const uint32_t x = from + 16 * k;
    const uint4 v = *reinterpret_cast<const uint4*>(win + (x - wbase));
    *reinterpret_cast<du64u*>(out + x) = ((uint64_t)v.y << 32) | v.x;
    *reinterpret_cast<du64u*>(out + x + 8) = ((uint64_t)v.w << 32) | v.z;
  }
  from += nb << 4;
  if (lane < to - from) out[from + lane] = win[from + lane - wbase];
}

// Tag walk over a 255-byte window by pointer doubling (VALU + LDS, no serial loop).
// cw = the 8 stream bytes at window position 4*lane; rlim = the parse limit relative to the
// window (window end or N-1, internal.jl:416), clamped to 255.  Every lane computes the
// speculative sizes of its 4 positions (packed u8 in `sizes`, 255 = a literal too long for a
// batch).  J0[p] = p + size(p), clamped to 255 (beyond the window: position 255 is never a tag
// of this window, and its entry maps to itself, so no read is conditional); a long literal is a
// stop node (J0[p] = p).  Positions at or after rlim need no stops: a chain's positions increase,
// so the tags before rlim are a prefix of lanes and the final count drops the rest.
// J_k = J_{k-1} o J_{k-1}, k < 5, in LDS as u8 rows (positions are bytes: a read's address is the
// row base plus the value, and five rows take 1.25 KB), J5 = J4 o J4 applied as two J4 reads:
// 64 tags = chain elements 0..63.  Lane t then holds tag t directly -- J_k applied for every set
// bit k of t -- with its window position cpos and size csz; stop nodes are fixed points, so the
// tags are a prefix of lanes.  Returns their count.
__device__ inline uint32_t walk_window(uint64_t cw, uint32_t rlim, uint16_t* jt16, uint32_t lane, uint32_t& cpos,
                                       uint32_t& csz, uint32_t& sizes) {
  uint8_t* const jt = reinterpret_cast<uint8_t*>(jt16);
  rlim = min(rlim, 255u);
  sizes = pack_sizes((uint32_t)cw, (uint32_t)(cw >> 32));
  auto rd = [&](int k, uint32_t x) -> uint32_t { return jt[k * kJtRow + x]; };
  auto row = [&](int k, const uint32_t (&J)[4]) {
    *reinterpret_cast<uint32_t*>(jt + k * kJtRow + 4 * lane) = J[0] | (J[1] << 8) | (J[2] << 16) | (J[3] << 24);
  };
  uint32_t J[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t p = 4 * lane + j;
    const uint32_t sz = (sizes >> (8 * j)) & 0xff;
    J[j] = sz == 255 ? p : min(p + sz, 255u);  // 255: beyond the window
  }
  row(0, J);
  // The J_k are powers of J0, so they commute: lane t applies J_k for bit k of t as soon as row k
  // is built, its read issued with the next row's reads (the chain does not wait for every row)
  uint32_t c = 0;
#pragma unroll
  for (int k = 1; k < kWalkLevels; ++k) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint32_t t = rd(k - 1, c);
#pragma unroll
    for (int j = 0; j < 4; ++j) J[j] = rd(k - 1, J[j]);
    c = ((lane >> (k - 1)) & 1u) ? t : c;
    row(k, J);
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the u8 reads below follow the row stores
  {
    const uint32_t t = rd(kWalkLevels - 1, c);
    c = ((lane >> (kWalkLevels - 1)) & 1u) ? t : c;
  }
  if (lane >= 32) {  // J5 = J4 o J4
    c = rd(kWalkLevels - 1, c);
    c = rd(kWalkLevels - 1, c);
  }
  // (the shuffle runs with every lane active: a ds_bpermute from an inactive lane reads 0)
  const uint32_t szw = __shfl(sizes, (c >> 2) & 63u, 64);
  const uint32_t sz = (szw >> (8 * (c & 3))) & 0xffu;
  cpos = c;
  csz = sz;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the next walk's stores follow these reads
  return (uint32_t)__builtin_popcountll(ballot(c < rlim && sz != 255));
}

// Decodes the tags that start in [ip, ip_end) -- ip_end = N for a whole stream, whose loop
// stops at N-1 (internal.jl:416) -- into out[op0, ...).  Copy sources below frag_lo are
// refused with kErrCross: a fragment of a block-structured stream must not read output that
// other waves produce (the caller then decodes the whole stream in order instead).  Error
// checks use stream-global positions, so they are the reference's whatever the range.
// kLit: 16-byte loads per lane in flight in a long literal's bulk copy (4 in the batch kernels,
// whose VGPR budget sets their occupancy; 16 in the lone-stream kernel, where one wave's copy is
// latency-bound)
template <uint32_t kLit = 4>
__device__ int32_t decode_stream_batch(const uint8_t* __restrict__ in, uint32_t N, uint32_t ip, uint32_t ip_end,
                                       uint32_t size, uint8_t* out, uint32_t op0, uint32_t frag_lo, uint8_t* ring,
                                       uint16_t* jt, uint8_t* win, uint32_t lane, uint32_t& op_end,
                                       uint32_t op_lim = 0xffffffffu) {
  // ring holds stream bytes [wb, wb+768); pre1 = [wb+768, wb+1024) (loaded a batch ago),
  // pre2 = [wb+1024, wb+1280) issued at the end of the previous batch -- so a round's fence
  // (s_waitcnt vmcnt(0)) never waits for a freshly issued prefetch.
  uint32_t wb = ip & ~255u;
  uint32_t pre1, pre2;
  ring_fill(in, N, wb, ring, pre1, pre2, lane);
  bool issue_pre2 = false;
  uint32_t op = op0, flushed = op0;  // output produced / already in HBM
  const uint32_t wlo = op0 & ~15u;   // (the window never starts below the first output block)
  uint32_t wbase = wlo;              // output position of the window's first byte
  win_init(win, lane);
  const uint32_t winA = lds_addr(win), ringA = lds_addr(ring);
  const bool in_al = (((uintptr_t)in) & 3) == 0;
  const int64_t Nm1 = min((int64_t)N - 1, (int64_t)ip_end);  // parse limit

  // every batch consumes input (ip strictly increases): more than N batches means the wave is
  // not whole (a caller that split it) -- a status, never a hang
  uint32_t guard = N + 1;
  while ((int64_t)ip < Nm1 && op < op_lim) {
    if (__builtin_expect(--guard == 0, 0)) return kErrDevice;
    if (ip >= wb + 256) {
      if (__builtin_expect(ip < wb + 512, 1)) {
        ring_put(ring, wb + 768, pre1, lane);
        pre1 = pre2;
        wb += 256;
        issue_pre2 = true;  // [wb+1024, wb+1280) loads after this batch
      } else {  // jumped (long literal): refill
        wb = ip & ~255u;
        ring_fill(in, N, wb, ring, pre1, pre2, lane);
        issue_pre2 = false;
      }
    }
    // the window [ip, ip+256) (inside the ring: ip < wb+256; a batch's literals end before
    // ip+256+200 < wb+768)
    const uint32_t wlim = (int64_t)(ip + 256) < Nm1 ? ip + 256 : (uint32_t)Nm1;
    uint32_t cpos, csz, sizes;
    const uint32_t ntok = walk_window(ring_get8(ring, ip + 4 * lane), wlim - ip, jt, lane, cpos, csz, sizes);
    uint32_t tpos = 0, ipw = ip, tnext = 0;
    bool big = false;
    if (__builtin_expect(ntok != 0, 1)) {
      tpos = ip + cpos;
      tnext = cpos + csz;
      ipw = ip + readlane(tnext, ntok - 1);
    }
    if (ipw < wlim) {
      const uint32_t rel = ipw - ip;
      big = ((readlane(sizes, rel >> 2) >> ((rel & 3) * 8)) & 0xff) == 255;
    }

    if (__builtin_expect(ntok != 0, 1)) {
      const bool mine = lane < ntok;
      // one tag per lane: its fields, output offset (wave scan) and the reference's checks as
      // selects (no exec branches), in the same first-failing order
      struct TagDec {
        uint32_t len, taglen, offset, litlen, osat, incl, opt, lsrc;
        bool iscopy;
        int32_t err;
      };
      auto tag_decode = [&](uint32_t tp) -> TagDec {
        TagDec d;
        const uint64_t hv = ring_get8(ring, mine ? tp : wb);
        const uint32_t c = (uint32_t)hv & 0xff;
        const uint32_t entry = char_entry(c);  // (a 512-byte table in global memory instead: 1.510 against 1.455 ms)
        d.len = entry & 0xff;
        d.taglen = entry >> 11;
        const uint32_t tr_raw = (uint32_t)(hv >> 8);
        // the low taglen bytes (0..4) of tr_raw: the low dword of ~0 << 8 taglen (64-bit: 0 for 4)
        // clears them in a mask, one v_bfi_b32 keeps them
        uint64_t hm;
        asm("v_lshlrev_b64 %0, %1, -1" : "=v"(hm) : "v"(8 * d.taglen));
        const uint32_t trailer = tr_raw & ~(uint32_t)hm;
        d.iscopy = (c & 3) != 0;
        d.offset = (entry & 0x700) + trailer;
        d.litlen = d.len + trailer;
        const uint32_t olen = d.iscopy ? d.len : d.litlen;
        d.osat = mine ? min(olen, 65537u) : 0u;
        d.incl = scan_dpp(d.osat);
        d.opt = op + d.incl - d.osat;
        d.lsrc = tp + 1 + d.taglen;
        const int64_t avail_out = (int64_t)size - (int64_t)d.opt;
        const int64_t avail_in = (int64_t)N - (int64_t)d.lsrc;
        const bool e_off = (int64_t)d.opt <= (int64_t)(uint32_t)(d.offset - 1u);                                // :499
        const bool e_cross = d.opt - d.offset < frag_lo;
        const bool e_len = !((d.len <= 16) & (d.offset >= 8) & (avail_out >= 16)) & (avail_out < (int64_t)d.len);  // :505
        const bool e_lit = (avail_out < (int64_t)d.litlen) | (avail_in < (int64_t)d.litlen);                     // :518
        const int32_t ec = e_off ? kErrCopyOffset : (e_cross ? kErrCross : (e_len ? kErrCopyLength : kOk));
        d.err = !mine ? kOk : (d.iscopy ? ec : (e_lit ? kErrLiteral : kOk));
        return d;
      };
      const TagDec d = tag_decode(tpos);
      const uint32_t len = d.len, offset = d.offset, litlen = d.litlen, incl = d.incl, opt = d.opt, lsrc = d.lsrc;
      const bool iscopy = d.iscopy;
      const int32_t err = d.err;
      const uint64_t em = ballot(err != kOk);
      if (__builtin_expect(em != 0, 0)) return (int32_t)readlane((uint32_t)err, ctz64(em));
      // cap the batch output at kBatchOut bytes (the window bound; one tag is <= 200 B) and at
      // the output limit (a fragment ends where the next one starts)
      uint32_t nt = ntok;
      if (__builtin_expect(readlane(incl, ntok - 1) > kBatchOut || readlane(opt, ntok - 1) >= op_lim, 0)) {
        nt = (uint32_t)__builtin_popcountll(ballot(mine && incl <= kBatchOut && opt < op_lim));
        ipw = ip + readlane(tnext, nt - 1);
        big = false;  // the next tag is a batch tag inside the window
      }
      const uint32_t X = readlane(incl, nt - 1);

      if (op - wbase + X + 32 > kWin) win_shift(win, wbase, op, lane);  // (uniform)
      const uint32_t O0 = op;
      const uint32_t slo = opt - offset;
      const uint32_t shi = slo + min(len, offset);
      // a source before the window comes from HBM, which holds it whole: the window starts at
      // least kKeep bytes before the output (after a shift or a big literal) or at the first
      // output block, a source ends at most 64 bytes after its start, and every byte before the
      // batch but the last partial 16-byte block is flushed
      // (lane sets as SGPR masks: a ballot of a compare is one v_cmp, and inverse_ballot turns a
      // mask back into a lane predicate for free -- a ballot of a combined bool costs two VALU)
      const uint64_t all = nt == 64 ? ~0ull : ((1ull << nt) - 1);
      const uint64_t copym = ballot(iscopy) & all;
      const uint64_t longm = ballot(litlen > 64) & ~copym & all;
      const uint64_t gm = ballot(slo < wbase) & copym;
      const bool gsrc = inverse_ballot(gm);
      uint64_t done = longm | ~all;
      // HBM sources: this wave's earlier flushes (and big literals) must have landed
      if (gm) __threadfence_block();

      // long literals (65..200 B, no dependencies, inside the input ring): whole-wave passes
      uint64_t lm = longm;
      while (lm) {
        const uint32_t t = ctz64(lm);
        lm &= lm - 1;
        const uint32_t o = readlane(opt, t), sr = readlane(lsrc, t), L = readlane(litlen, t);
        const uint32_t k = 16 * lane;
        if (k < L) lds_or16(winA + (o - wbase) + k, 0, trim16(lds_get16(ringA + ((sr + k) & (kRing - 1)), 0), min(16u, L - k)));
      }

      // One round (all in LDS, or HBM for sources before the window) runs every tag whose source
      // is final before the batch and whose bytes can be read straight: a literal (<= 64 B, from
      // the input ring) or a copy with offset >= 16 -- output byte j is S[j mod offset]
      // (incremental_copy_slow!, internal.jl:477-481), which for j >= offset is the copy's own
      // output byte j - offset = out[slo + j], written by an earlier 16-byte pass.  So every tag
      // reads out[slo + j] (or its literal bytes) in 16-byte pieces.  The writes never touch
      // bytes another ready tag reads.
      if (__builtin_expect(done != ~0ull, 1)) {
        const uint64_t rm = ~done & (~copym | (ballot(shi <= O0) & ballot(offset >= 16)));
        const uint32_t L = iscopy ? len : litlen;
        const uint32_t sa = iscopy ? winA + (slo - wbase) : ringA + (lsrc & (kRing - 1));
        const uint32_t da = winA + (opt - wbase);
        const uint8_t* gs = out + slo;
#pragma unroll
        for (uint32_t base = 0; base < 64; base += 16) {
          const uint64_t am = rm & ballot(L > base);
          if (!am) break;
          if (inverse_ballot(am)) {
            uint4 v;
            if (gsrc) {
              const du64u* g = reinterpret_cast<const du64u*>(gs + base);
              const uint64_t a = g[0], b = g[1];
              v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
            } else {
              v = lds_get16(sa, base);
            }
            lds_or16(da, base, trim16(v, min(L - base, 16u)));
          }
        }
        done |= rm;
      }
      // The copies left -- their source overlaps earlier tags of this batch, or offset < 16 --
      // run in stream order, one tag at a time, a byte per lane: byte k = S[k mod offset] with S
      // final by then (LDS accesses of a wave are serviced in order).
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      uint64_t rest = ~done;
      while (rest) {
        const uint32_t t = ctz64(rest);
        rest &= rest - 1;
        const uint32_t o = readlane(opt, t), sl = readlane(slo, t), L = readlane(len, t), off = readlane(offset, t);
        if (lane < L) {
          uint32_t k = lane;
          if (k >= off) {  // k mod off for k, off <= 64: exact through the f32 reciprocal
            const uint32_t q = (uint32_t)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)off));
            k -= q * off;
          }
          win[o + lane - wbase] = win[sl + k - wbase];
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
      }
      op += X;
      if (__builtin_expect(op > op_lim, 0)) return kErrCross;  // a tag crosses the fragment end
      win_flush(out, win, wbase, flushed, op & ~15u, lane);  // whole 16-byte blocks to HBM
      flushed = max(flushed, op & ~15u);
      ip = ipw;
    }
    if (issue_pre2) {
      // (a whole slot inside the stream at a 4-aligned base: one plain load, the test uniform)
      pre2 = (in_al && wb + 1280 <= N) ? reinterpret_cast<const uint32_t*>(in + wb + 1024)[lane]
                                       : load_word(in, N, wb + 1024 + 4 * lane);
      issue_pre2 = false;
    }

    if (__builtin_expect(big && op < op_lim, 0)) {  // (at op_lim the literal opens the next fragment)
      // one literal too long for the batch path (or a wrapped length): straight to HBM
      const uint64_t hv = ring_get8(ring, ip);
      const uint32_t c = uniform((uint32_t)hv & 0xff);
      const uint32_t entry = char_entry(c);
      const uint32_t taglen = entry >> 11;
      const uint32_t tr_raw = uniform((uint32_t)(hv >> 8));
      const uint32_t trailer = taglen >= 4 ? tr_raw : (tr_raw & ((1u << (8 * taglen)) - 1u));
      const uint32_t litlen = (entry & 0xff) + trailer;
      const uint32_t lsrc = ip + 1 + taglen;
      const int64_t avail_out = (int64_t)size - (int64_t)op;
      const int64_t avail_in = (int64_t)N - (int64_t)lsrc;
      if (avail_out < (int64_t)litlen || avail_in < (int64_t)litlen) return kErrLiteral;  // :518
      if ((uint64_t)op + litlen > op_lim) return kErrCross;
      if (litlen <= kMaxBatchLit) {
        // a short literal with 2-4 length bytes (a non-minimal encoding, or a wrapped length): its
        // bytes are in the ring (the tag is in the batch window, ip < wb + 512, so lsrc + litlen <
        // wb + 717 < wb + 768), so the whole wave ors them into the window as the batch round does
        // its long literals, then flushes whole 16-byte blocks as a batch does -- no full flush and
        // window reload from HBM per such tag.  (Every byte before op & ~15 is in
        // HBM here, as after a batch: a shift drops only flushed bytes.)
        if (op - wbase + litlen + 32 > kWin) win_shift(win, wbase, op, lane);  // (uniform)
        const uint32_t k = 16 * lane;
        if (k < litlen)
          lds_or16(winA + (op - wbase) + k, 0, trim16(lds_get16(ringA + ((lsrc + k) & (kRing - 1)), 0), min(16u, litlen - k)));
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        op += litlen;
        win_flush(out, win, wbase, flushed, op & ~15u, lane);
        flushed = max(flushed, op & ~15u);
        ip = lsrc + litlen;
        continue;
      }
      win_flush(out, win, wbase, flushed, op, lane);  // HBM holds everything before the literal
      // bulk copy: head bytes to 16-B source alignment, then 16 B per lane, kLit in flight
      const uint8_t* s = in + lsrc;
      uint32_t head = (uint32_t)((16 - ((uintptr_t)s & 15)) & 15);
      if (head > litlen) head = litlen;
      if (lane < head) out[op + lane] = s[lane];
      const uint4* s16 = reinterpret_cast<const uint4*>(s + head);
      const uint32_t n16 = (litlen - head) >> 4;
      uint8_t* d = out + op + head;
      uint32_t k = lane;
      for (; k + (kLit - 1) * kWave < n16; k += kLit * kWave) {
        uint4 v[kLit];
#pragma unroll
        for (uint32_t j = 0; j < kLit; ++j) v[j] = s16[k + j * kWave];
#pragma unroll
        for (uint32_t j = 0; j < kLit; ++j) {
          *reinterpret_cast<du64u*>(d + 16 * (k + j * kWave)) = ((uint64_t)v[j].y << 32) | v[j].x;
          *reinterpret_cast<du64u*>(d + 16 * (k + j * kWave) + 8) = ((uint64_t)v[j].w << 32) | v[j].z;
        }
      }
      for (; k < n16; k += kWave) {
        uint4 v0 = s16[k];
        *reinterpret_cast<du64u*>(d + 16 * k) = ((uint64_t)v0.y << 32) | v0.x;
        *reinterpret_cast<du64u*>(d + 16 * k + 8) = ((uint64_t)v0.w << 32) | v0.z;
      }
      const uint32_t done16 = head + (n16 << 4);
      if (lane < litlen - done16) out[op + done16 + lane] = s[done16 + lane];
      // the window restarts at nb = the 16-byte output boundary at or below op + litlen - kKeep
      // (not below the decode's first output block), filled from HBM -- which now holds all
      // output before op + litlen -- with zeros past op + litlen (any literal length, a wrapped
      // 0 included); older sources come from HBM
      const uint32_t opn = op + litlen;
      const uint32_t nb = (opn - min(opn - wlo, kKeep)) & ~15u;
      const uint32_t nk = opn - nb;
      __threadfence_block();  // (this wave's stores above land before the loads below)
      const uint8_t* q = out + nb;
      for (uint32_t u = lane; u < kWin / 16; u += kWave) {
        const uint32_t x = 16 * u;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (x + 16 <= nk) {
          const du64u* g = reinterpret_cast<const du64u*>(q + x);
          const uint64_t a = g[0], b = g[1];
          v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
        } else if (x < nk) {  // the last bytes: never read past the output
          uint64_t lo = 0, hi = 0;
          for (uint32_t i = 0; i < nk - x; ++i) {
            const uint64_t bt = (uint64_t)q[x + i] << (8 * (i & 7));
            if (i < 8) lo |= bt;
            else hi |= bt;
          }
          v = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        }
        reinterpret_cast<uint4*>(win)[u] = v;
      }
      wbase = nb;
      op += litlen;
      flushed = op;
      ip = lsrc + litlen;
    }
  }
  win_flush(out, win, wbase, flushed, op, lane);
  op_end = op;
  return kOk;
}

// varint32 stream header (varint.jl:12-37): size and the first tag's position; kErrVarint on
// more than 5 bytes, a 5th byte >= 0x10 or a truncated header
__device__ inline int32_t parse_header(const uint8_t* in, uint32_t N, uint32_t lane, uint32_t& size, uint32_t& ip) {
  const uint32_t hb = (lane < 5 && lane < N) ? in[lane] : 0;
  int32_t st = kErrVarint;
  size = 0;
  ip = 0;
  for (uint32_t i = 0; i < 5; ++i) {
    if (i >= N) break;
    const uint32_t bt = readlane(hb, i);
    if (i < 4) {
      size |= (bt & 0x7f) << (7 * i);
      if (bt < 0x80) {
        st = kOk;
        ip = i + 1;
        break;
      }
    } else {
      size |= (bt & 0x7f) << 28;
      if (bt < 0x10) {
        st = kOk;
        ip = 5;
      }
    }
  }
  return st;
}

#ifndef SM_DEC_OCC
#define SM_DEC_OCC 7  // waves per SIMD: 67 VGPRs, 5.0 KB LDS per wave (8: 64 VGPRs with a spill, 1.444 against 1.357 ms)
#endif
// one stream of the batch (block b) by one wave
template <uint32_t kLit = 4>
__device__ inline void decompress_block(const DecompressArgs& a, uint32_t b, uint8_t* sring, uint16_t* sjt, uint8_t* swin,
                                        uint32_t lane) {
  const uint8_t* in = a.one_n ? a.in : a.in + a.in_off[b];
  const uint32_t N = a.one_n ? a.one_n : a.in_len[b];
  uint8_t* dst = a.one_n ? a.out : a.out + a.out_off[b];
  const uint32_t cap = a.one_n ? a.one_cap : a.out_cap[b];

  uint32_t size = cap, ip = 0;
  if (N >= kOutLenError) {  // a compressor error mark, not a length: the slot holds no stream
    if (lane == 0) {
      a.status[b] = kErrDevice;
      a.out_len[b] = 0;
    }
    return;
  }
  int32_t st = a.raw ? kOk : parse_header(in, N, lane, size, ip);
  if (st == kOk && size > cap) st = kBufferTooSmall;
  if (st == kOk) {
    uint32_t op_end = 0;
    st = decode_stream_batch<kLit>(in, N, ip, N, size, dst, 0, 0, sring, sjt, swin, lane, op_end);
    if (st == kOk && op_end != size) st = kErrInvalid;                                    // Snappy.jl:50
  }
  if (lane == 0) {
    a.status[b] = st;
    a.out_len[b] = st == kOk ? size : 0;
  }
}

__global__ __launch_bounds__(64, SM_DEC_OCC) void k_decompress(DecompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sring[kRing + kRingMirror];
  __shared__ __attribute__((aligned(16))) uint16_t sjt[kJt];  // tag-walk jump tables
  __shared__ __attribute__((aligned(16))) uint8_t swin[kWinPad + kWin];  // output window
  decompress_block(a, blockIdx.x, sring, sjt, swin + kWinPad, lane_id());
}

// sm_uncompress's in-order path (a.one_n: one stream, one wave): the same engine with 16 loads a
// lane in flight in long literals -- a lone wave's bulk copy is bound by load latency, not by the
// VGPRs that set the batch kernel's occupancy (fireworks.jpeg's literal-only stream: see
// DESIGN.md section 3.4)
__global__ __launch_bounds__(64, 1) void k_decompress_one(DecompressArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sring[kRing + kRingMirror];
  __shared__ __attribute__((aligned(16))) uint16_t sjt[kJt];
  __shared__ __attribute__((aligned(16))) uint8_t swin[kWinPad + kWin];
  decompress_block<16>(a, 0, sring, sjt, swin + kWinPad, lane_id());
}

// ---- one large stream, decoded in parallel ------------------------
// Snappy.jl (src/Snappy.jl:29-33), libsnappy and this library compress 64 KiB blocks
// independently, so in their streams every output multiple of 65536 is a tag start and no copy
// reaches into an earlier block.  Finding those tags needs the tag boundaries, which the format
// does not index:
//  1. k_stream_index, one wave per 4 KiB chunk of the compressed body: the wave walks the tags
//     speculatively from the chunk's first byte (walk_window, 256 bytes per step: "lane 0's
//     path"), recording each visited position and the output before it; lanes l = 1..63 walk
//     from byte l (window-wise pointer doubling, the path's positions as stop nodes) until they
//     meet lane 0's path (tag walks resynchronise) or leave the chunk.  Each chunk then
//     knows, for entry offsets 0..63, where the walk leaves it and how much output it makes.
//  2. The host chains the true path (sm_api.hip) and locates each fragment's chunk.
//  3. k_decompress_frags, one wave per fragment: walk (window-parallel) from the chunk entry to
//     the tag at output F, then the batch engine with frag_lo = F and the output limit F + 65536.
// Anything unexpected (kErrCross, an error, a length mismatch) sends the caller to the in-order
// decode, which reproduces the reference's accept/reject exactly.

// stream tag at byte rel of an LDS copy: its size in the stream and its output bytes
// (char_entry / zero-padded lookahead: internal.jl:426-462)
__device__ inline void tag_at(const uint8_t* buf, uint32_t rel, uint64_t& size, uint64_t& outb) {
  const uint64_t hv = lds_ld64(buf, rel);
  const uint32_t c = (uint32_t)hv & 0xff;
  const uint32_t entry = char_entry(c);
  const uint32_t taglen = entry >> 11;
  const uint32_t tr_raw = (uint32_t)(hv >> 8);
  const uint32_t trailer = taglen >= 4 ? tr_raw : (tr_raw & ((1u << (8 * taglen)) - 1u));
  if (c & 3) {
    size = 1 + taglen;
    outb = entry & 0xff;
  } else {
    const uint32_t lit = (entry & 0xff) + trailer;  // u32 wrap, as the reference
    size = 1ull + taglen + lit;
    outb = lit;
  }
}

// bytes [s, s+len) of the stream into LDS, zero past N (the reference's zero-padded lookahead)
__device__ inline void stage_bytes(uint8_t* buf, const uint8_t* __restrict__ in, uint32_t N, uint32_t s, uint32_t len,
                                   uint32_t lane) {
  // dword k = stream bytes [s+4k, s+4k+4): two aligned global dwords + v_alignbyte, all of a
  // lane's loads issued before its LDS stores (len % 256 == 0 words per lane is not assumed)
  // Branch-free, so that every load is in flight at once (loads under divergent branches get a
  // wait at each join: six serial round trips per stage).  Aligned dwords are clamped to the one
  // holding byte N - 1 (the aligned dword at in + s - mis shares in[s]'s page), and the bytes at
  // or past N are masked to zero.
  constexpr int kU = 6;
  uint32_t* dst = reinterpret_cast<uint32_t*>(buf);
  const uint32_t nw = (len + 3) / 4;
  if (N == 0) {
    for (uint32_t k = lane; k < nw; k += kWave) dst[k] = 0;
    return;
  }
  const uint32_t mis = (uint32_t)((uintptr_t)(in + s) & 3u);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(in + s - mis);
  const int64_t klast = ((intptr_t)((uintptr_t)(in + N - 1) & ~(uintptr_t)3) - (intptr_t)src) / 4;  // (< 0: s >= N)
  for (uint32_t k0 = lane; k0 < nw; k0 += kU * kWave) {
    uint32_t w[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t k = k0 + u * kWave;
      w[u] = __builtin_amdgcn_alignbyte(src[min(k + 1, klast)], src[min(k, klast)], mis);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t b = (uint64_t)s + 4 * (k0 + u * kWave);  // stream offset of word k
      const uint64_t v = b < N ? (uint64_t)N - b : 0u;       // its bytes below N
      w[u] &= v >= 4 ? 0xffffffffu : (uint32_t)((1ull << (8 * v)) - 1);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (k0 + u * kWave < nw) dst[k0 + u * kWave] = w[u];
  }
}

// Tags of the staged window at chunk byte rel0 (walk_window over buf, rlim <= 256): lane t <
// ntok gets tag t's chunk position, its output bytes and the exclusive scan of them.  ntok == 0
// means a long literal (or nothing parseable) at rel0: the caller takes one scalar step.
__device__ inline uint32_t window_tags(const uint8_t* buf, uint32_t rel0, uint32_t rlim, uint16_t* jt, uint32_t lane,
                                       uint32_t& rel, uint32_t& next, uint32_t& outb, uint32_t& excl) {
  uint32_t cpos, csz, sizes;
  const uint32_t ntok = walk_window(lds_ld64(buf, rel0 + 4 * lane), rlim, jt, lane, cpos, csz, sizes);
  const bool mine = lane < ntok;
  const uint32_t c = buf[rel0 + (mine ? cpos : 0u)];
  const uint32_t e = char_entry(c);
  outb = !mine ? 0u : (c & 3) ? (e & 0xff) : csz - 1 - (e >> 11);  // a batch literal: csz = 1 + taglen + len
  excl = scan_dpp(outb) - outb;
  rel = rel0 + cpos;
  next = rel + csz;
  return ntok;
}

__device__ inline uint64_t load8z(const uint8_t* __restrict__ in, uint32_t N, uint32_t p) {
  return (uint64_t)load_word(in, N, p) | ((uint64_t)load_word(in, N, p + 4) << 32);
}

// Host tag walk (sm_api.hip host_walk) by one wave: where the tags from p leave [p, lim) and
// their output -- for chunk entries deeper than the index covers (lim - p <= kSmallChunk).  The
// bytes [p, lim + 256 + 32) are staged in stg (LDS, kDevWalkStage bytes) first; a 256-byte
// window of tags per step (walk_window, as k_origin_fill), a literal too long for a window by
// itself (its far end read from HBM).
template <uint32_t kC>  // (the chunk size: lim - p <= kC)
__device__ inline void dev_walk(const uint8_t* __restrict__ in, uint32_t N, uint64_t p, uint64_t lim, uint16_t* jt,
                                uint32_t lane, uint8_t* stg, uint64_t& exit_pos, uint64_t& produced) {
  constexpr uint32_t kStage = kC + kIdxPad;
  uint64_t o = 0;
  {  // Quick path: up to kQuickTags tags decoded one by one from a single load of the 256 bytes
     // at p's dword (zero past N, as the stage), no staging and no window walk.  A deep entry a
     // few bytes before its chunk's end, or one soon followed by a long literal, then costs one
     // round trip (most deep levels and walks of literal-heavy streams: paper-100k.pdf).
    constexpr uint32_t kQuickTags = 8;
    const uint32_t base = (uint32_t)p & ~3u;
    const uint32_t w = load_word(in, N, base + 4 * lane);
    uint64_t q = p, oq = 0;
    for (uint32_t k = 0; k < kQuickTags && q < lim; ++k) {
      const uint64_t rel = q - base;
      if (rel + 12 > 4 * kWave) break;
      const uint32_t i = (uint32_t)rel >> 2, sh = (uint32_t)rel & 3u;
      const uint32_t w0 = readlane(w, i), w1 = readlane(w, i + 1), w2 = readlane(w, i + 2);
      const uint32_t c = __builtin_amdgcn_alignbyte(w1, w0, sh) & 0xff;
      const uint32_t tr = __builtin_amdgcn_alignbyte(w2, w1, sh) << 24 | (__builtin_amdgcn_alignbyte(w1, w0, sh) >> 8);
      const uint32_t entry = char_entry(c);
      const uint32_t taglen = entry >> 11;
      const uint32_t trailer = taglen >= 4 ? tr : (tr & ((1u << (8 * taglen)) - 1u));
      if (c & 3) {
        q += 1 + taglen;
        oq += entry & 0xff;
      } else {
        const uint32_t lit = (entry & 0xff) + trailer;  // u32 wrap, as the reference
        q += 1ull + taglen + lit;
        oq += lit;
      }
    }
    p = q;  // (the window walk goes on from here when the quick path did not leave)
    o = oq;
  }
  const uint64_t sp = p;
  if (p < lim) {
    stage_bytes(stg, in, N, (uint32_t)sp, kStage, lane);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (one wave: its LDS stores land before its loads)
  }
  auto rd8 = [&](uint64_t x) -> uint64_t {
    return x >= sp && x - sp + 8 <= kStage ? lds_ld64(stg, (uint32_t)(x - sp)) : load8z(in, N, (uint32_t)x);
  };
  while (p < lim) {
    const uint32_t rlim = (uint32_t)min((uint64_t)256, lim - p);
    uint32_t cpos, csz, sizes;
    const uint32_t ntok = walk_window(rd8(p + 4 * lane), rlim, jt, lane, cpos, csz, sizes);
    if (ntok == 0) {  // a literal too long for a window walk (or a wrapped length)
      const uint64_t hv = rd8(p);
      const uint32_t c = uniform((uint32_t)hv & 0xff);
      const uint32_t entry = char_entry(c);
      const uint32_t taglen = entry >> 11;
      const uint32_t tr = uniform((uint32_t)(hv >> 8));
      const uint32_t trailer = taglen >= 4 ? tr : (tr & ((1u << (8 * taglen)) - 1u));
      if (c & 3) {
        p += 1 + taglen;
        o += entry & 0xff;
      } else {
        const uint32_t lit = (entry & 0xff) + trailer;  // u32 wrap, as the reference
        p += 1ull + taglen + lit;
        o += lit;
      }
      continue;
    }
    const bool mine = lane < ntok;
    const uint32_t c = (uint32_t)rd8(p + (mine ? cpos : 0u)) & 0xff;
    const uint32_t e = char_entry(c);
    const uint32_t ob = !mine ? 0u : (c & 3) ? (e & 0xff) : csz - 1 - (e >> 11);  // a window literal: csz = 1 + taglen + len
    const uint32_t incl = scan_dpp(ob);
    o += readlane(incl, ntok - 1);
    p += readlane(cpos + csz, ntok - 1);
  }
  exit_pos = p;
  produced = o;
}

// kDeep (path 4): also deep[kDeepLevels (kDeepChains c + ch)] = (x, exit, output, 1) for entering
// the chunk where this one's entry walks leave it, x, when x lies kIdxEntries or more bytes into
// it (a long literal across the boundary): the entry the device chain needs there whenever its
// walk passed through this chunk from one of the entries (chain 0: lane 0's exit, chains 1..:
// other distinct entry exits).  Level k + 1 likewise enters where level k's walk leaves
// (consecutive long literals: the chunks between start inside a literal, and their own lane-0
// paths need not be the stream's).  .w = 0: no such level.
// kDeep: one wave per deep-record chain (kDeepChains waves): wave 0 indexes the chunk, then each
// wave walks its chain's levels (serial dev_walks) at the same time as the others.
constexpr uint32_t index_threads(bool deep) { return deep ? kDeepChains * kWave : kWave; }
// copy_to (path 4 from a host call, else null): `in` is the call's input in device-mapped pinned
// host memory, and chunk c's bytes (chunk 0: also the header before ip0) go on to copy_to, the
// device copy the later kernels read -- the upload folded into the index launch.
template <uint32_t kC, bool kDeep>  // compressed bytes per chunk (kIdxChunk; path 4: kSmallChunk)
__global__ __launch_bounds__(index_threads(kDeep)) void k_stream_index(const uint8_t* __restrict__ in, uint32_t N,
                                                                          uint32_t ip0, uint2* rec, uint4* deep,
                                                                          uint8_t* __restrict__ copy_to) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kC + kIdxPad];
  __shared__ __attribute__((aligned(16))) uint16_t jt[6 * 256];  // walk tables, then the entry walk's 3 KiB
  __shared__ uint32_t bm[kC / 32];  // positions on lane 0's path
  __shared__ uint32_t cum[kC];      // output before each such position
  constexpr uint32_t kXw = kDeep ? kDeepChains - 1 : 1;  // waves 1.. : their own walk stage and tables
  __shared__ __attribute__((aligned(16))) uint8_t xstg[kXw][kC + kIdxPad + 16];
  __shared__ __attribute__((aligned(16))) uint16_t xjt[kXw][kJt];
  __shared__ uint64_t xs[kDeepChains];  // each chain's first entry (~0: none)
  const uint32_t c = blockIdx.x, lane = lane_id(), wv = threadIdx.x / kWave;
  const uint32_t s = ip0 + c * kC;
  if (copy_to) {
    const uint32_t a = c == 0 ? 0u : s, e = min(s + kC, N);
    for (uint32_t k = a + threadIdx.x; k < e; k += blockDim.x) copy_to[k] = in[k];
  }
  if (wv == 0) {  // (one wave from here to the chain starts: LDS in order, signal fences only)
    stage_bytes(buf, in, N, s, kC + kIdxPad, lane);
    for (uint32_t k = lane; k < kC / 32; k += kWave) bm[k] = 0;
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint64_t lim = min((uint64_t)s + kC, (uint64_t)N - 1);  // tags start below N-1 (:416)
    // lane 0's path: the tag walk from the chunk's first byte, a 256-byte window at a time
    uint64_t p = s, acc = 0, size, outb;
    while (p < lim) {
      const uint32_t rel0 = (uint32_t)(p - s);
      uint32_t rel, next, ob, excl;
      const uint32_t ntok = window_tags(buf, rel0, (uint32_t)min(lim - p, (uint64_t)256), jt, lane, rel, next, ob, excl);
      if (ntok == 0) {  // long literal
        if (lane == 0) {
          bm[rel0 >> 5] |= 1u << (rel0 & 31);
          cum[rel0] = (uint32_t)acc;
        }
        tag_at(buf, rel0, size, outb);
        acc += outb;
        p += size;
        continue;
      }
      if (lane < ntok) {
        atomicOr(&bm[rel >> 5], 1u << (rel & 31));
        cum[rel] = (uint32_t)acc + excl;
      }
      acc += readlane(excl + ob, ntok - 1);
      p = s + readlane(next, ntok - 1);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint64_t exit0 = p;
    const uint32_t tot0 = (uint32_t)acc;
    // Lanes 1..63 (entries at chunk bytes 1..63) walk until they meet lane 0's path or leave the
    // chunk, a 256-byte window at a time, by pointer doubling with lane 0's path as stop nodes:
    // J0[x] = x + size(x), O0[x] = its output bytes; a path position, a long literal or a
    // position at/after the limit is a fixed point (O = 0).  Seven doublings give 128 steps --
    // more tags than 256 bytes hold -- so J7[x] is where the walk from x meets the path, stops or
    // leaves the window, and O7[x] the output on the way.  Long literals take a scalar step.
    const uint64_t rl = lim > s ? lim - s : 0;  // chunk-relative parse limit
    uint64_t x = lane, ex = exit0;
    uint32_t pre = 0, res = tot0;
    bool done = lane == 0;
    uint16_t* tj = jt;                                   // 2 x 256 u16
    uint32_t* to = reinterpret_cast<uint32_t*>(jt + 512);  // 2 x 256 u32 (jt holds 3 KiB here)
    while (true) {
      bool again = true;
      while (ballot(again)) {  // settle: out of the chunk, on the path, or a long literal
        again = false;
        if (!done) {
          if (x >= rl) {
            ex = s + x;
            res = pre;
            done = true;
          } else if ((bm[x >> 5] >> (x & 31)) & 1u) {  // met lane 0's path
            res = pre + (tot0 - cum[x]);
            done = true;
          } else {
            tag_at(buf, (uint32_t)x, size, outb);
            if (walk_stop_literal(buf[x], outb)) {
              pre += (uint32_t)outb;
              x += size;
              again = true;
            }
          }
        }
      }
      if (!ballot(!done)) break;
      uint32_t base = done ? 0xffffffffu : (uint32_t)x;
  #pragma unroll
      for (int d = 1; d < 64; d <<= 1) base = min(base, (uint32_t)__shfl_xor(base, d, 64));
      const uint32_t rlim = (uint32_t)min(rl - base, (uint64_t)256);
      const uint64_t cw = lds_ld64(buf, base + 4 * lane);
      const uint32_t sizes = pack_sizes((uint32_t)cw, (uint32_t)(cw >> 32));
      uint32_t J[4], O[4];
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t r = 4 * lane + j, a = base + r, sz = (sizes >> (8 * j)) & 0xff, cb = (uint32_t)(cw >> (8 * j)) & 0xff;
        const uint32_t e = char_entry(cb);
        const bool stop = r >= rlim || ((bm[a >> 5] >> (a & 31)) & 1u) || sz == 255;  // (bm read below rlim only)
        J[j] = stop ? r : r + sz;
        O[j] = stop ? 0u : (cb & 3) ? (e & 0xff) : sz - 1 - (e >> 11);
      }
  #pragma unroll
      for (int k = 0; k < 8; ++k) {  // k = 7: the final tables for the lanes' read
        uint16_t* bj = tj + (k & 1) * 256;
        uint32_t* bo = to + (k & 1) * 256;
  #pragma unroll
        for (int j = 0; j < 4; ++j) {
          bj[4 * lane + j] = (uint16_t)J[j];
          bo[4 * lane + j] = O[j];
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (k == 7) break;
  #pragma unroll
        for (int j = 0; j < 4; ++j)
          if (J[j] < 256) {
            O[j] += bo[J[j]];
            J[j] = bj[J[j]];
          }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
      }
      if (!done && x < base + 256) {
        const uint32_t r = (uint32_t)x - base;
        pre += to[256 + r];
        x = base + tj[256 + r];
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the next window's stores follow these reads
    }
    // (exit, output) pairs side by side: the host's walk over the records reads one cache line
    rec[c * kIdxEntries + lane] = make_uint2((uint32_t)min(ex, (uint64_t)0xffffffffu), res);
    if constexpr (kDeep) {
      // chain 0 starts at lane 0's exit; chains 1.. at other distinct exits of the entry lanes that
      // land kIdxEntries or more bytes into a chunk (the records there do not cover them: a walk
      // that did not meet lane 0's path, e.g. one inside a long literal).  tools/chain_model.py
      // --distinct: paper-100k.pdf's fast stream 19 chain walks with one chain, 7 with four.
      auto deep_at = [&](uint64_t v) {
        const uint64_t db = ip0 + ((v - ip0) / kC) * kC;
        return v < (uint64_t)N - 1 && v - db >= kIdxEntries;
      };
      // (only exits inside the next chunk: the entry lanes that are not on the stream's path read
      // garbage as tags and often jump far -- chains for those cost alice29.txt 10 us, and the
      // model finds the same 7 walks on paper-100k.pdf without them)
      const uint32_t ex32 = (uint32_t)min(ex, (uint64_t)0xffffffffu);
      uint64_t more = ballot(ex != exit0 && ex < (uint64_t)s + 2 * kC && deep_at(ex));
      for (uint32_t ch = 0; ch < kDeepChains; ++ch) {
        uint64_t x = ~0ull;  // (no chain: zero records)
        if (ch == 0) {
          x = exit0;
        } else if (more) {
          x = readlane(ex32, ctz64(more));
          more &= ballot(ex32 != (uint32_t)x);
        }
        if (lane == 0) xs[ch] = x;
      }
    }
  }  // (wave 0)
  if constexpr (kDeep) {
    __syncthreads();
    const uint32_t ch = wv;
    uint64_t x = xs[ch];
    uint8_t* const stg = ch == 0 ? buf : xstg[ch - 1];  // (buf: free now)
    uint16_t* const wjt = ch == 0 ? jt : xjt[ch - 1];
    auto deep_at = [&](uint64_t v) {
      const uint64_t db = ip0 + ((v - ip0) / kC) * kC;
      return v < (uint64_t)N - 1 && v - db >= kIdxEntries;
    };
    uint4* const dc = deep + (size_t)(kDeepChains * c + ch) * kDeepLevels;
    for (uint32_t k = 0; k < kDeepLevels; ++k) {
      uint4 dr = make_uint4(0, 0, 0, 0);
      if (x != ~0ull && deep_at(x)) {
        const uint64_t db = ip0 + ((x - ip0) / kC) * kC;
        uint64_t dex, dot;
        dev_walk<kC>(in, N, x, min(db + kC, (uint64_t)N - 1), wjt, lane, stg, dex, dot);
        dr = make_uint4((uint32_t)x, (uint32_t)min(dex, (uint64_t)0xffffffffu),
                        (uint32_t)min(dot, (uint64_t)0xffffffffu), 1u);
        x = dex;
      }
      if (lane == 0) dc[k] = dr;
      if (!dr.w) {
        for (uint32_t j = k + 1; j < kDeepLevels; ++j)
          if (lane == 0) dc[j] = make_uint4(0, 0, 0, 0);
        break;
      }
    }
  }
}

__global__ __launch_bounds__(64, 4) void k_decompress_frags(const uint8_t* __restrict__ in, uint32_t N, uint32_t size,
                                                            uint8_t* out, const StreamFrag* frags, int32_t* status) {
  __shared__ __attribute__((aligned(16))) uint8_t sring[kRing + kRingMirror];
  __shared__ __attribute__((aligned(16))) uint16_t sjt[kJt];
  __shared__ __attribute__((aligned(16))) uint8_t swin[kWinPad + kWin];
  __shared__ __attribute__((aligned(16))) uint8_t sbuf[kIdxChunk + kIdxPad];
  const uint32_t f = blockIdx.x, lane = lane_id();
  const StreamFrag fr = frags[f];
  // walk from the chunk entry to the tag that starts at output F (inside that chunk), a
  // 256-byte window at a time: the first tag whose preceding output reaches F
  stage_bytes(sbuf, in, N, fr.y, kIdxChunk + kIdxPad, lane);
  __syncthreads();
  uint64_t p = fr.y, o = fr.O, tsz, outb;
  int32_t st = kOk;
  while (o < fr.F) {
    const uint32_t rel0 = (uint32_t)(p - fr.y);
    if (rel0 >= kIdxChunk + 16) {
      st = kErrCross;
      break;
    }
    uint32_t rel, next, ob, excl;
    const uint32_t ntok = window_tags(sbuf, rel0, min(kIdxChunk + 16 - rel0, 256u), sjt, lane, rel, next, ob, excl);
    if (ntok == 0) {  // long literal
      tag_at(sbuf, rel0, tsz, outb);
      o += outb;
      p += tsz;
      continue;
    }
    const uint64_t hit = ballot(lane < ntok && o + excl >= fr.F);
    if (hit) {
      const uint32_t t = ctz64(hit);
      o += readlane(excl, t);
      p = fr.y + readlane(rel, t);
      break;
    }
    o += readlane(excl + ob, ntok - 1);
    p = fr.y + readlane(next, ntok - 1);
  }
  if (st == kOk && o != fr.F) st = kErrCross;  // no tag starts at F: not block-structured
  if (st == kOk) {
    uint32_t op_end = 0;
    st = decode_stream_batch(in, N, (uint32_t)p, N, size, out, fr.F, fr.F, sring, sjt, swin + kWinPad, lane, op_end, fr.lim);
    if (st == kOk && op_end != (fr.lim == 0xffffffffu ? size : fr.lim)) st = kErrCross;
  }
  if (lane == 0) status[f] = st;
}

// ---- validation and declared lengths, no output -----------------------
// k_validate: the decoder's tag walk and checks (decode_stream_batch, internal.jl:411-527)
// without moving data: a block's status is exactly what uncompress(block) returns with an
// unlimited output buffer (snappy-c.h snappy_validate_compressed_buffer).  One wave per block,
// a 256-byte window per step, staged from HBM into LDS.
__global__ __launch_bounds__(64) void k_validate(const uint8_t* __restrict__ d_in, const uint64_t* in_off,
                                                 const uint32_t* in_len, int32_t* status) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[320];
  __shared__ __attribute__((aligned(16))) uint16_t jt[kJt];
  const uint32_t b = blockIdx.x, lane = lane_id();
  const uint8_t* in = d_in + in_off[b];
  const uint32_t N = in_len[b];
  if (N >= kOutLenError) {  // a compressor error mark (k_decompress): no read of the slot
    if (lane == 0) status[b] = kErrDevice;
    return;
  }
  uint32_t size, ip;
  int32_t st = parse_header(in, N, lane, size, ip);
  uint64_t op = 0, p = ip;
  const uint64_t lim = N ? N - 1 : 0;  // tags start below N-1 (:416)
  while (st == kOk && p < lim) {
    stage_bytes(buf, in, N, (uint32_t)p, 320, lane);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint32_t rel, next, ob, excl;
    const uint32_t ntok = window_tags(buf, 0, (uint32_t)min(lim - p, (uint64_t)256), jt, lane, rel, next, ob, excl);
    const bool mine = lane < ntok || (ntok == 0 && lane == 0);  // ntok == 0: a long literal at p
    const uint64_t hv = lds_ld64(buf, mine ? rel : 0u);
    const uint32_t c = (uint32_t)hv & 0xff;
    const uint32_t entry = char_entry(c);
    const uint32_t len = entry & 0xff;
    const uint32_t taglen = entry >> 11;
    const uint32_t tr_raw = (uint32_t)(hv >> 8);
    const uint32_t trailer = taglen >= 4 ? tr_raw : (tr_raw & ((1u << (8 * taglen)) - 1u));
    const uint32_t offset = (entry & 0x700) + trailer;
    const uint32_t litlen = len + trailer;  // u32 wrap, as the reference
    const uint64_t opt = op + (ntok ? excl : 0u);
    const int64_t avail_out = (int64_t)size - (int64_t)opt;
    int32_t err = kOk;
    if (mine) {
      if (c & 3) {
        if ((int64_t)opt <= (int64_t)(uint32_t)(offset - 1u)) err = kErrCopyOffset;                                  // :499
        else if (!(len <= 16 && offset >= 8 && avail_out >= 16) && avail_out < (int64_t)len) err = kErrCopyLength;  // :505
      } else {
        const int64_t avail_in = (int64_t)N - (int64_t)(p + (ntok ? rel : 0u) + 1 + taglen);
        if (avail_out < (int64_t)litlen || avail_in < (int64_t)litlen) err = kErrLiteral;  // :518
      }
    }
    const uint64_t em = ballot(err != kOk);
    if (em) {
      st = (int32_t)readlane((uint32_t)err, ctz64(em));
      break;
    }
    if (ntok == 0) {
      op += readlane(litlen, 0);
      p += 1 + readlane(taglen, 0) + (uint64_t)readlane(litlen, 0);
    } else {
      op += readlane(excl + ob, ntok - 1);
      p += readlane(next, ntok - 1);
    }
  }
  if (st == kOk && op != size) st = kErrInvalid;  // Snappy.jl:50
  if (lane == 0) status[b] = st;
}

// k_uncompressed_length: the varint header of each block (length_uncompressed,
// src/Snappy.jl:90-92), one thread per block
__global__ __launch_bounds__(256) void k_uncompressed_length(const uint8_t* __restrict__ d_in, const uint64_t* in_off,
                                                             const uint32_t* in_len, uint32_t nblk, uint32_t* out_len,
                                                             int32_t* status) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const uint8_t* in = d_in + in_off[b];
  const uint32_t N = in_len[b];
  uint32_t v = 0;
  int32_t st = N >= kOutLenError ? kErrDevice : kErrVarint;  // (a compressor error mark: no read)
  for (uint32_t i = 0; i < 5 && N < kOutLenError && i < N; ++i) {
    const uint32_t bt = in[i];
    v |= (bt & 0x7f) << (7 * i);
    if (i < 4 ? bt < 0x80 : bt < 0x10) {
      st = kOk;
      break;
    }
  }
  out_len[b] = st == kOk ? v : 0;
  status[b] = st;
}

hipError_t launch_validate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t nblk,
                           int32_t* status, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_validate, dim3(nblk), dim3(64), 0, s, in, in_off, in_len, status);
  return hipGetLastError();
}

hipError_t launch_uncompressed_length(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                      uint32_t nblk, uint32_t* out_len, int32_t* status, hipStream_t s) {
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_uncompressed_length, dim3((nblk + 255) / 256), dim3(256), 0, s, in, in_off, in_len, nblk,
                     out_len, status);
  return hipGetLastError();
}

// ---- any large stream, decoded in parallel by origin pointers ---------
// A stream whose copies reach into earlier 64 KiB blocks (not block-structured) cannot be cut
// into independent fragments.  Its output is still a pure function of the tags: output byte x
// is a literal byte in[i] or, inside a copy with offset d, the byte at x - d.  With the tag
// path of k_stream_index (host-chained: path element e = the tags starting in [y_e, ex_e),
// whose output starts at O_e):
//  1. k_origin_fill, one wave per path element: walk the element's tags (walk_window over
//     64-B-strided global words), apply the reference's checks (src/internal.jl:499,505,518),
//     and write P[x] for every output byte: 0x80000000 | i for a literal byte in[i], x - d for
//     a copy byte;
//  2. k_origin_resolve rounds: P[x] = P[P[x]] while P[x] names a copy byte.  Every value stays
//     an earlier byte of x's copy chain (in-place updates only move along it), and round k
//     moves an unresolved pointer at least 2^k steps, so ceil(log2(size)) rounds finish;
//  3. k_origin_gather: out[x] = in[P[x] & 0x7fffffff].
// The result is the plain LZ77 meaning of the tags -- decompress_all_tags!'s output for a valid
// stream (incremental_copy_slow!, internal.jl:477-481).  Any check that fails sends the caller
// to the in-order decode, which returns the reference's exact status.


// One path element's tags by one wave (window walks, internal.jl:411-466), with the reference's
// checks; kFill: the origin pointer of every output byte into P.  Returns the element's status.
// stg (optional): the stream bytes [sb, sb + sl) staged in LDS (stage_bytes), read instead of HBM
template <bool kFill>
__device__ __attribute__((always_inline)) inline int32_t origin_walk(const uint8_t* __restrict__ in, uint32_t N,
                                                                   uint32_t size, const OriginPath pe,
                                                                   uint32_t* __restrict__ P, uint16_t* jt,
                                                                   uint32_t lane, const uint8_t* stg = nullptr,
                                                                   uint32_t sb = 0, uint32_t sl = 0) {
  auto load8z = [&](const uint8_t* __restrict__ in_, uint32_t N_, uint32_t p) -> uint64_t {
    return (stg && p >= sb && p - sb + 8 <= sl) ? lds_ld64(stg, p - sb) : sm::load8z(in_, N_, p);
  };
  uint32_t ip = pe.y, op = pe.O;
  int32_t st = kOk;
  const uint32_t end = min(pe.ex, N - 1);  // a tag on the last byte is never parsed (internal.jl:416)
  while (ip < end) {
    const uint32_t rlim = min(256u, end - ip);  // tags that start before ex
    uint32_t cpos, csz, sizes;
    const uint32_t ntok = walk_window(load8z(in, N, ip + 4 * lane), rlim, jt, lane, cpos, csz, sizes);
    if (ntok == 0) {  // a literal too long for a window walk (or a wrapped length): whole wave
      const uint64_t hv = load8z(in, N, ip);
      const uint32_t c = uniform((uint32_t)hv & 0xff);
      const uint32_t entry = char_entry(c);
      const uint32_t taglen = entry >> 11;
      const uint32_t tr_raw = uniform((uint32_t)(hv >> 8));
      const uint32_t trailer = taglen >= 4 ? tr_raw : (tr_raw & ((1u << (8 * taglen)) - 1u));
      const uint32_t litlen = (entry & 0xff) + trailer;  // u32 wrap, as the reference
      const uint64_t lsrc = (uint64_t)ip + 1 + taglen;
      if ((c & 3) || lsrc + litlen > N || (uint64_t)op + litlen > size) {  // :518 (a copy here: bad path)
        st = (c & 3) ? (kFill ? kErrInvalid : kErrCross) : kErrLiteral;
        break;
      }
      if (kFill)
        for (uint32_t i = lane; i < litlen; i += kWave) P[op + i] = 0x80000000u | (uint32_t)(lsrc + i);
      op += litlen;
      ip = (uint32_t)(lsrc + litlen);
      continue;
    }
    const bool mine = lane < ntok;
    const uint32_t tpos = ip + (mine ? cpos : 0u);
    const uint64_t hv = load8z(in, N, tpos);
    const uint32_t c = (uint32_t)hv & 0xff;
    const uint32_t entry = char_entry(c);
    const uint32_t len = entry & 0xff;
    const uint32_t taglen = entry >> 11;
    const uint32_t tr_raw = (uint32_t)(hv >> 8);
    const uint32_t trailer = taglen >= 4 ? tr_raw : (tr_raw & ((1u << (8 * taglen)) - 1u));
    const bool iscopy = (c & 3) != 0;
    const uint32_t offset = (entry & 0x700) + trailer;
    const uint32_t litlen = len + trailer;
    const uint32_t olen = mine ? (iscopy ? len : litlen) : 0u;
    const uint32_t incl = scan_dpp(olen);
    const uint32_t opt = op + incl - olen;
    const uint32_t lsrc = tpos + 1 + taglen;
    const bool bad_off = iscopy && (offset == 0 || offset > opt);                                  // :499
    const bool bad = mine && (iscopy ? (bad_off || (uint64_t)opt + len > size)                     // :505
                                     : ((uint64_t)lsrc + litlen > N || (uint64_t)opt + litlen > size));  // :518
    const uint64_t bm = ballot(bad);
    if (bm) {  // the first failing tag in stream order decides
      const int32_t code = iscopy ? (bad_off ? kErrCopyOffset : kErrCopyLength) : kErrLiteral;
      st = kFill ? kErrInvalid : (int32_t)readlane((uint32_t)code, ctz64(bm));
      break;
    }
    // every output byte of the window's tags: tag t's bytes by the whole wave.  A copy's byte i
    // points at o - f + (i mod f): for i >= f its source lies inside the same copy, whose byte
    // i - f is byte (i mod f) of the period (incremental_copy!, internal.jl:491-509) -- so a run
    // (offset 1, 2, ...) adds one chain step, not one per period.
    if (kFill) {  // each lane its own tag's pointers, four a store (P[o + i] = base + i')
      const uint32_t base = iscopy ? opt - offset : 0x80000000u | lsrc;
      const uint32_t f = iscopy && offset < olen ? offset : 0xffffffffu;  // a copy overlapping itself
      uint32_t* const dst = P + opt;
      uint32_t i = 0, r = 0;  // r = i mod f
      auto nx = [&]() { r = r + 1 == f ? 0u : r + 1; };
      while (ballot(i + 4 <= olen)) {
        if (i + 4 <= olen) {
          uint4 v;
          v.x = base + r;
          nx();
          v.y = base + r;
          nx();
          v.z = base + r;
          nx();
          v.w = base + r;
          nx();
          *reinterpret_cast<uint4 __attribute__((aligned(4)))*>(dst + i) = v;
          i += 4;
        }
      }
      while (ballot(i < olen)) {
        if (i < olen) {
          dst[i] = base + r;
          nx();
          ++i;
        }
      }
    }
    op += readlane(incl, ntok - 1);
    ip += readlane(cpos + csz, ntok - 1);
  }
  if (st == kOk && ip != pe.ex && !(ip >= end && pe.ex >= end)) st = kFill ? kErrInvalid : kErrCross;  // tags tile the path
  if (st == kOk && op != pe.O + pe.out) st = kFill ? kErrInvalid : kErrCross;
  return st;
}

// kFill = false (k_path_check): the same walk without P, recording the reference's exact status
// of the element's first failing tag (src/internal.jl:499, :505, :518) -- a stream's first error
// is then the first failing element in path order, found in parallel instead of by the in-order
// decode.  kErrCross marks an element whose tags do not tile it (the caller falls back).
template <bool kFill>
__global__ __launch_bounds__(64) void k_origin_fill(const uint8_t* __restrict__ in, uint32_t N, uint32_t size,
                                                    const OriginPath* path, uint32_t* __restrict__ P,
                                                    int32_t* status) {
  __shared__ __attribute__((aligned(16))) uint16_t jt[kJt];
  const int32_t st = origin_walk<kFill>(in, N, size, path[blockIdx.x], P, jt, lane_id());
  if (lane_id() == 0) status[blockIdx.x] = st;
}

// ---- a small stream, all on the device (sm_uncompress): the index records chained by one wave
// instead of the host, the origin pointers filled per path element, resolved in a fixed number of
// launches and gathered -- one synchronisation for the whole call.  Any stream (no block
// structure assumed); anything unexpected (an error, no progress, a length mismatch) is reported
// in ctl[1] and the caller decodes the old way, which also finds the first error.
// The chain's LDS pool (u32 words): the entry records of the first chunks, compact (below), then
// the deep records of as many chunks as still fit.  Everything else is read from HBM.
constexpr uint32_t kChainThreads = 1024;  // all of them load the pool and take part in the runs
constexpr uint32_t kChainPool = 96u * 1024 / 4;
constexpr uint32_t kChainPath = 1024;  // path elements kept in LDS until the end (more: straight to HBM)
constexpr uint32_t kDeepWords = kDeepChains * kDeepLevels * 4;  // a chunk's deep records
constexpr uint32_t kRecNone = 0xffffffffu;                       // compact record: not representable
constexpr uint32_t kChainNodes = kChainThreads;  // chunks the parallel runs cover, one thread each
constexpr uint32_t kLift = 10;                   // 2^kLift >= kChainNodes: jump tables J[0..kLift)
constexpr uint32_t kMinRun = 8;                  // links ahead that make a parallel run worth two barriers
constexpr uint32_t kRunDone = 0xffffffffu;
#ifndef SM_CHAIN_DEEPLINK
#define SM_CHAIN_DEEPLINK 1  // links through chain 0's deep records (0: entry records only)
#endif
static_assert((1u << kLift) >= kChainNodes, "the jump tables must reach every node");
// k_stream_chain's static LDS, summed against the 160 KiB a workgroup may declare (ADVICE round 5:
// at kC = 1024 the kernel uses ~159 KiB, so growing kChainPool, kChainPath, kLift, kIdxPad or
// OriginPath by a little fails here, where these constants are tuned, not in the compiler)
template <uint32_t kC>
constexpr uint32_t chain_lds_bytes() {
  return 4 * kChainPool + (uint32_t)sizeof(OriginPath) * kChainPath + 2 * kLift * kChainNodes +
         (5 * 4 + 1) * kChainNodes + 4 * 5 + 2 * kJt + (kC + kIdxPad + 16) + 64 /* alignment slack */;
}
static_assert(chain_lds_bytes<1024>() <= 160u * 1024 && chain_lds_bytes<512>() <= 160u * 1024 &&
                  chain_lds_bytes<kSmallChunkTiny>() <= 160u * 1024,
              "k_stream_chain's LDS arrays exceed 160 KiB");
// an entry record (exit, output) of chunk base `base`, compact: (output << 16) | (exit - base)
__device__ inline uint32_t rec_compact(uint2 r, uint64_t base) {
  const uint64_t d = (uint64_t)r.x - base;
  return r.x >= base && d < 0xffffu && r.y <= 0xffffu ? (r.y << 16) | (uint32_t)d : kRecNone;
}

// The chain, in parallel where it can be.  Chunk c's lane-0 walk exits at E(c); entered anywhere,
// its walk usually meets lane 0's path and exits there too.  The link c -> c' holds when E(c)
// enters c' at an entry the records cover (offset < kIdxEntries) AND that entry's walk exits at
// E(c') -- then the element after the one in c' is again decided by a link.  A link may also pass
// through chain 0's deep records of c first (E(c) deep in a later chunk, consecutive long
// literals: the deep elements the serial chain would take there).  Pointer jumping over the
// links (one thread per chunk, kLift rounds) gives every chunk its distance D to the end of its
// links, the elements and the output (SS) on the way, and the jump tables J[k] (2^k links).
// When the serial chain (wave 0) stands on an entry whose walk exits at E(c1) with D(c1) >=
// kMinRun links ahead, every chunk t tests in parallel whether it lies i = D(c1) - D(t) links
// along from c1 (J0 of the node i - 1 along is t) and writes its own path element and its link's
// deep elements; wave 0 continues after the last.  Every run element is one the serial chain
// would take (same record, same exit), so the path is identical; anything else (other deep
// entries, walks) stays serial.
__device__ inline uint4 chain_deep0(const uint4* sdeep, const uint4* __restrict__ deep, uint32_t nsdeep, uint32_t c,
                                    uint32_t k) {
  const uint32_t i = kDeepLevels * kDeepChains * c + k;
  uint4 v;
  if (i < nsdeep)
    v = sdeep[i];
  else
    v = deep[i];
  return v;
}

// ctl[0] = path elements, ctl[1] = 0 (the path covers exactly `size` bytes of output) or 1 (fall back)
template <uint32_t kC>  // bytes per index chunk
__global__ __launch_bounds__(kChainThreads) void k_stream_chain(const uint8_t* __restrict__ in, uint32_t N, uint32_t ip0,
                                                                uint32_t size, uint32_t nchunks,
                                                                const uint2* __restrict__ rec,
                                                                const uint4* __restrict__ deep, OriginPath* path,
                                                                uint32_t* ctl, uint32_t nrounds) {
  __shared__ __attribute__((aligned(16))) uint32_t pool[kChainPool];
  __shared__ __attribute__((aligned(16))) OriginPath spath[kChainPath];
  __shared__ uint16_t J[kLift][kChainNodes];
  // per chunk node: D (links to the end, low 16 bits) | elements before the end's (high 16), the
  // output on the way (saturating), E, the output of the linked element, of the deep elements
  // before it, and their count
  __shared__ uint32_t Dsh[kChainNodes], SSsh[kChainNodes], Esh[kChainNodes], Wsh[kChainNodes], Wdsh[kChainNodes];
  __shared__ uint8_t Lsh[kChainNodes];
  __shared__ uint32_t run[5];  // the run wave 0 asks for: c1 (kRunDone: finished), y, O, np, output of c1's element
  __shared__ __attribute__((aligned(16))) uint16_t jt[kJt];
  __shared__ __attribute__((aligned(16))) uint8_t stg[kC + kIdxPad + 16];
  // one round trip for the whole pool: every thread's loads are in flight before its stores
  const uint32_t nrec = min(nchunks, kChainPool / kIdxEntries);                    // chunks with LDS records
  const uint32_t ndeep = min(nchunks, (kChainPool - nrec * kIdxEntries) / kDeepWords);  // ... and LDS deep records
  uint32_t* const srec = pool;
  uint4* const sdeep = reinterpret_cast<uint4*>(pool + nrec * kIdxEntries);  // (16-B aligned: nrec * 64 words)
  const uint32_t t = threadIdx.x;
  {  // (clamped indices, no branches around the loads: they all issue before the first wait)
    const uint32_t nr = nrec * kIdxEntries, nd = ndeep * kDeepWords / 4;
    for (uint32_t k0 = t; k0 < nr; k0 += 8 * kChainThreads) {
      uint2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = rec[min(k0 + u * kChainThreads, nr - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t k = k0 + u * kChainThreads;
        if (k < nr) srec[k] = rec_compact(v[u], ip0 + (uint64_t)(k / kIdxEntries) * kC);
      }
    }
    for (uint32_t k0 = t; k0 < nd; k0 += 4 * kChainThreads) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = deep[min(k0 + u * kChainThreads, nd - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) sdeep[min(k0 + u * kChainThreads, nd - 1)] = v[u];  // (past nd: the last again)
    }
  }
  __syncthreads();
  const bool par = nchunks <= kChainNodes;
  // a compact entry record from LDS, or from HBM past the pool
  auto crec = [&](uint32_t cc, uint32_t l) {
    return cc < nrec ? srec[cc * kIdxEntries + l]
                     : rec_compact(rec[cc * kIdxEntries + l], ip0 + (uint64_t)cc * kC);
  };
  // chain 0's deep record k of chunk c (LDS, or HBM past the pool)
  const uint32_t nsdeep = ndeep * kDeepChains * kDeepLevels;
#define drec0(c, k) chain_deep0(sdeep, deep, nsdeep, (c), (k))
  if (par) {  // the links and their pointer jumping (a root links to itself)
    uint32_t link = t, w = 0, wd = 0, nd = 0, e = 0xffffffffu;
    if (t < nchunks) {
      const uint32_t v0 = crec(t, 0);
      if (v0 != kRecNone) {
        e = ip0 + t * kC + (v0 & 0xffffu);
        // from E(t): through chain 0's deep records while the exits land deep in later chunks
        // (the serial chain takes exactly those: level 0 from the chains of t's chunk, level k + 1
        // as the next level of the record it came from), then a recorded entry that exits at E
        uint32_t X = e;
        for (uint32_t k = 0; k <= kDeepLevels; ++k) {
          const uint32_t xr = X - ip0, cx = xr / kC, lx = xr % kC;
          if ((uint64_t)X >= (uint64_t)N - 1 || cx >= nchunks || cx <= t) break;
          if (lx < kIdxEntries) {
            const uint32_t v2 = crec(cx, lx), v20 = crec(cx, 0);
            if (v2 != kRecNone && v20 != kRecNone && (v2 & 0xffffu) == (v20 & 0xffffu) && (v2 & 0xffffu) > lx) {
              link = cx;
              w = v2 >> 16;
            }
            break;
          }
          if (!SM_CHAIN_DEEPLINK || k == kDeepLevels) break;
          const uint4 dr = drec0(t, k);
          if (!(dr.w && dr.x == X && dr.y > X && dr.z <= size)) break;
          ++nd;
          wd += dr.z;  // (<= kDeepLevels * size: no wrap for size < 2^30)
          X = dr.y;
        }
        if (link == t || wd > size) {
          link = t;
          w = wd = nd = 0;
        }
      }
    }
    Esh[t] = e;
    Wsh[t] = w;
    Wdsh[t] = wd;
    Lsh[t] = (uint8_t)nd;
    J[0][t] = (uint16_t)link;
    uint32_t d = link != t ? 1u | ((1u + nd) << 16) : 0u, ss = w + wd, p = link;
    Dsh[t] = d;
    SSsh[t] = ss;
    __syncthreads();
    for (uint32_t r = 1; r <= kLift; ++r) {  // d, ss: over 2^r links; J[r] = J[r-1] o J[r-1]
      const uint32_t dp = Dsh[p], sp = SSsh[p], pn = J[r - 1][p];
      __syncthreads();
      d += dp;  // (both halves: at most kChainNodes each)
      ss = ss + sp < ss ? 0xffffffffu : ss + sp;  // (saturating: a run then ends past `size`, rejected)
      Dsh[t] = d;
      SSsh[t] = ss;
      if (r < kLift) J[r][t] = (uint16_t)pn;
      p = pn;
      __syncthreads();
    }
  }
  auto lift = [&](uint32_t x, uint32_t n) {
#pragma unroll
    for (uint32_t k = 0; k < kLift; ++k)
      if ((n >> k) & 1u) x = J[k][x];
    return x;
  };
  auto put = [&](uint32_t k, const OriginPath& pe) {
    if (k < kChainPath)
      spath[k] = pe;
    else
      path[k] = pe;
  };
  const uint32_t lane = lane_id();
  const bool w0 = t < kWave;
  uint64_t y = ip0, O = 0;
  uint32_t np = 0, bad = 0, cprev = 0xffffffffu;  // the chunk of the previous element
  uint32_t dsrc = 0xffffffffu, dlev = 0;          // the deep record the previous element came from
  while (true) {
    if (w0) {
      uint32_t c1 = kRunDone, out1 = 0;
      while (y < (uint64_t)N - 1) {  // internal.jl:416
        {  // the common step, an entry record in LDS, in a tight 32-bit loop (the general step below
           // takes everything else, and re-checks what ended this loop)
          uint32_t yr = (uint32_t)(y - ip0);
          bool stop = false;
          while (true) {
            const uint32_t c = yr / kC, l = yr % kC;
            if (l >= kIdxEntries || c >= nchunks) break;
            const uint32_t v = uniform(crec(c, l)), d = v & 0xffffu;
            if (v == kRecNone || d <= l || np >= nchunks) break;
            const uint32_t ot = v >> 16, exr = c * kC + d, Oc = (uint32_t)O;  // (O <= size here)
            if (par && (uniform(Dsh[c]) & 0xffffu) >= kMinRun && ip0 + exr == uniform(Esh[c])) {  // a run from here
              c1 = c;
              out1 = ot;
              break;
            }
            const OriginPath pe = {ip0 + yr, ip0 + exr, Oc, ot < 0xffffffffu - Oc ? ot : 0xffffffffu - Oc};
            if (lane == 0) put(np, pe);
            ++np;
            O += ot;
            cprev = c;
            dsrc = 0xffffffffu;
            yr = exr;
            if (O > size || (uint64_t)ip0 + exr >= (uint64_t)N - 1) {
              stop = true;
              break;
            }
          }
          y = ip0 + (uint64_t)yr;
          if (stop || c1 != kRunDone) break;
        }
        const uint32_t c = (uint32_t)((y - ip0) / kC);
        const uint64_t base = ip0 + (uint64_t)c * kC, l = y - base;
        uint64_t ex, ot;
        if (l < kIdxEntries) {
          const uint32_t v = c < nrec ? srec[c * kIdxEntries + l] : kRecNone;
          if (v != kRecNone) {
            ex = base + (v & 0xffffu);
            ot = v >> 16;
          } else {
            const uint2 r = rec[c * kIdxEntries + l];
            ex = uniform(r.x);
            ot = uniform(r.y);
          }
          dsrc = 0xffffffffu;
        } else {
          // candidates, one lane each, read at once: lane 0 the next level of the deep record the
          // previous element came from, lanes 1..kDeepChains level 0 of the previous element's chunk's
          // chains (it left where one of that chunk's entry walks does); the first that starts at y
          // wins, else a walk
          uint32_t idx = 0xffffffffu;
          if (lane == 0 && dsrc != 0xffffffffu && dlev + 1 < kDeepLevels) idx = kDeepLevels * dsrc + dlev + 1;
          if (lane >= 1 && lane <= kDeepChains && cprev != 0xffffffffu) idx = kDeepLevels * (kDeepChains * cprev + lane - 1);
          uint4 dr = make_uint4(0, 0, 0, 0);
          if (idx != 0xffffffffu) dr = idx < ndeep * kDeepChains * kDeepLevels ? sdeep[idx] : deep[idx];
          const uint64_t hit = ballot(dr.w && dr.x == (uint32_t)y && y <= 0xffffffffull);
          if (hit) {
            const uint32_t h = ctz64(hit);
            ex = readlane(dr.y, h);
            ot = readlane(dr.z, h);
            const uint32_t i = readlane(idx, h);
            dsrc = i / kDeepLevels;
            dlev = i % kDeepLevels;
          } else {
            dev_walk<kC>(in, N, y, min(base + kC, (uint64_t)N - 1), jt, lane, stg, ex, ot);
            dsrc = 0xffffffffu;
          }
        }
        cprev = c;
        if (np >= nchunks || ex <= y) {  // (never for a well-formed index: every element leaves its chunk)
          bad = 1;
          break;
        }
        {  // (into LDS: a global store per element made every step wait for the previous one's)
          const uint32_t Oc = O < 0xffffffffull ? (uint32_t)O : 0xffffffffu;
          const uint32_t e32 = ex < 0xffffffffull ? (uint32_t)ex : 0xffffffffu;
          const uint32_t o32 = ot < (uint64_t)(0xffffffffu - Oc) ? (uint32_t)ot : 0xffffffffu - Oc;
          if (lane == 0) put(np, {(uint32_t)y, e32, Oc, o32});
        }
        ++np;
        O += ot;
        y = ex;
        if (O > size) break;
      }
      if (lane == 0) {
        run[0] = c1;
        run[1] = (uint32_t)y;
        run[2] = (uint32_t)O;  // (O <= size when c1 is set)
        run[3] = np;
        run[4] = out1;
      }
    }
    __syncthreads();
    const uint32_t c1 = run[0];
    if (c1 == kRunDone) break;
    {  // every chunk: is it i links along from c1?  Then its element is path element np + (the
       // elements between), followed by its link's deep elements.
      const uint32_t y1 = run[1], O1 = run[2], np1 = run[3], out1 = run[4];
      const uint32_t D1 = Dsh[c1] & 0xffffu, E1 = Dsh[c1] >> 16;
      if (t < nchunks && t >= c1 && (Dsh[t] & 0xffffu) <= D1) {
        const uint32_t i = D1 - (Dsh[t] & 0xffffu), et = np1 + E1 - (Dsh[t] >> 16);
        bool on = false;
        uint32_t Ot = O1, ot = out1;
        if (i == 0) {
          if (t == c1) {
            put(np1, {y1, Esh[c1], O1, out1});
            on = true;
          }
        } else {
          const uint32_t p = lift(c1, i - 1);
          if (J[0][p] == t && p != t) {
            const uint32_t np_ = Lsh[p];
            const uint32_t yt = np_ ? drec0(p, np_ - 1).y : Esh[p];
            Ot = O1 + out1 + SSsh[c1] - SSsh[p] + Wdsh[p];
            ot = Wsh[p];
            put(et, {yt, Esh[t], Ot, ot});
            on = true;
          }
        }
        if (on && J[0][t] != t) {  // (a root's deep elements are the serial chain's)
          uint32_t Ok = Ot + ot;
          for (uint32_t k = 0; k < Lsh[t]; ++k) {
            const uint4 dr = drec0(t, k);
            put(et + 1 + k, {dr.x, dr.y, Ok, dr.z});
            Ok += dr.z;
          }
        }
      }
      if (w0) {  // wave 0 goes on after the run's last element
        const uint32_t root = lift(c1, D1);
        np = np1 + E1 + 1;
        O = (uint64_t)O1 + out1 + SSsh[c1];
        y = Esh[root];
        cprev = root;
        dsrc = 0xffffffffu;
        if (O > size) {  // (the serial chain stops there too; the path is then rejected)
          y = N;
        }
      }
    }
    __syncthreads();  // (run[] is rewritten next round; the run's LDS path elements are in place)
  }
  if (!w0) return;
  if (O != size) bad = 1;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (lane 0's LDS stores before the copy's reads; the runs': barrier)
  for (uint32_t k = lane; k < min(np, kChainPath); k += kWave) path[k] = spath[k];
  if (lane == 0) {
    ctl[0] = np;
    ctl[1] = bad;
  }
  if (lane >= 2 && lane < 4 + nrounds) ctl[lane] = 0;  // the fill's flag and the resolve counters
#undef drec0
}

// k_origin_fill for the device chain's path: elements past ctl[0] exit; a failing element sets ctl[2]
template <uint32_t kC>  // bytes per index chunk
__global__ __launch_bounds__(64) void k_origin_fill_dev(const uint8_t* __restrict__ in, uint32_t N, uint32_t size,
                                                        const OriginPath* path, uint32_t* __restrict__ P,
                                                        uint32_t* ctl) {
  __shared__ __attribute__((aligned(16))) uint16_t jt[kJt];
  __shared__ __attribute__((aligned(16))) uint8_t buf[kC + kIdxPad + 256 + 16];  // an element's tags and a window past them
  const uint32_t npath = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t fail = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (both in flight)
  if (blockIdx.x >= uniform(npath) || uniform(fail)) return;
  const OriginPath pe = path[blockIdx.x];
  stage_bytes(buf, in, N, pe.y, kC + kIdxPad + 256, lane_id());  // (zero past N, as load8z)
  __syncthreads();
  const int32_t st = origin_walk<true>(in, N, size, pe, P, jt, lane_id(), buf, pe.y, kC + kIdxPad + 256);
  if (st != kOk && lane_id() == 0) atomicOr(&ctl[2], 1u);
}

// Pointer jumping with up to `hops` chain steps per pointer per launch: after launch r every
// unresolved pointer has moved >= hops^(r+1) steps, so ceil(log_hops(size)) launches resolve
// all.  One pointer per thread (a pointer's hops are one dependent chain, so more threads hide
// more); a byte is written to out in the launch in which its pointer resolves (the gather folded
// in: a pointer resolved at the start of launch r > 0 was written before).  Launch r > 0 returns
// at once when launch r - 1 left nothing pending (pend[r] counts waves with unresolved pointers
// after launch r).  Launch 0's first thread publishes
// the call's verdict words (ctl[1], ctl[2]); nothing else runs when the chain or a fill failed (P
// is then not all written).  out and words may be device-mapped pinned host memory.
// (hops: kSmallHops, or up to kOneLaunchHops for a stream that small -- one launch then resolves
// every chain, whose length is at most size, without a second launch's dispatch)
__global__ __launch_bounds__(256) void k_small_resolve(const uint8_t* __restrict__ in, uint32_t* P, uint32_t size,
                                                       uint32_t* ctl, uint32_t r, uint32_t last, uint32_t hops,
                                                       uint8_t* __restrict__ out, uint32_t* words) {
  uint32_t* const pend = ctl + 4;
  const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
  // (the three control words in one round trip: later launches usually return here)
  const uint32_t f1 = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t f2 = __hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t pprev = __hip_atomic_load(&pend[r > 0 ? r - 1 : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (r == 0 && t0 == 0) {
    words[0] = f1;
    words[1] = f2;
  }
  if ((f1 | f2) != 0 || (r > 0 && pprev == 0)) return;
  uint32_t left = 0;
  for (uint32_t x = t0; x < size; x += gridDim.x * blockDim.x) {
    uint32_t v = P[x];
    if (v >> 31) {
      if (r == 0) out[x] = in[v & 0x7fffffffu];  // (r > 0: written by an earlier launch)
      continue;
    }
    // v < x: an earlier byte of the chain.  Every few hops the progress is published, so chains
    // through x jump over it (any value a thread stores or reads is a point of the same chain, so
    // stale or racing values are still correct): a run's chain then shrinks by doubling in
    // practice, while `hops` per launch bounds the work the round count assumes.
#pragma unroll 1
    for (uint32_t h = 0; h < hops && !(v >> 31); ++h) {
      v = P[v];
      if ((h & 3) == 3) P[x] = v;
    }
    P[x] = v;
    if (v >> 31)
      out[x] = in[v & 0x7fffffffu];
    else
      ++left;
  }
  const bool any_left = __builtin_amdgcn_ballot_w64(left != 0) != 0;
  if (any_left && lane_id() == 0) atomicAdd(&pend[r], 1u);
  // the last launch: a pointer still unresolved (the round count's bound broken) is reported in the
  // third verdict word (the host zeroes it before the call; every writer writes 1), so the host falls
  // back instead of returning bytes this call never wrote
  if (last && any_left && lane_id() == 0) words[2] = 1u;
}

__global__ __launch_bounds__(256) void k_origin_resolve(uint32_t* P, uint32_t size, uint32_t* pending) {
  uint32_t left = 0;
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < size; x += gridDim.x * blockDim.x) {
    const uint32_t v = P[x];
    if (!(v >> 31)) {
      const uint32_t w = P[v];  // v < x: an earlier byte of the chain
      P[x] = w;
      left += !(w >> 31);
    }
  }
  if (__builtin_amdgcn_ballot_w64(left != 0) && lane_id() == 0) atomicAdd(pending, 1u);
}

__global__ __launch_bounds__(256) void k_origin_gather(const uint8_t* __restrict__ in, const uint32_t* __restrict__ P,
                                                       uint32_t size, uint8_t* __restrict__ out) {
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < size; x += gridDim.x * blockDim.x)
    out[x] = in[P[x] & 0x7fffffffu];
}

// src[0, n) -> dst and nw control words -> words (dst / words: pinned host memory, device-mapped;
// sm_api.hip's upload_input runs it the other way, from mapped host pages into device memory),
// 16 bytes a thread; src and dst 16-byte aligned.
__global__ __launch_bounds__(256) void k_to_host(const uint8_t* __restrict__ src, uint32_t n, uint8_t* __restrict__ dst,
                                                 const uint32_t* wsrc, uint32_t nw, uint32_t* words) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nw) words[t] = wsrc[t];
  const uint32_t n16 = n / 16;
  for (uint32_t i = t; i < n16; i += gridDim.x * blockDim.x)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  if (t < n - 16 * n16) dst[16 * n16 + t] = src[16 * n16 + t];
}

// path 5 (sm_uncompress): the literals of a literal-only stream to their output positions --
// copy_literal! (internal.jl:500-527) for every tag at once.  A thread takes 16 output bytes: one
// literal's bytes as five dword loads and four funnel shifts, one 16-byte store; a unit that
// straddles two literals or the end goes byte by byte.
__global__ __launch_bounds__(256) void k_literal_spans(const uint8_t* __restrict__ in, LitSpans sp,
                                                       uint8_t* __restrict__ out, uint32_t* words) {
  const uint32_t total = sp.dst[sp.n];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) {
    words[0] = total;
    words[1] = 0;  // SM_OK
  }
  for (uint32_t x = 16 * t; x < total; x += 16 * blockDim.x * gridDim.x) {
    uint32_t s = 0;
    for (uint32_t k = 1; k < sp.n; ++k) s = sp.dst[k] <= x ? k : s;
    if (x + 16 <= sp.dst[s + 1]) {
      const uint32_t p = sp.src[s] + (x - sp.dst[s]);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (p & ~3u));
      const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
      *reinterpret_cast<uint4*>(out + x) =
          make_uint4(__builtin_amdgcn_alignbyte(w1, w0, p), __builtin_amdgcn_alignbyte(w2, w1, p),
                     __builtin_amdgcn_alignbyte(w3, w2, p), __builtin_amdgcn_alignbyte(w4, w3, p));
    } else {
      for (uint32_t y = x; y < min(x + 16, total); ++y) {
        while (s + 1 < sp.n && sp.dst[s + 1] <= y) ++s;
        out[y] = in[sp.src[s] + (y - sp.dst[s])];
      }
    }
  }
}

hipError_t launch_literal_spans(const uint8_t* in, const LitSpans& sp, uint8_t* out, uint32_t* words, hipStream_t s) {
  if (sp.n == 0 || sp.n > kLitSpans) return hipErrorInvalidValue;
  const uint32_t units = (sp.dst[sp.n] + 15) / 16;
  const uint32_t grid = min(1024u, max(1u, (units + 255) / 256));
  hipLaunchKernelGGL(k_literal_spans, dim3(grid), dim3(256), 0, s, in, sp, out, words);
  return hipGetLastError();
}

hipError_t launch_to_host(const uint8_t* src, uint32_t n, uint8_t* dst, const uint32_t* wsrc, uint32_t nw,
                          uint32_t* words, hipStream_t s) {
  if (nw > 256) return hipErrorInvalidValue;
  const uint32_t grid = min(1024u, max(1u, (n / 16 + 255) / 256));
  hipLaunchKernelGGL(k_to_host, dim3(grid), dim3(256), 0, s, src, n, dst, wsrc, nw, words);
  return hipGetLastError();
}

hipError_t launch_origin_fill(const uint8_t* in, uint32_t N, uint32_t size, const OriginPath* path, uint32_t npath,
                              uint32_t* P, int32_t* status, hipStream_t s) {
  if (npath == 0) return hipSuccess;
  hipLaunchKernelGGL(k_origin_fill<true>, dim3(npath), dim3(64), 0, s, in, N, size, path, P, status);
  return hipGetLastError();
}

hipError_t launch_path_check(const uint8_t* in, uint32_t N, uint32_t size, const OriginPath* path, uint32_t npath,
                             int32_t* status, hipStream_t s) {
  if (npath == 0) return hipSuccess;
  hipLaunchKernelGGL(k_origin_fill<false>, dim3(npath), dim3(64), 0, s, in, N, size, path, nullptr, status);
  return hipGetLastError();
}

static uint32_t origin_grid(uint32_t size) { return min(8192u, max(1u, (size + 1023) / 1024)); }

hipError_t launch_origin_resolve(uint32_t* P, uint32_t size, uint32_t* pending, hipStream_t s) {
  if (size == 0) return hipSuccess;
  hipLaunchKernelGGL(k_origin_resolve, dim3(origin_grid(size)), dim3(256), 0, s, P, size, pending);
  return hipGetLastError();
}

template <uint32_t kC>
static void launch_small_front(const uint8_t* in, const uint8_t* in_host, uint32_t N, uint32_t ip0, uint32_t size,
                               uint32_t nchunks, uint32_t* rec, OriginPath* path, uint32_t* ctl, uint32_t* P,
                               uint32_t rounds, hipStream_t s) {
  uint4* deep = reinterpret_cast<uint4*>(rec + (size_t)nchunks * kIdxEntries * 2);  // kDeepChains x kDeepLevels per chunk
  // (in_host: the index launch reads the input there and leaves its device copy at in)
  hipLaunchKernelGGL((k_stream_index<kC, true>), dim3(nchunks), dim3(index_threads(true)), 0, s, in_host ? in_host : in,
                     N, ip0, reinterpret_cast<uint2*>(rec), deep, in_host ? const_cast<uint8_t*>(in) : nullptr);
  hipLaunchKernelGGL(k_stream_chain<kC>, dim3(1), dim3(kChainThreads), 0, s, in, N, ip0, size, nchunks,
                     reinterpret_cast<const uint2*>(rec), deep, path, ctl, rounds);
  hipLaunchKernelGGL(k_origin_fill_dev<kC>, dim3(nchunks), dim3(64), 0, s, in, N, size, path, P, ctl);
}

hipError_t launch_small_decode(const uint8_t* in, const uint8_t* in_host, uint32_t N, uint32_t ip0, uint32_t size, uint32_t chunk,
                               uint32_t nchunks, uint32_t* rec, OriginPath* path, uint32_t* ctl, uint32_t* P,
                               uint32_t rounds, uint32_t hops, uint8_t* out, uint32_t* words, hipStream_t s) {
  if (nchunks == 0 || size == 0 || rounds == 0 || 4 + rounds > kWave || hops == 0 || hops > kOneLaunchHops)
    return hipErrorInvalidValue;
  if (chunk == kSmallChunk)
    launch_small_front<kSmallChunk>(in, in_host, N, ip0, size, nchunks, rec, path, ctl, P, rounds, s);
  else if (chunk == kSmallChunkFine)
    launch_small_front<kSmallChunkFine>(in, in_host, N, ip0, size, nchunks, rec, path, ctl, P, rounds, s);
  else if (chunk == kSmallChunkTiny)
    launch_small_front<kSmallChunkTiny>(in, in_host, N, ip0, size, nchunks, rec, path, ctl, P, rounds, s);
  else
    return hipErrorInvalidValue;
  // later launches usually find nothing pending and return at once: a small grid dispatches
  // faster, and strides over the pointers when some are left
  const uint32_t g1 = min(32768u, max(1u, (size + 255) / 256));
  for (uint32_t r = 0; r < rounds; ++r)
    hipLaunchKernelGGL(k_small_resolve, dim3(r == 0 ? g1 : min(g1, 32u)), dim3(256), 0, s, in, P, size, ctl, r,
                       (uint32_t)(r + 1 == rounds), hops, out, words);
  return hipGetLastError();
}

hipError_t launch_origin_gather(const uint8_t* in, const uint32_t* P, uint32_t size, uint8_t* out, hipStream_t s) {
  if (size == 0) return hipSuccess;
  hipLaunchKernelGGL(k_origin_gather, dim3(origin_grid(size)), dim3(256), 0, s, in, P, size, out);
  return hipGetLastError();
}

hipError_t launch_stream_index(const uint8_t* in, uint32_t N, uint32_t ip0, uint32_t nchunks, uint32_t* rec,
                               hipStream_t s) {
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL((k_stream_index<kIdxChunk, false>), dim3(nchunks), dim3(64), 0, s, in, N, ip0,
                     reinterpret_cast<uint2*>(rec), nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_decompress_frags(const uint8_t* in, uint32_t N, uint32_t size, uint8_t* out,
                                   const StreamFrag* frags, uint32_t nfrag, int32_t* status, hipStream_t s) {
  if (nfrag == 0) return hipSuccess;
  hipLaunchKernelGGL(k_decompress_frags, dim3(nfrag), dim3(64), 0, s, in, N, size, out, frags, status);
  return hipGetLastError();
}

hipError_t launch_decompress(const DecompressArgs& a, int /*large*/, hipStream_t s) {
  if (a.nblk == 0) return hipSuccess;
  if (a.one_n && a.nblk == 1)
    hipLaunchKernelGGL(k_decompress_one, dim3(1), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_decompress, dim3(a.nblk), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace sm
