// sm_compress_sc.hip -- fast-mode batched snappy compression for gfx950 (MI355X), round 3:
// super-chunks with a token-passed insert, a wave-parallel verify and a LANE-SERIAL greedy walk.
//
// Output is a valid snappy stream per <= 64 KiB block: it decodes bit-exactly under Snappy.jl's
// uncompress (src/internal.jl:411-466).  It is the reference's greedy parse (internal.jl:127-250)
// with two changes that make it parallel: every position gets its candidates from an in-order
// insert of ALL positions (not only the probed ones), and the block is cut into 1 KiB
// super-chunks whose copies stop at the super-chunk end.
//
// Persistent: one 16-wave workgroup per CU walks its blocks; the block (64 KiB) and a 32 KiB hash
// table live in LDS.  Each of 15 worker waves takes the next super-chunk of the block from an LDS
// counter and:
//  A. hashes its 16 groups of 64 positions (the reference's multiply, internal.jl:94, 13 bits);
//  B. waits for the insert token, then ONE ds_mskor_rtn_b32 per group exchanges the positions into
//     the table and hands the token on.  A table dword holds two u16 slots (position + 1): group
//     parity g & 1 picks the slot a position is written to, and the returned dword gives both
//     candidates at once -- the latest earlier position of the same hash in the own slot (exact:
//     a wave's LDS instructions execute in order, and the conflicting lanes of one instruction in
//     ascending lane order -- observed on gfx950, not an ISA guarantee) and the latest one of the
//     other parity.  Correctness never depends on that order: a candidate is used only when it is
//     an earlier position (C checks c - 1 < q, the one compare a nonzero test costs) and its
//     bytes match; only the ratio depends on it;
//  C. checks both candidates' first 4 bytes and keeps the more recent one that matches, or the
//     older one when the recent one is nearer than SC_FAR (256) bytes and the older matches too
//     (fewer copies that read the decoder's own tag batch): per position its offset (u16, rows of
//     16 positions, swizzled) and the row's match bitmask.  No match length is computed here;
//  D. each LANE walks its row's 16 positions greedily and serially (the reference's loop): at a
//     match position it computes the match length (a 16-byte compare; the walk's last token is
//     extended 16 bytes a step up to 255 bytes), records it, and jumps to the first match at or
//     after the copy's end.  Only the positions a walk visits get a length (about a fifth).  A copy
//     can end inside a later lane's positions, so the walks are resynchronised: every lane starts
//     at its first position; a lane whose true start (the previous lane's end) differs walks from
//     there until it lands on its old path, and keeps the old tokens from that point on; repeated
//     until no start changes;
//  E. literal runs that cross lanes get one tag (segmented by a ballot), token sizes, a DPP scan;
//  F. the wave waits for its staging slot (super-chunk k takes slot k mod 8);
//  G. the lanes or their tokens and literal bytes into the zeroed slot, and
//  W. the writer wave (wave 15) copies the staged super-chunks out in order at the running output
//     offset with aligned 16-byte stores, and writes the block's length.
// Output is deterministic.
#include "sm_device.h"
#include "sm_internal.h"

namespace sm {

constexpr uint32_t kScreenTodoSc = 0xfffffffeu;  // k_literal_screen's "parse this block" mark

constexpr uint32_t kScS = 1024;           // super-chunk bytes
constexpr uint32_t kScC = kScS / 64;      // positions per lane (16)
constexpr uint32_t kScG = kScS / 64;      // 64-position groups per super-chunk (16)
constexpr uint32_t kScW = 16;             // waves per workgroup: kScW - 1 workers and the writer
constexpr uint32_t kScWorkers = kScW - 1;
#ifndef SC_RING
#define SC_RING 16
#endif
// staging slots between the workers and the writer: one per worker and one more, so a worker that
// finishes its super-chunk stages it at once (with 8 slots, the workers 8 or more super-chunks ahead
// of the writer waited for one: half of their wave time in the section stamps, tools/sc_stamps.py)
constexpr uint32_t kScRing = SC_RING;
static_assert((kScRing & (kScRing - 1)) == 0, "the span kernel's slot sequence needs a power of 2");
// bytes per slot: a super-chunk's output is at most 1,040 bytes (1,024 input bytes; every copy tag
// is shorter than its copy, every maximal literal run adds a 1-byte tag, 2 or 3 bytes only for runs
// over 60 bytes, of which at most 15 fit between copies), plus the 20-byte reach of the last piece's
// or and the writer's one-unit read-ahead
constexpr uint32_t kScSlot = 1088;
constexpr uint32_t kScThreads = 64 * kScW;
constexpr uint32_t kScTabBits = 13;       // 8 K dword buckets of two u16 slots
constexpr uint32_t kScTabWords = 1u << kScTabBits;
constexpr uint32_t kScExt = 17;           // length byte: the 16-byte window was full (the walk extends it)
constexpr uint32_t kScMaxL = 255;         // longest copy token (u8 lengths)
#ifndef SC_SPIN_BITS
#define SC_SPIN_BITS 22
#endif
constexpr uint32_t kScSpinMax = 1u << SC_SPIN_BITS;  // hand-off polls (64+ cycles each) before a wait gives up
static_assert(kScC == 16 && kScG == 16, "a lane's 16 positions: one u16 mask, one 16-byte row");

#ifndef SC_CB  // fast mode: section C's groups per batch of candidate loads in flight
#define SC_CB 2
#endif
#ifndef SC_FAR  // fast mode: the older of two matching candidates when the recent one is nearer
#define SC_FAR 256
#endif
constexpr uint32_t kMaskPasses = 16;  // resync passes that may use the covered-lane proposal (the loop)
#ifndef SC_WPRIO
#define SC_WPRIO 3
#endif
#ifndef SC_TPRIO
#define SC_TPRIO 3
#endif
#ifndef SC_TSLEEP  // s_sleep units (64 cycles) between polls of the insert token
#define SC_TSLEEP 1
#endif
#ifndef SC_WSLEEP  // ... and of a staging slot's hand-off words
#define SC_WSLEEP 1
#endif


// per-wave LDS: rows of 16 positions (row r = lane r's positions)
struct ScWaveLds {
  uint8_t L[kScS];   // match length per walked position (4..16; kScExt: extend from 16), rows of 16
                     // bytes, the row's dwords swizzled by (row >> 3) & 3 (conflict-free byte stores)
  uint16_t O[kScS];  // candidate offset per position, rows of 16, dword pairs swizzled by (row >> 2) & 7
};
struct ScLds {
  uint8_t pre[16];                     // (read as the byte before position 0, then replaced by a tag)
  uint8_t blk[kBlockSize + 64];        // the block (+ pad: reads run up to 20 bytes past a position)
  uint32_t T[kScTabWords + 4];         // hash table (two u16 slots a dword); T[kScTabWords] is the dummy for invalid lanes
  ScWaveLds w[kScWorkers];
  uint8_t ring[kScRing][kScSlot];      // staged outputs: super-chunk k in slot k % kScRing
  uint32_t rsize[kScRing];             // the staged super-chunk's output size + 1 (0: slot not staged)
  uint32_t rseq[kScRing];              // the super-chunk a slot takes next (the writer frees it so)
  uint32_t ins;                        // insert token: super-chunks inserted so far
  uint32_t next;                       // the next super-chunk to take
  uint32_t err;                        // a hand-off wait timed out (never expected)
};
static_assert(sizeof(ScLds) <= 160 * 1024, "LDS");
static_assert(sizeof(ScWaveLds) % 32 == 0 && offsetof(ScLds, w) % 32 == 0 && offsetof(ScWaveLds, O) % 32 == 0,
              "rows are 32-byte aligned (section C's O addresses XOR the swizzle into bits 2..4)");
static_assert(kScSlot % 16 == 0 && offsetof(ScLds, ring) % 16 == 0, "slots are 16-byte aligned");
static_assert(kScSlot == kSpanSlot, "the host sizes part pitches by the staging slot");

// wait (bounded) until the LDS word at p satisfies pred; false if the wait gave up
template <typename Pred>
__device__ __attribute__((always_inline)) inline uint32_t sc_wait(uint32_t* p, Pred pred, uint32_t& err, uint32_t code) {
  uint32_t v;
  for (uint32_t it = 0; !pred(v = uniform(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))); ++it) {
    if (it > kScSpinMax) {  // never expected: a broken hand-off must not hang the GPU
      err |= code;
      break;
    }
    if (SC_WSLEEP) __builtin_amdgcn_s_sleep(SC_WSLEEP);
  }
  return v;
}


__device__ inline uint32_t sc_ld32(const uint8_t* blk, uint32_t a) { return *reinterpret_cast<const uint32_t*>(blk + a); }


// (v_alignbyte_b32 shifts by 8 * S2[1:0]: the shift operands below are byte addresses, unmasked --
// a `& 3` costs a VALU the compiler does not drop)
__device__ inline uint32_t sc_abyte(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

// the 4 bytes of the block at p (two aligned dwords, one funnel shift)
__device__ inline uint32_t sc_ld32u(const uint8_t* blk, uint32_t p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(blk + (p & ~3u));
  return sc_abyte(w[1], w[0], p);
}

// 16 bytes of the block at p (five aligned dwords, four funnel shifts)
__device__ inline uint4 sc_ld128(const uint8_t* blk, uint32_t p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(blk + (p & ~3u));
  const uint32_t s = p;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, s), __builtin_amdgcn_alignbyte(w2, w1, s),
                    __builtin_amdgcn_alignbyte(w3, w2, s), __builtin_amdgcn_alignbyte(w4, w3, s));
}

// first differing byte of two 8-byte values given as dword pairs (8: equal)
__device__ inline uint32_t sc_diff8(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
  const uint64_t d = ((uint64_t)(a1 ^ b1) << 32) | (a0 ^ b0);
  return d ? (uint32_t)__builtin_ctzll(d) >> 3 : 8u;
}

// v with the bytes from len (0..16) on cleared
__device__ inline uint4 sc_trim(uint4 v, uint32_t len) {
  const uint64_t mlo = len >= 8 ? ~0ull : (1ull << (8 * (len & 7))) - 1;
  const uint64_t mhi = len >= 16 ? ~0ull : (len <= 8 ? 0ull : (1ull << (8 * (len & 7))) - 1);
  return make_uint4(v.x & (uint32_t)mlo, v.y & (uint32_t)(mlo >> 32), v.z & (uint32_t)mhi, v.w & (uint32_t)(mhi >> 32));
}

// v with the bytes from len (1..16) on cleared, by two 64-bit right shifts of all-ones (the shift
// amounts stay in 0..56 for len >= 1; the high half is dropped by a select when len <= 8)
__device__ inline uint4 sc_trim1(uint4 v, uint32_t len) {
  uint32_t l8 = len << 3;
  asm("" : "+v"(l8));  // (else the compiler folds 128 - 8 len into a quarter-rate multiply by 56)
  uint64_t mlo, mhi;  // (v_lshrrev_b64 of the inline constant -1 reads 6 bits of the amount; len > 8: 0..56;
                      // written out, the compiler splits the halves into four shifts)
  asm("v_lshrrev_b64 %0, %1, -1" : "=v"(mlo) : "v"(64 - min(l8, 64u)));
  asm("v_lshrrev_b64 %0, %1, -1" : "=v"(mhi) : "v"(128 - l8));
  const bool hi = len > 8;
  return make_uint4(v.x & (uint32_t)mlo, v.y & (uint32_t)(mlo >> 32), hi ? v.z & (uint32_t)mhi : 0u,
                    hi ? v.w & (uint32_t)(mhi >> 32) : 0u);
}

// ors the 16 bytes v (zero past the piece) into the zeroed LDS byte array at byte address a (any
// alignment): five ds_or_b32, unconditionally (an or of zeros leaves a neighbour's bytes alone)
__device__ inline void sc_lds_or(uint32_t a, uint4 v) {
  // the five dwords from (a - 1) & ~3: alignbyte(hi, lo, t) = (hi:lo) >> 8 (t & 3) with t = 4 - (a & 3),
  // so an aligned a (t = 0) shifts the whole piece one dword up and or-s a zero below it (no selects)
  const uint32_t wa = (a - 1u) & ~3u, t = 0u - a;
  const uint32_t u0 = __builtin_amdgcn_alignbyte(v.x, 0u, t);
  const uint32_t u1 = __builtin_amdgcn_alignbyte(v.y, v.x, t);
  const uint32_t u2 = __builtin_amdgcn_alignbyte(v.z, v.y, t);
  const uint32_t u3 = __builtin_amdgcn_alignbyte(v.w, v.z, t);
  const uint32_t u4 = __builtin_amdgcn_alignbyte(0u, v.w, t);
  asm volatile("ds_or_b32 %0, %1\nds_or_b32 %0, %2 offset:4\nds_or_b32 %0, %3 offset:8\nds_or_b32 %0, %4 offset:12\n"
               "ds_or_b32 %0, %5 offset:16"
               : : "v"(wa), "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(u4) : "memory");
}

// sc_lds_or for a piece of nb (1..16) bytes: the last three dwords only when the piece reaches
// them (most literal runs are a few bytes: two ds_or_b32 instead of five)
__device__ inline void sc_lds_orn(uint32_t a, uint4 v, uint32_t nb) {
  const uint32_t wa = (a - 1u) & ~3u, t = 0u - a, d = a - wa;  // (d: 1..4, the piece starts in dword 0 or 1)
  const uint32_t u0 = __builtin_amdgcn_alignbyte(v.x, 0u, t);
  const uint32_t u1 = __builtin_amdgcn_alignbyte(v.y, v.x, t);
  asm volatile("ds_or_b32 %0, %1" : : "v"(wa), "v"(u0) : "memory");
  asm volatile("ds_or_b32 %0, %1 offset:4" : : "v"(wa), "v"(u1) : "memory");
  if (d + nb > 8) {
    const uint32_t u2 = __builtin_amdgcn_alignbyte(v.z, v.y, t);
    const uint32_t u3 = __builtin_amdgcn_alignbyte(v.w, v.z, t);
    const uint32_t u4 = __builtin_amdgcn_alignbyte(0u, v.w, t);
    asm volatile("ds_or_b32 %0, %1 offset:8\nds_or_b32 %0, %2 offset:12\nds_or_b32 %0, %3 offset:16"
                 : : "v"(wa), "v"(u2), "v"(u3), "v"(u4) : "memory");
  }
}

// ors the (up to 3) bytes of cv into the zeroed LDS byte array at byte address a
__device__ inline void sc_lds_or3(uint32_t a, uint32_t cv, uint32_t cs = 3) {
  const uint32_t wa = (a - 1u) & ~3u, t = 0u - a;  // (as sc_lds_or)
  const uint32_t lo = __builtin_amdgcn_alignbyte(cv, 0u, t), hi = __builtin_amdgcn_alignbyte(0u, cv, t);
  asm volatile("ds_or_b32 %0, %1\nds_or_b32 %0, %2 offset:4" : : "v"(wa), "v"(lo), "v"(hi) : "memory");
}

// v shifted up by t (0..3) bytes with the t-byte value tag below it
__device__ inline uint4 sc_prepend(uint4 v, uint32_t tag, uint32_t t) {
  if (t == 0) return v;
  const uint32_t s = 4 - t;  // alignbyte(hi, lo, s) = (hi:lo) >> 8s
  return make_uint4(__builtin_amdgcn_alignbyte(v.x, tag << (8 * s), s), __builtin_amdgcn_alignbyte(v.y, v.x, s),
                    __builtin_amdgcn_alignbyte(v.z, v.y, s), __builtin_amdgcn_alignbyte(v.w, v.z, s));
}

// emit_literal! tag (internal.jl:271-284) for a run of len >= 1 bytes, and its size
__device__ inline uint32_t sc_lit_tag(uint32_t len, uint32_t& sz) {
  const uint32_t l1 = len - 1;
  sz = len <= 60 ? 1u : (len <= 256 ? 2u : 3u);
  return sz == 1 ? (l1 << 2) : (sz == 2 ? (60u << 2) | (l1 << 8) : (61u << 2) | (l1 << 8));
}

// the bucket of a word: the reference's multiply (internal.jl:94), its top kScTabBits bits, as one
// v_bfe_u32 (the compiler's shift + mask + add of the bucket address is one VALU more)
__device__ inline uint32_t sc_hash_bucket(uint32_t w) {
  uint32_t h;
  asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(h) : "v"(w * kHashMul), "n"(32 - kScTabBits), "n"(kScTabBits));
  return h;
}

// lane l: bit l of the lane mask m ? a : b (one v_cndmask on the SGPR pair)
__device__ inline uint32_t sc_select(uint64_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}

// c ? a : b on values (a conditional on lvalues can become a select of their addresses)
__device__ inline uint32_t sc_sel(uint32_t c, uint32_t a, uint32_t b) { return c ? a : b; }

// one emit_copy_upto_64! piece (internal.jl:289-304), L in 4..64: copy-1 or copy-2, and its size
__device__ inline uint32_t sc_copy_piece(uint32_t off, uint32_t L, uint32_t& sz) {
  const bool c1 = L < 12 && off < 2048;
  sz = c1 ? 2u : 3u;
  // (both encodings, then a select: the compiler otherwise branches on c1)
  const uint32_t e1 = (1u + ((L - 4) << 2) + ((off >> 3) & 0xe0u)) | ((off & 0xffu) << 8);
  const uint32_t e2 = (2u + ((L - 1) << 2)) | (off << 8);
  return sc_sel(c1, e1, e2);
}

__device__ inline uint32_t sc_extend(const uint8_t* blk, uint32_t q, uint32_t off, uint32_t L, uint32_t cap) {
  for (;;) {
    const uint4 x = sc_ld128(blk, q + L), y = sc_ld128(blk, q + L - off);
    const uint32_t f0 = sc_diff8(x.x, x.y, y.x, y.y);
    const uint32_t fb = f0 < 8 ? f0 : 8u + sc_diff8(x.z, x.w, y.z, y.w);
    L = min(L + fb, cap);
    if (fb < 16 || L >= cap) return L;
  }
}

// copy_tag_bytes (emit_copy!, internal.jl:306-329) for 4 <= L <= 255 in closed form.  emit_copy!
// cuts 64-byte pieces while L >= 68, a 60-byte piece if more than 64 remain, then the last piece R:
// (L - 1) >> 6 three-byte pieces before the last, and R < 12 exactly when ((L - 1) & 63) < 11
// (R = m + 4 for m = ((L - 1) & 63) + 1 < 4, else m) -- checked for every L and both offset
// classes against the loop (tests/test_host_logic.py); no multiply (3 n as n + 2 n)
__device__ inline uint32_t sc_copy_bytes(uint32_t off, uint32_t L) {
  const uint32_t t = L - 1, n = t >> 6;
  return n + 2 * n + (((t & 63) < 11 && off < 2048) ? 2u : 3u);
}

// lowest set bit of x, ~0 for 0 (v_ffbl_b32)
__device__ inline uint32_t sc_ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));  // (the compiler does not know ffbl(0) = ~0)
  return r;
}

// equal leading bytes (0..16) of the 16 bytes X0..X3 and the 16 bytes at w + (s & 3) (w dword-aligned LDS)
__device__ __attribute__((always_inline)) inline uint32_t sc_eq16(uint32_t X0, uint32_t X1, uint32_t X2, uint32_t X3,
                                                                  const uint32_t* w, uint32_t s) {
  const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4];
  // first differing bit (ffbl(0) = ~0 survives the | and loses the min)
  const uint32_t b0 = sc_ffbl(X0 ^ __builtin_amdgcn_alignbyte(a1, a0, s));
  const uint32_t b1 = sc_ffbl(X1 ^ __builtin_amdgcn_alignbyte(a2, a1, s)) | 32u;
  const uint32_t b2 = sc_ffbl(X2 ^ __builtin_amdgcn_alignbyte(a3, a2, s)) | 64u;
  const uint32_t b3 = sc_ffbl(X3 ^ __builtin_amdgcn_alignbyte(a4, a3, s)) | 96u;
  return min(min(b0, b1), min(min(b2, b3), 128u)) >> 3;
}


// 13 when the 12 bytes at x and at y of the LDS array blk are equal, else their equal leading
// bytes (0..11): the walk's length code, 4 + this = 4..15 or kScExt (blk: 4-byte aligned)
__device__ __attribute__((always_inline)) inline uint32_t sc_eq12x(const uint8_t* blk, uint32_t x, uint32_t y) {
  const uint32_t* a = reinterpret_cast<const uint32_t*>(blk + (x & ~3u));
  const uint32_t* b = reinterpret_cast<const uint32_t*>(blk + (y & ~3u));
  const uint32_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
  const uint32_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
  const uint32_t f0 = sc_ffbl(sc_abyte(a1, a0, x) ^ sc_abyte(b1, b0, y));
  const uint32_t f1 = sc_ffbl(sc_abyte(a2, a1, x) ^ sc_abyte(b2, b1, y)) | 32u;
  const uint32_t f2 = sc_ffbl(sc_abyte(a3, a2, x) ^ sc_abyte(b3, b2, y)) | 64u;
  return min(min(f0, f1), min(f2, 104u)) >> 3;
}

// inclusive wave-64 max-scan with DPP (scan_dpp's pattern; 0 is the identity for these values)
__device__ inline uint32_t scan_max_dpp(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
  return v;
}

// bits [a, b) of a u32 (0 <= a <= b <= 31)
__device__ inline uint32_t sc_bits(uint32_t a, uint32_t b) { return ((1u << b) - 1u) & ~((1u << a) - 1u); }

// a lane's tokens: the copies of its walk (at most 4 in 16 positions), offset | length << 16 |
// position-in-row << 24, in position order
struct ScToks {
  uint32_t t[4];
  uint32_t n;
};

// The next block at or after `from` (stride gridDim.x) that the screen left for the parse, or nblk
// (wave-uniform; 64 candidates per step)
__device__ __attribute__((always_inline)) inline uint32_t sc_next_block(const CompressArgs& a, uint32_t from, uint32_t lane) {
  for (uint32_t b0 = from; b0 < a.nblk; b0 += 64 * gridDim.x) {
    const uint32_t bb = b0 + lane * gridDim.x;
    const bool todo = bb < a.nblk && (!a.screened || a.out_len[bb] == kScreenTodoSc);
    const uint64_t m = ballot(todo);
    if (m) return b0 + ctz64(m) * gridDim.x;
  }
  return a.nblk;
}

// One super-chunk, by one wave (sections A-G2 above).
template <int kDense>
__device__ __attribute__((always_inline)) inline void sc_superchunk(ScLds& S, const uint32_t k, const uint32_t n,
                                                                   const uint32_t wave, const uint32_t lane_in) {
  // (the lane index laundered per super-chunk: otherwise the compiler hoists dozens of lane-derived
  // addresses out of the super-chunk loop, and the registers they hold serialise section C)
  uint32_t lane = lane_in;
  asm volatile("" : "+v"(lane));
  ScWaveLds& Wl = S.w[wave];
  const uint32_t sc0 = k * kScS, sce = min(sc0 + kScS, n);
  const uint32_t Tbase = lds_addr(S.T);
  // ---- A. hashes of the 16 groups: LDS byte address of the bucket dword, the slot value ----
  // (group g's position is ql + 64 g: its dword address and byte shift are ql's plus a constant,
  // so the loads take immediate offsets; only the block's last super-chunk has positions whose 4
  // bytes run past the block, and only it checks them)
  uint32_t ha[kScG], hvv[kScG], wq[kScG];
  const uint32_t ql = sc0 + lane, qa = ql & ~3u, qb = ql;
  // (slots hold positions: a never-written slot reads as candidate 0, which the reference's table
  // gives too, Snappy.jl:30 -- a real candidate, verified like any other)
  const uint32_t hv0 = ql, hv1 = ql << 16;
#pragma unroll
  for (int g = 0; g < (int)kScG; ++g) {
    const uint32_t w = sc_abyte(sc_ld32(S.blk, qa + 64 * g + 4), sc_ld32(S.blk, qa + 64 * g), qb);
    wq[g] = w;
    ha[g] = Tbase + 4 * sc_hash_bucket(w);
    hvv[g] = (g & 1) ? hv1 + ((64u * g) << 16) : hv0 + 64u * g;
  }
  if (sc0 + kScS + 3 > n) {  // (uniform) positions without 4 bytes exchange into the dummy word
    asm volatile("");         // (a real branch: the selects are not speculated into every super-chunk)
#pragma unroll
    for (int g = 0; g < (int)kScG; ++g) ha[g] = ql + 64 * g + 4 <= n ? ha[g] : Tbase + 4 * kScTabWords;
  }
  const uint32_t mk0 = 0xffffu, mk1 = 0xffff0000u;
  // ---- B. the insert token: 16 masked exchanges in position order, then hand it on ----
  __builtin_amdgcn_s_setprio(SC_TPRIO);
  for (uint32_t it = 0; uniform(__hip_atomic_load(&S.ins, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != k; ++it) {
    if (it > kScSpinMax) {  // never expected: a broken hand-off must not hang the GPU
      S.err |= 1;  // (the insert token)
      break;
    }
    if (SC_TSLEEP) __builtin_amdgcn_s_sleep(SC_TSLEEP);
  }
  __builtin_amdgcn_s_setprio(3);
  const uint32_t tok_a = lds_addr(&S.ins), tok_v = k + 1;
  uint32_t r[kScG];
  asm volatile(
      "ds_mskor_rtn_b32 %0, %16, %32, %34\n"
      "ds_mskor_rtn_b32 %1, %17, %33, %35\n"
      "ds_mskor_rtn_b32 %2, %18, %32, %36\n"
      "ds_mskor_rtn_b32 %3, %19, %33, %37\n"
      "ds_mskor_rtn_b32 %4, %20, %32, %38\n"
      "ds_mskor_rtn_b32 %5, %21, %33, %39\n"
      "ds_mskor_rtn_b32 %6, %22, %32, %40\n"
      "ds_mskor_rtn_b32 %7, %23, %33, %41\n"
      "ds_mskor_rtn_b32 %8, %24, %32, %42\n"
      "ds_mskor_rtn_b32 %9, %25, %33, %43\n"
      "ds_mskor_rtn_b32 %10, %26, %32, %44\n"
      "ds_mskor_rtn_b32 %11, %27, %33, %45\n"
      "ds_mskor_rtn_b32 %12, %28, %32, %46\n"
      "ds_mskor_rtn_b32 %13, %29, %33, %47\n"
      "ds_mskor_rtn_b32 %14, %30, %32, %48\n"
      "ds_mskor_rtn_b32 %15, %31, %33, %49\n"
      "ds_write_b32 %50, %51\n"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]),
        "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
      : "v"(ha[0]), "v"(ha[1]), "v"(ha[2]), "v"(ha[3]), "v"(ha[4]), "v"(ha[5]), "v"(ha[6]), "v"(ha[7]), "v"(ha[8]),
        "v"(ha[9]), "v"(ha[10]), "v"(ha[11]), "v"(ha[12]), "v"(ha[13]), "v"(ha[14]), "v"(ha[15]), "v"(mk0), "v"(mk1),
        "v"(hvv[0]), "v"(hvv[1]), "v"(hvv[2]), "v"(hvv[3]), "v"(hvv[4]), "v"(hvv[5]), "v"(hvv[6]), "v"(hvv[7]),
        "v"(hvv[8]), "v"(hvv[9]), "v"(hvv[10]), "v"(hvv[11]), "v"(hvv[12]), "v"(hvv[13]), "v"(hvv[14]), "v"(hvv[15]),
        "v"(tok_a), "v"(tok_v)
      : "memory");
  __builtin_amdgcn_s_setprio(0);

  // ---- C. one candidate per position: the latest earlier position of the same hash (own slot or
  // the other's, the more recent first) whose first 4 bytes equal the position's.  Only its offset
  // is stored (row-major, swizzled); match lengths are computed by the walks (D), and only at the
  // positions a walk visits.  (Choosing the longer of the two by an 8-byte compare instead gives
  // ratio 0.5625 against 0.5738 on the bench text, but 3.21 against 2.96 ms, and a round trip
  // 3.6% slower: DESIGN.md section 3.2d.) ----
  uint64_t mbs[kScG];
  // a position's O entry: row r4 = 4 g + (lane >> 4), entry i = lane & 15, at u16 index 16 r4 + (i ^ 2 (g & 7))
  // (dword pairs swizzled by the group): byte offset (Orel ^ 4 (g & 7)) + 128 g, Orel = the entry's
  // unswizzled offset in group 0 (bits 2..4 are 2 i's) -- one XOR a group, 128 g an immediate offset
  uint8_t* const Ob8 = reinterpret_cast<uint8_t*>(Wl.O);
  const uint32_t Orel = 32 * (lane >> 4) + 2 * (lane & 15);
  // A candidate is valid when it is an earlier position: c < q.  The table is cleared per block and
  // filled in position order, so every slot value is an earlier position whenever the conflicting
  // lanes of one ds_mskor_rtn are serviced in ascending lane order (observed on gfx950); the compare
  // makes validity independent of that order.  c2 <= c1: when c1 is valid so is
  // c2; when it is not -- the order broke -- both are dropped.  Positions without 4 bytes before the
  // block end exchanged with the dummy word, and positions without 4 bytes before the super-chunk
  // end may not start a copy: the walks' row masks leave both out (D), so no per-group check here.
  // (A candidate's loads read inside the block copy whatever its value: c < 65536.)
  if constexpr (kDense) {
#pragma unroll
    for (int g = 0; g < (int)kScG; ++g) {
      const uint32_t q = sc0 + 64 * g + lane;
      const uint32_t sh = 16 * (g & 1);
      const uint32_t ca = (r[g] >> sh) & 0xffffu, cb = (r[g] >> (16 - sh)) & 0xffffu;  // positions
      const uint32_t c1 = max(ca, cb), c2 = min(ca, cb);
      const bool ok1 = c1 < q;
      const uint32_t d1 = q - c1, d2 = q - c2;  // the offsets
      uint16_t* const Og = reinterpret_cast<uint16_t*>(Ob8 + (Orel ^ (4u * (g & 7))) + 128u * g);
      const uint32_t r4 = 4 * g + (lane >> 4), i = lane & 15;  // row, entry
      // dense mode: both candidates compared over 16 bytes, the longer kept, its length stored
      // for the walks; on a tie the SC_FAR rule below (the older when the more recent is near)
      const uint4 X = sc_ld128(S.blk, q);
      uint32_t lw1 = sc_eq16(X.x, X.y, X.z, X.w, reinterpret_cast<const uint32_t*>(S.blk + (c1 & ~3u)), c1);
      uint32_t lw2 = sc_eq16(X.x, X.y, X.z, X.w, reinterpret_cast<const uint32_t*>(S.blk + (c2 & ~3u)), c2);
      asm("" : "+v"(lw1), "+v"(lw2));  // (keeps the loads unconditional)
      const uint32_t l1 = ok1 ? lw1 : 0u, l2 = ok1 ? lw2 : 0u;
      const bool take2 = l2 == l1 ? (l2 >= 4 && d1 < (uint32_t)SC_FAR) : l2 > l1;
      const uint32_t l = take2 ? l2 : l1;
      const uint32_t avail = sce - q;  // (>= 4 where l >= 4: room)
      const uint32_t enc = l < 4 ? 0u : ((l == 16 && avail > 16) ? kScExt : min(l, avail));
      *Og = (uint16_t)(take2 ? d2 : d1);
      Wl.L[16 * r4 + 4 * ((i >> 2) ^ ((g >> 1) & 3)) + (i & 3)] = (uint8_t)enc;
      mbs[g] = ballot(l >= 4);
    }
  } else {
    // fast mode: SC_CB groups at a time, all their candidate loads issued before any is waited for
#pragma unroll
    for (int g0 = 0; g0 < (int)kScG; g0 += SC_CB) {
      uint32_t c1s[SC_CB], c2s[SC_CB], v1s[SC_CB], v2s[SC_CB];
#pragma unroll
      for (int j = 0; j < SC_CB; ++j) {
        const int g = g0 + j;
        const uint32_t sh = 16 * (g & 1);
        const uint32_t ca = (r[g] >> sh) & 0xffffu, cb = (r[g] >> (16 - sh)) & 0xffffu;  // positions
        c1s[j] = max(ca, cb);
        c2s[j] = min(ca, cb);
        v1s[j] = sc_ld32u(S.blk, c1s[j]);
        v2s[j] = sc_ld32u(S.blk, c2s[j]);
      }
#pragma unroll
      for (int j = 0; j < SC_CB; ++j) asm("" : "+v"(v1s[j]), "+v"(v2s[j]));  // (keeps the loads unconditional)
#pragma unroll
      for (int j = 0; j < SC_CB; ++j) {
        const int g = g0 + j;
        const uint32_t q = sc0 + 64 * g + lane;
        const uint32_t c1 = c1s[j], c2 = c2s[j], w = wq[g];
        const bool ok1 = c1 < q;
        const uint32_t d1 = q - c1, d2 = q - c2;  // the offsets
        uint16_t* const Og = reinterpret_cast<uint16_t*>(Ob8 + (Orel ^ (4u * (g & 7))) + 128u * g);
        // the matches as lane masks (ballots of plain compares, combined by SALU: a ballot of an
        // and-ed bool costs a v_cndmask + v_cmp, and a select on a combined bool two v_cndmask)
        const uint64_t OK = ballot(ok1);
        const uint64_t M1 = ballot(v1s[j] == w) & OK, M2 = ballot(v2s[j] == w) & OK;
        // the older candidate when the more recent one is nearer than SC_FAR bytes: a copy whose
        // source is that close often reads the output of the decoder's own batch of tags, which
        // then runs it in order ("Candidates for the decoder")
        const uint64_t U = M2 & (~M1 | ballot(d1 < (uint32_t)SC_FAR));
        *Og = (uint16_t)sc_select(U, d2, d1);  // (a position without a match: never read)
        mbs[g] = M1 | M2;
      }
    }
  }
  // the row masks: lane d holds dword d of the 16 group ballots (v_writelane), lane l reads its
  // row's 16 bits from lane l / 2 (one ds_bpermute; no LDS array, no single-lane stores)
  uint32_t mdw = 0;
#define SC_WL(g)                                                                                  \
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(mdw) : "s"((uint32_t)mbs[g]), "n"(2 * (g)));   \
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(mdw) : "s"((uint32_t)(mbs[g] >> 32)), "n"(2 * (g) + 1));
  SC_WL(0) SC_WL(1) SC_WL(2) SC_WL(3) SC_WL(4) SC_WL(5) SC_WL(6) SC_WL(7)
  SC_WL(8) SC_WL(9) SC_WL(10) SC_WL(11) SC_WL(12) SC_WL(13) SC_WL(14) SC_WL(15)
#undef SC_WL
  __atomic_signal_fence(__ATOMIC_SEQ_CST);

  // ---- D. lane-serial walks over the row, resynchronised ----
  // A lane walks its row greedily: at a match position it computes the match length (16-byte
  // compare; kScExt: the 16 bytes were equal, the walk's last token is extended), records it, and
  // jumps to the first match position at or after the copy's end (the row's match bitmask).
  const uint32_t c0 = sc0 + kScC * lane;
  const uint32_t ce = c0 < sce ? min(c0 + kScC, sce) : c0;
  // (a match may cover 4 bytes before the super-chunk end: positions c0 + i with c0 + i + 4 <= sce)
  const uint32_t nroom = c0 + 3 < sce ? min(sce - c0 - 3, 16u) : 0u;
  const uint32_t mask16 = (__shfl(mdw, (int)(lane >> 1), 64) >> (16 * (lane & 1))) & ((1u << nroom) - 1u);
  // the row's swizzles as index XORs: entry i of the row is u16 i ^ osw2 of the O row and byte
  // i ^ lsw4 of the L row (2 ((i >> 1) ^ osw) + (i & 1) = i ^ 2 osw; likewise for L)
  const uint32_t osw2 = ((lane >> 2) & 7) << 1, lsw4 = ((lane >> 3) & 3) << 2;
  const uint16_t* const Orow = Wl.O + 16 * lane;
  auto offAt = [&](uint32_t i) -> uint32_t { return Orow[i ^ osw2]; };
  uint8_t* const Lrow = Wl.L + 16 * lane;
  // the last token's extended length (one per lane: resync walks often end on the same token)
  uint32_t xpos = 16, xlen = 0;
  // Walk from row position sr (16: none) until the walk leaves the row or lands on a token of
  // `stop` (kStop; the first walk has none): the token bits, the merge position (16: none), the
  // lane's end position.  A divergent loop: a lane leaves it when its walk ends (the next match
  // position is past the row), so no values are carried through an exec-masked region; every
  // iteration moves i forward by >= 4, so each lane leaves within 4 iterations.
  auto walk = [&](auto kStop, uint32_t sr, uint32_t stop, uint32_t& path, uint32_t& mpos, uint32_t& pend)
      __attribute__((always_inline)) {
    const uint32_t m0 = sr < 16 ? mask16 >> sr : 0u;
    uint32_t i = sr + sc_ffbl(m0);  // (m0 == 0: no walk)
    path = 0;
    mpos = 16;
    uint32_t last = 16, lastL = 0;
    bool act = m0 != 0;
    while (act) {
      if constexpr (decltype(kStop)::value) {
        if ((stop >> i) & 1u) {
          mpos = i;
          break;
        }
      }
      path |= 1u << i;
      last = i;
      uint32_t enc;
      if constexpr (kDense) {
        enc = Lrow[i ^ lsw4];  // (computed in C)
      } else {
        const uint32_t q = c0 + i, off = offAt(i);
        const uint32_t p = q - off;
        // the match length over 16 bytes: the first 4 are equal (the candidate check, C), so bytes
        // [4, 16) of both sides decide it: 4 + the equal leading bytes of 12, or kScExt (17) when
        // all 12 are equal (the min's cap 104 >> 3 = 13); then capped at the super-chunk end
        // (all 16 equal and more than 16 bytes left: kScExt, the walk's last token is extended)
        enc = min(4u + sc_eq12x(S.blk + 4, q, p), sce - q);  // (blk + 4: the +4 in the loads' offsets)
        Lrow[i ^ lsw4] = (uint8_t)enc;
      }
      lastL = enc;
      const uint32_t t = i + min(enc, 16u);  // <= 31: mask16 >> t is 0 past the row
      const uint32_t m = mask16 >> t;
      i = t + sc_ffbl(m);
      act = m != 0;
    }
    // the end: the last token's end when it leaves the row, else the row end (literals follow)
    pend = ce;
    if (last < 16) {
      uint32_t L = lastL;
      const bool ext = L == kScExt;
      if (last + min(L, 16u) >= 16) {
        if (ballot(ext)) {
          if (ext) {
            if (xpos != last) {
              xlen = sc_extend(S.blk, c0 + last, offAt(last), 16u, min(kScMaxL, sce - (c0 + last)));
              xpos = last;
            }
            L = xlen;
          }
        }
        pend = c0 + last + L;
      }
    }
  };
  const bool row = c0 < sce;  // the lane has positions
  uint32_t s = c0, e, P;
  {
    uint32_t mp;
    walk(std::false_type{}, row ? 0u : 16u, 0u, P, mp, e);
    if (!row) e = c0;
  }
  for (uint32_t pass = 0;; ++pass) {
    // every lane's start: the furthest end of the lanes before it (an exclusive max-scan), not only
    // the previous lane's -- a copy that covers several rows reaches every covered lane in one round
    // instead of one lane a round.  The fixed point is the same (ends are non-decreasing there, so
    // the max is the previous lane's end), so are the bytes; config 5's corpus 2.478 -> 2.367 ms,
    // the bench text unchanged
    const uint32_t pe = __builtin_amdgcn_update_dpp(0u, scan_max_dpp(e), 0x138, 0xf, 0xf, false);  // wave_shr:1
    const uint32_t st = lane == 0 ? sc0 : pe;
    uint32_t sn = st;
    // A lane whose start is past its row is covered: it forwards that start, and its own end (from
    // an earlier walk) is stale.  Stale ends only overestimate, and fed to the scan they push every
    // later lane too far, so data of long matches corrected one row a pass (geo.protodata 13.8
    // passes a super-chunk, a 427-byte period 50).  The proposal leaves covered lanes out of the
    // scan (a few cheap scans, until the covered set is stable).  The loop still ends only where
    // the plain scan agrees (the unique fixed point: the bytes are unchanged), takes the plain
    // scan's starts whenever the proposal changes nothing, and after kMaskPasses passes uses the
    // plain rule alone (which settles lane k by pass k + 1).  Same bytes on every corpus file and
    // the bench sets (tools/ab_bytes.py); config 5's fragments 2.369 -> 2.258 ms, geo.protodata
    // 2,000 windows 0.750 -> 0.584, the bench text 2.020 -> 2.033 (the proposal after the plain
    // fixed-point test, so the last pass does not pay for it: profiles/r06_ab_experiments.txt)
    bool chg = st != s;
    if (!ballot(chg)) break;  // the fixed point of the plain rule
    if (pass < kMaskPasses) {
      uint64_t cov = ballot(st >= ce);
      for (int it = 0; cov && it < 3; ++it) {
        const uint32_t x = sn >= ce ? 0u : e;
        const uint32_t pm = __builtin_amdgcn_update_dpp(0u, scan_max_dpp(x), 0x138, 0xf, 0xf, false);
        sn = lane == 0 ? sc0 : pm;
        const uint64_t c = ballot(sn >= ce);
        if (c == cov) break;
        cov = c;
      }
      chg = sn != s;
      if (!ballot(chg)) {  // (the proposal changes nothing: the plain rule's starts this pass)
        sn = st;
        chg = st != s;
      }
    }

    const bool inrow = chg && sn < ce;  // (an entry is never before the row)
    uint32_t nP, mp, ne;
    walk(std::true_type{}, inrow ? sn - c0 : 16u, P, nP, mp, ne);  // (rows not walking: stop at once)
    if (chg) {
      s = sn;
      if (!inrow) {  // past the row (a copy jumped over it) or a lane without positions
        P = 0;
        e = sn;
      } else if (mp == 16) {
        P = nP;
        e = ne;
      } else {  // the new tokens, then the old ones from the merge position on (e unchanged)
        P = nP | (P & ~sc_bits(0, mp));
      }
    }
  }
  // the lengths the walks recorded (every token of P has one), read back per token
  auto getL = [&](uint32_t i) -> uint32_t { return Lrow[i ^ lsw4]; };
  // the lane's tokens from its token bits: offset | length << 16 | position-in-row << 24
  ScToks tk;
  {
    uint32_t pm = P;
    tk.n = (uint32_t)__builtin_popcount(P);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = pm ? (uint32_t)__builtin_ctz(pm) : 0u;
      pm &= pm - 1;
      uint32_t L = getL(i);
      L = L == kScExt ? xlen : L;  // (only the last token can be an extended one, and it was)
      const uint32_t off = offAt(i);
      tk.t[j] = off | (L << 16) | (i << 24);
    }
  }

  // ---- E. the lane's summary, literal runs across lanes, sizes, offsets ----
  // lead: the first literal run; trail: the last one when the row ends on literals (no copies:
  // lead == trail); body: every other byte of the lane's output
  const bool live = s >= c0 && s < ce;
  uint32_t lead = 0, body = 0, trail = 0;
  {  // (selects, no branches: every lane runs all four token slots)
    uint32_t p = s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool has = (uint32_t)j < tk.n;
      const uint32_t tv = tk.t[j];
      const uint32_t q = c0 + (tv >> 24), L = (tv >> 16) & 0xffu, run = q - p;
      if (j == 0)
        lead = sc_sel(has, run, 0u);
      else
        body += sc_sel(has && run, run + 1, 0u);  // an internal run (< 16 bytes: a one-byte tag)
      body += sc_sel(has, sc_copy_bytes(tv & 0xffffu, L), 0u);
      p = sc_sel(has, q + L, p);
    }
    trail = (live && p < ce) ? ce - p : 0u;
    lead = tk.n == 0 ? trail : lead;
  }
  const uint32_t ptrail = __builtin_amdgcn_update_dpp(0u, trail, 0x138, 0xf, 0xf, false);  // wave_shr:1 (lane 0: 0)
  const bool cont = ptrail > 0 && lead > 0;  // this lane's first run continues the previous lane's last one
  const bool mid = cont && tk.n == 0;         // ... and is all the lane has: the run goes on
  const uint32_t Cs = scan_dpp(cont ? lead : 0u);
  // fn: the first lane after this one where a run stops passing through (63 if none)
  const uint64_t above = ballot(!mid) & (~1ull << lane);
  const uint32_t fn = above ? ctz64(above) : 63u;
  const uint32_t Cf = __shfl(Cs, fn, 64);
  const bool starts = trail > 0 && !mid;
  const uint32_t merged = starts ? trail + Cf - Cs : 0u;  // the run this lane's last run starts
  uint32_t mts;
  (void)sc_lit_tag(merged ? merged : 1u, mts);
  uint32_t size;
  if (tk.n == 0)
    size = lead == 0 ? 0u : (cont ? lead : mts + trail);
  else
    size = (lead ? (cont ? lead : 1u + lead) : 0u) + body + (trail ? mts + trail : 0u);
  const uint32_t incl = scan_dpp(size);
  const uint32_t total = readlane(incl, 63);

  // ---- F. a staging slot: super-chunk k takes slot k % kScRing once the writer has written
  // super-chunk k - kScRing out of it ----
  const uint32_t slot = k % kScRing;
  (void)sc_wait(&S.rseq[slot], [&](uint32_t v) { return v == k; }, S.err, 2u);

  // ---- G. the lanes' tokens into the slot, then the slot to the writer ----
  uint8_t* const stg = S.ring[slot];
  {
    // the output bytes are or-ed into a zeroed slot: no masks, no branches per piece (the zeroes
    // land first: a wave's LDS operations execute in order)
    for (uint32_t u = lane; 16 * u < total; u += 64) reinterpret_cast<uint4*>(stg)[u] = make_uint4(0, 0, 0, 0);
    const uint32_t stga = lds_addr(stg);
    uint32_t at = incl - size, p = s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if ((uint32_t)j < tk.n) {
        const uint32_t tv = tk.t[j];
        const uint32_t q = c0 + (tv >> 24), L = (tv >> 16) & 0xffu, off = tv & 0xffffu;
        const uint32_t run = q - p;  // < 16
        const uint32_t ts = (j == 0 && cont) ? 0u : 1u;
        const uint32_t len = run ? ts + run : 0u;
        if (ballot(len != 0)) {  // (uniform: skipped when no lane has a run before this token)
          // the run with the byte before it: the tag replaces that byte (ts = 1), or (ts = 0: the
          // run continues the previous lane's, which ends on that very byte) it is or-ed again
          // onto itself one byte early -- no prepend shifts
          uint4 v = sc_ld128(S.blk - 4, p + 3);  // bytes from position p - 1
          v.x = ts ? ((v.x & ~0xffu) | ((run - 1) << 2)) : v.x;
          // (lanes without a run write nothing: a shared dummy address serialises the atomics)
          if (run) sc_lds_orn(stga + at + ts - 1u, sc_trim1(v, run + 1), run + 1);
        }
        at += len;
        if (L <= 64) {
          uint32_t cs;
          const uint32_t cv = sc_copy_piece(off, L, cs);
          sc_lds_or3(stga + at, cv, cs);
          at += cs;
        } else {  // emit_copy! (internal.jl:306-329): 64-byte pieces while >= 68, a 60 if > 64, the rest
          uint32_t R = L;
          while (R >= 68) {
            sc_lds_or3(stga + at, (2u + (63u << 2)) | (off << 8));
            at += 3;
            R -= 64;
          }
          if (R > 64) {
            sc_lds_or3(stga + at, (2u + (59u << 2)) | (off << 8));
            at += 3;
            R -= 60;
          }
          uint32_t cs;
          const uint32_t cv = sc_copy_piece(off, R, cs);
          sc_lds_or3(stga + at, cv, cs);
          at += cs;
        }
        p = q + L;
      }
    }
    if (live && p < ce) {  // the lane's last run: it starts the merged run, unless it only continues one
      const uint32_t run = ce - p;
      uint32_t tag = 0, ts = 0;
      if (!(tk.n == 0 && cont)) tag = sc_lit_tag(merged, ts);
      sc_lds_orn(stga + at, sc_trim(sc_prepend(sc_ld128(S.blk, p), tag, ts), min(ts + run, 16u)), min(ts + run, 16u));
      if (ts + run > 16) sc_lds_or(stga + at + 16, sc_trim(sc_ld128(S.blk, p + 16 - ts), ts + run - 16));
    }
  }
  // (a wave's LDS operations execute in order: the writer that sees the size sees the bytes)
  __hip_atomic_store(&S.rsize[slot], total + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // (all lanes: same value)
}

// the staged bytes [0, len) of an LDS buffer (16-byte aligned) to global g (any alignment): aligned
// 16-byte stores of byte-shifted units, bytes at the two partial ends (one wave)
__device__ __attribute__((always_inline)) inline void sc_copy_out(uint8_t* const g, const uint8_t* stg, uint32_t len,
                                                                 uint32_t lane) {
  const uint32_t ad = (uint32_t)((uintptr_t)g & 15);
  const uint32_t u0 = ad ? 1u : 0u, u1 = (len + ad) >> 4;  // full units [u0, u1); unit u = bytes [16u - ad, +16)
  uint4* const g16 = reinterpret_cast<uint4*>(g - ad);
  const uint32_t* const s32 = reinterpret_cast<const uint32_t*>(stg);
  for (uint32_t u = u0 + lane; u < u1; u += 64) {
    const uint32_t j = 16 * u - ad;  // staging offset of the unit: five aligned dwords from j & ~3, funnel shifts
    const uint32_t* w = s32 + (j >> 2);  // (j + 20 <= len + 4: inside the slot)
    const uint32_t r0 = w[0], r1 = w[1], r2 = w[2], r3 = w[3], r4 = w[4];
    g16[u] = make_uint4(__builtin_amdgcn_alignbyte(r1, r0, j), __builtin_amdgcn_alignbyte(r2, r1, j),
                        __builtin_amdgcn_alignbyte(r3, r2, j), __builtin_amdgcn_alignbyte(r4, r3, j));
  }
  const uint32_t nh = min(u0 ? 16 - ad : 0u, len);              // head bytes [0, nh)
  const uint32_t tb = max(16 * u1 > ad ? 16 * u1 - ad : 0u, nh);  // tail bytes [tb, len)
  const uint32_t nt = len - tb;
  if (lane < nh + nt) {
    const uint32_t jj = lane < nh ? lane : tb + (lane - nh);
    g[jj] = stg[jj];
  }
}

// The writer wave: the staged super-chunks k0..k1-1 in order, each at the running output offset (no
// wave waits for another's offset), then the output's length into *len_out.  A whole block
// (whole) whose parse came out larger than one literal of the block (a nearly incompressible block
// past the screen) is rewritten as that literal (emit_literal!, internal.jl:271-284): the output
// never exceeds the literal size.  (A part of a block, k_compress_sc_span: the gather checks its
// block's sum instead.)
__device__ __attribute__((always_inline)) inline void sc_writer(ScLds& S, uint32_t n, uint8_t* const dst, uint32_t hv,
                                                               uint32_t k0, uint32_t k1, bool whole,
                                                               uint32_t* len_out, uint32_t lane) {
  uint32_t o = hv, err = 0;
  // (the next slot's size word is read together with this slot's bytes: when the workers are ahead,
  // as they mostly are, the next link starts without a poll round trip of its own)
  uint32_t vpre = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t slot = k % kScRing;
    const uint32_t sz =
        (vpre ? vpre : sc_wait(&S.rsize[slot], [](uint32_t v) { return v != 0; }, err, 4u)) - 1;
    if (err) break;
    vpre = k + 1 < k1 ? uniform(__hip_atomic_load(&S.rsize[(k + 1) % kScRing], __ATOMIC_ACQUIRE,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP))
                        : 0u;
    sc_copy_out(dst + o, S.ring[slot], sz, lane);
    o += sz;
    // (this wave's slot reads are issued before these writes, and LDS runs them in order)
    __hip_atomic_store(&S.rsize[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&S.rseq[slot], k + kScRing, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const uint32_t h = hv + (n ? literal_tag_bytes(n) : 0u);
  if (whole && !err && n && o > h + n) {  // one literal: the tag after the varint, the block from LDS
    uint8_t* const g = dst + hv;
    const uint32_t tb = h - hv, len = tb + n;  // literal stream bytes j: the tag (j < tb), then blk[j - tb]
    const uint32_t ad = (uint32_t)((uintptr_t)g & 15);
    uint4* const g16 = reinterpret_cast<uint4*>(g - ad);
    const uint32_t u1 = (len + ad) >> 4;              // units [ua, u1) are whole and past the tag
    const uint32_t ua = (tb + ad + 15) >> 4;
    for (uint32_t u = ua + lane; u < u1; u += 64) g16[u] = sc_ld128(S.blk, 16 * u - ad - tb);
    const uint32_t he = ua < u1 ? 16 * ua - ad : len;  // bytes [0, he) and [te, len) one by one
    const uint32_t te = ua < u1 ? 16 * u1 - ad : len;
    for (uint32_t j = lane; j < he + (len - te); j += 64) {
      const uint32_t jj = j < he ? j : te + (j - he);
      uint8_t c;
      if (jj < tb) {
        c = tb == 1 ? (uint8_t)((n - 1) << 2) : (jj == 0 ? (uint8_t)((58 + tb) << 2) : (uint8_t)((n - 1) >> (8 * (jj - 1))));
      } else {
        c = S.blk[jj - tb];
      }
      g[jj] = c;
    }
    o = h + n;
  }
  err |= uniform(__hip_atomic_load(&S.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  if (lane == 0) *len_out = err ? 0xfff00000u | err : o;  // (an error mark: > any block's length)
}

// Persistent: one workgroup per CU walks blocks blockIdx.x, + gridDim.x, ...; each wave loads its
// share of the next block into registers as soon as it runs out of super-chunks, so the HBM
// latency of the staging hides behind the block's tail.
template <int kDense>
__global__ __launch_bounds__(kScThreads) void k_compress_sc(CompressArgs a) {
  __shared__ __attribute__((aligned(16))) ScLds S;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);
  const uint32_t lane = tid & 63;
  static_assert(kBlockSize / 16 / kScThreads == 4, "four 16-byte pieces per thread of a full block");
  uint4 pf0, pf1, pf2, pf3;
  // block b's length, source, and whether its bytes are in pf0..3 (a 16-byte aligned full block)
  uint32_t b = sc_next_block(a, blockIdx.x, lane);
  uint32_t n = 0;
  const uint8_t* src = nullptr;
  bool inpf = false;
#define SC_FETCH(bb)                                                              \
  {                                                                               \
    n = (bb) < a.nblk ? a.in_len[bb] : 0u;                                        \
    src = (bb) < a.nblk ? a.in + a.in_off[bb] : nullptr;                          \
    inpf = (bb) < a.nblk && n == kBlockSize && ((uintptr_t)src & 15) == 0;        \
    if (inpf) {                                                                   \
      const uint4* s16 = reinterpret_cast<const uint4*>(src);                     \
      pf0 = s16[tid];                                                             \
      pf1 = s16[tid + kScThreads];                                                \
      pf2 = s16[tid + 2 * kScThreads];                                            \
      pf3 = s16[tid + 3 * kScThreads];                                            \
    }                                                                             \
  }
  SC_FETCH(b)
  while (b < a.nblk) {
    uint8_t* const dst = a.out + a.out_off[b];
    if (n > kBlockSize) {  // (uniform) not a block: error mark, next
      if (tid == 0) a.out_len[b] = 0xffffffffu;
      b = sc_next_block(a, b + gridDim.x, lane);
      SC_FETCH(b)
      continue;
    }
    // ---- stage the block, clear the table ----
    if (inpf) {
      uint4* d16 = reinterpret_cast<uint4*>(S.blk);
      d16[tid] = pf0;
      d16[tid + kScThreads] = pf1;
      d16[tid + 2 * kScThreads] = pf2;
      d16[tid + 3 * kScThreads] = pf3;
    } else if (((uintptr_t)src & 15) == 0) {
      const uint4* s16 = reinterpret_cast<const uint4*>(src);
      uint4* d16 = reinterpret_cast<uint4*>(S.blk);
      const uint32_t n16 = n >> 4;
      for (uint32_t k = tid; k < n16; k += kScThreads) d16[k] = s16[k];
      for (uint32_t k = (n & ~15u) + tid; k < n; k += kScThreads) S.blk[k] = src[k];
    } else {
      for (uint32_t k = tid; k < n; k += kScThreads) S.blk[k] = src[k];
    }
    if (tid < 64) S.blk[n + tid] = 0;  // bytes past the block read as zeros (never part of a match)
    {
      uint4* t16 = reinterpret_cast<uint4*>(S.T);
      for (uint32_t k = tid; k < 4 * kScTabWords / 16; k += kScThreads) t16[k] = make_uint4(0, 0, 0, 0);
    }
    const uint32_t hv = a.header ? varint_len(n) : 0u;
    if (tid < hv) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < hv ? 0x80 : 0));
    if (wave == 0) {  // the hand-off words (the previous block's users are past the barrier)
      if (lane < kScRing) {
        S.rsize[lane] = 0;
        S.rseq[lane] = lane;
      }
      if (lane == 0) {
        S.ins = 0;
        S.next = 0;
        S.err = 0;
      }
    }
    // the block after this one (its stride scan now, its bytes when this wave runs out of work)
    const uint32_t bn = sc_next_block(a, b + gridDim.x, lane);
    __syncthreads();

    const uint32_t nsc = (n + kScS - 1) / kScS;
    if (wave == kScWorkers) {
      __builtin_amdgcn_s_setprio(SC_WPRIO);  // (the writer's chain gates the slots)
      sc_writer(S, n, dst, hv, 0, nsc, true, &a.out_len[b], lane);
      __builtin_amdgcn_s_setprio(0);
    } else {
      // (no lane-0-only code here or at the end of a super-chunk: the compiler merged two such
      // regions across the loop's back edge into a divergent loop that hung the wave)
      for (;;) {
        // every lane adds 1 (one ds_add of 64 after the atomic optimizer); lane 0 sees a multiple of 64
        const uint32_t k = uniform(__hip_atomic_fetch_add(&S.next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 6;
        if (k >= nsc) break;
        sc_superchunk<kDense>(S, k, n, wave, lane);
      }
    }
    SC_FETCH(bn)  // the next block's bytes, in flight behind the other waves' last super-chunks
    __syncthreads();
    b = bn;
  }
#undef SC_FETCH
}

// ---- one block in parts, for latency (sm_compress of small inputs) ------------------------
// Item i = (block i / parts, part j = i % parts) parses super-chunks [j span, (j + 1) span) of its
// block on its own workgroup, so a few blocks use many CUs.  The parse of a super-chunk depends on
// the block's bytes and the table state before it (every earlier position inserted in order), so
// the item first rebuilds that state: a slot ends up holding the LATEST earlier position of its
// hash and parity, i.e. the maximum -- order-free, so all waves insert with ds_max_u32: the odd
// groups' slots (high halves) first, then the even groups' (low halves, the high half read back
// and kept).  Everything after that is the whole-block kernel's code, so the output equals the
// concatenation of the block's output in k_compress_sc (sans its literal fallback, which the
// gather checks per block).  Item outputs at out + out_off[block] + j pitch, lengths in
// part_len[i]; a block the screen emitted as a literal has that literal as its part 0.
template <int kDense>
__global__ __launch_bounds__(kScThreads) void k_compress_sc_span(CompressArgs a, ScSpan sp) {
  __shared__ __attribute__((aligned(16))) ScLds S;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = uniform(tid >> 6);
  const uint32_t lane = tid & 63;
  const uint32_t b = blockIdx.x / sp.parts, j = blockIdx.x % sp.parts;
  if (b >= a.nblk) return;
  uint32_t* const plen = sp.part_len + blockIdx.x;
  const uint32_t n = a.in_len[b];
  if (n > kBlockSize) {  // not a block: an error mark in part 0 (the gather refuses it)
    if (tid == 0) *plen = j == 0 ? 0xffffffffu : 0u;
    return;
  }
  const uint32_t nsc = (n + kScS - 1) / kScS;
  const uint32_t k0 = j * sp.span, k1 = min(k0 + sp.span, nsc);
  const bool todo = !a.screened || a.out_len[b] == kScreenTodoSc;
  if (!todo || k0 >= k1) {  // a screened literal (part 0 is its output) or a part past the block
    if (tid == 0) *plen = (!todo && j == 0) ? a.out_len[b] : 0u;
    return;
  }
  const uint8_t* const src = a.in + a.in_off[b];
  uint8_t* const dst = a.out + a.out_off[b] + (uint64_t)j * sp.pitch;
  // ---- stage the block, clear the table (as k_compress_sc) ----
  if (((uintptr_t)src & 15) == 0) {
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(S.blk);
    const uint32_t n16 = n >> 4;
    for (uint32_t k = tid; k < n16; k += kScThreads) d16[k] = s16[k];
    for (uint32_t k = (n & ~15u) + tid; k < n; k += kScThreads) S.blk[k] = src[k];
  } else {
    for (uint32_t k = tid; k < n; k += kScThreads) S.blk[k] = src[k];
  }
  if (tid < 64) S.blk[n + tid] = 0;
  {
    uint4* t16 = reinterpret_cast<uint4*>(S.T);
    for (uint32_t k = tid; k < 4 * kScTabWords / 16; k += kScThreads) t16[k] = make_uint4(0, 0, 0, 0);
  }
  const uint32_t hv = (a.header && j == 0) ? varint_len(n) : 0u;
  if (tid < hv) dst[tid] = (uint8_t)(((n >> (7 * tid)) & 0x7f) | (tid + 1 < hv ? 0x80 : 0));
  if (wave == 0) {  // the hand-off words, starting at super-chunk k0
    if (lane < kScRing) {
      S.rsize[lane] = 0;
      S.rseq[lane] = k0 + ((lane - k0) & (kScRing - 1));
    }
    if (lane == 0) {
      S.ins = k0;
      S.next = 64 * k0;
      S.err = 0;
    }
  }
  __syncthreads();
  // ---- the table as the in-order insert of positions [0, kScS k0) leaves it (section B's values:
  // positions, group parity = slot; positions without 4 bytes before the block end never enter;
  // a never-written slot and position 0 both read 0, the same candidate)
  const uint32_t pe = kScS * k0;
  // (a lane takes four consecutive positions of one group -- two aligned dwords give their four
  // words -- and a wave four groups of the phase's parity per step)
  const uint32_t sub = lane & 15, gq = lane >> 4;
  for (int ph = 1; ph >= 0; --ph) {
    for (uint32_t i = wave; 128 * (4 * i) < pe; i += kScW) {
      const uint32_t G = 2 * (4 * i + gq) + (uint32_t)ph;  // this lane's group
      const uint32_t q = 64 * G + 4 * sub;
      if (q >= pe) continue;
      const uint32_t d0 = sc_ld32(S.blk, q), d1 = sc_ld32(S.blk, q + 4);
      uint32_t* t[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t w = j ? __builtin_amdgcn_alignbyte(d1, d0, j) : d0;
        t[j] = &S.T[(w * kHashMul) >> (32 - kScTabBits)];
      }
      if (ph) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (q + j + 4 <= n) __hip_atomic_fetch_max(t[j], (q + j) << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {  // (the high half is final: only low halves change in this phase)
        uint32_t hi[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) hi[j] = __hip_atomic_load(t[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (q + j + 4 <= n)
            __hip_atomic_fetch_max(t[j], (hi[j] & 0xffff0000u) | (q + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __syncthreads();
  }
  if (wave == kScWorkers) {
    __builtin_amdgcn_s_setprio(SC_WPRIO);
    sc_writer(S, n, dst, hv, k0, k1, false, plen, lane);
    __builtin_amdgcn_s_setprio(0);
  } else {
    for (;;) {
      const uint32_t k = uniform(__hip_atomic_fetch_add(&S.next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 6;
      if (k >= k1) break;
      sc_superchunk<kDense>(S, k, n, wave, lane);
    }
  }
}

hipError_t launch_compress_sc_span(const CompressArgs& a, int mode, const ScSpan& sp, hipStream_t s) {
  if (sp.parts == 0 || sp.span == 0 || sp.parts * sp.span < (kBlockSize + kScS - 1) / kScS ||
      sp.pitch < (uint64_t)sp.span * kScSlot)
    return hipErrorInvalidValue;
  const uint32_t grid = a.nblk * sp.parts;
  if (grid == 0) return hipSuccess;
  if (mode == 2)
    hipLaunchKernelGGL(k_compress_sc_span<1>, dim3(grid), dim3(kScThreads), 0, s, a, sp);
  else
    hipLaunchKernelGGL(k_compress_sc_span<0>, dim3(grid), dim3(kScThreads), 0, s, a, sp);
  return hipGetLastError();
}


// mode 1 (SM_MODE_FAST): the more recent 4-byte match per position; mode 2 (SM_MODE_FAST_DENSE): the
// longer of the two candidates over 16 bytes (smaller output, about 15% slower)
hipError_t launch_compress_sc(const CompressArgs& a, int mode, hipStream_t s) {
  static uint32_t ncu_cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  uint32_t ncu = __atomic_load_n(&ncu_cache[dev], __ATOMIC_RELAXED);
  if (!ncu) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    ncu = (uint32_t)v;
    __atomic_store_n(&ncu_cache[dev], ncu, __ATOMIC_RELAXED);
  }
  const uint32_t grid = min(a.nblk, ncu);  // one workgroup per CU (the LDS holds one)
  if (mode == 2)
    hipLaunchKernelGGL(k_compress_sc<1>, dim3(grid), dim3(kScThreads), 0, s, a);
  else
    hipLaunchKernelGGL(k_compress_sc<0>, dim3(grid), dim3(kScThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace sm
