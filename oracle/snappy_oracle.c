/*
 * snappy_oracle.c -- CPU restatement of krm01/Snappy.jl (TEST INFRASTRUCTURE ONLY).
 * See snappy_oracle.h for what pins it.  Reference paths are relative to /root/reference.
 * Indices are 0-based here; the reference is 1-based, so every bound is re-derived at the
 * cited line rather than transliterated.
 */
#include "snappy_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define K_BLOCK_SIZE 65536u        /* internal.jl:31 */
#define K_INPUT_MARGIN_BYTES 15u   /* internal.jl:32 */
#define K_MAX_HASH_TABLE_SIZE 16384u /* internal.jl:33 */

static inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* Snappy.jl:80-82 */
size_t smo_max_compressed_length(size_t n) { return 32 + n + n / 6; }

/* varint.jl:12-37 -- fails when the buffer ends or on a 5th byte >= 0x10 */
int smo_parse32(const uint8_t* buf, size_t len, size_t off, uint32_t* val, size_t* next) {
  uint32_t result = 0;
  for (int i = 0; i < 5; ++i) {
    if (off + i >= len) return SMO_ERR_VARINT;
    uint32_t b = buf[off + i];
    if (i < 4) {
      result |= (b & 0x7f) << (7 * i);
      if (b < 0x80) { *val = result; *next = off + i + 1; return SMO_OK; }
    } else {
      result |= (b & 0x7f) << 28;
      if (b < 0x10) { *val = result; *next = off + 5; return SMO_OK; }
    }
  }
  return SMO_ERR_VARINT;
}

/* varint.jl:46-69 */
size_t smo_encode32(uint8_t* buf, uint32_t v) {
  size_t i = 0;
  while (v >= 0x80) { buf[i++] = (uint8_t)(v | 0x80); v >>= 7; }
  buf[i++] = (uint8_t)v;
  return i;
}

/* internal.jl:107-113: smallest power of two >= n, clamped to [256, 16384] */
uint32_t smo_hashtable_size(size_t n) {
  uint32_t ht = 256;
  while (ht < K_MAX_HASH_TABLE_SIZE && ht < n) ht <<= 1;
  return ht;
}

/* internal.jl:47-80 + the comment at :35-46: bits 0-7 length, 8-10 offset>>8, 11-13 extra
 * bytes.  Derived from the tag rules instead of transcribing the 256 literals. */
uint16_t smo_char_table(uint8_t c) {
  uint32_t kind = c & 3, hi = c >> 2;
  if (kind == 0) {
    if (hi < 60) return (uint16_t)(hi + 1);
    return (uint16_t)(((hi - 59) << 11) | 1);
  }
  if (kind == 1) return (uint16_t)((1u << 11) | ((uint32_t)(c >> 5) << 8) | (4 + ((c >> 2) & 7)));
  if (kind == 2) return (uint16_t)((2u << 11) | (hi + 1));
  return (uint16_t)((4u << 11) | (hi + 1));
}

/* internal.jl:343-387 (64-bit LE variant).  limit is INCLUSIVE, as in the reference.
 * Reads exactly the bytes the reference reads; reports -1 if any is outside a[0..alen). */
long smo_find_match_length(const uint8_t* a, size_t alen, size_t i1, size_t i2, size_t limit) {
  long matched = 0;
  if (i2 + 7 <= limit) {                                  /* :356 i2 <= limit-7 */
    if (i2 + 8 > alen || i1 + 8 > alen) return -1;
    uint64_t a1 = ld64(a + i1), a2 = ld64(a + i2);
    if (a1 != a2) return __builtin_ctzll(a1 ^ a2) >> 3;   /* :359-360 */
    i2 += 8; matched = 8;
  }
  while (i2 + 7 <= limit) {                               /* :371 */
    if (i2 + 8 > alen || i1 + matched + 8 > alen) return -1;
    uint64_t x = ld64(a + i2) ^ ld64(a + i1 + matched);
    if (x == 0) { i2 += 8; matched += 8; }
    else return matched + (__builtin_ctzll(x) >> 3);      /* :376-379 */
  }
  while (i2 <= limit) {                                   /* :382 */
    if (i2 >= alen || i1 + matched >= alen) return -1;
    if (a[i1 + matched] != a[i2]) break;
    ++i2; ++matched;
  }
  return matched;
}

/* internal.jl:94 */
static inline uint32_t hashdword(uint32_t bytes, uint32_t shift) {
  return (uint32_t)(bytes * 0x1e35a7bdu) >> shift;
}

/* internal.jl:252-287.  The fast path writes the same bytes as the slow one (its 16-byte
 * over-copy lands in slack that later emits overwrite or the final resize! drops).
 * Quirk Q3: the one-byte tag is used only for len < 60 (:271); C++ snappy uses it for
 * len-1 < 60, so a 60-byte literal is f0 3b here and ec in libsnappy.  compat flips it. */
static size_t emit_literal(uint8_t* out, size_t op, const uint8_t* lit, size_t len, int compat) {
  uint32_t n = (uint32_t)(len - 1);
  if (compat ? (n < 60) : (len < 60)) {
    out[op++] = (uint8_t)(n << 2);
  } else {
    size_t base = op++;
    uint32_t count = 0;
    while (n > 0) { out[op++] = (uint8_t)n; n >>= 8; ++count; }
    out[base] = (uint8_t)((59 + count) << 2);
  }
  memcpy(out + op, lit, len);
  return op + len;
}

/* internal.jl:289-304 */
static size_t emit_copy_upto_64(uint8_t* out, size_t op, uint32_t offset, uint32_t len) {
  if (len < 12 && offset < 2048) {
    out[op] = (uint8_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0));
    out[op + 1] = (uint8_t)(offset & 0xff);
    return op + 2;
  }
  out[op] = (uint8_t)(2 + ((len - 1) << 2));
  out[op + 1] = (uint8_t)offset;
  out[op + 2] = (uint8_t)(offset >> 8);
  return op + 3;
}

/* internal.jl:306-329 */
static size_t emit_copy(uint8_t* out, size_t op, uint32_t offset, uint32_t len) {
  if (len < 12) return emit_copy_upto_64(out, op, offset, len);
  while (len >= 68) { op = emit_copy_upto_64(out, op, offset, 64); len -= 64; }
  if (len > 64) { op = emit_copy_upto_64(out, op, offset, 60); len -= 60; }
  return emit_copy_upto_64(out, op, offset, len);
}

/* internal.jl:127-250, fragment in[s .. e] (e inclusive, may be s-1 for empty).
 * compat=1 flips quirks Q1 (ip_limit one byte later, as C++ snappy) and Q3. */
static size_t compress_fragment(uint8_t* out, size_t op, const uint8_t* in, long s, long e,
                                uint16_t* table, uint32_t table_size, int compat) {
  uint32_t shift = 32 - (31 - __builtin_clz(table_size));     /* :128 */
  long base = s, ip = s, next_emit = s, cand;
  long n = e - s + 1;                                        /* :130 */
  /* :131  1-based ip_limit = ip_end - 15  ==  0-based (e - 15); C++: e + 1 - 15 */
  long ip_limit = compat ? e + 1 - (long)K_INPUT_MARGIN_BYTES : e - (long)K_INPUT_MARGIN_BYTES;
  if (n >= (long)K_INPUT_MARGIN_BYTES) {                     /* :133 */
    for (;;) {
      uint32_t skip = 32;                                    /* :162 */
      ++ip;                                                  /* :163 */
      uint32_t next_hash = hashdword(ld32(in + ip), shift);
      long next_ip = ip;
      for (;;) {                                             /* :167-194 */
        ip = next_ip;
        uint32_t cur_hash = next_hash;
        uint32_t step = skip >> 5;
        skip += step;
        next_ip = ip + step;
        if (next_ip > ip_limit) goto emit_remainder;         /* :175 */
        next_hash = hashdword(ld32(in + next_ip), shift);
        cand = base + (uint16_t)(table[cur_hash] + 1);       /* :190 */
        table[cur_hash] = (uint16_t)(ip - base - 1);         /* :191 */
        if (ld32(in + cand) == ld32(in + ip)) break;         /* :193 */
      }
      op = emit_literal(out, op, in + next_emit, (size_t)(ip - next_emit), compat); /* :200 */
      for (;;) {                                             /* :211-239 */
        long m = smo_find_match_length(in, (size_t)(e + 1), (size_t)(cand + 4),
                                       (size_t)(ip + 4), (size_t)e);
        uint32_t matched = 4 + (uint32_t)m;                  /* :216 */
        op = emit_copy(out, op, (uint32_t)(ip - cand), matched);
        ip += matched;
        next_emit = ip;
        if (ip >= ip_limit) goto emit_remainder;             /* :222 */
        uint32_t prev_hash = hashdword(ld32(in + ip - 1), shift);
        uint32_t input_bytes = ld32(in + ip);
        uint32_t cur_hash = hashdword(input_bytes, shift);
        table[prev_hash] = (uint16_t)(ip - base - 2);        /* :233 */
        cand = base + (uint16_t)(table[cur_hash] + 1);       /* :234 */
        table[cur_hash] = (uint16_t)(ip - base - 1);         /* :235 */
        if (input_bytes != ld32(in + cand)) break;           /* :238 */
      }
    }
  }
emit_remainder:
  if (next_emit <= e)                                        /* :244-248 */
    op = emit_literal(out, op, in + next_emit, (size_t)(e - next_emit + 1), compat);
  return op;
}

/* Snappy.jl:20-36.  compat=1 flips quirk Q2 (table sized per fragment, as C++ snappy). */
int smo_compress(const uint8_t* in, size_t n, uint8_t* out, size_t* out_len, int compat) {
  if (n > 0xffffffffull) return SMO_ERR_INPUT_TOO_LARGE;    /* :21 */
  size_t op = smo_encode32(out, (uint32_t)n);                /* :26 */
  uint16_t table[K_MAX_HASH_TABLE_SIZE];
  uint32_t tsize_total = smo_hashtable_size(n);              /* :27 */
  for (size_t i = 0; i <= n; i += K_BLOCK_SIZE) {            /* :29  0:K_BLOCK_SIZE:n */
    size_t end = (i + K_BLOCK_SIZE < n) ? i + K_BLOCK_SIZE : n;
    uint32_t tsize = compat ? smo_hashtable_size(end - i) : tsize_total;
    memset(table, 0xff, tsize * sizeof(uint16_t));           /* :30 */
    op = compress_fragment(out, op, in, (long)i, (long)end - 1, table, tsize, compat);
    if (i + K_BLOCK_SIZE > n) break;
  }
  *out_len = op;
  return SMO_OK;
}

/* One fragment of a larger stream, as the block loop of Snappy.jl:29-33 runs it: no header,
 * table size from the stream's total length (Q2).  n <= 65536. */
int smo_compress_fragment(const uint8_t* in, size_t n, uint8_t* out, size_t* out_len, size_t total_len,
                          int compat) {
  if (n > K_BLOCK_SIZE) return SMO_INVALID_INPUT;
  uint16_t table[K_MAX_HASH_TABLE_SIZE];
  uint32_t tsize = compat ? smo_hashtable_size(n) : smo_hashtable_size(total_len);
  memset(table, 0xff, tsize * sizeof(uint16_t));
  *out_len = compress_fragment(out, 0, in, 0, (long)n - 1, table, tsize, compat);
  return SMO_OK;
}

int smo_uncompressed_length(const uint8_t* in, size_t n, size_t* result) {
  uint32_t v; size_t next;
  int st = smo_parse32(in, n, 0, &v, &next);                 /* Snappy.jl:90-92 */
  if (st == SMO_OK) *result = v;
  return st;
}

/* internal.jl:411-466 + incremental_copy! :492-509 + copy_literal! :515-527,
 * then the produced == declared check of Snappy.jl:50. */
int smo_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, size_t* out_len) {
  uint32_t size; size_t ip;
  int st = smo_parse32(in, n, 0, &size, &ip);
  if (st != SMO_OK) return st;
  if (size > out_cap) return SMO_BUFFER_TOO_SMALL;
  int64_t op = 0;
  const int64_t N = (int64_t)n, S = (int64_t)size;
  int64_t p = (int64_t)ip;
  static const uint32_t wordmask[5] = {0, 0xff, 0xffff, 0xffffff, 0xffffffffu}; /* :83-85 */
  while (p < N - 1) {                                        /* :416  ip < endof(input) */
    uint8_t c = in[p++];
    uint32_t tag = 0;                                        /* :426-430 zero-padded lookahead */
    for (int k = 0; k < 4; ++k)
      if (p + k < N) tag |= (uint32_t)in[p + k] << (8 * k);
    uint16_t entry = smo_char_table(c);                      /* :435-439 */
    uint32_t len = entry & 0xff;
    uint32_t taglen = entry >> 11;
    uint32_t trailer = tag & wordmask[taglen];
    p += taglen;
    if (c & 3) {                                             /* :458-460 copy */
      uint32_t offset = (uint32_t)(entry & 0x700) + trailer;
      int64_t avail_out = S - op;
      if (op <= (int64_t)(uint32_t)(offset - 1u)) return SMO_ERR_COPY_OFFSET; /* :499 */
      if (!(len <= 16 && offset >= 8 && avail_out >= 16)) {  /* :500 fast path needs no check */
        if (avail_out < (int64_t)len) return SMO_ERR_COPY_LENGTH;              /* :505 */
      }
      for (uint32_t k = 0; k < len; ++k) out[op + k] = out[op - offset + k];
      op += len;
    } else {                                                 /* :461-462 literal */
      uint32_t litlen = len + trailer;                       /* UInt32 wrap, as Julia */
      int64_t avail_out = S - op, avail_in = N - p;
      if (avail_out < (int64_t)litlen || avail_in < (int64_t)litlen) return SMO_ERR_LITERAL;
      memcpy(out + op, in + p, litlen);
      op += litlen; p += litlen;
    }
  }
  if (op != S) return SMO_ERR_INVALID;                       /* Snappy.jl:50 */
  *out_len = (size_t)op;
  return SMO_OK;
}

int smo_compress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                       uint32_t nblk, uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                       int compat, int nthreads) {
  int bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1) reduction(|:bad)
#endif
  for (long b = 0; b < (long)nblk; ++b) {
    size_t ol = 0;
    int st = smo_compress(in + in_off[b], in_len[b], out + out_off[b], &ol, compat);
    out_len[b] = (uint32_t)ol;
    bad |= (st != SMO_OK);
  }
  (void)nthreads;
  return bad ? SMO_INVALID_INPUT : SMO_OK;
}

int smo_uncompress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                         uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                         const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                         int nthreads) {
  int bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1) reduction(|:bad)
#endif
  for (long b = 0; b < (long)nblk; ++b) {
    size_t ol = 0;
    int st = smo_uncompress(in + in_off[b], in_len[b], out + out_off[b], out_cap[b], &ol);
    out_len[b] = (uint32_t)ol;
    status[b] = st;
    bad |= (st != SMO_OK);
  }
  (void)nthreads;
  return bad ? SMO_INVALID_INPUT : SMO_OK;
}
