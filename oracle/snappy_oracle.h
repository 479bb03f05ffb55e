/*
 * snappy_oracle.h -- CPU restatement of krm01/Snappy.jl (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X codec.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / CPU baseline.
 * The product library (snappy.jl_amd/csrc) never links or calls it.
 *
 * Every function restates the Julia reference with 0-based indices; the file:line of the
 * reference each one follows is cited at its definition in snappy_oracle.c.
 *
 * Pinning (see DESIGN.md "Oracle"): the Julia reference cannot run here (no Julia
 * toolchain).  The restatement is pinned by
 *   (1) the 45 find_match_length known-answer tests of test/runtests.jl:176-267,
 *   (2) the reference-mode golden sizes/SHA-256 table of SURVEY.md 8(c) (16 corpus files),
 *   (3) compat mode (quirks Q1/Q2/Q3 flipped) == libsnappy 1.1.8 byte-for-byte (SURVEY.md F5;
 *       Q3, the 60-byte literal tag, found in this build and checked by tests/test_oracle.py),
 *   (4) decode of test/testdata/alice29.snappy == alice29.txt, and the corrupted-input
 *       cases of test/runtests.jl:62-123 all rejected.
 */
#ifndef SNAPPY_ORACLE_H_
#define SNAPPY_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/snappy_mi355x.h */
enum {
  SMO_OK = 0,
  SMO_INVALID_INPUT = 1,
  SMO_BUFFER_TOO_SMALL = 2,
  SMO_ERR_INPUT_TOO_LARGE = 16, /* "Input too large."                    Snappy.jl:21   */
  SMO_ERR_INVALID = 17,         /* "Invalid input."                      Snappy.jl:50   */
  SMO_ERR_VARINT = 18,          /* "Could not decode varint32."          varint.jl:36   */
  SMO_ERR_COPY_OFFSET = 19,     /* "Invalid input: corrupt copy offset"  internal.jl:499 */
  SMO_ERR_COPY_LENGTH = 20,     /* "Invalid input: corrupt copy length"  internal.jl:505 */
  SMO_ERR_LITERAL = 21          /* "Invalid input: corrupt literal"      internal.jl:518 */
};

size_t smo_max_compressed_length(size_t n);
/* returns status; sets val and next on success.  off is 0-based. */
int smo_parse32(const uint8_t* buf, size_t len, size_t off, uint32_t* val, size_t* next);
/* writes 1..5 bytes, returns count */
size_t smo_encode32(uint8_t* buf, uint32_t v);
/* find_match_length with the reference's inclusive limit; 0-based indices into a[0..alen).
 * Returns -1 where the reference would read a[] out of bounds (the @test_broken KAT). */
long smo_find_match_length(const uint8_t* a, size_t alen, size_t i1, size_t i2, size_t limit);
/* hash table size the reference allocates for an n-byte input (internal.jl:107-113) */
uint32_t smo_hashtable_size(size_t n);
/* reference CHAR_TABLE entry (internal.jl:47-80), derived from the format rules */
uint16_t smo_char_table(uint8_t c);

/* compress(): compat=0 -> Snappy.jl byte-exact ("reference mode");
 *             compat=1 -> quirks Q1/Q2/Q3 flipped (== libsnappy 1.1.8). out must hold
 *             smo_max_compressed_length(n) bytes. */
int smo_compress(const uint8_t* in, size_t n, uint8_t* out, size_t* out_len, int compat);
/* uncompress(): reference accept/reject semantics (internal.jl:411-527, Snappy.jl:46-52).
 * If the declared length exceeds out_cap returns SMO_BUFFER_TOO_SMALL before decoding. */
int smo_uncompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, size_t* out_len);
int smo_uncompressed_length(const uint8_t* in, size_t n, size_t* result);
/* one <= 64 KiB fragment of a stream of total_len bytes (no header; Q2 table size) */
int smo_compress_fragment(const uint8_t* in, size_t n, uint8_t* out, size_t* out_len, size_t total_len,
                          int compat);

/* batch helpers used by bench.py's cpu_baseline leg (OpenMP over blocks when nthreads>1) */
int smo_compress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                       uint32_t nblk, uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                       int compat, int nthreads);
int smo_uncompress_batch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                         uint32_t nblk, uint8_t* out, const uint64_t* out_off,
                         const uint32_t* out_cap, uint32_t* out_len, int32_t* status,
                         int nthreads);

#ifdef __cplusplus
}
#endif
#endif
