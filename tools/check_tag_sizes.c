// Design check for the decoder's SWAR tag-size computation (pack_sizes in
// snappy.jl_amd/csrc/sm_decompress.hip): the packed formula must equal the per-byte
// definition (char_entry / spec_size, internal.jl:435-462 semantics) for every input.
// v_perm_b32 is emulated.  Run by tests/test_host_logic.py.
#include <stdint.h>
#include <stdio.h>
static uint32_t char_entry(uint32_t c) {
  uint32_t kind = c & 3, hi = c >> 2;
  if (kind == 0) return hi < 60 ? hi + 1 : (((hi - 59) << 11) | 1);
  if (kind == 1) return (1u << 11) | ((c >> 5) << 8) | (4 + ((c >> 2) & 7));
  if (kind == 2) return (2u << 11) | (hi + 1);
  return (4u << 11) | (hi + 1);
}
static uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (s & 3))); }
static uint32_t spec_size(uint32_t c, uint32_t trailer) {
  uint32_t entry = char_entry(c), taglen = entry >> 11;
  if (c & 3) return 1 + taglen;
  uint32_t len = entry & 0xff;
  uint32_t tr = taglen >= 4 ? trailer : (trailer & ((1u << (8 * taglen)) - 1u));
  uint32_t lit = len + tr;
  return lit > 200 ? 255u : 1 + taglen + lit;
}
static uint32_t pack_slow(uint32_t cur, uint32_t nxt) {
  uint32_t s = 0;
  for (int j = 0; j < 4; ++j) {
    uint32_t c = (cur >> (8 * j)) & 0xff;
    uint32_t tr = j == 3 ? nxt : alignbyte(nxt, cur, j + 1);
    s |= spec_size(c, tr) << (8 * j);
  }
  return s;
}
static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t v = ((uint64_t)s0 << 32) | s1; uint32_t r = 0;
  for (int i = 0; i < 4; ++i) { uint32_t b = (sel >> (8 * i)) & 0xff; r |= (uint32_t)((v >> (8 * b)) & 0xff) << (8 * i); }
  return r;
}
static uint32_t pack_fast(uint32_t cur, uint32_t nxt, int* slow) {
  const uint32_t K = cur & 0x03030303u, H = (cur >> 2) & 0x3f3f3f3fu;
  const uint32_t csz = perm(0u, 0x05030200u, K);
  const uint32_t nz = ((K + 0x7f7f7f7fu) & 0x80808080u) >> 7;
  const uint32_t ml = (nz ^ 0x01010101u) * 0xffu;
  uint32_t s = (csz & ~ml) | ((H + 0x02020202u) & ml);
  *slow = ((H + 0x44444444u) & 0x80808080u & ml) != 0;
  if (*slow) s = pack_slow(cur, nxt);
  return s;
}
int main() {
  uint64_t x = 88172645463325252ull; long bad = 0, nslow = 0, N = 20000000;
  for (long i = 0; i < N; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    uint32_t cur = (uint32_t)x, nxt = (uint32_t)(x >> 32);
    if (i < 256 * 256) cur = (uint32_t)(i & 0xff) | ((uint32_t)(i >> 8) << 24) | (cur & 0x00ffff00);
    int sl; uint32_t a = pack_fast(cur, nxt, &sl), b = pack_slow(cur, nxt);
    nslow += sl; if (a != b) { if (bad < 5) printf("mismatch %08x %08x: %08x vs %08x\n", cur, nxt, a, b); ++bad; }
  }
  printf("bad %ld, slow-path fraction %.4f (uniform random bytes)\n", bad, (double)nslow / N);
  return bad != 0;
}
