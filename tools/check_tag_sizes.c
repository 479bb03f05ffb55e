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
// the per-byte definition (255: a literal the batch walk leaves to the general path)
static uint32_t spec_size(uint32_t c, uint32_t trailer) {
  uint32_t entry = char_entry(c), taglen = entry >> 11;
  if (c & 3) return 1 + taglen;
  uint32_t hi = c >> 2;
  if (hi < 60) return 1 + (entry & 0xff);
  if (hi > 60) return 255u;  // two to four length bytes
  uint32_t lit = 1 + (trailer & 0xff);
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
  const uint32_t ml = perm(0u, 0x000000ffu, K);
  uint32_t s = (csz & ~ml) | ((H + 0x02020202u) & ml);
  const uint32_t h60 = (H + 0x44444444u) & 0x80808080u & ml;
  *slow = h60 != 0;
  if (h60) {
    const uint32_t hm = h60 | (h60 - (h60 >> 7));
    const uint32_t b = alignbyte(nxt, cur, 1);
    const uint32_t e = cur ^ 0xf0f0f0f0u;
    const uint32_t ne = (((e & 0x7f7f7f7fu) + 0x7f7f7f7fu) | e) & 0x80808080u;
    const uint32_t bb = (((b >> 1) & 0x7f7f7f7fu) + 0x1c1c1c1cu) & 0x80808080u;
    const uint32_t st = ne | bb;
    const uint32_t sm = st | (st - (st >> 7));
    const uint32_t v = (b | sm) + (0x03030303u & ~sm);
    s = (s & ~hm) | (v & hm);
  }
  return s;
}
int main() {
  uint64_t x = 88172645463325252ull; long bad = 0, nslow = 0, N = 20000000;
  for (long i = 0; i < N; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    uint32_t cur = (uint32_t)x, nxt = (uint32_t)(x >> 32);
    if (i < 4 * 65536) {  // every (tag byte, next byte) pair at each of the 4 positions
      const uint32_t j = (uint32_t)(i >> 16), c = (uint32_t)(i & 0xff), b = (uint32_t)((i >> 8) & 0xff);
      cur = (cur & ~(0xffu << (8 * j))) | (c << (8 * j));
      if (j < 3) cur = (cur & ~(0xffu << (8 * (j + 1)))) | (b << (8 * (j + 1)));
      else nxt = (nxt & ~0xffu) | b;
    }
    int sl; uint32_t a = pack_fast(cur, nxt, &sl), b = pack_slow(cur, nxt);
    nslow += sl; if (a != b) { if (bad < 5) printf("mismatch %08x %08x: %08x vs %08x\n", cur, nxt, a, b); ++bad; }
  }
  printf("bad %ld, length-byte fix-up fraction %.4f (uniform random bytes)\n", bad, (double)nslow / N);
  return bad != 0;
}
