// parallel-gcn_amd/csrc/rng.cpp -- xorshift128+ on the host: stepping, GF(2) jump-ahead
// and the byte tables the dropout kernel uses to advance chunk states by one epoch.
//
// The generator is hpdga-spring23/src/rand.cpp:17-28 (seed from rand.cpp:6-14). Its state
// update is linear over GF(2)^128, so "k draws later" is a 128x128 bit-matrix power. The
// reference GPU path uses curand Philox instead (src/variable.cu:5-61), which cannot
// reproduce the CPU masks; this engine reproduces them bit-for-bit.
#include "rng.hpp"

#include <cstdlib>
#include <cstring>

namespace pgcn {

// columns[i] = M * e_i, where bits 0..63 are s[0], bits 64..127 are s[1].
void BitMatrix::identity() {
  for (int i = 0; i < 128; i++) {
    col[i][0] = i < 64 ? (1ull << i) : 0;
    col[i][1] = i < 64 ? 0 : (1ull << (i - 64));
  }
}

void BitMatrix::apply(const uint64_t in[2], uint64_t out[2]) const {
  uint64_t a = 0, b = 0;
  for (int i = 0; i < 64; i++)
    if ((in[0] >> i) & 1) { a ^= col[i][0]; b ^= col[i][1]; }
  for (int i = 0; i < 64; i++)
    if ((in[1] >> i) & 1) { a ^= col[64 + i][0]; b ^= col[64 + i][1]; }
  out[0] = a;
  out[1] = b;
}

BitMatrix BitMatrix::mul(const BitMatrix &rhs) const {  // (*this) * rhs
  BitMatrix r;
  for (int i = 0; i < 128; i++) apply(rhs.col[i], r.col[i]);
  return r;
}

BitMatrix xs_step_matrix() {
  BitMatrix m;
  for (int i = 0; i < 128; i++) {
    uint64_t s[2] = {i < 64 ? (1ull << i) : 0, i < 64 ? 0 : (1ull << (i - 64))};
    xs_advance(s);
    m.col[i][0] = s[0];
    m.col[i][1] = s[1];
  }
  return m;
}

BitMatrix xs_jump_matrix(uint64_t k) {
  BitMatrix result, base = xs_step_matrix();
  result.identity();
  while (k) {
    if (k & 1) result = base.mul(result);
    k >>= 1;
    if (k) base = base.mul(base);
  }
  return result;
}

void xs_jump(uint64_t s[2], uint64_t k) {
  if (k == 0) return;
  if (k < 4096) {
    for (uint64_t i = 0; i < k; i++) xs_advance(s);
    return;
  }
  BitMatrix m = xs_jump_matrix(k);
  uint64_t o[2];
  m.apply(s, o);
  s[0] = o[0];
  s[1] = o[1];
}

// table[b][v] (16 x 256 entries of 2 x u64) = M * (v << 8b) : 16 lookups + xors apply M.
void xs_byte_tables(const BitMatrix &m, uint64_t *table) {
  for (int b = 0; b < 16; b++)
    for (int v = 0; v < 256; v++) {
      uint64_t a = 0, c = 0;
      for (int bit = 0; bit < 8; bit++)
        if ((v >> bit) & 1) {
          a ^= m.col[8 * b + bit][0];
          c ^= m.col[8 * b + bit][1];
        }
      table[(b * 256 + v) * 2 + 0] = a;
      table[(b * 256 + v) * 2 + 1] = c;
    }
}

}  // namespace pgcn

extern "C" {

void pgcn_rng_seed(uint64_t state[2]) {
  // hpdga-spring23/src/rand.cpp:6-14: x = rand(), y = rand() of an unseeded glibc rand().
  state[0] = 1804289383u;
  state[1] = 846930886u;
}

void pgcn_rng_seed_glibc(unsigned int seed, uint64_t state[2]) {
  // srand(seed); x = rand(); y = rand(): glibc rand() is random() on a TYPE_3 (128-byte)
  // state; a private one leaves the process's rand() alone.  seed 0 and 1 = unseeded.
  char buf[128];
  struct random_data rd;
  std::memset(&rd, 0, sizeof(rd));
  int32_t x = 0, y = 0;
  initstate_r(seed, buf, sizeof(buf), &rd);
  random_r(&rd, &x);
  random_r(&rd, &y);
  state[0] = (uint32_t)x;
  state[1] = (uint32_t)y;
}

void pgcn_rng_jump(uint64_t state[2], uint64_t k) { pgcn::xs_jump(state, k); }

int pgcn_rng_jump_table(uint64_t period, void *host_table) {
  if (!host_table) return PGCN_E_INVALID;
  pgcn::xs_byte_tables(pgcn::xs_jump_matrix(period), static_cast<uint64_t *>(host_table));
  return PGCN_OK;
}

}  // extern "C"
