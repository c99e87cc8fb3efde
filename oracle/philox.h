/* oracle/philox.h — TEST INFRASTRUCTURE (oracle only).
 *
 * Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11; Random123 reference constants).  The oracle's counter-RNG mode uses it
 * to reproduce, independently of the product code, the random stream defined in
 * DESIGN.md "RNG contract".  Known-answer vectors are checked in
 * tests/test_oracle_kat.py.
 */
#ifndef ORACLE_PHILOX_H
#define ORACLE_PHILOX_H
#include <stdint.h>

static inline void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                                        uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* Two 53-bit uniforms in [0,1) from one Philox block. */
// Four uniforms in [0,1) (x * 2^-32) from one Philox4x32-10 block for
// (pixel, stratum, bounce, slot) — DESIGN.md "RNG contract".
static inline void oracle_philox_u01x4(uint64_t seed, uint32_t pixel, uint32_t sample,
                                       uint32_t bounce, uint32_t slot, double out[4]) {
  uint32_t ctr[4] = {pixel, sample, bounce, slot};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t x[4];
  oracle_philox4x32_10(ctr, key, x);
  for (int k = 0; k < 4; ++k) out[k] = (double)x[k] * 0x1.0p-32;
}
#endif
