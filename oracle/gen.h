/*
 * oracle/gen.h — deterministic synthetic-input generator shared by every
 * side of the parity chain (TEST INFRASTRUCTURE, not product code).
 *
 * SplitMix64 (Steele, Lea & Flood 2014) with a 53-bit uniform mantissa.
 * Only exactly-rounded IEEE operations (+, -, *, /, sqrt) are used on the
 * generated uniforms, so the Python mirror in tests/gen.py reproduces every
 * array bit-for-bit on any machine.  Inputs that need transcendental
 * functions (the GP's y = sin(x) + noise) are generated once by the
 * reference harness and stored in tests/golden/ instead of regenerated.
 */
#ifndef SMG_ORACLE_GEN_H
#define SMG_ORACLE_GEN_H

#include <stdint.h>
#include <stddef.h>

typedef struct smg_rng {
  uint64_t s;
} smg_rng;

static inline smg_rng smg_rng_make(uint64_t seed) {
  smg_rng r;
  r.s = seed;
  return r;
}

static inline uint64_t smg_rng_next(smg_rng* r) {
  uint64_t z = (r->s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* uniform on [0, 1) with 53 random bits */
static inline double smg_rng_u01(smg_rng* r) {
  return (double)(smg_rng_next(r) >> 11) * (1.0 / 9007199254740992.0);
}

/* a + (b - a) * u, evaluated exactly in that order (no FMA contraction) */
static inline double smg_rng_unif(smg_rng* r, double a, double b) {
  volatile double w = (b - a) * smg_rng_u01(r);
  return a + w;
}

static inline void smg_fill_unif(uint64_t seed, size_t n, double a, double b,
                                 double* out) {
  smg_rng r = smg_rng_make(seed);
  for (size_t i = 0; i < n; ++i) out[i] = smg_rng_unif(&r, a, b);
}

/* y_i = (u < p) for Bernoulli draws */
static inline void smg_fill_bernoulli(uint64_t seed, size_t n, double p,
                                      int* out) {
  smg_rng r = smg_rng_make(seed);
  for (size_t i = 0; i < n; ++i) out[i] = smg_rng_u01(&r) < p ? 1 : 0;
}

#endif
