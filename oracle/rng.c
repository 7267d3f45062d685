/*
 * rng.c -- numpy legacy RandomState (MT19937) draws used by MAGICAL resets.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Reference RNG: base_env.py:134-141 (np.random.RandomState(seed)).  Draw
 * semantics restated from numpy's legacy generator (numpy/random/_legacy,
 * mt19937 seeding, random_standard_uniform, masked bounded integers,
 * random_interval); pinned bit-for-bit against numpy in tests/test_oracle_golden.py.
 */
#include "oracle.h"

void o_mt_seed(o_mt *s, uint32_t seed) {
    /* mt19937_seed: key[0]=seed; key[i] = 1812433253*(key[i-1]^(key[i-1]>>30)) + i */
    uint32_t v = seed;
    for (int i = 0; i < 624; i++) {
        s->key[i] = v;
        v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(i + 1);
    }
    s->pos = 624;
}

static void mt_gen(o_mt *s) {
    const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX_A = 0x9908b0dfu;
    int i;
    uint32_t y;
    for (i = 0; i < 624 - 397; i++) {
        y = (s->key[i] & UPPER) | (s->key[i + 1] & LOWER);
        s->key[i] = s->key[i + 397] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
    }
    for (; i < 623; i++) {
        y = (s->key[i] & UPPER) | (s->key[i + 1] & LOWER);
        s->key[i] = s->key[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
    }
    y = (s->key[623] & UPPER) | (s->key[0] & LOWER);
    s->key[623] = s->key[396] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
    s->pos = 0;
}

uint32_t o_mt_next32(o_mt *s) {
    if (s->pos == 624) mt_gen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double o_mt_double(o_mt *s) {
    int32_t a = (int32_t)(o_mt_next32(s) >> 5), b = (int32_t)(o_mt_next32(s) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* RandomState.uniform(lo, hi) = lo + (hi - lo) * random_sample() */
double o_mt_uniform(o_mt *s, double lo, double hi) {
    double range = hi - lo;
    return lo + range * o_mt_double(s);
}

static uint32_t gen_mask32(uint32_t max) {
    uint32_t m = max;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    return m;
}

/* RandomState.randint(lo, hi): masked rejection on 32-bit words, range < 2^32 */
int64_t o_mt_randint(o_mt *s, int64_t lo, int64_t hi) {
    uint64_t rng = (uint64_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    uint32_t mask = gen_mask32((uint32_t)rng), val;
    while ((val = (o_mt_next32(s) & mask)) > (uint32_t)rng) {}
    return lo + (int64_t)val;
}

/* random_interval(max): used by RandomState.shuffle */
uint64_t o_mt_interval(o_mt *s, uint64_t max) {
    if (max == 0) return 0;
    uint32_t mask = gen_mask32((uint32_t)max), val;
    while ((val = (o_mt_next32(s) & mask)) > (uint32_t)max) {}
    return val;
}
