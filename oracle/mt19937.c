/*
 * CPU oracle -- TEST INFRASTRUCTURE ONLY (see oracle/sac_oracle.py header).
 *
 * Plain-C restatement of the random stream the reference draws from: NumPy's
 * legacy ``RandomState`` (MT19937), as used by
 *   sac_eo/common/buffers.py:136           np.random.randint(current_size, size=B)
 *   sac_eo/actors/continuous_actors.py:351 np.random.normal(size=(B, A))
 *   sac_eo/common/seeding.py:12            np.random.seed(seed)
 * NumPy is a third-party dependency of the reference (unpinned; the legacy
 * stream is frozen by NEP 19).  The published algorithms restated here:
 *   - MT19937 init_genrand + twist + tempering (Matsumoto & Nishimura 1998,
 *     NumPy random/src/mt19937),
 *   - legacy bounded integers: masked rejection on 32-bit draws
 *     (NumPy random/src/distributions random_bounded_uint64, use_masked=1),
 *   - legacy_gauss: Marsaglia polar method with a cached second value,
 *   - random_standard_uniform: (a>>5, b>>6) 53-bit double.
 * Pinned bit-exactly against np.random.RandomState in tests/test_oracle.py
 * and by the committed vectors in tests/golden/rng_golden.npz.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -shared -fPIC).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define MT_N 624
#define MT_M 397
#define MATRIX_A 0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU

typedef struct {
    uint32_t key[MT_N];
    int32_t pos;
    int32_t has_gauss;
    double gauss;
} mto_state;

void mto_seed(mto_state *st, uint32_t seed) {
    for (int pos = 0; pos < MT_N; pos++) {
        st->key[pos] = seed;
        seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)pos + 1U;
    }
    st->pos = MT_N;
    st->has_gauss = 0;
    st->gauss = 0.0;
}

void mto_set_state(mto_state *st, const uint32_t *key, int32_t pos, int32_t has_gauss, double gauss) {
    memcpy(st->key, key, sizeof(st->key));
    st->pos = pos;
    st->has_gauss = has_gauss;
    st->gauss = gauss;
}

void mto_get_state(const mto_state *st, uint32_t *key, int32_t *pos, int32_t *has_gauss, double *gauss) {
    memcpy(key, st->key, sizeof(st->key));
    *pos = st->pos;
    *has_gauss = st->has_gauss;
    *gauss = st->gauss;
}

static uint32_t twist_word(uint32_t cur, uint32_t next, uint32_t far) {
    uint32_t y = (cur & UPPER_MASK) | (next & LOWER_MASK);
    return far ^ (y >> 1) ^ ((0U - (y & 1U)) & MATRIX_A);
}

static void mto_twist(mto_state *st) {
    int i;
    for (i = 0; i < MT_N - MT_M; i++)
        st->key[i] = twist_word(st->key[i], st->key[i + 1], st->key[i + MT_M]);
    for (; i < MT_N - 1; i++)
        st->key[i] = twist_word(st->key[i], st->key[i + 1], st->key[i + MT_M - MT_N]);
    st->key[MT_N - 1] = twist_word(st->key[MT_N - 1], st->key[0], st->key[MT_M - 1]);
    st->pos = 0;
}

static uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

uint32_t mto_next32(mto_state *st) {
    if (st->pos == MT_N) mto_twist(st);
    return temper(st->key[st->pos++]);
}

double mto_next_double(mto_state *st) {
    int32_t a = (int32_t)(mto_next32(st) >> 5), b = (int32_t)(mto_next32(st) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* legacy randint(high, size=n) for 1 <= high <= 2**32: masked rejection. */
int mto_randint(mto_state *st, int64_t high, int64_t n, int64_t *out) {
    if (high < 1 || high > 4294967296LL) return -1;
    uint64_t rng = (uint64_t)(high - 1);
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    for (int64_t i = 0; i < n; i++) {
        if (rng == 0) { out[i] = 0; continue; }
        if (rng == 0xFFFFFFFFULL) { out[i] = mto_next32(st); continue; }
        uint64_t val;
        while ((val = (mto_next32(st) & (uint32_t)mask)) > rng) {}
        out[i] = (int64_t)val;
    }
    return 0;
}

double mto_gauss(mto_state *st) {
    if (st->has_gauss) {
        st->has_gauss = 0;
        double g = st->gauss;
        st->gauss = 0.0;
        return g;
    }
    double f, x1, x2, r2;
    do {
        x1 = 2.0 * mto_next_double(st) - 1.0;
        x2 = 2.0 * mto_next_double(st) - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    f = sqrt(-2.0 * log(r2) / r2);
    st->gauss = f * x1;
    st->has_gauss = 1;
    return f * x2;
}

void mto_normal(mto_state *st, int64_t n, double *out) {
    for (int64_t i = 0; i < n; i++) out[i] = mto_gauss(st);
}

int64_t mto_state_size(void) { return (int64_t)sizeof(mto_state); }
