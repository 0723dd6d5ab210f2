// MT19937 jump-ahead coefficients (mt_jump.h): the characteristic polynomial by Berlekamp-Massey
// and x^(k L) mod phi by square-and-multiply over GF(2).  Host only; tests/mtjump_check.cpp
// checks the jumped windows against a directly generated stream.
#include "mt_jump.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <stdexcept>
#include <utility>
#include <vector>

namespace sacx {
namespace {

using Poly = std::vector<uint64_t>;   // bit i = coefficient of x^i

inline bool bit(const Poly& p, int64_t i) { return (p[(size_t)(i >> 6)] >> (i & 63)) & 1u; }
inline void flip(Poly& p, int64_t i) { p[(size_t)(i >> 6)] ^= 1ULL << (i & 63); }

// p ^= q << s over the first qbits bits of q (bits past p's end dropped)
void xor_shifted(Poly& p, const Poly& q, int64_t qbits, int64_t s) {
    const int64_t ws = s >> 6, bs = s & 63;
    const int64_t nq = (qbits + 63) >> 6;
    for (int64_t w = 0; w < nq; ++w) {
        const uint64_t v = q[(size_t)w];
        if (!v) continue;
        if ((size_t)(w + ws) < p.size()) p[(size_t)(w + ws)] ^= v << bs;
        if (bs && (size_t)(w + ws + 1) < p.size()) p[(size_t)(w + ws + 1)] ^= v >> (64 - bs);
    }
}

struct Charpoly {
    Poly phi;                    // monic, degree MT_DEG
    std::vector<int> terms;      // exponents e < MT_DEG with phi_e = 1
};

// Berlekamp-Massey on bit 0 of the raw words x[624 ..] of init_genrand(5489)'s stream
Charpoly find_charpoly() {
    const int N = 2 * MT_DEG;
    std::vector<uint32_t> x(624 + (size_t)N);
    x[0] = 5489U;
    for (int i = 1; i < 624; ++i) x[i] = 1812433253U * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    for (size_t n = 624; n < x.size(); ++n) {
        const uint32_t y = (x[n - 624] & 0x80000000U) | (x[n - 623] & 0x7fffffffU);
        x[n] = x[n - 227] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
    }
    // r: the sequence reversed, so that s[n - i] = r[N - 1 - n + i] is an ascending window
    const int NW = (N + 64) / 64 + 2;
    Poly r((size_t)NW, 0);
    for (int j = 0; j < N; ++j)
        if (x[624 + (size_t)(N - 1 - j)] & 1U) flip(r, j);
    const int CW = NW + 2;
    Poly C((size_t)CW, 0), B((size_t)CW, 0), T;
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int n = 0; n < N; ++n) {
        // d = s[n] ^ sum_{i=1..L} C_i s[n-i]
        const int64_t off = (int64_t)N - 1 - n;
        uint64_t acc = 0;
        const int nw = (L >> 6) + 1;
        for (int w = 0; w < nw; ++w) {
            const int64_t b0 = off + 64 * (int64_t)w;
            const int64_t wi = b0 >> 6, sh = b0 & 63;
            uint64_t win = r[(size_t)wi] >> sh;
            if (sh && (size_t)(wi + 1) < r.size()) win |= r[(size_t)(wi + 1)] << (64 - sh);
            uint64_t cw = C[(size_t)w];
            if (w == 0) cw &= ~1ULL;
            acc ^= cw & win;
        }
        const int d = (int)((x[624 + (size_t)n] & 1U) ^ (__builtin_popcountll(acc) & 1));
        if (!d) {
            ++m;
        } else if (2 * L <= n) {
            T = C;
            xor_shifted(C, B, (int64_t)B.size() * 64, m);
            L = n + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, (int64_t)B.size() * 64, m);
            ++m;
        }
    }
    if (L != MT_DEG) throw std::runtime_error("MT19937 characteristic polynomial: unexpected degree");
    Charpoly cp;
    cp.phi.assign((MT_DEG + 64) / 64 + 1, 0);
    for (int j = 0; j <= MT_DEG; ++j)      // phi_j = C_{L - j}
        if (bit(C, MT_DEG - j)) flip(cp.phi, j);
    for (int e = 0; e < MT_DEG; ++e)
        if (bit(cp.phi, e)) cp.terms.push_back(e);
    return cp;
}

const Charpoly& charpoly() {
    static const Charpoly cp = find_charpoly();
    return cp;
}

constexpr int PW = (2 * MT_DEG + 64) / 64 + 2;   // words of an unreduced product

// p (degree < 2 MT_DEG) mod phi, in place; the result has degree < MT_DEG
void reduce(Poly& p) {
    const Charpoly& cp = charpoly();
    for (int64_t b = 2 * (int64_t)MT_DEG; b >= MT_DEG; --b) {
        if (!bit(p, b)) continue;
        const int64_t s = b - MT_DEG;
        flip(p, b);
        for (int e : cp.terms) flip(p, e + s);
    }
}

Poly mulmod(const Poly& a, const Poly& b) {
    Poly p((size_t)PW, 0);
    for (int64_t i = 0; i < MT_DEG; ++i)
        if (bit(a, i)) xor_shifted(p, b, MT_DEG, i);
    reduce(p);
    p.resize((MT_DEG + 63) / 64 + 1);
    return p;
}

Poly sqrmod(const Poly& a) {
    Poly p((size_t)PW, 0);
    for (int64_t i = 0; i < MT_DEG; ++i)
        if (bit(a, i)) flip(p, 2 * i);
    reduce(p);
    p.resize((MT_DEG + 63) / 64 + 1);
    return p;
}

Poly xpow(uint64_t D) {
    Poly r((MT_DEG + 63) / 64 + 1, 0);
    r[0] = 1;
    int top = 63;
    while (top >= 0 && !((D >> top) & 1)) --top;
    const Charpoly& cp = charpoly();
    for (int k = top; k >= 0; --k) {
        r = sqrmod(r);
        if ((D >> k) & 1) {   // r *= x
            Poly s(r.size() + 1, 0);
            for (size_t w = 0; w < r.size(); ++w) {
                s[w] ^= r[w] << 1;
                s[w + 1] ^= r[w] >> 63;
            }
            if (bit(s, MT_DEG)) {
                flip(s, MT_DEG);
                for (int e : cp.terms) flip(s, e);
            }
            s.resize(r.size());
            r.swap(s);
        }
    }
    return r;
}

}  // namespace

void mt_jump_polys(int64_t L, int n, uint32_t* out) {
    static std::mutex mu;
    static std::map<std::pair<int64_t, int>, std::vector<uint32_t>> cache;
    if (L <= 0 || n <= 0) return;
    std::vector<uint32_t> v;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find({L, n});
        if (it != cache.end()) v = it->second;
    }
    if (v.empty()) {
        v.assign((size_t)n * MT_JUMP_WORDS, 0);
        const Poly c1 = xpow((uint64_t)L);
        Poly ck = c1;
        for (int k = 1; k <= n; ++k) {
            if (k > 1) ck = mulmod(ck, c1);
            for (int i = 0; i < MT_DEG; ++i)
                if (bit(ck, i)) v[(size_t)(k - 1) * MT_JUMP_WORDS + (i >> 5)] |= 1U << (i & 31);
        }
        std::lock_guard<std::mutex> g(mu);
        cache[{L, n}] = v;
    }
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
}

int64_t mt_jump_lists(int64_t L, int n, int ch, int32_t* out) {
    std::vector<uint32_t> c((size_t)n * MT_JUMP_WORDS);
    mt_jump_polys(L, n, c.data());
    const int nc = (MT_DEG + ch - 1) / ch;
    int32_t* off = out;
    int32_t* ent = out + (int64_t)n * nc + 1;
    int32_t e = 0;
    for (int k = 0; k < n; ++k)
        for (int j = 0; j < nc; ++j) {
            off[k * nc + j] = e;
            for (int i = j * ch; i < std::min(MT_DEG, (j + 1) * ch); ++i)
                if ((c[(size_t)k * MT_JUMP_WORDS + (i >> 5)] >> (i & 31)) & 1U) ent[e++] = i - j * ch;
        }
    off[(int64_t)n * nc] = e;
    return (int64_t)n * nc + 1 + e;
}

}  // namespace sacx
