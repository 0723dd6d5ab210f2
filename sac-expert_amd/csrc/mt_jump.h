// MT19937 jump-ahead coefficients for the segmented sampler (k_sac.hip, k_mtj_*).
//
// The raw word stream x[n] of MT19937 (before tempering) is a GF(2)-linear recurrence whose
// 19937-bit state advances by a fixed matrix T with characteristic polynomial phi (degree
// 19937).  Every word bit is a linear function of the state, so for any D with
//     x^D mod phi = sum_{i < 19937} c_i x^i
// the stream satisfies  x[n + D + j] = XOR_{i : c_i = 1} x[n + i + j]  for every j >= -623
// (relative to a state n whose 624-word window is x[n-624 .. n-1]; word n-624 holds only its
// top bit of state).  The segmented sampler uses it to start generating at k * L words past a
// key block from the first 20,561 words after it, instead of twisting the 623-word rounds in
// between on one workgroup.
//
// phi is found once per process by Berlekamp-Massey on one bit of a generated stream (it is
// irreducible, so any nonzero bit sequence of the generator has it as minimal polynomial).
#pragma once
#include <cstdint>

namespace sacx {

constexpr int MT_DEG = 19937;        // degree of phi
constexpr int MT_JUMP_WORDS = 624;   // uint32 words of one coefficient vector (bit i = c_i)

// c^(k) = x^(k * L) mod phi for k = 1 .. n, stored at out[(k - 1) * MT_JUMP_WORDS ...], bit i of
// the vector at word i >> 5, bit i & 31.  Deterministic; cached per (L, n) for the process.
void mt_jump_polys(int64_t L, int n, uint32_t* out);

// The same coefficients as the kernels read them (k_mtj_jump): for k = 1 .. n and coefficient
// chunk c of ch bits, the offsets of chunk (k, c)'s set-bit list, then the lists (bit index
// minus c * ch).  out: (n * nc + 1) offsets (relative to the lists' start) followed by the
// entries, nc = ceil(MT_DEG / ch); at most mt_jump_lists_words(n, ch) int32 words.
inline int64_t mt_jump_lists_words(int n, int ch) { return (int64_t)n * ((MT_DEG + ch - 1) / ch) + 1 + (int64_t)n * MT_DEG; }
int64_t mt_jump_lists(int64_t L, int n, int ch, int32_t* out);

}  // namespace sacx
