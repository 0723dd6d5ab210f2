"""The bf16 operand-shadow layout (sacx_internal.h wbf_pos / wbf_ld_of / wbf_per_of) against an
emulation of the consumer: the 32x32 bf16 forward tile splits K over 4 waves of `per` 16-wide
slabs, pairs each wave's slabs from its first, and packs lane group grp's operand as k = s0 + 4 grp
+ j then s1 + 4 grp + j (j < 4), zero past K and for a wave's unpaired last slab.  The shadow must
put every k < K exactly where that operand element is read, inside the row (< ld), and leave no
other position holding a k -- for the K of every shadowed matrix (S = 17, S + A = 23 and 393,
Humanoid S = 376, hidden 256) and a sweep.  The refresh kernel's inverse map (k_wbf_refresh) is
checked the same way.  CPU only: the formulas, restated from the header."""
import pytest


def per_of(K):
    return (((K + 15) >> 4) + 3) >> 2


def ld_of(K):
    return 4 * ((per_of(K) + 1) >> 1) * 32


def pos(k, per):
    s = k >> 4
    w = s // per
    i = s - w * per
    return (w * ((per + 1) >> 1) + (i >> 1)) * 32 + ((k >> 2) & 3) * 8 + (i & 1) * 4 + (k & 3)


def consumer_slots(K):
    """{shadow position: k} as the tile reads it (None: the operand element is zero)."""
    n_it = (K + 15) >> 4
    per = per_of(K)
    out = {}
    for w in range(4):
        it0, it1 = w * per, min(n_it, w * per + per)
        for it in range(it0, it1, 2):
            pp = w * ((per + 1) >> 1) + ((it - it0) >> 1)
            for grp in range(4):
                for u in range(2):
                    for j in range(4):
                        k = (it + u) * 16 + grp * 4 + j
                        ok = it + u < it1 and k < K
                        out[pp * 32 + grp * 8 + u * 4 + j] = k if ok else None
    return out


def refresh_inverse(p, K):
    """k_wbf_refresh's map from a shadow position to its k (None: zero)."""
    per, n_it = per_of(K), (K + 15) >> 4
    ppw = (per + 1) >> 1
    q, e = p // 8, p % 8
    pair, grp = q >> 2, q & 3
    w = pair // ppw
    i = (pair - w * ppw) * 2 + (e >> 2)
    sl = w * per + i
    k = sl * 16 + grp * 4 + (e & 3)
    return k if (i < per and sl < n_it and k < K) else None


@pytest.mark.parametrize("K", [1, 4, 16, 17, 23, 31, 64, 100, 128, 255, 256, 257, 376, 393, 512, 1000])
def test_shadow_layout_matches_consumer(K):
    per, ld = per_of(K), ld_of(K)
    slots = consumer_slots(K)
    assert all(p < ld for p in slots)
    placed = {pos(k, per): k for k in range(K)}
    assert len(placed) == K                                   # injective
    for p, k in placed.items():
        assert p < ld and slots.get(p) == k, (p, k, slots.get(p))
    for p, k in slots.items():
        assert (k is None) == (p not in placed)
    for p in range(ld):
        assert refresh_inverse(p, K) == placed.get(p)


def test_activation_shadows_are_dense_at_multiples_of_128():
    """abf rows have stride K: every position must hold a k (no zero slots) when K % 128 == 0."""
    for K in (128, 256, 384, 512):
        assert ld_of(K) == K
        assert sorted(pos(k, per_of(K)) for k in range(K)) == list(range(K))


def test_even_per_fast_path():
    """wbf_pos's branch for an even `per` (every wave starts on an even slab) equals the general form."""
    for K in range(1, 1100, 7):
        per = per_of(K)
        if per % 2:
            continue
        for k in range(K):
            s = k >> 4
            fast = (s >> 1) * 32 + ((k >> 2) & 3) * 8 + (s & 1) * 4 + (k & 3)
            assert fast == pos(k, per), (K, k)
