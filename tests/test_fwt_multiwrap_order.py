"""The reverse cascade's multi-wrap levels (h < M): the term order the kernels use.

Wavelet.reverse (Wavelet.java:277-303) scatters out[(2i + j) mod h] += (a_i sR_j) + (d_i wR_j)
for i ascending, then j ascending.  For h < M the kernels gather output k = 2U + p directly:
rev_pair_mw (compile-time h, U) takes for each i ascending j = p + 2((U - i) mod h/2) + m h,
m ascending; the STRICT line cascades (rev_pair_wrapped<..., ENUM>) take j = (k - 2i) mod h,
+ h, ...  Both must list exactly the scatter's (i, j) pairs for k, in the scatter's order --
the sums are then bit-identical to the reference's (the GPU tests check the values)."""
import pytest


def scatter_order(M, h, k):
    return [(i, j) for i in range(h // 2) for j in range(M) if (2 * i + j) % h == k]


def mw_order(M, h, U, p):
    half = h // 2
    out = []
    for i in range(half):
        s = ((U - i) % half + half) % half
        out += [(i, j) for j in range(p + 2 * s, M, h)]
    return out


def enum_order(M, h, k):
    out = []
    for i in range(h // 2):
        out += [(i, j) for j in range((k - 2 * i) & (h - 1), M, h)]
    return out


@pytest.mark.parametrize("M", list(range(2, 42, 2)))
def test_multiwrap_orders_match_the_scatter(M):
    h = 2
    while h < M:
        for k in range(h):
            ref = scatter_order(M, h, k)
            assert len(ref) == M // 2
            assert enum_order(M, h, k) == ref
            if M <= 20:
                assert mw_order(M, h, k // 2, k % 2) == ref
        h *= 2
