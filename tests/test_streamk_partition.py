"""The stream-K work split of the plane GEMMs (conv_p3_fwd.h, SK instantiations) on the host:
workgroup g owns iterations [g*T/G, (g+1)*T/G) of the flattened (tile, k-slot) space, and the
workgroups sharing tile t are g(f) .. g(l) with g(i) = ceil((i+1)*G/T) - 1 (f, l: the tile's first /
last iteration). Mirrors the kernel's integer math: every iteration is computed by exactly one
workgroup, every tile's shares are counted and indexed consistently (0 .. parts-1, the slab index
of splitk_gather), and parts never exceeds the slab reservation the binding makes
(sk_smax = min(G, ceil(nk / floor(T/G)) + 1))."""
import random


def g_of(i, G, T):
    return ((i + 1) * G + T - 1) // T - 1


def check(tiles, nk, G):
    T = tiles * nk
    G = min(G, T)
    q = T // G
    smax = min(G, -(-nk // q) + 1)
    owner = [None] * T
    shares = {}
    for g in range(G):
        it, end = g * T // G, (g + 1) * T // G
        while it < end:
            tile, kb = divmod(it, nk)
            n = min(nk - kb, end - it)
            f, l = tile * nk, tile * nk + nk - 1
            gf, gl = g_of(f, G, T), g_of(l, G, T)
            parts, part = gl - gf + 1, g - gf
            assert 0 <= part < parts <= smax, (tiles, nk, G, tile, part, parts, smax)
            shares.setdefault(tile, set()).add((part, parts))
            for i in range(it, it + n):
                assert owner[i] is None
                owner[i] = g
            it += n
    assert all(o is not None for o in owner)
    for tile, s in shares.items():
        parts = {p for _, p in s}
        assert len(parts) == 1 and sorted(p for p, _ in s) == list(range(parts.pop())), (tile, s)


def test_streamk_partition_covers_every_iteration_once():
    random.seed(0)
    for tiles, nk, G in [(196, 72, 256), (196, 72, 512), (98, 36, 256), (100, 144, 768), (7, 3, 256), (1, 1, 1),
                         (784, 2, 256), (25, 144, 300)]:
        check(tiles, nk, G)
    for _ in range(300):
        check(random.randint(1, 400), random.randint(1, 160), random.randint(1, 1024))
