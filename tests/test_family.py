"""tag36h11 codebook checks (CPU).

The 587 codewords are third-party data (cgpadwick/apriltag@3.3.0 tag36h11.c,
fetched by src/external/CMakeLists.txt:86-95, not vendored).  The pinned entries
are checked here arithmetically, without the upstream file:
  * ids 0..72, mapped to the 2.x row-major layout, lie on the generator
    progression v0 + k * 982451653 (mod 2^36), v0 = Java Random(361110).nextLong(),
    with k strictly increasing in id order;
  * ids 554 / 585 are the codes read from the reference's fixture photographs
    (tools/read_fixture_codes.py) and are found by the detector on those images
    (tests/test_oracle.py, tests/test_gpu_parity.py);
  * every pair of pinned codes keeps Hamming distance >= 11 over the four
    rotations (the family's minimum distance), and no code is within 11 of its
    own rotations;
  * the product library and the oracle carry the same table.
"""
import pytest

M36 = (1 << 36) - 1
PRIME = 982451653
# apriltag 3.x tag36h11 bit_x / bit_y (bit i is code bit 35 - i)
BX = [1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4, 1, 1, 1, 1, 1, 2, 2, 2, 3]
BY = [1, 1, 1, 1, 1, 2, 2, 2, 3, 1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4]


def java_next_long(seed):
    s = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def nxt():
        nonlocal s
        s = (s * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        r = s >> 16
        return r - (1 << 32) if r & (1 << 31) else r
    hi = nxt()
    lo = nxt()
    return ((hi << 32) + lo) & ((1 << 64) - 1)


def to_row_major(code):
    """3.x bit order -> 2.x row-major 6x6 (MSB = top-left)."""
    grid = [[0] * 6 for _ in range(6)]
    for i in range(36):
        grid[BY[i] - 1][BX[i] - 1] = (code >> (35 - i)) & 1
    v = 0
    for y in range(6):
        for x in range(6):
            v = (v << 1) | grid[y][x]
    return v


def rot90(v):
    g = [[(v >> (35 - (y * 6 + x))) & 1 for x in range(6)] for y in range(6)]
    out = 0
    for y in range(6):
        for x in range(6):
            out = (out << 1) | g[5 - x][y]
    return out


@pytest.fixture(scope="module")
def entries(oracle_mod):
    return oracle_mod.family_entries()


def test_product_and_oracle_tables_match(entries):
    import ros_vision_amd as rva
    assert rva.family_entries() == entries
    assert [i for i, _ in entries] == list(range(73)) + [554, 585]


def test_generator_progression(entries):
    v0 = java_next_long(361110) & M36
    assert v0 == 0xCE84479FA
    inv = pow(PRIME, -1, 1 << 36)
    ks = [((to_row_major(c) - v0) * inv) & M36 for i, c in entries]
    head = ks[:73]
    assert head == sorted(head) and len(set(head)) == 73 and head[0] == 2 and head[-1] == 409
    # the fixture codes lie far along the same progression, in id order
    assert ks[73] == 6235272729 and ks[74] == 42477048845


def test_minimum_hamming_distance(entries):
    vs = [to_row_major(c) for _, c in entries]
    rots = []
    for v in vs:
        r = [v]
        for _ in range(3):
            r.append(rot90(r[-1]))
        rots.append(r)
        assert min(bin(v ^ r[j]).count("1") for j in (1, 2, 3)) >= 11
    for a in range(len(vs)):
        for b in range(a + 1, len(vs)):
            assert min(bin(vs[a] ^ rb).count("1") for rb in rots[b]) >= 11, (entries[a][0], entries[b][0])
