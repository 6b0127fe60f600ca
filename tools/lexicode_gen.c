/* Offline regeneration of the small classic AprilTag families (tag16h5, tag25h9).
 *
 * Same lexicode procedure as tools/tag36h11_gen.c, for a d x d data grid:
 *
 *   V0 = java.util.Random(d*d*10000 + minham*100 + mincomplexity).nextLong()
 *        & (2^(d*d)-1)
 *   for k = 1 .. 2^(d*d):  V = V0 + k * 982451653  (mod 2^(d*d)), row-major,
 *                          MSB = top-left cell
 *     accept V iff its rotations are >= minham from it, its greedy rectangle
 *     complexity is >= mincomplexity, and it is >= minham from every rotation
 *     of every accepted code.
 *
 * (For tag36h11 the seed 361110 = 36*10000 + 11*100 + 10 carries the fitted
 * complexity threshold 10; this generator takes the threshold as a parameter
 * and tools/make_small_families.py selects it by the recalled tables.)
 *
 * Output: one line per accepted code, "id k code_rowmajor code_3x" (hex), the
 * 3.x code being the same pattern in the 3.x bit_x/bit_y order (the quadrant
 * spiral: rows y = 1.. of the upper triangle, rotated four times, the centre
 * cell last for odd d).
 *
 * Build: gcc -O2 tools/lexicode_gen.c -o /tmp/lexicode_gen
 * Usage: /tmp/lexicode_gen d minham mincomplexity
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint64_t u64;
static int D, NB, MINHAM, MINCOMPLEX;
static u64 kMask;
static const u64 kPrime = 982451653ULL;

static u64 java_next_long(u64 seed) {
    u64 s = (seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
    int32_t part[2];
    for (int i = 0; i < 2; ++i) {
        s = (s * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        part[i] = (int32_t)(s >> 16);
    }
    return ((u64)(int64_t)part[0] << 32) + (u64)(int64_t)part[1];
}

static int bit_at(u64 v, int y, int x) { return (int)((v >> (NB - 1 - (y * D + x))) & 1); }

static u64 rot90(u64 v) {
    u64 r = 0;
    for (int y = 0; y < D; ++y)
        for (int x = 0; x < D; ++x) r = (r << 1) | (u64)bit_at(v, D - 1 - x, y);
    return r;
}

static u64 g_rects[1024];
static int g_nrects;
static void build_rects(void) {
    g_nrects = 0;
    for (int y1 = 0; y1 < D; ++y1)
        for (int y0 = 0; y0 <= y1; ++y0)
            for (int x0 = 0; x0 < D; ++x0)
                for (int x1 = x0; x1 < D; ++x1) {
                    u64 m = 0;
                    for (int y = y0; y <= y1; ++y)
                        for (int x = x0; x <= x1; ++x) m |= 1ULL << (NB - 1 - (y * D + x));
                    g_rects[g_nrects++] = m;
                }
}

static int complexity(u64 t) {
    u64 tb = kMask & ~t, w = 0, b = 0;
    int cnt = 0;
    while (!(w == t && b == tb)) {
        int bs = -1;
        u64 bw = 0, bb = 0;
        for (int i = 0; i < g_nrects; ++i) {
            u64 m = g_rects[i];
            u64 nw = w | m, nb = b & ~m;
            int s = __builtin_popcountll(nw & t) + __builtin_popcountll(nb & tb);
            if (s >= bs) { bs = s; bw = nw; bb = nb; }
            nw = w & ~m; nb = b | m;
            s = __builtin_popcountll(nw & t) + __builtin_popcountll(nb & tb);
            if (s >= bs) { bs = s; bw = nw; bb = nb; }
        }
        w = bw; b = bb;
        if (++cnt >= MINCOMPLEX) return cnt;
    }
    return cnt;
}

static int g_bx[64], g_by[64];
static void build_layout(void) {
    int n = 0;
    for (int r = 0; r < 4; ++r)
        for (int y = 1; y <= D / 2; ++y)
            for (int x = y; x <= D - y; ++x) {
                int xx = x, yy = y; /* rotate (x, y) -> (D+1-y, x) r times */
                for (int i = 0; i < r; ++i) { int t = xx; xx = D + 1 - yy; yy = t; }
                g_bx[n] = xx; g_by[n] = yy; ++n;
            }
    if (D & 1) { g_bx[n] = D / 2 + 1; g_by[n] = D / 2 + 1; ++n; }
    if (n != NB) { fprintf(stderr, "layout has %d cells, want %d\n", n, NB); exit(1); }
}

static u64 to_3x(u64 rm) {
    u64 c = 0;
    for (int i = 0; i < NB; ++i) c = (c << 1) | (u64)bit_at(rm, g_by[i] - 1, g_bx[i] - 1);
    return c;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s d minham mincomplexity\n", argv[0]); return 2; }
    D = atoi(argv[1]); MINHAM = atoi(argv[2]); MINCOMPLEX = atoi(argv[3]);
    NB = D * D;
    if (D < 3 || D > 7 || NB > 63) return 2;
    kMask = (1ULL << NB) - 1;
    build_rects();
    build_layout();
    const u64 v0 = java_next_long((u64)(NB * 10000 + MINHAM * 100 + MINCOMPLEX)) & kMask;
    static u64 words[1 << 16];
    int nw = 0, ncodes = 0;
    for (u64 k = 1; k <= kMask + 1; ++k) {
        u64 v = (v0 + k * kPrime) & kMask;
        int ok = 1;
        for (int j = 0; j < nw && ok; ++j) ok = __builtin_popcountll(v ^ words[j]) >= MINHAM;
        if (!ok) continue;
        u64 r1 = rot90(v), r2 = rot90(r1), r3 = rot90(r2);
        if (__builtin_popcountll(v ^ r1) < MINHAM || __builtin_popcountll(v ^ r2) < MINHAM ||
            __builtin_popcountll(v ^ r3) < MINHAM)
            continue;
        if (complexity(v) < MINCOMPLEX) continue;
        printf("%d %llu 0x%llx 0x%llx\n", ncodes++, (unsigned long long)k, (unsigned long long)v,
               (unsigned long long)to_3x(v));
        words[nw++] = v; words[nw++] = r1; words[nw++] = r2; words[nw++] = r3;
    }
    fprintf(stderr, "done: %d codes\n", ncodes);
    return 0;
}
