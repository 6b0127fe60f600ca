"""Adversarial frames for the CCL: 1-px-featured patterns whose
components run through every block row of a CCL tile, so the unions of k_thr_ccl's
waves (and the finds that follow them, with no barrier between) race inside a tile,
and whose long chains cross tile borders (k_ccl_merge / k_ccl_border).

* interleaved combs: a fg comb from the top bar and one from the bottom bar, teeth
  every other column, so the background between them is ONE 4-connected serpentine
  through the whole region (its label, the minimum node id, sits at one end);
* square spirals: a 1-px fg line with a 1-px bg gap between turns;
* slope-1 staircases: 8-connected fg chains with 4-disconnected bg diagonals between;
* combs turned by 90 degrees (horizontal teeth: the serpentine crosses every wave's
  block rows once per tooth).

Regions of random size and offset (seeded) tile a decimated canvas, so the
patterns straddle CCL tile borders at every phase; each decimated pixel becomes a
2x2 full-resolution block of gray 230 (fg) or 25 (bg).  Test data only.
"""
import numpy as np


def comb(h, w):
    p = np.zeros((h, w), np.uint8)
    p[0] = p[h - 1] = 1
    for x in range(w):
        if x % 4 == 0:
            p[0:h - 2, x] = 1
        elif x % 4 == 2:
            p[2:h, x] = 1
    return p


def spiral(h, w):
    p = np.zeros((h, w), np.uint8)
    y0, x0, y1, x1 = 0, 0, h - 1, w - 1
    while y1 - y0 >= 2 and x1 - x0 >= 2:
        p[y0, x0:x1 + 1] = 1
        p[y0:y1 + 1, x1] = 1
        p[y1, x0 + 2:x1 + 1] = 1
        p[y0 + 2:y1 + 1, x0] = 1
        y0 += 2
        x0 += 2
        y1 -= 2
        x1 -= 2
        if y1 >= y0 and x1 >= x0:
            p[y0 - 1, x0 - 1] = 1  # the step into the next turn
    return p


def stairs(h, w):
    yy, xx = np.mgrid[0:h, 0:w]
    return (((xx + yy) % 3) == 0).astype(np.uint8)


def comb_turned(h, w):
    return comb(w, h).T.copy()


def canvas(hd, wd, seed):
    """Decimated canvas (1 = fg) of pattern regions (seeded sizes, offsets, kinds)."""
    rng = np.random.default_rng(seed)
    c = np.zeros((hd, wd), np.uint8)
    gens = [comb, spiral, stairs, comb_turned]
    y = int(rng.integers(0, 9))
    while y < hd - 8:
        rh = int(rng.integers(24, 72))
        x = int(rng.integers(0, 17))
        while x < wd - 8:
            rw = int(rng.integers(40, 140))
            hh, ww = min(rh, hd - y), min(rw, wd - x)
            c[y:y + hh, x:x + ww] = gens[int(rng.integers(0, len(gens)))](hh, ww)
            x += ww + int(rng.integers(1, 4))
        y += rh + int(rng.integers(1, 4))
    return c


def frame(width, height, seed):
    """GRAY8 frame (height, width): the canvas at full resolution, 230 / 25."""
    c = canvas(height // 2, width // 2, seed)
    return np.where(np.kron(c, np.ones((2, 2), np.uint8)) > 0, 230, 25).astype(np.uint8)
