"""Seeded synthetic tag boards (tag36h11 unless a
family is named).

A frame is a mid-gray background with ``ntags`` tags on a jittered grid; each
tag gets a random side length, rotation and perspective (corner jitter), is
rendered with bilinear interpolation from a (d+4)x(d+4)-cell bitmap (white
quiet zone, black border, d x d data cells in the apriltag 3.x bit layout; d = 6
for tag36h11, 5 for tag25h9, 4 for tag16h5) and the frame gets Gaussian noise.  Output is the gray plane or
packed YUYV with U = V = 128 (what cvtColor(BGR2YUV_YUYV) produces for a gray
image, apriltags_cuda_detector.cu:401).  Stream frames (configs C2-C4) carry
ids 10f .. 10f+ntags-1 mod 587, so a run of frames walks
the whole tag36h11 family.
"""
import numpy as np

# tag36h11 bit layout (apriltag 3.x), data cells in border coordinates 1..6
BIT_X = [1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4, 1, 1, 1, 1, 1, 2, 2, 2, 3]
BIT_Y = [1, 1, 1, 1, 1, 2, 2, 2, 3, 1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4]

# data grid side of the classic families the detector supports
FAMILY_D = {"tag36h11": 6, "tag25h9": 5, "tag16h5": 4}


def family_layout(family: str = "tag36h11"):
    """3.x bit_x / bit_y of a classic family: the upper triangle of the top-left
    quadrant row by row, rotated by 90 degrees three more times ((x, y) ->
    (d+1-y, x)), the centre cell last for odd d."""
    d = FAMILY_D[family]
    xs, ys = [], []
    for r in range(4):
        for y in range(1, d // 2 + 1):
            for x in range(y, d - y + 1):
                xx, yy = x, y
                for _ in range(r):
                    xx, yy = d + 1 - yy, xx
                xs.append(xx)
                ys.append(yy)
    if d % 2:
        xs.append(d // 2 + 1)
        ys.append(d // 2 + 1)
    return xs, ys


def tag_cells(code: int, family: str = "tag36h11") -> np.ndarray:
    """(d+4)x(d+4) cell image (1 = white) of a codeword incl. the quiet zone."""
    d = FAMILY_D[family]
    n = d * d
    bx, by = family_layout(family)
    cells = np.ones((d + 4, d + 4), np.float32)
    cells[1:d + 3, 1:d + 3] = 0.0  # black border ring
    for i in range(n):
        if (code >> (n - 1 - i)) & 1:
            cells[by[i] + 1, bx[i] + 1] = 1.0
    return cells


def homography(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    A = []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y, -u])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y, -v])
    _, _, vt = np.linalg.svd(np.asarray(A, np.float64))
    Hm = vt[-1].reshape(3, 3)
    return Hm / Hm[2, 2]


def _codes(family: str = "tag36h11"):
    from .detector import family_entries  # codebook lives in the C library
    return dict(family_entries(family))


def render_board(width: int, height: int, seed: int, ntags: int = 15, noise_sigma: float = 2.0,
                 side_range=(64, 128), ids=None, background: int = 128, codes=None, family: str = "tag36h11"):
    """Render one gray frame; returns (gray uint8 [H,W], list of (id, corners[4,2]))."""
    rng = np.random.default_rng(seed)
    codes = codes if codes is not None else _codes(family)
    nc = FAMILY_D[family] + 4  # cells across, quiet zone included
    known = sorted(codes)
    if ids is None:
        start = int(rng.integers(0, len(known)))
        ids = [known[(start + j) % len(known)] for j in range(ntags)]
    img = np.full((height, width), float(background), np.float32)
    rows = int(np.floor(np.sqrt(ntags * height / width))) or 1
    cols = int(np.ceil(ntags / rows))
    cw, ch = width / cols, height / rows
    truth = []
    sup = 8  # bitmap pixels per cell
    for j, tid in enumerate(ids):
        r, c = divmod(j, cols)
        side = float(rng.uniform(*side_range))
        side = min(side, 0.8 * min(cw, ch))
        cx = (c + 0.5) * cw + rng.uniform(-0.08, 0.08) * cw
        cy = (r + 0.5) * ch + rng.uniform(-0.08, 0.08) * ch
        ang = np.deg2rad(rng.uniform(-10, 10))
        # square of the full tag (quiet zone included), then perspective jitter
        half = side / 2 * nc / (nc - 2)
        base = np.array([[-half, -half], [half, -half], [half, half], [-half, half]])
        rot = np.array([[np.cos(ang), -np.sin(ang)], [np.sin(ang), np.cos(ang)]])
        corners = base @ rot.T + np.array([cx, cy])
        corners += rng.uniform(-0.15, 0.15, size=(4, 2)) * half * 0.5
        src = np.array([[0, 0], [nc, 0], [nc, nc], [0, nc]], np.float64)
        Hm = homography(src, corners)
        Hinv = np.linalg.inv(Hm)
        bmp = np.kron(tag_cells(codes[tid], family), np.ones((sup, sup), np.float32)) * 255.0
        x0, y0 = np.floor(corners.min(0)).astype(int) - 1
        x1, y1 = np.ceil(corners.max(0)).astype(int) + 1
        x0, y0, x1, y1 = max(x0, 0), max(y0, 0), min(x1, width - 1), min(y1, height - 1)
        xs, ys = np.meshgrid(np.arange(x0, x1 + 1), np.arange(y0, y1 + 1))
        pts = np.stack([xs.ravel() + 0.5, ys.ravel() + 0.5, np.ones(xs.size)])
        tp = Hinv @ pts
        u, v = tp[0] / tp[2], tp[1] / tp[2]
        inside = (u >= 0) & (u < nc) & (v >= 0) & (v < nc)
        bu, bv = u * sup - 0.5, v * sup - 0.5
        iu = np.clip(np.floor(bu).astype(int), 0, nc * sup - 2)
        iv = np.clip(np.floor(bv).astype(int), 0, nc * sup - 2)
        fu = np.clip(bu - iu, 0, 1)
        fv = np.clip(bv - iv, 0, 1)
        val = (bmp[iv, iu] * (1 - fu) * (1 - fv) + bmp[iv, iu + 1] * fu * (1 - fv) +
               bmp[iv + 1, iu] * (1 - fu) * fv + bmp[iv + 1, iu + 1] * fu * fv)
        flat = img[y0:y1 + 1, x0:x1 + 1].ravel()
        flat[inside] = val[inside]
        img[y0:y1 + 1, x0:x1 + 1] = flat.reshape(ys.shape)
        # tag black-border corners (cells 1 and nc-1) in image space
        bc = np.array([[1, 1], [nc - 1, 1], [nc - 1, nc - 1], [1, nc - 1]], np.float64)
        hb = Hm @ np.vstack([bc.T, np.ones(4)])
        truth.append((tid, (hb[:2] / hb[2]).T))
    if noise_sigma > 0:
        img += rng.normal(0.0, noise_sigma, size=img.shape).astype(np.float32)
    gray = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    return gray, truth


def render_dots(width: int, height: int, seed: int, side: int = 20, pitch: int = 40, noise_sigma: float = 2.0):
    """Dark squares on a light background on a jittered grid: every square is a
    blob pair that fits a quad (more accepted quads than tags fit in a frame)."""
    rng = np.random.default_rng(seed)
    img = np.full((height, width), 220.0, np.float32)
    n = 0
    for y in range(pitch // 2, height - pitch // 2 - side, pitch):
        for x in range(pitch // 2, width - pitch // 2 - side, pitch):
            jx, jy = rng.integers(-pitch // 6, pitch // 6 + 1, size=2)
            img[y + jy:y + jy + side, x + jx:x + jx + side] = 30.0
            n += 1
    if noise_sigma > 0:
        img += rng.normal(0.0, noise_sigma, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), n


def render_edge_board(width: int, height: int, seed: int, codes=None, family: str = "tag36h11"):
    """A board whose tags and blobs touch the right and bottom image borders: the
    partial last tile column / row of every tiled kernel at geometries whose
    decimated size is not a multiple of the tile (800x600 -> 400x300, the deployed
    camera of system_config.json:21-25).  A tag board fills the frame; tags are
    pasted with their quiet zone flush against the right edge, the bottom edge and
    the bottom-right corner (and one cut by the right edge); dark bars and a
    checker strip cross both borders.  Returns (gray, ids of the pasted tags)."""
    rng = np.random.default_rng(seed)
    codes = codes if codes is not None else _codes(family)
    known = sorted(codes)
    gray, truth = render_board(width, height, seed=seed, ntags=6, side_range=(56, 80), codes=codes, family=family)
    img = gray.astype(np.float32)
    ids = [t[0] for t in truth]
    used = set(ids)
    free = [k for k in known if k not in used]
    rng.shuffle(free)
    side = min(width, height) // 5

    def tag_crop(s, tid, sd):
        """One tag (quiet zone included) cropped to its bounding box."""
        sub, _ = render_board(s, s, seed=sd, ntags=1, side_range=(0.55 * s,) * 2, ids=[tid], codes=codes,
                              family=family, noise_sigma=0.0, background=128)
        ys, xs = np.nonzero(sub != 128)
        return sub[ys.min():ys.max() + 1, xs.min():xs.max() + 1].astype(np.float32)

    # dark bars crossing the right border, light bars crossing the bottom one, a
    # checker strip along the bottom rows (small blobs cut by the border)
    for k in range(4):
        yb = int(rng.integers(8, height - 40))
        img[yb:yb + int(rng.integers(6, 20)), width - int(rng.integers(12, 60)):] = 20.0
        xb = int(rng.integers(8, width - 40))
        img[height - int(rng.integers(12, 60)):, xb:xb + int(rng.integers(6, 20))] = 235.0
    yy, xx = np.mgrid[0:10, 0:width]
    img[height - 10:, :] = np.where(((xx // 5) + (yy // 5)) & 1, 230.0, 25.0)
    s = side
    # (anchor x or None = right-flush, anchor y or None = bottom-flush, gap to the border)
    spots = [(None, (height - s) // 3, 0), (width // 3, None, 1), (None, None, 2), (None, 2, 1)]
    for (ax, ay, gap) in spots:
        tid = free.pop()
        crop = tag_crop(s, tid, int(rng.integers(1 << 30)))
        h, w = crop.shape
        x0 = width - w - gap if ax is None else ax
        y0 = height - h - gap if ay is None else ay
        region = img[y0:y0 + h, x0:x0 + w]
        img[y0:y0 + h, x0:x0 + w] = np.where(crop != 128, crop, region)
        ids.append(tid)
    # a tag cut by the right border (its quads are partial: both sides must agree on them)
    crop = tag_crop(s, free.pop(), seed + 1)
    h, w = crop.shape
    y0 = (2 * (height - s)) // 3
    region = img[y0:y0 + h, width - w // 2:]
    img[y0:y0 + h, width - w // 2:] = np.where(crop[:, :w // 2] != 128, crop[:, :w // 2], region)
    img += rng.normal(0.0, 2.0, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), ids


def to_yuyv(gray: np.ndarray) -> np.ndarray:
    """Pack a gray plane as YUYV 4:2:2 (Y0 U Y1 V) with U = V = 128."""
    h, w = gray.shape
    out = np.empty((h, 2 * w), np.uint8)
    out[:, 0::2] = gray
    out[:, 1::2] = 128
    return out


def stream_ids(frame: int, ntags: int = 15, nfamily: int = 587):
    """Config C2 ids of one frame: 10f .. 10f+ntags-1 mod 587, unique per frame."""
    return [(10 * frame + j) % nfamily for j in range(ntags)]


def stream_frame(width: int, height: int, frame: int, camera: int = 0, ntags: int = 15, codes=None):
    """Config C2/C3 frame: seed 766000 + frame (+ camera * 10**6), ids stream_ids(frame)."""
    codes = codes if codes is not None else _codes()
    gray, truth = render_board(width, height, seed=766000 + frame + camera * 10 ** 6, ntags=ntags,
                               ids=stream_ids(frame, ntags, len(codes)), codes=codes)
    return to_yuyv(gray), gray, truth
