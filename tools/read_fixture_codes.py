"""Read the 36 data bits of the upright printed tag in each reference fixture image.

The reference's test data holds photographs of printed tag36h11 tags whose caption
states the id ("april.tag.Tag36h11, id = N"): colorimage.jpg (id 554) and
grayimage.jpg (id 585).  The codewords are third-party data (the un-vendored
tag36h11.c), so these photographs are the reference-held evidence
for those two entries.  This script finds the tag's outer black square with the
CPU oracle's quad stage, samples the 8x8 cell centres through the quad's
homography, thresholds them at the midpoint of the black border and the white
quiet zone, and prints the code in the apriltag 3.x bit order (bit_x / bit_y).
Reads /root/reference at generation time only; the result is committed in the
codebook include files.
"""
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ao  # noqa: E402  (checker library: only its quad stage is used)

SRC = "/root/reference/src/apriltags_cuda/test/data/"
BX = [1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4, 1, 1, 1, 1, 1, 2, 2, 2, 3]
BY = [1, 1, 1, 1, 1, 2, 2, 2, 3, 1, 2, 3, 4, 5, 2, 3, 4, 3, 6, 6, 6, 6, 6, 5, 5, 5, 4, 6, 5, 4, 3, 2, 5, 4, 3, 4]


def y_bt601(rgb):
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((269484 * r + 528482 * g + 102760 * b + (1 << 19) + (16 << 20)) >> 20).astype(np.uint8)


def homography(src, dst):
    A = []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y, -u])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y, -v])
    _, _, vt = np.linalg.svd(np.array(A, np.float64))
    return vt[-1].reshape(3, 3)


def read_code(gray, corners):
    """corners: outer black-square corners in image pixels, any order."""
    c = np.asarray(corners, np.float64)
    ctr = c.mean(0)
    ang = np.arctan2(c[:, 1] - ctr[1], c[:, 0] - ctr[0])
    c = c[np.argsort(ang)]                       # y-down image: TL, TR, BR, BL by angle from -pi
    k = int(np.argmin(c[:, 0] + c[:, 1]))        # top-left first
    c = np.roll(c, -k, axis=0)
    Hm = homography([(0, 0), (8, 0), (8, 8), (0, 8)], c)

    def sample(u, v):
        p = Hm @ np.array([u, v, 1.0])
        x, y = p[0] / p[2], p[1] / p[2]
        xi, yi = int(round(x)), int(round(y))
        return float(gray[yi - 2:yi + 3, xi - 2:xi + 3].mean())

    border = [sample(i + 0.5, j + 0.5) for i in range(8) for j in range(8) if i in (0, 7) or j in (0, 7)]
    quiet = [sample(-0.5, t + 0.5) for t in range(8)] + [sample(8.5, t + 0.5) for t in range(8)]
    thr = 0.5 * (np.mean(border) + np.mean(quiet))
    code = 0
    margin = 1e9
    for i in range(36):
        v = sample(BX[i] + 0.5, BY[i] + 0.5)
        code = (code << 1) | int(v > thr)
        margin = min(margin, abs(v - thr))
    return code, margin


def main():
    out = {}
    for name, fmt in [("colorimage.jpg", "rgb"), ("grayimage.jpg", "rgb")]:
        rgb = np.asarray(Image.open(SRC + name).convert("RGB"))
        gray = y_bt601(rgb)
        H, W = gray.shape
        orc = ao.Oracle(W, H)
        orc.detect(np.ascontiguousarray(gray), 2)
        best = None
        for corners, _ in orc.quads():
            area = 0.5 * abs(np.cross(corners[2] - corners[0], corners[3] - corners[1]))
            if best is None or area > best[0]:
                best = (area, corners)
        code, margin = read_code(gray, best[1])
        out[name] = code
        print("%s: code 0x%09x, min |sample - threshold| %.1f gray levels" % (name, code, margin))
    return out


if __name__ == "__main__":
    main()
