"""Build the real-image fixtures from the reference's own test data.

The reference test (test/gpu_detector_test.cu:40-47) does
imread(colorimage.jpg) -> cvtColor(BGR2YUV_YUYV) -> GpuDetector::Detect.
OpenCV is absent offline, so the JPEG is decoded once here with PIL and the
Y plane is computed with OpenCV's BT.601 fixed-point formula (the one the
YUYV conversion uses, ITUR_BT_601_SHIFT = 20).  The result is committed as a
lossless PNG so JPEG-decoder differences can never move the fixture.
Reads /root/reference at generation time only.
"""
import numpy as np
from PIL import Image

SRC = "/root/reference/src/apriltags_cuda/test/data/"
DST = "/root/repo/tests/golden/"


def y_bt601(rgb: np.ndarray) -> np.ndarray:
    r = rgb[..., 0].astype(np.int64)
    g = rgb[..., 1].astype(np.int64)
    b = rgb[..., 2].astype(np.int64)
    y = (269484 * r + 528482 * g + 102760 * b + (1 << 19) + (16 << 20)) >> 20
    return y.astype(np.uint8)


# real-world frames without tags from the reference's game-piece data (outdoor
# textures: many quads, no detections) -- natural-image parity cases
EXTRA = {"frc_rebuilt_frame1": "/root/reference/src/game_piece_detection/data/rebuilt/frame1.png",
         "frc_reefscape_frame6141": "/root/reference/src/game_piece_detection/data/reefscape/frame_6141.jpg"}

if __name__ == "__main__":
    for name in ["colorimage", "colorimage_notags", "grayimage"]:
        rgb = np.asarray(Image.open(SRC + name + ".jpg").convert("RGB"))
        Image.fromarray(y_bt601(rgb)).save(DST + name + "_y.png", optimize=True)
        print(name, rgb.shape)
    for name, path in EXTRA.items():
        rgb = np.asarray(Image.open(path).convert("RGB"))
        Image.fromarray(y_bt601(rgb)).save(DST + name + "_y.png", optimize=True)
        print(name, rgb.shape)
    # colour input of the game-piece preprocessing row (8(f)4): the 640x640 frame
    # as decoded, RGB PNG (the tests flip it to the node's bgr8)
    rgb = np.asarray(Image.open(EXTRA["frc_reefscape_frame6141"]).convert("RGB"))
    Image.fromarray(rgb).save(DST + "frc_reefscape_frame6141_rgb.png", optimize=True)
    print("frc_reefscape_frame6141_rgb", rgb.shape)
