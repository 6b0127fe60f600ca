"""Row 8(f)4: shared game-piece preprocessing.

preprocess_image (src/game_piece_detection/src/game_piece_detection_node.cu:347-379):
cv::resize (INTER_LINEAR) to the network input, BGR->RGB (3 channels) or BGR->GRAY
(1 channel), x 1/255, NCHW float.  OpenCV is third-party and absent offline, so the
oracle (oracle/ao_gp.c) restates its 8-bit arithmetic -- parity against OpenCV
itself is UNPINNED (no fixture in the reference holds a preprocessed tensor).

CPU: the oracle against a float bilinear resize (torch, same half-pixel sampling)
within one gray level, plus closed-form cases.  GPU: the HIP path (standalone and
inside a BGR8 detection batch) bit-identical to the oracle.
"""
import ctypes as C

import numpy as np
import pytest
from PIL import Image

SIZES = [(1280, 720, 640, 640), (1280, 720, 640, 360), (1920, 1080, 416, 416), (640, 480, 640, 640),
         (640, 640, 320, 320), (100, 60, 333, 211)]


def _torch_ref(bgr, ow, oh):
    import torch
    t = torch.from_numpy(bgr[:, :, ::-1].copy()).permute(2, 0, 1)[None].double()
    return torch.nn.functional.interpolate(t, size=(oh, ow), mode="bilinear", align_corners=False)[0].numpy() / 255


@pytest.mark.parametrize("w,h,ow,oh", SIZES)
def test_oracle_close_to_float_bilinear(oracle_mod, w, h, ow, oh):
    rng = np.random.default_rng(w + oh)
    bgr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    out = oracle_mod.gp_preprocess(bgr, ow, oh, 3)
    assert out.shape == (3, oh, ow) and out.dtype == np.float32
    assert np.abs(out - _torch_ref(bgr, ow, oh)).max() <= 1.0 / 255 + 1e-6


def test_oracle_closed_forms(oracle_mod):
    rng = np.random.default_rng(7)
    bgr = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    # same size: the bytes themselves, planes in RGB order
    out = oracle_mod.gp_preprocess(bgr, 96, 64, 3)
    a = np.float32(1.0 / 255.0)
    assert np.array_equal(out, np.stack([bgr[:, :, 2], bgr[:, :, 1], bgr[:, :, 0]]).astype(np.float32) * a)
    # exact halving: INTER_AREA's 2x2 mean, rounded half up
    out = oracle_mod.gp_preprocess(bgr, 48, 32, 3)
    s = bgr.astype(np.int32)
    m = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
    assert np.array_equal(out, np.stack([m[:, :, 2], m[:, :, 1], m[:, :, 0]]).astype(np.float32) * a)
    # gray: BGR2GRAY fixed point of the resized pixel
    g = oracle_mod.gp_preprocess(bgr, 96, 64, 1)
    y = (s[:, :, 0] * 1868 + s[:, :, 1] * 9617 + s[:, :, 2] * 4899 + 8192) >> 14
    assert np.array_equal(g[0], y.astype(np.float32) * a)
    # a constant image stays constant at any scale
    c = np.full((37, 53, 3), (10, 200, 77), np.uint8)
    out = oracle_mod.gp_preprocess(c, 128, 91, 3)
    assert np.array_equal(np.unique(out[0]), [np.float32(77) * a]) and np.array_equal(np.unique(out[2]), [np.float32(10) * a])


# ---------------------------------------------------------------------------- GPU


def _bgr_cases():
    from ros_vision_amd import synth
    rng = np.random.default_rng(11)
    yield "random_720p", rng.integers(0, 256, (720, 1280, 3), dtype=np.uint8)
    gray, _ = synth.render_board(1280, 720, seed=3, ntags=15)
    tint = np.stack([gray, (gray.astype(np.int32) * 3 // 4).astype(np.uint8), 255 - gray], axis=2)
    yield "board_720p", tint
    import os
    rgb = np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "golden", "frc_reefscape_frame6141_rgb.png")))
    yield "reefscape_640", np.ascontiguousarray(rgb[:, :, ::-1])


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [3, 1])
def test_gpu_standalone_matches_oracle(oracle_mod, channels):
    import torch
    import ros_vision_amd as rva
    for name, bgr in _bgr_cases():
        h, w, _ = bgr.shape
        d_in = torch.from_numpy(bgr).cuda()
        for ow, oh in [(640, 640), (w // 2, h // 2), (416, 416), (w, h), (333, 211)]:
            d_out = torch.empty((channels, oh, ow), dtype=torch.float32, device="cuda")
            rva.game_piece_preprocess_device(d_in.data_ptr(), w, h, d_out.data_ptr(), ow, oh, channels,
                                             torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = oracle_mod.gp_preprocess(bgr, ow, oh, channels)
            assert np.array_equal(d_out.cpu().numpy(), want), (name, ow, oh, channels)


@pytest.mark.gpu
def test_gpu_fused_in_detection_batch(oracle_mod):
    """at_gp_enable: the tensor of every BGR8 frame of a batch comes out of the same
    launch sequence, bit-identical to the oracle; the detections are unchanged."""
    import ros_vision_amd as rva
    from ros_vision_amd import synth
    frames, grays = [], []
    for f in range(3):
        gray, _ = synth.render_board(1280, 720, seed=766000 + f, ntags=15)
        grays.append(gray)
        frames.append(np.ascontiguousarray(np.repeat(gray[:, :, None], 3, axis=2)))
    det = rva.GpuDetector(1280, 720, max_batch=3)
    base = det.detect_batch(frames, rva.AT_FMT_BGR8)
    det.enable_game_piece_input(640, 640, 3)
    got = det.detect_batch(frames, rva.AT_FMT_BGR8)
    assert [[d.id for d in fr] for fr in got] == [[d.id for d in fr] for fr in base]
    for f in range(3):
        assert det.game_piece_tensor_ptr(f) != 0
        assert np.array_equal(det.game_piece_tensor(f), oracle_mod.gp_preprocess(frames[f], 640, 640, 3))
    # a non-BGR batch has no tensor
    det.detect(synth.to_yuyv(grays[0]), rva.AT_FMT_YUYV)
    with pytest.raises(RuntimeError):
        det.game_piece_tensor(0)
