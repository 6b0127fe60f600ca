/* CPU oracle for the shared game-piece preprocessing.
 *
 * TEST INFRASTRUCTURE ONLY (never linked into the product).  Restates
 * preprocess_image() of src/game_piece_detection/src/game_piece_detection_node.cu:347-379:
 *   cv::resize(img, resized, Size(iw, ih))            default INTER_LINEAR, 8UC3
 *   cvtColor(BGR2RGB) (3 channels) or cvtColor(BGR2GRAY) (1 channel)
 *   convertTo(CV_32F, 1/255)
 *   HWC -> CHW (NCHW, batch 1)
 * OpenCV 4.9.0 is third-party and not in the image (src/external/CMakeLists.txt
 * fetches it), so its 8-bit arithmetic is restated from its published sources
 * (imgproc/src/resize.cpp, color_rgb.simd.hpp) -- PARITY UNPINNED: no fixture in
 * the reference holds a preprocessed tensor.
 *
 * resize, 8U, INTER_LINEAR (hal::resize -> resizeGeneric_ with HResizeLinear /
 * VResizeLinear<uchar, int, short, FixedPtCast<int, uchar, 22>>):
 *   scale_x = 1 / ((double)ow / w), scale_y likewise;
 *   when both scales are exactly 2 the call is rerouted to INTER_AREA's fast
 *   2x2 path: dst = (s00 + s01 + s10 + s11 + 2) >> 2;
 *   otherwise, per output column: fx = (float)((dx + 0.5) * scale_x - 0.5),
 *   sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0); sx >= w - 1 ->
 *   (sx, fx) = (w - 1, 0) and the column takes S[sx] * 2048 alone (xmax);
 *   alpha = (saturate_cast<short>((1 - fx) * 2048), saturate_cast<short>(fx * 2048));
 *   per output row the same with sy, fy -> beta, and the two source rows sy, sy + 1
 *   clamped to [0, h - 1];
 *   horizontal: H = S[sx] * a0 + S[sx + 1] * a1 (int);
 *   vertical:   dst = (((b0 * (H0 >> 4)) >> 16) + ((b1 * (H1 >> 4)) >> 16) + 2) >> 2.
 * BGR2GRAY, 8U: Y = (B * 1868 + G * 9617 + R * 4899 + (1 << 13)) >> 14.
 * convertTo: (float)v * (float)(1.0 / 255.0).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "ao_oracle.h"

static short sat_short(float v) {
  const long r = lrintf(v); /* cvRound: round half to even */
  return (short)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}

/* resize of one 8-bit 3-channel image to ow x oh (BGR order kept) */
static void resize_bgr(const uint8_t *src, int w, int h, uint8_t *dst, int ow, int oh) {
  const double scale_x = 1. / ((double)ow / w), scale_y = 1. / ((double)oh / h);
  const int iscale_x = (int)lrint(scale_x), iscale_y = (int)lrint(scale_y);
  const double eps = 2.220446049250313e-16;
  if (fabs(scale_x - iscale_x) < eps && fabs(scale_y - iscale_y) < eps && iscale_x == 2 && iscale_y == 2) {
    for (int dy = 0; dy < oh; dy++)
      for (int dx = 0; dx < ow; dx++)
        for (int c = 0; c < 3; c++) {
          const uint8_t *s0 = src + ((size_t)(2 * dy) * w + 2 * dx) * 3 + c, *s1 = s0 + (size_t)w * 3;
          dst[((size_t)dy * ow + dx) * 3 + c] = (uint8_t)((s0[0] + s0[3] + s1[0] + s1[3] + 2) >> 2);
        }
    return;
  }
  int *xofs = (int *)malloc(sizeof(int) * ow), *xone = (int *)malloc(sizeof(int) * ow);
  short *alpha = (short *)malloc(sizeof(short) * 2 * ow);
  for (int dx = 0; dx < ow; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    xone[dx] = 0;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= w) { xone[dx] = 1; if (sx >= w - 1) { fx = 0; sx = w - 1; } }
    xofs[dx] = sx;
    alpha[2 * dx] = sat_short((1.f - fx) * 2048);
    alpha[2 * dx + 1] = sat_short(fx * 2048);
  }
  /* xmax: columns from the first one whose sx + 1 >= w take S[sx] * 2048 */
  int xmax = ow;
  for (int dx = 0; dx < ow; dx++)
    if (xone[dx]) { xmax = dx; break; }
  int *H0 = (int *)malloc(sizeof(int) * ow * 3), *H1 = (int *)malloc(sizeof(int) * ow * 3);
  for (int dy = 0; dy < oh; dy++) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
    int r0 = sy, r1 = sy + 1;
    r0 = r0 < 0 ? 0 : r0 > h - 1 ? h - 1 : r0;
    r1 = r1 < 0 ? 0 : r1 > h - 1 ? h - 1 : r1;
    for (int k = 0; k < 2; k++) {
      const uint8_t *S = src + (size_t)(k ? r1 : r0) * w * 3;
      int *Hk = k ? H1 : H0;
      for (int dx = 0; dx < ow; dx++)
        for (int c = 0; c < 3; c++) {
          const int sx = xofs[dx] * 3 + c;
          Hk[dx * 3 + c] = dx < xmax ? S[sx] * alpha[2 * dx] + S[sx + 3] * alpha[2 * dx + 1] : S[sx] * 2048;
        }
    }
    for (int i = 0; i < ow * 3; i++)
      dst[(size_t)dy * ow * 3 + i] = (uint8_t)((((b0 * (H0[i] >> 4)) >> 16) + ((b1 * (H1[i] >> 4)) >> 16) + 2) >> 2);
  }
  free(xofs); free(xone); free(alpha); free(H0); free(H1);
}

int ao_gp_preprocess(const uint8_t *bgr, int w, int h, float *out, int ow, int oh, int channels) {
  if (!bgr || !out || w < 2 || h < 2 || ow < 1 || oh < 1 || (channels != 1 && channels != 3)) return -1;
  uint8_t *rs = (uint8_t *)malloc((size_t)ow * oh * 3);
  resize_bgr(bgr, w, h, rs, ow, oh);
  const float a = (float)(1.0 / 255.0);
  const size_t plane = (size_t)ow * oh;
  for (size_t i = 0; i < plane; i++) {
    const int B = rs[3 * i], G = rs[3 * i + 1], R = rs[3 * i + 2];
    if (channels == 3) {
      out[i] = (float)R * a;
      out[plane + i] = (float)G * a;
      out[2 * plane + i] = (float)B * a;
    } else {
      out[i] = (float)((B * 1868 + G * 9617 + R * 4899 + (1 << 13)) >> 14) * a;
    }
  }
  free(rs);
  return 0;
}
