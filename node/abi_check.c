/* abi_check.c -- a plain C11 consumer of include/at_api.h.
 *
 * Compile-time: the struct layouts every binding mirrors (ctypes in
 * ros_vision_amd/detector.py, the node core, INTEGRATION.md's bindings) are
 * pinned with _Static_assert, so an ABI drift fails the build of this file.
 *   abi_check layout                      prints the layout as JSON (no GPU)
 *   abi_check detect W H FMT FRAME_FILE   one at_detect on the GPU; detections as JSON
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/at_api.h"

_Static_assert(AT_ABI_VERSION == 5, "at_api.h ABI version");
_Static_assert(sizeof(at_camera) == 72, "at_camera");
_Static_assert(sizeof(at_config) == 72, "at_config");
_Static_assert(offsetof(at_config, family) == 8 && offsetof(at_config, decode_sharpening) == 24 &&
                   offsetof(at_config, cos_critical_rad) == 48 && offsetof(at_config, tag_size) == 64,
               "at_config layout");
_Static_assert(sizeof(at_detection) == 168, "at_detection");
_Static_assert(offsetof(at_detection, H) == 16 && offsetof(at_detection, c) == 88 && offsetof(at_detection, p) == 104,
               "at_detection layout");
_Static_assert(sizeof(at_pose) == 112 && offsetof(at_pose, R) == 8 && offsetof(at_pose, err) == 104, "at_pose");
_Static_assert(sizeof(at_tag_detection) == 72 && offsetof(at_tag_detection, robot) == 32 &&
                   offsetof(at_tag_detection, err) == 64,
               "at_tag_detection");
_Static_assert(sizeof(at_quad_record) == 52 && offsetof(at_quad_record, corners) == 20, "at_quad_record");

#define OFF(T, f) printf("\"%s.%s\": %zu, ", #T, #f, offsetof(T, f))

static int layout(void) {
  printf("{\"abi_version\": %d, ", AT_ABI_VERSION);
  printf("\"sizeof.at_camera\": %zu, \"sizeof.at_config\": %zu, \"sizeof.at_detection\": %zu, ", sizeof(at_camera),
         sizeof(at_config), sizeof(at_detection));
  printf("\"sizeof.at_pose\": %zu, \"sizeof.at_tag_detection\": %zu, \"sizeof.at_quad_record\": %zu, ",
         sizeof(at_pose), sizeof(at_tag_detection), sizeof(at_quad_record));
  OFF(at_config, width); OFF(at_config, height); OFF(at_config, family); OFF(at_config, quad_decimate);
  OFF(at_config, refine_edges); OFF(at_config, decode_sharpening); OFF(at_config, min_white_black_diff);
  OFF(at_config, min_cluster_pixels); OFF(at_config, max_nmaxima); OFF(at_config, max_line_fit_mse);
  OFF(at_config, cos_critical_rad); OFF(at_config, device); OFF(at_config, max_batch); OFF(at_config, tag_size);
  OFF(at_camera, fx); OFF(at_camera, fy); OFF(at_camera, cx); OFF(at_camera, cy); OFF(at_camera, k1);
  OFF(at_camera, k2); OFF(at_camera, p1); OFF(at_camera, p2); OFF(at_camera, k3);
  OFF(at_detection, id); OFF(at_detection, hamming); OFF(at_detection, decision_margin); OFF(at_detection, H);
  OFF(at_detection, c); OFF(at_detection, p);
  OFF(at_pose, id); OFF(at_pose, R); OFF(at_pose, t); OFF(at_pose, err);
  OFF(at_tag_detection, id); OFF(at_tag_detection, camera); OFF(at_tag_detection, robot);
  OFF(at_tag_detection, distance); OFF(at_tag_detection, err);
  OFF(at_quad_record, blob_index); OFF(at_quad_record, valid); OFF(at_quad_record, accepted);
  OFF(at_quad_record, indices); OFF(at_quad_record, corners);
  printf("\"library_abi_version\": %d}\n", at_abi_version());
  return 0;
}

static int detect(int W, int H, int fmt, const char* path) {
  const size_t fb = (size_t)W * H * (fmt == AT_FMT_BGR8 ? 3 : (fmt == AT_FMT_YUYV ? 2 : 1));
  unsigned char* frame = malloc(fb);
  FILE* f = fopen(path, "rb");
  if (!frame || !f || fread(frame, 1, fb, f) != fb) {
    fprintf(stderr, "cannot read %zu bytes from %s\n", fb, path);
    return 1;
  }
  fclose(f);
  at_config cfg;
  at_camera cam = {905.495617, 907.909470, 609.916016, 352.682645, 0.059238, -0.075154, -0.003801, 0.001113, 0.0};
  at_detector* d = NULL;
  int rc = at_config_default(&cfg, W, H);
  if (rc == AT_OK) rc = at_create(&cfg, &cam, &d);
  if (rc != AT_OK) {
    fprintf(stderr, "at_create: %s\n", at_strerror(rc));
    return 1;
  }
  at_detection dets[256];
  int n = 0;
  rc = at_detect(d, frame, (at_pixfmt)fmt, dets, 256, &n);
  if (rc != AT_OK) {
    fprintf(stderr, "at_detect: %s\n", at_strerror(rc));
    at_destroy(d);
    return 1;
  }
  printf("[");
  for (int i = 0; i < n && i < 256; i++)
    printf("%s{\"id\": %d, \"hamming\": %d, \"p\": [[%.17g, %.17g], [%.17g, %.17g], [%.17g, %.17g], [%.17g, %.17g]]}",
           i ? ", " : "", dets[i].id, dets[i].hamming, dets[i].p[0][0], dets[i].p[0][1], dets[i].p[1][0],
           dets[i].p[1][1], dets[i].p[2][0], dets[i].p[2][1], dets[i].p[3][0], dets[i].p[3][1]);
  printf("]\n");
  at_destroy(d);
  free(frame);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && argv[1][0] == 'l') return layout();
  if (argc >= 6 && argv[1][0] == 'd') return detect(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), argv[5]);
  fprintf(stderr, "usage: %s layout | detect W H FMT FRAME_FILE\n", argv[0]);
  return 2;
}
