/* CPU-baseline driver for the oracle (test/bench infrastructure only).
 * Reads N raw YUYV frames (W*H*2 bytes each) from a file and times
 * ao_detect: per-frame latency single-threaded, and throughput with one
 * frame stream per thread.  Prints one JSON line. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sched.h>
#include "ao_oracle.h"

static double now_s(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
typedef struct { const unsigned char *frames; int nframes, W, H, iters; double secs; long dets; } job_t;
static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  ao_params p; ao_default_params(&p, j->W, j->H);
  ao_state *s = ao_create(&p);
  double t0 = now_s();
  for (int i = 0; i < j->iters; i++) j->dets += ao_detect(s, j->frames + (size_t)(i % j->nframes) * j->W * j->H * 2, 0);
  j->secs = now_s() - t0;
  ao_destroy(s);
  return NULL;
}
static int cmpd(const void *a, const void *b) { double x = *(const double *)a, y = *(const double *)b; return x < y ? -1 : x > y; }
int main(int argc, char **argv) {
  if (argc < 7) { fprintf(stderr, "usage: %s frames.raw W H nframes lat_iters thr_iters [threads]\n", argv[0]); return 2; }
  const char *fn = argv[1]; int W = atoi(argv[2]), H = atoi(argv[3]), nf = atoi(argv[4]);
  int lat_iters = atoi(argv[5]), thr_iters = atoi(argv[6]);
  int threads = argc > 7 ? atoi(argv[7]) : 0;
  if (threads <= 0) { cpu_set_t cs; sched_getaffinity(0, sizeof(cs), &cs); threads = CPU_COUNT(&cs); }
  size_t fb = (size_t)W * H * 2;
  unsigned char *frames = malloc(fb * nf);
  FILE *f = fopen(fn, "rb"); if (!f || fread(frames, 1, fb * nf, f) != fb * nf) { fprintf(stderr, "read fail\n"); return 1; } fclose(f);
  ao_params p; ao_default_params(&p, W, H); ao_state *s = ao_create(&p);
  for (int i = 0; i < 3 && i < nf; i++) ao_detect(s, frames + fb * i, 0);
  double *lat = malloc(sizeof(double) * (lat_iters > 0 ? lat_iters : 1)); long dets = 0;
  double tl0 = now_s();
  for (int i = 0; i < lat_iters; i++) { double t0 = now_s(); dets += ao_detect(s, frames + fb * (i % nf), 0); lat[i] = now_s() - t0; }
  double tl = now_s() - tl0;
  qsort(lat, lat_iters, sizeof(double), cmpd);
  ao_destroy(s);
  pthread_t *th = malloc(sizeof(pthread_t) * threads); job_t *jobs = calloc(threads, sizeof(job_t));
  double t0 = now_s();
  for (int t = 0; t < threads; t++) { jobs[t] = (job_t){frames, nf, W, H, thr_iters, 0, 0}; pthread_create(&th[t], NULL, worker, &jobs[t]); }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  double tt = now_s() - t0;
  printf("{\"lat_frames\": %d, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"single_thread_fps\": %.3f, \"threads\": %d, \"thr_frames\": %d, \"throughput_fps\": %.3f, \"dets_per_frame\": %.3f}\n",
         lat_iters, 1e3 * lat[lat_iters / 2], 1e3 * lat[(int)(lat_iters * 0.99)], lat_iters / tl, threads, threads * thr_iters,
         threads * thr_iters / tt, lat_iters ? (double)dets / lat_iters : 0.0);
  return 0;
}
