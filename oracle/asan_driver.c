/*
 * asan_driver.c — TEST INFRASTRUCTURE ONLY: a standalone driver of the CPU reference physics
 * (physics_ref.c, f64 and f32 variants) built with AddressSanitizer + UndefinedBehaviorSanitizer
 * by `make -C oracle asan` (sanitizer runs of the host code).  tests/test_oracle_asan.py
 * writes a scenario file, runs this executable and compares its outputs with libphysref.so.
 *
 * Scenario file (little endian, no padding between fields):
 *   int32 n, steps, hf_rows, hf_cols;  hg_cfg;  hg_model;  int16 hf[hf_rows * hf_cols];
 *   f64 root[n][13], q[n][12], qd[n][12], mass0[n], fric[n], actions[steps][n][12]
 * Output file: for f64 then f32 (as f64): root, q, qd, torques, contact[n][13][3], then int32
 *   nonfinite[n], dropped[n] per precision.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hgsim.h"

int ref_step_f64(const hg_cfg*, const hg_model*, const int16_t*, int, double*, double*, double*, double*,
                 const double*, const double*, const double*, double*, double*, double*, int32_t*, int32_t*);
int ref_step_f32(const hg_cfg*, const hg_model*, const int16_t*, int, float*, float*, float*, float*,
                 const float*, const float*, const float*, float*, float*, float*, int32_t*, int32_t*);
int ref_lamw_f64(void);

static void must_read(FILE* f, void* p, size_t bytes) {
  if (fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "asan_driver: short scenario file\n");
    exit(2);
  }
}

static void* xcalloc(size_t count, size_t size) {
  void* p = calloc(count ? count : 1, size);
  if (!p) exit(3);
  return p;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s scenario.bin out.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hdr[4];
  must_read(f, hdr, sizeof(hdr));
  const int n = hdr[0], steps = hdr[1], hr = hdr[2], hc = hdr[3];
  hg_cfg cfg;
  hg_model model;
  must_read(f, &cfg, sizeof(cfg));
  must_read(f, &model, sizeof(model));
  int16_t* hf = NULL;
  if (hr > 0 && hc > 0) {
    hf = (int16_t*)xcalloc((size_t)hr * hc, sizeof(int16_t));
    must_read(f, hf, (size_t)hr * hc * sizeof(int16_t));
  }
  cfg.heightfield = hf;
  cfg.terrain_origins = NULL;
  const int lamw = ref_lamw_f64();
  double* root0 = (double*)xcalloc((size_t)n * 13, 8);
  double* q0 = (double*)xcalloc((size_t)n * 12, 8);
  double* qd0 = (double*)xcalloc((size_t)n * 12, 8);
  double* mass0 = (double*)xcalloc(n, 8);
  double* fric = (double*)xcalloc(n, 8);
  double* act = (double*)xcalloc((size_t)steps * n * 12, 8);
  must_read(f, root0, (size_t)n * 13 * 8);
  must_read(f, q0, (size_t)n * 12 * 8);
  must_read(f, qd0, (size_t)n * 12 * 8);
  must_read(f, mass0, (size_t)n * 8);
  must_read(f, fric, (size_t)n * 8);
  must_read(f, act, (size_t)steps * n * 12 * 8);
  fclose(f);
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;

  /* f64 */
  {
    double* root = (double*)xcalloc((size_t)n * 13, 8);
    double* q = (double*)xcalloc((size_t)n * 12, 8);
    double* qd = (double*)xcalloc((size_t)n * 12, 8);
    double* lam = (double*)xcalloc((size_t)n * lamw, 8);
    double* tau = (double*)xcalloc((size_t)n * 12, 8);
    double* con = (double*)xcalloc((size_t)n * 13 * 3, 8);
    double* rig = (double*)xcalloc((size_t)n * 13 * 13, 8);
    int32_t* bad = (int32_t*)xcalloc(n, 4);
    int32_t* drop = (int32_t*)xcalloc(n, 4);
    memcpy(root, root0, (size_t)n * 13 * 8);
    memcpy(q, q0, (size_t)n * 12 * 8);
    memcpy(qd, qd0, (size_t)n * 12 * 8);
    for (int s = 0; s < steps; s++)
      ref_step_f64(&cfg, &model, hf, n, root, q, qd, lam, act + (size_t)s * n * 12, mass0, fric, tau, con, rig, bad,
                   drop);
    fwrite(root, 8, (size_t)n * 13, o);
    fwrite(q, 8, (size_t)n * 12, o);
    fwrite(qd, 8, (size_t)n * 12, o);
    fwrite(tau, 8, (size_t)n * 12, o);
    fwrite(con, 8, (size_t)n * 13 * 3, o);
    fwrite(bad, 4, n, o);
    fwrite(drop, 4, n, o);
    free(root); free(q); free(qd); free(lam); free(tau); free(con); free(rig); free(bad); free(drop);
  }
  /* f32 */
  {
    float* root = (float*)xcalloc((size_t)n * 13, 4);
    float* q = (float*)xcalloc((size_t)n * 12, 4);
    float* qd = (float*)xcalloc((size_t)n * 12, 4);
    float* lam = (float*)xcalloc((size_t)n * lamw, 4);
    float* a = (float*)xcalloc((size_t)n * 12, 4);
    float* m0 = (float*)xcalloc(n, 4);
    float* fr = (float*)xcalloc(n, 4);
    float* tau = (float*)xcalloc((size_t)n * 12, 4);
    float* con = (float*)xcalloc((size_t)n * 13 * 3, 4);
    float* rig = (float*)xcalloc((size_t)n * 13 * 13, 4);
    int32_t* bad = (int32_t*)xcalloc(n, 4);
    int32_t* drop = (int32_t*)xcalloc(n, 4);
    for (size_t i = 0; i < (size_t)n * 13; i++) root[i] = (float)root0[i];
    for (size_t i = 0; i < (size_t)n * 12; i++) { q[i] = (float)q0[i]; qd[i] = (float)qd0[i]; }
    for (int e = 0; e < n; e++) { m0[e] = (float)mass0[e]; fr[e] = (float)fric[e]; }
    for (int s = 0; s < steps; s++) {
      for (size_t i = 0; i < (size_t)n * 12; i++) a[i] = (float)act[(size_t)s * n * 12 + i];
      ref_step_f32(&cfg, &model, hf, n, root, q, qd, lam, a, m0, fr, tau, con, rig, bad, drop);
    }
    double* buf = (double*)xcalloc((size_t)n * 13 * 3, 8);
#define PUT(p, cnt)                                              \
  do {                                                           \
    for (size_t i = 0; i < (size_t)(cnt); i++) buf[i] = (p)[i];  \
    fwrite(buf, 8, (size_t)(cnt), o);                            \
  } while (0)
    PUT(root, (size_t)n * 13);
    PUT(q, (size_t)n * 12);
    PUT(qd, (size_t)n * 12);
    PUT(tau, (size_t)n * 12);
    PUT(con, (size_t)n * 13 * 3);
#undef PUT
    fwrite(bad, 4, n, o);
    fwrite(drop, 4, n, o);
    free(buf); free(root); free(q); free(qd); free(lam); free(a); free(m0); free(fr); free(tau); free(con);
    free(rig); free(bad); free(drop);
  }
  fclose(o);
  free(hf); free(root0); free(q0); free(qd0); free(mass0); free(fric); free(act);
  return 0;
}
