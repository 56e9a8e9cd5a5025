/*
 * Sanitizer driver for the oracle's C code (test infrastructure): oracle/fxp_oracle.c and
 * oracle/fxp_gmp.c built with -fsanitize=address,undefined (or thread, for the threaded CPU
 * baseline) and run over seeded inputs — special values, random bit patterns, ragged thread
 * splits, random and malformed hex text. Exit status 0 = every cross-check held and the
 * sanitizer reported nothing. Driven by tests/test_sanitizers.py (CPU-side
 * ASan/TSan of the host code).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_encode_f32(const float* x, int64_t* M, int64_t* E, int64_t n, int dp);
void oracle_encode_f64(const double* x, int64_t* M, int64_t* E, int64_t n, int dp);
void oracle_encode_int(const void* x, int elem_bytes, int64_t* M, int64_t* E, int64_t n);
void oracle_decode_f32(const int64_t* M, const int64_t* E, float* y, int64_t n, int ftz);
void oracle_decode_f64(const int64_t* M, const int64_t* E, double* y, int64_t n);
int oracle_decode_hex_d(const char* s, int64_t len, int64_t E, uint64_t* dbits);
void gmp_decode_i64(const int64_t* M, const int64_t* E, void* y, int out_f64, int64_t n, int ftz);
int64_t gmp_decode_hex(const char* buf, const int64_t* offs, const int64_t* E, void* y, int out_f64, int64_t n,
                       int ftz);
void baseline_encode_f32_literal(const float* x, int64_t* M, int64_t* E, int64_t n, int dp);
void baseline_encode_f32_mt(const float* x, int64_t* M, int64_t* E, int64_t n, int dp, int nthreads);
void baseline_decode_f32_mt(const int64_t* M, const int64_t* E, float* y, int64_t n, int nthreads, int ftz);

static uint64_t s_rng = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
  s_rng ^= s_rng << 13;
  s_rng ^= s_rng >> 7;
  s_rng ^= s_rng << 17;
  return s_rng;
}

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);           \
      fprintf(stderr, "\n");                  \
      if (++fails > 20) exit(1);              \
    }                                         \
  } while (0)

int main(int argc, char** argv) {
  const int threads_only = argc > 1 && strcmp(argv[1], "threads") == 0;
  const int64_t n = 100003;   /* ragged: blocks of uneven size over the threads */
  uint32_t* xb = malloc(n * 4);
  for (int64_t i = 0; i < n; ++i) xb[i] = (uint32_t)rnd();
  const uint32_t special[] = {0u, 0x80000000u, 1u, 0x80000001u, 0x007FFFFFu, 0x00800000u, 0x4B000000u,
                              0x4B000001u, 0x4B400000u, 0x4B800000u, 0x7F800000u, 0xFF800000u, 0x7FC00000u,
                              0x3F800000u, 0xBFC00000u, 0x7F7FFFFFu};
  memcpy(xb, special, sizeof special);
  const float* x = (const float*)xb;
  int64_t *M = malloc(n * 8), *E = malloc(n * 8), *M2 = malloc(n * 8), *E2 = malloc(n * 8);
  float *y = malloc(n * 4), *y2 = malloc(n * 4);

  for (int dp = 0; dp < 2; ++dp) {
    if (!threads_only) {
      oracle_encode_f32(x, M, E, n, dp);
      baseline_encode_f32_literal(x, M2, E2, n, dp);
      CHECK(!memcmp(M, M2, n * 8) && !memcmp(E, E2, n * 8), "literal loop != restatement (dp %d)", dp);
    }
    for (int t = 1; t <= 7; t += 3) {
      baseline_encode_f32_mt(x, M2, E2, n, dp, t);
      if (threads_only) continue;
      CHECK(!memcmp(M, M2, n * 8) && !memcmp(E, E2, n * 8), "threaded encode (%d threads)", t);
    }
    for (int ftz = 0; ftz < 2; ++ftz) {
      if (!threads_only) {
        oracle_decode_f32(M, E, y, n, ftz);
        gmp_decode_i64(M, E, y2, 0, n, ftz);
        CHECK(!memcmp(y, y2, n * 4), "decode restatement != GMP (dp %d ftz %d)", dp, ftz);
      }
      baseline_decode_f32_mt(M2, E2, y2, n, 5, ftz);
      if (!threads_only) CHECK(!memcmp(y, y2, n * 4), "threaded decode (ftz %d)", ftz);
    }
  }
  if (!threads_only) {
    /* fp64 and integer encode, fp64 decode vs GMP over wide (M, E) */
    double* xd = malloc(n * 8);
    for (int64_t i = 0; i < n; ++i) {
      uint64_t b = rnd();
      memcpy(&xd[i], &b, 8);
    }
    oracle_encode_f64(xd, M, E, n, 0);
    oracle_encode_f64(xd, M, E, n, 1);
    int16_t* xi = malloc(n * 2);
    for (int64_t i = 0; i < n; ++i) xi[i] = (int16_t)rnd();
    oracle_encode_int(xi, 2, M, E, n);
    for (int64_t i = 0; i < n; ++i) CHECK(M[i] == xi[i] && E[i] == 0, "int16 encode at %lld", (long long)i);
    for (int64_t i = 0; i < n; ++i) {
      M[i] = (int64_t)(rnd() >> (rnd() & 63));
      if (rnd() & 1) M[i] = -M[i];
      E[i] = (int64_t)(rnd() % 2400) - 1250;
    }
    double *d1 = malloc(n * 8), *d2 = malloc(n * 8);
    oracle_decode_f64(M, E, d1, n);
    gmp_decode_i64(M, E, d2, 1, n, 0);
    CHECK(!memcmp(d1, d2, n * 8), "f64 decode restatement != GMP");
    /* hex text: random widths up to 300 digits, signs, and malformed strings */
    const int nh = 4000;
    char* buf = malloc((size_t)nh * 304);
    int64_t* offs = malloc((nh + 1) * 8);
    int64_t* Eh = malloc(nh * 8);
    double* dh = malloc(nh * 8);
    static const char digits[] = "0123456789abcdefABCDEF";
    int64_t pos = 0;
    for (int i = 0; i < nh; ++i) {
      offs[i] = pos;
      const int len = 1 + (int)(rnd() % 300);
      if (rnd() % 3 == 0) buf[pos++] = '-';
      for (int j = 0; j < len; ++j) buf[pos++] = digits[rnd() % 22];
      if (i % 97 == 5) buf[pos - 1] = 'x';   /* malformed */
      Eh[i] = (int64_t)(rnd() % 400) - 1400;
    }
    offs[nh] = pos;
    int64_t bad = 0;
    for (int i = 0; i < nh; ++i) {
      uint64_t bits;
      const int rc = oracle_decode_hex_d(buf + offs[i], offs[i + 1] - offs[i], Eh[i], &bits);
      if (rc) { ++bad; continue; }
      dh[i] = 0;
      memcpy(&dh[i], &bits, 8);
    }
    double* dg = malloc(nh * 8);
    const int64_t gbad = gmp_decode_hex(buf, offs, Eh, dg, 1, nh, 0);
    CHECK(bad == gbad, "malformed count %lld vs GMP %lld", (long long)bad, (long long)gbad);
    for (int i = 0; i < nh; ++i)
      if (i % 97 != 5) CHECK(!memcmp(&dh[i], &dg[i], 8), "hex decode %d", i);
    free(xd); free(xi); free(d1); free(d2); free(buf); free(offs); free(Eh); free(dh); free(dg);
  }
  free(xb); free(M); free(E); free(M2); free(E2); free(y); free(y2);
  if (fails) return 1;
  printf("oracle sanitizer driver: ok (%s)\n", threads_only ? "threads" : "all");
  return 0;
}
