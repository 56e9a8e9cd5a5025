/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see fxp_oracle.c header).
 *
 * GMP-backed decode in the reference's own call order, used for two things:
 *   1. pinning the plain-C decode restatement (fxp_oracle.c) against GMP 6.2.1 itself — the
 *      third-party library in which FixedPointToFloatPoint's arithmetic lives
 *      (efls-train/cc/efl/math/fixed_point.cc:235-248, :255-265; GMP is an un-vendored
 *      dependency, `libgmp3-dev` in docker/Dockerfile.efls-train:5);
 *   2. the timing-faithful CPU baseline for bench.py (`cpu_baseline`, kind "port"): the
 *      reference's per-element GMP mpf sequence, sharded over host threads in contiguous blocks
 *      like TF's Shard (fixed_point.cc:140-141, :250-251).
 *
 * `ftz` runs the loop with MXCSR FTZ|DAZ set, i.e. the state TensorFlow's CPU threadpool
 * threads run kernels in (the reference op runs inside those threads).
 */
#include <gmp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <xmmintrin.h>

#define EFL_EXPORT __attribute__((visibility("default")))

void oracle_encode_f32(const float* x, int64_t* M, int64_t* E, int64_t n, int dp);

/* efls-train/cc/efl/math/gmp_utils.cc:19-33 semantics: |x| imported as one 64-bit word. */
static void set_sll(mpz_t rop, long long v) {
  unsigned long long u = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
  mpz_import(rop, 1, -1, sizeof(u), 0, 0, &u);
  if (v < 0) mpz_neg(rop, rop);
}

static inline void scale_2exp(mpf_t op, int64_t e) {
  if (e > 0) mpf_mul_2exp(op, op, (mp_bitcnt_t)e);
  else if (e < 0) mpf_div_2exp(op, op, (mp_bitcnt_t)(0 - (uint64_t)e));
}

static void decode_i64_range(const int64_t* M, const int64_t* E, void* y, int out_f64,
                             int64_t s, int64_t e) {
  mpf_t op;
  mpz_t z;
  mpf_init(op);
  mpz_init(z);
  for (int64_t i = s; i < e; ++i) {
    set_sll(z, M[i]);
    mpf_set_z(op, z);
    scale_2exp(op, E[i]);
    double d = mpf_get_d(op);
    if (out_f64) ((double*)y)[i] = d;
    else ((float*)y)[i] = (float)d;
  }
  mpz_clear(z);
  mpf_clear(op);
}

static unsigned set_ftz(int ftz) {
  unsigned old = _mm_getcsr();
  if (ftz) _mm_setcsr(old | 0x8040u);   /* FTZ (bit 15) | DAZ (bit 6) */
  return old;
}

/* Single-threaded GMP decode, int64 mantissa. */
EFL_EXPORT void gmp_decode_i64(const int64_t* M, const int64_t* E, void* y, int out_f64,
                               int64_t n, int ftz) {
  unsigned old = set_ftz(ftz);
  decode_i64_range(M, E, y, out_f64, 0, n);
  _mm_setcsr(old);
}

/* Single-threaded GMP decode, hex-string mantissas packed as a flat buffer + offsets[n+1].
 * Returns the number of strings mpf_set_str rejected (their output is left as NaN). */
EFL_EXPORT int64_t gmp_decode_hex(const char* buf, const int64_t* offs, const int64_t* E,
                                  void* y, int out_f64, int64_t n, int ftz) {
  unsigned old = set_ftz(ftz);
  mpf_t op;
  mpf_init(op);
  int64_t bad = 0;
  char* tmp = NULL;
  size_t cap = 0;
  for (int64_t i = 0; i < n; ++i) {
    size_t len = (size_t)(offs[i + 1] - offs[i]);
    if (len + 1 > cap) {
      cap = (len + 1) * 2;
      tmp = (char*)realloc(tmp, cap);
    }
    memcpy(tmp, buf + offs[i], len);
    tmp[len] = 0;
    if (mpf_set_str(op, tmp, 16) != 0) {
      ++bad;
      if (out_f64) ((double*)y)[i] = __builtin_nan("");
      else ((float*)y)[i] = __builtin_nanf("");
      continue;
    }
    scale_2exp(op, E[i]);
    double d = mpf_get_d(op);
    if (out_f64) ((double*)y)[i] = d;
    else ((float*)y)[i] = (float)d;
  }
  free(tmp);
  mpf_clear(op);
  _mm_setcsr(old);
  return bad;
}

/* ---------------------------- threaded CPU baseline ---------------------------------- */

/* The reference's encode loop body as it runs (fixed_point.cc:107-137), statement for statement,
 * for the timed baseline: the trailing-zero count is taken the reference's way, by converting the
 * lowest set bit to float and reading its biased exponent (:126-127), not with a ctz instruction.
 * The mant == 0 case shifts by (0u - 127) like the reference; gcc on x86-64 gives M = 0,
 * E = exp - 127 there, which tests/test_oracle.py checks against the
 * restatement in fxp_oracle.c. */
static void encode_f32_literal(const float* x, int64_t* M, int64_t* E, int64_t s, int64_t e,
                               int dp) {
  for (int64_t i = s; i < e; ++i) {
    uint32_t bits;
    memcpy(&bits, &x[i], sizeof bits);
    uint32_t se = bits >> 23;
    uint32_t sign = se >> 8;
    int exp = (int)(se & 0xFFu) - 127 - 23;
    int mant = (int)(bits & 0x7FFFFFu);
    if (exp) mant |= 0x800000;
    if (dp) {
      mant >>= 13;
      exp += 13;
    }
    float low = (float)(mant & -mant);
    uint32_t lbits;
    memcpy(&lbits, &low, sizeof lbits);
    unsigned r = (lbits >> 23) - 127u;
    mant = (int)((unsigned)mant >> (r & 31u));
    exp = (int)((unsigned)exp + r);
    M[i] = sign ? -(int64_t)mant : (int64_t)mant;
    E[i] = exp;
  }
}

/* Single-threaded literal loop (checked against the restatement by tests/test_oracle.py). */
EFL_EXPORT void baseline_encode_f32_literal(const float* x, int64_t* M, int64_t* E, int64_t n,
                                            int dp) {
  encode_f32_literal(x, M, E, 0, n, dp);
}

typedef struct {
  const void* x;
  const int64_t* Mi;
  const int64_t* Ei;
  int64_t* M;
  int64_t* E;
  void* y;
  int64_t s, e;
  int mode;   /* 0 encode f32, 1 decode f32 */
  int dp, ftz;
} job_t;

static void* worker(void* p) {
  job_t* j = (job_t*)p;
  unsigned old = set_ftz(j->ftz);
  if (j->mode == 0) {
    encode_f32_literal((const float*)j->x, j->M, j->E, j->s, j->e, j->dp);
  } else {
    decode_i64_range(j->Mi, j->Ei, j->y, 0, j->s, j->e);
  }
  _mm_setcsr(old);
  return NULL;
}

static void run_sharded(job_t proto, int64_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  job_t* jobs = (job_t*)malloc(sizeof(job_t) * (size_t)nthreads);
  int64_t blk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = proto;
    jobs[t].s = t * blk < n ? t * blk : n;
    jobs[t].e = (t + 1) * blk < n ? (t + 1) * blk : n;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* Reference encode loop (fixed_point.cc:107-137, literal form above) sharded over nthreads
 * contiguous blocks like TF Shard (:140-141). */
EFL_EXPORT void baseline_encode_f32_mt(const float* x, int64_t* M, int64_t* E, int64_t n, int dp,
                                       int nthreads) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.x = x; j.M = M; j.E = E; j.mode = 0; j.dp = dp; j.ftz = 1;
  run_sharded(j, n, nthreads);
}

/* Reference decode loop (fixed_point.cc:235-248, GMP mpf) sharded over nthreads blocks; ftz = the
 * MXCSR state of a TF threadpool thread (FTZ|DAZ), the mode the GPU leg decodes in. */
EFL_EXPORT void baseline_decode_f32_mt(const int64_t* M, const int64_t* E, float* y, int64_t n,
                                       int nthreads, int ftz) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.Mi = M; j.Ei = E; j.y = y; j.mode = 1; j.ftz = ftz;
  run_sharded(j, n, nthreads);
}

/* ------------------------- exhaustive fp32 check (tools/exhaustive_fxp.py) ------------------- */

/* Position-weighted sums mod 2^64 over fp32 bit patterns start .. start+count-1 (uint32 wrap) of
 *   h[0] = sum (M K1 + E K2) (2 i + 1)      the literal encode loop (fixed_point.cc:107-137)
 *   h[1] = sum y0 K3 (2 i + 1)               y0 = GMP decode of (M, E), MXCSR default
 *   h[2] = sum y1 K3 (2 i + 1)               y1 = the same under FTZ|DAZ (TF threadpool state)
 * i = the global pattern index (start + offset), y = float bits. Sums mod 2^64 do not depend on the
 * order of the additions, so the GPU side (torch int64 arithmetic) reproduces them exactly. */
#define EH_K1 0x9E3779B97F4A7C15ull
#define EH_K2 0xC2B2AE3D27D4EB4Full
#define EH_K3 0x165667B19E3779F9ull

typedef struct {
  uint32_t start;
  int64_t s, e;
  int dp;
  uint64_t h[3];
} eh_job_t;

static void* eh_worker(void* p) {
  eh_job_t* j = (eh_job_t*)p;
  enum { B = 4096 };
  float x[B];
  int64_t M[B], E[B];
  mpf_t op;
  mpz_t z;
  mpf_init(op);
  mpz_init(z);
  uint64_t h0 = 0, h1 = 0, h2 = 0;
  for (int64_t b0 = j->s; b0 < j->e; b0 += B) {
    const int64_t nb = j->e - b0 < B ? j->e - b0 : B;
    for (int64_t k = 0; k < nb; ++k) {
      const uint32_t bits = j->start + (uint32_t)(b0 + k);
      memcpy(&x[k], &bits, 4);
    }
    encode_f32_literal(x, M, E, 0, nb, j->dp);
    for (int mode = 0; mode < 2; ++mode) {
      const unsigned old = set_ftz(mode);
      uint64_t acc = 0;
      for (int64_t k = 0; k < nb; ++k) {
        set_sll(z, M[k]);
        mpf_set_z(op, z);
        scale_2exp(op, E[k]);
        const float y = (float)mpf_get_d(op);
        uint32_t yb;
        memcpy(&yb, &y, 4);
        const uint64_t w = 2 * ((uint64_t)j->start + (uint64_t)(b0 + k)) + 1;
        acc += (uint64_t)yb * EH_K3 * w;
        if (mode == 0) h0 += ((uint64_t)M[k] * EH_K1 + (uint64_t)E[k] * EH_K2) * w;
      }
      _mm_setcsr(old);
      if (mode == 0) h1 += acc;
      else h2 += acc;
    }
  }
  mpz_clear(z);
  mpf_clear(op);
  j->h[0] = h0;
  j->h[1] = h1;
  j->h[2] = h2;
  return NULL;
}

EFL_EXPORT void exhaustive_hash_f32(uint32_t start, int64_t count, int dp, int nthreads, uint64_t* out) {
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  eh_job_t* jobs = (eh_job_t*)malloc(sizeof(eh_job_t) * (size_t)nthreads);
  const int64_t blk = (count + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].start = start;
    jobs[t].dp = dp;
    jobs[t].s = t * blk < count ? t * blk : count;
    jobs[t].e = (t + 1) * blk < count ? (t + 1) * blk : count;
    pthread_create(&th[t], NULL, eh_worker, &jobs[t]);
  }
  out[0] = out[1] = out[2] = 0;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    for (int k = 0; k < 3; ++k) out[k] += jobs[t].h[k];
  }
  free(th);
  free(jobs);
}
