/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see fxp_oracle.c header).
 *
 * Paillier arithmetic of efls-train through GMP 6.2.1, in the reference's own call order, used to
 * pin the Python-int restatement (oracle/paillier.py) and to produce the golden known-answer
 * vectors in tests/golden/ (the reference ships none: efls-train/test/paillier_test.py uses fresh
 * time-seeded keys and allclose). Restated from:
 *   keygen   GeneratePaillierKeypairOp::Compute   efls-train/cc/efl/math/paillier.cc:833-904
 *   keys     SetPublicKey / SetPrivateKey         paillier.cc:70-101, h-function :28-37
 *   encrypt  PaillierKeypair::Encrypt             paillier.cc:103-131 (hsa given)
 *   decrypt  _Decrypt + m-function                paillier.cc:296-312, :39-48
 *   fbpowm   FixedBasePowm::init_table/mpz_fbpowm gmp_utils.cc:56-144
 *   ops      Add / MulScalar / MulExp2 / Invert   paillier.cc:157-285, :722-733
 *   matmul   PaillierMatmulOp::Compute            paillier.cc:987-1035
 * Strings are lowercase hex as mpz_get_str(..., 16) writes them (gmp_utils.cc:146-150).
 */
#include <gmp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EFL_EXPORT __attribute__((visibility("default")))

static void put(char* out, size_t cap, const mpz_t v) {
  char* s = mpz_get_str(NULL, 16, v);
  strncpy(out, s, cap - 1);
  out[cap - 1] = 0;
  void (*freefunc)(void*, size_t);
  mp_get_memory_functions(NULL, NULL, &freefunc);
  freefunc(s, strlen(s) + 1);
}

/* keygen with an explicit MT seed (the reference seeds with time(), paillier.cc:845-849) */
static void draw_prime(mpz_t r, gmp_randstate_t st, int bits, int reps) {
  do {
    mpz_urandomb(r, st, (mp_bitcnt_t)bits);
    mpz_setbit(r, 0);
    mpz_setbit(r, 1);
    mpz_setbit(r, (mp_bitcnt_t)(bits - 1));
  } while (!mpz_probab_prime_p(r, reps));
}

EFL_EXPORT void pl_gmp_keygen(int n_bytes, int reps, unsigned long seed, char* n_out, char* hs_out,
                              char* p_out, char* q_out, size_t cap) {
  mpz_t p, q, n, hs, t1, t2;
  gmp_randstate_t st;
  mpz_inits(p, q, n, hs, t1, t2, NULL);
  gmp_randinit_mt(st);
  gmp_randseed_ui(st, seed);
  const int bits = n_bytes * 4;                           /* paillier.cc:852 n_bytes << 2 */
  for (;;) {                                              /* gcd(p-1, q-1) must be 2 */
    draw_prime(p, st, bits, reps);
    draw_prime(q, st, bits, reps);
    mpz_sub_ui(t1, p, 1);
    mpz_sub_ui(t2, q, 1);
    mpz_gcd(t1, t1, t2);
    if (mpz_cmp_ui(t1, 2) == 0) break;
  }
  mpz_mul(n, p, q);
  do {                                                    /* x in Z_n^* */
    mpz_urandomm(t1, st, n);
    mpz_gcd(t2, t1, n);
  } while (mpz_cmp_ui(t2, 1) != 0);
  mpz_mul(hs, t1, t1);                                    /* hs = (-x^2)^n mod n^2 */
  mpz_neg(hs, hs);
  mpz_mod(hs, hs, n);
  mpz_mul(t1, n, n);
  mpz_powm(hs, hs, n, t1);
  put(n_out, cap, n);
  put(hs_out, cap, hs);
  put(p_out, cap, p);
  put(q_out, cap, q);
  mpz_clears(p, q, n, hs, t1, t2, NULL);
  gmp_randclear(st);
}

/* Encrypt given hsa (non-zero): c = (1 + |m| n)^(+-1) * hsa mod n^2 */
EFL_EXPORT void pl_gmp_encrypt(const char* n_hex, long long m, const char* hsa_hex, char* out, size_t cap) {
  mpz_t n, n2, c, h;
  mpz_inits(n, n2, c, h, NULL);
  mpz_set_str(n, n_hex, 16);
  mpz_mul(n2, n, n);
  mpz_set_str(h, hsa_hex, 16);
  unsigned long long u = m < 0 ? 0ull - (unsigned long long)m : (unsigned long long)m;
  mpz_import(c, 1, -1, sizeof(u), 0, 0, &u);
  mpz_mul(c, c, n);
  mpz_add_ui(c, c, 1);
  if (m < 0) mpz_invert(c, c, n2);
  mpz_mul(c, c, h);
  mpz_mod(c, c, n2);
  put(out, cap, c);
  mpz_clears(n, n2, c, h, NULL);
}

/* h(x) = (L_x((n+1)^(x-1) mod x^2))^-1 mod x */
static void h_func(mpz_t r, const mpz_t n, const mpz_t x, const mpz_t x2) {
  mpz_t g;
  mpz_init(g);
  mpz_add_ui(g, n, 1);
  mpz_sub_ui(r, x, 1);
  mpz_powm(r, g, r, x2);
  mpz_sub_ui(r, r, 1);
  mpz_divexact(r, r, x);
  mpz_invert(r, r, x);
  mpz_clear(g);
}

/* m_x(c) = L_x(c^(x-1) mod x^2) * h mod x */
static void m_func(mpz_t r, const mpz_t c, const mpz_t x, const mpz_t x2, const mpz_t h) {
  mpz_t e;
  mpz_init(e);
  mpz_sub_ui(e, x, 1);
  mpz_powm(r, c, e, x2);
  mpz_sub_ui(r, r, 1);
  mpz_divexact(r, r, x);
  mpz_mul(r, r, h);
  mpz_mod(r, r, x);
  mpz_clear(e);
}

EFL_EXPORT void pl_gmp_decrypt(const char* p_hex, const char* q_hex, const char* c_hex, char* out, size_t cap) {
  mpz_t p, q, n, p2, q2, hp, hq, qinv, mx, c, m, cq;
  mpz_inits(p, q, n, p2, q2, hp, hq, qinv, mx, c, m, cq, NULL);
  mpz_set_str(p, p_hex, 16);
  mpz_set_str(q, q_hex, 16);
  mpz_mul(n, p, q);
  mpz_mul(p2, p, p);
  mpz_mul(q2, q, q);
  h_func(hp, n, p, p2);
  h_func(hq, n, q, q2);
  mpz_invert(qinv, q, p);
  mpz_mul_2exp(mx, n, 1);                                /* max = ceil(2n/3), paillier.cc:76-77 */
  mpz_cdiv_q_ui(mx, mx, 3);
  mpz_set_str(c, c_hex, 16);
  m_func(m, c, p, p2, hp);
  m_func(cq, c, q, q2, hq);
  mpz_sub(m, m, cq);                                      /* CRT */
  mpz_mul(m, m, qinv);
  mpz_mod(m, m, p);
  mpz_mul(m, m, q);
  mpz_add(m, m, cq);
  mpz_mod(m, m, n);
  if (mpz_cmp(m, mx) > 0) mpz_sub(m, m, n);
  put(out, cap, m);
  mpz_clears(p, q, n, p2, q2, hp, hq, qinv, mx, c, m, cq, NULL);
}

/* fixed-base powm through the reference's table and lookup order */
EFL_EXPORT int pl_gmp_fbpowm(const char* base_hex, const char* mod_hex, unsigned exp_bits, unsigned g,
                             const char* a_hex, char* out, size_t cap) {
  mpz_t base, mod, a, acc;
  mpz_inits(base, mod, a, acc, NULL);
  mpz_set_str(base, base_hex, 16);
  mpz_set_str(mod, mod_hex, 16);
  mpz_set_str(a, a_hex, 16);
  const unsigned long long cols = (1ull << g) - 1;
  const unsigned rows = exp_bits / g + (exp_bits % g ? 1 : 0);
  mpz_t* T = (mpz_t*)malloc(sizeof(mpz_t) * rows * cols);
  for (unsigned long long i = 0; i < rows * cols; ++i) mpz_init(T[i]);
  /* row 0: base^1 .. base^cols; row i: row i-1 raised to 2^g */
  mpz_set(T[0], base);
  for (unsigned long long j = 1; j < cols; ++j) {
    mpz_mul(T[j], T[j - 1], base);
    mpz_mod(T[j], T[j], mod);
  }
  for (unsigned i = 1; i < rows; ++i)
    for (unsigned long long j = 0; j < cols; ++j)
      mpz_powm_ui(T[i * cols + j], T[(i - 1) * cols + j], 1ul << g, mod);
  int rc = 1;
  size_t size = mpz_sizeinbase(a, 2);
  if (mpz_sgn(a) == 0) size = 1;                         /* sizeinbase(0) = 1 */
  if (size > exp_bits) {
    rc = -1;
  } else {
    mpz_set_ui(acc, 1);
    const size_t full = size / g;
    for (size_t i = 0; i < full; ++i) {
      unsigned long idx = 0;
      for (unsigned j = 0; j < g; ++j) idx = (idx << 1) | (unsigned long)mpz_tstbit(a, i * g + j);
      if (idx) {
        mpz_mul(acc, acc, T[i * cols + idx - 1]);
        mpz_mod(acc, acc, mod);
      }
    }
    if (size % g) {
      unsigned long idx = 0;
      for (size_t b = full * g; b < size; ++b) idx = (idx << 1) | (unsigned long)mpz_tstbit(a, b);
      /* the reference indexes with --idx unconditionally here (gmp_utils.cc:133-137): the top
       * partial group holds the leading 1 bit of a, so idx >= 1 — except a == 0 with g > 1, an
       * out-of-bounds read in the reference (probability 2^-a_bits); defined here as a^0 = 1. */
      if (idx) {
        mpz_mul(acc, acc, T[full * cols + idx - 1]);
        mpz_mod(acc, acc, mod);
      }
    }
    put(out, cap, acc);
  }
  for (unsigned long long i = 0; i < rows * cols; ++i) mpz_clear(T[i]);
  free(T);
  mpz_clears(base, mod, a, acc, NULL);
  return rc;
}

/* plain powm, for spot checks */
EFL_EXPORT void pl_gmp_powm(const char* b_hex, const char* e_hex, const char* m_hex, char* out, size_t cap) {
  mpz_t b, e, m, r;
  mpz_inits(b, e, m, r, NULL);
  mpz_set_str(b, b_hex, 16);
  mpz_set_str(e, e_hex, 16);
  mpz_set_str(m, m_hex, 16);
  mpz_powm(r, b, e, m);
  put(out, cap, r);
  mpz_clears(b, e, m, r, NULL);
}

/* ------------------------------------------------------------------------------------------
 * Homomorphic ops through GMP in the reference's call order (known answers for tests/golden).
 * Every ciphertext / scalar crosses as the hex text the TF ops carry (mpz_init_set_str(.., 16)).
 * ------------------------------------------------------------------------------------------ */
static void n_square(mpz_t n2, const char* n_hex) {
  mpz_set_str(n2, n_hex, 16);
  mpz_mul(n2, n2, n2);
}

/* PaillierKeypair::Add(string, string, string), paillier.cc:157-169 */
EFL_EXPORT void pl_gmp_add(const char* n_hex, const char* x_hex, const char* y_hex, char* out, size_t cap) {
  mpz_t n2, op, rop;
  mpz_inits(n2, op, rop, NULL);
  n_square(n2, n_hex);
  mpz_set_str(rop, x_hex, 16);
  mpz_set_str(op, y_hex, 16);
  mpz_mul(rop, rop, op);
  mpz_mod(rop, rop, n2);
  put(out, cap, rop);
  mpz_clears(n2, op, rop, NULL);
}

/* MulScalar(mpz x, mpz y, mpz z), paillier.cc:197-212: y < 0 inverts x mod n^2, then powm by |y|.
 * The int64 and string overloads (:227-248) reach it with y = mpz_set_sll(y) / mpz_init_set_str(y,
 * 16); the int32 overload (:180-195) computes the same value with powm_ui. y_hex is signed hex.
 * Returns 0, or -1 when y < 0 and x has no inverse mod n^2 (the reference's result is undefined). */
EFL_EXPORT int pl_gmp_mul_scalar(const char* n_hex, const char* x_hex, const char* y_hex, char* out, size_t cap) {
  mpz_t n2, x, y, z, abs_y;
  mpz_inits(n2, x, y, z, abs_y, NULL);
  n_square(n2, n_hex);
  mpz_set_str(x, x_hex, 16);
  mpz_set_str(y, y_hex, 16);
  int rc = 0;
  if (mpz_sgn(y) < 0) {
    mpz_neg(abs_y, y);
    if (!mpz_invert(z, x, n2)) rc = -1;
    else mpz_powm(z, z, abs_y, n2);
  } else {
    mpz_powm(z, x, y, n2);
  }
  if (!rc) put(out, cap, z);
  mpz_clears(n2, x, y, z, abs_y, NULL);
  return rc;
}

/* PaillierMulExp2Op::Compute per element, paillier.cc:722-733: y < 0 is an InvalidArgument
 * (returns -1); else op = 2^y and MulScalar(x, op). */
EFL_EXPORT int pl_gmp_mul_exp2(const char* n_hex, const char* x_hex, long long y, char* out, size_t cap) {
  if (y < 0) return -1;
  mpz_t n2, x, op, z;
  mpz_inits(n2, x, op, z, NULL);
  n_square(n2, n_hex);
  mpz_set_str(x, x_hex, 16);
  mpz_set_si(op, 1);
  mpz_mul_2exp(op, op, (mp_bitcnt_t)y);
  mpz_powm(z, x, op, n2);
  put(out, cap, z);
  mpz_clears(n2, x, op, z, NULL);
  return 0;
}

/* Invert(string, string), paillier.cc:275-285. Returns -1 when x has no inverse mod n^2. */
EFL_EXPORT int pl_gmp_invert(const char* n_hex, const char* x_hex, char* out, size_t cap) {
  mpz_t n2, op;
  mpz_inits(n2, op, NULL);
  n_square(n2, n_hex);
  mpz_set_str(op, x_hex, 16);
  int rc = mpz_invert(op, op, n2) ? 0 : -1;
  if (!rc) put(out, cap, op);
  mpz_clears(n2, op, NULL);
  return rc;
}

/* PaillierMatmulOp::Compute, paillier.cc:987-1035, statement for statement: y transposed into
 * yt (:988-993), every x inverted mod n^2 (:994-999), then per output i the minimum exponent
 * (:1006-1014) and per term MulScalar(x, y) for y >= 0 (:250-265 with y >= 0) or
 * MulScalar(x^-1, -y) (:1020-1021), MulScalar by 2^(exp - min) (:1023-1025), and Add into the
 * sum (:1026-1031). xs: u*v hex strings; xe [u][v]; ym, ye [v][w]; out: u*w strings of `cap`
 * bytes each (row-major), ze [u][w]. Returns -1 if an x has no inverse. */
EFL_EXPORT int pl_gmp_matmul(const char* n_hex, const char* const* xs, const long long* xe, const long long* ym,
                             const long long* ye, int u, int v, int w, char* out, size_t cap, long long* ze) {
  mpz_t n2, addend, e, sum;
  mpz_inits(n2, addend, e, sum, NULL);
  n_square(n2, n_hex);
  const long long N = (long long)v * w;
  long long* yt_m = (long long*)malloc(sizeof(long long) * (size_t)(N ? N : 1));
  long long* yt_e = (long long*)malloc(sizeof(long long) * (size_t)(N ? N : 1));
  for (long long i = 0; i < N; ++i) {
    yt_m[i / w + i % w * v] = ym[i];
    yt_e[i / w + i % w * v] = ye[i];
  }
  const long long NX = (long long)u * v;
  mpz_t* xm = (mpz_t*)malloc(sizeof(mpz_t) * (size_t)(NX ? NX : 1));
  mpz_t* xinv = (mpz_t*)malloc(sizeof(mpz_t) * (size_t)(NX ? NX : 1));
  int rc = 0;
  for (long long i = 0; i < NX; ++i) {
    mpz_init_set_str(xm[i], xs[i], 16);
    mpz_init(xinv[i]);
    if (!mpz_invert(xinv[i], xm[i], n2)) rc = -1;
  }
  for (long long i = 0; rc == 0 && i < (long long)u * w; ++i) {
    const long long sx = i / w * v, sy = i % w * v;
    long long mn = 0x7FFFFFFFFFFFFFFFLL;
    for (int j = 0; j < v; ++j) {
      const long long ex = xe[sx + j] + yt_e[sy + j];
      if (ex < mn) mn = ex;
    }
    for (int j = 0; j < v; ++j) {
      const long long ex = xe[sx + j] + yt_e[sy + j] - mn;
      const long long y = yt_m[sy + j];
      const unsigned long long ay = y < 0 ? 0ull - (unsigned long long)y : (unsigned long long)y;
      mpz_import(e, 1, -1, sizeof(ay), 0, 0, &ay);
      mpz_powm(addend, y >= 0 ? xm[sx + j] : xinv[sx + j], e, n2);
      mpz_set_si(e, 1);
      mpz_mul_2exp(e, e, (mp_bitcnt_t)ex);
      mpz_powm(addend, addend, e, n2);
      if (!j) {
        mpz_set(sum, addend);
      } else {
        mpz_mul(sum, addend, sum);
        mpz_mod(sum, sum, n2);
      }
    }
    ze[i] = mn;
    put(out + (size_t)i * cap, cap, sum);
  }
  for (long long i = 0; i < NX; ++i) mpz_clears(xm[i], xinv[i], NULL);
  free(xm);
  free(xinv);
  free(yt_m);
  free(yt_e);
  mpz_clears(n2, addend, e, sum, NULL);
  return rc;
}

/* ------------------------------------------------------------------------------------------
 * CPU baseline of Stage P (bench.py --stage p, cpu_baseline leg only): the reference's per-element
 * work with the key state built ONCE, as the PaillierKeypair resource holds it (paillier.cc:70-101:
 * n^2, hp, hq, q^-1 mod p, the fbpowm table of gmp_utils.cc:56-89), then `count` encryptions with
 * fresh randomness (urandomb a of a_bits, fbpowm, (1+|m|n)^(+-1) * hsa mod n^2; paillier.cc:103-131)
 * and `count` CRT decryptions (paillier.cc:296-312), split into contiguous blocks over `threads`
 * pthreads like TF Shard. Each thread owns its MT state (the reference shares one, unlocked).
 * times[0] = encrypt seconds, times[1] = decrypt seconds (wall).
 * ------------------------------------------------------------------------------------------ */
#include <pthread.h>
#include <time.h>

typedef struct {
  mpz_t n, n2, p, q, p2, q2, hp, hq, qinv, mx;
  mpz_t* T;
  unsigned long long cols;
  unsigned rows, g, a_bits;
} bench_key;

typedef struct {
  bench_key* k;
  long long lo, hi;
  int op;   /* 0 encrypt, 1 decrypt */
  char** cts;
  unsigned long seed;
} bench_job;

static void bench_fbpowm(mpz_t acc, const bench_key* k, const mpz_t a) {
  const size_t size = mpz_sgn(a) ? mpz_sizeinbase(a, 2) : 1;
  mpz_set_ui(acc, 1);
  for (size_t s = 0, row = 0; s < size; s += k->g, ++row) {
    const size_t w = size - s < k->g ? size - s : k->g;
    unsigned long idx = 0;
    for (size_t j = 0; j < w; ++j) idx = (idx << 1) | (unsigned long)mpz_tstbit(a, s + j);
    if (idx) {
      mpz_mul(acc, acc, k->T[row * k->cols + idx - 1]);
      mpz_mod(acc, acc, k->n2);
    }
  }
}

static void* bench_worker(void* arg) {
  bench_job* jb = (bench_job*)arg;
  bench_key* k = jb->k;
  mpz_t a, h, c, m, cq;
  mpz_inits(a, h, c, m, cq, NULL);
  gmp_randstate_t st;
  gmp_randinit_mt(st);
  gmp_randseed_ui(st, jb->seed);
  for (long long i = jb->lo; i < jb->hi; ++i) {
    if (jb->op == 0) {
      long long mv = (i * 2654435761LL) % 1000003LL - 500001LL;
      mpz_urandomb(a, st, k->a_bits);
      bench_fbpowm(h, k, a);
      unsigned long long u = mv < 0 ? 0ull - (unsigned long long)mv : (unsigned long long)mv;
      mpz_import(c, 1, -1, sizeof(u), 0, 0, &u);
      mpz_mul(c, c, k->n);
      mpz_add_ui(c, c, 1);
      if (mv < 0) mpz_invert(c, c, k->n2);
      mpz_mul(c, c, h);
      mpz_mod(c, c, k->n2);
      char* s = mpz_get_str(NULL, 16, c);   /* the op's DT_STRING output */
      if (jb->cts) jb->cts[i] = s;
      else {
        void (*freefunc)(void*, size_t);
        mp_get_memory_functions(NULL, NULL, &freefunc);
        freefunc(s, strlen(s) + 1);
      }
    } else {
      mpz_set_str(c, jb->cts[i], 16);
      m_func(m, c, k->p, k->p2, k->hp);
      m_func(cq, c, k->q, k->q2, k->hq);
      mpz_sub(m, m, cq);
      mpz_mul(m, m, k->qinv);
      mpz_mod(m, m, k->p);
      mpz_mul(m, m, k->q);
      mpz_add(m, m, cq);
      mpz_mod(m, m, k->n);
      if (mpz_cmp(m, k->mx) > 0) mpz_sub(m, m, k->n);
      char* s = mpz_get_str(NULL, 16, m);
      void (*freefunc)(void*, size_t);
      mp_get_memory_functions(NULL, NULL, &freefunc);
      freefunc(s, strlen(s) + 1);
    }
  }
  gmp_randclear(st);
  mpz_clears(a, h, c, m, cq, NULL);
  return NULL;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void bench_run(bench_key* k, int op, char** cts, long long count, int threads) {
  pthread_t th[256];
  bench_job jobs[256];
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    jobs[t].k = k;
    jobs[t].op = op;
    jobs[t].cts = cts;
    jobs[t].lo = count * t / threads;
    jobs[t].hi = count * (t + 1) / threads;
    jobs[t].seed = 12345ul + (unsigned long)t;
    pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

EFL_EXPORT void pl_gmp_bench(const char* p_hex, const char* q_hex, const char* hs_hex, unsigned a_bits,
                             unsigned g, long long count, int threads, double* times) {
  bench_key k;
  mpz_inits(k.n, k.n2, k.p, k.q, k.p2, k.q2, k.hp, k.hq, k.qinv, k.mx, NULL);
  mpz_set_str(k.p, p_hex, 16);
  mpz_set_str(k.q, q_hex, 16);
  mpz_mul(k.n, k.p, k.q);
  mpz_mul(k.n2, k.n, k.n);
  mpz_mul(k.p2, k.p, k.p);
  mpz_mul(k.q2, k.q, k.q);
  h_func(k.hp, k.n, k.p, k.p2);
  h_func(k.hq, k.n, k.q, k.q2);
  mpz_invert(k.qinv, k.q, k.p);
  mpz_mul_2exp(k.mx, k.n, 1);
  mpz_cdiv_q_ui(k.mx, k.mx, 3);
  k.g = g;
  k.a_bits = a_bits;
  k.cols = (1ull << g) - 1;
  k.rows = a_bits / g + (a_bits % g ? 1 : 0);
  k.T = (mpz_t*)malloc(sizeof(mpz_t) * k.rows * k.cols);
  mpz_t hs;
  mpz_init_set_str(hs, hs_hex, 16);
  for (unsigned long long i = 0; i < k.rows * k.cols; ++i) mpz_init(k.T[i]);
  mpz_set(k.T[0], hs);
  for (unsigned long long j = 1; j < k.cols; ++j) {
    mpz_mul(k.T[j], k.T[j - 1], hs);
    mpz_mod(k.T[j], k.T[j], k.n2);
  }
  for (unsigned i = 1; i < k.rows; ++i)
    for (unsigned long long j = 0; j < k.cols; ++j)
      mpz_powm_ui(k.T[i * k.cols + j], k.T[(i - 1) * k.cols + j], 1ul << g, k.n2);
  char** cts = (char**)calloc((size_t)count, sizeof(char*));
  double t0 = now_s();
  bench_run(&k, 0, cts, count, threads);
  times[0] = now_s() - t0;
  t0 = now_s();
  bench_run(&k, 1, cts, count, threads);
  times[1] = now_s() - t0;
  void (*freefunc)(void*, size_t);
  mp_get_memory_functions(NULL, NULL, &freefunc);
  for (long long i = 0; i < count; ++i)
    if (cts[i]) freefunc(cts[i], strlen(cts[i]) + 1);
  free(cts);
  for (unsigned long long i = 0; i < k.rows * k.cols; ++i) mpz_clear(k.T[i]);
  free(k.T);
  mpz_clear(hs);
  mpz_clears(k.n, k.n2, k.p, k.q, k.p2, k.q2, k.hp, k.hq, k.qinv, k.mx, NULL);
}

/* ------------------------------------------------------------------------------------------
 * CPU baseline of PaillierMatmul (bench.py --stage p, cpu_baseline leg only), restating the op's
 * compute (paillier.cc:987-1041): every x ciphertext is inverted mod n^2 serially before the
 * sharded loop (:994-999); each output (i, k) takes min_j(xe + ye), then per term
 * powm(x, y) (y >= 0, x parsed from its hex string) or powm(x^-1, -y), powm by 2^(exp - min) and
 * a multiply mod n^2 into the sum (:1015-1032), and prints the sum as hex (:1034). Outputs are
 * split into contiguous blocks over `threads` pthreads. x: `rows * v` ciphertexts drawn uniformly
 * below n^2 from a fixed MT seed; xe [rows][v], ym / ye [v][w] as given. times[0] = inversion
 * seconds, times[1] = output-loop seconds (wall).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  mpz_srcptr n2;
  char** xs;
  mpz_t* xinv;
  const long long *xe, *ym, *ye;
  int v, w;
  long long lo, hi;
} mm_job;

static void* mm_worker(void* arg) {
  mm_job* jb = (mm_job*)arg;
  mpz_t addend, e, sum, x;
  mpz_inits(addend, e, sum, x, NULL);
  const int v = jb->v, w = jb->w;
  for (long long o = jb->lo; o < jb->hi; ++o) {
    const long long i = o / w, kk = o % w;
    long long mn = 0x7FFFFFFFFFFFFFFFLL;
    for (int j = 0; j < v; ++j) {
      const long long ex = jb->xe[i * v + j] + jb->ye[(long long)j * w + kk];
      if (ex < mn) mn = ex;
    }
    for (int j = 0; j < v; ++j) {
      const long long ex = jb->xe[i * v + j] + jb->ye[(long long)j * w + kk] - mn;
      const long long y = jb->ym[(long long)j * w + kk];
      const unsigned long long ay = y < 0 ? 0ull - (unsigned long long)y : (unsigned long long)y;
      mpz_import(e, 1, -1, sizeof(ay), 0, 0, &ay);
      if (y >= 0) {
        mpz_set_str(x, jb->xs[i * v + j], 16);
        mpz_powm(addend, x, e, jb->n2);
      } else {
        mpz_powm(addend, jb->xinv[i * v + j], e, jb->n2);
      }
      mpz_set_ui(e, 1);
      mpz_mul_2exp(e, e, (mp_bitcnt_t)ex);
      mpz_powm(addend, addend, e, jb->n2);
      if (!j) {
        mpz_set(sum, addend);
      } else {
        mpz_mul(sum, addend, sum);
        mpz_mod(sum, sum, jb->n2);
      }
    }
    char* s = mpz_get_str(NULL, 16, sum);
    void (*freefunc)(void*, size_t);
    mp_get_memory_functions(NULL, NULL, &freefunc);
    freefunc(s, strlen(s) + 1);
  }
  mpz_clears(addend, e, sum, x, NULL);
  return NULL;
}

EFL_EXPORT void pl_gmp_matmul_bench(const char* n_hex, const long long* xe, const long long* ym,
                                    const long long* ye, int rows, int v, int w, int threads, double* times) {
  mpz_t n, n2, c;
  mpz_inits(n, n2, c, NULL);
  mpz_set_str(n, n_hex, 16);
  mpz_mul(n2, n, n);
  const long long nx = (long long)rows * v;
  char** xs = (char**)calloc((size_t)nx, sizeof(char*));
  mpz_t* xinv = (mpz_t*)malloc(sizeof(mpz_t) * (size_t)nx);
  gmp_randstate_t st;
  gmp_randinit_mt(st);
  gmp_randseed_ui(st, 2024ul);
  for (long long t = 0; t < nx; ++t) {
    do {
      mpz_urandomm(c, st, n2);
    } while (mpz_sgn(c) == 0);
    xs[t] = mpz_get_str(NULL, 16, c);
    mpz_init(xinv[t]);
  }
  double t0 = now_s();
  for (long long t = 0; t < nx; ++t) {
    mpz_set_str(c, xs[t], 16);
    mpz_invert(xinv[t], c, n2);
  }
  times[0] = now_s() - t0;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  mm_job jobs[256];
  const long long outs = (long long)rows * w;
  t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (mm_job){n2, xs, xinv, xe, ym, ye, v, w, outs * t / threads, outs * (t + 1) / threads};
    pthread_create(&th[t], NULL, mm_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  times[1] = now_s() - t0;
  void (*freefunc)(void*, size_t);
  mp_get_memory_functions(NULL, NULL, &freefunc);
  for (long long t = 0; t < nx; ++t) {
    freefunc(xs[t], strlen(xs[t]) + 1);
    mpz_clear(xinv[t]);
  }
  free(xs);
  free(xinv);
  gmp_randclear(st);
  mpz_clears(n, n2, c, NULL);
}
