/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the product
 * path (libefl_hip.so / the `efl` package). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the fixed-point codec of efls-train:
 *   encode  = Convert2FixedPointOp<float|double|intX>::Compute
 *             efls-train/cc/efl/math/fixed_point.cc:53-69 (ints), :106-138 (float), :156-188 (double)
 *   decode  = FixedPointToFloatPointOp<int64, float|double>::Compute
 *             efls-train/cc/efl/math/fixed_point.cc:235-248, Input2Mpf :259-265
 *             (GMP mpf_set_z -> mpf_mul_2exp / mpf_div_2exp -> mpf_get_d -> implicit double->Tout)
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - encode: against the reference-loop outputs recorded in SURVEY.md Appendix A (the survey ran
 *     the reference loop body in this container) and against an independent numpy restatement
 *     (oracle/fxp.py, np_encode_*).
 *   - decode: against GMP 6.2.1 itself (oracle/fxp_gmp.c calls mpf_* in the reference's call
 *     order, fixed_point.cc:238-246), golden vectors in tests/golden/.
 *
 * Every rule below is written out explicitly; the one C++ UB of the reference (shift by
 * 0u-127 when the mantissa is 0, fixed_point.cc:127-129) is given the value x86-64 gcc
 * produces (rule A5): M = 0, E = exp - 127.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

#define EFL_EXPORT __attribute__((visibility("default")))

/* --------------------------------------------------------------------------------------- */
/* encode                                                                                   */
/* --------------------------------------------------------------------------------------- */

/* fixed_point.cc:108-136, one fp32 word. */
static inline void enc_f32_one(uint32_t bits, int dp, int64_t* M, int64_t* E) {
  uint32_t sign = bits >> 31;                         /* :109-110 */
  int32_t exp = (int32_t)((bits >> 23) & 0xFFu) - 150; /* :111  bias 127 + 23 fraction bits */
  /* :113 `exp == 0xFF` can never hold (exp in [-150, 105]); inf/NaN fall through (A2). */
  int32_t mant = (int32_t)(bits & 0x7FFFFFu);          /* :116 */
  if (exp != 0) mant |= 0x800000;                      /* :117-119 test on the SHIFTED exponent (A3) */
  if (dp) {                                            /* :121-124 decrease_precision */
    mant >>= 13;
    exp += 13;
  }
  if (mant == 0) {
    /* :126-129 with mant == 0: f = 0.0f, r = 0u - 127; mant stays 0, exp wraps to exp - 127 (A5). */
    exp -= 127;
  } else {
    int r = __builtin_ctz((uint32_t)mant);             /* :126-127 lowest set bit via float exponent */
    mant >>= r;                                        /* :128 */
    exp += r;                                          /* :129 */
  }
  *M = sign ? -(int64_t)mant : (int64_t)mant;          /* :131-135 */
  *E = (int64_t)exp;                                   /* :136 */
}

/* fixed_point.cc:158-186, one fp64 word. */
static inline void enc_f64_one(uint64_t bits, int dp, int64_t* M, int64_t* E) {
  uint64_t sign = bits >> 63;                             /* :159-160 */
  int64_t exp = (int64_t)((bits >> 52) & 0x7FFu) - 1075;   /* :161 */
  int64_t mant = (int64_t)(bits & 0xFFFFFFFFFFFFFull);     /* :166 */
  if (exp != 0) mant |= 0x10000000000000ll;                /* :167-169 */
  if (dp) {                                                /* :171-174 */
    mant >>= 42;
    exp += 42;
  }
  if (mant == 0) {
    exp -= 1023;                                           /* :176-179 with mant == 0 (A5, fp64 form) */
  } else {
    int r = __builtin_ctzll((uint64_t)mant);
    mant >>= r;
    exp += r;
  }
  *M = sign ? -mant : mant;
  *E = exp;
}

EFL_EXPORT void oracle_encode_f32(const float* x, int64_t* M, int64_t* E, int64_t n, int dp) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t b;
    memcpy(&b, &x[i], 4);
    enc_f32_one(b, dp, &M[i], &E[i]);
  }
}

EFL_EXPORT void oracle_encode_f64(const double* x, int64_t* M, int64_t* E, int64_t n, int dp) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t b;
    memcpy(&b, &x[i], 8);
    enc_f64_one(b, dp, &M[i], &E[i]);
  }
}

/* fixed_point.cc:53-69: M = x (sign-extended), E = 0. elem_bytes in {1,2,4,8}. */
EFL_EXPORT void oracle_encode_int(const void* x, int elem_bytes, int64_t* M, int64_t* E, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t v = 0;
    switch (elem_bytes) {
      case 1: v = ((const int8_t*)x)[i]; break;
      case 2: v = ((const int16_t*)x)[i]; break;
      case 4: v = ((const int32_t*)x)[i]; break;
      default: v = ((const int64_t*)x)[i]; break;
    }
    M[i] = v;
    E[i] = 0;
  }
}

/* --------------------------------------------------------------------------------------- */
/* decode                                                                                   */
/* --------------------------------------------------------------------------------------- */

/*
 * Value of GMP's mpf_get_d for the exact quantity (-1)^neg * a * 2^e, a > 0 (GMP 6.x
 * mpn_get_d, IEEE-double path): the top 53 bits of a are kept by TRUNCATION; with L the
 * position of the leading bit of a*2^e:
 *   L >= 1024          -> +-inf
 *   -1022 <= L < 1024  -> normal double, truncated
 *   -1074 <= L < -1022 -> denormal double, truncated toward zero (sign kept)
 *   L <= -1075         -> +0.0 (sign dropped)
 * fixed_point.cc:238-245 reaches exactly this value: mpf_set_z, mpf_mul_2exp and mpf_div_2exp
 * are exact for a one-limb operand at the default precision.
 */
EFL_EXPORT uint64_t oracle_gmp_get_d_bits(uint64_t a, int neg, int64_t e) {
  const uint64_t sgn = neg ? (1ull << 63) : 0;
  if (a == 0) return 0;                                   /* mpf zero -> +0.0 */
  int p = 63 - __builtin_clzll(a);
  if (e > 4096) return sgn | 0x7FF0000000000000ull;
  if (e < -8192) return 0;
  int64_t L = (int64_t)p + e;
  if (L >= 1024) return sgn | 0x7FF0000000000000ull;
  if (L <= -1075) return 0;
  uint64_t m53 = p >= 52 ? (a >> (p - 52)) : (a << (52 - p));   /* leading bit at 52 */
  uint64_t bits;
  if (L >= -1022) {
    bits = ((uint64_t)(L + 1023) << 52) | (m53 & 0xFFFFFFFFFFFFFull);
  } else {
    bits = m53 >> (-1022 - L);                            /* 1..52 */
  }
  return sgn | bits;
}

static inline double bits2d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static inline uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/*
 * double -> float as the reference's implicit conversion (fixed_point.cc:245, y is float):
 * round-to-nearest-even. `ftz` = 1 reproduces the MXCSR state TensorFlow's CPU threadpool
 * threads run kernels in (FTZ+DAZ). x86 detects tininess AFTER rounding to 24 bits with an
 * unbounded exponent, so the result is flushed to a zero of d's sign exactly when
 * |d| < 2^-126 - 2^-151 (= 0x1.ffffffp-127); DAZ is subsumed (denormal doubles are far below).
 */
EFL_EXPORT uint32_t oracle_d2f_bits(uint64_t dbits, int ftz) {
  double d = bits2d(dbits);
  if (ftz && fabs(d) < 0x1.ffffffp-127) return (uint32_t)(dbits >> 32) & 0x80000000u;
  return f2bits((float)d);                                /* host default rounding: RNE */
}

static inline uint64_t dec_one_d(int64_t M, int64_t E) {
  uint64_t a = M < 0 ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  return oracle_gmp_get_d_bits(a, M < 0, E);
}

EFL_EXPORT void oracle_decode_f32(const int64_t* M, const int64_t* E, float* y, int64_t n, int ftz) {
  for (int64_t i = 0; i < n; ++i) y[i] = bits2f(oracle_d2f_bits(dec_one_d(M[i], E[i]), ftz));
}

EFL_EXPORT void oracle_decode_f64(const int64_t* M, const int64_t* E, double* y, int64_t n) {
  for (int64_t i = 0; i < n; ++i) y[i] = bits2d(dec_one_d(M[i], E[i]));
}

/*
 * Hex-string mantissa (FixedPointToFloatPointOp<string, *>, fixed_point.cc:255-257:
 * mpf_set_str(rop, s, 16)). Lower-case or upper-case digits, optional leading '-'. The value is
 * truncated at every mpf step, which composes to: keep the leading 64 bits of |m|, remember
 * its bit length. Returns -1 on a malformed string (the reference ignores mpf_set_str's return
 * code; the build reports InvalidArgument instead).
 */
EFL_EXPORT int oracle_hex_top64(const char* s, int64_t len, uint64_t* top, int64_t* shift, int* neg) {
  int64_t i = 0;
  *neg = 0;
  if (len > 0 && s[0] == '-') { *neg = 1; i = 1; }
  if (i >= len) return -1;
  /* skip leading zeros */
  while (i < len && s[i] == '0') ++i;
  uint64_t acc = 0;
  int64_t nbits = 0;          /* significant bits consumed into acc (max 64) */
  int64_t extra = 0;          /* bits dropped below acc */
  for (; i < len; ++i) {
    char c = s[i];
    int v;
    if (c >= '0' && c <= '9') v = c - '0';
    else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v = c - 'A' + 10;
    else return -1;
    if (nbits == 0) {
      if (v == 0) continue;   /* unreachable after zero skip, kept for safety */
      acc = (uint64_t)v;
      nbits = 64 - __builtin_clzll(acc);
    } else if (nbits + 4 <= 64) {
      acc = (acc << 4) | (uint64_t)v;
      nbits += 4;
    } else {
      int room = (int)(64 - nbits);            /* 0..3 */
      if (room > 0) {
        acc = (acc << room) | ((uint64_t)v >> (4 - room));
        nbits = 64;
      }
      extra += 4 - room;
    }
  }
  *top = acc;
  *shift = extra;                               /* |m| ~ acc * 2^extra (truncated) */
  if (acc == 0) { *neg = 0; *shift = 0; }
  return 0;
}

/* Decode of one hex mantissa; returns 0 / -1 like oracle_hex_top64. */
EFL_EXPORT int oracle_decode_hex_d(const char* s, int64_t len, int64_t E, uint64_t* dbits) {
  uint64_t top; int64_t sh; int neg;
  if (oracle_hex_top64(s, len, &top, &sh, &neg)) return -1;
  *dbits = oracle_gmp_get_d_bits(top, neg, E + sh);
  return 0;
}
