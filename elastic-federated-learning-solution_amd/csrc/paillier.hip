// Stage P — Paillier cipher of EFLS-train's forward-encryption path on MI355X (gfx950).
//
// Reference: efls-train/cc/efl/math/paillier.cc
//   PaillierKeypair::Encrypt :103-131 (hsa given, or hsa = fbpowm(random a) when "0")
//   _Decrypt :296-312 with m-function :39-48, h-function :28-37
//   FixedBasePowm (table + lookup with per-group bit-reversed index) gmp_utils.cc:56-144
//   Add/MulScalar/MulExp2/Invert :157-285
//
// One ciphertext per lane. Big numbers are little-endian 32-bit limbs, element-major in HBM
// ([N][L]); per lane they live in VGPRs (operand a, accumulator t) and in the lane's LDS column
// (operand b, stride = workgroup size). Moduli and key constants are wave-uniform (scalar loads).
// The per-element randomness `a` of hsa = hs^a comes from Philox4x32-10 keyed by the broadcast
// seed with counter = global element index (counter-based: independent of GPU count/launch shape).
#include "bignum.h"
#include "common.h"

#include <type_traits>
#include "pl_common.h"

namespace efl {
namespace {

using namespace big;
using pl::Key;
using pl::philox;

constexpr int kPlBlock = 64;   // one wave per workgroup: LDS columns are per lane

// a = Philox stream of `words` 32-bit words for element counter ctr, written to an LDS column.
__device__ __forceinline__ void draw_a(uint32_t* col, int S, int words, int a_bits, uint64_t seed,
                                       uint64_t ctr) {
  for (int b = 0; b * 4 < words; ++b) {
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)b, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (b * 4 + j < words) col[(b * 4 + j) * S] = c[j];
  }
  const int rem = a_bits & 31;
  if (rem) col[(words - 1) * S] &= (1u << rem) - 1u;
}

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------

template <int L>
__device__ __forceinline__ void load_g(uint32_t (&x)[L], const uint32_t* __restrict__ g) {
#pragma unroll
  for (int j = 0; j < L; j += 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(g + j);
    x[j] = v.x; x[j + 1] = v.y; x[j + 2] = v.z; x[j + 3] = v.w;
  }
}

template <int L>
__device__ __forceinline__ void store_g(uint32_t* __restrict__ g, const uint32_t (&x)[L]) {
#pragma unroll
  for (int j = 0; j < L; j += 4) *reinterpret_cast<uint4*>(g + j) = make_uint4(x[j], x[j + 1], x[j + 2], x[j + 3]);
}

template <int L>
__device__ __forceinline__ void load_uniform(uint32_t (&x)[L], const uint32_t* __restrict__ g) {
#pragma unroll
  for (int j = 0; j < L; ++j) x[j] = g[j];
}

// copy L limbs from global (per lane) into the lane's LDS column
template <int L>
__device__ __forceinline__ void g_to_lds(uint32_t* col, int S, const uint32_t* __restrict__ g) {
#pragma unroll
  for (int j = 0; j < L; j += 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(g + j);
    col[j * S] = v.x; col[(j + 1) * S] = v.y; col[(j + 2) * S] = v.z; col[(j + 3) * S] = v.w;
  }
}

// g = 1 + a*n  (a = |m|, 64-bit) or its inverse mod n^2, 1 - a*n = n^2 + 1 - a*n  (m < 0).
// paillier.cc:110-124: (1+|m|n)^-1 mod n^2 is exactly n^2 + 1 - |m|n because (1+an)(1-an) = 1 - a^2 n^2.
template <int LN>
__device__ __forceinline__ void make_g(uint32_t (&g)[2 * LN], long long m, const uint32_t* __restrict__ n,
                                       const uint32_t* __restrict__ n2) {
  constexpr int LC = 2 * LN;
  const uint64_t a = m < 0 ? 0ull - (uint64_t)m : (uint64_t)m;
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
  // prod = a * n (LN + 2 limbs)
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int j = 0; j < LC; ++j) g[j] = 0;
#pragma unroll
  for (int j = 0; j < LN; ++j) {
    const uint64_t p = mad(a0, n[j], (uint64_t)g[j] + c0);
    g[j] = (uint32_t)p;
    c0 = (uint32_t)(p >> 32);
  }
  g[LN] = c0;
#pragma unroll
  for (int j = 0; j < LN; ++j) {
    const uint64_t p = mad(a1, n[j], (uint64_t)g[j + 1] + c1);
    g[j + 1] = (uint32_t)p;
    c1 = (uint32_t)(p >> 32);
  }
  g[LN + 1] += c1;
  if (m < 0) {
    // g = n2 - g + 1
    uint32_t borrow = 0;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const uint64_t d = (uint64_t)n2[j] - g[j] - borrow;
      g[j] = (uint32_t)d;
      borrow = (uint32_t)(d >> 63);
    }
  }
  // + 1
  uint32_t c = 1;
#pragma unroll
  for (int j = 0; j < LC; ++j) {
    const uint64_t s = (uint64_t)g[j] + c;
    g[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
}

// ------------------------------------------------------------------------------------------
// fixed-base exponentiation hs^(a') mod n^2 through the table (gmp_utils.cc:107-144): a' = a with
// every group_size-bit group bit-reversed (the reference's index order, pl_common.h), formed in
// place in the lane's column, then taken in plain windows of the table's width W. Table entries
// T[i][j] = hs^((j+1) 2^(W i)) in Montgomery form. Returns acc = hs^(a') * R mod n^2.
// ------------------------------------------------------------------------------------------
template <int LC>
__device__ __forceinline__ void fbpowm_mont(uint32_t (&acc)[LC], const Key& k, uint32_t* acol,
                                            uint32_t* bcol, int S) {
  const int words = (k.d.a_bits + 31) >> 5;
  const int size = pl::col_bit_length(acol, S, words);
  pl::regroup_exponent(acol, S, size, k.d.group_size, words);
  const int W = pl::table_window(k.d);
  load_uniform<LC>(acc, k.at(k.d.off_n2_one));
  const uint32_t* n2 = k.at(k.d.off_n2);
  const uint32_t* table = k.at(k.d.off_table);
  const int cols = k.d.table_cols;
  for (int s = 0, row = 0; s < size; s += W, ++row) {
    const uint32_t idx = pl::col_bits(acol, S, s, size - s < W ? size - s : W, words);
    if (idx) {
      g_to_lds<LC>(bcol, S, table + ((int64_t)row * cols + (idx - 1)) * LC);
      mont_mul<LC>(acc, LdsCol{bcol, S}, n2, k.d.n2_minv);
    }
  }
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------

// Encrypt (paillier.cc:103-131). hsa: [N][LC] normal-form limbs, or null -> fbpowm of a fresh a.
template <int LN>
__global__ __launch_bounds__(kPlBlock) void k_encrypt(Key k, const long long* __restrict__ m,
                                                      const uint32_t* hsa, uint32_t* out, long long N,
                                                      uint64_t seed, long long ctr0, int hsa_mont) {
  constexpr int LC = 2 * LN;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  const int awords = (k.d.a_bits + 31) >> 5;
  uint32_t* acol = lds + threadIdx.x;                               // a (or squaring scratch)
  uint32_t* bcol = lds + (awords > LC ? awords : LC) * S + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t* n = k.at(k.d.off_n);
  const uint32_t* n2 = k.at(k.d.off_n2);
  uint32_t c[LC];
  if (hsa) {
    // c = g * hsa mod n^2 = mont(mont(g, hsa), R^2)
    make_g<LN>(c, m[i], n, n2);
    g_to_lds<LC>(bcol, S, hsa + i * LC);
    mont_mul<LC>(c, LdsCol{bcol, S}, n2, k.d.n2_minv);
    if (!hsa_mont) mont_mul<LC>(c, Uniform{k.at(k.d.off_n2_r2)}, n2, k.d.n2_minv);   // hsa_mont: hsa R given
  } else {
    draw_a(acol, S, (k.d.a_bits + 31) >> 5, k.d.a_bits, seed, (uint64_t)(ctr0 + i));
    fbpowm_mont<LC>(c, k, acol, bcol, S);      // hs^a' * R
    to_lds<LC>(bcol, S, c);
    make_g<LN>(c, m[i], n, n2);
    mont_mul<LC>(c, LdsCol{bcol, S}, n2, k.d.n2_minv);   // g * hs^a'
  }
  store_g<LC>(out + i * LC, c);
}

// hsa only (hs^a' for a given / drawn a), normal form — exposed for parity with FixedBasePowm.
template <int LN>
__global__ __launch_bounds__(kPlBlock) void k_fbpowm(Key k, const uint32_t* __restrict__ a_in,
                                                     uint32_t* __restrict__ out, long long N,
                                                     uint64_t seed, long long ctr0) {
  constexpr int LC = 2 * LN;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* acol = lds + threadIdx.x;
  uint32_t* bcol = lds + (words > LC ? words : LC) * S + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (a_in) {
    for (int w = 0; w < words; ++w) acol[w * S] = a_in[i * words + w];
  } else {
    draw_a(acol, S, words, k.d.a_bits, seed, (uint64_t)(ctr0 + i));
  }
  uint32_t acc[LC];
  fbpowm_mont<LC>(acc, k, acol, bcol, S);
  redc<LC>(acc, k.at(k.d.off_n2), k.d.n2_minv);
  store_g<LC>(out + i * LC, acc);
}

// z (2 L + 1 words) += f y for a uniform L-word f and a register L-word y, row R onwards. The rows
// are a template recursion so every index is a compile-time constant (a fully unrolled L x L
// nest leaves z in scratch).
template <int L, int R>
__device__ __forceinline__ void add_product(uint32_t (&z)[2 * L + 1], const uint32_t (&y)[L],
                                            const uint32_t* __restrict__ f, uint32_t over = 0) {
  if constexpr (R < L) {
    const uint32_t fr = f[R];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t p = mad(fr, y[j], (uint64_t)z[R + j] + c);
      z[R + j] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    const uint64_t t = (uint64_t)z[R + L] + c + over;   // over: carry out of word R + L - 1's row
    z[R + L] = (uint32_t)t;
    add_product<L, R + 1>(z, y, f, (uint32_t)(t >> 32));
  } else {
    z[2 * L] += over;
  }
}

// CRT join (efl_pl_crt_join): z = q^2 yp + p^2 yq mod n^2 for yp < p^2, yq < q^2 ([N][LN] words,
// LN = the key's ln; z [N][2 LN]). With yp = x (q^2)^-1 mod p^2 and yq = x (p^2)^-1 mod q^2, z is x
// mod n^2 (z = x mod p^2 and mod q^2). The key owner's encryption gets yp and yq straight from the
// fixed-base walks mod p^2 and mod q^2, whose accumulators start from (q^2)^-1 and (p^2)^-1 instead
// of 1 (KeyBlock walk_start), so the join is two plain LN x LN products, a sum and at most one
// subtraction of n^2 — no modular product. One lane per element, the operand in registers; the sum
// (2 LN + 1 words: q^2 yp + p^2 yq < 2 n^2) in registers for LN <= 32 (at LN = 64 that takes 766
// registers and spills), else row by row into the lane's LDS column.
template <int LN>
__global__ __launch_bounds__(kPlBlock) void k_crt_join(Key k, const uint32_t* __restrict__ yp,
                                                       const uint32_t* __restrict__ yq,
                                                       uint32_t* __restrict__ out, long long N) {
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  uint32_t* zcol = lds + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if constexpr (LN <= 32) {
    // the sum in registers (2 LN + 1 words), both products fully unrolled: no LDS round trips
    uint32_t z[2 * LN + 1], y[LN];
#pragma unroll
    for (int j = 0; j <= 2 * LN; ++j) z[j] = 0u;
    load_g<LN>(y, yp + i * LN);
    add_product<LN, 0>(z, y, k.at(k.d.off_q2));
    load_g<LN>(y, yq + i * LN);
    add_product<LN, 0>(z, y, k.at(k.d.off_p2));
    const uint32_t* n2 = k.at(k.d.off_n2);
    uint32_t borrow = 0;
#pragma unroll
    for (int j = 0; j < 2 * LN; ++j) borrow = (uint32_t)(((uint64_t)z[j] - n2[j] - borrow) >> 63);
    const bool ge = z[2 * LN] >= borrow;
    borrow = 0;
#pragma unroll
    for (int j = 0; j < 2 * LN; ++j) {
      const uint64_t d = (uint64_t)z[j] - (ge ? n2[j] : 0u) - borrow;
      z[j] = (uint32_t)d;
      borrow = (uint32_t)(d >> 63);
    }
    uint32_t zz[2 * LN];
#pragma unroll
    for (int j = 0; j < 2 * LN; ++j) zz[j] = z[j];
    store_g<2 * LN>(out + i * (2 * LN), zz);
    return;
  }
#pragma unroll 4
  for (int j = 0; j <= 2 * LN; ++j) zcol[j * S] = 0u;
  uint32_t y[LN];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    load_g<LN>(y, (pass ? yq : yp) + i * LN);
    const uint32_t* f = k.at(pass ? k.d.off_p2 : k.d.off_q2);
    uint32_t over = 0;   // carry out of word r + LN of the previous row
#pragma unroll 1
    for (int r = 0; r < LN; ++r) {
      asm volatile("" ::: "memory");
      const uint32_t fr = f[r];
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < LN; ++j) {
        const uint64_t p = mad(fr, y[j], (uint64_t)zcol[(r + j) * S] + c);
        zcol[(r + j) * S] = (uint32_t)p;
        c = (uint32_t)(p >> 32);
      }
      const uint64_t t = (uint64_t)zcol[(r + LN) * S] + c + over;
      zcol[(r + LN) * S] = (uint32_t)t;
      over = (uint32_t)(t >> 32);
    }
    zcol[2 * LN * S] += over;
  }
  // z >= n^2 ? z - n^2 : z
  const uint32_t* n2 = k.at(k.d.off_n2);
  uint32_t borrow = 0;
#pragma unroll 4
  for (int j = 0; j < 2 * LN; ++j) borrow = (uint32_t)(((uint64_t)zcol[j * S] - n2[j] - borrow) >> 63);
  const bool ge = zcol[2 * LN * S] >= borrow;   // word 2 LN is 0 or 1
  borrow = 0;
  uint32_t* o = out + i * (2 * LN);
#pragma unroll 2
  for (int j = 0; j < 2 * LN; j += 4) {
    uint32_t w[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t d = (uint64_t)zcol[(j + t) * S] - (ge ? n2[j + t] : 0u) - borrow;
      w[t] = (uint32_t)d;
      borrow = (uint32_t)(d >> 63);
    }
    *reinterpret_cast<uint4*>(o + j) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// m_x(c) = L_x(c^(x-1) mod x^2) * h mod x   (paillier.cc:39-48), x = p or q.
// lo/hi: the 2*LP limbs of c (consumed). Result: LH limbs.
template <int LP>
__device__ __forceinline__ void m_func(uint32_t (&res)[LP / 2], uint32_t (&lo)[LP], uint32_t (&hi)[LP],
                                       const Key& k, bool second, uint32_t* acol, uint32_t* bcol, int S) {
  constexpr int LH = LP / 2;
  const uint32_t* x2 = k.at(second ? k.d.off_q2 : k.d.off_p2);
  const uint32_t x2_minv = second ? k.d.q2_minv : k.d.p2_minv;
  const uint32_t* r3 = k.at(second ? k.d.off_q2_r3 : k.d.off_p2_r3);
  const uint32_t* e = k.at(second ? k.d.off_qm1 : k.d.off_pm1);
  const int ebits = second ? k.d.qm1_bits : k.d.pm1_bits;
  const uint32_t* x = k.at(second ? k.d.off_q : k.d.off_p);
  const uint32_t x_minv = second ? k.d.q_minv : k.d.p_minv;
  const uint32_t* xinv_w = k.at(second ? k.d.off_qinv_w : k.d.off_pinv_w);
  const uint32_t* h_m = k.at(second ? k.d.off_hq : k.d.off_hp);

  redc_wide<LP>(lo, hi, x2, x2_minv);                        // hi = c R^-1 mod x^2
  mont_mul<LP>(hi, Uniform{r3}, x2, x2_minv);                 // c R mod x^2 (Montgomery form)
  to_lds<LP>(bcol, S, hi);
  // left-to-right binary exponentiation by the (uniform) exponent x - 1; top bit is 1
#pragma unroll 1
  for (int b = ebits - 2; b >= 0; --b) {
    mont_sqr<LP>(hi, acol, S, x2, x2_minv);
    if ((e[b >> 5] >> (b & 31)) & 1u) mont_mul<LP>(hi, LdsCol{bcol, S}, x2, x2_minv);
  }
  redc<LP>(hi, x2, x2_minv);                                  // y = c^(x-1) mod x^2
  const uint32_t (&y)[LP] = hi;
  // L: (y - 1) / x exactly = (y - 1) * x^-1 mod 2^(32 LH)   (quotient < x)
  uint32_t y1[LH];
  uint32_t borrow = 1;
#pragma unroll
  for (int j = 0; j < LH; ++j) {
    const uint64_t d = (uint64_t)y[j] - borrow;
    y1[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  uint32_t q[LH];
#pragma unroll
  for (int j = 0; j < LH; ++j) q[j] = 0;
#pragma unroll
  for (int i = 0; i < LH; ++i) {
    uint32_t c = 0;
    const uint32_t yi = y1[i];
#pragma unroll
    for (int j = 0; i + j < LH; ++j) {
      const uint64_t p = mad(yi, xinv_w[j], (uint64_t)q[i + j] + c);
      q[i + j] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
  }
  // * h mod x  (h in Montgomery form -> normal result)
  mont_mul<LH>(q, Uniform{h_m}, x, x_minv);
  copy<LH>(res, q);
}

// Decrypt (paillier.cc:296-312). ct: [N][2LP]; out magnitude [N][LP], neg [N] (1 if m < 0).
template <int LP>
__global__ __launch_bounds__(kPlBlock) void k_decrypt(Key k, const uint32_t* __restrict__ ct,
                                                      uint32_t* __restrict__ mag,
                                                      signed char* __restrict__ neg, long long N) {
  constexpr int LH = LP / 2;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  uint32_t* acol = lds + threadIdx.x;
  uint32_t* bcol = lds + LP * S + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t* c = ct + i * 2 * LP;
  uint32_t lo[LP], hi[LP], mp[LH], mq[LH];
  load_g<LP>(lo, c);
  load_g<LP>(hi, c + LP);
  m_func<LP>(mp, lo, hi, k, false, acol, bcol, S);
  load_g<LP>(lo, c);
  load_g<LP>(hi, c + LP);
  m_func<LP>(mq, lo, hi, k, true, acol, bcol, S);
  // CRT: m = ((mp - mq) mod p) * (q^-1 mod p) mod p * q + mq
  const uint32_t* p = k.at(k.d.off_p);
  const uint32_t* q = k.at(k.d.off_q);
  uint32_t mqp[LH];
  copy<LH>(mqp, mq);
  csub<LH>(mqp, p, geq<LH>(mqp, p));                        // mq < q < 2p
  uint32_t d[LH];
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < LH; ++j) {
    const uint64_t x = (uint64_t)mp[j] - mqp[j] - borrow;
    d[j] = (uint32_t)x;
    borrow = (uint32_t)(x >> 63);
  }
  if (borrow) {
    uint32_t c2 = 0;
#pragma unroll
    for (int j = 0; j < LH; ++j) {
      const uint64_t s = (uint64_t)d[j] + p[j] + c2;
      d[j] = (uint32_t)s;
      c2 = (uint32_t)(s >> 32);
    }
  }
  mont_mul<LH>(d, Uniform{k.at(k.d.off_qinvp)}, p, k.d.p_minv);
  const uint32_t (&h)[LH] = d;
  // m = h * q + mq  (< n)
  uint32_t m[LP];
#pragma unroll
  for (int j = 0; j < LP; ++j) m[j] = j < LH ? mq[j < LH ? j : 0] : 0;
#pragma unroll
  for (int a = 0; a < LH; ++a) {
    uint32_t cc = 0;
#pragma unroll
    for (int b = 0; b < LH; ++b) {
      const uint64_t pr = mad(h[a], q[b], (uint64_t)m[a + b] + cc);
      m[a + b] = (uint32_t)pr;
      cc = (uint32_t)(pr >> 32);
    }
#pragma unroll
    for (int b = a + LH; b < LP; ++b) {
      const uint64_t s = (uint64_t)m[b] + cc;
      m[b] = (uint32_t)s;
      cc = (uint32_t)(s >> 32);
    }
  }
  // signed: if m > max (= ceil(2n/3)) then m - n  (paillier.cc:308-310)
  const uint32_t* mx = k.at(k.d.off_max);
  uint32_t bb = 0;
#pragma unroll
  for (int j = 0; j < LP; ++j) {   // borrow of max - m  -> set iff m > max
    const uint64_t x = (uint64_t)mx[j] - m[j] - bb;
    bb = (uint32_t)(x >> 63);
  }
  const bool isneg = bb != 0;
  if (isneg) {   // |m - n| = n - m
    const uint32_t* n = k.at(k.d.off_n);
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const uint64_t x = (uint64_t)n[j] - m[j] - br;
      m[j] = (uint32_t)x;
      br = (uint32_t)(x >> 63);
    }
  }
  store_g<LP>(mag + i * LP, m);
  neg[i] = isneg ? 1 : 0;
}

// c = x * y mod n^2 (PaillierAdd, paillier.cc:157-178)
template <int LN>
__global__ __launch_bounds__(kPlBlock) void k_add(Key k, const uint32_t* __restrict__ x,
                                                  const uint32_t* __restrict__ y,
                                                  uint32_t* __restrict__ out, long long N) {
  constexpr int LC = 2 * LN;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  uint32_t* bcol = lds + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t* n2 = k.at(k.d.off_n2);
  uint32_t a[LC];
  load_g<LC>(a, x + i * LC);
  g_to_lds<LC>(bcol, S, y + i * LC);
  mont_mul<LC>(a, LdsCol{bcol, S}, n2, k.d.n2_minv);
  mont_mul<LC>(a, Uniform{k.at(k.d.off_n2_r2)}, n2, k.d.n2_minv);
  store_g<LC>(out + i * LC, a);
}

// c = x^e mod n^2 for a per-element non-negative exponent read through `xs` (pl_common.h: 32-bit
// words, |int64| or 2^int64; MulScalar / MulExp2, paillier.cc:180-265, 683-719; a negative scalar
// is finished by an inversion, efl_pl_mul_scalar). Elements whose exponent is not ok get 0 and
// their index in `bad`.
template <int LN, class XS>
__global__ __launch_bounds__(kPlBlock) void k_powm(Key k, const uint32_t* __restrict__ x, XS xs,
                                                   uint32_t* __restrict__ out, long long N,
                                                   unsigned long long* bad) {
  constexpr int LC = 2 * LN;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  uint32_t* acol = lds + threadIdx.x;
  uint32_t* bcol = lds + LC * S + threadIdx.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t* n2 = k.at(k.d.off_n2);
  const auto ex = xs.at(i);
  const int ebits = ex.ok ? ex.bits() : 0;
  uint32_t t[LC];
  if (ebits == 0) {
    // x^0 = 1 (mpz_powm: 1 mod n^2)
#pragma unroll
    for (int j = 0; j < LC; ++j) t[j] = (ex.ok && j == 0) ? 1u : 0u;
    store_g<LC>(out + i * LC, t);
    if (!ex.ok) atomicMin(bad, (unsigned long long)i);
    return;
  }
  load_g<LC>(t, x + i * LC);
  mont_mul<LC>(t, Uniform{k.at(k.d.off_n2_r2)}, n2, k.d.n2_minv);   // x R
  to_lds<LC>(bcol, S, t);
#pragma unroll 1
  for (int b = ebits - 2; b >= 0; --b) {
    mont_sqr<LC>(t, acol, S, n2, k.d.n2_minv);
    if (ex.bit(b)) mont_mul<LC>(t, LdsCol{bcol, S}, n2, k.d.n2_minv);
  }
  redc<LC>(t, n2, k.d.n2_minv);
  store_g<LC>(out + i * LC, t);
}

// ------------------------------------------------------------------------------------------
// x^-1 mod n^2 (mpz_invert, paillier.cc:267-285): limb helpers over numbers kept in a lane's LDS
// column (LdsNum) or, for the Bezout coefficients of keys up to 1024 bits, in registers (RegNum);
// the kernel (k_invert, Pornin's batched binary GCD) is below.
// ------------------------------------------------------------------------------------------
template <int L>
struct LdsNum {
  uint32_t* p;
  int S;
  __device__ __forceinline__ uint32_t& operator[](int j) const { return p[j * S]; }
};

// a number in registers: only ever indexed by fully unrolled loops (constant j)
template <int L>
struct RegNum {
  uint32_t v[L];
  __device__ __forceinline__ uint32_t& operator[](int j) { return v[j]; }
  __device__ __forceinline__ uint32_t operator[](int j) const { return v[j]; }
};

template <int L>
__device__ __forceinline__ bool lds_is_zero(const LdsNum<L>& x) {
  uint32_t o = 0;
  for (int j = 0; j < L; ++j) o |= x[j];
  return o == 0;
}

// x >>= k (0 < k < 32)
template <int L>
__device__ __forceinline__ void lds_shr(const LdsNum<L>& x, int k) {
  uint32_t lo = x[0];
  for (int j = 0; j < L - 1; ++j) {
    const uint32_t hi = x[j + 1];
    x[j] = (lo >> k) | (hi << (32 - k));
    lo = hi;
  }
  x[L - 1] = lo >> k;
}

// A <- A * 2^-k mod M (A < M, 0 < k < 32)
template <int L>
__device__ __forceinline__ void lds_half_k(const LdsNum<L>& A, int k, const uint32_t* __restrict__ M, uint32_t minv) {
  const uint32_t t = (A[0] * minv) & ((1u << k) - 1u);
  // A + t*M  (L+1 limbs), then >> k
  uint32_t c = 0;
  uint32_t prev = 0;
  for (int j = 0; j < L; ++j) {
    const uint64_t s = mad(t, M[j], (uint64_t)A[j] + c);
    const uint32_t w = (uint32_t)s;
    c = (uint32_t)(s >> 32);
    if (j) A[j - 1] = (prev >> k) | (w << (32 - k));
    prev = w;
  }
  A[L - 1] = (prev >> k) | (c << (32 - k));
}

// x >= y
template <int L>
__device__ __forceinline__ bool lds_geq(const LdsNum<L>& x, const LdsNum<L>& y) {
  for (int j = L - 1; j >= 0; --j) {
    const uint32_t a = x[j], b = y[j];
    if (a != b) return a > b;
  }
  return true;
}

// x -= y (x >= y)
template <int L>
__device__ __forceinline__ void lds_sub(const LdsNum<L>& x, const LdsNum<L>& y) {
  uint32_t br = 0;
  for (int j = 0; j < L; ++j) {
    const uint64_t d = (uint64_t)x[j] - y[j] - br;
    x[j] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
}

// x = x - y mod M (x, y < M)
template <int L>
__device__ __forceinline__ void lds_modsub(const LdsNum<L>& x, const LdsNum<L>& y, const uint32_t* __restrict__ M) {
  uint32_t br = 0;
  for (int j = 0; j < L; ++j) {
    const uint64_t d = (uint64_t)x[j] - y[j] - br;
    x[j] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  if (br) {
    uint32_t c = 0;
    for (int j = 0; j < L; ++j) {
      const uint64_t s = (uint64_t)x[j] + M[j] + c;
      x[j] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
  }
}

// 33 bits of x starting at bit `pos` (pos >= 0; bits past the top limb read as 0)
template <int L>
__device__ __forceinline__ uint64_t lds_bits33(const LdsNum<L>& x, int pos) {
  const int w = pos >> 5, off = pos & 31;
  const uint64_t lo = x[w];
  const uint64_t mid = w + 1 < L ? x[w + 1] : 0u;
  const uint64_t hi = w + 2 < L ? x[w + 2] : 0u;
  const uint64_t v = (lo >> off) | (mid << (32 - off)) | (off ? hi << (64 - off) : 0ull);
  return v & ((1ull << 33) - 1);
}

// one signed limb of sum(p_i) + c, p_i = int64 products: low 32 bits out, signed carry kept
__device__ __forceinline__ uint32_t signed_limb(int64_t p0, int64_t p1, int64_t& c) {
  const uint64_t lo = (uint64_t)(uint32_t)p0 + (uint32_t)p1 + (uint32_t)c;
  c = (p0 >> 32) + (p1 >> 32) + (c >> 32) + (int64_t)(lo >> 32);
  return (uint32_t)lo;
}

__device__ __forceinline__ uint32_t signed_limb3(int64_t p0, int64_t p1, int64_t p2, int64_t& c) {
  const uint64_t lo = (uint64_t)(uint32_t)p0 + (uint32_t)p1 + (uint32_t)p2 + (uint32_t)c;
  c = (p0 >> 32) + (p1 >> 32) + (p2 >> 32) + (c >> 32) + (int64_t)(lo >> 32);
  return (uint32_t)lo;
}

// x <- -x over limbs [0, n) (two's complement)
template <int L>
__device__ __forceinline__ void lds_neg(const LdsNum<L>& x, int n) {
  uint32_t br = 0;
  for (int j = 0; j < n; ++j) {
    const uint64_t d = 0ull - x[j] - br;
    x[j] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
}

// PaillierInvert (paillier.cc:267-273 mpz_invert): x^-1 mod n^2, Pornin's binary GCD with 31-step
// batches ("Optimized Binary GCD for Modular Inversion", 2020, Algorithm 2). Each outer pass runs
// 31 binary-GCD steps on 64-bit approximations of a and b (low 31 bits and top 33 bits, exact once
// both fit 64 bits), collecting the update factors f0, g0, f1, g1 (|.| <= 2^31), then applies them
// to the full numbers: (a, b) <- ((f0 a + g0 b) / 2^31, (f1 a + g1 b) / 2^31) with sign fixes, and
// (u, v) <- the same combinations times 2^-31 mod M (one Montgomery-style step), keeping
// a = u x, b = v x (mod M). About 2 len(M) / 31 passes of a few limb sweeps each, instead of one
// sweep per bit; the 31 inner steps are branch-free, so a wave does not diverge in them.
//
// REG (n^2 of up to 2048 bits): u and v, which every pass sweeps in full, live in registers with
// the sweeps unrolled; a and b (swept only up to their shrinking top limb) stay in LDS. That halves
// the LDS per lane and takes four LDS accesses off every limb step of the u, v update: 32,768
// inverses 1.96 -> 1.66 ms at 1024-bit n, 0.63 -> 0.54 ms at 512-bit; the LDS sweeps of larger keys
// unrolled by 4, 13.0 -> 12.4 ms at 2048-bit (tools/bench_invert.py, profiles/r02/invert_ab.jsonl).
//
// sel_kind selects the elements to invert (the others are copied, or left alone when out == x; x
// is read in full before out is written, so the op runs in place): 0 every element, 1 where the
// int8 flag sel[i] != 0 (a parsed hex scalar's sign), 2 where the int64 sel[i] < 0 (MulScalar's y).
template <int LN, bool REG>
__global__ __launch_bounds__(kPlBlock) void k_invert(Key k, const uint32_t* x, uint32_t* out, long long N,
                                                     unsigned long long* bad, const void* sel, int sel_kind) {
  constexpr int LC = 2 * LN;
  constexpr int UR = REG ? LC : 4;    // unroll of the u, v sweeps (full in registers)
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (sel_kind) {
    const bool inv = sel_kind == 1 ? ((const signed char*)sel)[i] != 0 : ((const long long*)sel)[i] < 0;
    if (!inv) {
      if (out != x)
        for (int j = 0; j < LC; j += 4)
          *reinterpret_cast<uint4*>(out + i * LC + j) = *reinterpret_cast<const uint4*>(x + i * LC + j);
      return;
    }
  }
  const uint32_t* M = k.at(k.d.off_n2);
  const uint32_t minv = k.d.n2_minv;   // -M^-1 mod 2^32
  LdsNum<LC> A{lds + threadIdx.x, S}, B{lds + LC * S + threadIdx.x, S};
  using UV = typename std::conditional<REG, RegNum<LC>, LdsNum<LC>>::type;
  UV U, V;
  if constexpr (!REG) {
    U = LdsNum<LC>{lds + 2 * LC * S + threadIdx.x, S};
    V = LdsNum<LC>{lds + 3 * LC * S + threadIdx.x, S};
  }
  const uint32_t* xi = x + i * LC;
  uint32_t any = 0;
  for (int j = 0; j < LC; ++j) {
    A[j] = xi[j];
    any |= xi[j];
    B[j] = M[j];
  }
#pragma unroll UR
  for (int j = 0; j < LC; ++j) {
    U[j] = j == 0 ? 1u : 0u;
    V[j] = 0u;
  }
  // total binary-GCD steps <= 2 len(M) - 1 (Pornin, Theorem 1); a few passes of slack
  const int max_pass = (2 * 32 * LC - 1 + 30) / 31 + 4;
  int top = LC - 1;
  bool a_zero = any == 0;
  for (int pass = 0; pass < max_pass && !a_zero; ++pass) {
    while (top > 0 && (A[top] | B[top]) == 0u) --top;
    const uint32_t th = A[top] | B[top];
    int nb = 32 * top + 32 - __clz(th);
    nb = nb < 64 ? 64 : nb;
    uint64_t ab = (A[0] & 0x7FFFFFFFu) | (lds_bits33<LC>(A, nb - 33) << 31);
    uint64_t bb = (B[0] & 0x7FFFFFFFu) | (lds_bits33<LC>(B, nb - 33) << 31);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
    for (int s = 0; s < 31; ++s) {
      const bool odd = ab & 1ull;
      const bool sw = odd && ab < bb;
      const uint64_t ta = sw ? bb : ab, tb = sw ? ab : bb;
      const int64_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      ab = (odd ? ta - tb : ta) >> 1;
      bb = tb;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      f1 = tf1 << 1;
      g1 = tg1 << 1;
    }
    // (a, b) <- ((f0 a + g0 b) >> 31, (f1 a + g1 b) >> 31) over limbs [0, top]; values do not grow
    {
      int64_t ca = 0, cb = 0;
      uint32_t pa = 0, pb = 0, nz = 0;
      for (int j = 0; j <= top; ++j) {
        const int64_t aj = A[j], bj = B[j];
        const uint32_t da = signed_limb(aj * f0, bj * g0, ca);
        const uint32_t db = signed_limb(aj * f1, bj * g1, cb);
        if (j) {
          A[j - 1] = (pa >> 31) | (da << 1);
          B[j - 1] = (pb >> 31) | (db << 1);
          nz |= A[j - 1];
        }
        pa = da;
        pb = db;
      }
      A[top] = (pa >> 31) | ((uint32_t)ca << 1);
      B[top] = (pb >> 31) | ((uint32_t)cb << 1);
      nz |= A[top];
      if (ca < 0) {
        lds_neg<LC>(A, top + 1);
        f0 = -f0;
        g0 = -g0;
      }
      if (cb < 0) {
        lds_neg<LC>(B, top + 1);
        f1 = -f1;
        g1 = -g1;
      }
      a_zero = nz == 0u;
    }
    // (u, v) <- ((f0 u + g0 v) 2^-31, (f1 u + g1 v) 2^-31) mod M: add t M with the low 31 bits of
    // the sum zeroed, shift, then bring the result (|r| < 3M) into [0, M)
    {
      const uint32_t s0u = U[0] * (uint32_t)f0 + V[0] * (uint32_t)g0;
      const uint32_t s0v = U[0] * (uint32_t)f1 + V[0] * (uint32_t)g1;
      const int64_t tu = (int64_t)((s0u * minv) & 0x7FFFFFFFu), tv = (int64_t)((s0v * minv) & 0x7FFFFFFFu);
      int64_t cu = 0, cv = 0;
      uint32_t pu = 0, pv = 0;
#pragma unroll UR
      for (int j = 0; j < LC; ++j) {
        const int64_t uj = U[j], vj = V[j], mj = M[j];
        const uint32_t ru = signed_limb3(uj * f0, vj * g0, tu * mj, cu);
        const uint32_t rv = signed_limb3(uj * f1, vj * g1, tv * mj, cv);
        if (j) {
          U[j - 1] = (pu >> 31) | (ru << 1);
          V[j - 1] = (pv >> 31) | (rv << 1);
        }
        pu = ru;
        pv = rv;
      }
      U[LC - 1] = (pu >> 31) | ((uint32_t)cu << 1);
      V[LC - 1] = (pv >> 31) | ((uint32_t)cv << 1);
      int64_t eu = cu >> 31, ev = cv >> 31;   // limb LC of the shifted results (small, signed)
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        UV& R = which ? V : U;
        int64_t& ext = which ? ev : eu;
        while (ext < 0) {   // R += M
          uint32_t c = 0;
#pragma unroll UR
          for (int j = 0; j < LC; ++j) {
            const uint64_t t = (uint64_t)R[j] + M[j] + c;
            R[j] = (uint32_t)t;
            c = (uint32_t)(t >> 32);
          }
          ext += c;
        }
        for (;;) {          // R >= M (or ext > 0): R -= M
          bool ge = ext > 0;
          if (!ge) {
            // R >= M, from the top limb down: branch-free over all limbs in registers (so the
            // loop stays unrolled), an early exit over LDS (the first differing limb decides)
            if constexpr (REG) {
              int cmp = 0;
#pragma unroll
              for (int j = LC - 1; j >= 0; --j) {
                const uint32_t r = R[j], m = M[j];
                cmp = cmp ? cmp : (r > m) - (r < m);
              }
              ge = cmp >= 0;
            } else {
              ge = true;
              for (int j = LC - 1; j >= 0; --j) {
                const uint32_t r = R[j], m = M[j];
                if (r != m) {
                  ge = r > m;
                  break;
                }
              }
            }
          }
          if (!ge) break;
          uint32_t br = 0;
#pragma unroll UR
          for (int j = 0; j < LC; ++j) {
            const uint64_t d = (uint64_t)R[j] - M[j] - br;
            R[j] = (uint32_t)d;
            br = (uint32_t)(d >> 63);
          }
          ext -= br;
        }
      }
    }
  }
  // gcd in b: invertible iff a reached 0 with b == 1
  bool ok = a_zero && B[0] == 1u;
  for (int j = 1; j < LC && ok; ++j) ok = B[j] == 0u;
  uint32_t* o = out + i * LC;
#pragma unroll UR
  for (int j = 0; j < LC; ++j) o[j] = ok ? V[j] : 0u;
  if (!ok) atomicMin(bad, (unsigned long long)i);
}

// PaillierMatmul core (paillier.cc:941-1051): one lane per output (i, k). Terms with y >= 0 are
// multiplied into `pos`, terms with y < 0 (the reference's (x^-1)^|y|) into `neg`; the caller
// finishes z = pos * neg^-1, the same group element the reference's ordered product gives.
// Each term is (x^|y|)^(2^(xe + ye - min)).
template <int LN>
__global__ __launch_bounds__(kPlBlock) void k_matmul(Key k, const uint32_t* __restrict__ X,
                                                     const long long* __restrict__ xe,
                                                     const long long* __restrict__ ym,
                                                     const long long* __restrict__ ye,
                                                     uint32_t* __restrict__ zpos, uint32_t* __restrict__ zneg,
                                                     long long* __restrict__ ze, int u, int v, int w) {
  constexpr int LC = 2 * LN;
  extern __shared__ uint32_t lds[];
  const int S = blockDim.x;
  uint32_t* acol = lds + threadIdx.x;
  uint32_t* bcol = lds + LC * S + threadIdx.x;
  uint32_t* pcol = lds + 2 * LC * S + threadIdx.x;   // running positive product (Montgomery)
  const long long lin = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (lin >= (long long)u * w) return;
  // column by column: the lanes of a wave share every term's |y| (no divergence in x^|y|)
  const int i = (int)(lin % u), kk = (int)(lin / u);
  const long long o = (long long)i * w + kk;
  const uint32_t* n2 = k.at(k.d.off_n2);
  const uint32_t* one = k.at(k.d.off_n2_one);
  long long mn = 0x7FFFFFFFFFFFFFFFll;
  for (int j = 0; j < v; ++j) {
    const long long e = xe[(long long)i * v + j] + ye[(long long)j * w + kk];
    mn = e < mn ? e : mn;
  }
  uint32_t t[LC], neg[LC];
  load_uniform<LC>(t, one);
  to_lds<LC>(pcol, S, t);
  load_uniform<LC>(neg, one);
  for (int j = 0; j < v; ++j) {
    const long long y = ym[(long long)j * w + kk];
    if (y == 0) continue;                                     // x^0 = 1
    const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
    const long long delta = xe[(long long)i * v + j] + ye[(long long)j * w + kk] - mn;
    // base = x_ij * R
    load_g<LC>(t, X + ((long long)i * v + j) * LC);
    mont_mul<LC>(t, Uniform{k.at(k.d.off_n2_r2)}, n2, k.d.n2_minv);
    to_lds<LC>(bcol, S, t);
    const int bits = 64 - __clzll((long long)ay);
    for (int b = bits - 2; b >= 0; --b) {
      mont_sqr<LC>(t, acol, S, n2, k.d.n2_minv);
      if ((ay >> b) & 1ull) mont_mul<LC>(t, LdsCol{bcol, S}, n2, k.d.n2_minv);
    }
    for (long long d = 0; d < delta; ++d) mont_sqr<LC>(t, acol, S, n2, k.d.n2_minv);
    if (y > 0) {
      mont_mul<LC>(t, LdsCol{pcol, S}, n2, k.d.n2_minv);
      to_lds<LC>(pcol, S, t);
    } else {
      to_lds<LC>(bcol, S, neg);
      mont_mul<LC>(t, LdsCol{bcol, S}, n2, k.d.n2_minv);
      copy<LC>(neg, t);
    }
  }
  // back to normal form
  for (int j = 0; j < LC; ++j) t[j] = pcol[j * S];
  redc<LC>(t, n2, k.d.n2_minv);
  store_g<LC>(zpos + o * LC, t);
  redc<LC>(neg, n2, k.d.n2_minv);
  store_g<LC>(zneg + o * LC, neg);
  ze[o] = mn;
}

// ------------------------------------------------------------------------------------------
// limbs <-> hex text (mpz_get_str(..., 16) / mpz_set_str(..., 16))
// ------------------------------------------------------------------------------------------

// number of characters of each element's hex text ('-' included), "0" for zero
__global__ __launch_bounds__(256) void k_hex_len(const uint32_t* __restrict__ limbs, int L,
                                                 const signed char* __restrict__ neg,
                                                 long long* __restrict__ lens, long long N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t* x = limbs + i * L;
  int digits = 1;
  for (int w = L - 1; w >= 0; --w)
    if (x[w]) { digits = w * 8 + (32 - __clz(x[w]) + 3) / 4; break; }
  const bool zero = digits == 1 && x[0] == 0;
  lens[i] = digits + ((neg && neg[i] && !zero) ? 1 : 0);
}

// One wave per element for the text itself: a ciphertext's text is hundreds to thousands of
// characters (512 at 1024-bit n), so one lane per element made every byte access a 64-way
// scatter (lanes one text apart). Here the 64 lanes of a wave walk ONE text together, lane c on
// characters c, c + 64, ...: every byte load / store instruction covers 64 consecutive bytes, and
// the limb words the lanes need are 8 consecutive words (broadcast within groups of 8 lanes).
constexpr int kHexWaves = 4;   // waves (elements) per 256-lane workgroup

__device__ __forceinline__ char hex_char(uint32_t v) { return (char)(v < 10 ? '0' + v : 'a' + v - 10); }

// value of a hex digit, or 16 for anything else
__device__ __forceinline__ uint32_t hex_val(char c) {
  if (c >= '0' && c <= '9') return (uint32_t)(c - '0');
  if (c >= 'a' && c <= 'f') return (uint32_t)(c - 'a' + 10);
  if (c >= 'A' && c <= 'F') return (uint32_t)(c - 'A' + 10);
  return 16u;
}

__global__ __launch_bounds__(256) void k_hex_write(const uint32_t* __restrict__ limbs, int L,
                                                   const signed char* __restrict__ neg,
                                                   const long long* __restrict__ offs,
                                                   char* __restrict__ chars, long long N) {
  const long long i = (long long)blockIdx.x * kHexWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  const uint32_t* x = limbs + i * L;
  const long long o0 = offs[i], len = offs[i + 1] - o0;
  const bool sign = len > 1 && neg && neg[i];
  if (sign && lane == 0) chars[o0] = '-';
  char* o = chars + o0 + (sign ? 1 : 0);
  const long long digits = len - (sign ? 1 : 0);
  for (long long c = lane; c < digits; c += 64) {
    const long long d = digits - 1 - c;   // digit index from the least significant
    o[c] = hex_char((x[d >> 3] >> ((d & 7) * 4)) & 15u);
  }
}

// parse [-]hexdigits into L limbs; bad <- smallest index of a malformed / too-wide string.
// Lane w assembles limbs w, w + 64, ... from their 8 digits; digits past 8 L must be '0'.
__global__ __launch_bounds__(256) void k_hex_parse(const char* __restrict__ chars,
                                                   const long long* __restrict__ offs, int L,
                                                   uint32_t* __restrict__ limbs,
                                                   signed char* __restrict__ neg, long long N,
                                                   unsigned long long* bad) {
  const long long i = (long long)blockIdx.x * kHexWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  long long s = offs[i];
  const long long e = offs[i + 1];
  bool ok = e > s;
  const bool ng = ok && chars[s] == '-';
  if (ng) {
    ++s;
    ok = e > s;
  }
  const long long nd = ok ? e - s : 0;
  uint32_t* x = limbs + i * L;
  for (int w = lane; w < L; w += 64) {
    uint32_t acc = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const long long d = 8ll * w + t;
      if (d < nd) {
        const uint32_t v = hex_val(chars[e - 1 - d]);
        ok = ok && v < 16u;
        acc |= (v & 15u) << (4 * t);
      }
    }
    x[w] = acc;
  }
  for (long long d = 8ll * L + lane; d < nd; d += 64) ok = ok && chars[e - 1 - d] == '0';
  if (neg && lane == 0) neg[i] = ng ? 1 : 0;
  // one report per element: any lane that saw a bad character
  if (__any(!ok) && lane == 0) atomicMin(bad, (unsigned long long)i);
}

// decrypt -> int64 (mpz_get_sll semantics, gmp_utils.cc:38-45: low 64 bits of |m|, then sign)
__global__ __launch_bounds__(256) void k_to_int64(const uint32_t* __restrict__ mag, int L,
                                                  const signed char* __restrict__ neg,
                                                  long long* __restrict__ out, long long N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint64_t v = (uint64_t)mag[i * L] | ((uint64_t)mag[i * L + 1] << 32);
  out[i] = neg[i] ? (long long)(0ull - v) : (long long)v;
}

// ------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------

inline bool key_ok(const void* kb, const efl_pl_key* d, bool need_private, int ln_max) {
  if (!d) { set_error("null key descriptor"); return false; }
  if (!kb) { set_error("null key block"); return false; }   // e.g. a context whose table build failed
  if (d->a_bits <= 0 || d->a_bits > 8192) { set_error("a_bits must be in [1, 8192]"); return false; }
  if (d->ln != 16 && d->ln != 32 && d->ln != 64 && d->ln != 128 && d->ln != 256) {
    set_error("unsupported limb count %d (n of 512/1024/2048/4096/8192 bits)", d->ln);
    return false;
  }
  if (d->ln > ln_max) {
    set_error("n of %d bits is not supported by this operation on the GPU yet (max %d)", d->ln * 32, ln_max * 32);
    return false;
  }
  if (need_private && !d->has_private) { set_error("No private key."); return false; }
  return true;
}

// the fixed-base table covers a: W-bit windows (1..24), 2^W - 1 columns, ceil(a_bits / W) rows;
// group_size (the API's, used to form a') in 1..32
inline int table_ok(const efl_pl_key* d) {
  const int W = d->table_window > 0 ? d->table_window : d->group_size;
  if (d->table_rows <= 0 || d->group_size <= 0) {
    set_error("no fixed-base table: set the public key first");
    return EFL_E_ABORTED;
  }
  if (W < 1 || W > 24 || d->group_size > 32 || d->table_cols != (1 << W) - 1 ||
      (int64_t)d->table_rows * W < d->a_bits) {
    set_error("fixed-base table %d x %d (window %d) does not cover %d-bit exponents", d->table_rows,
              d->table_cols, W, d->a_bits);
    return EFL_E_INVALID_ARGUMENT;
  }
  return EFL_OK;
}

// kernel family per key size: 0 = one lane per element (paillier.hip), C = sliced over 2ln/C (n^2
// ops) or ln/C (decryption) lanes of C limbs (paillier_sliced.hip). [ln 16/32/64/128/256][n^2 ops, decrypt]
// measured: decryption profiles/r01/bench_pl*.jsonl; n^2 ops profiles/r02/sweep_pl_family.jsonl — with
// the round-2 table window, 32 limbs per lane is the fastest encryption at every key size (512-bit
// 1.7x, 1024-bit 1.06x incl. the MNIST matmul, 2048-bit 1.14x, 4096-bit 1.51x the round-1 choice)
// 8192-bit n (round 4): n^2 ops over 16 lanes of 32 limbs, decryption over 8 (the 4096-bit key's
// n^2 family), both without a one-lane alternative
constexpr int kDefaultSlicing[5][2] = {{32, 8}, {32, 32}, {32, 32}, {32, 32}, {32, 32}};
int g_slicing[5][2] = {{32, 8}, {32, 32}, {32, 32}, {32, 32}, {32, 32}};
inline int ln_index(int ln) { return ln == 16 ? 0 : ln == 32 ? 1 : ln == 64 ? 2 : ln == 128 ? 3 : 4; }
inline int slicing(int ln, int dec) { return g_slicing[ln_index(ln)][dec]; }
bool g_slicing_set[5][2] = {};   // set explicitly through efl_pl_tune: used as given for every size

// Decryption family for n elements: the default (C = 32) unless the launch would give fewer than
// 768 waves (3 per 4 SIMDs) of that family; then C = 8 (four times the lanes per element). Round 3
// sweep (tools/sweep_dec_family.py, profiles/r03/dec_family.jsonl): 2048-bit 16,384: 31.7 (C = 8)
// against 37.2 (32); 4096-bit 4,096: 90 against 143. C = 16 is never the fastest (at 2048 / 4096 bits
// it spills into its window loop and runs 3-5x slower), so the sizing skips it; round 1's rule
// halved C step by step. The 1024-bit key's C = 32 family holds a number in ONE lane and squares by
// product scanning (sliced28.h sqr_fips1, 1.3-1.4x faster than its CIOS squaring), which moves its
// crossover down to 384 waves: 32,768 elements 6.5 ms (C = 32) against 7.8 (C = 8), 16,384 6.4
// against 5.9 (profiles/r03/dec_family_fips.jsonl).
inline int decrypt_family(int ln, long long n) {
  const int C = slicing(ln, 1);
  if (!C || g_slicing_set[ln_index(ln)][1]) return C;
  const long long few_waves = (ln == 32 ? 384ll : 768ll) * 64;   // lanes
  if (C == 32 && n * (ln / 32) < few_waves && pl::sliced_available(ln, 8)) return 8;
  return C;
}

inline unsigned grid_of(long long N) { return (unsigned)((N + kPlBlock - 1) / kPlBlock); }

template <template <int> class F, class... A>
hipError_t dispatch_ln(int ln, A... args) {
  switch (ln) {
    case 16: return F<16>::run(args...);
    case 32: return F<32>::run(args...);
    case 64: return F<64>::run(args...);
    default: return hipErrorInvalidValue;
  }
}

template <int LN>
struct RunEncrypt {
  static hipError_t run(Key k, const long long* m, const uint32_t* hsa, uint32_t* out, long long N,
                        uint64_t seed, long long ctr0, hipStream_t s, int hsa_mont = 0) {
    const int aw = (k.d.a_bits + 31) / 32;
    const size_t lds = (size_t)((aw > 2 * LN ? aw : 2 * LN) + 2 * LN) * kPlBlock * 4;
    hipLaunchKernelGGL((k_encrypt<LN>), dim3(grid_of(N)), dim3(kPlBlock), lds, s, k, m, hsa, out, N, seed, ctr0,
                       hsa_mont);
    return hipGetLastError();
  }
};
template <int LN>
struct RunFbpowm {
  static hipError_t run(Key k, const uint32_t* a, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                        hipStream_t s) {
    const int aw = (k.d.a_bits + 31) / 32;
    const size_t lds = (size_t)((aw > 2 * LN ? aw : 2 * LN) + 2 * LN) * kPlBlock * 4;
    hipLaunchKernelGGL((k_fbpowm<LN>), dim3(grid_of(N)), dim3(kPlBlock), lds, s, k, a, out, N, seed, ctr0);
    return hipGetLastError();
  }
};
template <int LN>
struct RunAdd {
  static hipError_t run(Key k, const uint32_t* x, const uint32_t* y, uint32_t* out, long long N, hipStream_t s) {
    const size_t lds = (size_t)(2 * LN) * kPlBlock * 4;
    hipLaunchKernelGGL((k_add<LN>), dim3(grid_of(N)), dim3(kPlBlock), lds, s, k, x, y, out, N);
    return hipGetLastError();
  }
};
template <int LN>
struct RunPowm {
  template <class XS>
  static hipError_t run(Key k, const uint32_t* x, XS xs, uint32_t* out, long long N, unsigned long long* bad,
                        hipStream_t s) {
    const size_t lds = (size_t)2 * (2 * LN) * kPlBlock * 4;
    hipLaunchKernelGGL((k_powm<LN, XS>), dim3(grid_of(N)), dim3(kPlBlock), lds, s, k, x, xs, out, N, bad);
    return hipGetLastError();
  }
};

template <int LN>
hipError_t run_invert(Key k, const uint32_t* x, uint32_t* out, long long N, unsigned long long* bad, hipStream_t s,
                      const void* sel = nullptr, int sel_kind = 0) {
  // four LDS numbers per lane: 32 lanes per workgroup for n^2 of 8192 bits (128 KiB), 16 for n^2
  // of 16384 bits (128 KiB)
  constexpr int block = LN >= 256 ? 16 : LN >= 128 ? 32 : kPlBlock;
  constexpr bool reg = 2 * LN <= 64;   // u, v in registers (k_invert)
  const size_t lds = (size_t)(reg ? 2 : 4) * (2 * LN) * block * 4;
  hipLaunchKernelGGL((k_invert<LN, reg>), dim3((unsigned)((N + block - 1) / block)), dim3(block), lds, s, k, x, out,
                     N, bad, sel, sel_kind);
  return hipGetLastError();
}

hipError_t invert_ln(Key k, const uint32_t* x, uint32_t* out, long long N, unsigned long long* bad, hipStream_t s,
                     const void* sel, int sel_kind) {
  switch (k.d.ln) {
    case 16: return run_invert<16>(k, x, out, N, bad, s, sel, sel_kind);
    case 32: return run_invert<32>(k, x, out, N, bad, s, sel, sel_kind);
    case 64: return run_invert<64>(k, x, out, N, bad, s, sel, sel_kind);
    case 128: return run_invert<128>(k, x, out, N, bad, s, sel, sel_kind);
    default: return run_invert<256>(k, x, out, N, bad, s, sel, sel_kind);
  }
}

// z = x^e mod n^2 with the exponent source xs, in the family chosen for n^2 ops
template <class XS>
hipError_t powm_family(Key k, const uint32_t* x, XS xs, uint32_t* z, long long n, unsigned long long* bad,
                       hipStream_t s);
template <int LN>
struct RunMatmul {
  static hipError_t run(Key k, const uint32_t* X, const long long* xe, const long long* ym, const long long* ye,
                        uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w, hipStream_t s) {
    const size_t lds = (size_t)3 * (2 * LN) * kPlBlock * 4;
    hipLaunchKernelGGL((k_matmul<LN>), dim3(grid_of((long long)u * w)), dim3(kPlBlock), lds, s, k, X, xe, ym, ye,
                       zpos, zneg, ze, u, v, w);
    return hipGetLastError();
  }
};

template <int LP>
hipError_t run_decrypt(Key k, const uint32_t* ct, uint32_t* mag, signed char* neg, long long N, hipStream_t s) {
  const size_t lds = (size_t)2 * LP * kPlBlock * 4;
  hipLaunchKernelGGL((k_decrypt<LP>), dim3(grid_of(N)), dim3(kPlBlock), lds, s, k, ct, mag, neg, N);
  return hipGetLastError();
}

}  // namespace
}  // namespace efl

using namespace efl;

EFL_API int efl_pl_encrypt(const void* key_block, const efl_pl_key* key, const int64_t* plaintext,
                           const uint32_t* hsa, uint32_t* ciphertext, int64_t n, uint64_t seed,
                           int64_t counter_base, void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (n < 0) { set_error("negative count"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  if (!hsa) {
    const int rc = table_ok(key);
    if (rc != EFL_OK) return rc;
  }
  Key k{(const uint32_t*)key_block, *key};
  const int C = slicing(key->ln, 0);
  return hip_status(C ? pl::sl_encrypt(k, C, (const long long*)plaintext, hsa, ciphertext, (long long)n, seed,
                                       (long long)counter_base, (hipStream_t)stream)
                      : dispatch_ln<RunEncrypt>(key->ln, k, (const long long*)plaintext, hsa, ciphertext,
                                                (long long)n, seed, (long long)counter_base, (hipStream_t)stream),
                    "efl_pl_encrypt");
}

EFL_API int efl_pl_fbpowm(const void* key_block, const efl_pl_key* key, const uint32_t* a, uint32_t* hsa,
                          int64_t n, uint64_t seed, int64_t counter_base, void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  const int rc = table_ok(key);
  if (rc != EFL_OK) return rc;
  Key k{(const uint32_t*)key_block, *key};
  const int C = slicing(key->ln, 0);
  return hip_status(C ? pl::sl_fbpowm(k, C, a, hsa, (long long)n, seed, (long long)counter_base, (hipStream_t)stream)
                      : dispatch_ln<RunFbpowm>(key->ln, k, a, hsa, (long long)n, seed, (long long)counter_base,
                                               (hipStream_t)stream),
                    "efl_pl_fbpowm");
}

EFL_API int efl_pl_crt_join(const void* key_block, const efl_pl_key* key, const uint32_t* xp, const uint32_t* xq,
                            const int64_t* plaintext, uint32_t* z, int64_t n, void* stream) {
  if (!key_ok(key_block, key, true, 256)) return key && !key->has_private ? EFL_E_ABORTED : EFL_E_INVALID_ARGUMENT;
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  Key k{(const uint32_t*)key_block, *key};
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = grid_of((long long)n);
  const size_t lds = (size_t)(2 * key->ln + 1) * kPlBlock * 4;
  switch (key->ln) {
    case 16: hipLaunchKernelGGL((k_crt_join<16>), dim3(g), dim3(kPlBlock), lds, s, k, xp, xq, z, (long long)n); break;
    case 32: hipLaunchKernelGGL((k_crt_join<32>), dim3(g), dim3(kPlBlock), lds, s, k, xp, xq, z, (long long)n); break;
    case 64: hipLaunchKernelGGL((k_crt_join<64>), dim3(g), dim3(kPlBlock), lds, s, k, xp, xq, z, (long long)n); break;
    case 128: hipLaunchKernelGGL((k_crt_join<128>), dim3(g), dim3(kPlBlock), lds, s, k, xp, xq, z, (long long)n); break;
    default: hipLaunchKernelGGL((k_crt_join<256>), dim3(g), dim3(kPlBlock), lds, s, k, xp, xq, z, (long long)n); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !plaintext) return hip_status(e, "efl_pl_crt_join");
  // encryption: z holds hsa R mod n^2; g(m) hsa = mont(g, hsa R), one product, in place (each lane
  // reads its element's words of z before it writes them)
  const int C = slicing(key->ln, 0);
  const long long* m = (const long long*)plaintext;
  e = C ? pl::sl_encrypt(k, C, m, z, z, (long long)n, 0, 0, s, 1)
        : dispatch_ln<RunEncrypt>(key->ln, k, m, (const uint32_t*)z, z, (long long)n, (uint64_t)0, 0ll, s, 1);
  return hip_status(e, "efl_pl_crt_join");
}

EFL_API int efl_pl_decrypt(const void* key_block, const efl_pl_key* key, const uint32_t* ciphertext,
                           uint32_t* magnitude, int8_t* negative, int64_t n, void* stream) {
  if (!key_ok(key_block, key, true, 256)) return key && !key->has_private ? EFL_E_ABORTED : EFL_E_INVALID_ARGUMENT;
  if (n < 0) { set_error("negative count"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  Key k{(const uint32_t*)key_block, *key};
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  const int C = decrypt_family(key->ln, n);
  if (C) return hip_status(pl::sl_decrypt(k, C, ciphertext, magnitude, (signed char*)negative, n, s), "efl_pl_decrypt");
  switch (key->ln) {
    case 16: e = run_decrypt<16>(k, ciphertext, magnitude, (signed char*)negative, n, s); break;
    case 32: e = run_decrypt<32>(k, ciphertext, magnitude, (signed char*)negative, n, s); break;
    case 64: e = run_decrypt<64>(k, ciphertext, magnitude, (signed char*)negative, n, s); break;
    case 128: e = run_decrypt<128>(k, ciphertext, magnitude, (signed char*)negative, n, s); break;
    default: set_error("no one-lane decryption for p^2 of %d bits", 32 * key->ln); return EFL_E_INVALID_ARGUMENT;
  }
  return hip_status(e, "efl_pl_decrypt");
}

EFL_API int efl_pl_add(const void* key_block, const efl_pl_key* key, const uint32_t* x, const uint32_t* y,
                       uint32_t* z, int64_t n, void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  Key k{(const uint32_t*)key_block, *key};
  const int C = slicing(key->ln, 0);
  return hip_status(C ? pl::sl_add(k, C, x, y, z, (long long)n, (hipStream_t)stream)
                      : dispatch_ln<RunAdd>(key->ln, k, x, y, z, (long long)n, (hipStream_t)stream),
                    "efl_pl_add");
}

EFL_API int efl_pl_powm(const void* key_block, const efl_pl_key* key, const uint32_t* x, const uint32_t* exps,
                        int exp_words, uint32_t* z, int64_t n, void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (exp_words <= 0) { set_error("exp_words must be positive"); return EFL_E_INVALID_ARGUMENT; }
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  Key k{(const uint32_t*)key_block, *key};
  const int C = slicing(key->ln, 0);
  return hip_status(C ? pl::sl_powm(k, C, x, exps, exp_words, z, (long long)n, (hipStream_t)stream)
                      : dispatch_ln<RunPowm>(key->ln, k, x, pl::ExpWords{exps, exp_words}, z, (long long)n,
                                             (unsigned long long*)nullptr, (hipStream_t)stream),
                    "efl_pl_powm");
}

namespace efl {
namespace {
template <>
hipError_t powm_family<pl::ExpAbs64>(Key k, const uint32_t* x, pl::ExpAbs64 xs, uint32_t* z, long long n,
                                     unsigned long long* bad, hipStream_t s) {
  const int C = slicing(k.d.ln, 0);
  return C ? pl::sl_powm_abs64(k, C, x, xs.y, z, n, bad, s) : dispatch_ln<RunPowm>(k.d.ln, k, x, xs, z, n, bad, s);
}
template <>
hipError_t powm_family<pl::ExpPow2>(Key k, const uint32_t* x, pl::ExpPow2 xs, uint32_t* z, long long n,
                                    unsigned long long* bad, hipStream_t s) {
  const int C = slicing(k.d.ln, 0);
  return C ? pl::sl_powm_pow2(k, C, x, xs.y, z, n, bad, s) : dispatch_ln<RunPowm>(k.d.ln, k, x, xs, z, n, bad, s);
}
template <>
hipError_t powm_family<pl::ExpShift>(Key k, const uint32_t* x, pl::ExpShift xs, uint32_t* z, long long n,
                                     unsigned long long* bad, hipStream_t s) {
  const int C = slicing(k.d.ln, 0);
  return C ? pl::sl_powm_shift(k, C, x, xs.own, xs.other, z, n, bad, s)
           : dispatch_ln<RunPowm>(k.d.ln, k, x, xs, z, n, bad, s);
}
template <>
hipError_t powm_family<pl::ExpWords>(Key k, const uint32_t* x, pl::ExpWords xs, uint32_t* z, long long n,
                                     unsigned long long* bad, hipStream_t s) {
  const int C = slicing(k.d.ln, 0);
  return C ? pl::sl_powm(k, C, x, xs.e, xs.ew, z, n, s) : dispatch_ln<RunPowm>(k.d.ln, k, x, xs, z, n, bad, s);
}

// common prologue of the ops with a device status word: argument checks, bad <- -1
int status_prologue(const void* key_block, const efl_pl_key* key, int64_t n, int64_t* bad, hipStream_t s, const char* op) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (!bad) { set_error("%s: null status word", op); return EFL_E_INVALID_ARGUMENT; }
  if (n < 0) { set_error("%s: negative count", op); return EFL_E_INVALID_ARGUMENT; }
  return hip_status(hipMemsetAsync(bad, 0xFF, sizeof(int64_t), s), op);
}
}  // namespace
}  // namespace efl

EFL_API int efl_pl_mul_exp2(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* y,
                            uint32_t* z, int64_t n, int64_t* bad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int rc = status_prologue(key_block, key, n, bad, s, "efl_pl_mul_exp2");
  if (rc != EFL_OK || n == 0) return rc;
  Key k{(const uint32_t*)key_block, *key};
  return hip_status(powm_family(k, x, pl::ExpPow2{(const long long*)y}, z, (long long)n, (unsigned long long*)bad, s),
                    "efl_pl_mul_exp2");
}

EFL_API int efl_pl_mul_scalar(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* y,
                              uint32_t* z, int64_t n, int64_t* bad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int rc = status_prologue(key_block, key, n, bad, s, "efl_pl_mul_scalar");
  if (rc != EFL_OK || n == 0) return rc;
  Key k{(const uint32_t*)key_block, *key};
  unsigned long long* b = (unsigned long long*)bad;
  hipError_t e = powm_family(k, x, pl::ExpAbs64{(const long long*)y}, z, (long long)n, b, s);
  if (e == hipSuccess) e = invert_ln(k, z, z, (long long)n, b, s, y, 2);
  return hip_status(e, "efl_pl_mul_scalar");
}

EFL_API int efl_pl_mul_scalar_big(const void* key_block, const efl_pl_key* key, const uint32_t* x,
                                  const uint32_t* y_magnitude, int y_words, const int8_t* y_negative, uint32_t* z,
                                  int64_t n, int64_t* bad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int rc = status_prologue(key_block, key, n, bad, s, "efl_pl_mul_scalar_big");
  if (rc != EFL_OK || n == 0) return rc;
  if (y_words <= 0) { set_error("y_words must be positive"); return EFL_E_INVALID_ARGUMENT; }
  Key k{(const uint32_t*)key_block, *key};
  unsigned long long* b = (unsigned long long*)bad;
  hipError_t e = powm_family(k, x, pl::ExpWords{y_magnitude, y_words}, z, (long long)n, b, s);
  if (e == hipSuccess && y_negative) e = invert_ln(k, z, z, (long long)n, b, s, y_negative, 1);
  return hip_status(e, "efl_pl_mul_scalar_big");
}

EFL_API int efl_pl_fxp_add(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* x_exponent,
                           const uint32_t* y, const int64_t* y_exponent, uint32_t* z, int64_t n, int64_t* bad,
                           void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int rc = status_prologue(key_block, key, n, bad, s, "efl_pl_fxp_add");
  if (rc != EFL_OK || n == 0) return rc;
  Key k{(const uint32_t*)key_block, *key};
  unsigned long long* b = (unsigned long long*)bad;
  const long long* xe = (const long long*)x_exponent;
  const long long* ye = (const long long*)y_exponent;
  const int C = slicing(key->ln, 0);
  if (C) {
    const hipError_t e = pl::sl_fxp_add(k, C, x, xe, y, ye, z, (long long)n, b, s);
    if (e != hipErrorNotSupported) return hip_status(e, "efl_pl_fxp_add");
  }
  // families without the fused kernel: the reference's composition, (x << dl) + (y << dr)
  uint32_t* tmp = nullptr;
  const size_t words = (size_t)n * 2 * key->ln;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&tmp), 2 * words * 4, s);
  if (e != hipSuccess) return hip_status(e, "efl_pl_fxp_add");
  e = powm_family(k, x, pl::ExpShift{xe, ye}, tmp, (long long)n, b, s);
  if (e == hipSuccess) e = powm_family(k, y, pl::ExpShift{ye, xe}, tmp + words, (long long)n, b, s);
  if (e == hipSuccess)
    e = C ? pl::sl_add(k, C, tmp, tmp + words, z, (long long)n, s)
          : dispatch_ln<RunAdd>(key->ln, k, tmp, tmp + words, z, (long long)n, s);
  const hipError_t fe = hipFreeAsync(tmp, s);
  return hip_status(e != hipSuccess ? e : fe, "efl_pl_fxp_add");
}

EFL_API int efl_pl_invert(const void* key_block, const efl_pl_key* key, const uint32_t* x, uint32_t* z,
                          int64_t n, int64_t* bad, void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (!bad) { set_error("null status word"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(bad, 0xFF, sizeof(int64_t), s);
  if (e != hipSuccess || n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : hip_status(e, "efl_pl_invert");
  Key k{(const uint32_t*)key_block, *key};
  unsigned long long* b = (unsigned long long*)bad;
  switch (key->ln) {
    case 16: e = run_invert<16>(k, x, z, (long long)n, b, s); break;
    case 32: e = run_invert<32>(k, x, z, (long long)n, b, s); break;
    case 64: e = run_invert<64>(k, x, z, (long long)n, b, s); break;
    case 128: e = run_invert<128>(k, x, z, (long long)n, b, s); break;
    default: e = run_invert<256>(k, x, z, (long long)n, b, s); break;
  }
  return hip_status(e, "efl_pl_invert");
}

EFL_API int efl_pl_matmul(const void* key_block, const efl_pl_key* key, const uint32_t* x_mantissa,
                          const int64_t* x_exponent, const int64_t* y_mantissa, const int64_t* y_exponent,
                          uint32_t* z_pos, uint32_t* z_neg, int64_t* z_exponent, int u, int v, int w,
                          void* stream) {
  if (!key_ok(key_block, key, false, 256)) return EFL_E_INVALID_ARGUMENT;
  if (u < 0 || v <= 0 || w < 0) { set_error("bad matmul shape"); return EFL_E_INVALID_ARGUMENT; }
  if ((long long)u * w == 0) return EFL_OK;
  Key k{(const uint32_t*)key_block, *key};
  const int C = slicing(key->ln, 0);
  if (C)
    return hip_status(pl::sl_matmul(k, C, x_mantissa, (const long long*)x_exponent, (const long long*)y_mantissa,
                                    (const long long*)y_exponent, z_pos, z_neg, (long long*)z_exponent, u, v, w,
                                    (hipStream_t)stream),
                      "efl_pl_matmul");
  return hip_status(dispatch_ln<RunMatmul>(key->ln, k, x_mantissa, (const long long*)x_exponent,
                                            (const long long*)y_mantissa, (const long long*)y_exponent, z_pos,
                                            z_neg, (long long*)z_exponent, u, v, w, (hipStream_t)stream),
                    "efl_pl_matmul");
}

EFL_API int efl_pl_tune(int ln, int decrypt, int limbs_per_lane) {
  if (ln != 16 && ln != 32 && ln != 64 && ln != 128 && ln != 256) { set_error("unsupported limb count %d", ln); return EFL_E_INVALID_ARGUMENT; }
  if (decrypt == 2) {   // sliced decryption's exponentiation: 1 sliding window (default), 0 binary
    if (limbs_per_lane < 0) return pl::sl_dec_window(-1);
    if (limbs_per_lane > 1) { set_error("decryption method must be 0 (binary) or 1 (window)"); return EFL_E_INVALID_ARGUMENT; }
    return pl::sl_dec_window(limbs_per_lane);
  }
  if (decrypt == 4) {   // row-split fixed-base walks: 0 chosen per launch, 1 never, 2..5 parts
    if (limbs_per_lane < 0) return pl::sl_walk_parts(-1);
    if (limbs_per_lane > 5) { set_error("walk parts must be 0 (auto) or 1..5"); return EFL_E_INVALID_ARGUMENT; }
    return pl::sl_walk_parts(limbs_per_lane);
  }
  if (decrypt == 5) {   // the key owner's CRT encryption: 0 chosen per launch, 1 per key, 2 paired lanes
    if (limbs_per_lane < 0) return pl::sl_crt_fused(-1);
    if (limbs_per_lane > 2) { set_error("CRT walk mode must be 0 (chosen), 1 (per key) or 2 (paired lanes)"); return EFL_E_INVALID_ARGUMENT; }
    return pl::sl_crt_fused(limbs_per_lane);
  }
  if (decrypt == 6) {   // the paired CRT encryption's tail: 0 mixed launch, 1 split + join, 2/4/8/16 tree S
    if (limbs_per_lane < 0) return pl::sl_crt_tail(-1);
    if (limbs_per_lane != 0 && limbs_per_lane != 1 && limbs_per_lane != 2 && limbs_per_lane != 4 &&
        limbs_per_lane != 8 && limbs_per_lane != 16) {
      set_error("CRT tail mode must be 0 (tree waves in the whole launch), 1 (split and join) or 2, 4, 8, 16 (tree parts)");
      return EFL_E_INVALID_ARGUMENT;
    }
    return pl::sl_crt_tail(limbs_per_lane);
  }
  if (decrypt == 3) {   // efl_pl_matmul term splits: 0 chosen per launch, 1..16 fixed
    if (limbs_per_lane < 0) return pl::sl_mat_splits(-1);
    if (limbs_per_lane > 16) { set_error("matmul term splits must be 0 (auto) or 1..16"); return EFL_E_INVALID_ARGUMENT; }
    return pl::sl_mat_splits(limbs_per_lane);
  }
  const int dec = decrypt ? 1 : 0;
  if (limbs_per_lane == -2) {                       // back to the measured default, sized per launch
    const int prev = slicing(ln, dec);
    g_slicing[ln_index(ln)][dec] = kDefaultSlicing[ln_index(ln)][dec];
    g_slicing_set[ln_index(ln)][dec] = false;
    return prev;
  }
  if (limbs_per_lane < 0) return slicing(ln, dec);   // query
  if (limbs_per_lane == 0) {
    if (!dec && ln > 64) { set_error("no one-lane kernels for n^2 of %d bits", 64 * ln); return EFL_E_INVALID_ARGUMENT; }
    if (dec && ln > 128) { set_error("no one-lane decryption for p^2 of %d bits", 32 * ln); return EFL_E_INVALID_ARGUMENT; }
  } else if (!pl::sliced_available(dec ? ln : 2 * ln, limbs_per_lane)) {
    set_error("no sliced kernels with %d limbs per lane for %d-limb moduli", limbs_per_lane, dec ? ln : 2 * ln);
    return EFL_E_INVALID_ARGUMENT;
  }
  const int prev = slicing(ln, dec);
  g_slicing[ln_index(ln)][dec] = limbs_per_lane;
  g_slicing_set[ln_index(ln)][dec] = true;
  return prev;
}

EFL_API int efl_hex_lengths(const uint32_t* limbs, int limbs_per_elem, const int8_t* negative,
                            int64_t* lengths, int64_t n, void* stream) {
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  hipLaunchKernelGGL(k_hex_len, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, limbs,
                     limbs_per_elem, (const signed char*)negative, (long long*)lengths, (long long)n);
  return hip_status(hipGetLastError(), "efl_hex_lengths");
}

EFL_API int efl_hex_write(const uint32_t* limbs, int limbs_per_elem, const int8_t* negative,
                          const int64_t* offsets, char* chars, int64_t n, void* stream) {
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  hipLaunchKernelGGL(k_hex_write, dim3((unsigned)((n + kHexWaves - 1) / kHexWaves)), dim3(256), 0, (hipStream_t)stream, limbs,
                     limbs_per_elem, (const signed char*)negative, (const long long*)offsets, chars, (long long)n);
  return hip_status(hipGetLastError(), "efl_hex_write");
}

EFL_API int efl_hex_parse(const char* chars, const int64_t* offsets, int limbs_per_elem, uint32_t* limbs,
                          int8_t* negative, int64_t n, int64_t* bad, void* stream) {
  if (!bad) { set_error("null status word"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(bad, 0xFF, sizeof(int64_t), s);
  if (e != hipSuccess || n <= 0) return hip_status(e, "efl_hex_parse");
  hipLaunchKernelGGL(k_hex_parse, dim3((unsigned)((n + kHexWaves - 1) / kHexWaves)), dim3(256), 0, s, chars,
                     (const long long*)offsets, limbs_per_elem, limbs, (signed char*)negative, (long long)n,
                     (unsigned long long*)bad);
  return hip_status(hipGetLastError(), "efl_hex_parse");
}

EFL_API int efl_pl_to_int64(const uint32_t* magnitude, int limbs_per_elem, const int8_t* negative,
                            int64_t* out, int64_t n, void* stream) {
  if (n <= 0) return n < 0 ? EFL_E_INVALID_ARGUMENT : EFL_OK;
  if (limbs_per_elem < 2) { set_error("need >= 2 limbs"); return EFL_E_INVALID_ARGUMENT; }
  hipLaunchKernelGGL(k_to_int64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     magnitude, limbs_per_elem, (const signed char*)negative, (long long*)out, (long long)n);
  return hip_status(hipGetLastError(), "efl_pl_to_int64");
}
