// Pieces shared by the one-lane (paillier.hip) and the sliced (paillier_sliced.hip) Paillier kernels.
#pragma once

#include "common.h"

namespace efl {
namespace pl {

// key block (device, 32-bit limbs) + the descriptor of where each constant lives in it
struct Key {
  const uint32_t* base;
  efl_pl_key d;
  __device__ __forceinline__ const uint32_t* at(int64_t off) const { return base + off; }
};

// Philox4x32-10 (Salmon et al., SC'11): counter (ctr_lo, ctr_hi, block, 0), key = seed.
// NB independent blocks advance round by round together (philox_n), so the chains interleave.
template <int NB>
__device__ __forceinline__ void philox_n(uint32_t (&c)[NB][4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c[b][0];
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[b][2];
      // three-input XORs in one v_bitop3_b32 each (truth table 0x96); the compiler emits two v_xor
      const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c[b][1], k0, 0x96);
      const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c[b][3], k1, 0x96);
      c[b][0] = n0;
      c[b][1] = (uint32_t)p1;
      c[b][2] = n2;
      c[b][3] = (uint32_t)p0;
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ void philox(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  philox_n<1>(reinterpret_cast<uint32_t (&)[1][4]>(c), k0, k1);
}

// ---- the fixed-base exponent (FixedBasePowm, gmp_utils.cc:107-144) --------------------------
// An element's exponent a lives as `words` little-endian 32-bit words in an LDS column of stride
// S. The reference's mpz_fbpowm builds each g-bit group's table index MSB-first from the group's
// LOW bit (the top group is as wide as a's remaining bit length), so what it computes is hs^(a'),
// a' = a with every group bit-reversed. The kernels form a' in place
// with the API group size and then walk a' in plain windows of the table's OWN width
// (efl_pl_key.table_window): the result is the same group element for any window, and the window
// only sets the cost (one product per non-zero window).

// bits [s, s + w) of the column's number, 1 <= w <= 32
__device__ __forceinline__ uint32_t col_bits(const uint32_t* col, int S, int s, int w, int words) {
  const int q = s >> 5, r = s & 31;
  uint64_t v = col[q * S];
  if (r + w > 32 && q + 1 < words) v |= (uint64_t)col[(q + 1) * S] << 32;
  return (uint32_t)(v >> r) & (uint32_t)((1ull << w) - 1ull);
}

__device__ __forceinline__ void col_put_bits(uint32_t* col, int S, int s, int w, uint32_t val, int words) {
  const int q = s >> 5, r = s & 31;
  const bool two = r + w > 32 && q + 1 < words;
  uint64_t v = col[q * S];
  if (two) v |= (uint64_t)col[(q + 1) * S] << 32;
  const uint64_t mask = ((1ull << w) - 1ull) << r;
  v = (v & ~mask) | (((uint64_t)val << r) & mask);
  col[q * S] = (uint32_t)v;
  if (two) col[(q + 1) * S] = (uint32_t)(v >> 32);
}

// bit length of the column's number
__device__ __forceinline__ int col_bit_length(const uint32_t* col, int S, int words) {
  for (int w = words - 1; w >= 0; --w) {
    const uint32_t v = col[w * S];
    if (v) return w * 32 + 32 - __clz(v);
  }
  return 0;
}

// a -> a' in place: every g-bit group of a's `size` bits (the top one `size mod g` wide)
// bit-reversed. g == 1 is the identity.
__device__ __forceinline__ void regroup_exponent(uint32_t* col, int S, int size, int g, int words) {
  if (g <= 1) return;
  for (int s = 0; s < size; s += g) {
    const int w = size - s < g ? size - s : g;
    const uint32_t v = col_bits(col, S, s, w, words);
    col_put_bits(col, S, s, w, __brev(v) >> (32 - w), words);
  }
}

// width of the table's windows (0 in a descriptor from before the field existed: the API group
// size, whose table is the same T[i][j] = hs^((j+1) 2^(g i)))
__device__ __forceinline__ int table_window(const efl_pl_key& d) {
  return d.table_window > 0 ? d.table_window : d.group_size;
}

// ---- per-element exponents of the powm kernels (PaillierMulScalar / PaillierMulExp2) ----------
// `xs.at(i)` gives element i's exponent: ok (false -> the op's InvalidArgument for that element),
// bits (bit length; 0 -> x^0 = 1) and bit(b). The kernels run left to right: for b = bits-2 .. 0,
// one squaring, then a multiply by x when bit(b) is set.
//
// Shifts (2^y) are capped: the reference's mpz_mul_2exp(1, y) + mpz_powm (paillier.cc:724-732)
// does y squarings too, so a y far past any fixed-point exponent difference (fp64 spans ~2,200)
// is hours of work there; here y > kMaxShift is reported like a negative y instead of occupying a
// wave for minutes.
constexpr long long kMaxShift = 1ll << 16;

// |e| as `ew` little-endian 32-bit words per element (efl_pl_powm)
struct ExpWords {
  const uint32_t* e;
  int ew;
  struct El {
    const uint32_t* p;
    int nbits;
    bool ok;
    __device__ __forceinline__ int bits() const { return nbits; }
    __device__ __forceinline__ bool bit(int b) const { return (p[b >> 5] >> (b & 31)) & 1u; }
  };
  __device__ __forceinline__ El at(long long i) const {
    const uint32_t* p = e + i * ew;
    int nb = 0;
    for (int w = ew - 1; w >= 0; --w)
      if (p[w]) { nb = w * 32 + 32 - __clz(p[w]); break; }
    return El{p, nb, true};
  }
};

// |y| of an int64 scalar (PaillierMulScalar<int64>: mpz_set_sll, then the sign picks x or x^-1)
struct ExpAbs64 {
  const long long* y;
  struct El {
    uint64_t v;
    bool ok;
    __device__ __forceinline__ int bits() const { return v ? 64 - __clzll(v) : 0; }
    __device__ __forceinline__ bool bit(int b) const { return (v >> b) & 1ull; }
  };
  __device__ __forceinline__ El at(long long i) const {
    const long long s = y[i];
    return El{s < 0 ? 0ull - (uint64_t)s : (uint64_t)s, true};
  }
};

// 2^y (PaillierMulExp2: y squarings, no multiply); y < 0 or y > kMaxShift -> not ok
struct ExpPow2 {
  const long long* y;
  struct El {
    long long s;
    bool ok;
    __device__ __forceinline__ int bits() const { return (int)s + 1; }
    __device__ __forceinline__ bool bit(int) const { return false; }
  };
  __device__ __forceinline__ El at(long long i) const {
    const long long s = y[i];
    return El{s, s >= 0 && s <= kMaxShift};
  }
};

// 2^(own - min(own, other)): one side of FixedPointTensor.__add__'s exponent alignment
// (paillier.py:119-132: dl = max(d, 0), dr = |min(d, 0)|, d = self.exponent - another.exponent)
struct ExpShift {
  const long long* own;
  const long long* other;
  __device__ __forceinline__ ExpPow2::El at(long long i) const {
    const long long a = own[i], b = other[i];
    if (a <= b) return ExpPow2::El{0, true};
    const uint64_t d = (uint64_t)a - (uint64_t)b;
    return ExpPow2::El{d <= (uint64_t)kMaxShift ? (long long)d : 0, d <= (uint64_t)kMaxShift};
  }
};

// Sliced kernels (paillier_sliced.hip): one number over L/C lanes of C limbs. L = limbs of the
// modulus the op works in (2*ln for n^2 ops, ln for decryption's p^2 / q^2).
bool sliced_available(int L, int C);
hipError_t sl_encrypt(const Key& k, int C, const long long* m, const uint32_t* hsa, uint32_t* out, long long N,
                      uint64_t seed, long long ctr0, hipStream_t s, int hsa_mont = 0);
hipError_t sl_fbpowm(const Key& k, int C, const uint32_t* a, uint32_t* out, long long N, uint64_t seed,
                     long long ctr0, hipStream_t s);
// the key owner's CRT walk from the element's own start (y^2)^-1 g(m) mod x^2 (k_fbpowm28g; the
// sub-key's off_gn28 / off_gstart28): hipErrorNotSupported when the sub-key has no such constants or
// its radix-2^28 table does not serve family C
hipError_t sl_fbpowm_g(const Key& k, int C, const long long* m, const uint32_t* a, uint32_t* out, long long N,
                       uint64_t seed, long long ctr0, hipStream_t s);
int sl_crt_fused(int v);
int sl_crt_tail(int v);
// the key owner's whole CRT encryption (or hs^(a') for m NULL) with an element's two walks in one
// wave and the CRT join at its end: the ciphertext mod n^2 (n2w = n^2 in 32-bit words) into out
// ([N][2 C] words). hipErrorNotSupported unless the one-lane family C = 32 serves both sub-keys
// with equal tables (and under efl_pl_tune(ln, 5, 1))
hipError_t sl_crt_encrypt_pair(const Key& kp, const Key& kq, int C, const uint32_t* n2w, const long long* m,
                               const uint32_t* a, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                               hipStream_t s);
hipError_t sl_add(const Key& k, int C, const uint32_t* x, const uint32_t* y, uint32_t* out, long long N,
                  hipStream_t s);
hipError_t sl_powm(const Key& k, int C, const uint32_t* x, const uint32_t* e, int ew, uint32_t* out, long long N,
                   hipStream_t s);
// the same exponentiation with the exponent read from an int64 tensor: |y| (MulScalar) or 2^y
// (MulExp2); elements whose exponent is not ok get z = 0 and their index atomically min'ed into bad
hipError_t sl_powm_abs64(const Key& k, int C, const uint32_t* x, const long long* y, uint32_t* out, long long N,
                         unsigned long long* bad, hipStream_t s);
hipError_t sl_powm_pow2(const Key& k, int C, const uint32_t* x, const long long* y, uint32_t* out, long long N,
                        unsigned long long* bad, hipStream_t s);
hipError_t sl_powm_shift(const Key& k, int C, const uint32_t* x, const long long* own, const long long* other,
                         uint32_t* out, long long N, unsigned long long* bad, hipStream_t s);
// z = x^(2^(xe - m)) y^(2^(ye - m)) mod n^2, m = min(xe, ye): FixedPointTensor.__add__ in one launch
// (radix-2^28 family only: hipErrorNotSupported otherwise, and the caller composes powm + add)
hipError_t sl_fxp_add(const Key& k, int C, const uint32_t* x, const long long* xe, const uint32_t* y,
                      const long long* ye, uint32_t* out, long long N, unsigned long long* bad, hipStream_t s);
hipError_t sl_matmul(const Key& k, int C, const uint32_t* X, const long long* xe, const long long* ym,
                     const long long* ye, uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w,
                     hipStream_t s);
hipError_t sl_decrypt(const Key& k, int C, const uint32_t* ct, uint32_t* mag, signed char* neg, long long N,
                      hipStream_t s);
// sliced decryption's exponentiation method: 1 sliding window (default), 0 binary; v < 0 queries.
// Returns the previous setting.
int sl_dec_window(int v);
// efl_pl_matmul's term splits: 0 chosen per launch (default), else 1..16 (rounded down to a power of
// two); v < 0 queries. Returns the previous setting.
int sl_mat_splits(int v);
int sl_walk_parts(int v);

}  // namespace pl
}  // namespace efl
