// Host big-integer arithmetic for the Paillier key setup (csrc/keyset.hip): what the reference's
// PaillierKeypair resource does with GMP when a key is set (paillier.cc:70-101: mpz_set_str base 16,
// mpz_mul, mpz_cdiv_q_ui, mpz_divexact, mpz_invert; gmp_utils.cc:56-89 for the table), plus the
// constants the gfx950 kernels need on top (Montgomery radices, -m^-1 mod 2^32 / 2^28, exact-division
// inverses). Once per key, never on the device: plain schoolbook products and Knuth's algorithm D over
// 32-bit limbs are enough (an 8192-bit key's constants take milliseconds).
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

namespace efl {
namespace hb {

// Non-negative integer, little-endian 32-bit limbs, no high zero limbs (zero = empty).
struct Big {
  std::vector<uint32_t> w;

  Big() = default;
  explicit Big(uint64_t v) {
    while (v) {
      w.push_back((uint32_t)v);
      v >>= 32;
    }
  }
  bool zero() const { return w.empty(); }
  void trim() {
    while (!w.empty() && !w.back()) w.pop_back();
  }
  int bits() const {
    if (w.empty()) return 0;
    return 32 * ((int)w.size() - 1) + (32 - __builtin_clz(w.back()));
  }
  bool bit(int i) const {
    const size_t k = (size_t)i >> 5;
    return k < w.size() && ((w[k] >> (i & 31)) & 1);
  }
  bool odd() const { return !w.empty() && (w[0] & 1); }
};

inline int cmp(const Big& a, const Big& b) {
  if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
  for (size_t i = a.w.size(); i-- > 0;)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
inline bool operator==(const Big& a, const Big& b) { return a.w == b.w; }
inline bool operator!=(const Big& a, const Big& b) { return a.w != b.w; }

inline Big add(const Big& a, const Big& b) {
  const Big& x = a.w.size() >= b.w.size() ? a : b;
  const Big& y = a.w.size() >= b.w.size() ? b : a;
  Big r;
  r.w.resize(x.w.size() + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < x.w.size(); ++i) {
    c += (uint64_t)x.w[i] + (i < y.w.size() ? y.w[i] : 0);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  r.w[x.w.size()] = (uint32_t)c;
  r.trim();
  return r;
}

// a - b, a >= b
inline Big sub(const Big& a, const Big& b) {
  Big r;
  r.w.resize(a.w.size());
  int64_t br = 0;
  for (size_t i = 0; i < a.w.size(); ++i) {
    int64_t d = (int64_t)a.w[i] - (i < b.w.size() ? b.w[i] : 0) - br;
    br = d < 0;
    r.w[i] = (uint32_t)(d + (br << 32));
  }
  r.trim();
  return r;
}

inline Big mul(const Big& a, const Big& b) {
  Big r;
  if (a.zero() || b.zero()) return r;
  r.w.assign(a.w.size() + b.w.size(), 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    uint64_t c = 0;
    const uint64_t ai = a.w[i];
    for (size_t j = 0; j < b.w.size(); ++j) {
      c += ai * b.w[j] + r.w[i + j];
      r.w[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r.w[i + b.w.size()] = (uint32_t)c;
  }
  r.trim();
  return r;
}

inline Big shl(const Big& a, int s) {
  if (a.zero()) return a;
  Big r;
  const int q = s >> 5, b = s & 31;
  r.w.assign(a.w.size() + q + 1, 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    r.w[i + q] |= a.w[i] << b;
    if (b) r.w[i + q + 1] |= a.w[i] >> (32 - b);
  }
  r.trim();
  return r;
}

inline Big shr(const Big& a, int s) {
  const size_t q = (size_t)s >> 5;
  const int b = s & 31;
  Big r;
  if (q >= a.w.size()) return r;
  r.w.assign(a.w.size() - q, 0);
  for (size_t i = 0; i < r.w.size(); ++i) {
    r.w[i] = a.w[i + q] >> b;
    if (b && i + q + 1 < a.w.size()) r.w[i] |= a.w[i + q + 1] << (32 - b);
  }
  r.trim();
  return r;
}

inline Big pow2(int e) { return shl(Big(1), e); }

// a mod 2^e
inline Big low_bits(const Big& a, int e) {
  Big r = a;
  const size_t words = ((size_t)e + 31) >> 5;
  if (r.w.size() > words) r.w.resize(words);
  if ((e & 31) && r.w.size() == words) r.w[words - 1] &= (1u << (e & 31)) - 1;
  r.trim();
  return r;
}

// Knuth, TAOCP vol. 2, 4.3.1 algorithm D: q = a / b, r = a mod b (b != 0). q or r may be null.
inline void divmod(const Big& a, const Big& b, Big* q, Big* r) {
  if (cmp(a, b) < 0) {
    if (q) *q = Big();
    if (r) *r = a;
    return;
  }
  const size_t n = b.w.size(), m = a.w.size() - n;
  if (n == 1) {
    Big qq;
    qq.w.assign(a.w.size(), 0);
    uint64_t rem = 0;
    for (size_t i = a.w.size(); i-- > 0;) {
      const uint64_t cur = (rem << 32) | a.w[i];
      qq.w[i] = (uint32_t)(cur / b.w[0]);
      rem = cur % b.w[0];
    }
    qq.trim();
    if (q) *q = qq;
    if (r) *r = Big(rem);
    return;
  }
  const int s = __builtin_clz(b.w.back());
  std::vector<uint32_t> v(n), u(a.w.size() + 1);
  for (size_t i = n; i-- > 0;) v[i] = (b.w[i] << s) | (s && i ? b.w[i - 1] >> (32 - s) : 0);
  u[a.w.size()] = s ? a.w.back() >> (32 - s) : 0;
  for (size_t i = a.w.size(); i-- > 0;) u[i] = (a.w[i] << s) | (s && i ? a.w[i - 1] >> (32 - s) : 0);
  Big qq;
  qq.w.assign(m + 1, 0);
  for (size_t j = m + 1; j-- > 0;) {
    const uint64_t num = ((uint64_t)u[j + n] << 32) | u[j + n - 1];
    uint64_t qhat = num / v[n - 1], rhat = num % v[n - 1];
    while (qhat >> 32 || qhat * v[n - 2] > ((rhat << 32) | u[j + n - 2])) {
      --qhat;
      rhat += v[n - 1];
      if (rhat >> 32) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t p = qhat * v[i] + carry;
      carry = p >> 32;
      const int64_t t = (int64_t)u[i + j] - (int64_t)(uint32_t)p - borrow;
      u[i + j] = (uint32_t)t;
      borrow = t < 0;
    }
    const int64_t t = (int64_t)u[j + n] - (int64_t)carry - borrow;
    u[j + n] = (uint32_t)t;
    if (t < 0) {                          // qhat one too large: add v back
      --qhat;
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        c += (uint64_t)u[i + j] + v[i];
        u[i + j] = (uint32_t)c;
        c >>= 32;
      }
      u[j + n] += (uint32_t)c;
    }
    qq.w[j] = (uint32_t)qhat;
  }
  qq.trim();
  if (q) *q = qq;
  if (r) {
    Big rr;
    rr.w.assign(n, 0);
    for (size_t i = 0; i < n; ++i) rr.w[i] = (u[i] >> s) | (s ? (uint32_t)((uint64_t)u[i + 1] << (32 - s)) : 0);
    rr.trim();
    *r = rr;
  }
}

inline Big mod(const Big& a, const Big& m) {
  Big r;
  divmod(a, m, nullptr, &r);
  return r;
}

// ceil(a / b)
inline Big cdiv(const Big& a, const Big& b) {
  Big q, r;
  divmod(a, b, &q, &r);
  return r.zero() ? q : add(q, Big(1));
}

// a^-1 mod m (extended Euclid); false when gcd(a, m) != 1 (mpz_invert's failure)
inline bool modinv(const Big& a, const Big& m, Big* out) {
  Big r0 = m, r1 = mod(a, m);
  Big s0, s1(1);               // Bezout coefficients of a, as magnitude + sign
  bool n0 = false, n1 = false;
  while (!r1.zero()) {
    Big q, r2;
    divmod(r0, r1, &q, &r2);
    // s2 = s0 - q s1
    const Big t = mul(q, s1);
    Big s2;
    bool n2;
    if (n0 != n1) {            // s0 and -q s1 have the same sign
      s2 = add(s0, t);
      n2 = n0;
    } else if (cmp(s0, t) >= 0) {
      s2 = sub(s0, t);
      n2 = n0;
    } else {
      s2 = sub(t, s0);
      n2 = !n0;
    }
    r0 = r1;
    r1 = r2;
    s0 = s1;
    n0 = n1;
    s1 = s2;
    n1 = n2;
  }
  if (r0 != Big(1)) return false;
  Big v = mod(s0, m);
  if (n0 && !v.zero()) v = sub(m, v);
  *out = v;
  return true;
}

// -m^-1 mod 2^32 (m odd): the Montgomery constant of the 32-bit limb kernels
inline uint32_t minv32(const Big& m) {
  const uint32_t m0 = m.w.empty() ? 0 : m.w[0];
  uint32_t x = m0;                        // Newton: x = m0^-1 mod 2^32
  for (int i = 0; i < 5; ++i) x *= 2 - m0 * x;
  return (uint32_t)0 - x;
}
// -m^-1 mod 2^28 (radix-2^28 kernels)
inline uint32_t minv28(const Big& m) { return minv32(m) & 0xFFFFFFFu; }

// fixed-width little-endian 32-bit words (zero-padded; the caller checks the width)
inline void put_words(const Big& a, int L, uint32_t* out) {
  for (int i = 0; i < L; ++i) out[i] = (size_t)i < a.w.size() ? a.w[i] : 0;
}
// L radix-2^28 limbs, one per 32-bit word (csrc/sliced28.h)
inline void put_limbs28(const Big& a, int L, uint32_t* out) {
  for (int k = 0; k < L; ++k) {
    const int bit = 28 * k, q = bit >> 5, r = bit & 31;
    uint64_t v = (size_t)q < a.w.size() ? a.w[q] : 0;
    if ((size_t)q + 1 < a.w.size()) v |= (uint64_t)a.w[q + 1] << 32;
    out[k] = (uint32_t)(v >> r) & 0xFFFFFFFu;
  }
}

// mpz_set_str(x, s, 16) of a non-negative hex text: digits in either case, white space anywhere
// ignored (as GMP ignores it); false on an empty text or any other character (mpz_set_str returns -1)
inline bool from_hex(const char* s, size_t len, Big* out) {
  std::vector<uint8_t> dg;
  dg.reserve(len);
  for (size_t i = 0; i < len; ++i) {
    const char c = s[i];
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') continue;
    if (c >= '0' && c <= '9') dg.push_back((uint8_t)(c - '0'));
    else if (c >= 'a' && c <= 'f') dg.push_back((uint8_t)(c - 'a' + 10));
    else if (c >= 'A' && c <= 'F') dg.push_back((uint8_t)(c - 'A' + 10));
    else return false;
  }
  if (dg.empty()) return false;
  Big r;
  const size_t nd = dg.size();
  r.w.assign((nd + 7) / 8, 0);
  for (size_t k = 0; k < nd; ++k) r.w[k >> 3] |= (uint32_t)dg[nd - 1 - k] << (4 * (k & 7));
  r.trim();
  *out = r;
  return true;
}

inline std::string to_hex(const Big& a) {
  if (a.zero()) return "0";
  static const char* dg = "0123456789abcdef";
  std::string s;
  for (size_t i = a.w.size(); i-- > 0;)
    for (int k = 7; k >= 0; --k) {
      const char c = dg[(a.w[i] >> (4 * k)) & 15];
      if (s.empty() && c == '0') continue;
      s.push_back(c);
    }
  return s;
}

}  // namespace hb
}  // namespace efl
