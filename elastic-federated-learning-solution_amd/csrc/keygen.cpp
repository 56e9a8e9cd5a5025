// Host arithmetic of GeneratePaillierKeypair (efls-train/cc/efl/math/paillier.cc:833-904): the
// prime search's probable-prime tests and hs = (-x^2)^n mod n^2. The reference runs them with GMP
// inside its CPU op; the Python host side of this build hands the candidates it drew (and sieved)
// to these functions instead of running CPython's big-integer pow, which is about 10x slower per
// modular exponentiation at 2048 bits. Montgomery arithmetic over 64-bit limbs (CIOS, unsigned
// __int128 products), fixed 4-bit windows; the candidates of one call are tested on `threads`
// host threads. Keys are made once per session (and on each re-key), never on the device.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "efl_hip.h"

#define EFL_API extern "C" __attribute__((visibility("default")))

namespace efl {
void set_error(const char* fmt, ...);
}

namespace {

typedef unsigned __int128 u128;

struct Mont {
  int L = 0;                    // 64-bit limbs
  std::vector<uint64_t> m;      // odd modulus
  uint64_t minv = 0;            // -m^-1 mod 2^64
  std::vector<uint64_t> one;    // R mod m (Montgomery form of 1)
  std::vector<uint64_t> r2;     // R^2 mod m
  std::vector<uint64_t> t;      // CIOS scratch, L + 2 limbs

  // a >= b, both L limbs
  static bool geq(const uint64_t* a, const uint64_t* b, int L) {
    for (int i = L - 1; i >= 0; --i)
      if (a[i] != b[i]) return a[i] > b[i];
    return true;
  }
  static void sub(uint64_t* a, const uint64_t* b, int L) {
    uint64_t br = 0;
    for (int i = 0; i < L; ++i) {
      const u128 d = (u128)a[i] - b[i] - br;
      a[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
  }
  // x <- 2x mod m (x < m)
  void dbl(uint64_t* x) const {
    uint64_t top = x[L - 1] >> 63;
    for (int i = L - 1; i > 0; --i) x[i] = (x[i] << 1) | (x[i - 1] >> 63);
    x[0] <<= 1;
    if (top || geq(x, m.data(), L)) sub(x, m.data(), L);
  }

  explicit Mont(const std::vector<uint64_t>& mod) : L((int)mod.size()), m(mod), one(mod.size()), r2(mod.size()),
                                                     t(mod.size() + 2) {
    uint64_t x = m[0];                      // Newton: x = m0^-1 mod 2^64
    for (int i = 0; i < 6; ++i) x *= 2 - m[0] * x;
    minv = (uint64_t)0 - x;
    std::vector<uint64_t> v(L, 0);
    v[0] = 1;
    if (L == 1 && m[0] == 1) v[0] = 0;
    for (int i = 0; i < 64 * L; ++i) dbl(v.data());   // 2^(64 L) mod m
    one = v;
    for (int i = 0; i < 64 * L; ++i) dbl(v.data());   // 2^(128 L) mod m
    r2 = v;
  }

  // CIOS with the limb count fixed at compile time: the inner loops unroll and the carries stay
  // in registers (3-4x the generic loop's rate at 2048-4096 bits)
  template <int N>
  void mul_fixed(uint64_t* out, const uint64_t* a, const uint64_t* b) {
    uint64_t T[N + 2] = {0};
    const uint64_t* M = m.data();
    for (int i = 0; i < N; ++i) {
      uint64_t c = 0;
      const uint64_t bi = b[i];
#pragma GCC unroll 16
      for (int j = 0; j < N; ++j) {
        const u128 s = (u128)a[j] * bi + T[j] + c;
        T[j] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      u128 s = (u128)T[N] + c;
      T[N] = (uint64_t)s;
      T[N + 1] = (uint64_t)(s >> 64);
      const uint64_t u = T[0] * minv;
      s = (u128)u * M[0] + T[0];
      c = (uint64_t)(s >> 64);
#pragma GCC unroll 16
      for (int j = 1; j < N; ++j) {
        s = (u128)u * M[j] + T[j] + c;
        T[j - 1] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      s = (u128)T[N] + c;
      T[N - 1] = (uint64_t)s;
      T[N] = T[N + 1] + (uint64_t)(s >> 64);
    }
    if (T[N] || geq(T, M, N)) sub(T, M, N);
    memcpy(out, T, 8 * (size_t)N);
  }

  // out <- a b R^-1 mod m (a, b < m); out may alias a or b
  void mul(uint64_t* out, const uint64_t* a, const uint64_t* b) {
    switch (L) {
      case 8: return mul_fixed<8>(out, a, b);
      case 16: return mul_fixed<16>(out, a, b);
      case 32: return mul_fixed<32>(out, a, b);
      case 64: return mul_fixed<64>(out, a, b);
      case 128: return mul_fixed<128>(out, a, b);
      default: break;
    }
    uint64_t* T = t.data();
    std::fill(t.begin(), t.end(), 0);
    for (int i = 0; i < L; ++i) {
      uint64_t c = 0;
      const uint64_t bi = b[i];
      for (int j = 0; j < L; ++j) {
        const u128 s = (u128)a[j] * bi + T[j] + c;
        T[j] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      u128 s = (u128)T[L] + c;
      T[L] = (uint64_t)s;
      T[L + 1] = (uint64_t)(s >> 64);
      const uint64_t u = T[0] * minv;
      s = (u128)u * m[0] + T[0];
      c = (uint64_t)(s >> 64);
      for (int j = 1; j < L; ++j) {
        s = (u128)u * m[j] + T[j] + c;
        T[j - 1] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      s = (u128)T[L] + c;
      T[L - 1] = (uint64_t)s;
      T[L] = T[L + 1] + (uint64_t)(s >> 64);
    }
    if (T[L] || geq(T, m.data(), L)) sub(T, m.data(), L);
    memcpy(out, T, 8 * (size_t)L);
  }

  // out <- base^exp mod m in Montgomery form (base < m, ordinary form); exp: ew 64-bit words
  void powm_mont(uint64_t* out, const uint64_t* base, const uint64_t* exp, int ew) {
    std::vector<uint64_t> tab(16 * (size_t)L);
    memcpy(tab.data(), one.data(), 8 * (size_t)L);
    mul(&tab[L], base, r2.data());
    for (int k = 2; k < 16; ++k) mul(&tab[(size_t)k * L], &tab[(size_t)(k - 1) * L], &tab[L]);
    std::vector<uint64_t> acc(one);
    int top = ew * 64 - 1;
    while (top >= 0 && !((exp[top >> 6] >> (top & 63)) & 1)) --top;
    const int nib = (top + 4) / 4;          // 4-bit windows from the top
    for (int w = nib - 1; w >= 0; --w) {
      if (w != nib - 1)
        for (int s = 0; s < 4; ++s) mul(acc.data(), acc.data(), acc.data());
      const int bit = 4 * w;
      const unsigned d = (unsigned)((exp[bit >> 6] >> (bit & 63)) & 15);
      if (d) mul(acc.data(), acc.data(), &tab[(size_t)d * L]);
    }
    memcpy(out, acc.data(), 8 * (size_t)L);
  }
};

std::vector<uint64_t> to64(const uint32_t* w, int words, int L) {
  std::vector<uint64_t> v(L, 0);
  for (int i = 0; i < words; ++i) v[i >> 1] |= (uint64_t)w[i] << (32 * (i & 1));
  return v;
}

bool is_zero(const std::vector<uint64_t>& v) {
  for (uint64_t x : v)
    if (x) return false;
  return true;
}

// Miller-Rabin of odd n > 3 with the given bases (each in [2, n - 2]); true = probable prime
bool miller_rabin(const std::vector<uint64_t>& n, const uint32_t* bases, int reps, int words) {
  const int L = (int)n.size();
  Mont M(n);
  std::vector<uint64_t> d(n);
  d[0] -= 1;                                    // n odd: no borrow
  int s = 0;
  while (!(d[0] & 1)) {
    for (int i = 0; i < L - 1; ++i) d[i] = (d[i] >> 1) | (d[i + 1] << 63);
    d[L - 1] >>= 1;
    ++s;
  }
  std::vector<uint64_t> mone(n);                 // (n - 1) R mod n = n - (R mod n)
  Mont::sub(mone.data(), M.one.data(), L);
  std::vector<uint64_t> x(L);
  for (int r = 0; r < reps; ++r) {
    const std::vector<uint64_t> a = to64(bases + (size_t)r * words, words, L);
    M.powm_mont(x.data(), a.data(), d.data(), L);
    if (x == M.one || x == mone) continue;
    bool witness = true;
    for (int k = 1; k < s && witness; ++k) {
      M.mul(x.data(), x.data(), x.data());
      if (x == mone) witness = false;
      else if (x == M.one) break;              // a non-trivial square root of 1: composite
    }
    if (witness) return false;
  }
  return true;
}

}  // namespace

// base^exp mod mod (mod odd, base < mod), all little-endian 32-bit words; out has mod_words words.
EFL_API int efl_host_powm(const uint32_t* base, int base_words, const uint32_t* exp, int exp_words,
                          const uint32_t* mod, int mod_words, uint32_t* out) {
  if (!base || !exp || !mod || !out || mod_words <= 0 || base_words < 0 || exp_words < 0 || base_words > mod_words) {
    efl::set_error("efl_host_powm: bad arguments");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!(mod[0] & 1)) {
    efl::set_error("efl_host_powm: the modulus must be odd");
    return EFL_E_INVALID_ARGUMENT;
  }
  const int L = (mod_words + 1) / 2;
  const std::vector<uint64_t> m = to64(mod, mod_words, L), b = to64(base, base_words, L);
  if (Mont::geq(b.data(), m.data(), L)) {
    efl::set_error("efl_host_powm: base must be below the modulus");
    return EFL_E_INVALID_ARGUMENT;
  }
  const int EL = std::max(1, (exp_words + 1) / 2);
  const std::vector<uint64_t> e = to64(exp, exp_words, EL);
  Mont M(m);
  std::vector<uint64_t> r(L), plain(L, 0);
  plain[0] = 1;
  M.powm_mont(r.data(), b.data(), e.data(), EL);
  M.mul(r.data(), r.data(), plain.data());      // out of Montgomery form
  if (is_zero(e)) {                             // x^0 = 1 (mod 1 = 0)
    r.assign(L, 0);
    if (!(mod_words == 1 && mod[0] == 1)) r[0] = 1;
  }
  for (int i = 0; i < mod_words; ++i) out[i] = (uint32_t)(r[i >> 1] >> (32 * (i & 1)));
  return 0;
}

// The fixed-base table's row bases (gmp_utils.cc:73-88 raises the base by 2^W per row):
// out[i] = base^(2^(k i)) mod mod for i in [0, steps), mod odd, base < mod; out is [steps][mod_words].
// One Montgomery setup for the whole chain of k (steps - 1) squarings.
EFL_API int efl_host_sqr_chain(const uint32_t* base, int base_words, int k, int steps, const uint32_t* mod,
                               int mod_words, uint32_t* out) {
  if (!base || !mod || !out || mod_words <= 0 || base_words < 0 || base_words > mod_words || k < 0 || steps < 0) {
    efl::set_error("efl_host_sqr_chain: bad arguments");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!(mod[0] & 1)) {
    efl::set_error("efl_host_sqr_chain: the modulus must be odd");
    return EFL_E_INVALID_ARGUMENT;
  }
  const int L = (mod_words + 1) / 2;
  const std::vector<uint64_t> m = to64(mod, mod_words, L), b = to64(base, base_words, L);
  if (Mont::geq(b.data(), m.data(), L)) {
    efl::set_error("efl_host_sqr_chain: base must be below the modulus");
    return EFL_E_INVALID_ARGUMENT;
  }
  Mont M(m);
  std::vector<uint64_t> x(L), y(L), one(L, 0);
  one[0] = 1;
  M.mul(x.data(), b.data(), M.r2.data());      // base R
  for (int i = 0; i < steps; ++i) {
    if (i)
      for (int s = 0; s < k; ++s) M.mul(x.data(), x.data(), x.data());
    M.mul(y.data(), x.data(), one.data());      // out of Montgomery form
    uint32_t* o = out + (size_t)i * mod_words;
    for (int j = 0; j < mod_words; ++j) o[j] = (uint32_t)(y[j >> 1] >> (32 * (j & 1)));
  }
  return 0;
}

// Miller-Rabin of `count` odd candidates ([count][words] 32-bit words, each > 3) with `reps` bases
// each ([count][reps][words], in [2, c - 2]); out[i] = 1 probable prime, 0 composite. Candidates
// are shared out over `threads` host threads (<= 0: hardware concurrency).
EFL_API int efl_host_probable_primes(const uint32_t* cands, int words, int count, const uint32_t* bases, int reps,
                                     int threads, int8_t* out) {
  if (!cands || !bases || !out || words <= 0 || count < 0 || reps < 1) {
    efl::set_error("efl_host_probable_primes: bad arguments");
    return EFL_E_INVALID_ARGUMENT;
  }
  for (int i = 0; i < count; ++i)
    if (!(cands[(size_t)i * words] & 1)) {
      efl::set_error("efl_host_probable_primes: candidate %d is even", i);
      return EFL_E_INVALID_ARGUMENT;
    }
  int T = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  T = std::min(T, std::max(1, count));
  const int L = (words + 1) / 2;
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int i = next++; i < count; i = next++)
      out[i] = miller_rabin(to64(cands + (size_t)i * words, words, L), bases + (size_t)i * reps * words, reps, words)
                   ? 1 : 0;
  };
  std::vector<std::thread> pool;
  for (int k = 1; k < T; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}
