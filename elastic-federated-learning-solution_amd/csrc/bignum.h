// Multi-precision arithmetic for the Paillier kernels (gfx950), one big number per lane.
//
// Numbers are L little-endian 32-bit limbs. Products use v_mad_u64_u32 (32x32+64 -> 64).
// Montgomery multiplication is CIOS (coarsely integrated operand scanning): for each limb b_i,
// t += a*b_i, then t += u*m with u = t_0 * (-m^-1 mod 2^32), then t >>= 32. The outer loop runs
// over limbs of b, read either from the lane's LDS column (stride = workgroup size, so a wave's 64
// reads of one limb index hit 64 consecutive dwords: conflict-free) or from a wave-uniform
// constant (scalar loads); the inner loops are fully unrolled so a and t stay in VGPRs.
// Every operation is in place on its register operand so at most two L-limb arrays are live
// (the operand and the accumulator): 2L+1 VGPRs for the arithmetic itself.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace efl {
namespace big {

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;
}

template <int L>
__device__ __forceinline__ void copy(uint32_t (&d)[L], const uint32_t (&s)[L]) {
#pragma unroll
  for (int j = 0; j < L; ++j) d[j] = s[j];
}

// x >= m ?  (m uniform)
template <int L>
__device__ __forceinline__ bool geq(const uint32_t (&x)[L], const uint32_t* __restrict__ m) {
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const uint64_t d = (uint64_t)x[j] - m[j] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow == 0;
}

// x -= m if cond (branch-free select)
template <int L>
__device__ __forceinline__ void csub(uint32_t (&x)[L], const uint32_t* __restrict__ m, bool cond) {
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const uint64_t d = (uint64_t)x[j] - m[j] - borrow;
    borrow = (uint32_t)(d >> 63);
    x[j] = cond ? (uint32_t)d : x[j];
  }
}

// Sources of the b operand: a lane's LDS column (stride S words) or a wave-uniform constant.
struct LdsCol {
  const uint32_t* p;
  int S;
  __device__ __forceinline__ uint32_t operator()(int i) const { return p[i * S]; }
};
struct Uniform {
  const uint32_t* __restrict__ p;
  __device__ __forceinline__ uint32_t operator()(int i) const { return p[i]; }
};

// a <- a * b * 2^(-32L) mod m, for a, b < m.
template <int L, class B>
__device__ __forceinline__ void mont_mul(uint32_t (&a)[L], const B& b, const uint32_t* __restrict__ m,
                                         uint32_t minv) {
  uint32_t t[L + 1];
#pragma unroll
  for (int j = 0; j <= L; ++j) t[j] = 0;
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    // keep the modulus limbs as per-iteration scalar loads: hoisting L of them out of the loop
    // would pin L SGPRs (spilled to VGPRs for L >= 64)
    asm volatile("" ::: "memory");
    const uint32_t bi = b(i);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t p = mad(a[j], bi, (uint64_t)t[j] + c);
      t[j] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    uint64_t s = (uint64_t)t[L] + c;
    t[L] = (uint32_t)s;
    const uint32_t top = (uint32_t)(s >> 32);
    const uint32_t u = t[0] * minv;
    c = (uint32_t)(mad(m[0], u, t[0]) >> 32);
#pragma unroll
    for (int j = 1; j < L; ++j) {
      const uint64_t p = mad(m[j], u, (uint64_t)t[j] + c);
      t[j - 1] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    s = (uint64_t)t[L] + c;
    t[L - 1] = (uint32_t)s;
    t[L] = top + (uint32_t)(s >> 32);
  }
#pragma unroll
  for (int j = 0; j < L; ++j) a[j] = t[j];
  const bool ge = t[L] != 0 || geq<L>(a, m);
  csub<L>(a, m, ge);
}

// store this lane's LDS column
template <int L>
__device__ __forceinline__ void to_lds(uint32_t* col, int S, const uint32_t (&x)[L]) {
#pragma unroll
  for (int j = 0; j < L; ++j) col[j * S] = x[j];
}

// a <- a^2 R^-1 mod m (a staged through the lane's scratch column)
template <int L>
__device__ __forceinline__ void mont_sqr(uint32_t (&a)[L], uint32_t* scratch, int S,
                                         const uint32_t* __restrict__ m, uint32_t minv) {
  to_lds<L>(scratch, S, a);
  mont_mul<L>(a, LdsCol{scratch, S}, m, minv);
}

// a <- a * 2^(-32L) mod m for an L-limb a < 2^(32L) (Montgomery -> normal form).
template <int L>
__device__ __forceinline__ void redc(uint32_t (&a)[L], const uint32_t* __restrict__ m, uint32_t minv) {
  uint32_t top = 0;   // limb L of the running value
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    asm volatile("" ::: "memory");
    const uint32_t u = a[0] * minv;
    uint32_t c = (uint32_t)(mad(m[0], u, a[0]) >> 32);
#pragma unroll
    for (int j = 1; j < L; ++j) {
      const uint64_t p = mad(m[j], u, (uint64_t)a[j] + c);
      a[j - 1] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    const uint64_t s = (uint64_t)top + c;
    a[L - 1] = (uint32_t)s;
    top = (uint32_t)(s >> 32);
  }
  const bool ge = top != 0 || geq<L>(a, m);
  csub<L>(a, m, ge);
}

// hi <- (hi:lo) * 2^(-32L) mod m for (hi:lo) < m * 2^(32L)   (lo is consumed)
template <int L>
__device__ __forceinline__ void redc_wide(uint32_t (&lo)[L], uint32_t (&hi)[L], const uint32_t* __restrict__ m,
                                          uint32_t minv) {
  // one Montgomery step per low limb: add u*m at offset i (the limb becomes 0), carries ripple
  // into hi; `over` collects the carry out of limb 2L-1 (bounded by 1).
  uint32_t over = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t u = lo[i] * minv;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int k = i + j;
      uint32_t& tk = k < L ? lo[k < L ? k : 0] : hi[k >= L ? k - L : 0];
      const uint64_t p = mad(m[j], u, (uint64_t)tk + c);
      tk = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    // carry lands on limb i + L (= hi[i]) and ripples up
#pragma unroll
    for (int k = i; k < L; ++k) {
      const uint64_t s = (uint64_t)hi[k] + c;
      hi[k] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    over += c;
  }
  const bool ge = over != 0 || geq<L>(hi, m);
  csub<L>(hi, m, ge);
}

}  // namespace big
}  // namespace efl
