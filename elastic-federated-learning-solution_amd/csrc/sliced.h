// Sliced multi-precision arithmetic: one big number spread over G lanes (C limbs per lane,
// L = C*G limbs), for moduli too wide for one lane's registers (n^2 of 2048- and 4096-bit keys).
//
// Lane g of a group holds limbs [g*C, (g+1)*C). Montgomery multiplication is CIOS with the
// accumulator sliced the same way: per outer step i every lane adds its C products a_j*b_i and
// u*m_j (u = t_0 * m' broadcast from lane 0 of the group), then the number shifts down one limb
// (lane g's new top limb is lane g+1's old bottom limb: one __shfl_down). The carry out of a
// lane's slice is not rippled into the next lane at every step: it stays "pending" at position
// (g+1)*C, which after the shift is exactly the lane's own new top limb, so it is added there
// without any cross-lane traffic. Pending carries are resolved once per multiplication
// (G-1 shuffle rounds), followed by the conditional subtraction of m.
//
// b operands are read with a per-element LDS broadcast (all G lanes read the same address) or from
// wave-uniform key constants; per-lane slices of the modulus stay in VGPRs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace efl {
namespace sl {

__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// Cross-lane moves inside aligned groups of G lanes. The two on every CIOS step (bcast0,
// from_next) are DPP moves (one VALU instruction, no LDS round trip) wherever one instruction
// does it; ds_bpermute (__shfl) otherwise. DPP controls (GFX9 encoding): quad_perm 0x00-0xFF,
// row_shl:1 0x101 (lane i <- i+1 in its 16-lane row), row_shr:1 0x111, row_shr:4 0x114,
// wave_shl:1 0x130, wave_shr:1 0x138, row_newbcast:0 0x150 (lane 0 of the row to the row).
template <int G>
__device__ __forceinline__ uint32_t bcast0(uint32_t v) {
  if constexpr (G == 1) {
    return v;
  } else if constexpr (G == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, false);   // quad_perm [0,0,2,2]
  } else if constexpr (G == 4) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);   // quad_perm [0,0,0,0]
  } else if constexpr (G == 8) {
    // lane 0 of every quad, then the upper quad of each 8-lane group (banks 1, 3) copies the
    // lower quad's value from 4 lanes down
    const int q = __builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(q, q, 0x114, 0xF, 0xA, false);
  } else if constexpr (G == 16) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150, 0xF, 0xF, false);  // row_newbcast:0
  } else {
    return __shfl(v, 0, G);
  }
}
// lane g <- lane g+1 (the caller zeroes lane G-1)
template <int G>
__device__ __forceinline__ uint32_t from_next(uint32_t v) {
  if constexpr (G == 1) return 0u;
  else if constexpr (G <= 16) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xF, 0xF, true);
  else if constexpr (G == 32) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
  else return __shfl_down(v, 1, G);
}
// lane g <- lane g-1 (the caller zeroes lane 0)
template <int G>
__device__ __forceinline__ uint32_t from_prev(uint32_t v) {
  if constexpr (G == 1) return 0u;
  else if constexpr (G <= 16) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
  else if constexpr (G == 32) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
  else return __shfl_up(v, 1, G);
}
template <int G>
__device__ __forceinline__ uint32_t from_lane(uint32_t v, int src) { return G == 1 ? v : __shfl(v, src, G); }

// element's number in LDS: limb i at base[i * E] (E = elements per workgroup), read by all G lanes
struct LdsElem {
  const uint32_t* base;
  int E;
  __device__ __forceinline__ uint32_t operator()(int i) const { return base[i * E]; }
};
struct Uniform {
  const uint32_t* __restrict__ p;
  __device__ __forceinline__ uint32_t operator()(int i) const { return p[i]; }
};

template <int C>
__device__ __forceinline__ void to_lds(uint32_t* base, int E, int g, const uint32_t (&x)[C]) {
#pragma unroll
  for (int j = 0; j < C; ++j) base[(g * C + j) * E] = x[j];
}

// lane's slice of a uniform number
template <int C>
__device__ __forceinline__ void slice_uniform(uint32_t (&x)[C], const uint32_t* __restrict__ p, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = p[g * C + j];
}

template <int C>
__device__ __forceinline__ void load_slice(uint32_t (&x)[C], const uint32_t* __restrict__ p, int g) {
  const uint32_t* q = p + g * C;
#pragma unroll
  for (int j = 0; j < C; j += 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(q + j);
    x[j] = v.x; x[j + 1] = v.y; x[j + 2] = v.z; x[j + 3] = v.w;
  }
}

template <int C>
__device__ __forceinline__ void store_slice(uint32_t* __restrict__ p, int g, const uint32_t (&x)[C]) {
  uint32_t* q = p + g * C;
#pragma unroll
  for (int j = 0; j < C; j += 4) *reinterpret_cast<uint4*>(q + j) = make_uint4(x[j], x[j + 1], x[j + 2], x[j + 3]);
}

// Resolve per-lane pending carries (carry = lane's carry into the next lane's limb 0). Returns
// the carry out of the whole number (valid in every lane).
template <int C, int G>
__device__ __forceinline__ uint32_t resolve_carries(uint32_t (&t)[C], uint32_t carry, int g) {
  uint32_t top = g == G - 1 ? carry : 0u;
  uint32_t out = g == G - 1 ? 0u : carry;
#pragma unroll
  for (int r = 0; r < G - 1; ++r) {
    uint32_t c = from_prev<G>(out);
    if (g == 0) c = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const uint64_t s = (uint64_t)t[j] + c;
      t[j] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    if (g == G - 1) { top += c; out = 0; }
    else out = c;
  }
  return from_lane<G>(top, G - 1);
}

// Resolve per-lane pending borrows (borrow = lane's borrow out of its slice). Returns the borrow
// out of the whole number (valid in every lane).
template <int C, int G>
__device__ __forceinline__ uint32_t resolve_borrows(uint32_t (&t)[C], uint32_t borrow, int g) {
  uint32_t top = g == G - 1 ? borrow : 0u;
  uint32_t out = g == G - 1 ? 0u : borrow;
#pragma unroll
  for (int r = 0; r < G - 1; ++r) {
    uint32_t b = from_prev<G>(out);
    if (g == 0) b = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const uint64_t d = (uint64_t)t[j] - b;
      t[j] = (uint32_t)d;
      b = (uint32_t)(d >> 63);
    }
    if (g == G - 1) { top += b; out = 0; }
    else out = b;
  }
  return from_lane<G>(top, G - 1);
}

// t += v (v at limb 0 of the number); returns the carry out of the number
template <int C, int G>
__device__ __forceinline__ uint32_t add_small(uint32_t (&t)[C], uint32_t v, int g) {
  uint32_t c = g == 0 ? v : 0u;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t s = (uint64_t)t[j] + c;
    t[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return resolve_carries<C, G>(t, c, g);
}

// t -= v; returns the borrow out of the number
template <int C, int G>
__device__ __forceinline__ uint32_t sub_small(uint32_t (&t)[C], uint32_t v, int g) {
  uint32_t b = g == 0 ? v : 0u;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t d = (uint64_t)t[j] - b;
    t[j] = (uint32_t)d;
    b = (uint32_t)(d >> 63);
  }
  return resolve_borrows<C, G>(t, b, g);
}

// t += x; returns the carry out
template <int C, int G>
__device__ __forceinline__ uint32_t add(uint32_t (&t)[C], const uint32_t (&x)[C], int g) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t s = (uint64_t)t[j] + x[j] + c;
    t[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return resolve_carries<C, G>(t, c, g);
}

// t -= x; returns the borrow out
template <int C, int G>
__device__ __forceinline__ uint32_t sub(uint32_t (&t)[C], const uint32_t (&x)[C], int g) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t d = (uint64_t)t[j] - x[j] - b;
    t[j] = (uint32_t)d;
    b = (uint32_t)(d >> 63);
  }
  return resolve_borrows<C, G>(t, b, g);
}

// t = x - t (x >= t)
template <int C, int G>
__device__ __forceinline__ void rsub(uint32_t (&t)[C], const uint32_t (&x)[C], int g) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t d = (uint64_t)x[j] - t[j] - b;
    t[j] = (uint32_t)d;
    b = (uint32_t)(d >> 63);
  }
  resolve_borrows<C, G>(t, b, g);
}

// the integer 1 as a b operand (Montgomery reduction: mont_mul(a, Unit) = a R^-1 mod m)
struct Unit {
  __device__ __forceinline__ uint32_t operator()(int i) const { return i == 0 ? 1u : 0u; }
};

// order this lane's LDS writes before the group's following reads (one wave per workgroup:
// LDS instructions of a wave execute in order, this only pins the compiler)
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x -= m if cond; borrow rippled across the group (m: lane slice). cond uniform per group.
template <int C, int G>
__device__ __forceinline__ void csub(uint32_t (&x)[C], const uint32_t (&m)[C], bool cond, int g) {
  // local subtract with borrow-in 0, then G-1 rounds of borrow propagation
  uint32_t d[C];
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t v = (uint64_t)x[j] - m[j] - b;
    d[j] = (uint32_t)v;
    b = (uint32_t)(v >> 63);
  }
  uint32_t out = g == G - 1 ? 0u : b;
#pragma unroll
  for (int r = 0; r < G - 1; ++r) {
    uint32_t bi = from_prev<G>(out);
    if (g == 0) bi = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const uint64_t v = (uint64_t)d[j] - bi;
      d[j] = (uint32_t)v;
      bi = (uint32_t)(v >> 63);
    }
    out = g == G - 1 ? 0u : bi;
  }
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = cond ? d[j] : x[j];
}

// x >= m (group-uniform answer)
template <int C, int G>
__device__ __forceinline__ bool geq(const uint32_t (&x)[C], const uint32_t (&m)[C], int g) {
  // per-lane compare of the slice: 1 greater, -1 less, 0 equal; the most significant lane with a
  // nonzero verdict decides
  int v = 0;
#pragma unroll
  for (int j = C - 1; j >= 0; --j)
    if (v == 0 && x[j] != m[j]) v = x[j] > m[j] ? 1 : -1;
  int decided = 0;
#pragma unroll
  for (int s = G - 1; s >= 0; --s) {
    const int vs = (int)from_lane<G>((uint32_t)v, s);
    if (decided == 0) decided = vs;
  }
  return decided >= 0;
}

// t += x * y over one slice; returns the carry word out of the slice. The C products
// x_j * y + t_j are independent 64-bit mads; only their high halves ripple, through a 32-bit
// add-with-carry chain (no 64-bit carry pairs to assemble).
template <int C>
__device__ __forceinline__ uint32_t row(uint32_t (&t)[C], const uint32_t (&x)[C], uint32_t y) {
  uint32_t prev_hi = 0, cf = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t p = (uint64_t)x[j] * y + t[j];
    uint32_t co;
    t[j] = __builtin_addc((uint32_t)p, prev_hi, cf, &co);
    cf = co;
    prev_hi = (uint32_t)(p >> 32);
  }
  return prev_hi + cf;   // t + x*y < 2^(32(C+1)): no overflow
}

// a <- a * b * 2^(-32L) mod m  (L = C*G; a, b < m). m: this lane's slice, minv = -m^-1 mod 2^32.
template <int C, int G, class B>
__device__ __forceinline__ void mont_mul(uint32_t (&a)[C], const B& b, const uint32_t (&m)[C], uint32_t minv,
                                         int g) {
  constexpr int L = C * G;
  uint32_t t[C];
#pragma unroll
  for (int j = 0; j < C; ++j) t[j] = 0;
  uint32_t pend = 0;
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    const uint32_t c1 = row<C>(t, a, b(i));
    const uint32_t u = bcast0<G>(t[0] * minv);
    const uint32_t c2 = row<C>(t, m, u);
    uint32_t in = from_next<G>(t[0]);
    if (g == G - 1) in = 0;
#pragma unroll
    for (int j = 0; j < C - 1; ++j) t[j] = t[j + 1];
    const uint64_t s = (uint64_t)in + pend + c1 + c2;
    t[C - 1] = (uint32_t)s;
    pend = (uint32_t)(s >> 32);
  }
  const uint32_t top = resolve_carries<C, G>(t, pend, g);
  const bool ge = top != 0 || geq<C, G>(t, m, g);
  csub<C, G>(t, m, ge, g);
#pragma unroll
  for (int j = 0; j < C; ++j) a[j] = t[j];
}

// a <- a^2 R^-1 mod m through the element's LDS scratch array
template <int C, int G>
__device__ __forceinline__ void mont_sqr(uint32_t (&a)[C], uint32_t* scratch, int E, const uint32_t (&m)[C],
                                         uint32_t minv, int g) {
  to_lds<C>(scratch, E, g, a);
  lds_sync();
  mont_mul<C, G>(a, LdsElem{scratch, E}, m, minv, g);
}

// a <- a R^-1 mod m (to normal form)
template <int C, int G>
__device__ __forceinline__ void redc(uint32_t (&a)[C], const uint32_t (&m)[C], uint32_t minv, int g) {
  mont_mul<C, G>(a, Unit{}, m, minv, g);
}

}  // namespace sl
}  // namespace efl
