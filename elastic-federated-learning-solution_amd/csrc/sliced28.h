// Radix-2^28 Montgomery arithmetic with lazy carries, sliced over G lanes (C28 limbs per lane),
// for the exponentiation loops of the Paillier kernels.
//
// Why: with 32-bit limbs every limb product needs v_mad_u64_u32 plus an add-with-carry, and the
// compiler re-zeroes the high half of each 64-bit addend (one v_mov per product): about three VALU
// instructions per product (csrc/sliced.h). With 28-bit limbs a product is < 2^56, so each limb
// position keeps a 64-bit accumulator and one CIOS step is just 2 C28 v_mad_u64_u32 whose addend
// IS the accumulator: no carry chain inside the step. Only the limb shifted out at the bottom
// passes its carry (>> 28) up. (32/28)^2 = 1.31x more products, about 2.5x fewer instructions.
//
// Bounds. Limbs of a and b are < 2^28, so one step adds < 2^57 to a position; a position
// accumulates for at most L steps before it leaves, so accumulators stay < 2 L 2^56 < 2^63 for
// L <= 64; longer numbers are carry-normalised every 64 steps (lazy_normalize). R = 2^(28 L) > 4 m
// (L = C28 G chosen so), so Montgomery products of inputs < 2m stay < 2m and no conditional
// subtraction is needed inside the exponentiation; redc of a value < 2m is fully reduced (< m).
//
// Layout: lane g of a group holds 28-bit limbs [g C28, (g+1) C28) of the number, each in the low
// bits of a 32-bit register; the b operand is read per limb from LDS (all G lanes read the same
// word) or from a wave-uniform constant, exactly as in sliced.h.
#pragma once

#include "sliced.h"

namespace efl {
namespace s28 {

// Unroll of the CIOS step loop for numbers sliced over G >= 2 lanes (build knob). Two steps per
// loop pass: same-box A/B (profiles/r02/ab_mont_unroll.jsonl) 1024-bit encrypt +2-4 %, 4096-bit
// encrypt +5 %, 4096-bit decrypt +2 %, MNIST matmul +1 %. G = 1 (the 1024-bit decryption's
// one-lane family) keeps one step per pass: unrolled, its register spills grew 191 -> 1087 VGPRs
// and it ran 7.6x slower.
#ifndef EFL_MONT28_UNROLL
#define EFL_MONT28_UNROLL 2
#endif

// Decryption squarings of numbers over G >= 2 lanes in the folded layout, symmetric (round 6; build
// knob for A/B: EFL_SQR_FOLD=0 builds the blocked CIOS squaring)
#ifndef EFL_SQR_FOLD
#define EFL_SQR_FOLD 0
#endif
// Decryption squarings of numbers over G = 2 or 4 lanes by separated operand scanning (round 6,
// sos_sqr; build knob for A/B: EFL_SQR_SOS=0 builds the blocked CIOS squaring)
#ifndef EFL_SQR_SOS
#define EFL_SQR_SOS 1
#endif
// One-lane squarings by product scanning (sqr_fips1) instead of CIOS through LDS (build knob for
// A/B: EFL_SQR_FIPS=0 builds the round-2 squaring)
#ifndef EFL_SQR_FIPS
#define EFL_SQR_FIPS 1
#endif
// One-lane multiplies by a register operand by product scanning (mul_fips1) in the fixed-base walks
// (build knob for A/B: EFL_MUL_FIPS=0 builds the CIOS loop through LDS)
#ifndef EFL_MUL_FIPS
#define EFL_MUL_FIPS 1
#endif

constexpr int kBits = 28;
constexpr uint32_t kMask = (1u << kBits) - 1;

// limbs needed for a modulus of `bits32 * 32` bits with R > 4 m, per lane of G
__host__ __device__ constexpr int limbs_per_lane(int L32, int G) { return ((32 * L32 + 2 + 27) / 28 + G - 1) / G; }

template <int G>
__device__ __forceinline__ uint64_t from_next64(uint64_t v) {
  const uint32_t lo = sl::from_next<G>((uint32_t)v);
  const uint32_t hi = sl::from_next<G>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int G>
__device__ __forceinline__ uint64_t from_prev64(uint64_t v) {
  const uint32_t lo = sl::from_prev<G>((uint32_t)v);
  const uint32_t hi = sl::from_prev<G>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Fold every accumulator's bits above 28 into the next position (the slice's top carry moves to
// the next lane's bottom position); values stay lazy (< 2^37) but far from overflow.
template <int C, int G>
__device__ __forceinline__ void lazy_normalize(uint64_t (&T)[C], int g) {
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t v = T[j] + c;
    T[j] = v & kMask;
    c = v >> kBits;
  }
  uint64_t in = from_prev64<G>(c);
  if (g == 0) in = 0;
  T[0] += in;   // the top lane's carry is 0: the number is < R
}

// Accumulators -> normalised 28-bit limbs (full carry ripple across the group).
template <int C, int G>
__device__ __forceinline__ void normalize(uint32_t (&a)[C], const uint64_t (&T)[C], int g) {
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t v = T[j] + c;
    a[j] = (uint32_t)v & kMask;
    c = v >> kBits;
  }
  // carry out of each slice into the next lane; ripples at most G-1 lanes
#pragma unroll
  for (int r = 0; r < G - 1; ++r) {
    uint64_t in = from_prev64<G>(c);
    if (g == 0) in = 0;
    c = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const uint64_t v = (uint64_t)a[j] + in;
      a[j] = (uint32_t)v & kMask;
      in = v >> kBits;
    }
    c = in;
  }
}

// a <- a b R^-1 mod m (lazy: inputs < 2m, output < 2m). m: this lane's slice; minv = -m^-1 mod 2^28.
template <int C, int G, class B>
__device__ __forceinline__ void mont_mul(uint32_t (&a)[C], const B& b, const uint32_t (&m)[C], uint32_t minv,
                                         int g) {
  constexpr int L = C * G;
  // one step per pass for one-lane numbers and for short slices (C < 32: the 128-VGPR decryption
  // families C = 8 / 16, where two steps per pass spilled 736-1,092 VGPRs into the loop)
  constexpr int kUnroll = (G == 1 || C < 32) ? 1 : EFL_MONT28_UNROLL;
  uint64_t T[C];
#pragma unroll
  for (int j = 0; j < C; ++j) T[j] = 0;
#pragma unroll kUnroll
  for (int i = 0; i < L; ++i) {
    const uint32_t bi = b(i);
#pragma unroll
    for (int j = 0; j < C; ++j) T[j] = (uint64_t)a[j] * bi + T[j];
    const uint32_t u = sl::bcast0<G>(((uint32_t)T[0] * minv) & kMask);
#pragma unroll
    for (int j = 0; j < C; ++j) T[j] = (uint64_t)m[j] * u + T[j];
    uint64_t in = from_next64<G>(T[0]);
    if (g == G - 1) in = 0;
    const uint64_t c0 = T[0] >> kBits;   // lane 0: the bottom limb is now 0 mod 2^28
#pragma unroll
    for (int j = 0; j < C - 1; ++j) T[j] = T[j + 1];
    T[C - 1] = in;
    if (g == 0) T[0] += c0;
    if (L > 64 && (i & 63) == 63) lazy_normalize<C, G>(T, g);
  }
  normalize<C, G>(a, T, g);
}

// a <- a b 2^(-28 steps) mod m for a b operand of only `steps` limbs (the rest zero): the first
// `steps` CIOS steps of mont_mul. Inputs a < 2m, b < 2^(28 steps): output < a b 2^(-28 steps) + m.
template <int C, int G, class B>
__device__ __forceinline__ void mont_mul_steps(uint32_t (&a)[C], const B& b, const uint32_t (&m)[C], uint32_t minv,
                                               int g, int steps) {
  uint64_t T[C];
#pragma unroll
  for (int j = 0; j < C; ++j) T[j] = 0;
  for (int i = 0; i < steps; ++i) {
    const uint32_t bi = b(i);
#pragma unroll
    for (int j = 0; j < C; ++j) T[j] = (uint64_t)a[j] * bi + T[j];
    const uint32_t u = sl::bcast0<G>(((uint32_t)T[0] * minv) & kMask);
#pragma unroll
    for (int j = 0; j < C; ++j) T[j] = (uint64_t)m[j] * u + T[j];
    uint64_t in = from_next64<G>(T[0]);
    if (g == G - 1) in = 0;
    const uint64_t c0 = T[0] >> kBits;
#pragma unroll
    for (int j = 0; j < C - 1; ++j) T[j] = T[j + 1];
    T[C - 1] = in;
    if (g == 0) T[0] += c0;
  }
  normalize<C, G>(a, T, g);
}

// a <- a^2 R^-1 mod m for a number held in ONE lane (G = 1: the 1024-bit key's decryption family,
// n^2 of 512-bit keys): finely integrated product scanning (Koc, Acar, Kaliski 1996, "FIPS").
// Column k of the square takes every cross product a_i a_j (i < j) once and doubles the column, and
// the reduction's u_i m_j terms land in the same column, so a squaring is C(C+1)/2 + C^2 limb
// products instead of CIOS's 2 C^2 (C = 37: 2,072 instead of 2,738), all from registers — no LDS
// operand, no accumulator array (two column accumulators and the u_i instead of C 64-bit ones).
// Bounds: a column holds at most C/2 doubled cross products, one diagonal, C reduction products and
// a carry < 2^36: < (2C + 2) 2^56 < 2^64 for C < 127. Output < 2m for input < 2m (R > 4m), as CIOS.
// u_k is known only once column k is complete; column k's own m_0 u_k is the last term added.
template <int C>
__device__ __forceinline__ void sqr_fips1(uint32_t (&a)[C], const uint32_t (&m)[C], uint32_t minv) {
  static_assert(C < 127, "column accumulator bound");
  uint32_t u[C];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * C - 1; ++k) {
    const int ilo = k < C ? 0 : k - C + 1;
    uint64_t x = 0, r0 = carry, r1 = 0;
#pragma unroll
    for (int i = ilo; i < k - i; ++i) x = (uint64_t)a[i] * a[k - i] + x;
#pragma unroll
    for (int i = ilo; i < k && i < C; ++i) {   // j = k - i in [1, C)
      if ((i & 1) == 0) r0 = (uint64_t)m[k - i] * u[i] + r0;
      else r1 = (uint64_t)m[k - i] * u[i] + r1;
    }
    uint64_t t = (x << 1) + r0 + r1;
    if ((k & 1) == 0) t = (uint64_t)a[k >> 1] * a[k >> 1] + t;
    if (k < C) {
      u[k] = ((uint32_t)t * minv) & kMask;
      t = (uint64_t)m[0] * u[k] + t;   // now 0 mod 2^28
    } else {
      a[k - C] = (uint32_t)t & kMask;  // limb k - C of the result; a_(k-C) is no longer read
    }
    carry = t >> kBits;
  }
  a[C - 1] = (uint32_t)carry;          // < 2^28: the result is < 2m < R
}

// a <- a b R^-1 mod m for numbers held in ONE lane, b in registers too (the fixed-base walk's table
// entry, loaded straight from HBM): product scanning as in sqr_fips1, without the symmetry. Column k
// takes a_i b_(k-i) and the reduction's u_i m_(k-i); 2 C^2 limb products like CIOS, but CIOS in one
// lane runs its steps as a loop whose 64-bit accumulator array shifts down one position per step (2 C
// register moves per 2 C products) and reads b_i from LDS; here the columns are unrolled, nothing
// moves, and nothing goes through LDS. Four accumulators per column (two chains of a b, two of
// m u) keep the dependent mads apart. Bounds as sqr_fips1: a column holds at most C products a b,
// C products m u and a carry < 2^36: < (2C + 1) 2^56 < 2^64 for C < 127; output < 2m for inputs
// < 2m (R > 4m). a_(k-C) is written once column k no longer reads it.
template <int C>
__device__ __forceinline__ void mul_fips1(uint32_t (&a)[C], const uint32_t (&b)[C], const uint32_t (&m)[C],
                                          uint32_t minv) {
  static_assert(C < 127, "column accumulator bound");
  uint32_t u[C];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * C - 1; ++k) {
    const int ilo = k < C ? 0 : k - C + 1;
    uint64_t x0 = carry, x1 = 0, r0 = 0, r1 = 0;
#pragma unroll
    for (int i = ilo; i <= k && i < C; ++i) {      // a_i b_(k-i), k - i in [0, C)
      if ((i & 1) == 0) x0 = (uint64_t)a[i] * b[k - i] + x0;
      else x1 = (uint64_t)a[i] * b[k - i] + x1;
    }
#pragma unroll
    for (int i = ilo; i < k && i < C; ++i) {       // u_i m_(k-i), k - i in [1, C)
      if ((i & 1) == 0) r0 = (uint64_t)m[k - i] * u[i] + r0;
      else r1 = (uint64_t)m[k - i] * u[i] + r1;
    }
    uint64_t t = x0 + x1 + r0 + r1;
    if (k < C) {
      u[k] = ((uint32_t)t * minv) & kMask;
      t = (uint64_t)m[0] * u[k] + t;   // now 0 mod 2^28
    } else {
      a[k - C] = (uint32_t)t & kMask;
    }
    carry = t >> kBits;
  }
  a[C - 1] = (uint32_t)carry;
}

// a <- a^2 R^-1 mod m through the element's LDS scratch array (limb i at scratch[i * E]); one-lane
// numbers square in registers (sqr_fips1)
template <int C, int G>
__device__ __forceinline__ void mont_sqr(uint32_t (&a)[C], uint32_t* scratch, int E, const uint32_t (&m)[C],
                                         uint32_t minv, int g) {
  if constexpr (G == 1 && EFL_SQR_FIPS) {
    sqr_fips1<C>(a, m, minv);
  } else {
    sl::to_lds<C>(scratch, E, g, a);
    sl::lds_sync();
    s28::mont_mul<C, G>(a, sl::LdsElem{scratch, E}, m, minv, g);
  }
}

// ---- folded layout and symmetric squaring (round 6; the G >= 2 decryption families) -----------
// Squaring by CIOS forms every cross product a_i a_j twice (steps i and j). Forming 2 a_i a_j once,
// at step min(i, j), and a_i^2 at step i gives every column c all its terms by step c, so the
// reduction digits u and the result are those of CIOS exactly (tools: the round-6 simulation in
// DESIGN.md §5). But in SIMD a step's products only shrink if the limbs at or above i are spread
// over the lanes: with the blocked layout (lane g: limbs g C .. g C + C - 1) the top lane stays busy
// until the last chunk and the square saves 1/(2G) of its products. FOLDED: lane g holds a low chunk
// (positions H1 g + j, j < H1 = ceil(C / 2)) and a high chunk (positions G H1 + H2 (G - 1 - g) + j,
// j < H2 = floor(C / 2)). While i is in the low half every lane's high chunk lies above i (all
// doubled products), the low slots of lanes past i's chunk are doubled, i's own slot single, the
// slots below zero; in the high half no low slot has products at all. A squaring then issues
// (L/2)(C + C) + (L/2)(H2 + C) limb products instead of 2 L C: 7/8 of CIOS's, the product half
// 3/4. The accumulator shift crosses chunks in position order: a low chunk's top takes the next
// lane's low bottom (lane G-1: its own high bottom), a high chunk's top the previous lane's high
// bottom (lane 0: zero), so a step moves two 64-bit values between lanes (from_next64,
// from_prev64). Bounds as mont_mul: a step adds < 2^57 (doubled product) + 2^56 (m u) to a
// position, < 2^64 over the 64 steps between lazy normalisations.
constexpr __host__ __device__ int fold_h1(int C) { return (C + 1) / 2; }
constexpr __host__ __device__ int fold_h2(int C) { return C / 2; }
// position of folded slot j (j < H1: low chunk; else high chunk) of lane g
template <int C, int G>
__device__ __forceinline__ int fold_pos(int g, int j) {
  constexpr int H1 = fold_h1(C), H2 = fold_h2(C);
  return j < H1 ? H1 * g + j : G * H1 + H2 * (G - 1 - g) + (j - H1);
}

template <int C, int G>
__device__ __forceinline__ void to_lds_folded(uint32_t* base, int E, int g, const uint32_t (&x)[C]) {
#pragma unroll
  for (int j = 0; j < C; ++j) base[fold_pos<C, G>(g, j) * E] = x[j];
}
template <int C, int G>
__device__ __forceinline__ void from_lds_folded(uint32_t (&x)[C], const uint32_t* base, int E, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = base[fold_pos<C, G>(g, j) * E];
}
template <int C, int G>
__device__ __forceinline__ void slice_uniform_folded(uint32_t (&x)[C], const uint32_t* __restrict__ p, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = p[fold_pos<C, G>(g, j)];
}

// accumulators (folded) -> normalised 28-bit limbs: the carry ripples through the 2G chunks in
// position order (low chunks of lanes 0 .. G-1, then the high chunks of lanes G-1 .. 0)
template <int C, int G>
__device__ __forceinline__ void normalize_folded(uint32_t (&a)[C], const uint64_t (&T)[C], int g) {
  constexpr int H1 = fold_h1(C);
  uint64_t cl = 0, ch = 0;
#pragma unroll
  for (int j = 0; j < H1; ++j) {
    const uint64_t v = T[j] + cl;
    a[j] = (uint32_t)v & kMask;
    cl = v >> kBits;
  }
#pragma unroll
  for (int j = H1; j < C; ++j) {
    const uint64_t v = T[j] + ch;
    a[j] = (uint32_t)v & kMask;
    ch = v >> kBits;
  }
  // 2G - 1 rounds carry a chunk's carry into the next chunk in position order
#pragma unroll
  for (int r = 0; r < 2 * G - 1; ++r) {
    uint64_t inl = from_prev64<G>(cl);
    if (g == 0) inl = 0;
    uint64_t inh = from_next64<G>(ch);
    if (g == G - 1) inh = cl;          // lane G-1's high chunk follows its own low chunk
#pragma unroll
    for (int j = 0; j < H1; ++j) {
      const uint64_t v = (uint64_t)a[j] + inl;
      a[j] = (uint32_t)v & kMask;
      inl = v >> kBits;
    }
#pragma unroll
    for (int j = H1; j < C; ++j) {
      const uint64_t v = (uint64_t)a[j] + inh;
      a[j] = (uint32_t)v & kMask;
      inh = v >> kBits;
    }
    cl = inl;
    ch = g == 0 ? 0 : inh;             // the top chunk's carry out is 0: the number is < R
  }
}

template <int C, int G>
__device__ __forceinline__ void lazy_normalize_folded(uint64_t (&T)[C], int g) {
  constexpr int H1 = fold_h1(C);
  uint64_t cl = 0, ch = 0;
#pragma unroll
  for (int j = 0; j < H1; ++j) {
    const uint64_t v = T[j] + cl;
    T[j] = v & kMask;
    cl = v >> kBits;
  }
#pragma unroll
  for (int j = H1; j < C; ++j) {
    const uint64_t v = T[j] + ch;
    T[j] = v & kMask;
    ch = v >> kBits;
  }
  uint64_t inl = from_prev64<G>(cl);
  if (g == 0) inl = 0;
  uint64_t inh = from_next64<G>(ch);
  if (g == G - 1) inh = cl;
  T[0] += inl;
  T[H1] += inh;                        // values stay lazy (< 2^37) but far from overflow
}

// one CIOS step in the folded layout: bi the step's b limb, mul the multipliers of the low and high
// slots (LOW = false: the low slots take no product), then the reduction and the shift. No lazy
// normalisation here: the callers normalise between chunks (a branch inside the unrolled steps
// split them into blocks, and the compiler then moved every accumulator each step)
template <int C, int G, bool LOW>
__device__ __forceinline__ void fold_step(uint64_t (&T)[C], const uint32_t (&mul)[C], uint32_t bi,
                                          const uint32_t (&m)[C], uint32_t minv, int g) {
  constexpr int H1 = fold_h1(C);
  if constexpr (LOW) {
#pragma unroll
    for (int j = 0; j < H1; ++j) T[j] = (uint64_t)mul[j] * bi + T[j];
  }
#pragma unroll
  for (int j = H1; j < C; ++j) T[j] = (uint64_t)mul[j] * bi + T[j];
  const uint32_t u = sl::bcast0<G>(((uint32_t)T[0] * minv) & kMask);
#pragma unroll
  for (int j = 0; j < C; ++j) T[j] = (uint64_t)m[j] * u + T[j];
  uint64_t nl = from_next64<G>(T[0]);
  nl = g == G - 1 ? T[H1] : nl;
  uint64_t nh = from_prev64<G>(T[H1]);
  nh = g == 0 ? 0ull : nh;
  const uint64_t c0 = g == 0 ? T[0] >> kBits : 0ull;   // lane 0: the bottom limb is now 0 mod 2^28
#pragma unroll
  for (int j = 0; j < H1 - 1; ++j) T[j] = T[j + 1];
  T[H1 - 1] = nl;
#pragma unroll
  for (int j = H1; j < C - 1; ++j) T[j] = T[j + 1];
  T[C - 1] = nh;
  T[0] += c0;
}

// The L steps of a folded product (SQ = false: mul = a, every product) or square (SQ: mul = 2 a,
// the diagonal halved when its step comes and the slot zeroed after it; the high half's steps skip
// the low slots, all zero by then). Steps run a chunk at a time, unrolled (the low accumulators'
// shift is a full rotation per chunk: no moves), and the accumulators are lazily normalised between
// chunks, before any position could have gone 64 steps without one.
template <int C, int G, bool SQ>
__device__ __forceinline__ void fold_pass(uint64_t (&T)[C], uint32_t (&mul)[C], const uint32_t* bl, int E,
                                          const uint32_t (&m)[C], uint32_t minv, int g) {
  constexpr int H1 = fold_h1(C), H2 = fold_h2(C), L = C * G;
  static_assert(H1 <= 64, "chunk longer than the lazy-normalisation bound");
  int since = 0;
#pragma unroll 1
  for (int c = 0; c < G; ++c) {        // i in the low chunk of lane c
#pragma unroll
    for (int s = 0; s < H1; ++s) {
      const uint32_t bi = bl[(c * H1 + s) * E];
      const bool diag = SQ && g == c;
      if constexpr (SQ) mul[s] = diag ? mul[s] >> 1 : mul[s];   // the diagonal a_i^2, once
      fold_step<C, G, true>(T, mul, bi, m, minv, g);
      if constexpr (SQ) mul[s] = diag ? 0u : mul[s];            // below every later step
    }
    since += H1;
    if (L > 64 && since + H1 > 64) {
      lazy_normalize_folded<C, G>(T, g);
      since = 0;
    }
  }
#pragma unroll 1
  for (int c = 0; c < G; ++c) {        // i in the high chunk of lane G - 1 - c
#pragma unroll
    for (int s = 0; s < H2; ++s) {
      const uint32_t bi = bl[(G * H1 + c * H2 + s) * E];
      const bool diag = SQ && g == G - 1 - c;
      if constexpr (SQ) mul[H1 + s] = diag ? mul[H1 + s] >> 1 : mul[H1 + s];
      fold_step<C, G, !SQ>(T, mul, bi, m, minv, g);   // a square's low slots are all zero here
      if constexpr (SQ) mul[H1 + s] = diag ? 0u : mul[H1 + s];
    }
    since += H2;
    if (L > 64 && since + H2 > 64) {
      lazy_normalize_folded<C, G>(T, g);
      since = 0;
    }
  }
}

// a <- a b R^-1 mod m with b limb i read from the element's LDS array bl (position order), or, sq
// set, a <- a^2 R^-1 mod m (a is first written to bl). The exponentiation calls it at one site for
// its squarings and multiplies alike.
template <int C, int G>
__device__ __forceinline__ void fold_mont(uint32_t (&a)[C], uint32_t* bl, int E, const uint32_t (&m)[C],
                                          uint32_t minv, int g, bool sq) {
  uint64_t T[C];
#pragma unroll
  for (int j = 0; j < C; ++j) T[j] = 0;
  uint32_t mul[C];
  if (sq) {
    to_lds_folded<C, G>(bl, E, g, a);
    sl::lds_sync();
#pragma unroll
    for (int j = 0; j < C; ++j) mul[j] = a[j] << 1;   // < 2^29
    fold_pass<C, G, true>(T, mul, bl, E, m, minv, g);
  } else {
#pragma unroll
    for (int j = 0; j < C; ++j) mul[j] = a[j];
    fold_pass<C, G, false>(T, mul, bl, E, m, minv, g);
  }
  normalize_folded<C, G>(a, T, g);
}

// the constant b of a folded product (a uniform number, or 1 for the conversion out) goes to the
// element's LDS array first, so every product runs through fold_mont
template <int C, int G, class B>
__device__ __forceinline__ void mont_mul_folded(uint32_t (&a)[C], const B& b, uint32_t* bl, int E,
                                                const uint32_t (&m)[C], uint32_t minv, int g) {
  sl::lds_sync();
  for (int i = g; i < C * G; i += G) bl[i * E] = b(i);
  sl::lds_sync();
  fold_mont<C, G>(a, bl, E, m, minv, g, false);
}

// the element's number in 32-bit words in LDS (word k at w32[k * E], L32 words) -> this lane's
// folded 28-bit limbs
template <int C, int G>
__device__ __forceinline__ void from_words_folded(uint32_t (&a)[C], const uint32_t* w32, int E, int L32, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int bit = kBits * fold_pos<C, G>(g, j);
    const int w = bit >> 5, sft = bit & 31;
    const uint32_t lo = w < L32 ? w32[w * E] : 0u;
    const uint32_t hi = w + 1 < L32 ? w32[(w + 1) * E] : 0u;
    a[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sft) & kMask;
  }
}

// The element's number in 32-bit words in LDS (word k at w32[k * E], L32 words) -> this lane's
// 28-bit limbs. Words past L32 read as 0.
template <int C>
__device__ __forceinline__ void from_words(uint32_t (&a)[C], const uint32_t* w32, int E, int L32, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int bit = kBits * (g * C + j);
    const int w = bit >> 5, s = bit & 31;
    const uint32_t lo = w < L32 ? w32[w * E] : 0u;
    const uint32_t hi = w + 1 < L32 ? w32[(w + 1) * E] : 0u;
    a[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> s) & kMask;
  }
}

// 28-bit limbs in LDS (limb k at l28[k * E], L28 limbs) -> this lane's C32 32-bit words.
template <int C32>
__device__ __forceinline__ void to_words(uint32_t (&w)[C32], const uint32_t* l28, int E, int L28, int g) {
#pragma unroll
  for (int j = 0; j < C32; ++j) {
    const int bit = 32 * (g * C32 + j);
    const int k = bit / kBits, s = bit % kBits;
    const uint64_t l0 = k < L28 ? l28[k * E] : 0u;
    const uint64_t l1 = k + 1 < L28 ? l28[(k + 1) * E] : 0u;
    const uint64_t l2 = k + 2 < L28 ? l28[(k + 2) * E] : 0u;
    w[j] = (uint32_t)((l0 | (l1 << kBits) | (l2 << (2 * kBits))) >> s);
  }
}


// ---- separated operand scanning squaring (round 6; the G = 2 / 4 decryption families) -------------
// a^2 R^-1 mod m for a number over G lanes (lane g: limbs g C .. g C + C - 1), in two phases.
// Phase 1 forms the square a^2 (2 L limbs) in the element's LDS words T (the decryption's two LDS
// arrays, contiguous: T[p] at T0[p * E]) as sub-products scanned by columns in registers, each
// column's 28-bit limb added with ds_add_u32. Lane g takes A_g^2 (symmetric: C (C + 1) / 2 products),
// the full cross product 2 A_g A_(g+1 mod G) (G = 4), and half the rows of one more cross pair (G = 4:
// the distance-2 pairs (0, 2), (1, 3); G = 2: the one pair (0, 1)), the partner chunks taken by
// DPP lane rotations: C (C + 1) / 2 + C^2 + C H products per lane at G = 4 (2,812 at C = 37) against
// CIOS's 2 L C = 10,952 for the whole product. Phase 2 is the reduction alone: L CIOS steps of
// C products m u over the lane-sliced window holding the low half, and then the high half added.
// Bounds: a column holds at most C products < 2^57 (cross rows doubled) and a carry < 2^36; a T word
// at most 7 limbs < 2^29 (< 2^32); the window adds < 2^56 per step, lazily normalised every 64
// steps, and stays < R. Output <= 2m for input <= 2m (R > 4m), which later products accept.
// tools/sos_sim.py simulates the same steps lane by lane against (x^2 + U m) / R.

// lane g <- lane (g + D) mod G inside aligned groups (G = 2: D = 1; G = 4: D = 1, 2)
template <int G, int D>
__device__ __forceinline__ uint32_t rot_lane(uint32_t v) {
  static_assert(G == 2 || G == 4, "rotations for pairs and quads");
  if constexpr (G == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
  else if constexpr (D == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x39, 0xF, 0xF, false);  // [1,2,3,0]
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
}

// x (R rows) times y (C limbs) by columns; COLS column limbs added to T[k * E] (the last takes the
// rest of the carry). A template recursion over the column K, so every column's row range and every
// register index is a compile-time constant (a loop nest with run-time bounds went to scratch)
template <int R, int C, int COLS, int K>
__device__ __forceinline__ void scan_col(const uint32_t (&x)[R], const uint32_t (&y)[C], uint32_t* T, int E,
                                         uint64_t carry) {
  if constexpr (K < COLS) {
    constexpr int rlo = K - C + 1 > 0 ? K - C + 1 : 0;
    constexpr int rhi = K < R - 1 ? K : R - 1;
    uint64_t x0 = carry, x1 = 0;
#pragma unroll
    for (int r = rlo; r <= rhi; ++r) {
      if ((r - rlo) & 1) x1 = (uint64_t)x[r] * y[K - r] + x1;
      else x0 = (uint64_t)x[r] * y[K - r] + x0;
    }
    const uint64_t acc = x0 + x1;
    if constexpr (K < COLS - 1) {
      atomicAdd(&T[K * E], (uint32_t)acc & kMask);
      scan_col<R, C, COLS, K + 1>(x, y, T, E, acc >> kBits);
    } else {
      atomicAdd(&T[K * E], (uint32_t)acc);
    }
  }
}
template <int R, int C, int COLS>
__device__ __forceinline__ void scan_add(const uint32_t (&x)[R], const uint32_t (&y)[C], uint32_t* T, int E) {
  scan_col<R, C, COLS, 0>(x, y, T, E, 0);
}

// a^2 by columns (each cross product once, doubled), 2 C column limbs added to T[k * E]
template <int C, int K>
__device__ __forceinline__ void sqr_col(const uint32_t (&a)[C], uint32_t* T, int E, uint64_t carry) {
  if constexpr (K < 2 * C) {
    constexpr int ilo = K - C + 1 > 0 ? K - C + 1 : 0;   // j = K - i < C
    constexpr int ihi = K >= 1 ? (K - 1) / 2 : -1;        // i < j (none in column 0)
    uint64_t x0 = 0, x1 = 0;
#pragma unroll
    for (int i = ilo; i <= ihi; ++i) {
      if ((i - ilo) & 1) x1 = (uint64_t)a[i] * a[K - i] + x1;
      else x0 = (uint64_t)a[i] * a[K - i] + x0;
    }
    uint64_t acc = ((x0 + x1) << 1) + carry;
    if constexpr ((K & 1) == 0 && (K >> 1) < C) acc = (uint64_t)a[K >> 1] * a[K >> 1] + acc;
    if constexpr (K < 2 * C - 1) {
      atomicAdd(&T[K * E], (uint32_t)acc & kMask);
      sqr_col<C, K + 1>(a, T, E, acc >> kBits);
    } else {
      atomicAdd(&T[K * E], (uint32_t)acc);
    }
  }
}
template <int C>
__device__ __forceinline__ void sqr_scan_add(const uint32_t (&a)[C], uint32_t* T, int E) {
  sqr_col<C, 0>(a, T, E, 0);
}

template <int C, int G>
__device__ __forceinline__ void sos_sqr(uint32_t (&a)[C], uint32_t* T, int E, const uint32_t (&m)[C], uint32_t minv,
                                        int g) {
  static_assert(G == 2 || G == 4, "SOS squaring for pairs and quads of lanes");
  constexpr int L = C * G, H = (C + 1) / 2;
#pragma unroll
  for (int j = 0; j < 2 * C; ++j) T[(g * 2 * C + j) * E] = 0u;
  sl::lds_sync();
  sqr_scan_add<C>(a, T + (2 * g * C) * E, E);
  uint32_t y[C], x[H];
  if constexpr (G == 4) {
    // the full cross product with the next lane's chunk, doubled
#pragma unroll
    for (int j = 0; j < C; ++j) y[j] = rot_lane<G, 1>(a[j]) << 1;
    const int off1 = (g + ((g + 1) & 3)) * C;
    scan_add<C, C, 2 * C + 1>(a, y, T + off1 * E, E);
    // half the rows of the distance-2 pair: g < 2 rows [0, H) of A_g against 2 A_(g+2); g >= 2 rows
    // [H, C) of A_(g-2) against 2 A_g
    uint32_t p2[C];
#pragma unroll
    for (int j = 0; j < C; ++j) p2[j] = rot_lane<G, 2>(a[j]);
    const bool lo = g < 2;
#pragma unroll
    for (int r = 0; r < H; ++r) x[r] = lo ? a[r] : (H + r < C ? p2[H + r] : 0u);
#pragma unroll
    for (int j = 0; j < C; ++j) y[j] = (lo ? p2[j] : a[j]) << 1;
    const int off2 = lo ? (2 * g + 2) * C : (2 * g - 2) * C + H;
    scan_add<H, C, H + C + 1>(x, y, T + off2 * E, E);
  } else {
    // the one pair (0, 1): lane 0 rows [0, H) of A_0, lane 1 rows [H, C) of A_0, against 2 A_1
    uint32_t p1[C];
#pragma unroll
    for (int j = 0; j < C; ++j) p1[j] = rot_lane<G, 1>(a[j]);
    const bool lo = g == 0;
#pragma unroll
    for (int r = 0; r < H; ++r) x[r] = lo ? a[r] : (H + r < C ? p1[H + r] : 0u);
#pragma unroll
    for (int j = 0; j < C; ++j) y[j] = (lo ? p1[j] : a[j]) << 1;
    const int off2 = lo ? C : C + H;
    scan_add<H, C, H + C + 1>(x, y, T + off2 * E, E);
  }
  sl::lds_sync();
  // phase 2: the low half's reduction over the lane-sliced window, then the high half added:
  // (T + U m) / R = T_hi + (T_lo + U m) / R (U depends on T_lo only; the window stays < R, so the
  // top lane takes nothing in, as in mont_mul)
  uint64_t W[C];
#pragma unroll
  for (int j = 0; j < C; ++j) W[j] = T[(g * C + j) * E];
#pragma unroll 2
  for (int i = 0; i < L; ++i) {
    const uint32_t u = sl::bcast0<G>(((uint32_t)W[0] * minv) & kMask);
#pragma unroll
    for (int j = 0; j < C; ++j) W[j] = (uint64_t)m[j] * u + W[j];
    uint64_t in = from_next64<G>(W[0]);
    if (g == G - 1) in = 0;
    const uint64_t c0 = W[0] >> kBits;   // lane 0: the bottom limb is now 0 mod 2^28
#pragma unroll
    for (int j = 0; j < C - 1; ++j) W[j] = W[j + 1];
    W[C - 1] = in;
    if (g == 0) W[0] += c0;
    if (L > 64 && (i & 63) == 63) lazy_normalize<C, G>(W, g);
  }
#pragma unroll
  for (int j = 0; j < C; ++j) W[j] += T[(L + g * C + j) * E];
  normalize<C, G>(a, W, g);
}

}  // namespace s28
}  // namespace efl
