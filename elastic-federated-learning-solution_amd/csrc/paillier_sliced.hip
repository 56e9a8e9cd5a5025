// Stage P, sliced kernels: the Paillier ops for moduli too wide for one lane (n^2 of 2048/4096-bit
// keys, p^2 of 4096-bit keys), and a lower-register alternative for 1024-bit keys.
//
// Reference: efls-train/cc/efl/math/paillier.cc — Encrypt :103-131, _Decrypt :296-312 with the
// m/h-functions :28-48, Add/MulScalar/MulExp2 :157-265, Matmul :941-1051; fixed-base powm
// gmp_utils.cc:107-144. Same algorithms, same outputs as paillier.hip's one-lane kernels (the
// parity tests run both); only the data placement differs.
//
// One 64-lane wave per workgroup, G = L/C lanes per element, E = 64/G elements per workgroup.
// Every element owns LDS arrays (limb i of array A at A[i*E]) for its b operands: squaring scratch,
// the exponentiation base, the fixed-base table entry, running products. All G lanes read the
// same word (broadcast); the E elements of the wave hit consecutive banks.
#include <atomic>
#include <type_traits>

#include "pl_common.h"
#include "sliced.h"
#include "sliced28.h"

namespace efl {
namespace pl {
namespace {

using namespace sl;

constexpr int kSlBlock = 64;

// lane's slice of a uniform number that has only `len` limbs (zero above)
template <int C>
__device__ __forceinline__ void slice_prefix(uint32_t (&x)[C], const uint32_t* __restrict__ p, int len, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = g * C + j < len ? p[g * C + j] : 0u;
}

template <int C>
__device__ __forceinline__ void from_lds(uint32_t (&x)[C], const uint32_t* base, int E, int g) {
#pragma unroll
  for (int j = 0; j < C; ++j) x[j] = base[(g * C + j) * E];
}

// the element's a (Philox stream, as paillier.hip's draw_a) into LDS; Philox blocks split over the group
template <int G>
__device__ __forceinline__ void draw_a(uint32_t* A, int E, int words, int a_bits, uint64_t seed, uint64_t ctr,
                                       int g) {
  const int rem = a_bits & 31;
  for (int b = g; b * 4 < words; b += G) {
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)b, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int w = b * 4 + j;
      if (w < words) A[w * E] = (w == words - 1 && rem) ? c[j] & ((1u << rem) - 1u) : c[j];
    }
  }
}

// g = 1 + |m| n, or n^2 + 1 - |m| n for m < 0 (= (1 + |m| n)^-1 mod n^2), sliced over L = 2 ln limbs
template <int C, int G>
__device__ __forceinline__ void make_g(uint32_t (&t)[C], long long m, const Key& k, const uint32_t (&n2)[C],
                                       int g) {
  const uint64_t a = m < 0 ? 0ull - (uint64_t)m : (uint64_t)m;
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
  uint32_t ns[C];
  slice_prefix<C>(ns, k.at(k.d.off_n), k.d.ln, g);
  uint32_t c0 = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint64_t p = mad(a0, ns[j], c0);
    t[j] = (uint32_t)p;
    c0 = (uint32_t)(p >> 32);
  }
  uint32_t c1 = 0;
#pragma unroll
  for (int j = 0; j < C - 1; ++j) {
    const uint64_t p = mad(a1, ns[j], (uint64_t)t[j + 1] + c1);
    t[j + 1] = (uint32_t)p;
    c1 = (uint32_t)(p >> 32);
  }
  const uint64_t top = mad(a1, ns[C - 1], c1);
  // spill of this slice into the next lane: limb 0 += c0 + lo(top), limb 1 += hi(top)
  uint32_t in0 = from_prev<G>(c0), in1 = from_prev<G>((uint32_t)top), in2 = from_prev<G>((uint32_t)(top >> 32));
  if (g == 0) in0 = in1 = in2 = 0;
  uint64_t s = (uint64_t)t[0] + in0 + in1;
  t[0] = (uint32_t)s;
  s = (uint64_t)t[1] + in2 + (s >> 32);
  t[1] = (uint32_t)s;
  uint32_t cc = (uint32_t)(s >> 32);
#pragma unroll
  for (int j = 2; j < C; ++j) {
    s = (uint64_t)t[j] + cc;
    t[j] = (uint32_t)s;
    cc = (uint32_t)(s >> 32);
  }
  resolve_carries<C, G>(t, cc, g);
  if (m < 0) rsub<C, G>(t, n2, g);
  add_small<C, G>(t, 1u, g);
}

// a -> a' (pl_common.h regroup_exponent) on the element's group leader, then every lane of the
// group sees it; returns a's bit length
__device__ __forceinline__ int regroup_shared(uint32_t* A, int E, int words, int gs, int g) {
  const int size = col_bit_length(A, E, words);
  if (gs > 1) {
    if (g == 0) regroup_exponent(A, E, size, gs, words);
    lds_sync();
  }
  return size;
}

// hs^(a') R mod n^2 through the fixed-base table (gmp_utils.cc:107-144; see paillier.hip)
template <int C, int G>
__device__ __forceinline__ void fbpowm_mont(uint32_t (&acc)[C], const Key& k, uint32_t* A, uint32_t* B, int E,
                                            int words, const uint32_t (&n2)[C], int g) {
  constexpr int L = C * G;
  const int size = regroup_shared(A, E, words, k.d.group_size, g);
  const int W = table_window(k.d);
  slice_uniform<C>(acc, k.at(k.d.off_n2_one), g);
  const uint32_t* table = k.at(k.d.off_table);
  const int cols = k.d.table_cols;
  for (int s = 0, row = 0; s < size; s += W, ++row) {
    const uint32_t idx = col_bits(A, E, s, size - s < W ? size - s : W, words);
    if (idx) {
      uint32_t ent[C];
      load_slice<C>(ent, table + ((int64_t)row * cols + (idx - 1)) * L, g);
      to_lds<C>(B, E, g, ent);
      lds_sync();
      mont_mul<C, G>(acc, LdsElem{B, E}, n2, k.d.n2_minv, g);
    }
  }
}

// Optional register cap (waves per SIMD) for the C = 16 / C = 32 kernels: build knob for tuning
// (EFL_SL_WAVES16 / EFL_SL_WAVES32); default: the compiler's choice.
#if defined(EFL_SL_WAVES16) && defined(EFL_SL_WAVES32)
#define SL_OCC __attribute__((amdgpu_waves_per_eu(C == 16 ? EFL_SL_WAVES16 : EFL_SL_WAVES32)))
#else
#define SL_OCC
#endif

// Minimum waves per SIMD for the decryption kernels with C <= 16 limbs per lane (caps their VGPRs
// at 512 / EFL_DEC_WAVES; C = 32 keeps 2 waves, it spills heavily below 256 VGPRs):
// the radix-2^28 exponentiation needs latency hiding across waves more than registers.
#ifndef EFL_DEC_WAVES
#define EFL_DEC_WAVES 4
#endif

// k_matmul28's waves per SIMD (build knobs EFL_MAT_WAVES16 / EFL_MAT_WAVES32) and whether its event
// loop loads the next multiply's operand while the current product runs (EFL_MAT_PREFETCH: C28
// more registers, so it pays only where the register cap leaves room)
#ifndef EFL_MAT_WAVES16
#define EFL_MAT_WAVES16 EFL_DEC_WAVES
#endif
#ifndef EFL_MAT_WAVES32
#define EFL_MAT_WAVES32 2
#endif
#ifndef EFL_WALK_PROBE
#define EFL_WALK_PROBE 0
#endif
#ifndef EFL_MAT_PREFETCH
#define EFL_MAT_PREFETCH 0
#endif

#define SL_ELEMENT(E_, G_)                                   \
  const int g = (int)threadIdx.x % (G_);                     \
  const int e = (int)threadIdx.x / (G_);                     \
  const long long i = (long long)blockIdx.x * (E_) + e;

// ------------------------------------------------------------------------------------------
template <int C, int G>
__global__ __launch_bounds__(kSlBlock) SL_OCC void k_encrypt(Key k, const long long* __restrict__ m,
                                                      const uint32_t* hsa, uint32_t* out, long long N,
                                                      uint64_t seed, long long ctr0, int hsa_mont) {
  constexpr int L = C * G, E = kSlBlock / G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + e;
  uint32_t* A = lds + L * E + e;
  uint32_t n2[C];
  slice_uniform<C>(n2, k.at(k.d.off_n2), g);
  const uint32_t minv = k.d.n2_minv;
  uint32_t c[C];
  if (hsa) {
    load_slice<C>(c, hsa + i * L, g);
    to_lds<C>(B, E, g, c);
    make_g<C, G>(c, m[i], k, n2, g);
    lds_sync();
    mont_mul<C, G>(c, LdsElem{B, E}, n2, minv, g);
    // hsa_mont: hsa is hsa R mod n^2 (efl_pl_crt_join), so the one product above is g hsa
    if (!hsa_mont) mont_mul<C, G>(c, Uniform{k.at(k.d.off_n2_r2)}, n2, minv, g);
  } else {
    draw_a<G>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + i), g);
    lds_sync();
    fbpowm_mont<C, G>(c, k, A, B, E, words, n2, g);
    to_lds<C>(B, E, g, c);
    make_g<C, G>(c, m[i], k, n2, g);
    lds_sync();
    mont_mul<C, G>(c, LdsElem{B, E}, n2, minv, g);
  }
  store_slice<C>(out + i * L, g, c);
}

template <int C, int G>
__global__ __launch_bounds__(kSlBlock) SL_OCC void k_fbpowm(Key k, const uint32_t* __restrict__ a_in,
                                                     uint32_t* __restrict__ out, long long N, uint64_t seed,
                                                     long long ctr0) {
  constexpr int L = C * G, E = kSlBlock / G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + e;
  uint32_t* A = lds + L * E + e;
  if (a_in) {
    for (int w = g; w < words; w += G) A[w * E] = a_in[i * words + w];
  } else {
    draw_a<G>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + i), g);
  }
  lds_sync();
  uint32_t n2[C], acc[C];
  slice_uniform<C>(n2, k.at(k.d.off_n2), g);
  fbpowm_mont<C, G>(acc, k, A, B, E, words, n2, g);
  redc<C, G>(acc, n2, k.d.n2_minv, g);
  store_slice<C>(out + i * L, g, acc);
}

// Waves per SIMD the one-lane (G = 1) walk kernels are compiled for (build knob for A/B): with the
// entry and the product-scanning multiply in registers (s28::mul_fips1) the walk takes about 200
// VGPRs at 2 waves
#ifndef EFL_WALK1_WAVES
#define EFL_WALK1_WAVES 2
#endif
// One-lane walks load the next non-zero window's entry while the current product runs (build knob
// for A/B: 0 loads each entry right before its product)
#ifndef EFL_WALK1_PREFETCH
#define EFL_WALK1_PREFETCH 1
#endif

// entry of table row `row`, column idx (1-based) for this lane's slice
template <int C28, int L28>
__device__ __forceinline__ const uint32_t* walk_entry(const uint32_t* table, int row, uint32_t idx, int cols, int g) {
#if EFL_WALK_PROBE   // latency probe build (tools/walk_probe.py): every product reads entry (0, 0), L2-resident
  return table + g * C28;
#else
  return table + ((int64_t)row * cols + (idx - 1)) * L28 + g * C28;
#endif
}

// hs^(a') mod n^2 through the radix-2^28 table (same lookup order as fbpowm_mont), result in
// NORMAL form as this lane's C 32-bit words. Scratch: B (entry / conversion, L28 words per element).
template <int C, int G>
__device__ __forceinline__ void fbpowm28_walk(uint32_t (&acc)[s28::limbs_per_lane(C * G, G)], const Key& k,
                                              uint32_t* A, uint32_t* B, int E, int words,
                                              const uint32_t (&m28)[s28::limbs_per_lane(C * G, G)], int g) {
  constexpr int L = C * G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  const int size = regroup_shared(A, E, words, k.d.group_size, g);
  const int W = table_window(k.d);
  const uint32_t minv28 = k.d.n2_minv28;
  const uint32_t* table = k.at(k.d.off_table28);
  const int cols = k.d.table_cols;
  if constexpr (G == 1 && EFL_MUL_FIPS && EFL_WALK1_PREFETCH) {
    // one lane holds the whole number (round 4): entries go straight into registers, and the next
    // non-zero window's entry is in flight while the current product runs
    int s = 0, row = 0;
    auto next_entry = [&]() -> const uint32_t* {
      for (; s < size; s += W, ++row) {
        const uint32_t idx = col_bits(A, E, s, size - s < W ? size - s : W, words);
        if (idx) {
          const uint32_t* e = walk_entry<C28, L28>(table, row, idx, cols, g);
          s += W;
          ++row;
          return e;
        }
      }
      return nullptr;
    };
    const uint32_t* cur = next_entry();
    uint32_t b[C28], nb[C28];
    if (cur) {
#pragma unroll
      for (int j = 0; j < C28; ++j) b[j] = cur[j];
    }
    while (cur) {
      const uint32_t* nxt = next_entry();
      if (nxt) {
#pragma unroll
        for (int j = 0; j < C28; ++j) nb[j] = nxt[j];
      }
      s28::mul_fips1<C28>(acc, b, m28, minv28);
      cur = nxt;
#pragma unroll
      for (int j = 0; j < C28; ++j) b[j] = nb[j];
    }
    return;
  }
  for (int s = 0, row = 0; s < size; s += W, ++row) {
    const uint32_t idx = col_bits(A, E, s, size - s < W ? size - s : W, words);
    if (idx) {
      const uint32_t* ent = walk_entry<C28, L28>(table, row, idx, cols, g);
      if constexpr (G == 1 && EFL_MUL_FIPS) {
        // one lane holds the whole number: the entry goes straight into registers (round 4)
        uint32_t b[C28];
#pragma unroll
        for (int j = 0; j < C28; ++j) b[j] = ent[j];
        s28::mul_fips1<C28>(acc, b, m28, minv28);
      } else {
#pragma unroll
        for (int j = 0; j < C28; ++j) B[(g * C28 + j) * E] = ent[j];
        lds_sync();
        s28::mont_mul<C28, G>(acc, LdsElem{B, E}, m28, minv28, g);
        lds_sync();
      }
    }
  }
}

// hs^(a') mod n^2 through the radix-2^28 table (gmp_utils.cc:107-144), as 32-bit words
template <int C, int G>
__device__ __forceinline__ void fbpowm28(uint32_t (&out)[C], const Key& k, uint32_t* A, uint32_t* B, int E,
                                         int words, int g, const uint32_t* start = nullptr) {
  constexpr int L = C * G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  if (start) {                                    // the element's own walk start (k_gstart28)
    constexpr int CP = (C28 + 3) & ~3;
#pragma unroll
    for (int j = 0; j < C28; ++j) acc[j] = start[g * CP + j];
  } else {
    slice_uniform<C28>(acc, k.at(k.d.off_n2_one28), g);
  }
  fbpowm28_walk<C, G>(acc, k, A, B, E, words, m28, g);
  s28::mont_mul<C28, G>(acc, Unit{}, m28, k.d.n2_minv28, g);   // hs^(a') mod n^2 (< n^2)
  lds_sync();
  to_lds<C28>(B, E, g, acc);
  lds_sync();
  s28::to_words<C>(out, B, E, L28, g);
  lds_sync();
}

template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? (G == 1 ? EFL_WALK1_WAVES : 2) : EFL_DEC_WAVES) void k_fbpowm28(Key k, const uint32_t* __restrict__ a_in,
                                                                         uint32_t* __restrict__ out, long long N,
                                                                         uint64_t seed, long long ctr0,
                                                                         const uint32_t* __restrict__ start) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int L28 = s28::limbs_per_lane(L, G) * G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + e;
  uint32_t* A = lds + L28 * E + e;
  if (a_in) {
    for (int w = g; w < words; w += G) A[w * E] = a_in[i * words + w];
  } else {
    draw_a<G>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + i), g);
  }
  lds_sync();
  uint32_t h[C];
  fbpowm28<C, G>(h, k, A, B, E, words, g, start ? start + (size_t)i * G * ((s28::limbs_per_lane(L, G) + 3) & ~3) : nullptr);
  store_slice<C>(out + i * L, g, h);
}

// |m|'s 28-bit limbs as a b operand (three steps cover |m| < 2^84)
struct MLimbs {
  unsigned long long v;
  __device__ __forceinline__ uint32_t operator()(int i) const {
    return i < 3 ? (uint32_t)(v >> (28 * i)) & s28::kMask : 0u;
  }
};

// The key owner's CRT walk mod x^2 (x = p or q, y the other prime) started from the element's own
// (y^2)^-1 g(m) instead of the key's fixed walk start: the walk (k_fbpowm28 with `start`) then gives
// (y^2)^-1 g(m) hs^(a') mod x^2, so the CRT join of the two walks (efl_pl_crt_join without a
// plaintext: q^2 yp + p^2 yq mod n^2) IS the ciphertext g(m) hs^(a') mod n^2 (paillier.cc:103-131),
// with no product mod n^2 left. This kernel makes the starts, in the walk's radix-2^28 Montgomery
// form, into scratch (a separate launch keeps the walk's registers as they are):
// g(m) mod x^2 = 1 + |m| n, or (1 + |m| n)^-1 = 1 - |m| n for m < 0 (n^2 = 0 mod x^2); |m| (n mod
// x^2) by three Montgomery steps against (n mod x^2) 2^84 (key constant off_gn28), one conditional
// subtraction, then one product by (y^2)^-1 R28^2 (off_gstart28) gives (y^2)^-1 g R28. About 1.1
// products per walk against the 32-bit product mod n^2 it replaces. m NULL: g = 1 (FixedBasePowm).
template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? (G == 1 ? EFL_WALK1_WAVES : 2) : EFL_DEC_WAVES) void k_gstart28(
    Key k, const long long* __restrict__ m, uint32_t* __restrict__ start, long long N) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* B = lds + e;
  const uint32_t minv28 = k.d.n2_minv28;
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const long long mi = m ? m[i] : 0;
  const unsigned long long am = mi < 0 ? 0ull - (unsigned long long)mi : (unsigned long long)mi;
  slice_uniform<C28>(acc, k.at(k.d.off_gn28), g);
  s28::mont_mul_steps<C28, G>(acc, MLimbs{am}, m28, minv28, g, 3);         // |m| (n mod x^2), < x^2 (1 + 2^-21)
  to_lds<C28>(B, E, g, acc);
  lds_sync();
  {
    uint32_t t[C], x2[C];
    s28::to_words<C>(t, B, E, L28, g);
    lds_sync();
    slice_uniform<C>(x2, k.at(k.d.off_n2), g);
    csub<C, G>(t, x2, geq<C, G>(t, x2, g), g);                              // < x^2
    if (mi < 0) rsub<C, G>(t, x2, g);                                        // x^2 - t
    add_small<C, G>(t, 1u, g);                                               // g(m) mod x^2 (<= x^2)
    to_lds<C>(B, E, g, t);
    lds_sync();
  }
  s28::from_words<C28>(acc, B, E, L, g);
  s28::mont_mul<C28, G>(acc, Uniform{k.at(k.d.off_gstart28)}, m28, minv28, g);   // (y^2)^-1 g R28
  constexpr int CP = (C28 + 3) & ~3;            // padded slices, as k_fbpowm28 reads them
#pragma unroll
  for (int j = 0; j < C28; ++j) start[(size_t)i * G * CP + g * CP + j] = acc[j];
}

template <int C, int G>
__global__ __launch_bounds__(kSlBlock) SL_OCC void k_add(Key k, const uint32_t* __restrict__ x,
                                                  const uint32_t* __restrict__ y, uint32_t* __restrict__ out,
                                                  long long N) {
  constexpr int L = C * G, E = kSlBlock / G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* B = lds + e;
  uint32_t n2[C], a[C];
  slice_uniform<C>(n2, k.at(k.d.off_n2), g);
  load_slice<C>(a, y + i * L, g);
  to_lds<C>(B, E, g, a);
  load_slice<C>(a, x + i * L, g);
  lds_sync();
  mont_mul<C, G>(a, LdsElem{B, E}, n2, k.d.n2_minv, g);
  mont_mul<C, G>(a, Uniform{k.at(k.d.off_n2_r2)}, n2, k.d.n2_minv, g);
  store_slice<C>(out + i * L, g, a);
}

// x^e mod n^2 with the per-element exponent of `xs` (pl_common.h: words, |int64| or 2^int64)
template <int C, int G, class XS>
__global__ __launch_bounds__(kSlBlock) SL_OCC void k_powm(Key k, const uint32_t* __restrict__ x, XS xs,
                                                   uint32_t* __restrict__ out, long long N,
                                                   unsigned long long* bad) {
  constexpr int L = C * G, E = kSlBlock / G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* BASE = lds + e;
  uint32_t* SCR = lds + L * E + e;
  const auto ex = xs.at(i);
  const int ebits = ex.ok ? ex.bits() : 0;
  uint32_t t[C];
  if (ebits == 0) {
#pragma unroll
    for (int j = 0; j < C; ++j) t[j] = (ex.ok && g == 0 && j == 0) ? 1u : 0u;
    store_slice<C>(out + i * L, g, t);
    if (!ex.ok && g == 0) atomicMin(bad, (unsigned long long)i);
    return;
  }
  uint32_t n2[C];
  slice_uniform<C>(n2, k.at(k.d.off_n2), g);
  const uint32_t minv = k.d.n2_minv;
  load_slice<C>(t, x + i * L, g);
  mont_mul<C, G>(t, Uniform{k.at(k.d.off_n2_r2)}, n2, minv, g);
  to_lds<C>(BASE, E, g, t);
#pragma unroll 1
  for (int b = ebits - 2; b >= 0; --b) {
    mont_sqr<C, G>(t, SCR, E, n2, minv, g);
    if (ex.bit(b)) mont_mul<C, G>(t, LdsElem{BASE, E}, n2, minv, g);
  }
  redc<C, G>(t, n2, minv, g);
  store_slice<C>(out + i * L, g, t);
}

// ---- radix-2^28 variants of powm / matmul (the family the radix-2^28 table was built for) ----

// this lane's 28-bit slice of x R28 mod n^2 from x in normal form (32-bit words in HBM); SCR scratch
template <int C, int G>
__device__ __forceinline__ void to_mont28(uint32_t (&t)[s28::limbs_per_lane(C * G, G)], const uint32_t* x,
                                          const Key& k, const uint32_t (&m28)[s28::limbs_per_lane(C * G, G)],
                                          uint32_t* SCR, int E, int g) {
  constexpr int L = C * G, C28 = s28::limbs_per_lane(L, G);
  uint32_t w[C];
  load_slice<C>(w, x, g);
  lds_sync();
  to_lds<C>(SCR, E, g, w);
  lds_sync();
  s28::from_words<C28>(t, SCR, E, L, g);
  lds_sync();
  s28::mont_mul<C28, G>(t, Uniform{k.at(k.d.off_n2_r2_28)}, m28, k.d.n2_minv28, g);
}

// normal form (< n^2) from a radix-2^28 Montgomery slice, stored as 32-bit words. The final
// reduction leaves a residue of 0 as either 0 or m (lazy bound <= m); with `m32` (the modulus in
// 32-bit words) an m is written as 0, as mpz_powm gives for a non-unit x (e.g. n^2 mod n^2).
template <int C, int G>
__device__ __forceinline__ void store_from_mont28(uint32_t* out, uint32_t (&t)[s28::limbs_per_lane(C * G, G)],
                                                  const uint32_t (&m28)[s28::limbs_per_lane(C * G, G)],
                                                  uint32_t minv28, uint32_t* SCR, int E, int g,
                                                  const uint32_t* m32 = nullptr) {
  constexpr int L = C * G, C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  s28::mont_mul<C28, G>(t, Unit{}, m28, minv28, g);
  lds_sync();
  to_lds<C28>(SCR, E, g, t);
  lds_sync();
  uint32_t w[C];
  s28::to_words<C>(w, SCR, E, L28, g);
  if (m32) {
    uint32_t m[C];
    slice_uniform<C>(m, m32, g);
    if (geq<C, G>(w, m, g)) {
#pragma unroll
      for (int j = 0; j < C; ++j) w[j] = 0u;
    }
  }
  store_slice<C>(out, g, w);
}

// PaillierEncrypt with fresh randomness through the radix-2^28 table: c = g(m) * hs^(a') mod n^2.
// The walk starts from g(m) R instead of R, so it leaves c R and one conversion out gives c: one
// radix-2^28 product (g -> g R) instead of round 1's two 32-bit-limb products after the walk, which
// also spilled at C = 32. Same-box A/B (profiles/r02/ab_encrypt_tail.jsonl): 1024-bit n +7 %
// encrypts/s; 4096-bit n 1.2-1.8 % slower, with the hot loop identical instruction for instruction
// (tools/isa_loops.py) and only its code placement moved — keeping the round-1 tail there in the
// same build measured slower still (-3 %).
template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? (G == 1 ? EFL_WALK1_WAVES : 2) : EFL_DEC_WAVES) void k_encrypt28(Key k, const long long* __restrict__ m,
                                                                          uint32_t* __restrict__ out, long long N,
                                                                          uint64_t seed, long long ctr0) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + e;
  uint32_t* A = lds + L28 * E + e;
  uint32_t m28[C28], acc[C28];
  {
    uint32_t n2[C], c[C];
    slice_uniform<C>(n2, k.at(k.d.off_n2), g);
    make_g<C, G>(c, m[i], k, n2, g);
    to_lds<C>(B, E, g, c);
  }
  lds_sync();
  s28::from_words<C28>(acc, B, E, L, g);
  lds_sync();
  // R^2 as the LDS operand, like a table entry
  slice_uniform<C28>(m28, k.at(k.d.off_n2_r2_28), g);
  to_lds<C28>(B, E, g, m28);
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  lds_sync();
  s28::mont_mul<C28, G>(acc, LdsElem{B, E}, m28, k.d.n2_minv28, g);   // g R
  lds_sync();
  draw_a<G>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + i), g);
  lds_sync();
  fbpowm28_walk<C, G>(acc, k, A, B, E, words, m28, g);                 // g hs^(a') R
  lds_sync();
  store_from_mont28<C, G>(out + i * L, acc, m28, k.d.n2_minv28, B, E, g);
}

template <int C, int G, class XS>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? 2 : EFL_DEC_WAVES) void k_powm28(Key k, const uint32_t* __restrict__ x,
                                                                       XS xs, uint32_t* __restrict__ out,
                                                                       long long N, unsigned long long* bad) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* BASE = lds + e;
  uint32_t* SCR = lds + L28 * E + e;
  const auto ex = xs.at(i);
  const int ebits = ex.ok ? ex.bits() : 0;
  if (ebits == 0) {
    uint32_t one[C];
#pragma unroll
    for (int j = 0; j < C; ++j) one[j] = (ex.ok && g == 0 && j == 0) ? 1u : 0u;
    store_slice<C>(out + i * L, g, one);
    if (!ex.ok && g == 0) atomicMin(bad, (unsigned long long)i);
    return;
  }
  uint32_t m28[C28], t[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  to_mont28<C, G>(t, x + i * L, k, m28, SCR, E, g);
  lds_sync();
  to_lds<C28>(BASE, E, g, t);
#pragma unroll 1
  for (int b = ebits - 2; b >= 0; --b) {
    s28::mont_sqr<C28, G>(t, SCR, E, m28, minv28, g);
    if (ex.bit(b)) s28::mont_mul<C28, G>(t, LdsElem{BASE, E}, m28, minv28, g);
  }
  store_from_mont28<C, G>(out + i * L, t, m28, minv28, SCR, E, g, k.at(k.d.off_n2));
}

// FixedPointTensor.__add__ (paillier.py:116-133) in one launch: z = x^(2^(xe - m)) y^(2^(ye - m))
// mod n^2, m = min(xe, ye). The reference shifts both sides with PaillierMulExp2 (one of the two
// shifts is 2^0) and multiplies them with PaillierAdd: three ops, each a pass over HBM. Here the
// side with the larger exponent is squared d = |xe - ye| times and multiplied by the other side
// once: d + 4 radix-2^28 products (two conversions in, one out) instead of d + 6 over three launches.
// d > kMaxShift -> z = 0 and the index into bad (the caller raises, like a MulExp2 shift past it).
template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? 2 : EFL_DEC_WAVES) void k_fxp_add28(
    Key k, const uint32_t* __restrict__ x, const long long* __restrict__ xe, const uint32_t* __restrict__ y,
    const long long* __restrict__ ye, uint32_t* __restrict__ out, long long N, unsigned long long* bad) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* BASE = lds + e;
  uint32_t* SCR = lds + L28 * E + e;
  const long long a = xe[i], b = ye[i];
  const bool shift_x = a > b;
  const uint64_t d = shift_x ? (uint64_t)a - (uint64_t)b : (uint64_t)b - (uint64_t)a;
  if (d > (uint64_t)kMaxShift) {
    uint32_t zero[C];
#pragma unroll
    for (int j = 0; j < C; ++j) zero[j] = 0u;
    store_slice<C>(out + i * L, g, zero);
    if (g == 0) atomicMin(bad, (unsigned long long)i);
    return;
  }
  const uint32_t* A = (shift_x ? x : y) + i * L;   // raised to 2^d
  const uint32_t* B = (shift_x ? y : x) + i * L;
  uint32_t m28[C28], t[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  to_mont28<C, G>(t, B, k, m28, SCR, E, g);        // B R
  lds_sync();
  to_lds<C28>(BASE, E, g, t);
  to_mont28<C, G>(t, A, k, m28, SCR, E, g);        // A R
#pragma unroll 1
  for (int s = 0; s < (int)d; ++s) s28::mont_sqr<C28, G>(t, SCR, E, m28, minv28, g);
  lds_sync();
  s28::mont_mul<C28, G>(t, LdsElem{BASE, E}, m28, minv28, g);   // A^(2^d) B R
  store_from_mont28<C, G>(out + i * L, t, m28, minv28, SCR, E, g, k.at(k.d.off_n2));
}

// ---- PaillierMatmul in radix 2^28: x converted once, then one multi-exponentiation per output ----
//
// Output (i, k) is prod_j x_ij^(|y_jk| 2^(d_ijk)) over the terms of each sign, d = xe + ye - min.
// Instead of one square-and-multiply per term (bits(|y|) - 1 + d squarings each), the terms of
// one sign share the squarings (Straus): from the top bit level down, square the product once,
// then multiply in every x_ij whose exponent has that bit. Squarings drop from sum_j (bits + d) to
// max_j (bits + d) per sign; multiplies stay popcount(|y|) per term (the first is a copy). x_ij R (radix 2^28) is
// computed once per x element (k_tomont28) instead of once per output, and read from HBM as the
// register operand of the multiply; the two running products are the LDS operand.
//
// Groups walk the outputs column by column (consecutive groups: consecutive rows, the same column
// of y), so the groups of a wave share every term's |y| and differ only through d; they also have
// the same number of multiplies (sum of popcount(|y|)), so their event lists are about equally long.

// padded radix-2^28 slice of one element in HBM: lane g's C28 limbs at [g * CP, g * CP + C28)
template <int C28>
constexpr int pad4() { return (C28 + 3) & ~3; }

template <int C28>
__device__ __forceinline__ void store28(uint32_t* __restrict__ q, const uint32_t (&t)[C28]) {
  constexpr int CP = pad4<C28>();
#pragma unroll
  for (int j = 0; j < CP; j += 4)
    *reinterpret_cast<uint4*>(q + j) = make_uint4(t[j], j + 1 < C28 ? t[j + 1] : 0u, j + 2 < C28 ? t[j + 2] : 0u,
                                                  j + 3 < C28 ? t[j + 3] : 0u);
}

// Windowed terms (round 2): every term's exponent |y| is cut right to left into windows of up to
// kMatWin bits that start at a 1 bit (a window (s, v): bits s .. s + kMatWin - 1 of |y|, v odd), so
// x^|y| = prod over its windows of (x^v)^(2^s). Each x element gets its odd powers x, x^3, ...,
// x^(2^kMatWin - 1) once (k_tomont28: 1 squaring + 2^(kMatWin-1) - 1 products, shared by all w
// outputs of its row), and a term costs one multiply per window instead of one per set bit:
// ~2-2.5 instead of ~5.5 for the 11-bit mantissas decrease_precision leaves.
#ifndef EFL_MAT_WIN
#define EFL_MAT_WIN 5   // 3 / 4 / 5 / 6: 31.4 / 29.7 / 27.2 / 27.5 ms (profiles/r02/matmul_window_sweep.json)
#endif
constexpr int kMatWin = EFL_MAT_WIN, kMatEntries = 1 << (kMatWin - 1);
// term splits of efl_pl_matmul: 0 = chosen per launch (run_matmul28), else a fixed power of two
// (efl_pl_tune(ln, 3, S))
std::atomic<int> g_mat_splits{0};

// window starts of |y| (bit s set = a window begins at bit s), right to left
__global__ __launch_bounds__(256) void k_wmask(const long long* __restrict__ ym, unsigned long long* __restrict__ wm,
                                               long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long y = ym[i];
  uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
  uint64_t mask = 0;
  int s = 0;
  while (ay >> s) {
    if ((ay >> s) & 1ull) {
      mask |= 1ull << s;
      s += kMatWin;
    } else {
      ++s;
    }
    if (s >= 64) break;
  }
  wm[i] = mask;
}

// Multiply schedules of k_matmul28, built ahead by k_mmevents (round 2). Scanning every term at
// every bit level inside k_matmul28 cost as much as the Montgomery products themselves: ~15 scan
// steps per event on the MNIST product, each a handful of dependent cached loads, and the wave
// waits for its slowest group (tools/matmul_probe.py, EFL_MAT_PROBE=1: the kernel without its
// products still took half its time). Here one lane per (output, split) runs that scan once and
// writes the multiplies in the order the product consumes them (bit level descending, terms
// ascending within a level) as 32-bit words: bits [0,16) j - j0, [16,21) odd-power entry, [21]
// negative term, [22,32) level. Word e of list l is at EV[e * NL + l] (a wave's lists side by side,
// so k_matmul28's per-event reads are coalesced). hdr[l] = {events, top level}; -1 events: the list
// does not fit (more than `cap` events, a level past 1023, a split wider than 2^16 terms) and
// k_matmul28 scans that output's terms itself as before. mnv[l] = the output's minimum exponent.
constexpr int kEvLevelShift = 22, kEvNegBit = 21;
constexpr long long kEvLevels = 1ll << (32 - kEvLevelShift);
static_assert(kMatWin <= 6, "odd-power entry must fit the event word's 5 bits");

// Levels below kEvHistLevels are sorted by a per-lane counting sort in LDS (two passes over the
// terms: count events per level, then place each at its level's next slot — the same order as the
// level-major scan, which stays as the path for higher levels).
constexpr int kEvBlock = 128, kEvHistLevels = 128;

__device__ __forceinline__ uint32_t ev_word(int jr, uint64_t ay, long long y, long long p, long long b) {
  const uint32_t ent = (uint32_t)(((ay >> p) & ((1ull << kMatWin) - 1ull)) >> 1);
  return (uint32_t)jr | (ent << 16) | ((y < 0 ? 1u : 0u) << kEvNegBit) | ((uint32_t)b << kEvLevelShift);
}

__global__ __launch_bounds__(kEvBlock) void k_mmevents(const long long* __restrict__ xe,
                                                       const long long* __restrict__ ym,
                                                       const long long* __restrict__ ye,
                                                       const unsigned long long* __restrict__ wmask, int u, int v,
                                                       int w, int S, int cap, uint32_t* __restrict__ EV,
                                                       int2* __restrict__ hdr, long long* __restrict__ mnv) {
  __shared__ uint32_t hist[kEvHistLevels * kEvBlock];   // level-major, lane-minor: conflict-free
  const long long UW = (long long)u * w, NL = UW * S;
  const long long l = (long long)blockIdx.x * kEvBlock + threadIdx.x;
  if (l >= NL) return;
  const int sp = (int)(l / UW);
  const int row = (int)(l % UW % u), kk = (int)(l % UW / u);
  const long long* xr = xe + (long long)row * v;
  const long long* yc = ym + kk;
  const long long* ec = ye + kk;
  const unsigned long long* wc = wmask + kk;
  long long mn = 0x7FFFFFFFFFFFFFFFll;
  for (int j = 0; j < v; ++j) {
    const long long ex = xr[j] + ec[(long long)j * w];
    mn = ex < mn ? ex : mn;
  }
  mnv[l] = mn;
  const int j0 = (int)((long long)v * sp / S), j1 = (int)((long long)v * (sp + 1) / S);
  long long top = 0;
  for (int j = j0; j < j1; ++j) {
    const long long y = yc[(long long)j * w];
    if (y == 0) continue;
    const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
    const long long lvl = xr[j] + ec[(long long)j * w] - mn + (64 - __clzll((long long)ay));
    top = lvl > top ? lvl : top;
  }
  int cnt = 0;
  bool ok = j1 - j0 <= 65536 && top <= kEvLevels;
  if (ok && top <= kEvHistLevels) {
    uint32_t* H = hist + threadIdx.x;
    for (int lv = 0; lv < (int)top; ++lv) H[lv * kEvBlock] = 0;
    for (int j = j0; j < j1; ++j) {
      const int d = (int)(xr[j] + ec[(long long)j * w] - mn);
      for (unsigned long long m = wc[(long long)j * w]; m; m &= m - 1) H[(d + __ffsll((long long)m) - 1) * kEvBlock]++;
    }
    uint32_t run = 0;   // exclusive offsets, top level first
    for (int lv = (int)top - 1; lv >= 0; --lv) {
      const uint32_t c = H[lv * kEvBlock];
      H[lv * kEvBlock] = run;
      run += c;
    }
    ok = run <= (uint32_t)cap;
    if (ok) {
      cnt = (int)run;
      for (int j = j0; j < j1; ++j) {
        const long long y = yc[(long long)j * w];
        const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
        const int d = (int)(xr[j] + ec[(long long)j * w] - mn);
        for (unsigned long long m = wc[(long long)j * w]; m; m &= m - 1) {
          const int p = __ffsll((long long)m) - 1;
          const uint32_t pos = H[(d + p) * kEvBlock]++;
          EV[(long long)pos * NL + l] = ev_word(j - j0, ay, y, p, d + p);
        }
      }
    }
  } else {
    for (long long b = top - 1; ok && b >= 0; --b) {
      for (int j = j0; j < j1; ++j) {
        const long long p = b - (xr[j] + ec[(long long)j * w] - mn);
        if (p >= 0 && p < 64 && ((wc[(long long)j * w] >> p) & 1ull)) {
          if (cnt == cap) {
            ok = false;
            break;
          }
          const long long y = yc[(long long)j * w];
          const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
          EV[(long long)cnt * NL + l] = ev_word(j - j0, ay, y, p, b);
          ++cnt;
        }
      }
    }
  }
  hdr[l] = make_int2(ok ? cnt : -1, ok ? (int)top : 0);
}

// x R mod n^2 and its odd powers (radix 2^28, Montgomery) for every x element (row r, term j of
// x [u, v]): entry e at Xm + mat_slot(j, e, r, u) * (CP * G), lane g's slice at + g * CP. Term-major,
// then entry, then row: a k_matmul28 wave's groups are consecutive rows of one output column, so at
// one event they read the same (term, entry) of consecutive rows — one contiguous span (round 2's
// row-major [r][j][e] put consecutive rows v * 16 slots, 2 MB at the MNIST shape, apart).
__device__ __forceinline__ long long mat_slot(long long j, int e, long long r, long long u) {
  return (j * kMatEntries + e) * u + r;
}

template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? 2 : EFL_DEC_WAVES) void k_tomont28(Key k, const uint32_t* __restrict__ X,
                                                                         uint32_t* __restrict__ Xm, long long N,
                                                                         int u, int v) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G, CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* B = lds + e;
  uint32_t* SCR = lds + L28 * E + e;
  uint32_t m28[C28], t[C28], x2[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  to_mont28<C, G>(t, X + i * L, k, m28, B, E, g);
  const long long r = i / v, jt = i % v;
  uint32_t* q = Xm + mat_slot(jt, 0, r, u) * (CP * G) + g * CP;
  const long long estride = (long long)u * (CP * G);   // entry e + 1 of the same element
  store28<C28>(q, t);
#pragma unroll
  for (int j = 0; j < C28; ++j) x2[j] = t[j];
  lds_sync();
  s28::mont_sqr<C28, G>(x2, SCR, E, m28, minv28, g);
  lds_sync();
  to_lds<C28>(B, E, g, x2);
  lds_sync();
#pragma unroll 1
  for (int e2 = 1; e2 < kMatEntries; ++e2) {
    s28::mont_mul<C28, G>(t, LdsElem{B, E}, m28, minv28, g);
    store28<C28>(q + (long long)e2 * estride, t);
  }
}

template <int C28>
__device__ __forceinline__ void load28(uint32_t (&t)[C28], const uint32_t* __restrict__ q) {
  constexpr int CP = pad4<C28>();
#pragma unroll
  for (int j = 0; j < CP; j += 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(q + j);
    t[j] = v.x;
    if (j + 1 < C28) t[j + 1] = v.y;
    if (j + 2 < C28) t[j + 2] = v.z;
    if (j + 3 < C28) t[j + 3] = v.w;
  }
}

// ---- row-split walks (round 5) -------------------------------------------------------------------
// A launch of W waves keeps every SIMD busy only when W is close to a multiple of the SIMD count:
// the paillier_mnist activation ([256, 392] = 100,352 elements, 1,568 one-lane waves on 1,024 SIMDs)
// leaves 480 SIMDs with one wave and 544 with two, so the launch lasts as long as two waves for 1.53
// waves of work (0.77). Splitting every element's fixed-base walk into P parts over disjoint ranges of
// table rows (P x the waves, each doing 1/P of the work) evens that out, e.g. 4.59 -> 5 waves per SIMD
// for P = 3 (0.92). Parts start from their first non-zero window's entry instead of the Montgomery
// one, so the P - 1 products of the join cost nothing extra; an encryption's join then multiplies
// the product (x R) by g(m) in normal form, which gives the ciphertext x g with no conversion, two
// products fewer than k_encrypt28 (g -> g R, and the conversion out). Same value, bit for bit: a
// product mod m does not depend on its grouping, and every part's lazy result (< 2m) is a valid
// Montgomery operand.

// the walk over table rows [r0, r1) of a' (regrouped, `size` bits) into acc; `have` = acc already
// holds a factor (the walk start, or g R); otherwise the first non-zero window's entry becomes acc.
// Returns whether acc holds a factor afterwards.
template <int C, int G>
__device__ __forceinline__ bool walk28_rows(uint32_t (&acc)[s28::limbs_per_lane(C * G, G)], const Key& k, const uint32_t* A,
                                            uint32_t* B, int E, int words, int size,
                                            const uint32_t (&m28)[s28::limbs_per_lane(C * G, G)], int g, int r0, int r1,
                                            bool have) {
  constexpr int L = C * G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  const int W = table_window(k.d);
  const uint32_t minv28 = k.d.n2_minv28;
  const uint32_t* table = k.at(k.d.off_table28);
  const int cols = k.d.table_cols;
  const int end = r1 * W < size ? r1 * W : size;
  int s = r0 * W, row = r0;
  auto next_entry = [&]() -> const uint32_t* {
    for (; s < end; s += W, ++row) {
      const uint32_t idx = col_bits(A, E, s, end - s < W ? end - s : W, words);
      if (idx) {
        const uint32_t* e = walk_entry<C28, L28>(table, row, idx, cols, g);
        s += W;
        ++row;
        return e;
      }
    }
    return nullptr;
  };
  const uint32_t* cur = next_entry();
  if constexpr (G == 1 && EFL_MUL_FIPS) {
    // as fbpowm28_walk's one-lane loop: the entry goes into registers, the next one is in flight
    // during the product
    uint32_t b[C28], nb[C28];
    if (cur) {
#pragma unroll
      for (int j = 0; j < C28; ++j) b[j] = cur[j];
    }
    if (!have) {
      if (!cur) return false;
#pragma unroll
      for (int j = 0; j < C28; ++j) acc[j] = b[j];
      cur = next_entry();
      if (cur) {
#pragma unroll
        for (int j = 0; j < C28; ++j) b[j] = cur[j];
      }
    }
    while (cur) {
      const uint32_t* nxt = next_entry();
      if (nxt) {
#pragma unroll
        for (int j = 0; j < C28; ++j) nb[j] = nxt[j];
      }
      s28::mul_fips1<C28>(acc, b, m28, minv28);
      cur = nxt;
#pragma unroll
      for (int j = 0; j < C28; ++j) b[j] = nb[j];
    }
  } else {
    if (!have) {
      if (!cur) return false;
#pragma unroll
      for (int j = 0; j < C28; ++j) acc[j] = cur[j];
      cur = next_entry();
    }
    while (cur) {
#pragma unroll
      for (int j = 0; j < C28; ++j) B[(g * C28 + j) * E] = cur[j];
      lds_sync();
      s28::mont_mul<C28, G>(acc, LdsElem{B, E}, m28, minv28, g);
      lds_sync();
      cur = next_entry();
    }
  }
  return true;
}

// part p of element i (virtual element v = p N + i): the product of its rows' entries in radix-2^28
// Montgomery form into P (padded slices, store28 layout), and whether it holds anything into F.
// FROM_START (efl_pl_fbpowm): part 0 starts from the key's walk start (off_n2_one28, the CRT
// sub-keys' R (q^2)^-1); otherwise (PaillierEncrypt) every part starts from its first entry and the
// join brings in g(m).
template <int C, int G, bool FROM_START>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? (G == 1 ? EFL_WALK1_WAVES : 2) : EFL_DEC_WAVES) void k_walk28_part(
    Key k, const uint32_t* __restrict__ a_in, uint32_t* __restrict__ P, unsigned char* __restrict__ F, long long N,
    int parts, uint64_t seed, long long ctr0) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G, CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N * parts) return;
  const long long v = i;
  const int part = (int)(v / N);
  const long long el = v - (long long)part * N;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + e;
  uint32_t* A = lds + L28 * E + e;
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  bool have = false;
  if (FROM_START && part == 0) {
    slice_uniform<C28>(acc, k.at(k.d.off_n2_one28), g);
    have = true;
  }
  if (a_in) {
    for (int w = g; w < words; w += G) A[w * E] = a_in[el * words + w];
  } else {
    draw_a<G>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + el), g);
  }
  lds_sync();
  const int size = regroup_shared(A, E, words, k.d.group_size, g);
  const int rows = k.d.table_rows;
  const int r0 = (int)((long long)rows * part / parts), r1 = (int)((long long)rows * (part + 1) / parts);
  have = walk28_rows<C, G>(acc, k, A, B, E, words, size, m28, g, r0, r1, have);
  store28<C28>(P + (size_t)v * G * CP + g * CP, acc);
  if (g == 0) F[v] = have ? 1 : 0;
}

// the join: element i's parts multiplied (parts without a factor skipped). m NULL (efl_pl_fbpowm):
// then out of Montgomery form, as k_fbpowm28 writes it. m given (PaillierEncrypt): the product (x R)
// times g(m) in normal form is x g, the ciphertext, with one conditional subtraction of n^2 (the
// walk's lazy bound is 2 n^2) and no conversion; no factor at all (a' = 0) leaves g(m) itself.
template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? (G == 1 ? EFL_WALK1_WAVES : 2) : EFL_DEC_WAVES) void k_walk28_join(
    Key k, const long long* __restrict__ m, const uint32_t* __restrict__ P, const unsigned char* __restrict__ F,
    uint32_t* __restrict__ out, long long N, int parts) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G, CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* B = lds + e;
  uint32_t* GW = lds + L28 * E + e;        // g(m) as 32-bit words, made before the products
  if (m) {
    uint32_t c[C], n2[C];
    slice_uniform<C>(n2, k.at(k.d.off_n2), g);
    make_g<C, G>(c, m[i], k, n2, g);
    to_lds<C>(GW, E, g, c);
    lds_sync();
  }
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  bool any = false;
  for (int p = 0; p < parts; ++p) {
    const long long v = (long long)p * N + i;
    if (!F[v]) continue;
    if (!any) {
      load28<C28>(acc, P + (size_t)v * G * CP + g * CP);
      any = true;
      continue;
    }
    uint32_t b[C28];
    load28<C28>(b, P + (size_t)v * G * CP + g * CP);
    if constexpr (G == 1 && EFL_MUL_FIPS) {
      s28::mul_fips1<C28>(acc, b, m28, minv28);
    } else {
      to_lds<C28>(B, E, g, b);
      lds_sync();
      s28::mont_mul<C28, G>(acc, LdsElem{B, E}, m28, minv28, g);
      lds_sync();
    }
  }
  if (!m) {
    store_from_mont28<C, G>(out + i * L, acc, m28, minv28, B, E, g);   // part 0 always holds a factor
    return;
  }
  uint32_t c[C];
  if (!any) {
    from_lds<C>(c, GW, E, g);              // a' = 0: the ciphertext is g(m)
  } else {
    uint32_t gb[C28];
    s28::from_words<C28>(gb, GW, E, L, g);
    lds_sync();
    if constexpr (G == 1 && EFL_MUL_FIPS) {
      s28::mul_fips1<C28>(acc, gb, m28, minv28);
    } else {
      to_lds<C28>(B, E, g, gb);
      lds_sync();
      s28::mont_mul<C28, G>(acc, LdsElem{B, E}, m28, minv28, g);
      lds_sync();
    }
    to_lds<C28>(B, E, g, acc);
    lds_sync();
    s28::to_words<C>(c, B, E, L28, g);
    lds_sync();
    uint32_t n2[C];
    slice_uniform<C>(n2, k.at(k.d.off_n2), g);
    csub<C, G>(c, n2, geq<C, G>(c, n2, g), g);
  }
  store_slice<C>(out + i * L, g, c);
}


template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? EFL_MAT_WAVES32 : EFL_MAT_WAVES16) void k_matmul28(
    Key k, const uint32_t* __restrict__ Xm, const long long* __restrict__ xe, const long long* __restrict__ ym,
    const long long* __restrict__ ye, uint32_t* __restrict__ zpos, uint32_t* __restrict__ zneg,
    long long* __restrict__ ze, int u, int v, int w, int S, uint32_t* __restrict__ P,
    const unsigned long long* __restrict__ wmask, const uint32_t* __restrict__ EV, const int2* __restrict__ hdr,
    const long long* __restrict__ mnv) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G, CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  const long long UW = (long long)u * w, NL = UW * S;
  if (i >= NL) return;
  const int sp = (int)(i / UW);                      // split of the terms this group takes
  const int row = (int)(i % UW % u), kk = (int)(i % UW / u);
  const long long o = (long long)row * w + kk;
  uint32_t* ACC[2] = {lds + e, lds + L28 * E + e};   // running products: y > 0, y < 0
  uint32_t m28[C28], t[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  const long long* xr = xe + (long long)row * v;
  const long long* yc = ym + kk;
  const long long* ec = ye + kk;
  const unsigned long long* wc = wmask + kk;
  const long long mn = mnv[i];                       // min over j of xe_ij + ye_jk (k_mmevents)
  // this split's terms [j0, j1); top bit level of any of their exponents |y| 2^d
  const int j0 = (int)((long long)v * sp / S), j1 = (int)((long long)v * (sp + 1) / S);
  const int2 h = hdr[i];
  const bool listed = h.x >= 0;                      // k_mmevents wrote this group's multiplies
  long long top = h.y;
  if (!listed) {
    top = 0;
    for (int j = j0; j < j1; ++j) {
      const long long y = yc[(long long)j * w];
      if (y == 0) continue;
      const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
      const long long lvl = xr[j] + ec[(long long)j * w] - mn + (64 - __clzll((long long)ay));
      top = lvl > top ? lvl : top;
    }
  }
  // Each group walks its own event list: per bit level from the top, a squaring of each started
  // product, then one multiply per term with a window starting at that level (by the term's odd
  // power x^v, v the window's value). Every pass of the loop below is one Montgomery product per
  // group (its first operand from LDS for a squaring, from HBM for a multiply), so a wave runs
  // max_group(events) products, not the union of its groups' levels.
  bool started0 = false, started1 = false;   // products still 1 take their first term as a copy
  long long b = top - 1;
  int j = 0, phase = 0;                      // phase 0: square POS, 1: square NEG, 2: terms
  // listed groups: the next multiply word, read one event ahead (it arrives while a product runs)
  int ev_i = 0;
  uint32_t ev = listed && h.x > 0 ? EV[i] : 0u;
  // The next event of this group's list: op 0/1 square POS/NEG, 2/3 multiply x_j^v into POS/NEG,
  // -1 at the end; `addr` = the multiply's operand in Xm, `copy` = it is its product's first term
  // (a product counts as started once its first multiply has been scanned).
  auto next = [&](int& op, long long& addr, bool& copy) {
    op = -1;
    copy = false;
    while (op < 0 && b >= 0) {
      if (phase == 0) {
        phase = 1;
        if (started0) op = 0;
      } else if (phase == 1) {
        phase = 2;
        j = j0;
        if (started1) op = 1;
      } else if (listed) {
        if (ev_i < h.x && (long long)(ev >> kEvLevelShift) == b) {
          const int ent = (int)((ev >> 16) & 31u);
          addr = mat_slot(j0 + (int)(ev & 0xFFFFu), ent, row, u) * (CP * G) + g * CP;
          if ((ev >> kEvNegBit) & 1u) {
            op = 3;
            copy = !started1;
            started1 = true;
          } else {
            op = 2;
            copy = !started0;
            started0 = true;
          }
          if (++ev_i < h.x) ev = EV[(long long)ev_i * NL + i];
        } else {
          --b;
          phase = 0;
        }
      } else if (j >= j1) {
        --b;
        phase = 0;
      } else {
        const long long p = b - (xr[j] + ec[(long long)j * w] - mn);
        if (p >= 0 && p < 64 && ((wc[(long long)j * w] >> p) & 1ull)) {
          const long long y = yc[(long long)j * w];
          const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
          const int ent = (int)(((ay >> p) & ((1ull << kMatWin) - 1ull)) >> 1);
          addr = mat_slot(j, ent, row, u) * (CP * G) + g * CP;
          if (y < 0) {
            op = 3;
            copy = !started1;
            started1 = true;
          } else {
            op = 2;
            copy = !started0;
            started0 = true;
          }
        }
        ++j;
      }
    }
  };
  int op;
  long long addr = 0;
  bool copy;
#if EFL_MAT_PREFETCH
  // scanned one event ahead: the next multiply's HBM operand loads while this product computes
  int op_n;
  long long addr_n = 0;
  bool copy_n;
  uint32_t nx[C28];
  next(op, addr, copy);
  if (op >= 2) load28<C28>(nx, Xm + addr);
  while (op >= 0) {
    uint32_t* acc = (op & 1) ? ACC[1] : ACC[0];
    if (op < 2) {
      from_lds<C28>(t, acc, E, g);
    } else {
#pragma unroll
      for (int q = 0; q < C28; ++q) t[q] = nx[q];
    }
    next(op_n, addr_n, copy_n);
    if (op_n >= 2) load28<C28>(nx, Xm + addr_n);
    if (!copy) {
      s28::mont_mul<C28, G>(t, LdsElem{acc, E}, m28, minv28, g);
      lds_sync();
    }
    to_lds<C28>(acc, E, g, t);
    lds_sync();
    op = op_n;
    addr = addr_n;
    copy = copy_n;
  }
#else
  for (;;) {
    next(op, addr, copy);
    if (op < 0) break;
    uint32_t* acc = (op & 1) ? ACC[1] : ACC[0];
    if (op < 2) from_lds<C28>(t, acc, E, g);
#if EFL_MAT_PROBE == 2   // timing probe (wrong results): every multiply operand from one cached slot
    else load28<C28>(t, Xm + g * CP);
#else
    else load28<C28>(t, Xm + addr);
#endif
    if (!copy) {
#if EFL_MAT_PROBE != 1   // timing probe (wrong results): EFL_MAT_PROBE=1 skips the products
      s28::mont_mul<C28, G>(t, LdsElem{acc, E}, m28, minv28, g);
#endif
      lds_sync();
    }
    to_lds<C28>(acc, E, g, t);
    lds_sync();
  }
#endif
  if (S > 1) {
    // partial products (radix-2^28 Montgomery form, < 2m) for k_matcomb28; 1 = R for an unused sign
#pragma unroll
    for (int sgn = 0; sgn < 2; ++sgn) {
      if (sgn ? started1 : started0) from_lds<C28>(t, ACC[sgn], E, g);
      else slice_uniform<C28>(t, k.at(k.d.off_n2_one28), g);
      uint32_t* q = P + (((long long)sp * UW + o) * 2 + sgn) * (CP * G) + g * CP;
#pragma unroll
      for (int jj = 0; jj < CP; jj += 4)
        *reinterpret_cast<uint4*>(q + jj) = make_uint4(t[jj], jj + 1 < C28 ? t[jj + 1] : 0u,
                                                       jj + 2 < C28 ? t[jj + 2] : 0u, jj + 3 < C28 ? t[jj + 3] : 0u);
    }
    if (sp == 0 && g == 0) ze[o] = mn;
    return;
  }
  uint32_t* out[2] = {zpos + o * L, zneg + o * L};
#pragma unroll
  for (int sgn = 0; sgn < 2; ++sgn) {
    if (sgn ? started1 : started0) {
      from_lds<C28>(t, ACC[sgn], E, g);
      lds_sync();
      store_from_mont28<C, G>(out[sgn], t, m28, minv28, ACC[sgn], E, g);   // the product's LDS is the scratch
    } else {
      uint32_t one[C];
#pragma unroll
      for (int j = 0; j < C; ++j) one[j] = (g == 0 && j == 0) ? 1u : 0u;
      store_slice<C>(out[sgn], g, one);
    }
    lds_sync();
  }
  if (g == 0) ze[o] = mn;
}

// z_pos / z_neg from the S partial products of each output (k_matmul28 with S > 1)
template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? 2 : EFL_DEC_WAVES) void k_matcomb28(
    Key k, const uint32_t* __restrict__ P, int S, long long UW, uint32_t* __restrict__ zpos,
    uint32_t* __restrict__ zneg) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= UW * 2) return;
  const long long o = i >> 1;
  const int sgn = (int)(i & 1);
  uint32_t* B = lds + e;
  uint32_t m28[C28], t[C28], r[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), g);
  const uint32_t minv28 = k.d.n2_minv28;
  const long long stride = UW * 2 * (CP * G);
  const uint32_t* q = P + (o * 2 + sgn) * (CP * G) + g * CP;
  load28<C28>(t, q);
  for (int sp = 1; sp < S; ++sp) {
    load28<C28>(r, q + sp * stride);
    lds_sync();
    to_lds<C28>(B, E, g, r);
    lds_sync();
    s28::mont_mul<C28, G>(t, LdsElem{B, E}, m28, minv28, g);
  }
  lds_sync();
  store_from_mont28<C, G>((sgn ? zneg : zpos) + o * L, t, m28, minv28, B, E, g);
}

// PaillierMatmul core, one group per output (see paillier.hip k_matmul)
template <int C, int G>
__global__ __launch_bounds__(kSlBlock) SL_OCC void k_matmul(Key k, const uint32_t* __restrict__ X,
                                                     const long long* __restrict__ xe,
                                                     const long long* __restrict__ ym,
                                                     const long long* __restrict__ ye, uint32_t* __restrict__ zpos,
                                                     uint32_t* __restrict__ zneg, long long* __restrict__ ze, int u,
                                                     int v, int w) {
  constexpr int L = C * G, E = kSlBlock / G;
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= (long long)u * w) return;
  const int row = (int)(i % u), kk = (int)(i / u);   // column by column, as k_matmul28
  const long long o = (long long)row * w + kk;
  uint32_t* BASE = lds + e;
  uint32_t* SCR = lds + L * E + e;
  uint32_t* POS = lds + 2 * L * E + e;
  uint32_t* NEG = lds + 3 * L * E + e;
  uint32_t n2[C], t[C];
  slice_uniform<C>(n2, k.at(k.d.off_n2), g);
  const uint32_t minv = k.d.n2_minv;
  long long mn = 0x7FFFFFFFFFFFFFFFll;
  for (int j = 0; j < v; ++j) {
    const long long ex = xe[(long long)row * v + j] + ye[(long long)j * w + kk];
    mn = ex < mn ? ex : mn;
  }
  slice_uniform<C>(t, k.at(k.d.off_n2_one), g);
  to_lds<C>(POS, E, g, t);
  to_lds<C>(NEG, E, g, t);
  for (int j = 0; j < v; ++j) {
    const long long y = ym[(long long)j * w + kk];
    if (y == 0) continue;
    const uint64_t ay = y < 0 ? 0ull - (uint64_t)y : (uint64_t)y;
    const long long delta = xe[(long long)row * v + j] + ye[(long long)j * w + kk] - mn;
    load_slice<C>(t, X + ((long long)row * v + j) * L, g);
    mont_mul<C, G>(t, Uniform{k.at(k.d.off_n2_r2)}, n2, minv, g);
    to_lds<C>(BASE, E, g, t);
    const int bits = 64 - __clzll((long long)ay);
    for (int b = bits - 2; b >= 0; --b) {
      mont_sqr<C, G>(t, SCR, E, n2, minv, g);
      if ((ay >> b) & 1ull) mont_mul<C, G>(t, LdsElem{BASE, E}, n2, minv, g);
    }
    for (long long d = 0; d < delta; ++d) mont_sqr<C, G>(t, SCR, E, n2, minv, g);
    uint32_t* acc = y > 0 ? POS : NEG;
    lds_sync();
    mont_mul<C, G>(t, LdsElem{acc, E}, n2, minv, g);
    to_lds<C>(acc, E, g, t);
  }
  lds_sync();
  from_lds<C>(t, POS, E, g);
  redc<C, G>(t, n2, minv, g);
  store_slice<C>(zpos + o * L, g, t);
  from_lds<C>(t, NEG, E, g);
  redc<C, G>(t, n2, minv, g);
  store_slice<C>(zneg + o * L, g, t);
  if (g == 0) ze[o] = mn;
}

// ------------------------------------------------------------------------------------------
// decryption: L = ln limbs (x^2 for x = p, q), half slices of C/2 limbs for numbers mod x
// ------------------------------------------------------------------------------------------

// Sliding-window exponentiation by the decryption exponent x - 1 (the same for every element, so
// the window walk is wave-uniform): the element's odd powers c^1, c^3, ..., c^(2^kDecWin - 1) in
// radix-2^28 Montgomery form go to a global scratch slab (kDecEntries x G x CP words per element,
// this lane's CP-word slice at +g*CP), and every multiply stages its entry in LDS. Products per
// modulus: bits(x-1) - 1 squarings + ~bits/(kDecWin+1) multiplies + 2^(kDecWin-1) for the table,
// against bits - 1 + popcount - 1 for the binary method: 2404 instead of ~3071 at 4096-bit n.
constexpr int kDecWin = 5, kDecEntries = 1 << (kDecWin - 1);

// bit b of the uniform exponent
__device__ __forceinline__ uint32_t ebit(const uint32_t* ex, int b) { return (ex[b >> 5] >> (b & 31)) & 1u; }

// res = L_x(c^(x-1) mod x^2) * h mod x   (paillier.cc:28-48). tab: this element's odd-power slab
// (sliding window), or null for the binary method.
template <int C, int G>
__device__ __forceinline__ void m_func(uint32_t (&res)[C / 2], const uint32_t* __restrict__ c, const Key& k,
                                       bool second, uint32_t* BASE, uint32_t* SCR, int E, int g,
                                       uint32_t* __restrict__ tab) {
  constexpr int L = C * G, CH = C / 2, LH = L / 2;
  uint32_t x2[C];
  slice_uniform<C>(x2, k.at(second ? k.d.off_q2 : k.d.off_p2), g);
  const uint32_t x2_minv = second ? k.d.q2_minv : k.d.p2_minv;
  const uint32_t* r3 = k.at(second ? k.d.off_q2_r3 : k.d.off_p2_r3);
  const uint32_t* ex = k.at(second ? k.d.off_qm1 : k.d.off_pm1);
  const int ebits = second ? k.d.qm1_bits : k.d.pm1_bits;

  // c R mod x^2 = hi R^2 + lo R  with c = hi 2^(32L) + lo
  uint32_t t[C], lo[C];
  load_slice<C>(t, c + L, g);
  mont_mul<C, G>(t, Uniform{r3}, x2, x2_minv, g);   // hi R^2
  load_slice<C>(lo, c, g);
  mont_mul<C, G>(lo, Uniform{r3}, x2, x2_minv, g);  // lo R^2
  redc<C, G>(lo, x2, x2_minv, g);                   // lo R
  const uint32_t top = add<C, G>(t, lo, g);
  csub<C, G>(t, x2, top != 0 || geq<C, G>(t, x2, g), g);
  // The exponentiation runs in radix 2^28 with lazy carries (csrc/sliced28.h: one v_mad_u64_u32
  // per limb product instead of about three instructions): c mod x^2 in normal form -> 28-bit
  // limbs through LDS -> c R28 mod x^2 -> square-and-multiply by x - 1 -> redc (< x^2) -> 32-bit.
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  constexpr int kLog2G = G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : 5;
  redc<C, G>(t, x2, x2_minv, g);   // c mod x^2
  to_lds<C>(SCR, E, g, t);
  lds_sync();
  // keep the key constants the code after the exponentiation needs from being loaded (and held
  // in VGPRs) across it: the loop wants its registers for the accumulators
  asm volatile("" ::: "memory");
  // the running value's limb layout: folded (symmetric squarings, sliced28.h) for the 32-word-slice
  // families over G >= 2 lanes (the 2048- to 8192-bit keys' defaults, 37-limb slices), blocked
  // otherwise (the short-slice families keep CIOS: their unrolled folded loops cost compile time
  // for little)
  constexpr bool kFold = G > 1 && C == 32 && EFL_SQR_FOLD;
  // SOS squarings for the 37-limb slices over 2 or 4 lanes (the 2048- and 4096-bit keys' defaults)
  // when the sliding window's table slab is there (the binary method keeps CIOS)
  constexpr bool kSos = !kFold && (G == 2 || G == 4) && C == 32 && EFL_SQR_SOS;
  const uint32_t minv28 = second ? k.d.q2_minv28 : k.d.p2_minv28;
  const uint32_t* r2_28 = k.at(second ? k.d.off_q2_r2_28[kLog2G] : k.d.off_p2_r2_28[kLog2G]);
  const uint32_t* m28_at = k.at(second ? k.d.off_q2_28 : k.d.off_p2_28);
  if constexpr (kFold) {
    uint32_t a[C28], m28[C28];
    s28::from_words_folded<C28, G>(a, SCR, E, L, g);
    s28::slice_uniform_folded<C28, G>(m28, m28_at, g);
    s28::mont_mul_folded<C28, G>(a, Uniform{r2_28}, BASE, E, m28, minv28, g);   // c R28
    lds_sync();
    if (tab) {
      constexpr int CP = pad4<C28>();
      uint32_t* slot = tab + g * CP;               // entry e at slot + e * G * CP (folded slices)
      store28<C28>(slot, a);
      uint32_t c2[C28];
#pragma unroll
      for (int j = 0; j < C28; ++j) c2[j] = a[j];
      s28::fold_mont<C28, G>(c2, SCR, E, m28, minv28, g, true);
      lds_sync();
      s28::to_lds_folded<C28, G>(BASE, E, g, c2);
      lds_sync();
#pragma unroll 1
      for (int e2 = 1; e2 < kDecEntries; ++e2) {
        s28::fold_mont<C28, G>(a, BASE, E, m28, minv28, g, false);
        store28<C28>(slot + (size_t)e2 * G * CP, a);
      }
      lds_sync();
      int b = ebits - 1;
      int j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
      while (!ebit(ex, j)) ++j;
      uint32_t v = 0;
      for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
      load28<C28>(a, slot + (size_t)(v >> 1) * G * CP);
      b = j - 1;
      // The window walk with one fold_mont call site for its squarings and multiplies alike: the
      // next operation is planned at the top of the loop (a lone squaring for a 0 bit, or a window's
      // squarings, then its multiply). The entry is loaded just before its multiply, not held in
      // VGPRs across the squarings (the squaring needs them; the other wave on the SIMD covers the
      // load, once per window)
      size_t ent_at = 0;
      int sq_left = 0;
      bool mul_next = false;
#pragma unroll 1
      for (;;) {
        if (sq_left == 0 && !mul_next) {
          if (b < 0) break;
          if (!ebit(ex, b)) {
            sq_left = 1;
            --b;
          } else {
            j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
            while (!ebit(ex, j)) ++j;
            v = 0;
            for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
            ent_at = (size_t)(v >> 1) * G * CP;
            sq_left = b - j + 1;
            mul_next = true;
            b = j - 1;
          }
        }
        const bool sq = sq_left > 0;
        if (!sq) {
          uint32_t ent[C28];
          load28<C28>(ent, slot + ent_at);
          s28::to_lds_folded<C28, G>(BASE, E, g, ent);
          lds_sync();
        }
        s28::fold_mont<C28, G>(a, sq ? SCR : BASE, E, m28, minv28, g, sq);
        lds_sync();
        if (sq) --sq_left;
        else mul_next = false;
      }
    } else {
      s28::to_lds_folded<C28, G>(BASE, E, g, a);
      lds_sync();
#pragma unroll 1
      for (int b = ebits - 2; b >= 0; --b) {
        s28::fold_mont<C28, G>(a, SCR, E, m28, minv28, g, true);
        lds_sync();
        if (ebit(ex, b)) {
          s28::fold_mont<C28, G>(a, BASE, E, m28, minv28, g, false);
          lds_sync();
        }
      }
    }
    s28::mont_mul_folded<C28, G>(a, Unit{}, BASE, E, m28, minv28, g);   // y = c^(x-1) mod x^2
    lds_sync();
    s28::to_lds_folded<C28, G>(SCR, E, g, a);
    lds_sync();
  } else if constexpr (kSos) {
    // the SOS squarings (sliced28.h sos_sqr) take both LDS arrays as the square's 2 L words; one
    // call site for every squaring of the window walk (its code is about 3,500 instructions)
    uint32_t a[C28], m28[C28];
    s28::from_words<C28>(a, SCR, E, L, g);
    slice_uniform<C28>(m28, m28_at, g);
    s28::mont_mul<C28, G>(a, Uniform{r2_28}, m28, minv28, g);
    lds_sync();
    if (!tab) {                                    // the binary method (efl_pl_tune(ln, 2, 0)): CIOS
      to_lds<C28>(BASE, E, g, a);
#pragma unroll 1
      for (int b = ebits - 2; b >= 0; --b) {
        s28::mont_sqr<C28, G>(a, SCR, E, m28, minv28, g);
        if (ebit(ex, b)) s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
      }
    } else {
    constexpr int CP = pad4<C28>();
    uint32_t* slot = tab + g * CP;                 // entry e at slot + e * G * CP
    store28<C28>(slot, a);
    int b = ebits - 1;
    int j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
    while (!ebit(ex, j)) ++j;
    uint32_t v = 0;
    for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
    // phase -1: c^2, then the odd powers; phase 0: the window walk
    int nsq = 1;
    int e2 = 0;                                    // table entries built so far (after c^2)
    bool build = true;
    size_t ent_at = 0;
    bool mul = false;
#pragma unroll 1
    for (;;) {
#pragma unroll 1
      for (int t = 0; t < nsq; ++t) {
        s28::sos_sqr<C28, G>(a, BASE, E, m28, minv28, g);
        lds_sync();
      }
      if (build) {
        // a = c^2: stage it, then T[e] = T[e-1] c^2 from c
        to_lds<C28>(BASE, E, g, a);
        lds_sync();
        load28<C28>(a, slot);
#pragma unroll 1
        for (e2 = 1; e2 < kDecEntries; ++e2) {
          s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
          store28<C28>(slot + (size_t)e2 * G * CP, a);
        }
        lds_sync();
        load28<C28>(a, slot + (size_t)(v >> 1) * G * CP);
        b = j - 1;
        build = false;
      } else if (mul) {
        uint32_t ent[C28];
        load28<C28>(ent, slot + ent_at);
        to_lds<C28>(BASE, E, g, ent);
        lds_sync();
        s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
        lds_sync();
      }
      if (b < 0) break;
      if (!ebit(ex, b)) {
        nsq = 1;
        mul = false;
        --b;
      } else {
        j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
        while (!ebit(ex, j)) ++j;
        v = 0;
        for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
        ent_at = (size_t)(v >> 1) * G * CP;
        nsq = b - j + 1;
        mul = true;
        b = j - 1;
      }
    }
    }
    s28::mont_mul<C28, G>(a, Unit{}, m28, minv28, g);   // y = c^(x-1) mod x^2
    lds_sync();
    to_lds<C28>(SCR, E, g, a);
    lds_sync();
  } else {
  uint32_t a[C28], m28[C28];
  s28::from_words<C28>(a, SCR, E, L, g);
  slice_uniform<C28>(m28, m28_at, g);
  s28::mont_mul<C28, G>(a, Uniform{r2_28}, m28, minv28, g);
  lds_sync();
  if (tab) {
    constexpr int CP = pad4<C28>();
    uint32_t* slot = tab + g * CP;                 // entry e at slot + e * G * CP
    // odd powers: T[0] = c, T[e] = T[e-1] c^2
    store28<C28>(slot, a);
    uint32_t c2[C28];
#pragma unroll
    for (int j = 0; j < C28; ++j) c2[j] = a[j];
    s28::mont_sqr<C28, G>(c2, SCR, E, m28, minv28, g);
    lds_sync();
    to_lds<C28>(BASE, E, g, c2);
    lds_sync();
#pragma unroll 1
    for (int e2 = 1; e2 < kDecEntries; ++e2) {
      s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
      store28<C28>(slot + (size_t)e2 * G * CP, a);
    }
    lds_sync();
    // left to right: windows of up to kDecWin bits that end in a 1 bit (the top bit is 1)
    int b = ebits - 1;
    int j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
    while (!ebit(ex, j)) ++j;
    uint32_t v = 0;
    for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
    load28<C28>(a, slot + (size_t)(v >> 1) * G * CP);
    b = j - 1;
#pragma unroll 1
    while (b >= 0) {
      if (!ebit(ex, b)) {
        s28::mont_sqr<C28, G>(a, SCR, E, m28, minv28, g);
        --b;
        continue;
      }
      j = b - kDecWin + 1 > 0 ? b - kDecWin + 1 : 0;
      while (!ebit(ex, j)) ++j;
      v = 0;
      for (int t = b; t >= j; --t) v = (v << 1) | ebit(ex, t);
      uint32_t ent[C28];
      load28<C28>(ent, slot + (size_t)(v >> 1) * G * CP);   // in flight during the squarings
#pragma unroll 1
      for (int t = b; t >= j; --t) s28::mont_sqr<C28, G>(a, SCR, E, m28, minv28, g);
      // (mul_fips1 here, for one-lane numbers, measured 3 % slower: the 1024-bit decryption's 256
      // VGPRs were already full, round 4)
      to_lds<C28>(BASE, E, g, ent);
      lds_sync();
      s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
      lds_sync();
      b = j - 1;
    }
  } else {
    to_lds<C28>(BASE, E, g, a);
#pragma unroll 1
    for (int b = ebits - 2; b >= 0; --b) {
      s28::mont_sqr<C28, G>(a, SCR, E, m28, minv28, g);
      if (ebit(ex, b)) s28::mont_mul<C28, G>(a, LdsElem{BASE, E}, m28, minv28, g);
    }
  }
  s28::mont_mul<C28, G>(a, Unit{}, m28, minv28, g);   // y = c^(x-1) mod x^2 (< x^2; y = 1 mod x, so y >= 1)
  lds_sync();
  to_lds<C28>(SCR, E, g, a);
  lds_sync();
  }
  s28::to_words<C>(t, SCR, E, L28, g);
  lds_sync();
  asm volatile("" ::: "memory");
  sub_small<C, G>(t, 1u, g);
  to_lds<C>(SCR, E, g, t);
  lds_sync();
  // (y - 1) / x exactly = (y - 1) * x^-1 mod 2^(32 LH): operand scanning, limb ii of the
  // quotient leaves lane 0 after step ii
  uint32_t xi[CH], q[CH];
  slice_uniform<CH>(xi, k.at(second ? k.d.off_qinv_w : k.d.off_pinv_w), g);
#pragma unroll
  for (int j = 0; j < CH; ++j) q[j] = 0;
  uint32_t pend = 0;
#pragma unroll 1
  for (int ii = 0; ii < LH; ++ii) {
    const uint32_t yv = SCR[ii * E];
    uint32_t c1 = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const uint64_t p = mad(xi[j], yv, (uint64_t)q[j] + c1);
      q[j] = (uint32_t)p;
      c1 = (uint32_t)(p >> 32);
    }
    if (g == 0) BASE[ii * E] = q[0];
    uint32_t in = from_next<G>(q[0]);
    if (g == G - 1) in = 0;
#pragma unroll
    for (int j = 0; j < CH - 1; ++j) q[j] = q[j + 1];
    const uint64_t s = (uint64_t)in + pend + c1;
    q[CH - 1] = (uint32_t)s;
    pend = (uint32_t)(s >> 32);
  }
  lds_sync();
  from_lds<CH>(q, BASE, E, g);
  uint32_t xs[CH];
  slice_uniform<CH>(xs, k.at(second ? k.d.off_q : k.d.off_p), g);
  // * h mod x (h stored in Montgomery form -> normal result)
  mont_mul<CH, G>(q, Uniform{k.at(second ? k.d.off_hq : k.d.off_hp)}, xs, second ? k.d.q_minv : k.d.p_minv, g);
#pragma unroll
  for (int j = 0; j < CH; ++j) res[j] = q[j];
}

template <int C, int G>
__global__ __launch_bounds__(kSlBlock, C >= 32 ? 2 : EFL_DEC_WAVES) void k_decrypt(Key k, const uint32_t* __restrict__ ct,
                                                      uint32_t* __restrict__ mag, signed char* __restrict__ neg,
                                                      long long N, uint32_t* __restrict__ win) {
  constexpr int L = C * G, E = kSlBlock / G, CH = C / 2, LH = L / 2;
  constexpr int L28 = s28::limbs_per_lane(L, G) * G;   // LDS arrays also hold radix-2^28 numbers
  extern __shared__ uint32_t lds[];
  SL_ELEMENT(E, G)
  if (i >= N) return;
  uint32_t* BASE = lds + e;
  uint32_t* SCR = lds + L28 * E + e;
  const uint32_t* c = ct + i * 2 * L;
  // this element's odd-power slab (p's, then reused for q's)
  uint32_t* tab = win ? win + (size_t)i * kDecEntries * G * pad4<s28::limbs_per_lane(L, G)>() : nullptr;
  uint32_t mp[CH], mq[CH];
  m_func<C, G>(mp, c, k, false, BASE, SCR, E, g, tab);
  m_func<C, G>(mq, c, k, true, BASE, SCR, E, g, tab);
  // CRT (paillier.cc:296-307): h = ((mp - mq) mod p) * (q^-1 mod p) mod p; m = h q + mq
  uint32_t ph[CH], qh[CH], d[CH];
  slice_uniform<CH>(ph, k.at(k.d.off_p), g);
  slice_uniform<CH>(qh, k.at(k.d.off_q), g);
#pragma unroll
  for (int j = 0; j < CH; ++j) d[j] = mq[j];
  csub<CH, G>(d, ph, geq<CH, G>(d, ph, g), g);   // mq mod p (mq < q < 2p)
  {
    uint32_t r[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) r[j] = mp[j];
    if (sub<CH, G>(r, d, g)) add<CH, G>(r, ph, g);
#pragma unroll
    for (int j = 0; j < CH; ++j) d[j] = r[j];
  }
  mont_mul<CH, G>(d, Uniform{k.at(k.d.off_qinvp)}, ph, k.d.p_minv, g);
  // m = h q + mq by operand scanning; low limbs leave lane 0 into SCR, the high half follows
  to_lds<CH>(BASE, E, g, d);
  lds_sync();
  uint32_t t[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) t[j] = mq[j];
  uint32_t pend = 0;
#pragma unroll 1
  for (int ii = 0; ii < LH; ++ii) {
    const uint32_t hv = BASE[ii * E];
    uint32_t c1 = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const uint64_t p = mad(qh[j], hv, (uint64_t)t[j] + c1);
      t[j] = (uint32_t)p;
      c1 = (uint32_t)(p >> 32);
    }
    if (g == 0) SCR[ii * E] = t[0];
    uint32_t in = from_next<G>(t[0]);
    if (g == G - 1) in = 0;
#pragma unroll
    for (int j = 0; j < CH - 1; ++j) t[j] = t[j + 1];
    const uint64_t s = (uint64_t)in + pend + c1;
    t[CH - 1] = (uint32_t)s;
    pend = (uint32_t)(s >> 32);
  }
  resolve_carries<CH, G>(t, pend, g);
#pragma unroll
  for (int j = 0; j < CH; ++j) SCR[(LH + g * CH + j) * E] = t[j];
  lds_sync();
  uint32_t mm[C], ref[C];
  from_lds<C>(mm, SCR, E, g);
  // signed: m > max (= ceil(2n/3)) -> m - n  (paillier.cc:308-310)
  slice_uniform<C>(ref, k.at(k.d.off_max), g);
  const bool isneg = !geq<C, G>(ref, mm, g);
  if (isneg) {
    slice_uniform<C>(ref, k.at(k.d.off_n), g);
    rsub<C, G>(mm, ref, g);
  }
  store_slice<C>(mag + i * L, g, mm);
  if (g == 0) neg[i] = isneg ? 1 : 0;
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
inline unsigned grid_of(long long N, int G) {
  const long long E = kSlBlock / G;
  return (unsigned)((N + E - 1) / E);
}

template <int C, int G>
hipError_t run_encrypt(const Key& k, const long long* m, const uint32_t* hsa, uint32_t* out, long long N,
                       uint64_t seed, long long ctr0, hipStream_t s, int hsa_mont) {
  const int aw = (k.d.a_bits + 31) / 32;
  hipLaunchKernelGGL((k_encrypt<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), (size_t)(C * G + aw) * (kSlBlock / G) * 4, s, k, m,
                     hsa, out, N, seed, ctr0, hsa_mont);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_fbpowm(const Key& k, const uint32_t* a, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                      hipStream_t s) {
  const int aw = (k.d.a_bits + 31) / 32;
  hipLaunchKernelGGL((k_fbpowm<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), (size_t)(C * G + aw) * (kSlBlock / G) * 4, s, k, a,
                     out, N, seed, ctr0);
  return hipGetLastError();
}
// SIMDs of the current device (CUs x 4), read once per device index: a process that drives
// several GPUs (or partition modes with different CU counts) sizes each device's splits by its own
constexpr int kMaxDevices = 64;
int simd_count() {
  static std::atomic<int> n[kMaxDevices] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  std::atomic<int>& slot = n[dev < kMaxDevices ? dev : kMaxDevices - 1];
  int v = slot.load(std::memory_order_relaxed);
  if (!v) {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0) cu = 256;
    v = 4 * cu;
    slot.store(v, std::memory_order_relaxed);
  }
  return v;
}

// efl_pl_tune(ln, 4, P): parts of the row-split walks, 0 = chosen per launch (walk_parts), 1 = never
// split, 2..5 = that many whenever the launch is below 4 waves per SIMD
std::atomic<int> g_walk_parts{0};
constexpr int kMaxWalkParts = 5;

// Parts for a walk of N elements over G lanes each: the P maximising the share of busy lanes,
// x P / ceil(x P) for x = waves per SIMD, less about 3 % per extra part (the exponent's draw and
// regrouping per part, the join's loads); launches of 4 or more waves per SIMD are not split.
// MNIST activation, 1024-bit key: the two-lane n^2 walk x = 3.06 -> P = 3 (0.77 -> 0.92 of the lanes
// busy): 59.2 -> 77.4 M encryptions/s (profiles/r05/walk_split.jsonl). The one-lane walks (the key
// owner's CRT sub-keys, G = 1) are not split: their time goes to the table entries' HBM latency,
// and splitting them measured 1-3 % slower (107.7 -> 104.6 M/s at P = 3).
int walk_parts(long long N, int G) {
  const double x = (double)((N * G + 63) / 64) / simd_count();
  if (x <= 0.0 || x >= 4.0) return 1;
  const int fixed = g_walk_parts.load(std::memory_order_relaxed);
  if (fixed > 0) return fixed;        // (a fixed P splits the one-lane walks too: A/B, tests)
  if (G == 1) return 1;
  int best = 1;
  double bv = x / __builtin_ceil(x);
  for (int P = 2; P <= kMaxWalkParts; ++P) {
    const double u = x * P / __builtin_ceil(x * P) / (1.0 + 0.03 * (P - 1));
    if (u > bv * 1.02) {
      best = P;
      bv = u;
    }
  }
  return best;
}

// the row-split walk: P parts into stream-ordered scratch, then the join
template <int C, int G>
hipError_t run_walk28_split(const Key& k, const long long* m, const uint32_t* a, uint32_t* out, long long N,
                            uint64_t seed, long long ctr0, int parts, hipStream_t s) {
  constexpr int L = C * G, E = kSlBlock / G;
  constexpr int C28 = s28::limbs_per_lane(L, G), L28 = C28 * G;
  const size_t slot = (size_t)pad4<C28>() * G;
  const long long V = N * parts;
  uint32_t* P = nullptr;
  hipError_t err = hipMallocAsync(reinterpret_cast<void**>(&P), (size_t)V * slot * 4 + (size_t)V, s);
  if (err != hipSuccess) return err;
  unsigned char* F = reinterpret_cast<unsigned char*>(P + (size_t)V * slot);
  const int aw = (k.d.a_bits + 31) / 32;
  if (m)
    hipLaunchKernelGGL((k_walk28_part<C, G, false>), dim3(grid_of(V, G)), dim3(kSlBlock), (size_t)(L28 + aw) * E * 4,
                       s, k, a, P, F, N, parts, seed, ctr0);
  else
    hipLaunchKernelGGL((k_walk28_part<C, G, true>), dim3(grid_of(V, G)), dim3(kSlBlock), (size_t)(L28 + aw) * E * 4, s,
                       k, a, P, F, N, parts, seed, ctr0);
  err = hipGetLastError();
  if (err == hipSuccess) {
    hipLaunchKernelGGL((k_walk28_join<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), (size_t)2 * L28 * E * 4, s, k, m, P,
                       F, out, N, parts);
    err = hipGetLastError();
  }
  const hipError_t ferr = hipFreeAsync(P, s);
  return err != hipSuccess ? err : ferr;
}

template <int C, int G>
hipError_t run_encrypt28(const Key& k, const long long* m, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                         hipStream_t s) {
  const int parts = walk_parts(N, G);
  if (parts > 1) return run_walk28_split<C, G>(k, m, nullptr, out, N, seed, ctr0, parts, s);
  const int aw = (k.d.a_bits + 31) / 32;
  const size_t lds = (size_t)(s28::limbs_per_lane(C * G, G) * G + aw) * (kSlBlock / G) * 4;
  hipLaunchKernelGGL((k_encrypt28<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), lds, s, k, m, out, N, seed, ctr0);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_fbpowm28(const Key& k, const uint32_t* a, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                        hipStream_t s) {
  const int parts = walk_parts(N, G);
  if (parts > 1) return run_walk28_split<C, G>(k, nullptr, a, out, N, seed, ctr0, parts, s);
  const int aw = (k.d.a_bits + 31) / 32;
  const size_t lds = (size_t)(s28::limbs_per_lane(C * G, G) * G + aw) * (kSlBlock / G) * 4;
  hipLaunchKernelGGL((k_fbpowm28<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), lds, s, k, a, out, N, seed, ctr0,
                     (const uint32_t*)nullptr);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_fbpowm28g(const Key& k, const long long* m, const uint32_t* a, uint32_t* out, long long N,
                         uint64_t seed, long long ctr0, hipStream_t s) {
  constexpr int C28 = s28::limbs_per_lane(C * G, G), L28 = C28 * G;
  const int aw = (k.d.a_bits + 31) / 32;
  uint32_t* st = nullptr;
  hipError_t err = hipMallocAsync(reinterpret_cast<void**>(&st), (size_t)N * G * ((C28 + 3) & ~3) * 4, s);
  if (err != hipSuccess) return err;
  const size_t lds0 = (size_t)(L28 > C * G ? L28 : C * G) * (kSlBlock / G) * 4;
  hipLaunchKernelGGL((k_gstart28<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), lds0, s, k, m, st, N);
  err = hipGetLastError();
  if (err == hipSuccess) {
    const size_t lds = (size_t)(L28 + aw) * (kSlBlock / G) * 4;
    hipLaunchKernelGGL((k_fbpowm28<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), lds, s, k, a, out, N, seed, ctr0, st);
    err = hipGetLastError();
  }
  const hipError_t ferr = hipFreeAsync(st, s);
  return err != hipSuccess ? err : ferr;
}
// ---- the key owner's CRT encryption with an element's two walks in one wave (round 5) ------------
// The owner's encryption walks twice per element, mod p^2 and mod q^2, one lane each (family C = 32,
// G = 1 for the examples' 1024-bit key). Run per sub-key (k_gstart28 + k_fbpowm28 twice, then
// efl_pl_crt_join), each launch of the paillier_mnist activation is 1,568 waves: 1.53 per SIMD, so
// 480 of 1,024 SIMDs sit a wave short, and every launch pays its own tail. Here lanes 0-31 of a
// wave walk elements 32 w .. 32 w + 31 mod p^2 and lanes 32-63 the same elements mod q^2 (a Key per
// lane). Each lane makes its own walk start (y^2)^-1 g(m) first (what k_gstart28 writes, in
// registers) and, after the walk, its half of the CRT join: q^2 y_p in the p lane, p^2 y_q in the q
// lane (32 x 32 words each); the q lane hands its half to the p lane through LDS, which adds,
// subtracts n^2 at most once and stores the ciphertext. One pass per element: no k_gstart28 or
// join launch, no walk results in HBM. The list's whole rounds of waves run plain
// (k_crt_pair_whole: 3,072 waves, 3 per SIMD, at the MNIST activation); only the waves past them
// are split P ways over disjoint ranges of table rows (k_crt_pair_part, part 0 from the start) and
// joined (k_crt_pair_tjoin), so the split's overhead (each part draws and regroups a', the join's
// P - 1 products) falls on 2 % of the walks. Same values, bit for bit: a product mod x^2 does not
// depend on its grouping, and every lazy part < 2 x^2 is a valid Montgomery operand.

// the walk start of this lane's element: (y^2)^-1 g(m) R28 mod x^2 (k_gstart28's steps), B = this
// lane's LDS column (C28 words at stride E)
template <int C>
__device__ __forceinline__ void lane_gstart(uint32_t (&acc)[s28::limbs_per_lane(C, 1)], const Key& k,
                                            const uint32_t (&m28)[s28::limbs_per_lane(C, 1)], long long mi,
                                            uint32_t* B, int E) {
  constexpr int C28 = s28::limbs_per_lane(C, 1);
  const uint32_t minv28 = k.d.n2_minv28;
  const unsigned long long am = mi < 0 ? 0ull - (unsigned long long)mi : (unsigned long long)mi;
  slice_uniform<C28>(acc, k.at(k.d.off_gn28), 0);
  s28::mont_mul_steps<C28, 1>(acc, MLimbs{am}, m28, minv28, 0, 3);
  to_lds<C28>(B, E, 0, acc);
  lds_sync();
  {
    uint32_t t[C], x2[C];
    s28::to_words<C>(t, B, E, C28, 0);
    lds_sync();
    slice_uniform<C>(x2, k.at(k.d.off_n2), 0);
    csub<C, 1>(t, x2, geq<C, 1>(t, x2, 0), 0);
    if (mi < 0) rsub<C, 1>(t, x2, 0);
    add_small<C, 1>(t, 1u, 0);
    to_lds<C>(B, E, 0, t);
    lds_sync();
  }
  s28::from_words<C28>(acc, B, E, C, 0);
  s28::mont_mul<C28, 1>(acc, Uniform{k.at(k.d.off_gstart28)}, m28, minv28, 0);
}

// z (2 L + 1 words) += f y for an L-word f (this lane's pointer) and a register L-word y, rows R
// onwards (a template recursion, so every register index is a constant)
template <int L, int R>
__device__ __forceinline__ void add_rows(uint32_t (&z)[2 * L + 1], const uint32_t (&y)[L], const uint32_t* f,
                                         uint32_t over = 0) {
  if constexpr (R < L) {
    const uint32_t fr = f[R];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t p = (uint64_t)fr * y[j] + z[R + j] + c;
      z[R + j] = (uint32_t)p;
      c = (uint32_t)(p >> 32);
    }
    const uint64_t t = (uint64_t)z[R + L] + c + over;
    z[R + L] = (uint32_t)t;
    add_rows<L, R + 1>(z, y, f, (uint32_t)(t >> 32));
  } else {
    z[2 * L] += over;
  }
}

// the CRT join from the two lanes of element el: h = this lane's walk (normal form, C words); the
// p lane (q = false) ends with z = q^2 y_p + p^2 y_q - (n^2 if over) in out. Z = LDS area of
// (2 C + 1) x 32 words (column = lane & 31). Every lane of the wave calls it (lanes past N too,
// with el < 0: they only take part in the LDS order).
template <int C>
__device__ __forceinline__ void pair_join(const uint32_t (&h)[C], const uint32_t* other_x2, const uint32_t* n2w,
                                          uint32_t* Z, uint32_t* out, bool q, bool valid) {
  uint32_t z[2 * C + 1];
#pragma unroll
  for (int j = 0; j <= 2 * C; ++j) z[j] = 0u;
  if (valid) add_rows<C, 0>(z, h, other_x2);
  uint32_t* zc = Z + (threadIdx.x & 31);
  if (q && valid) {
#pragma unroll
    for (int j = 0; j <= 2 * C; ++j) zc[j * 32] = z[j];
  }
  lds_sync();
  if (q || !valid) return;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j <= 2 * C; ++j) {
    const uint64_t s = (uint64_t)z[j] + zc[j * 32] + c;
    z[j] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  uint32_t borrow = 0;
#pragma unroll
  for (int j = 0; j < 2 * C; ++j) borrow = (uint32_t)(((uint64_t)z[j] - n2w[j] - borrow) >> 63);
  const bool ge = z[2 * C] >= borrow;
  borrow = 0;
#pragma unroll
  for (int j = 0; j < 2 * C; ++j) {
    const uint64_t d = (uint64_t)z[j] - (ge ? n2w[j] : 0u) - borrow;
    z[j] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  uint32_t zz[2 * C];
#pragma unroll
  for (int j = 0; j < 2 * C; ++j) zz[j] = z[j];
  store_slice<2 * C>(out, 0, zz);
}

template <int C>
__device__ __forceinline__ bool pair_lane(long long w, long long N, long long& el, bool& q) {
  q = threadIdx.x >= 32;
  el = w * 32 + (threadIdx.x & 31);
  return el < N;
}

// wave w of the whole rounds: lanes 0-31 the p halves, 32-63 the q halves of elements 32 w ..
template <int C>
__device__ __forceinline__ void crt_pair_whole_wave(long long w, const Key& kp, const Key& kq,
                                                    const uint32_t* __restrict__ n2w, const long long* __restrict__ m,
                                                    const uint32_t* __restrict__ a_in, uint32_t* __restrict__ out,
                                                    long long N, uint64_t seed, long long ctr0, uint32_t* lds) {
  constexpr int E = kSlBlock, C28 = s28::limbs_per_lane(C, 1);
  long long el;
  bool q;
  const bool valid = pair_lane<C>(w, N, el, q);
  const Key k = q ? kq : kp;
  uint32_t h[C];
  if (valid) {
    const int words = (k.d.a_bits + 31) >> 5;
    uint32_t* B = lds + threadIdx.x;
    uint32_t* A = lds + C28 * E + threadIdx.x;
    if (a_in) {
      for (int wd = 0; wd < words; ++wd) A[wd * E] = a_in[el * words + wd];
    } else {
      draw_a<1>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + el), 0);
    }
    lds_sync();
    uint32_t m28[C28], acc[C28];
    slice_uniform<C28>(m28, k.at(k.d.off_n2_28), 0);
    lane_gstart<C>(acc, k, m28, m ? m[el] : 0, B, E);
    fbpowm28_walk<C, 1>(acc, k, A, B, E, words, m28, 0);
    s28::mont_mul<C28, 1>(acc, Unit{}, m28, k.d.n2_minv28, 0);
    lds_sync();
    to_lds<C28>(B, E, 0, acc);
    lds_sync();
    s28::to_words<C>(h, B, E, C28, 0);
  }
  lds_sync();
  const uint32_t* ox2 = q ? kp.at(kp.d.off_n2) : kq.at(kq.d.off_n2);   // the other prime's square
  pair_join<C>(h, ox2, n2w, lds, out + el * 2 * C, q, valid);
}

template <int C>
__global__ __launch_bounds__(kSlBlock, EFL_WALK1_WAVES) void k_crt_pair_whole(
    Key kp, Key kq, const uint32_t* __restrict__ n2w, const long long* __restrict__ m,
    const uint32_t* __restrict__ a_in, uint32_t* __restrict__ out, long long N, uint64_t seed, long long ctr0) {
  extern __shared__ uint32_t lds[];
  crt_pair_whole_wave<C>(blockIdx.x, kp, kq, n2w, m, a_in, out, N, seed, ctr0, lds);
}

// part `part` of tail wave t (global wave w0 + t): slot v = (part * tw + t) * 64 + lane
template <int C>
__global__ __launch_bounds__(kSlBlock, EFL_WALK1_WAVES) void k_crt_pair_part(
    Key kp, Key kq, const long long* __restrict__ m, const uint32_t* __restrict__ a_in, uint32_t* __restrict__ P,
    unsigned char* __restrict__ F, long long N, long long w0, long long tw, int parts, uint64_t seed, long long ctr0) {
  constexpr int E = kSlBlock, C28 = s28::limbs_per_lane(C, 1), CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  const int part = (int)(blockIdx.x / tw);
  const long long t = blockIdx.x - (long long)part * tw;
  long long el;
  bool q;
  if (!pair_lane<C>(w0 + t, N, el, q)) return;
  const Key k = q ? kq : kp;
  const long long v = (long long)blockIdx.x * kSlBlock + threadIdx.x;
  const int words = (k.d.a_bits + 31) >> 5;
  uint32_t* B = lds + threadIdx.x;
  uint32_t* A = lds + C28 * E + threadIdx.x;
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), 0);
  bool have = false;
  if (part == 0) {
    lane_gstart<C>(acc, k, m28, m ? m[el] : 0, B, E);
    have = true;
  }
  if (a_in) {
    for (int w = 0; w < words; ++w) A[w * E] = a_in[el * words + w];
  } else {
    draw_a<1>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + el), 0);
  }
  lds_sync();
  const int size = regroup_shared(A, E, words, k.d.group_size, 0);
  const int rows = k.d.table_rows;
  const int r0 = (int)((long long)rows * part / parts), r1 = (int)((long long)rows * (part + 1) / parts);
  have = walk28_rows<C, 1>(acc, k, A, B, E, words, size, m28, 0, r0, r1, have);
  store28<C28>(P + (size_t)v * CP, acc);
  F[v] = have ? 1 : 0;
}

template <int C>
__global__ __launch_bounds__(kSlBlock, EFL_WALK1_WAVES) void k_crt_pair_tjoin(
    Key kp, Key kq, const uint32_t* __restrict__ n2w, const uint32_t* __restrict__ P,
    const unsigned char* __restrict__ F, uint32_t* __restrict__ out, long long N, long long w0, long long tw,
    int parts) {
  constexpr int E = kSlBlock, C28 = s28::limbs_per_lane(C, 1), CP = pad4<C28>();
  extern __shared__ uint32_t lds[];
  long long el;
  bool q;
  const bool valid = pair_lane<C>(w0 + blockIdx.x, N, el, q);
  const Key k = q ? kq : kp;
  uint32_t h[C];
  if (valid) {
    uint32_t* B = lds + threadIdx.x;
    uint32_t m28[C28], acc[C28];
    slice_uniform<C28>(m28, k.at(k.d.off_n2_28), 0);
    const uint32_t minv28 = k.d.n2_minv28;
    load28<C28>(acc, P + ((size_t)blockIdx.x * kSlBlock + threadIdx.x) * CP);   // part 0: holds the start
    for (int p = 1; p < parts; ++p) {
      const long long v = ((long long)p * tw + blockIdx.x) * kSlBlock + threadIdx.x;
      if (!F[v]) continue;
      uint32_t b[C28];
      load28<C28>(b, P + (size_t)v * CP);
      s28::mul_fips1<C28>(acc, b, m28, minv28);
    }
    s28::mont_mul<C28, 1>(acc, Unit{}, m28, minv28, 0);
    lds_sync();
    to_lds<C28>(B, E, 0, acc);
    lds_sync();
    s28::to_words<C>(h, B, E, C28, 0);
  }
  lds_sync();
  const uint32_t* ox2 = q ? kp.at(kp.d.off_n2) : kq.at(kq.d.off_n2);   // the other prime's square
  pair_join<C>(h, ox2, n2w, lds, out + el * 2 * C, q, valid);
}

// The tail as a product tree across lanes (round 6). The element-halves past the whole rounds are
// split S ways over table rows INSIDE a wave: lane l walks rows [rows p / S, rows (p + 1) / S) of
// element-half (l >> 5, (l & 31) / S), p = l % S, part 0 from the walk start (lane_gstart). The S
// partial products then meet in log2 S levels: at level d the lanes with p % 2d == 0 take the
// partner's (p + d) product through LDS and multiply, so an element-half's S - 1 products cost
// log2 S products of wave time, where the split-and-join launches (k_crt_pair_part,
// k_crt_pair_tjoin) paid P - 1 in series, in a second launch, plus each part's store and reload.
// Part 0 then holds the element-half's walk, and the p / q halves join as in k_crt_pair_whole.
// Lanes diverge only in the walk's trip count (rows differ by at most one) and in part 0's
// lane_gstart; lds_sync is a wavefront fence, so the divergent calls are safe.
template <int C, int S>
__device__ __forceinline__ void crt_pair_tree_wave(long long wb, const Key& kp, const Key& kq,
                                                   const uint32_t* __restrict__ n2w, const long long* __restrict__ m,
                                                   const uint32_t* __restrict__ a_in, uint32_t* __restrict__ out,
                                                   long long N, long long el0, uint64_t seed, long long ctr0,
                                                   uint32_t* lds) {
  static_assert(S >= 2 && S <= 32 && (S & (S - 1)) == 0, "parts per element-half: a power of two dividing 32");
  constexpr int E = kSlBlock, C28 = s28::limbs_per_lane(C, 1);
  const int lane = (int)threadIdx.x;
  const bool q = lane >= 32;
  const int part = lane % S;
  const long long el = el0 + wb * (32 / S) + (lane & 31) / S;
  const bool live = el < N;
  const Key k = q ? kq : kp;
  uint32_t* B = lds + lane;
  uint32_t* A = lds + C28 * E + lane;
  uint32_t m28[C28], acc[C28];
  slice_uniform<C28>(m28, k.at(k.d.off_n2_28), 0);
  const uint32_t minv28 = k.d.n2_minv28;
  bool have = false;
  if (live) {
    const int words = (k.d.a_bits + 31) >> 5;
    if (part == 0) {
      lane_gstart<C>(acc, k, m28, m ? m[el] : 0, B, E);
      have = true;
    }
    if (a_in) {
      for (int w = 0; w < words; ++w) A[w * E] = a_in[el * words + w];
    } else {
      draw_a<1>(A, E, words, k.d.a_bits, seed, (uint64_t)(ctr0 + el), 0);
    }
    lds_sync();
    const int size = regroup_shared(A, E, words, k.d.group_size, 0);
    const int rows = k.d.table_rows;
    const int r0 = (int)((long long)rows * part / S), r1 = (int)((long long)rows * (part + 1) / S);
    have = walk28_rows<C, 1>(acc, k, A, B, E, words, size, m28, 0, r0, r1, have);
  }
  for (int d = 1; d < S; d <<= 1) {
    lds_sync();
#pragma unroll
    for (int j = 0; j < C28; ++j) B[j * E] = acc[j];
    A[0] = have ? 1u : 0u;
    lds_sync();
    if (live && part % (2 * d) == 0 && A[d]) {
      uint32_t b[C28];
#pragma unroll
      for (int j = 0; j < C28; ++j) b[j] = B[j * E + d];
      if (have) {
        s28::mul_fips1<C28>(acc, b, m28, minv28);
      } else {
#pragma unroll
        for (int j = 0; j < C28; ++j) acc[j] = b[j];
        have = true;
      }
    }
  }
  const bool valid = live && part == 0;
  uint32_t h[C];
  lds_sync();
  if (valid) {
    s28::mont_mul<C28, 1>(acc, Unit{}, m28, minv28, 0);
    to_lds<C28>(B, E, 0, acc);
  }
  lds_sync();
  if (valid) s28::to_words<C>(h, B, E, C28, 0);
  lds_sync();
  const uint32_t* ox2 = q ? kp.at(kp.d.off_n2) : kq.at(kq.d.off_n2);   // the other prime's square
  pair_join<C>(h, ox2, n2w, lds, out + (valid ? el : 0) * 2 * C, q, valid);
}

template <int C, int S>
__global__ __launch_bounds__(kSlBlock, EFL_WALK1_WAVES) void k_crt_pair_tree(
    Key kp, Key kq, const uint32_t* __restrict__ n2w, const long long* __restrict__ m,
    const uint32_t* __restrict__ a_in, uint32_t* __restrict__ out, long long N, long long el0, uint64_t seed,
    long long ctr0) {
  extern __shared__ uint32_t lds[];
  crt_pair_tree_wave<C, S>(blockIdx.x, kp, kq, n2w, m, a_in, out, N, el0, seed, ctr0, lds);
}

// The tail's tree waves and the whole rounds in ONE launch, the tree waves first (round 6, tail mode
// 0). Launched apart, the tail ran after the whole rounds, one wave per SIMD at most and latency
// bound (about 0.6 of a whole wave's time for 2 % of the work). Here blocks [0, tb) are tree waves of
// elements el0 .. N - 1 and blocks tb .. are whole waves 0 .. of elements 0 .. el0 - 1: each SIMD
// takes a short tree wave beside its first whole wave, and the dispatcher fills the slots the tree
// waves free with whole waves, so the tail's work spreads over the whole launch.
template <int C, int S>
__global__ __launch_bounds__(kSlBlock, EFL_WALK1_WAVES) void k_crt_pair_mixed(
    Key kp, Key kq, const uint32_t* __restrict__ n2w, const long long* __restrict__ m,
    const uint32_t* __restrict__ a_in, uint32_t* __restrict__ out, long long N, long long el0, long long tb,
    uint64_t seed, long long ctr0) {
  extern __shared__ uint32_t lds[];
  const long long b = blockIdx.x;
  if (b < tb) crt_pair_tree_wave<C, S>(b, kp, kq, n2w, m, a_in, out, N, el0, seed, ctr0, lds);
  else crt_pair_whole_wave<C>(b - tb, kp, kq, n2w, m, a_in, out, el0, seed, ctr0, lds);
}

// efl_pl_tune(ln, 6, v): the tail of the paired CRT encryption: 0 = the tail's tree waves in the same
// launch as the whole rounds, ahead of them (k_crt_pair_mixed, S chosen per launch; round 6), 1 = the
// split-and-join launches (round 5; tail_parts chooses the parts, 1 when the tail is not worth
// splitting), 2 / 4 / 8 / 16 = the product tree with that S as a launch of its own after the whole
// rounds (round 6: no faster than 1 at the MNIST shape)
std::atomic<int> g_crt_tail{0};

// efl_pl_tune(ln, 5, v): the key owner's CRT encryption, 0 = chosen per launch (the paired lanes
// whenever they apply), 1 = one launch per sub-key and the join launch, 2 = the paired lanes
std::atomic<int> g_crt_fused{0};
constexpr int kMaxTailParts = 8;

// Parts for the waves past the whole rounds: the P minimising (the tail's part rounds, each rows / P
// + 1.5 products' time) + (the join: P - 1 products and the conversion, about 2), in walk units of
// `rows` products; 1 = no split (the tail runs as plain walks, one more round). *cost = the whole
// list's time in walk units.
int tail_parts(long long waves, int rows, long long* whole, double* cost) {
  const long long S = simd_count();
  *whole = waves / S * S;
  const long long tail = waves - *whole;
  double best = tail ? 1.0 : 0.0;   // the unsplit tail: one more round
  int bp = 1;
  for (int P = 2; tail && rows >= 4 && P <= kMaxTailParts; ++P) {
    const double part_rounds = (double)((tail * P + S - 1) / S);
    const double c = part_rounds * ((double)rows / P + 1.5) / rows + (P + 1.0) / rows;
    if (c < best * 0.97) {
      best = c;
      bp = P;
    }
  }
  *cost = (double)(*whole / S) + best;
  return bp;
}


template <int C>
hipError_t run_crt_pair(const Key& kp, const Key& kq, const uint32_t* n2w, const long long* m, const uint32_t* a,
                        uint32_t* out, long long N, uint64_t seed, long long ctr0, hipStream_t s) {
  constexpr int E = kSlBlock, C28 = s28::limbs_per_lane(C, 1), CP = pad4<C28>();
  const long long waves = (N + 31) / 32;
  long long whole = 0;
  double cost = 0.0;
  const int mode = g_crt_tail.load(std::memory_order_relaxed);
  int S = mode;                        // >= 2: the tree tail with S parts, launched after the whole rounds
  const bool tree = S >= 2;
  int parts = 1;
  if (mode == 0) {
    // the largest S <= 16 whose tree waves (tail elements x S / 32) still fit one per SIMD; none: the
    // tail runs as plain whole waves
    whole = waves / simd_count() * simd_count();
    const long long tail_el = N - whole * 32;
    S = 1;
    for (int P = 2; P <= 16; P <<= 1)
      if (tail_el > 0 && (tail_el * P + 31) / 32 <= simd_count()) S = P;
    const size_t walk_lds0 = (size_t)(C28 + (kp.d.a_bits + 31) / 32) * E * 4, join_lds0 = (size_t)(2 * C + 1) * 32 * 4;
    const size_t lds0 = walk_lds0 > join_lds0 ? walk_lds0 : join_lds0;
    if (S == 1) {
      hipLaunchKernelGGL((k_crt_pair_whole<C>), dim3((unsigned)waves), dim3(kSlBlock), lds0, s, kp, kq, n2w, m, a, out,
                         N, seed, ctr0);
      return hipGetLastError();
    }
    const long long el0 = whole * 32, tb = (tail_el * S + 31) / 32;
    const unsigned grid = (unsigned)(tb + whole);
    switch (S) {
      case 2: hipLaunchKernelGGL((k_crt_pair_mixed<C, 2>), dim3(grid), dim3(kSlBlock), lds0, s, kp, kq, n2w, m, a, out,
                                 N, el0, tb, seed, ctr0); break;
      case 4: hipLaunchKernelGGL((k_crt_pair_mixed<C, 4>), dim3(grid), dim3(kSlBlock), lds0, s, kp, kq, n2w, m, a, out,
                                 N, el0, tb, seed, ctr0); break;
      case 8: hipLaunchKernelGGL((k_crt_pair_mixed<C, 8>), dim3(grid), dim3(kSlBlock), lds0, s, kp, kq, n2w, m, a, out,
                                 N, el0, tb, seed, ctr0); break;
      default: hipLaunchKernelGGL((k_crt_pair_mixed<C, 16>), dim3(grid), dim3(kSlBlock), lds0, s, kp, kq, n2w, m, a,
                                  out, N, el0, tb, seed, ctr0); break;
    }
    return hipGetLastError();
  }
  if (tree) {
    whole = waves / simd_count() * simd_count();   // the whole rounds; the rest is the tree tail
  } else {
    parts = tail_parts(waves, kp.d.table_rows, &whole, &cost);
    if (parts == 1) whole = waves;
  }
  const long long tw = waves - whole;
  const int aw = (kp.d.a_bits + 31) / 32;
  // LDS: the walk's columns (C28 + aw words per lane), at least the join's (2 C + 1) x 32 words
  const size_t walk_lds = (size_t)(C28 + aw) * E * 4, join_lds = (size_t)(2 * C + 1) * 32 * 4;
  const size_t lds = walk_lds > join_lds ? walk_lds : join_lds;
  hipError_t err = hipSuccess;
  if (whole > 0) {
    hipLaunchKernelGGL((k_crt_pair_whole<C>), dim3((unsigned)whole), dim3(kSlBlock), lds, s, kp, kq, n2w, m, a, out, N,
                       seed, ctr0);
    err = hipGetLastError();
  }
  if (err != hipSuccess || tw == 0) return err;
  if (tree) {
    const long long el0 = whole * 32, tail_el = N - el0;
    const unsigned grid = (unsigned)((tail_el * S + 31) / 32);
    switch (S) {
      case 2: hipLaunchKernelGGL((k_crt_pair_tree<C, 2>), dim3(grid), dim3(kSlBlock), lds, s, kp, kq, n2w, m, a, out, N,
                                 el0, seed, ctr0); break;
      case 4: hipLaunchKernelGGL((k_crt_pair_tree<C, 4>), dim3(grid), dim3(kSlBlock), lds, s, kp, kq, n2w, m, a, out, N,
                                 el0, seed, ctr0); break;
      case 8: hipLaunchKernelGGL((k_crt_pair_tree<C, 8>), dim3(grid), dim3(kSlBlock), lds, s, kp, kq, n2w, m, a, out, N,
                                 el0, seed, ctr0); break;
      default: hipLaunchKernelGGL((k_crt_pair_tree<C, 16>), dim3(grid), dim3(kSlBlock), lds, s, kp, kq, n2w, m, a, out,
                                  N, el0, seed, ctr0); break;
    }
    return hipGetLastError();
  }
  const size_t slots = (size_t)tw * parts * kSlBlock;
  uint32_t* P = nullptr;
  err = hipMallocAsync(reinterpret_cast<void**>(&P), slots * CP * 4 + slots, s);
  if (err != hipSuccess) return err;
  unsigned char* F = reinterpret_cast<unsigned char*>(P + slots * CP);
  hipLaunchKernelGGL((k_crt_pair_part<C>), dim3((unsigned)(tw * parts)), dim3(kSlBlock), walk_lds, s, kp, kq, m, a, P, F,
                     N, whole, tw, parts, seed, ctr0);
  err = hipGetLastError();
  if (err == hipSuccess) {
    const size_t tl = (size_t)C28 * E * 4 > join_lds ? (size_t)C28 * E * 4 : join_lds;
    hipLaunchKernelGGL((k_crt_pair_tjoin<C>), dim3((unsigned)tw), dim3(kSlBlock), tl, s, kp, kq, n2w, P, F, out, N, whole,
                       tw, parts);
    err = hipGetLastError();
  }
  const hipError_t ferr = hipFreeAsync(P, s);
  return err != hipSuccess ? err : ferr;
}

template <int C, int G, class XS>
hipError_t run_powm28(const Key& k, const uint32_t* x, XS xs, uint32_t* out, long long N, unsigned long long* bad,
                      hipStream_t s) {
  const size_t lds = (size_t)(2 * s28::limbs_per_lane(C * G, G) * G) * (kSlBlock / G) * 4;
  hipLaunchKernelGGL((k_powm28<C, G, XS>), dim3(grid_of(N, G)), dim3(kSlBlock), lds, s, k, x, xs, out, N, bad);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_fxp_add28(const Key& k, const uint32_t* x, const long long* xe, const uint32_t* y, const long long* ye,
                         uint32_t* out, long long N, unsigned long long* bad, hipStream_t s) {
  const size_t lds = (size_t)(2 * s28::limbs_per_lane(C * G, G) * G) * (kSlBlock / G) * 4;
  hipLaunchKernelGGL((k_fxp_add28<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), lds, s, k, x, xe, y, ye, out, N, bad);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_matmul28(const Key& k, const uint32_t* X, const long long* xe, const long long* ym, const long long* ye,
                        uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w, hipStream_t s) {
  constexpr int C28 = s28::limbs_per_lane(C * G, G), L28 = C28 * G, E = kSlBlock / G;
  const long long nx = (long long)u * v, UW = (long long)u * w;
  // terms split S ways over separate groups when one group per output would leave part of one
  // round of the kernel's waves per SIMD empty; every split repeats the squarings (982 / 1034 / 1133
  // products per output of the MNIST product at S = 1 / 2 / 4), and the partials are combined
  // after. Round 1 and the scan-per-event kernel wanted two rounds (S = 4 there) to even out the
  // groups' scan lengths; with the event lists (k_mmevents) one round is faster: 17.0 ms at S = 2
  // against 18.1 at S = 4 and 29.2 at S = 1 (profiles/r02/matmul_splits_events.jsonl).
  // bench.py mirrors this choice.
  constexpr long long kOneRound = 256ll * 4 * 64 * (C >= 32 ? EFL_MAT_WAVES32 : EFL_MAT_WAVES16);
  int S = 1;
  const int fixed = g_mat_splits.load();
  if (fixed > 0) {
    while (2 * S <= fixed && 2 * S <= v) S *= 2;
  } else {
    while (2 * S <= 8 && 2 * S <= v && UW * G * S < kOneRound) S *= 2;
  }
  const size_t slot = (size_t)pad4<C28>() * G;
  // event-list capacity per (output, split): five windows per term cover 24-bit mantissas (the
  // fp32 encode's), three the decrease_precision weights; a list past it falls back to the scan.
  // The lists take at most 1 GiB: larger products get shorter lists (more outputs scan).
  const long long NL = UW * S, terms = (v + S - 1) / S;
  long long cap = terms * 5 < 4096 ? terms * 5 : 4096;
  if (cap * NL > (1ll << 28)) cap = (1ll << 28) / NL;
  // stream-ordered scratch: the odd powers of every x (kMatEntries padded radix-2^28 slices each),
  // then the S > 1 partials, the event lists, then (8-byte aligned) the window masks of y, the list
  // headers and the outputs' minimum exponents
  const size_t x_words = (size_t)nx * kMatEntries * slot, p_words = S > 1 ? (size_t)S * UW * 2 * slot : 0;
  const size_t ev_words = ((size_t)NL * cap + 1) & ~(size_t)1;
  const size_t yw = (size_t)v * w;
  uint32_t* Xm = nullptr;
  hipError_t err = hipMallocAsync(reinterpret_cast<void**>(&Xm),
                                  (x_words + p_words + ev_words) * 4 + yw * 8 + (size_t)NL * 16, s);
  if (err != hipSuccess) return err;
  uint32_t* P = S > 1 ? Xm + x_words : nullptr;
  uint32_t* EV = Xm + x_words + p_words;
  unsigned long long* wm = reinterpret_cast<unsigned long long*>(EV + ev_words);
  int2* hdr = reinterpret_cast<int2*>(wm + yw);
  long long* mnv = reinterpret_cast<long long*>(hdr + NL);
  hipLaunchKernelGGL(k_wmask, dim3((unsigned)((yw + 255) / 256)), dim3(256), 0, s, ym, wm, (long long)yw);
  err = hipGetLastError();
  if (err == hipSuccess) {
    hipLaunchKernelGGL(k_mmevents, dim3((unsigned)((NL + kEvBlock - 1) / kEvBlock)), dim3(kEvBlock), 0, s, xe, ym, ye,
                       wm, u, v, w, S,
                       (int)cap, EV, hdr, mnv);
    err = hipGetLastError();
  }
  if (err == hipSuccess) {
    hipLaunchKernelGGL((k_tomont28<C, G>), dim3(grid_of(nx, G)), dim3(kSlBlock), (size_t)2 * L28 * E * 4, s, k, X, Xm,
                       nx, u, v);
    err = hipGetLastError();
  }
  if (err == hipSuccess) {
    hipLaunchKernelGGL((k_matmul28<C, G>), dim3(grid_of(UW * S, G)), dim3(kSlBlock), (size_t)2 * L28 * E * 4, s, k,
                       Xm, xe, ym, ye, zpos, zneg, ze, u, v, w, S, P, wm, EV, hdr, mnv);
    err = hipGetLastError();
  }
  if (err == hipSuccess && S > 1) {
    hipLaunchKernelGGL((k_matcomb28<C, G>), dim3(grid_of(UW * 2, G)), dim3(kSlBlock), (size_t)L28 * E * 4, s, k, P,
                       S, UW, zpos, zneg);
    err = hipGetLastError();
  }
  const hipError_t ferr = hipFreeAsync(Xm, s);
  return err != hipSuccess ? err : ferr;
}
template <int C, int G>
hipError_t run_add(const Key& k, const uint32_t* x, const uint32_t* y, uint32_t* out, long long N, hipStream_t s) {
  hipLaunchKernelGGL((k_add<C, G>), dim3(grid_of(N, G)), dim3(kSlBlock), (size_t)(C * G) * (kSlBlock / G) * 4, s, k, x, y, out, N);
  return hipGetLastError();
}
template <int C, int G, class XS>
hipError_t run_powm(const Key& k, const uint32_t* x, XS xs, uint32_t* out, long long N, unsigned long long* bad,
                    hipStream_t s) {
  hipLaunchKernelGGL((k_powm<C, G, XS>), dim3(grid_of(N, G)), dim3(kSlBlock), (size_t)(2 * C * G) * (kSlBlock / G) * 4, s, k, x,
                     xs, out, N, bad);
  return hipGetLastError();
}
template <int C, int G>
hipError_t run_matmul(const Key& k, const uint32_t* X, const long long* xe, const long long* ym, const long long* ye,
                      uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w, hipStream_t s) {
  hipLaunchKernelGGL((k_matmul<C, G>), dim3(grid_of((long long)u * w, G)), dim3(kSlBlock), (size_t)(4 * C * G) * (kSlBlock / G) * 4,
                     s, k, X, xe, ym, ye, zpos, zneg, ze, u, v, w);
  return hipGetLastError();
}
// Decryption launches in chunks of at most kDecChunk elements, each with a stream-ordered scratch
// slab for the sliding window's odd powers (kDecEntries x L28-padded words per element, e.g. 9.5 KB
// at 4096-bit n: 2.4 GiB at most per chunk), taken and released on `s` like efl_pl_matmul's.
constexpr long long kDecChunk = 1 << 18;
std::atomic<int> g_dec_window{1};   // efl_pl_tune(ln, 2, 0/1): binary method / sliding window

template <int C, int G>
hipError_t run_decrypt(const Key& k, const uint32_t* ct, uint32_t* mag, signed char* neg, long long N,
                       hipStream_t s) {
  constexpr int L = C * G;
  constexpr size_t slab = (size_t)kDecEntries * G * pad4<s28::limbs_per_lane(L, G)>();
  const size_t lds = (size_t)(2 * s28::limbs_per_lane(L, G) * G) * (kSlBlock / G) * 4;
  const long long chunk = N < kDecChunk ? N : kDecChunk;
  uint32_t* win = nullptr;
  if (g_dec_window.load(std::memory_order_relaxed)) {
    const hipError_t err = hipMallocAsync(reinterpret_cast<void**>(&win), (size_t)chunk * slab * 4, s);
    if (err != hipSuccess) return err;
  }
  hipError_t err = hipSuccess;
  for (long long o = 0; o < N && err == hipSuccess; o += chunk) {
    const long long n = N - o < chunk ? N - o : chunk;
    hipLaunchKernelGGL((k_decrypt<C, G>), dim3(grid_of(n, G)), dim3(kSlBlock), lds, s, k, ct + o * 2 * L,
                       mag + o * L, neg + o, n, win);
    err = hipGetLastError();
  }
  if (win) {
    const hipError_t ferr = hipFreeAsync(win, s);
    if (err == hipSuccess) err = ferr;
  }
  return err;
}

}  // namespace

// (L, C) pairs compiled: L = limbs of the modulus (2 ln for n^2 ops, ln for decryption)
bool sliced_available(int L, int C) {
  switch (L * 1000 + C) {
    case 16008: case 32008: case 64008: case 128008: case 256008:
    case 32016: case 32032: case 64016: case 64032: case 128016: case 128032: case 256016: case 256032:
    case 512032: return true;
    default: return false;
  }
}

#define SL_DISPATCH(L_, C_, EXPR)                            \
  switch ((L_) * 1000 + (C_)) {                              \
    case 16008: { constexpr int CC = 8, GG = 2; return EXPR; }   \
    case 32008: { constexpr int CC = 8, GG = 4; return EXPR; }   \
    case 64008: { constexpr int CC = 8, GG = 8; return EXPR; }   \
    case 128008: { constexpr int CC = 8, GG = 16; return EXPR; } \
    case 256008: { constexpr int CC = 8, GG = 32; return EXPR; } \
    case 32016: { constexpr int CC = 16, GG = 2; return EXPR; }  \
    case 32032: { constexpr int CC = 32, GG = 1; return EXPR; }  \
    case 64016: { constexpr int CC = 16, GG = 4; return EXPR; }  \
    case 64032: { constexpr int CC = 32, GG = 2; return EXPR; }  \
    case 128016: { constexpr int CC = 16, GG = 8; return EXPR; } \
    case 128032: { constexpr int CC = 32, GG = 4; return EXPR; } \
    case 256016: { constexpr int CC = 16, GG = 16; return EXPR; } \
    case 256032: { constexpr int CC = 32, GG = 8; return EXPR; } \
    case 512032: { constexpr int CC = 32, GG = 16; return EXPR; } \
    default: return hipErrorInvalidValue;                    \
  }

// the radix-2^28 table (include/efl_hip.h off_table28) serves a family whose lane count it was built for
inline bool table28_for(const Key& k, int C) {
  const int G = 2 * k.d.ln / C;
  return k.d.off_table28 >= 0 && (1 << k.d.table28_log2g) == G &&
         k.d.n2_28_len == s28::limbs_per_lane(2 * k.d.ln, G) * G;
}

hipError_t sl_encrypt(const Key& k, int C, const long long* m, const uint32_t* hsa, uint32_t* out, long long N,
                      uint64_t seed, long long ctr0, hipStream_t s, int hsa_mont) {
  if (!hsa && table28_for(k, C)) {
    SL_DISPATCH(2 * k.d.ln, C, (run_encrypt28<CC, GG>(k, m, out, N, seed, ctr0, s)))
  }
  SL_DISPATCH(2 * k.d.ln, C, (run_encrypt<CC, GG>(k, m, hsa, out, N, seed, ctr0, s, hsa_mont)))
}
hipError_t sl_fbpowm(const Key& k, int C, const uint32_t* a, uint32_t* out, long long N, uint64_t seed,
                     long long ctr0, hipStream_t s) {
  if (table28_for(k, C)) {
    SL_DISPATCH(2 * k.d.ln, C, (run_fbpowm28<CC, GG>(k, a, out, N, seed, ctr0, s)))
  }
  SL_DISPATCH(2 * k.d.ln, C, (run_fbpowm<CC, GG>(k, a, out, N, seed, ctr0, s)))
}
hipError_t sl_fbpowm_g(const Key& k, int C, const long long* m, const uint32_t* a, uint32_t* out, long long N,
                       uint64_t seed, long long ctr0, hipStream_t s) {
  if (!C || !table28_for(k, C) || k.d.off_gn28 < 0 || k.d.off_gstart28 < 0) return hipErrorNotSupported;
  SL_DISPATCH(2 * k.d.ln, C, (run_fbpowm28g<CC, GG>(k, m, a, out, N, seed, ctr0, s)))
}
hipError_t sl_crt_encrypt_pair(const Key& kp, const Key& kq, int C, const uint32_t* n2w, const long long* m,
                               const uint32_t* a, uint32_t* out, long long N, uint64_t seed, long long ctr0,
                               hipStream_t s) {
  if (g_crt_fused.load(std::memory_order_relaxed) == 1) return hipErrorNotSupported;
  if (C != 32 || 2 * kp.d.ln != 32 || 2 * kq.d.ln != 32 || !table28_for(kp, C) || !table28_for(kq, C) ||
      kp.d.off_gn28 < 0 || kp.d.off_gstart28 < 0 || kq.d.off_gn28 < 0 || kq.d.off_gstart28 < 0 ||
      kp.d.a_bits != kq.d.a_bits || kp.d.group_size != kq.d.group_size || kp.d.table_rows != kq.d.table_rows ||
      kp.d.table_window != kq.d.table_window || kp.d.table_cols != kq.d.table_cols)
    return hipErrorNotSupported;
  return run_crt_pair<32>(kp, kq, n2w, m, a, out, N, seed, ctr0, s);
}
int sl_crt_fused(int v) {
  return v < 0 ? g_crt_fused.load() : g_crt_fused.exchange(v);
}
int sl_crt_tail(int v) {
  return v < 0 ? g_crt_tail.load() : g_crt_tail.exchange(v);
}
hipError_t sl_add(const Key& k, int C, const uint32_t* x, const uint32_t* y, uint32_t* out, long long N,
                  hipStream_t s) {
  SL_DISPATCH(2 * k.d.ln, C, (run_add<CC, GG>(k, x, y, out, N, s)))
}
template <class XS>
hipError_t sl_powm_x(const Key& k, int C, const uint32_t* x, XS xs, uint32_t* out, long long N,
                     unsigned long long* bad, hipStream_t s) {
  if (table28_for(k, C)) {
    SL_DISPATCH(2 * k.d.ln, C, (run_powm28<CC, GG, XS>(k, x, xs, out, N, bad, s)))
  }
  SL_DISPATCH(2 * k.d.ln, C, (run_powm<CC, GG, XS>(k, x, xs, out, N, bad, s)))
}
hipError_t sl_powm(const Key& k, int C, const uint32_t* x, const uint32_t* e, int ew, uint32_t* out, long long N,
                   hipStream_t s) {
  return sl_powm_x(k, C, x, ExpWords{e, ew}, out, N, nullptr, s);
}
hipError_t sl_powm_abs64(const Key& k, int C, const uint32_t* x, const long long* y, uint32_t* out, long long N,
                         unsigned long long* bad, hipStream_t s) {
  return sl_powm_x(k, C, x, ExpAbs64{y}, out, N, bad, s);
}
hipError_t sl_powm_pow2(const Key& k, int C, const uint32_t* x, const long long* y, uint32_t* out, long long N,
                        unsigned long long* bad, hipStream_t s) {
  return sl_powm_x(k, C, x, ExpPow2{y}, out, N, bad, s);
}
hipError_t sl_powm_shift(const Key& k, int C, const uint32_t* x, const long long* own, const long long* other,
                         uint32_t* out, long long N, unsigned long long* bad, hipStream_t s) {
  return sl_powm_x(k, C, x, ExpShift{own, other}, out, N, bad, s);
}
hipError_t sl_fxp_add(const Key& k, int C, const uint32_t* x, const long long* xe, const uint32_t* y,
                      const long long* ye, uint32_t* out, long long N, unsigned long long* bad, hipStream_t s) {
  if (!table28_for(k, C)) return hipErrorNotSupported;
  SL_DISPATCH(2 * k.d.ln, C, (run_fxp_add28<CC, GG>(k, x, xe, y, ye, out, N, bad, s)))
}
hipError_t sl_matmul(const Key& k, int C, const uint32_t* X, const long long* xe, const long long* ym,
                     const long long* ye, uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w,
                     hipStream_t s) {
  if (table28_for(k, C)) {
    SL_DISPATCH(2 * k.d.ln, C, (run_matmul28<CC, GG>(k, X, xe, ym, ye, zpos, zneg, ze, u, v, w, s)))
  }
  SL_DISPATCH(2 * k.d.ln, C, (run_matmul<CC, GG>(k, X, xe, ym, ye, zpos, zneg, ze, u, v, w, s)))
}
int sl_dec_window(int v) {
  return v < 0 ? g_dec_window.load() : g_dec_window.exchange(v ? 1 : 0);
}
int sl_mat_splits(int v) {
  return v < 0 ? g_mat_splits.load() : g_mat_splits.exchange(v);
}
int sl_walk_parts(int v) {
  return v < 0 ? g_walk_parts.load() : g_walk_parts.exchange(v);
}
hipError_t sl_decrypt(const Key& k, int C, const uint32_t* ct, uint32_t* mag, signed char* neg, long long N,
                      hipStream_t s) {
  SL_DISPATCH(k.d.ln, C, (run_decrypt<CC, GG>(k, ct, mag, neg, N, s)))
}

}  // namespace pl
}  // namespace efl
