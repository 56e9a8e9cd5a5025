// Secret-sharing masks and DP-SGD noise: the additive float noise EFLS
// applies to a tensor before the communicator sends one share of it cross-silo, and the Gaussian
// noise its DP optimisers add to the summed microbatch gradients.
//
// Reference: efls-train/python/efl/privacy/secret_sharing.py
//   generate_suitable_noise(t) = tf.random.uniform(shape(t)) * t                        (:26-27)
//   share():       send a = noise(x), keep x - a                                        (:158-168)
//   Dense weights: send w - noise(w)/d, keep w + noise(w)/d                             (:137-143)
//   _matmul mode A (column pairs of e = noise(a)): send [a + e | e_even + e_odd],
//                  keep a - e and e_odd - e_even                                        (:30-41)
//   _matmul mode B (row pairs of f = noise(b)):    send [b/2 - f ; f_even - f_odd],
//                  keep b/2 + f and f_odd + f_even                                      (:42-53)
// TF draws the uniform from an unseeded Philox4x32-10 stream and converts each 32-bit word with
// Uint32ToFloat (23 mantissa bits under exponent 127, minus 1.0). The build uses the same
// generator and conversion, keyed by an explicit 64-bit seed with element i taking word i % 4 of
// Philox block ctr0 + i / 4, so every output is reproducible and checkable bit for bit
// (oracle/mask.py); the reference itself is only pinned statistically.
//
// Every kernel is one streaming pass: read x once, write each output once. One lane owns four
// consecutive elements (one Philox block, dwordx4 loads and stores). HBM-bound, no LDS, no MFMA.
#include <atomic>
#include <cmath>

#include "common.h"
#include "pl_common.h"
#include "box_muller_math.h"
#include "sincos_angle.h"

// Every product and sum rounds on its own, as TF's separate ops (and numpy in the oracle) do:
// hipcc contracts a*b+c into one FMA by default, which changes the last bit.
#pragma clang fp contract(off)

namespace efl {
namespace {

using pl::philox;

// Store flavour of the mask kernels (efl_fxp_tune kind 28): 0 plain stores, 2 nontemporal (`nt`),
// 7 `global_store_dwordx{2,4} ... nt sc1` (the line leaves the XCD's L2 as it is written; the
// streaming encode's flavour). The DP kernel keeps plain stores.
typedef int i4m __attribute__((ext_vector_type(4)));
typedef int i2m __attribute__((ext_vector_type(2)));
template <int ST = 0, class T>
__device__ __forceinline__ void stv(T* p, T v) {
  if constexpr (ST == 7 && sizeof(T) == 16) {
    const i4m w = __builtin_bit_cast(i4m, v);
    // a VALU write to the data VGPRs right after a >8-byte store needs a wait state the hazard
    // recognizer cannot see inside asm (tests/test_isa_guard.py checks the s_nop)
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr (ST == 7 && sizeof(T) == 8) {
    const i2m w = __builtin_bit_cast(i2m, v);
    asm volatile("global_store_dwordx2 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr (ST == 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

__device__ __forceinline__ float u01(uint32_t w) {
  return __uint_as_float(0x3f800000u | (w & 0x7fffffu)) - 1.0f;
}

__device__ __forceinline__ void draw4(uint64_t seed, uint64_t blk, float (&u)[4]) {
  uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = u01(c[j]);
}

// noise n = U * x (then / d when d != 1, as `noise / noise_divisor` in the reference). DIV is a
// template parameter (0 none, 1 times the exact reciprocal of a power-of-two d — the same rounding
// as the division — 2 the IEEE division): as a runtime flag the compiler computed the division for
// every element and selected (about 11 VALU instructions each, round 6 ISA).
template <int DIV>
__device__ __forceinline__ float noise(float u, float x, float d) {
  const float n = u * x;
  if constexpr (DIV == 1) return n * d;
  else if constexpr (DIV == 2) return n / d;
  else return n;
}

// Division of a lane-group index by the row length: q = g / d for g < 2^31 as one 64-bit product and
// a shift (Granlund-Montgomery: l = ceil(log2 d), m = floor(2^(31 + l) / d) + 1 < 2^32 is exact for
// every g < 2^31), from the magic (m, 31 + l) the host passes; m == 0 (more than 2^31 groups) takes
// the 64-bit division.
__device__ __forceinline__ long long div_groups(long long g, long long d, uint32_t m, int sh) {
  if (m) return (long long)(((uint64_t)(uint32_t)g * m) >> sh);
  return g / d;
}

// op 0: o0 = n            (generate_suitable_noise)
// op 1: o0 = n, o1 = x-n  (share: the sent share and the kept one)
// op 2: o0 = x-n, o1 = x+n (Dense weight noise: sent and kept)
// One lane owns NB Philox blocks (4 elements each) kBlock lanes apart, so a wave's accesses stay
// 64 x 16 contiguous bytes; the loads of all NB blocks are issued first and the NB Philox chains
// run round by round together while they travel (round 6, the DP kernel's round-5 structure: one
// block per lane drew the uniforms before loading x, with nothing in flight meanwhile).
template <int OP, int DIV>
__device__ __forceinline__ void noise_f4(const f4& v, const float (&u)[4], float d, f4& a, f4& b) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float nz = noise<DIV>(u[j], v[j], d);
    if (OP == 0) a[j] = nz;
    if (OP == 1) { a[j] = nz; b[j] = v[j] - nz; }
    if (OP == 2) { a[j] = v[j] - nz; b[j] = v[j] + nz; }
  }
}

template <int NB>
__device__ __forceinline__ void uniforms(uint64_t seed, const uint64_t (&blk)[NB], float (&u)[NB][4]) {
  uint32_t c[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    c[b][0] = (uint32_t)blk[b];
    c[b][1] = (uint32_t)(blk[b] >> 32);
    c[b][2] = 0u;
    c[b][3] = 0u;
  }
  pl::philox_n<NB>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int j = 0; j < 4; ++j) u[b][j] = u01(c[b][j]);
}

template <int OP, int DIV, int NB, int ST>
__global__ __launch_bounds__(kBlock) void k_noise(const float* __restrict__ x, float* __restrict__ o0,
                                                  float* __restrict__ o1, long long n, uint64_t seed,
                                                  uint64_t ctr0, float d) {
  const long long g0 = (long long)blockIdx.x * (kBlock * NB) + threadIdx.x;
  if (g0 * 4 >= n) return;
  if ((g0 + (long long)(NB - 1) * kBlock) * 4 + 4 <= n) {
    f4 v[NB];
    uint64_t blk[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      v[b] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + g0 + b * kBlock);
      blk[b] = ctr0 + (uint64_t)(g0 + b * kBlock);
    }
    float u[NB][4];
    uniforms<NB>(seed, blk, u);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f4 a, c;
      noise_f4<OP, DIV>(v[b], u[b], d, a, c);
      stv<ST>(reinterpret_cast<f4*>(o0) + g0 + b * kBlock, a);
      if (OP != 0) stv<ST>(reinterpret_cast<f4*>(o1) + g0 + b * kBlock, c);
    }
    return;
  }
  for (int b = 0; b < NB; ++b) {
    const long long g = g0 + b * kBlock, i0 = g * 4;
    if (i0 >= n) break;
    float u[4];
    draw4(seed, ctr0 + (uint64_t)g, u);
    if (i0 + 4 <= n) {
      const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + g);
      f4 a, c;
      noise_f4<OP, DIV>(v, u, d, a, c);
      stv<ST>(reinterpret_cast<f4*>(o0) + g, a);
      if (OP != 0) stv<ST>(reinterpret_cast<f4*>(o1) + g, c);
    } else {
      for (int j = 0; j < 4 && i0 + j < n; ++j) {
        const float xv = x[i0 + j];
        const float nz = noise<DIV>(u[j], xv, d);
        if (OP == 0) o0[i0 + j] = nz;
        if (OP == 1) { o0[i0 + j] = nz; o1[i0 + j] = xv - nz; }
        if (OP == 2) { o0[i0 + j] = xv - nz; o1[i0 + j] = xv + nz; }
      }
    }
  }
}

// Mode A, a [R, C] with C % 8 == 0 (every row of send, width 3C/2, then starts 16-byte aligned):
// lane group g owns a[r, 4q .. 4q+3] (element index 4g); a lane owns NB groups kBlock apart, loads
// first, Philox chains together (as k_noise).
// send [R, 3C/2] = [a + e | e_even + e_odd], keep0 [R, C] = a - e, keep1 [R, C/2] = e_odd - e_even.
template <int ST>
__device__ __forceinline__ void mask_cols_store(const f4& v, const float (&u)[4], long long g, long long q4,
                                                long long C, float* __restrict__ send, float* __restrict__ keep0,
                                                float* __restrict__ keep1, uint32_t dm, int ds) {
  const long long r = div_groups(g, q4, dm, ds), q = g - r * q4;
  f4 s, k;
  float e[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[j] = u[j] * v[j];
    s[j] = v[j] + e[j];
    k[j] = v[j] - e[j];
  }
  const long long W = C + C / 2;
  stv<ST>(reinterpret_cast<f4*>(send + r * W + 4 * q), s);
  stv<ST>(reinterpret_cast<f4*>(keep0) + g, k);
  f2 p, m;
  p[0] = e[0] + e[1];
  p[1] = e[2] + e[3];
  m[0] = e[1] - e[0];
  m[1] = e[3] - e[2];
  stv<ST>(reinterpret_cast<f2*>(send + r * W + C + 2 * q), p);
  stv<ST>(reinterpret_cast<f2*>(keep1 + r * (C / 2) + 2 * q), m);
}

template <int NB, int ST>
__global__ __launch_bounds__(kBlock) void k_mask_cols4(const float* __restrict__ a, float* __restrict__ send,
                                                       float* __restrict__ keep0, float* __restrict__ keep1,
                                                       long long R, long long C, uint64_t seed, uint64_t ctr0,
                                                       uint32_t dm, int ds) {
  const long long g0 = (long long)blockIdx.x * (kBlock * NB) + threadIdx.x;
  const long long q4 = C / 4, total = R * q4;
  if (g0 >= total) return;
  if (g0 + (long long)(NB - 1) * kBlock < total) {
    f4 v[NB];
    uint64_t blk[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      v[b] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(a) + g0 + b * kBlock);
      blk[b] = ctr0 + (uint64_t)(g0 + b * kBlock);
    }
    float u[NB][4];
    uniforms<NB>(seed, blk, u);
#pragma unroll
    for (int b = 0; b < NB; ++b) mask_cols_store<ST>(v[b], u[b], g0 + b * kBlock, q4, C, send, keep0, keep1, dm, ds);
    return;
  }
  for (int b = 0; b < NB; ++b) {
    const long long g = g0 + b * kBlock;
    if (g >= total) break;
    float u[4];
    draw4(seed, ctr0 + (uint64_t)g, u);
    mask_cols_store<ST>(__builtin_nontemporal_load(reinterpret_cast<const f4*>(a) + g), u, g, q4, C, send, keep0, keep1,
                        dm, ds);
  }
}

// Mode A for other even C: one lane per column pair (2 elements), Philox word chosen per element.
__global__ __launch_bounds__(kBlock) void k_mask_cols2(const float* __restrict__ a, float* __restrict__ send,
                                                       float* __restrict__ keep0, float* __restrict__ keep1,
                                                       long long R, long long C, uint64_t seed, uint64_t ctr0) {
  const long long g = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long h = C / 2;
  if (g >= R * h) return;
  const long long r = g / h, j = g - r * h;
  const long long i = 2 * g;   // element index of a[r, 2j]; i % 4 is 0 or 2
  float u[4];
  draw4(seed, ctr0 + (uint64_t)(i >> 2), u);
  const int w = (int)(i & 3);
  const float x0 = a[i], x1 = a[i + 1];
  const float e0 = u[w] * x0, e1 = u[w + 1] * x1;
  const long long W = C + h;
  send[r * W + 2 * j] = x0 + e0;
  send[r * W + 2 * j + 1] = x1 + e1;
  keep0[i] = x0 - e0;
  keep0[i + 1] = x1 - e1;
  send[r * W + C + j] = e0 + e1;
  keep1[r * h + j] = e1 - e0;
}

// Mode B, b [K, N] with K even: lane group g owns columns 4q..4q+3 of rows 2j and 2j+1 (N % 4 == 0)
// or one column (general N). Element index of b[r, c] is r*N + c.
// send [3K/2, N] = [b/2 - f ; f_even - f_odd], keep0 [K, N] = b/2 + f, keep1 [K/2, N] = f_odd + f_even.
template <int V, int ST>
__device__ __forceinline__ void mask_rows_store(const float (&xe)[V], const float (&xo)[V], const float (&ue)[4],
                                                const float (&uo)[4], long long ie, long long io, long long idf,
                                                long long ik, float* __restrict__ send, float* __restrict__ keep0,
                                                float* __restrict__ keep1) {
  float se[V], so[V], ke[V], ko[V], sd[V], kd[V];
#pragma unroll
  for (int t = 0; t < V; ++t) {
    const float fe = ue[V == 4 ? t : (int)(ie & 3)] * xe[t];
    const float fo = uo[V == 4 ? t : (int)(io & 3)] * xo[t];
    const float he = xe[t] / 2.0f, ho = xo[t] / 2.0f;
    se[t] = he - fe;
    so[t] = ho - fo;
    ke[t] = he + fe;
    ko[t] = ho + fo;
    sd[t] = fe - fo;
    kd[t] = fo + fe;
  }
  if (V == 4) {
    stv<ST>(reinterpret_cast<f4*>(send + ie), f4{se[0], se[1], se[2], se[3]});
    stv<ST>(reinterpret_cast<f4*>(send + io), f4{so[0], so[1], so[2], so[3]});
    stv<ST>(reinterpret_cast<f4*>(keep0 + ie), f4{ke[0], ke[1], ke[2], ke[3]});
    stv<ST>(reinterpret_cast<f4*>(keep0 + io), f4{ko[0], ko[1], ko[2], ko[3]});
    stv<ST>(reinterpret_cast<f4*>(send + idf), f4{sd[0], sd[1], sd[2], sd[3]});
    stv<ST>(reinterpret_cast<f4*>(keep1 + ik), f4{kd[0], kd[1], kd[2], kd[3]});
  } else {
    send[ie] = se[0];
    send[io] = so[0];
    keep0[ie] = ke[0];
    keep0[io] = ko[0];
    send[idf] = sd[0];
    keep1[ik] = kd[0];
  }
}

// V = 4: a lane owns NB groups kBlock apart (2 NB Philox blocks), loads first, chains together
template <int V, int NB, int ST>
__global__ __launch_bounds__(kBlock) void k_mask_rows(const float* __restrict__ b, float* __restrict__ send,
                                                      float* __restrict__ keep0, float* __restrict__ keep1,
                                                      long long K, long long N, uint64_t seed, uint64_t ctr0,
                                                      uint32_t dm, int ds) {
  const long long g0 = (long long)blockIdx.x * (kBlock * NB) + threadIdx.x;
  const long long nq = N / V, total = (K / 2) * nq;
  if (g0 >= total) return;
  if (V == 4 && g0 + (long long)(NB - 1) * kBlock < total) {
    long long ie[NB], io[NB];
    f4 ve[NB], vo[NB];
    uint64_t blk[2 * NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const long long g = g0 + t * kBlock;
      const long long j = div_groups(g, nq, dm, ds), q = g - j * nq;
      ie[t] = 2 * j * N + V * q;
      io[t] = ie[t] + N;
      ve[t] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(b + ie[t]));
      vo[t] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(b + io[t]));
      blk[2 * t] = ctr0 + (uint64_t)(ie[t] >> 2);
      blk[2 * t + 1] = ctr0 + (uint64_t)(io[t] >> 2);
    }
    float u[2 * NB][4];
    uniforms<2 * NB>(seed, blk, u);
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const long long g = g0 + t * kBlock;
      const long long j = div_groups(g, nq, dm, ds), q = g - j * nq;
      float xe[V], xo[V];
#pragma unroll
      for (int c = 0; c < V; ++c) {
        xe[c] = ve[t][c];
        xo[c] = vo[t][c];
      }
      mask_rows_store<V, ST>(xe, xo, u[2 * t], u[2 * t + 1], ie[t], io[t], K * N + j * N + V * q, j * N + V * q, send,
                         keep0, keep1);
    }
    return;
  }
  for (int t = 0; t < NB; ++t) {
    const long long g = g0 + t * kBlock;
    if (g >= total) break;
    const long long j = div_groups(g, nq, dm, ds), q = g - j * nq;
    const long long ie = 2 * j * N + V * q, io = ie + N;   // a[2j, Vq], a[2j+1, Vq]
    float ue[4], uo[4];
    draw4(seed, ctr0 + (uint64_t)(ie >> 2), ue);
    draw4(seed, ctr0 + (uint64_t)(io >> 2), uo);
    float xe[V], xo[V];
    if (V == 4) {
      const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(b + ie));
      const f4 c = __builtin_nontemporal_load(reinterpret_cast<const f4*>(b + io));
#pragma unroll
      for (int k = 0; k < V; ++k) { xe[k] = a[k]; xo[k] = c[k]; }
    } else {
      xe[0] = b[ie];
      xo[0] = b[io];
    }
    mask_rows_store<V, ST>(xe, xo, ue, uo, ie, io, K * N + j * N + V * q, j * N + V * q, send, keep0, keep1);
  }
}

// ---- DP-SGD noise (efls-train/python/efl/privacy/dp_optimizer.py) ------------
// TF's tf.random.normal (NormalDistribution<PhiloxRandom, float>, tensorflow/core/lib/random/
// random_distributions.h): every Philox4x32-10 block gives 4 normals, Box-Muller on the word pairs
// (0, 1) and (2, 3): u1 = max(Uint32ToFloat(x0), 1e-7), v1 = float(2 pi (double) * Uint32ToFloat(x1)),
// r = sqrt(-2 log u1), (f0, f1) = r (sin v1, cos v1). Element i takes normal i % 4 of block
// ctr0 + i / 4, as the uniform masks do.
//
// logf / sqrtf over the arguments Box-Muller reaches: box_muller_math.h.
__device__ __forceinline__ void box_muller(uint32_t x0, uint32_t x1, float& f0, float& f1) {
  const float u1 = u01(x0);
  const float v1 = efl_box_muller_angle(u01(x1));   // float(2 pi (double) u), no doubles
  // both arms computed and one selected: a branch around the logarithm costs more than it saves
  const float rr = sqrt_normal(-2.0f * log_unit(fmaxf(u1, 1.0e-7f)));
  const float r = u1 < 1.0e-7f ? __uint_as_float(kRClampBits) : rr;
  float sn, cs;
  efl_sincos_angle(v1, &sn, &cs);   // v1 in [0, 2 pi]: <= 1 ulp of the rounded sin / cos (sincos_angle.h)
  f0 = sn * r;
  f1 = cs * r;
}

__device__ __forceinline__ void normal4(uint64_t seed, uint64_t blk, float (&z)[4]) {
  uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(c[0], c[1], z[0], z[1]);
  box_muller(c[2], c[3], z[2], z[3]);
}

// The normals of NB blocks (blk0, blk0 + stride, ...), the same values as normal4 on each, computed
// stage by stage across the 2 NB Box-Muller pairs (Philox rounds, logarithms, square roots, angles)
// so that every stage has 2 NB independent chains to fill the transcendental and compare hazards
// with (round 5: before, each pair ran to the end on its own, with s_nop between dependent steps).
template <int NB>
__device__ __forceinline__ void normals(uint64_t seed, uint64_t blk0, uint64_t stride, float (&z)[NB][4]) {
  constexpr int P = 2 * NB;
  uint32_t c[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint64_t blk = blk0 + (uint64_t)b * stride;
    c[b][0] = (uint32_t)blk;
    c[b][1] = (uint32_t)(blk >> 32);
    c[b][2] = 0u;
    c[b][3] = 0u;
  }
  pl::philox_n<NB>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u1[P], v1[P], r[P], sn[P], cs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    u1[p] = u01(c[p >> 1][(p & 1) * 2]);
    v1[p] = efl_box_muller_angle(u01(c[p >> 1][(p & 1) * 2 + 1]));
  }
#pragma unroll
  for (int p = 0; p < P; ++p) r[p] = -2.0f * log_unit(fmaxf(u1[p], 1.0e-7f));
#pragma unroll
  for (int p = 0; p < P; ++p) r[p] = sqrt_normal(r[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) r[p] = u1[p] < 1.0e-7f ? __uint_as_float(kRClampBits) : r[p];
#pragma unroll
  for (int p = 0; p < P; ++p) efl_sincos_angle(v1[p], &sn[p], &cs[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    z[p >> 1][(p & 1) * 2] = sn[p] * r[p];
    z[p >> 1][(p & 1) * 2 + 1] = cs[p] * r[p];
  }
}

// MODE 0, ElementWiseGaussianSumQuery.add_noise (dp_optimizer.py:70-71): v + normal * v * sigma;
// MODE 1, GaussianSumQuery (tensorflow_privacy 0.3.0, TF 1.x branch): v + (normal * stddev + 0);
// then safe_normalize (dp_optimizer.py:210-214): / num_microbatches. Each op rounds on its own.
// POW2: the divisor is a power of two and `div` holds its reciprocal: x * 2^-k is the correctly
// rounded x / 2^k (the same exact real, one rounding), without the IEEE division sequence.
template <int MODE, bool POW2>
__device__ __forceinline__ float dp_one(float v, float z, float sigma, float div) {
  const float n = MODE == 0 ? (z * v) * sigma : z * sigma + 0.0f;
  return POW2 ? (v + n) * div : (v + n) / div;
}

// One lane owns NB Philox blocks (4 elements each) kBlock lanes apart, so a wave's accesses stay
// 64 x 16 contiguous bytes. Round 2 drew the normals first and then loaded x: every lane sat in
// Box-Muller (logf, sincosf, a double product) with nothing in flight, 0.68 of 8 TB/s. Now the
// loads of all of a lane's blocks are issued first and the normals computed while they travel.
template <int MODE, bool POW2, int NB>
__global__ __launch_bounds__(kBlock) void k_dp_noise(const float* x, float* o,   // in place allowed
                                                     long long n, uint64_t seed, uint64_t ctr0, float sigma,
                                                     float div) {
  const long long g0 = (long long)blockIdx.x * (kBlock * NB) + threadIdx.x;
  if (g0 * 4 >= n) return;
  if ((g0 + (long long)(NB - 1) * kBlock) * 4 + 4 <= n) {
    f4 v[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) v[b] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + g0 + b * kBlock);
    float z[NB][4];
    normals<NB>(seed, ctr0 + (uint64_t)g0, kBlock, z);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = dp_one<MODE, POW2>(v[b][j], z[b][j], sigma, div);
      stv(reinterpret_cast<f4*>(o) + g0 + b * kBlock, r);
    }
    return;
  }
  for (int b = 0; b < NB; ++b) {
    const long long g = g0 + b * kBlock, i0 = g * 4;
    if (i0 >= n) break;
    float z[4];
    normal4(seed, ctr0 + (uint64_t)g, z);
    if (i0 + 4 <= n) {
      const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + g);
      f4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = dp_one<MODE, POW2>(v[j], z[j], sigma, div);
      stv(reinterpret_cast<f4*>(o) + g, r);
    } else {
      for (int j = 0; j < 4 && i0 + j < n; ++j) o[i0 + j] = dp_one<MODE, POW2>(x[i0 + j], z[j], sigma, div);
    }
  }
}

unsigned grid_for(long long lanes) { return (unsigned)((lanes + kBlock - 1) / kBlock); }

template <int MODE, bool POW2>
void launch_dp(int nb, long long lanes, const float* x, float* o, long long n, uint64_t seed, uint64_t ctr0,
               float sigma, float d, hipStream_t s) {
  const unsigned g1 = grid_for(lanes);
  if (nb == 1) k_dp_noise<MODE, POW2, 1><<<g1, kBlock, 0, s>>>(x, o, n, seed, ctr0, sigma, d);
  else if (nb == 4) k_dp_noise<MODE, POW2, 4><<<(g1 + 3) / 4, kBlock, 0, s>>>(x, o, n, seed, ctr0, sigma, d);
  else k_dp_noise<MODE, POW2, 2><<<(g1 + 1) / 2, kBlock, 0, s>>>(x, o, n, seed, ctr0, sigma, d);
}

bool lanes_ok(long long lanes) { return lanes / kBlock < (1ll << 31); }

// one launch of a mask kernel at nb lane groups per lane (1, 2, 4) and store flavour st (0, 2, 7):
// KERNEL(NB, ST) names the instance
#define EFL_MASK_LAUNCH(nb, st, lanes, s, KERNEL, ...)                                                \
  do {                                                                                               \
    const unsigned g1_ = grid_for(lanes);                                                            \
    const int nb_ = (nb), st_ = (st);                                                                \
    const unsigned gr_ = nb_ == 4 ? (g1_ + 3) / 4 : nb_ == 2 ? (g1_ + 1) / 2 : g1_;                  \
    if (nb_ == 4 && st_ == 7) KERNEL(4, 7)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                      \
    else if (nb_ == 4 && st_ == 2) KERNEL(4, 2)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                 \
    else if (nb_ == 4) KERNEL(4, 0)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                             \
    else if (nb_ == 2 && st_ == 7) KERNEL(2, 7)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                 \
    else if (nb_ == 2 && st_ == 2) KERNEL(2, 2)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                 \
    else if (nb_ == 2) KERNEL(2, 0)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                             \
    else if (st_ == 7) KERNEL(1, 7)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                             \
    else if (st_ == 2) KERNEL(1, 2)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                             \
    else KERNEL(1, 0)<<<gr_, kBlock, 0, s>>>(__VA_ARGS__);                                           \
  } while (0)
#define EFL_K_NOISE0D0(NB, ST) k_noise<0, 0, NB, ST>
#define EFL_K_NOISE0D1(NB, ST) k_noise<0, 1, NB, ST>
#define EFL_K_NOISE0D2(NB, ST) k_noise<0, 2, NB, ST>
#define EFL_K_NOISE1D0(NB, ST) k_noise<1, 0, NB, ST>
#define EFL_K_NOISE1D1(NB, ST) k_noise<1, 1, NB, ST>
#define EFL_K_NOISE1D2(NB, ST) k_noise<1, 2, NB, ST>
#define EFL_K_NOISE2D0(NB, ST) k_noise<2, 0, NB, ST>
#define EFL_K_NOISE2D1(NB, ST) k_noise<2, 1, NB, ST>
#define EFL_K_NOISE2D2(NB, ST) k_noise<2, 2, NB, ST>

// the magic (m, shift) of div_groups for d, or m = 0 when the groups pass 2^31
void group_magic(long long total, long long d, uint32_t* m, int* sh) {
  *m = 0;
  *sh = 0;
  if (total <= 0 || total >= (1ll << 31) || d <= 0) return;
  int l = 0;
  while ((1ll << l) < d) ++l;
  *m = (uint32_t)(((1ull << (31 + l)) / (unsigned long long)d) + 1ull);
  *sh = 31 + l;
}
// share / weight noise (op 1 / 2) with the two outputs over the two halves of a wave
// (efl_fxp_tune(30, 1), the default since round 6): lanes l and l + 32 load the same 16-byte group
// (one HBM read; the second half's request hits the line the first fetched), draw the same Philox
// block, and store o0 (l < 32) or o1 (l >= 32): one load and one store per lane, as mask_rows'
// halves. 0.72 -> 0.75 of 8 TB/s on two boxes.
template <int OP, int DIV, int ST>
__global__ __launch_bounds__(kBlock) void k_noise_half(const float* __restrict__ x, float* __restrict__ o0,
                                                       float* __restrict__ o1, long long n, uint64_t seed,
                                                       uint64_t ctr0, float d) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int half = (int)((threadIdx.x >> 5) & 1);
  const long long g = (t >> 6) * 32 + (threadIdx.x & 31), i0 = g * 4;
  if (i0 >= n) return;
  float* o = half ? o1 : o0;
  float u[4];
  draw4(seed, ctr0 + (uint64_t)g, u);
  if (i0 + 4 <= n) {
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + g);
    f4 a, c;
    noise_f4<OP, DIV>(v, u, d, a, c);
    stv<ST>(reinterpret_cast<f4*>(o) + g, half ? c : a);
    return;
  }
  for (int j = 0; j < 4 && i0 + j < n; ++j) {
    const float xv = x[i0 + j];
    const float nz = noise<DIV>(u[j], xv, d);
    if (OP == 1) o[i0 + j] = half ? xv - nz : nz;
    if (OP == 2) o[i0 + j] = half ? xv + nz : xv - nz;
  }
}

// Mode B with the row pair split over the two halves of a wave (efl_fxp_tune(29, 1), the default
// since round 6): lane l < 32 owns row 2j, lane l + 32 row 2j + 1 of the same four columns, so a lane
// loads one 16-byte group and stores three (its send and keep0 rows, then the send difference row
// from the even half or the keep sum row from the odd half, f swapped between the halves). A wave
// owns NB runs of 32 groups (kind 25): all NB loads first, the NB Philox chains together. Same values
// and Philox blocks as k_mask_rows; 0.66 -> 0.78 of 8 TB/s at [65536, 1024].
template <int NB, int ST>
__global__ __launch_bounds__(kBlock) void k_mask_rows_half(const float* __restrict__ b, float* __restrict__ send,
                                                           float* __restrict__ keep0, float* __restrict__ keep1,
                                                           long long K, long long N, uint64_t seed, uint64_t ctr0,
                                                           uint32_t dm, int ds) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int l = (int)(threadIdx.x & 63), half = l >> 5;
  const long long g0 = (t >> 6) * (32 * NB) + (l & 31);
  const long long nq = N / 4, total = (K / 2) * nq;
  long long i[NB], o[NB];
  bool valid[NB];
  f4 x[NB];
  uint64_t blk[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const long long g = g0 + 32 * k;
    valid[k] = g < total;
    const long long gv = valid[k] ? g : 0;
    const long long j = div_groups(gv, nq, dm, ds), q = gv - j * nq;
    i[k] = (2 * j + half) * N + 4 * q;
    o[k] = half == 0 ? K * N + j * N + 4 * q : j * N + 4 * q;   // send difference row / keep sum row
    x[k] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    if (valid[k]) x[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(b + i[k]));
    blk[k] = ctr0 + (uint64_t)(i[k] >> 2);
  }
  float u[NB][4];
  uniforms<NB>(seed, blk, u);
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    float f[4], pf[4];
    f4 sv, kv, dv;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      f[c] = u[k][c] * x[k][c];
      const float h = x[k][c] / 2.0f;
      sv[c] = h - f[c];
      kv[c] = h + f[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) pf[c] = __shfl_xor(f[c], 32);   // every lane takes part
#pragma unroll
    for (int c = 0; c < 4; ++c) dv[c] = half == 0 ? f[c] - pf[c] : f[c] + pf[c];   // fe - fo ; fo + fe
    if (valid[k]) {
      stv<ST>(reinterpret_cast<f4*>(send + i[k]), sv);
      stv<ST>(reinterpret_cast<f4*>(keep0 + i[k]), kv);
      stv<ST>(reinterpret_cast<f4*>((half == 0 ? send : keep1) + o[k]), dv);
    }
  }
}

#define EFL_K_COLS4(NB, ST) k_mask_cols4<NB, ST>
#define EFL_K_ROWS4(NB, ST) k_mask_rows<4, NB, ST>
#define EFL_K_ROWSH(NB, ST) k_mask_rows_half<NB, ST>

}  // namespace

// efl_fxp_tune(20, nb): Philox blocks per lane of the DP noise kernel (defined in fxp.hip);
// efl_fxp_tune(25, nb) / (28, st): lane groups per lane / store flavour of the mask kernels
extern std::atomic<int> g_dp_blocks;
extern std::atomic<int> g_mask_blocks[4];   // [noise, share / weight noise, mask_cols, mask_rows]
extern std::atomic<int> g_mask_store[4];
extern std::atomic<int> g_noise_half;       // efl_fxp_tune(30, v): share / weight noise over wave halves (1, default)
extern std::atomic<int> g_rows_half;        // efl_fxp_tune(29, v): mode B over wave halves (1, default) or not (0)

}  // namespace efl

using namespace efl;

EFL_API int efl_ss_noise(const float* x, float* out0, float* out1, int64_t n, int op, uint64_t seed,
                         uint64_t ctr0, float divisor, void* stream) {
  if (n < 0) { set_error("negative element count"); return EFL_E_INVALID_ARGUMENT; }
  if (op < 0 || op > 2) { set_error("efl_ss_noise: op must be 0, 1 or 2"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  if (!x || !out0 || (op != 0 && !out1)) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  if (!aligned(x, 16) || !aligned(out0, 16) || (op != 0 && !aligned(out1, 16))) {
    set_error("efl_ss_noise: buffers must be 16-byte aligned");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!(divisor == divisor) || divisor == 0.0f) { set_error("efl_ss_noise: divisor must be non-zero"); return EFL_E_INVALID_ARGUMENT; }
  const long long lanes = (n + 3) / 4;
  if (!lanes_ok(lanes)) { set_error("efl_ss_noise: tensor too large"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  // divisor 1: no division; a power of two with a normal reciprocal: times the reciprocal (the same
  // correctly rounded value); otherwise the division
  int ex = 0;
  const bool pow2 = std::isfinite(divisor) && std::frexp(std::fabs(divisor), &ex) == 0.5f &&
                    std::isnormal(1.0f / divisor);
  const int dv = divisor == 1.0f ? 0 : pow2 ? 1 : 2;
  const float d = dv == 1 ? 1.0f / divisor : divisor;
  if (op != 0 && g_noise_half.load(std::memory_order_relaxed)) {
    const unsigned grid = (unsigned)(((lanes + 31) / 32 * 64 + kBlock - 1) / kBlock);
    const int st = g_mask_store[1].load(std::memory_order_relaxed);
#define EFL_NH(OP, DV) \
    (st == 7 ? k_noise_half<OP, DV, 7> : st == 2 ? k_noise_half<OP, DV, 2> : k_noise_half<OP, DV, 0>)
    auto* kern = op == 1 ? (dv == 0 ? EFL_NH(1, 0) : dv == 1 ? EFL_NH(1, 1) : EFL_NH(1, 2))
                         : (dv == 0 ? EFL_NH(2, 0) : dv == 1 ? EFL_NH(2, 1) : EFL_NH(2, 2));
#undef EFL_NH
    kern<<<grid, kBlock, 0, s>>>(x, out0, out1, n, seed, ctr0, d);
    return hip_status(hipGetLastError(), "efl_ss_noise");
  }
  const int fam = op == 0 ? 0 : 1;
  const int nb = g_mask_blocks[fam].load(std::memory_order_relaxed);
  const int st = g_mask_store[fam].load(std::memory_order_relaxed);
#define EFL_NOISE_OP(OPD) EFL_MASK_LAUNCH(nb, st, lanes, s, OPD, x, out0, out1, n, seed, ctr0, d)
  switch (op * 3 + dv) {
    case 0: EFL_NOISE_OP(EFL_K_NOISE0D0); break;
    case 1: EFL_NOISE_OP(EFL_K_NOISE0D1); break;
    case 2: EFL_NOISE_OP(EFL_K_NOISE0D2); break;
    case 3: EFL_NOISE_OP(EFL_K_NOISE1D0); break;
    case 4: EFL_NOISE_OP(EFL_K_NOISE1D1); break;
    case 5: EFL_NOISE_OP(EFL_K_NOISE1D2); break;
    case 6: EFL_NOISE_OP(EFL_K_NOISE2D0); break;
    case 7: EFL_NOISE_OP(EFL_K_NOISE2D1); break;
    default: EFL_NOISE_OP(EFL_K_NOISE2D2); break;
  }
#undef EFL_NOISE_OP
  return hip_status(hipGetLastError(), "efl_ss_noise");
}

EFL_API int efl_ss_mask_cols(const float* a, float* send, float* keep0, float* keep1, int64_t rows,
                             int64_t cols, uint64_t seed, uint64_t ctr0, void* stream) {
  if (rows < 0 || cols < 0 || (cols & 1)) {
    set_error("secret_sharing mode A: the columns of a must be even, got [%lld, %lld]", (long long)rows, (long long)cols);
    return EFL_E_INVALID_ARGUMENT;
  }
  if (rows == 0 || cols == 0) return EFL_OK;
  if (!a || !send || !keep0 || !keep1) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  const bool v4 = cols % 8 == 0 && aligned(a, 16) && aligned(send, 16) && aligned(keep0, 16) && aligned(keep1, 8);
  const long long lanes = v4 ? rows * (cols / 4) : rows * (cols / 2);
  if (!lanes_ok(lanes)) { set_error("efl_ss_mask_cols: tensor too large"); return EFL_E_INVALID_ARGUMENT; }
  if (v4) {
    uint32_t dm;
    int ds;
    group_magic(lanes, cols / 4, &dm, &ds);
    EFL_MASK_LAUNCH(g_mask_blocks[2].load(std::memory_order_relaxed), g_mask_store[2].load(std::memory_order_relaxed),
                    lanes, s, EFL_K_COLS4, a, send, keep0, keep1, rows, cols, seed, ctr0, dm, ds);
  }
  else k_mask_cols2<<<grid_for(lanes), kBlock, 0, s>>>(a, send, keep0, keep1, rows, cols, seed, ctr0);
  return hip_status(hipGetLastError(), "efl_ss_mask_cols");
}

EFL_API int efl_ss_mask_rows(const float* b, float* send, float* keep0, float* keep1, int64_t rows,
                             int64_t cols, uint64_t seed, uint64_t ctr0, void* stream) {
  if (rows < 0 || cols < 0 || (rows & 1)) {
    set_error("secret_sharing mode B: the rows of b must be even, got [%lld, %lld]", (long long)rows, (long long)cols);
    return EFL_E_INVALID_ARGUMENT;
  }
  if (rows == 0 || cols == 0) return EFL_OK;
  if (!b || !send || !keep0 || !keep1) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  const bool v4 = cols % 4 == 0 && aligned(b, 16) && aligned(send, 16) && aligned(keep0, 16) && aligned(keep1, 16);
  const long long lanes = (rows / 2) * (v4 ? cols / 4 : cols);
  if (!lanes_ok(lanes)) { set_error("efl_ss_mask_rows: tensor too large"); return EFL_E_INVALID_ARGUMENT; }
  uint32_t dm;
  int ds;
  group_magic(lanes, v4 ? cols / 4 : cols, &dm, &ds);
  if (v4 && g_rows_half.load(std::memory_order_relaxed)) {
    // a wave per 32 NB lane groups: (waves x 64) threads
    const int nb = g_mask_blocks[3].load(std::memory_order_relaxed);
    const long long waves = (lanes + 32 * nb - 1) / (32 * nb);
    EFL_MASK_LAUNCH(nb, g_mask_store[3].load(std::memory_order_relaxed), waves * 64 * nb, s, EFL_K_ROWSH, b, send,
                    keep0, keep1, rows, cols, seed, ctr0, dm, ds);
  } else if (v4)
    EFL_MASK_LAUNCH(g_mask_blocks[3].load(std::memory_order_relaxed), g_mask_store[3].load(std::memory_order_relaxed),
                    lanes, s, EFL_K_ROWS4, b, send, keep0, keep1, rows, cols, seed, ctr0, dm, ds);
  else k_mask_rows<1, 1, 0><<<grid_for(lanes), kBlock, 0, s>>>(b, send, keep0, keep1, rows, cols, seed, ctr0, dm, ds);
  return hip_status(hipGetLastError(), "efl_ss_mask_rows");
}

EFL_API int efl_dp_noise(const float* x, float* out, int64_t n, int mode, float sigma, float divisor, uint64_t seed,
                         uint64_t ctr0, void* stream) {
  if (n < 0) { set_error("negative element count"); return EFL_E_INVALID_ARGUMENT; }
  if (mode < 0 || mode > 1) { set_error("efl_dp_noise: mode must be 0 (element-wise) or 1 (Gaussian sum)"); return EFL_E_INVALID_ARGUMENT; }
  if (!(divisor == divisor) || divisor == 0.0f) { set_error("efl_dp_noise: divisor must be non-zero"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  if (!x || !out) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  if (!aligned(x, 16) || !aligned(out, 16)) { set_error("efl_dp_noise: buffers must be 16-byte aligned"); return EFL_E_INVALID_ARGUMENT; }
  const long long lanes = (n + 3) / 4;
  if (!lanes_ok(lanes)) { set_error("efl_dp_noise: tensor too large"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  int ex = 0;
  const bool pow2 = std::isfinite(divisor) && std::frexp(std::fabs(divisor), &ex) == 0.5f &&
                    std::isnormal(1.0f / divisor);
  const float d = pow2 ? 1.0f / divisor : divisor;   // exact for a power of two with a normal reciprocal
  const int nb = g_dp_blocks.load(std::memory_order_relaxed);
  if (mode == 0 && pow2) launch_dp<0, true>(nb, lanes, x, out, n, seed, ctr0, sigma, d, s);
  else if (mode == 0) launch_dp<0, false>(nb, lanes, x, out, n, seed, ctr0, sigma, d, s);
  else if (pow2) launch_dp<1, true>(nb, lanes, x, out, n, seed, ctr0, sigma, d, s);
  else launch_dp<1, false>(nb, lanes, x, out, n, seed, ctr0, sigma, d, s);
  return hip_status(hipGetLastError(), "efl_dp_noise");
}
