// Stage F — fixed-point codec of EFLS-train's forward-encryption path, as streaming HIP kernels
// for MI355X (gfx950).
//
// Reference: efls-train/cc/efl/math/fixed_point.cc
//   encode  Convert2FixedPointOp<T>::Compute          :53-69 (int), :106-138 (float), :156-188 (double)
//   decode  FixedPointToFloatPointOp<int64|string, T> :235-248 (GMP mpf), Input2Mpf :255-265
//
// Both directions are pure streams: per fp32 element encode reads 4 B and
// writes 16 B, decode reads 16 B and writes 4 B — 40 algorithmic bytes per element for
// encrypt+decrypt, no reuse, so the roofline is HBM bandwidth and the kernels are built to keep
// every wave instruction a contiguous 16-B-per-lane access:
//   * "pair" layout (default): lane i of a 64-lane wave owns elements 2i, 2i+1 of its 128-element
//     stripe, so the int64 M/E streams (the 4x-wide side) move as one contiguous 1 KiB
//     global_{load,store}_dwordx4 per wave instruction; the fp32 side moves as dwordx2.
//   * "quad" layout: lane owns 4 consecutive elements: dwordx4 on the fp32 side, the int64 side as
//     two dwordx4 per lane at a 32-B lane stride.
// No LDS, no MFMA (there is no reuse and no contraction). Branch-free integer arithmetic on the
// IEEE bit patterns; the decode reproduces GMP's truncating mpf_get_d exactly (see dec_bits).
#include "common.h"

#include <atomic>
#include <type_traits>

namespace efl {
namespace {

// ------------------------------------------------------------------------------------------
// element transforms
// ------------------------------------------------------------------------------------------

// fixed_point.cc:108-136 for one fp32 bit pattern (SURVEY.md Appendix A rules A1-A6).
__device__ __forceinline__ void enc_f32(uint32_t b, bool dp, long long& M, long long& E) {
  int exp = (int)((b >> 23) & 0xFFu) - 150;                 // A1: unbiased, minus 23
  int mant = (int)(b & 0x7FFFFFu) | (exp != 0 ? 0x800000 : 0);   // A3: test on shifted exp
  if (dp) {                                                 // A4
    mant >>= 13;
    exp += 13;
  }
  // A5: r = ctz(mant); mant == 0 is the reference's UB shift, defined as M = 0, E = exp - 127.
  const int r = mant ? __builtin_ctz((unsigned)mant) : -127;
  mant = (int)((unsigned)mant >> (r & 31));
  exp += r;
  const int sm = (b >> 31) ? -mant : mant;                  // A6
  M = (long long)sm;
  E = (long long)exp;
}

// fixed_point.cc:158-186 for one fp64 bit pattern.
__device__ __forceinline__ void enc_f64(unsigned long long b, bool dp, long long& M, long long& E) {
  long long exp = (long long)((b >> 52) & 0x7FFull) - 1075;
  long long mant = (long long)(b & 0xFFFFFFFFFFFFFull) | (exp != 0 ? 0x10000000000000ll : 0);
  if (dp) {
    mant >>= 42;
    exp += 42;
  }
  const int r = mant ? __builtin_ctzll((unsigned long long)mant) : -1023;
  mant = (long long)((unsigned long long)mant >> (r & 63));
  exp += r;
  M = (b >> 63) ? -mant : mant;
  E = exp;
}

// GMP mpf_get_d of (-1)^s * a * 2^e with the exact value, a = |M| (fixed_point.cc:238-245:
// mpf_set_z, mpf_mul_2exp / mpf_div_2exp are exact for one limb; mpf_get_d truncates):
//   leading-bit position L >= 1024 -> +-inf; -1022..1023 normal (top 53 bits, truncated);
//   -1074..-1023 denormal (truncated, sign kept); <= -1075 -> +0.0.
__device__ __forceinline__ unsigned long long get_d_bits(unsigned long long a, bool neg, long long e) {
  if (a == 0) return 0ull;
  const unsigned long long sgn = neg ? 0x8000000000000000ull : 0ull;
  const int p = 63 - __clzll((long long)a);
  const long long ec = e > 4096 ? 4096 : (e < -8192 ? -8192 : e);
  const long long L = p + ec;
  if (L >= 1024) return sgn | 0x7FF0000000000000ull;
  if (L <= -1075) return 0ull;
  const unsigned long long m53 = p >= 52 ? (a >> (p - 52)) : (a << (52 - p));
  unsigned long long bits;
  if (L >= -1022)
    bits = ((unsigned long long)(L + 1023) << 52) | (m53 & 0xFFFFFFFFFFFFFull);
  else
    bits = m53 >> (int)(-1022 - L);
  return sgn | bits;
}

__device__ __forceinline__ unsigned long long dec_bits(long long M, long long E) {
  const unsigned long long a = M < 0 ? 0ull - (unsigned long long)M : (unsigned long long)M;
  return get_d_bits(a, M < 0, E);
}

// implicit double -> float of fixed_point.cc:245 (round to nearest even, IEEE denormals).
// ftz: TF threadpool MXCSR FTZ|DAZ: |d| < 2^-126 - 2^-151 -> zero of d's sign.
__device__ __forceinline__ float d2f(unsigned long long dbits, bool ftz) {
  constexpr unsigned long long kTiny = 0x380FFFFFF0000000ull;   // 0x1.ffffffp-127
  if (ftz && (dbits & 0x7FFFFFFFFFFFFFFFull) < kTiny)
    return __uint_as_float((unsigned)(dbits >> 32) & 0x80000000u);
  return (float)__longlong_as_double((long long)dbits);
}

// Fast path of get_d_bits. For |M| < 2^53 and E >= -1022 the value M * 2^E is exact in a double
// (normal, zero, or >= 2^1024 where both GMP and the hardware give +-inf), so GMP's truncation
// never acts and mpf_get_d == ldexp((double)M, E) bit for bit: an exact int64 -> f64 convert and
// one v_ldexp_f64 instead of the bit-by-bit rebuild. Every mantissa ConvertToFixedPoint<float>
// produces takes it (|M| < 2^24, E >= -277); anything else falls back to dec_bits.
__device__ __forceinline__ bool dec_fast_ok(long long M, long long E) {
  return (unsigned long long)M + (1ull << 53) < (1ull << 54) && E >= -1022;
}
__device__ __forceinline__ unsigned long long dec_fast_bits(long long M, long long E) {
  const int e = E > 4096 ? 4096 : (int)E;   // anything past 2^1024 is inf already
  return (unsigned long long)__double_as_longlong(ldexp((double)M, e));
}
__device__ __forceinline__ unsigned long long dec_any_bits(long long M, long long E) {
  return dec_fast_ok(M, E) ? dec_fast_bits(M, E) : dec_bits(M, E);
}

// ------------------------------------------------------------------------------------------
// memory helpers (NT bit 0: nontemporal loads, bit 1: nontemporal stores, bit 2 (with bit 1):
// 16-B stores as `global_store_dwordx4 ... nt sc1`, which also drop the line from the XCD's L2
// (MI355X_MICROARCH.md, store flavours) so the next kernel inherits no dirty encode output)
// ------------------------------------------------------------------------------------------

typedef int i4 __attribute__((ext_vector_type(4)));

template <int NT, class T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT, class T>
__device__ __forceinline__ void st(T* p, T v) {
  if constexpr ((NT & 4) && sizeof(T) == 16) {
    const i4 w = __builtin_bit_cast(i4, v);
    // The compiler's hazard recognizer does not see a store inside inline asm: a VALU write to
    // the data VGPRs right after a >8-byte store needs a wait state on gfx950, so pad it here.
    // tests/test_isa_guard.py checks every such store in the built library keeps its s_nop.
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr ((NT & 4) && sizeof(T) == 8) {
    const i2 w = __builtin_bit_cast(i2, v);
    asm volatile("global_store_dwordx2 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr (NT & 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// ------------------------------------------------------------------------------------------
// per-"unit" ops. A unit is 2 (pair) or 4 (quad) consecutive elements; each op knows how to
// load a unit, transform it and store it. `scalar` handles the ragged tail / unaligned case.
// ------------------------------------------------------------------------------------------

struct EncArgs {
  const void* x;
  long long* M;
  long long* E;
  int flag;       // decrease_precision
  int e_first;    // fp32 streaming encode: store the exponent pair before the mantissa pair
};
struct DecArgs {
  const long long* M;
  const long long* E;
  void* y;
  int flag;   // EFL_FXP_FTZ
};

struct EncF32Pair {
  using Args = EncArgs;
  static constexpr int kElems = 2;
  using In = f2;
  template <int NT> __device__ static In load(const Args& a, long long u) { return ld<NT>((const f2*)a.x + u); }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    long long m0, e0, m1, e1;
    enc_f32(__float_as_uint(v.x), a.flag, m0, e0);
    enc_f32(__float_as_uint(v.y), a.flag, m1, e1);
    if (a.e_first) {
      st<NT>((ll2*)a.E + u, ll2{e0, e1});
      st<NT>((ll2*)a.M + u, ll2{m0, m1});
    } else {
      st<NT>((ll2*)a.M + u, ll2{m0, m1});
      st<NT>((ll2*)a.E + u, ll2{e0, e1});
    }
  }
  __device__ static void scalar(const Args& a, long long i) {
    long long m, e;
    enc_f32(__float_as_uint(((const float*)a.x)[i]), a.flag, m, e);
    a.M[i] = m;
    a.E[i] = e;
  }
};

struct EncF32Quad {
  using Args = EncArgs;
  static constexpr int kElems = 4;
  using In = f4;
  template <int NT> __device__ static In load(const Args& a, long long u) { return ld<NT>((const f4*)a.x + u); }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    long long m0, e0, m1, e1, m2, e2, m3, e3;
    enc_f32(__float_as_uint(v.x), a.flag, m0, e0);
    enc_f32(__float_as_uint(v.y), a.flag, m1, e1);
    enc_f32(__float_as_uint(v.z), a.flag, m2, e2);
    enc_f32(__float_as_uint(v.w), a.flag, m3, e3);
    st<NT>((ll2*)a.M + 2 * u, ll2{m0, m1});
    st<NT>((ll2*)a.M + 2 * u + 1, ll2{m2, m3});
    st<NT>((ll2*)a.E + 2 * u, ll2{e0, e1});
    st<NT>((ll2*)a.E + 2 * u + 1, ll2{e2, e3});
  }
  __device__ static void scalar(const Args& a, long long i) { EncF32Pair::scalar(a, i); }
};

struct EncF64Pair {
  using Args = EncArgs;
  static constexpr int kElems = 2;
  using In = ll2;
  template <int NT> __device__ static In load(const Args& a, long long u) { return ld<NT>((const ll2*)a.x + u); }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    long long m0, e0, m1, e1;
    enc_f64((unsigned long long)v.x, a.flag, m0, e0);
    enc_f64((unsigned long long)v.y, a.flag, m1, e1);
    st<NT>((ll2*)a.M + u, ll2{m0, m1});
    st<NT>((ll2*)a.E + u, ll2{e0, e1});
  }
  __device__ static void scalar(const Args& a, long long i) {
    long long m, e;
    enc_f64(((const unsigned long long*)a.x)[i], a.flag, m, e);
    a.M[i] = m;
    a.E[i] = e;
  }
};

// Int2FixedPoint (fixed_point.cc:53-69): M = x, E = 0.
template <class T, class V2>
struct EncIntPair {
  using Args = EncArgs;
  static constexpr int kElems = 2;
  using In = V2;
  template <int NT> __device__ static In load(const Args& a, long long u) { return ld<NT>((const V2*)a.x + u); }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    st<NT>((ll2*)a.M + u, ll2{(long long)v.x, (long long)v.y});
    st<NT>((ll2*)a.E + u, ll2{0, 0});
  }
  __device__ static void scalar(const Args& a, long long i) {
    a.M[i] = (long long)((const T*)a.x)[i];
    a.E[i] = 0;
  }
};

struct DecF32Pair {
  using Args = DecArgs;
  static constexpr int kElems = 2;
  struct In { ll2 m, e; };
  template <int NT> __device__ static In load(const Args& a, long long u) {
    return In{ld<NT>((const ll2*)a.M + u), ld<NT>((const ll2*)a.E + u)};
  }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    const bool ftz = a.flag & EFL_FXP_FTZ;
    f2 r{d2f(dec_any_bits(v.m.x, v.e.x), ftz), d2f(dec_any_bits(v.m.y, v.e.y), ftz)};
    st<NT>((f2*)a.y + u, r);
  }
  __device__ static void scalar(const Args& a, long long i) {
    ((float*)a.y)[i] = d2f(dec_any_bits(a.M[i], a.E[i]), a.flag & EFL_FXP_FTZ);
  }
};

struct DecF32Quad {
  using Args = DecArgs;
  static constexpr int kElems = 4;
  struct In { ll2 m0, m1, e0, e1; };
  template <int NT> __device__ static In load(const Args& a, long long u) {
    const ll2* M = (const ll2*)a.M + 2 * u;
    const ll2* E = (const ll2*)a.E + 2 * u;
    return In{ld<NT>(M), ld<NT>(M + 1), ld<NT>(E), ld<NT>(E + 1)};
  }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    const bool ftz = a.flag & EFL_FXP_FTZ;
    f4 r{d2f(dec_any_bits(v.m0.x, v.e0.x), ftz), d2f(dec_any_bits(v.m0.y, v.e0.y), ftz),
         d2f(dec_any_bits(v.m1.x, v.e1.x), ftz), d2f(dec_any_bits(v.m1.y, v.e1.y), ftz)};
    st<NT>((f4*)a.y + u, r);
  }
  __device__ static void scalar(const Args& a, long long i) { DecF32Pair::scalar(a, i); }
};

struct DecF64Pair {
  using Args = DecArgs;
  static constexpr int kElems = 2;
  struct In { ll2 m, e; };
  template <int NT> __device__ static In load(const Args& a, long long u) {
    return In{ld<NT>((const ll2*)a.M + u), ld<NT>((const ll2*)a.E + u)};
  }
  template <int NT> __device__ static void apply(const Args& a, long long u, In v) {
    ll2 r{(long long)dec_any_bits(v.m.x, v.e.x), (long long)dec_any_bits(v.m.y, v.e.y)};
    st<NT>((ll2*)a.y + u, r);
  }
  __device__ static void scalar(const Args& a, long long i) {
    ((unsigned long long*)a.y)[i] = dec_any_bits(a.M[i], a.E[i]);
  }
};

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------

// Streaming kernel: tiles of B*K units; a workgroup walks tiles blockIdx.x, +gridDim.x, ...
// Inside a full tile every lane issues its K loads back to back before any store, then transforms
// and stores. Tile t of a wave touches one contiguous span.
// xcd_per > 0: XCD-aware tile order. Workgroups are dispatched round-robin over the 8 XCDs
// (blockIdx % 8); workgroup b then takes tile (b % 8) * xcd_per + b / 8, so each XCD streams one
// contiguous eighth of the tensor instead of every eighth tile (gridDim.x = 8 * xcd_per).
// Kernel arguments as plain scalars (p0, p1, p2 = x, M, E for encode; M, E, y for decode), not the
// Args struct: scalars can be preloaded into SGPRs at wave launch (the Makefile builds this file with
// kernarg preload), and the empty asm below makes every argument the kernel reads arrive in one
// scalar round trip otherwise. Passing the struct, the compiler loaded xcd_per, waited and branched,
// then loaded nunits, waited and branched, then loaded the pointers: three dependent round trips
// at the head of every workgroup before its first data load (round 6, from the ISA).
template <class Args>
__device__ __forceinline__ Args make_args(const void* p0, const void* p1, void* p2, int flag, int e_first) {
  if constexpr (std::is_same<Args, EncArgs>::value) {
    return EncArgs{p0, (long long*)p1, (long long*)p2, flag, e_first};
  } else {
    return DecArgs{(const long long*)p0, (const long long*)p1, p2, flag};
  }
}
struct RawArgs {
  const void* p0;
  const void* p1;
  void* p2;
  int flag, e_first;
};
inline RawArgs raw_args(const EncArgs& a) { return {a.x, a.M, a.E, a.flag, a.e_first}; }
inline RawArgs raw_args(const DecArgs& a) { return {a.M, a.E, a.y, a.flag, 0}; }

template <class Op, int B, int K, int NT>
__global__ __launch_bounds__(B) void k_stream(const void* p0, const void* p1, void* p2, int flag, int e_first,
                                              long long nunits, int xcd_per) {
  asm volatile("" ::"s"(p0), "s"(p1), "s"(p2), "s"(flag), "s"(e_first), "s"(nunits), "s"(xcd_per));
  const typename Op::Args a = make_args<typename Op::Args>(p0, p1, p2, flag, e_first);
  const long long tile = (long long)B * K;
  const long long t0 = xcd_per > 0 ? (long long)(blockIdx.x & 7u) * xcd_per + (blockIdx.x >> 3) : blockIdx.x;
  for (long long base = t0 * tile; base < nunits;
       base += (long long)gridDim.x * tile) {
    typename Op::In v[K];
    if (base + tile <= nunits) {
#pragma unroll
      for (int k = 0; k < K; ++k) v[k] = Op::template load<NT>(a, base + k * B + threadIdx.x);
      // keep every load of the tile issued before any of the transform: without this fence the
      // scheduler may start converting the first stream and wait for it before issuing the second
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < K; ++k) Op::template apply<NT>(a, base + k * B + threadIdx.x, v[k]);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const long long u = base + k * B + threadIdx.x;
        if (u < nunits) v[k] = Op::template load<NT>(a, u);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const long long u = base + k * B + threadIdx.x;
        if (u < nunits) Op::template apply<NT>(a, u, v[k]);
      }
    }
  }
}

// Element-at-a-time kernel for the ragged tail and for unaligned buffers.
template <class Op>
__global__ __launch_bounds__(kBlock) void k_scalar(typename Op::Args a, long long start, long long n) {
  for (long long i = start + (long long)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock)
    Op::scalar(a, i);
}

// Batched (BASELINE config 3): tile `x` of tensor `t`, one launch for `count` tensors. Arrays of
// pointers / sizes live in device memory (t is wave-uniform: scalar loads). Same tile shape as
// k_stream (B lanes x K units, every load of a full tile issued before the transform).
// T > 1: the workgroup walks T consecutive tiles of its tensor (xg = tile group). Round 6 PMC
// (profiles/r06/c3_pmc*.json): per launch over the bench's 4,096 separate slices the batched kernels
// take 90-126 k UTCL1 translation misses (and 2.6-3.4 M misses under miss) against 20-374 for the
// streaming kernels over the same bytes in large allocations: every short workgroup pays its own
// translation of the small fragments its 8-16 KiB of each stream sit in. A workgroup covering T
// tiles pays it once per T tiles.
template <class Op, int B, int K, int NT, int T = 1>
__device__ __forceinline__ void batched_tile(const void* const* src, void* const* dst0, void* const* dst1,
                                             const long long* ns, int flag, long long t, long long xg) {
  // All four table entries in one scalar round trip. Left alone, the compiler loads ns[t], waits,
  // branches on it, and only then loads the three pointers: a second dependent L2 round trip at the
  // head of every workgroup, which the streaming kernel does not pay (round 6: per-launch the
  // batched kernels ran 4-6 % behind k_stream on the same contiguous bytes). The empty asm needs
  // all four values in SGPRs, so the loads issue together and one s_waitcnt covers them.
  const long long n = ns[t];
  const void* sp = src[t];
  void* p0 = dst0[t];
  void* p1 = dst1[t];
  asm volatile("" ::"s"(n), "s"(sp), "s"(p0), "s"(p1));
  typename Op::Args a;
  if constexpr (std::is_same<typename Op::Args, EncArgs>::value) {
    a = EncArgs{sp, (long long*)p0, (long long*)p1, flag};
  } else {
    a = DecArgs{(const long long*)sp, (const long long*)p0, p1, flag};
  }
  const long long tile = (long long)B * K * Op::kElems;
  // 16-B alignment of this tensor's streams decides vector vs element path (uniform branch).
  const bool vec = aligned(sp, 16) && aligned(p0, 16) && aligned(p1, 16);
  const long long nunits = n / Op::kElems;
#pragma unroll 1
  for (int st = 0; st < T; ++st) {
  const long long x = xg * T + st;
  const long long e0 = x * tile;
  if (e0 >= n) return;
  const long long u0 = x * B * K;
  if (vec) {
    typename Op::In v[K];
    if (u0 + (long long)B * K <= nunits) {
#pragma unroll
      for (int k = 0; k < K; ++k) v[k] = Op::template load<NT>(a, u0 + k * B + threadIdx.x);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < K; ++k) Op::template apply<NT>(a, u0 + k * B + threadIdx.x, v[k]);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const long long u = u0 + k * B + threadIdx.x;
        if (u < nunits) v[k] = Op::template load<NT>(a, u);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const long long u = u0 + k * B + threadIdx.x;
        if (u < nunits) Op::template apply<NT>(a, u, v[k]);
      }
    }
    // ragged tail (< kElems elements) of this tensor, handled by the tile that owns it
    const long long tail0 = nunits * Op::kElems;
    if (tail0 < n && tail0 >= e0 && tail0 < e0 + tile) {
      if (threadIdx.x < n - tail0) Op::scalar(a, tail0 + threadIdx.x);
    }
  } else {
    for (long long i = e0 + threadIdx.x; i < n && i < e0 + tile; i += B) Op::scalar(a, i);
  }
  }
}

// 2-D grid: blockIdx.y = tensor (from tile_base), blockIdx.x = group of T tiles of that tensor.
template <class Op, int B, int K, int NT, int T = 1>
__global__ __launch_bounds__(B) void k_batched(const void* const* src, void* const* dst0,
                                               void* const* dst1, const long long* ns,
                                               int flag, long long tile_base) {
  batched_tile<Op, B, K, NT, T>(src, dst0, dst1, ns, flag, tile_base + blockIdx.y, blockIdx.x);
}

// 1-D grid over count x gx tiles (tensor-major), XCD-aware like k_stream: workgroups are dispatched
// round-robin over the 8 XCDs, and workgroup b takes linear tile (b % 8) * per + b / 8, so each XCD
// streams one contiguous eighth of the tensors (and of their tiles) instead of every eighth tile.
template <class Op, int B, int K, int NT>
__global__ __launch_bounds__(B) void k_batched_flat(const void* const* src, void* const* dst0,
                                                    void* const* dst1, const long long* ns, int flag,
                                                    long long gx, long long total, long long per) {
  const long long lin = per > 0 ? (long long)(blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;
  if (lin >= total) return;
  batched_tile<Op, B, K, NT>(src, dst0, dst1, ns, flag, lin / gx, lin % gx);
}

// Persistent batched walk: gridDim.x workgroups over the count x gx tiles (tensor-major), workgroup
// b taking tiles b, b + grid, ... The NEXT tile's pointer-table entries and data loads are issued
// before the current tile's transform and stores (software pipelining), so a tile exposes neither
// the table latency nor its data latency. Full, aligned tiles take that path; the others (ragged
// ends, unaligned tensors) go through batched_tile.
template <class Op, int B, int K>
__device__ __forceinline__ bool persist_setup(const void* const* src, void* const* dst0, void* const* dst1,
                                              const long long* ns, int flag, long long lin, long long gx,
                                              typename Op::Args& a, long long& u0) {
  const long long t = lin / gx, x = lin % gx;
  const long long n = ns[t];
  if constexpr (std::is_same<typename Op::Args, EncArgs>::value) {
    a = EncArgs{src[t], (long long*)dst0[t], (long long*)dst1[t], flag};
  } else {
    a = DecArgs{(const long long*)src[t], (const long long*)dst0[t], dst1[t], flag};
  }
  u0 = x * B * K;
  return aligned(src[t], 16) && aligned(dst0[t], 16) && aligned(dst1[t], 16) &&
         u0 + (long long)B * K <= n / Op::kElems;
}

template <class Op, int B, int K, int NT>
__global__ __launch_bounds__(B) void k_batched_persist(const void* const* src, void* const* dst0,
                                                       void* const* dst1, const long long* ns, int flag,
                                                       long long gx, long long total) {
  long long lin = blockIdx.x;
  if (lin >= total) return;
  typename Op::Args a;
  long long u0;
  bool fast = persist_setup<Op, B, K>(src, dst0, dst1, ns, flag, lin, gx, a, u0);
  typename Op::In v[K];
  if (fast) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = Op::template load<NT>(a, u0 + k * B + threadIdx.x);
  }
  for (;;) {
    const long long nxt = lin + gridDim.x;
    typename Op::Args an;
    long long un = 0;
    bool fn = false;
    typename Op::In vn[K];
    if (nxt < total) {
      fn = persist_setup<Op, B, K>(src, dst0, dst1, ns, flag, nxt, gx, an, un);
      if (fn) {
#pragma unroll
        for (int k = 0; k < K; ++k) vn[k] = Op::template load<NT>(an, un + k * B + threadIdx.x);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (fast) {
#pragma unroll
      for (int k = 0; k < K; ++k) Op::template apply<NT>(a, u0 + k * B + threadIdx.x, v[k]);
    } else {
      batched_tile<Op, B, K, NT>(src, dst0, dst1, ns, flag, lin / gx, lin % gx);
    }
    if (nxt >= total) break;
    lin = nxt;
    a = an;
    u0 = un;
    fast = fn;
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = vn[k];
  }
}

// Hex mantissa decode (FixedPointToFloatPointOp<string, T>, fixed_point.cc:255-257): one lane per
// string; keeps the leading 64 bits of |m| and its bit length (mpf truncation composes to that).
template <bool F64>
__global__ __launch_bounds__(kBlock) void k_decode_hex(const char* chars, const long long* offs,
                                                       const long long* E, void* y, long long n,
                                                       int flag, long long* bad) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  long long s = offs[i];
  const long long end = offs[i + 1];
  bool neg = false, ok = end > s;
  if (ok && chars[s] == '-') {
    neg = true;
    ++s;
    ok = end > s;
  }
  unsigned long long acc = 0;
  int nbits = 0;
  long long extra = 0;
  for (long long j = s; j < end; ++j) {
    const char c = chars[j];
    int v;
    if (c >= '0' && c <= '9') v = c - '0';
    else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v = c - 'A' + 10;
    else { ok = false; break; }
    if (nbits == 0) {
      if (v) { acc = (unsigned long long)v; nbits = 64 - __clzll((long long)acc); }
    } else if (nbits + 4 <= 64) {
      acc = (acc << 4) | (unsigned long long)v;
      nbits += 4;
    } else {
      const int room = 64 - nbits;
      if (room > 0) { acc = (acc << room) | ((unsigned long long)v >> (4 - room)); nbits = 64; }
      extra += 4 - room;
    }
  }
  if (!ok) {
    atomicMin((unsigned long long*)bad, (unsigned long long)i);
    if (F64) ((unsigned long long*)y)[i] = 0x7FF8000000000000ull;
    else ((unsigned*)y)[i] = 0x7FC00000u;
    return;
  }
  const unsigned long long d = get_d_bits(acc, neg && acc != 0, E[i] + extra);
  if (F64) ((unsigned long long*)y)[i] = d;
  else ((float*)y)[i] = d2f(d, flag & EFL_FXP_FTZ);
}

// ------------------------------------------------------------------------------------------
// launch configuration (tunable; see efl_fxp_tune)
// ------------------------------------------------------------------------------------------

// Per-direction launch shape of the fp32 kernels. Defaults: the fastest shape of the interleaved
// sweep on MI355X (tools/sweep_fxp.py -> profiles/r01/sweep_*.jsonl), pair layout, one tile per
// workgroup. Decode: 128 lanes, nontemporal loads (+5 % over plain loads; plain stores: `nt sc1`
// stores cost 4 % of the step, profiles/r02/step_probe_*.json). Encode: 512 lanes, nontemporal
// loads and `nt sc1` stores (NT mask 7): 256 lanes took the bench step from 0.209 to 0.197 ms over
// 128 lanes / plain stores, and 512 lanes another 1-2 % (step_probe, two boxes); `nt sc1` is
// 1.5-3 % below plain `nt` stores (profiles/r01/ab_*.json, tools/enc_probe.hip on the bare mix)
// and also takes decode's time down (no inherited dirty lines).
struct Shape {
  std::atomic<int> variant;   // 0 pair, 1 quad
  std::atomic<int> block;     // 128, 256, 512, 1024
  std::atomic<int> k;         // units per lane per tile: 1, 2
  std::atomic<int> nt;        // bit0 nontemporal loads, bit1 nontemporal stores
};
Shape g_shape[2] = {{{0}, {512}, {1}, {7}}, {{0}, {128}, {1}, {1}}};
std::atomic<int> g_grid_cap{0};   // 0: one tile per workgroup; else max workgroups
// efl_fxp_tune 14 / 15: XCD-aware tile order (k_stream). Decode on: its kernel 2.3 % and the step
// 1.2 % faster, encode off: 2.5 % slower (profiles/r02/step_probe_xcd_*.json, same box)
std::atomic<int> g_xcd_order[2] = {{0}, {1}};
std::atomic<int> g_e_first{0};                  // efl_fxp_tune 16: encode stores E before M
// NT mask of the fp32 batched encode (efl_fxp_tune kind 9): 1 nontemporal loads, 3 loads + stores,
// 7 loads + `nt sc1` stores (default, as the streaming encode)
std::atomic<int> g_batch_enc_nt{7};
constexpr int kEnc = 0, kDec = 1;
// batched tile (efl_fxp_encode_batched / decode_batched): B lanes x K pairs per workgroup
constexpr int kBatchB = 256, kBatchK = 4;
constexpr long long kMaxGridY = 65535;
// fp32 [encode, decode]: encode 512 lanes x 1 pair (the streaming encode's tile, one 1024-element
// tile per workgroup), decode 512 x 2. Rounds 3-5 ran 512 x 2 both ways; the per-launch A/B in one
// process (tools/config3_coalesce_probe.py, profiles/r05/c3_coalesce.jsonl, c3_same_box.jsonl) put
// the encode's 512 x 1 at -8 % on a slow box (0.2279 -> 0.2103 ms) and -0.5 % on a fast one, and the
// decode's 512 x 2 ahead of 512 x 1 on the fast box (0.2007 against 0.2085 ms); round 6 re-took the
// A/B interleaved (profiles/r06/c3_shapes.jsonl)
std::atomic<int> g_batch_block[2] = {{512}, {512}};
std::atomic<int> g_batch_k[2] = {{1}, {2}};
// efl_fxp_tune 17 / 18: tile order of the fp32 batched encode / decode: 0 2-D grid (tensor =
// blockIdx.y), 1 one flat tensor-major grid, 2 the flat grid in XCD-aware order
std::atomic<int> g_batch_order[2] = {{0}, {0}};
// efl_fxp_tune 26 / 27: tiles per workgroup of the fp32 batched encode / decode (2-D grid, 512-lane
// tiles; 1, 2, 4, 8): fewer, longer workgroups, each translating its tensor's pages once
std::atomic<int> g_batch_tiles[2] = {{1}, {1}};
// efl_fxp_tune 19: workgroups of the persistent batched walk (order 3)
std::atomic<int> g_batch_persist_grid{2048};
// The fp64 encode (8 B read, 16 B written per element) through its own shape: efl_fxp_tune kinds
// 21 workgroup size, 22 units per lane, 23 NT mask, 24 XCD-aware order. Round 4 ran it at the fp32
// encode's shape (512 lanes, 1 unit, NT 7, linear order): 0.79 of 8 TB/s. Round 5 sweep of all 36
// shapes, interleaved, median of 3 (tools/fp64_shape_probe.py, profiles/r05/fp64_shape.jsonl):
// 1024 lanes, 1 unit, NT 7 and the XCD-aware order 0.2508 ms (0.803) against 0.2547 ms (0.790).
Shape g_shape64 = {{0}, {1024}, {1}, {7}};
std::atomic<int> g_xcd64{1};

template <class Op, int B, int K, int NT>
hipError_t launch_k(const typename Op::Args& a, long long nunits, hipStream_t s, int xcd = 0) {
  const long long tile = (long long)B * K;
  long long grid = (nunits + tile - 1) / tile;
  const int cap = g_grid_cap.load(std::memory_order_relaxed);
  int xcd_per = 0;
  if (cap > 0 && grid > cap) grid = cap;
  else if (xcd && grid >= 64 && grid < 0x7FFFFFF0ll) {
    xcd_per = (int)((grid + 7) / 8);
    grid = 8ll * xcd_per;
  }
  if (grid > 0x7FFFFFFFll) grid = 0x7FFFFFFFll;
  if (grid == 0) return hipSuccess;
  const RawArgs r = raw_args(a);
  hipLaunchKernelGGL((k_stream<Op, B, K, NT>), dim3((unsigned)grid), dim3(B), 0, s, r.p0, r.p1, r.p2, r.flag,
                     r.e_first, nunits, xcd_per);
  return hipGetLastError();
}

template <class Op, int B, int K>
hipError_t launch_nt(int nt, const typename Op::Args& a, long long nunits, hipStream_t s, int xcd) {
  switch (nt) {
    case 1: return launch_k<Op, B, K, 1>(a, nunits, s, xcd);
    case 2: return launch_k<Op, B, K, 2>(a, nunits, s, xcd);
    case 3: return launch_k<Op, B, K, 3>(a, nunits, s, xcd);
    case 7: return launch_k<Op, B, K, 7>(a, nunits, s, xcd);
    default: return launch_k<Op, B, K, 0>(a, nunits, s, xcd);
  }
}

template <class Op, int B>
hipError_t launch_bk(const Shape& sh, const typename Op::Args& a, long long nunits, hipStream_t s, int xcd) {
  const int nt = sh.nt.load(std::memory_order_relaxed);
  return sh.k.load(std::memory_order_relaxed) == 2 ? launch_nt<Op, B, 2>(nt, a, nunits, s, xcd)
                                                   : launch_nt<Op, B, 1>(nt, a, nunits, s, xcd);
}

// tunable launch (fp32 ops; the fp64 encode through its own shape, g_shape64)
template <class Op>
hipError_t launch_tuned(const Shape& sh, const typename Op::Args& a, long long nunits, hipStream_t s, int xcd) {
  switch (sh.block.load(std::memory_order_relaxed)) {
    case 128: return launch_bk<Op, 128>(sh, a, nunits, s, xcd);
    case 512: return launch_bk<Op, 512>(sh, a, nunits, s, xcd);
    case 1024: return launch_bk<Op, 1024>(sh, a, nunits, s, xcd);
    default: return launch_bk<Op, 256>(sh, a, nunits, s, xcd);
  }
}

// fixed launch (fp64 / integer ops): the fp32 default shape of the same direction. Encode: 512
// lanes, nontemporal loads and `nt sc1` 16-B stores; decode: 128 lanes, nontemporal loads, XCD-aware
// tile order (round 1 ran both at 128 lanes with nontemporal loads only; tools/bench_fxp_dtypes.py,
// profiles/r02/fxp_dtypes.jsonl)
template <class Op>
hipError_t launch_fixed(int dir, const typename Op::Args& a, long long nunits, hipStream_t s) {
  if (dir == kEnc) return launch_k<Op, 512, 1, 7>(a, nunits, s);
  return launch_k<Op, 128, 1, 1>(a, nunits, s, 1);
}

template <class Op>
hipError_t launch_scalar(const typename Op::Args& a, long long start, long long n, hipStream_t s) {
  if (n <= start) return hipSuccess;
  long long grid = (n - start + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL((k_scalar<Op>), dim3((unsigned)grid), dim3(kBlock), 0, s, a, start, n);
  return hipGetLastError();
}

// vector path over the aligned prefix + scalar tail, or all-scalar when unaligned.
template <class Op, bool TUNED>
hipError_t run(int dir, const typename Op::Args& a, const void* p0, const void* p1, const void* p2,
               long long n, hipStream_t s) {
  const uintptr_t need = 16;
  if (aligned(p0, need) && aligned(p1, need) && aligned(p2, need)) {
    const long long nunits = n / Op::kElems;
    hipError_t e;
    if constexpr (std::is_same<Op, EncF64Pair>::value)
      e = launch_tuned<Op>(g_shape64, a, nunits, s, g_xcd64.load(std::memory_order_relaxed));
    else if constexpr (TUNED)
      e = launch_tuned<Op>(g_shape[dir], a, nunits, s, g_xcd_order[dir].load(std::memory_order_relaxed));
    else
      e = launch_fixed<Op>(dir, a, nunits, s);
    if (e != hipSuccess) return e;
    return launch_scalar<Op>(a, nunits * Op::kElems, n, s);
  }
  return launch_scalar<Op>(a, 0, n, s);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// error reporting
// ------------------------------------------------------------------------------------------

namespace {
thread_local std::string t_err;
}

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
}

int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return EFL_OK;
  set_error("%s: %s", what, hipGetErrorString(e));
  return EFL_E_INTERNAL;
}

}  // namespace efl

using namespace efl;

EFL_API const char* efl_last_error(void) { return t_err.c_str(); }

namespace efl {
// efl_fxp_tune(20, nb): Philox blocks per lane of the DP noise kernel (csrc/mask.hip; 1, 2, 4). 4:
// 0.669 / 0.685 of 8 TB/s against 0.594 / 0.366 for one block on two boxes (profiles/r03/bench_mask*)
std::atomic<int> g_dp_blocks{4};
// efl_fxp_tune(25, nb) / (28, st): lane groups (Philox blocks) per lane (1, 2, 4) and store flavour
// (0 plain, 2 nontemporal, 7 `nt sc1`) of the secret-sharing mask kernels, per family [noise (op 0),
// share / weight noise (ops 1, 2), mask_cols, mask_rows]; setting a kind sets all four. Defaults:
// the best of the round-6 sweep on three boxes (tools/bench_mask.py, profiles/r06/bench_mask*.jsonl):
// noise 2 / plain 0.87-0.90, share 1 / nt sc1 0.71-0.78, mask_cols 1 / nt 0.89, mask_rows 1 / nt sc1
// 0.67
std::atomic<int> g_mask_blocks[4] = {{2}, {1}, {1}, {1}};
std::atomic<int> g_mask_store[4] = {{0}, {7}, {2}, {7}};
std::atomic<int> g_rows_half{1};
std::atomic<int> g_noise_half{1};
}  // namespace efl

EFL_API int efl_fxp_tune(int kind, int value) {
  if (kind >= 21 && kind <= 24) {   // fp64 encode shape
    switch (kind) {
      case 21:
        if (value != 128 && value != 256 && value != 512 && value != 1024) return EFL_E_INVALID_ARGUMENT;
        return g_shape64.block.exchange(value);
      case 22:
        if (value != 1 && value != 2) return EFL_E_INVALID_ARGUMENT;
        return g_shape64.k.exchange(value);
      case 23:
        if (value < 0 || (value > 3 && value != 7)) return EFL_E_INVALID_ARGUMENT;
        return g_shape64.nt.exchange(value);
      default:
        if (value != 0 && value != 1) return EFL_E_INVALID_ARGUMENT;
        return g_xcd64.exchange(value);
    }
  }
  if (kind == 25 || kind == 28) {   // mask kernels: lane groups per lane / store flavour, every family
    std::atomic<int>* v = kind == 25 ? g_mask_blocks : g_mask_store;
    if (value == -1) return v[0].load();
    if (value == -2) {              // back to the per-family defaults
      static const int kDef[2][4] = {{2, 1, 1, 1}, {0, 7, 2, 7}};
      for (int f = 0; f < 4; ++f) v[f].store(kDef[kind == 25 ? 0 : 1][f]);
      return 0;
    }
    if (kind == 25 && value != 1 && value != 2 && value != 4) return EFL_E_INVALID_ARGUMENT;
    if (kind == 28 && value != 0 && value != 2 && value != 7) return EFL_E_INVALID_ARGUMENT;
    const int prev = v[0].load();
    for (int f = 0; f < 4; ++f) v[f].store(value);
    return prev;
  }
  if (kind == 20) {                 // DP noise kernel: Philox blocks per lane (csrc/mask.hip)
    if (value == -1) return g_dp_blocks.load();
    if (value != 1 && value != 2 && value != 4) return EFL_E_INVALID_ARGUMENT;
    return g_dp_blocks.exchange(value);
  }
  if (kind == 14 || kind == 15) {   // XCD-aware tile order, streaming fp32 encode / decode
    if (value != 0 && value != 1) return EFL_E_INVALID_ARGUMENT;
    return g_xcd_order[kind - 14].exchange(value);
  }
  if (kind == 16) {                 // streaming fp32 encode: exponent stores first
    if (value != 0 && value != 1) return EFL_E_INVALID_ARGUMENT;
    return g_e_first.exchange(value);
  }
  if (kind == 29 || kind == 30) {   // mask_rows / share + weight noise: one lane (0) or wave halves (1)
    std::atomic<int>& v = kind == 29 ? g_rows_half : g_noise_half;
    if (value == -1) return v.load();
    if (value != 0 && value != 1) return EFL_E_INVALID_ARGUMENT;
    return v.exchange(value);
  }
  if (kind == 26 || kind == 27) {   // batched fp32 encode / decode: tiles per workgroup
    std::atomic<int>& v = g_batch_tiles[kind - 26];
    if (value == -1) return v.load();
    if (value != 1 && value != 2 && value != 4 && value != 8) return EFL_E_INVALID_ARGUMENT;
    return v.exchange(value);
  }
  if (kind == 19) {                 // persistent batched walk: workgroups
    if (value < 1) return EFL_E_INVALID_ARGUMENT;
    return g_batch_persist_grid.exchange(value);
  }
  if (kind == 17 || kind == 18) {   // batched fp32 tile order: 0 2-D, 1 flat, 2 flat XCD-aware, 3 persistent
    if (value < 0 || value > 3) return EFL_E_INVALID_ARGUMENT;
    return g_batch_order[kind - 17].exchange(value);
  }
  if (kind >= 10 && kind <= 13) {   // batched fp32: 10/11 encode block/K, 12/13 decode block/K
    const int dir = kind >= 12 ? kDec : kEnc;
    if (value == -1) return kind % 2 == 0 ? g_batch_block[dir].load() : g_batch_k[dir].load();   // query
    if (kind % 2 == 0) {
      if (value != 128 && value != 256 && value != 512) return EFL_E_INVALID_ARGUMENT;
      return g_batch_block[dir].exchange(value);
    }
    if (value != 1 && value != 2 && value != 4) return EFL_E_INVALID_ARGUMENT;
    return g_batch_k[dir].exchange(value);
  }
  if (kind == 9) {
    if (value != 1 && value != 3 && value != 7) return EFL_E_INVALID_ARGUMENT;
    return g_batch_enc_nt.exchange(value);
  }
  if (kind == 8) {
    if (value < 0) return EFL_E_INVALID_ARGUMENT;
    return g_grid_cap.exchange(value);
  }
  if (kind < 0 || kind > 7) return EFL_E_INVALID_ARGUMENT;
  Shape& sh = g_shape[kind & 1];
  switch (kind >> 1) {
    case 0:
      if (value < 0 || value > 1) return EFL_E_INVALID_ARGUMENT;
      return sh.variant.exchange(value);
    case 1:
      if (value != 1 && value != 2) return EFL_E_INVALID_ARGUMENT;
      return sh.k.exchange(value);
    case 2:
      if (value < 0 || (value > 3 && value != 7)) return EFL_E_INVALID_ARGUMENT;
      return sh.nt.exchange(value);
    default:
      if (value != 128 && value != 256 && value != 512 && value != 1024) return EFL_E_INVALID_ARGUMENT;
      return sh.block.exchange(value);
  }
}

EFL_API int efl_fxp_encode(const void* x, int dtype, int64_t* mantissa, int64_t* exponent,
                           int64_t n, int decrease_precision, void* stream) {
  if (n < 0) { set_error("negative element count"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  if (!x || !mantissa || !exponent) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  EncArgs a{x, (long long*)mantissa, (long long*)exponent, decrease_precision ? 1 : 0,
            g_e_first.load(std::memory_order_relaxed)};
  hipError_t e;
  switch (dtype) {
    case EFL_DT_FLOAT:
      e = g_shape[kEnc].variant.load() == 1 ? run<EncF32Quad, true>(kEnc, a, x, mantissa, exponent, n, s)
                                            : run<EncF32Pair, true>(kEnc, a, x, mantissa, exponent, n, s);
      break;
    case EFL_DT_DOUBLE: e = run<EncF64Pair, false>(kEnc, a, x, mantissa, exponent, n, s); break;
    case EFL_DT_INT8: e = run<EncIntPair<signed char, c2>, false>(kEnc, a, x, mantissa, exponent, n, s); break;
    case EFL_DT_INT16: e = run<EncIntPair<short, s2>, false>(kEnc, a, x, mantissa, exponent, n, s); break;
    case EFL_DT_INT32: e = run<EncIntPair<int, i2>, false>(kEnc, a, x, mantissa, exponent, n, s); break;
    case EFL_DT_INT64: e = run<EncIntPair<long long, ll2>, false>(kEnc, a, x, mantissa, exponent, n, s); break;
    default:
      set_error("ConvertToFixedPoint: unsupported dtype %d (int8/16/32/64, float, double)", dtype);
      return EFL_E_INVALID_ARGUMENT;
  }
  return hip_status(e, "efl_fxp_encode");
}

EFL_API int efl_fxp_decode(const int64_t* mantissa, const int64_t* exponent, void* y, int dtype,
                           int64_t n_mantissa, int64_t n_exponent, int flags, void* stream) {
  if (n_mantissa != n_exponent) {
    set_error("mantissa and exponent should be the same size.");
    return EFL_E_INVALID_ARGUMENT;
  }
  const int64_t n = n_mantissa;
  if (n < 0) { set_error("negative element count"); return EFL_E_INVALID_ARGUMENT; }
  if (n == 0) return EFL_OK;
  if (!mantissa || !exponent || !y) { set_error("null buffer"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  DecArgs a{(const long long*)mantissa, (const long long*)exponent, y, flags};
  hipError_t e;
  switch (dtype) {
    case EFL_DT_FLOAT:
      e = g_shape[kDec].variant.load() == 1 ? run<DecF32Quad, true>(kDec, a, mantissa, exponent, y, n, s)
                                            : run<DecF32Pair, true>(kDec, a, mantissa, exponent, y, n, s);
      break;
    case EFL_DT_DOUBLE: e = run<DecF64Pair, false>(kDec, a, mantissa, exponent, y, n, s); break;
    default:
      set_error("FixedPointToFloatPoint: unsupported dtype %d (float, double)", dtype);
      return EFL_E_INVALID_ARGUMENT;
  }
  return hip_status(e, "efl_fxp_decode");
}

EFL_API int efl_fxp_decode_hex(const char* chars, const int64_t* offsets, const int64_t* exponent,
                               void* y, int dtype, int64_t n, int flags, int64_t* bad,
                               void* stream) {
  if (n < 0) { set_error("negative element count"); return EFL_E_INVALID_ARGUMENT; }
  if (!bad) { set_error("null status word"); return EFL_E_INVALID_ARGUMENT; }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(bad, 0xFF, sizeof(int64_t), s);   // -1 == no error
  if (e != hipSuccess) return hip_status(e, "efl_fxp_decode_hex");
  if (n == 0) return EFL_OK;
  if (dtype != EFL_DT_FLOAT && dtype != EFL_DT_DOUBLE) {
    set_error("FixedPointToFloatPoint: unsupported dtype %d (float, double)", dtype);
    return EFL_E_INVALID_ARGUMENT;
  }
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  if (dtype == EFL_DT_DOUBLE)
    hipLaunchKernelGGL((k_decode_hex<true>), dim3(grid), dim3(kBlock), 0, s, chars,
                       (const long long*)offsets, (const long long*)exponent, y, (long long)n,
                       flags, (long long*)bad);
  else
    hipLaunchKernelGGL((k_decode_hex<false>), dim3(grid), dim3(kBlock), 0, s, chars,
                       (const long long*)offsets, (const long long*)exponent, y, (long long)n,
                       flags, (long long*)bad);
  return hip_status(hipGetLastError(), "efl_fxp_decode_hex");
}

namespace {
// batched tile: B lanes x K pairs, nontemporal loads: fewer, longer workgroups amortise the
// per-workgroup pointer-table reads. Default 256 x 4 (2048 elements, measured faster than the
// k_stream shape here); the fp32 shapes are tunable (efl_fxp_tune kinds 10-13).

template <class Op, int NT, int B, int K>
hipError_t launch_batched_bk(const void* const* src, void* const* d0, void* const* d1,
                             const long long* ns, long long count, long long max_n, int flag,
                             hipStream_t s, int dir = -1) {
  const long long tile = (long long)B * K * Op::kElems;
  const long long gx = (max_n + tile - 1) / tile;
  if (gx == 0 || count == 0) return hipSuccess;
  if (gx > 0x7FFFFFFFll) return hipErrorInvalidValue;
  const int order = dir >= 0 ? g_batch_order[dir].load(std::memory_order_relaxed) : 0;
  const long long total = count * gx;
  if (order == 3 && total < 0x7FFFFFF0ll) {
    const long long cap = g_batch_persist_grid.load(std::memory_order_relaxed);
    const long long grid = total < cap ? total : cap;
    hipLaunchKernelGGL((k_batched_persist<Op, B, K, NT>), dim3((unsigned)grid), dim3(B), 0, s, src, d0, d1, ns, flag,
                       gx, total);
    return hipGetLastError();
  }
  if (order > 0 && total < 0x7FFFFFF0ll) {
    const long long per = order == 2 && total >= 64 ? (total + 7) / 8 : 0;
    const long long grid = per ? 8 * per : total;
    hipLaunchKernelGGL((k_batched_flat<Op, B, K, NT>), dim3((unsigned)grid), dim3(B), 0, s, src, d0, d1, ns, flag,
                       gx, total, per);
    return hipGetLastError();
  }
  const int T = (dir >= 0 && B == 512) ? g_batch_tiles[dir].load(std::memory_order_relaxed) : 1;
  const long long gxt = (gx + T - 1) / T;
  for (long long b = 0; b < count; b += kMaxGridY) {
    const long long gy = count - b < kMaxGridY ? count - b : kMaxGridY;
    const dim3 grid((unsigned)gxt, (unsigned)gy);
    if constexpr (B == 512) {
      switch (T) {
        case 2: hipLaunchKernelGGL((k_batched<Op, B, K, NT, 2>), grid, dim3(B), 0, s, src, d0, d1, ns, flag, b); break;
        case 4: hipLaunchKernelGGL((k_batched<Op, B, K, NT, 4>), grid, dim3(B), 0, s, src, d0, d1, ns, flag, b); break;
        case 8: hipLaunchKernelGGL((k_batched<Op, B, K, NT, 8>), grid, dim3(B), 0, s, src, d0, d1, ns, flag, b); break;
        default: hipLaunchKernelGGL((k_batched<Op, B, K, NT>), grid, dim3(B), 0, s, src, d0, d1, ns, flag, b); break;
      }
    } else {
      hipLaunchKernelGGL((k_batched<Op, B, K, NT>), grid, dim3(B), 0, s, src, d0, d1, ns, flag, b);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <class Op, int NT>
hipError_t launch_batched(const void* const* src, void* const* d0, void* const* d1,
                          const long long* ns, long long count, long long max_n, int flag,
                          hipStream_t s) {
  return launch_batched_bk<Op, NT, kBatchB, kBatchK>(src, d0, d1, ns, count, max_n, flag, s);
}

// the fp32 ops, at the tuned shape of their direction
template <class Op, int NT>
hipError_t launch_batched_f32(int dir, const void* const* src, void* const* d0, void* const* d1,
                              const long long* ns, long long count, long long max_n, int flag,
                              hipStream_t s) {
  const int B = g_batch_block[dir].load(std::memory_order_relaxed);
  const int K = g_batch_k[dir].load(std::memory_order_relaxed);
#define EFL_BK(B_, K_) \
  if (B == B_ && K == K_) return launch_batched_bk<Op, NT, B_, K_>(src, d0, d1, ns, count, max_n, flag, s, dir);
  EFL_BK(128, 1) EFL_BK(128, 2) EFL_BK(256, 1) EFL_BK(256, 2) EFL_BK(256, 4) EFL_BK(512, 1) EFL_BK(512, 2)
  EFL_BK(512, 4)
#undef EFL_BK
  return launch_batched_bk<Op, NT, kBatchB, kBatchK>(src, d0, d1, ns, count, max_n, flag, s, dir);
}
}  // namespace

EFL_API int efl_fxp_encode_batched(const void* const* xs, int dtype, int64_t* const* mantissas,
                                   int64_t* const* exponents, const int64_t* ns, int64_t count,
                                   int64_t max_n, int decrease_precision, void* stream) {
  if (count < 0 || max_n < 0) { set_error("negative count"); return EFL_E_INVALID_ARGUMENT; }
  if (count == 0 || max_n == 0) return EFL_OK;
  hipStream_t s = (hipStream_t)stream;
  auto d0 = (void* const*)mantissas;
  auto d1 = (void* const*)exponents;
  auto nn = (const long long*)ns;
  const int f = decrease_precision ? 1 : 0;
  hipError_t e;
  switch (dtype) {
    case EFL_DT_FLOAT:
      switch (g_batch_enc_nt.load()) {
        case 7: e = launch_batched_f32<EncF32Pair, 7>(kEnc, xs, d0, d1, nn, count, max_n, f, s); break;
        case 3: e = launch_batched_f32<EncF32Pair, 3>(kEnc, xs, d0, d1, nn, count, max_n, f, s); break;
        default: e = launch_batched_f32<EncF32Pair, 1>(kEnc, xs, d0, d1, nn, count, max_n, f, s); break;
      }
      break;
    case EFL_DT_DOUBLE: e = launch_batched<EncF64Pair, 1>(xs, d0, d1, nn, count, max_n, f, s); break;
    case EFL_DT_INT8: e = launch_batched<EncIntPair<signed char, c2>, 1>(xs, d0, d1, nn, count, max_n, f, s); break;
    case EFL_DT_INT16: e = launch_batched<EncIntPair<short, s2>, 1>(xs, d0, d1, nn, count, max_n, f, s); break;
    case EFL_DT_INT32: e = launch_batched<EncIntPair<int, i2>, 1>(xs, d0, d1, nn, count, max_n, f, s); break;
    case EFL_DT_INT64: e = launch_batched<EncIntPair<long long, ll2>, 1>(xs, d0, d1, nn, count, max_n, f, s); break;
    default:
      set_error("ConvertToFixedPoint: unsupported dtype %d", dtype);
      return EFL_E_INVALID_ARGUMENT;
  }
  return hip_status(e, "efl_fxp_encode_batched");
}

EFL_API int efl_fxp_decode_batched(const int64_t* const* mantissas, const int64_t* const* exponents,
                                   void* const* ys, int dtype, const int64_t* ns, int64_t count,
                                   int64_t max_n, int flags, void* stream) {
  if (count < 0 || max_n < 0) { set_error("negative count"); return EFL_E_INVALID_ARGUMENT; }
  if (count == 0 || max_n == 0) return EFL_OK;
  hipStream_t s = (hipStream_t)stream;
  auto src = (const void* const*)mantissas;
  auto d0 = (void* const*)exponents;
  auto nn = (const long long*)ns;
  hipError_t e;
  switch (dtype) {
    case EFL_DT_FLOAT: e = launch_batched_f32<DecF32Pair, 1>(kDec, src, d0, ys, nn, count, max_n, flags, s); break;
    case EFL_DT_DOUBLE: e = launch_batched<DecF64Pair, 1>(src, d0, ys, nn, count, max_n, flags, s); break;
    default:
      set_error("FixedPointToFloatPoint: unsupported dtype %d", dtype);
      return EFL_E_INVALID_ARGUMENT;
  }
  return hip_status(e, "efl_fxp_decode_batched");
}
