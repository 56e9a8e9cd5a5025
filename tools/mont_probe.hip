// mont_probe — the sliced Montgomery squaring loop of the Paillier decrypt (1024-bit modulus,
// 2 lanes per element) in two limb radixes, timed and cross-checked:
//   variant 0: 32-bit limbs, carry chain per product (csrc/sliced.h, the production kernels)
//   variant 1: 28-bit limbs, lazy 64-bit accumulators (csrc/sliced28.h)
// Both compute x^(2^S) mod m for N elements. Driven from tools/mont_probe.py (ctypes + torch).
//
//   make -C tools libmont_probe.so
#include <hip/hip_runtime.h>

#include "sliced28.h"

using namespace efl;

namespace {

constexpr int kG = 2, kC32 = 16, kL32 = kC32 * kG;
constexpr int kC28 = s28::limbs_per_lane(kL32, kG), kL28 = kC28 * kG;
constexpr int kE = 64 / kG;   // elements per (one-wave) workgroup

struct Uni {
  const uint32_t* p;
  __device__ __forceinline__ uint32_t operator()(int i) const { return p[i]; }
};
struct One {
  __device__ __forceinline__ uint32_t operator()(int i) const { return i == 0 ? 1u : 0u; }
};

__global__ __launch_bounds__(64) void k_sq32(const uint32_t* __restrict__ m, const uint32_t* __restrict__ r2,
                                             uint32_t minv, const uint32_t* __restrict__ x, uint32_t* __restrict__ out,
                                             long long N, int S) {
  __shared__ uint32_t lds[kL32 * kE];
  const int g = threadIdx.x % kG, e = threadIdx.x / kG;
  const long long i = (long long)blockIdx.x * kE + e;
  if (i >= N) return;
  uint32_t ms[kC32], t[kC32];
  sl::slice_uniform<kC32>(ms, m, g);
  sl::load_slice<kC32>(t, x + i * kL32, g);
  sl::mont_mul<kC32, kG>(t, Uni{r2}, ms, minv, g);
  for (int s = 0; s < S; ++s) sl::mont_sqr<kC32, kG>(t, lds + e, kE, ms, minv, g);
  sl::mont_mul<kC32, kG>(t, One{}, ms, minv, g);
  sl::store_slice<kC32>(out + i * kL32, g, t);
}

__global__ __launch_bounds__(64) void k_sq28(const uint32_t* __restrict__ m28, const uint32_t* __restrict__ r2_28,
                                             uint32_t minv28, const uint32_t* __restrict__ x, uint32_t* __restrict__ out,
                                             long long N, int S) {
  __shared__ uint32_t lds[kL28 * kE];
  const int g = threadIdx.x % kG, e = threadIdx.x / kG;
  const long long i = (long long)blockIdx.x * kE + e;
  if (i >= N) return;
  uint32_t* col = lds + e;
  uint32_t w[kC32];
  sl::load_slice<kC32>(w, x + i * kL32, g);
  sl::to_lds<kC32>(col, kE, g, w);
  sl::lds_sync();
  uint32_t ms[kC28], a[kC28];
  s28::from_words<kC28>(a, col, kE, kL32, g);
  sl::lds_sync();
  sl::slice_uniform<kC28>(ms, m28, g);
  s28::mont_mul<kC28, kG>(a, Uni{r2_28}, ms, minv28, g);
  for (int s = 0; s < S; ++s) s28::mont_sqr<kC28, kG>(a, col, kE, ms, minv28, g);
  s28::mont_mul<kC28, kG>(a, One{}, ms, minv28, g);
  sl::lds_sync();
  sl::to_lds<kC28>(col, kE, g, a);
  sl::lds_sync();
  s28::to_words<kC32>(w, col, kE, kL28, g);
  sl::store_slice<kC32>(out + i * kL32, g, w);
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int mont_probe_limbs28() { return kL28; }

extern "C" __attribute__((visibility("default"))) int mont_probe(int variant, const uint32_t* m, const uint32_t* r2,
                                                                   uint32_t minv, const uint32_t* x, uint32_t* out,
                                                                   long long N, int S, void* stream) {
  const unsigned grid = (unsigned)((N + kE - 1) / kE);
  if (variant == 0)
    hipLaunchKernelGGL(k_sq32, dim3(grid), dim3(64), 0, (hipStream_t)stream, m, r2, minv, x, out, N, S);
  else
    hipLaunchKernelGGL(k_sq28, dim3(grid), dim3(64), 0, (hipStream_t)stream, m, r2, minv, x, out, N, S);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
