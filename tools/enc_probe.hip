// Encode traffic-mix layouts (4 B read, 16 B written per element, no compute), timed interleaved
// beside a mask-like 4:12 mix and efl_fxp_encode. Question: is the encode kernel's write-heavy mix
// bounded by the HBM mix itself or by its access layout? Not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "efl_hip.h"

typedef long long ll2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ ll2 mk(float a, float b, long long s) {
  return ll2{(long long)__float_as_uint(a) ^ s, (long long)__float_as_uint(b) ^ s};
}

// V0/V1: pair layout (lane = 2 elements), block BS
template <int BS>
__global__ __launch_bounds__(BS) void k_pair(const f2* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nu) {
  const long long u = (long long)blockIdx.x * BS + threadIdx.x;
  if (u >= nu) return;
  const f2 v = __builtin_nontemporal_load(x + u);
  M[u] = mk(v.x, v.y, 0);
  E[u] = mk(v.x, v.y, 1);
}

// V2: lane = 4 consecutive elements (f4 load), int64 stores at a 32-B lane stride
__global__ __launch_bounds__(256) void k_quad(const f4* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nq) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= nq) return;
  const f4 v = __builtin_nontemporal_load(x + g);
  M[2 * g] = mk(v.x, v.y, 0);
  M[2 * g + 1] = mk(v.z, v.w, 0);
  E[2 * g] = mk(v.x, v.y, 1);
  E[2 * g + 1] = mk(v.z, v.w, 1);
}

// V3: lane = 2 pairs of a 256-element wave span (elements 2l,2l+1 and 128+2l,128+2l+1), loads first
__global__ __launch_bounds__(256) void k_pair2(const f2* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nu) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long base = ((long long)blockIdx.x * 4 + w) * 128;   // in pair units: 128 pairs per wave
  if (base + 128 > nu) return;
  const f2 a = __builtin_nontemporal_load(x + base + lane);
  const f2 b = __builtin_nontemporal_load(x + base + 64 + lane);
  M[base + lane] = mk(a.x, a.y, 0);
  M[base + 64 + lane] = mk(b.x, b.y, 0);
  E[base + lane] = mk(a.x, a.y, 1);
  E[base + 64 + lane] = mk(b.x, b.y, 1);
}

// V4: nontemporal stores, pair layout, block 256
__global__ __launch_bounds__(256) void k_pair_nt(const f2* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nu) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const f2 v = __builtin_nontemporal_load(x + u);
  __builtin_nontemporal_store(mk(v.x, v.y, 0), M + u);
  __builtin_nontemporal_store(mk(v.x, v.y, 1), E + u);
}

// V6: stores with explicit cache-policy bits (gfx950 global_store_dwordx4 ... off <bits>)
typedef int i4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_sc1(ll2* p, ll2 v) {
  i4 w = __builtin_bit_cast(i4, v);
  asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ void st16_sc0sc1(ll2* p, ll2 v) {
  i4 w = __builtin_bit_cast(i4, v);
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ void st16_ntsc1(ll2* p, ll2 v) {
  i4 w = __builtin_bit_cast(i4, v);
  asm volatile("global_store_dwordx4 %0, %1, off nt sc1" :: "v"(p), "v"(w) : "memory");
}
template <int MODE>
__global__ __launch_bounds__(256) void k_pair_bits(const f2* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nu) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const f2 v = __builtin_nontemporal_load(x + u);
  if (MODE == 0) { st16_sc1(M + u, mk(v.x, v.y, 0)); st16_sc1(E + u, mk(v.x, v.y, 1)); }
  if (MODE == 1) { st16_sc0sc1(M + u, mk(v.x, v.y, 0)); st16_sc0sc1(E + u, mk(v.x, v.y, 1)); }
  if (MODE == 2) { st16_ntsc1(M + u, mk(v.x, v.y, 0)); st16_ntsc1(E + u, mk(v.x, v.y, 1)); }
}

// V5: all M of a workgroup tile, then all E (two phases, each one contiguous 4 KiB per block)
__global__ __launch_bounds__(256) void k_pair_phase(const f2* __restrict__ x, ll2* __restrict__ M, ll2* __restrict__ E, long long nu) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const f2 v = __builtin_nontemporal_load(x + u);
  M[u] = mk(v.x, v.y, 0);
  __builtin_amdgcn_s_barrier();
  E[u] = mk(v.x, v.y, 1);
}

// control: mask_cols-like 4:12 mix (f4 load; f4, f4, f2 stores)
__global__ __launch_bounds__(256) void k_mask_mix(const f4* __restrict__ x, f4* __restrict__ s, f4* __restrict__ k,
                                                  f2* __restrict__ h, long long nq) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= nq) return;
  const f4 v = __builtin_nontemporal_load(x + g);
  s[g] = v + 1.0f;
  k[g] = v - 1.0f;
  h[g] = f2{v.x + v.y, v.z + v.w};
}

struct Timed {
  const char* name;
  double bytes;
  std::function<void()> launch;
  std::vector<float> t;
};

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 65536LL * 1024;
  if (n <= 0 || n % 1024) return 2;
  float *x, *y;
  long long *M, *E;
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMalloc(&y, n * 4));
  CHECK(hipMalloc(&M, n * 8));
  CHECK(hipMalloc(&E, n * 8));
  CHECK(hipMemset(x, 0x3f, n * 4));
  CHECK(hipMemset(M, 1, n * 8));
  CHECK(hipMemset(E, 2, n * 8));
  const long long nu = n / 2, nq = n / 4;
  const double b20 = 20.0 * n, b16 = 16.0 * n;
  std::vector<Timed> ks = {
      {"pair128", b20, [&] { hipLaunchKernelGGL(k_pair<128>, dim3(nu / 128), dim3(128), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair256", b20, [&] { hipLaunchKernelGGL(k_pair<256>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair512", b20, [&] { hipLaunchKernelGGL(k_pair<512>, dim3(nu / 512), dim3(512), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"quad", b20, [&] { hipLaunchKernelGGL(k_quad, dim3(nq / 256), dim3(256), 0, 0, (const f4*)x, (ll2*)M, (ll2*)E, nq); }, {}},
      {"pair2", b20, [&] { hipLaunchKernelGGL(k_pair2, dim3(nu / 512), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair_nt", b20, [&] { hipLaunchKernelGGL(k_pair_nt, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair_phase", b20, [&] { hipLaunchKernelGGL(k_pair_phase, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair_sc1", b20, [&] { hipLaunchKernelGGL(k_pair_bits<0>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair_sc0sc1", b20, [&] { hipLaunchKernelGGL(k_pair_bits<1>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"pair_ntsc1", b20, [&] { hipLaunchKernelGGL(k_pair_bits<2>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu); }, {}},
      {"step_plain", 2 * b20, [&] { hipLaunchKernelGGL(k_pair<256>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu);
                                   if (efl_fxp_decode((const int64_t*)M, (const int64_t*)E, y, EFL_DT_FLOAT, n, n, 0, nullptr)) exit(3); }, {}},
      {"step_nt", 2 * b20, [&] { hipLaunchKernelGGL(k_pair_nt, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu);
                                if (efl_fxp_decode((const int64_t*)M, (const int64_t*)E, y, EFL_DT_FLOAT, n, n, 0, nullptr)) exit(3); }, {}},
      {"step_sc1", 2 * b20, [&] { hipLaunchKernelGGL(k_pair_bits<0>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu);
                                 if (efl_fxp_decode((const int64_t*)M, (const int64_t*)E, y, EFL_DT_FLOAT, n, n, 0, nullptr)) exit(3); }, {}},
      {"step_ntsc1", 2 * b20, [&] { hipLaunchKernelGGL(k_pair_bits<2>, dim3(nu / 256), dim3(256), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nu);
                                   if (efl_fxp_decode((const int64_t*)M, (const int64_t*)E, y, EFL_DT_FLOAT, n, n, 0, nullptr)) exit(3); }, {}},
      {"mask_mix", b16, [&] { hipLaunchKernelGGL(k_mask_mix, dim3(nq / 256), dim3(256), 0, 0, (const f4*)x, (f4*)M, (f4*)E, (f2*)(E + n / 2 + 1024), nq); }, {}},
      {"efl_encode", b20, [&] { if (efl_fxp_encode(x, EFL_DT_FLOAT, (int64_t*)M, (int64_t*)E, n, 0, nullptr)) exit(3); }, {}},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& k : ks)
    for (int i = 0; i < 3; ++i) k.launch();
  for (int r = 0; r < 10; ++r)
    for (auto& k : ks)
      for (int i = 0; i < 5; ++i) {
        CHECK(hipEventRecord(e0, 0));
        k.launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        k.t.push_back(ms);
      }
  CHECK(hipGetLastError());
  printf("{\"elements\": %lld", n);
  for (auto& k : ks) {
    std::sort(k.t.begin(), k.t.end());
    const float ms = k.t[k.t.size() / 2];
    printf(", \"%s\": [%.4f, %.1f]", k.name, ms, k.bytes / (ms * 1e-3) / 1e9);
  }
  printf("}\n");
  return 0;
}
