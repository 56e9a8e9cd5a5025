// stream_probe — practical HBM ceiling for the exact traffic mix of the Stage-F kernels.
//
// The fixed-point codec moves 20 B per fp32 element in each direction, with opposite mixes:
// encode reads 4 B and writes 16 B (two int64 streams), decode reads 16 B and writes 4 B. This
// probe runs compute-free kernels with the SAME access pattern as csrc/fxp.hip's default shape
// (pair layout: lane i owns elements 2i, 2i+1 of a 128-element stripe, dwordx2 on the 4-byte side,
// dwordx4 on each 8-byte side, one tile of 128 lanes per workgroup, nontemporal loads), plus a
// float4 copy, a read-only and a write-only stream of the same byte count, at the bench size
// (64 Mi elements). The codec kernels are then judged against the ceiling of their own mix as well
// as the 8 TB/s spec.
//
// The real codec kernels (libefl_hip.so through its C ABI, on the same buffers) are timed in the
// same interleaved rounds, so "kernel vs the ceiling of its own mix" is one measurement.
//
//   make -C tools probes        (hipcc, links ../elastic-federated-learning-solution_amd/efl/libefl_hip.so)
//   tools/stream_probe [elements]      -> one JSON line
#include <hip/hip_runtime.h>

#include "efl_hip.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

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

#define CHECK_EFL(x)                                                              \
  do {                                                                            \
    if ((x) != EFL_OK) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, efl_last_error());        \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int B = 128;

// encode mix: read f2, write ll2 to M and ll2 to E (values depend on the loads so nothing folds)
__global__ __launch_bounds__(B) void k_enc_mix(const f2* __restrict__ x, ll2* __restrict__ M,
                                               ll2* __restrict__ E, long long nunits) {
  const long long u = (long long)blockIdx.x * B + threadIdx.x;
  if (u >= nunits) return;
  const f2 v = __builtin_nontemporal_load(x + u);
  const long long a = (long long)__float_as_uint(v.x), b = (long long)__float_as_uint(v.y);
  M[u] = ll2{a, b};
  E[u] = ll2{a ^ 1, b ^ 1};
}

// decode mix: read ll2 from M and E, write f2
__global__ __launch_bounds__(B) void k_dec_mix(const ll2* __restrict__ M, const ll2* __restrict__ E,
                                               f2* __restrict__ y, long long nunits) {
  const long long u = (long long)blockIdx.x * B + threadIdx.x;
  if (u >= nunits) return;
  const ll2 m = __builtin_nontemporal_load(M + u);
  const ll2 e = __builtin_nontemporal_load(E + u);
  y[u] = f2{__uint_as_float((unsigned)(m.x ^ e.x)), __uint_as_float((unsigned)(m.y ^ e.y))};
}

// read-only and write-only streams (the two extremes of the mix)
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ a, float* __restrict__ sink, long long n4) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u >= n4) return;
  const f4 v = __builtin_nontemporal_load(a + u);
  if (v.x == 1.2345f && v.y == 6.789f) sink[0] = v.z + v.w;   // never true for the memset data
}
__global__ __launch_bounds__(256) void k_write(f4* __restrict__ a, long long n4) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u < n4) a[u] = f4{(float)u, 0.f, 0.f, 0.f};
}

// plain float4 copy (the guide's 6.29 TB/s reference shape)
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ a, f4* __restrict__ b, long long n4) {
  const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
  if (u < n4) b[u] = a[u];
}

// Interleaved timing (cdna_hip_programming.md §5.4 rule 24): every round times each kernel a few
// times in turn, so clock / power drift lands on all of them alike; the median is reported.
struct Timed {
  const char* name;
  std::function<void()> launch;
  std::vector<float> t;
};

static void time_all(std::vector<Timed>& ks, int rounds, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& k : ks)
    for (int i = 0; i < 3; ++i) k.launch();
  for (int r = 0; r < rounds; ++r)
    for (auto& k : ks)
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(e0, 0));
        k.launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        k.t.push_back(ms);
      }
  for (auto& k : ks) std::sort(k.t.begin(), k.t.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 65536LL * 1024;   // bench size: 256 MiB fp32
  if (n <= 0 || n % 256) {
    fprintf(stderr, "elements must be a positive multiple of 256\n");
    return 2;
  }
  float *x, *y, *sink;
  long long *M, *E;
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMalloc(&M, n * 8));
  CHECK(hipMalloc(&E, n * 8));
  CHECK(hipMalloc(&y, n * 4));
  CHECK(hipMalloc(&sink, 16));
  CHECK(hipMemset(x, 0x3f, n * 4));
  CHECK(hipMemset(M, 0x01, n * 8));
  CHECK(hipMemset(E, 0x02, n * 8));
  const long long nunits = n / 2;
  const unsigned grid = (unsigned)(nunits / B);
  const double bytes = 20.0 * n;   // per kernel, as the codec

  const long long n4 = n * 20 / 16 / 2;   // copy: half of the 20 B read, half written
  const long long r4 = n * 20 / 16;       // read-only / write-only: all 20 B one way
  f4 *big0, *big1;
  CHECK(hipMalloc(&big0, r4 * 16));
  CHECK(hipMalloc(&big1, n4 * 16));
  CHECK(hipMemset(big0, 0, r4 * 16));
  std::vector<Timed> ks = {
      {"enc_mix", [&] { hipLaunchKernelGGL(k_enc_mix, dim3(grid), dim3(B), 0, 0, (const f2*)x, (ll2*)M, (ll2*)E, nunits); }, {}},
      {"dec_mix", [&] { hipLaunchKernelGGL(k_dec_mix, dim3(grid), dim3(B), 0, 0, (const ll2*)M, (const ll2*)E, (f2*)y, nunits); }, {}},
      {"copy_f4", [&] { hipLaunchKernelGGL(k_copy, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const f4*)big0, big1, n4); }, {}},
      {"read_only", [&] { hipLaunchKernelGGL(k_read, dim3((unsigned)((r4 + 255) / 256)), dim3(256), 0, 0, (const f4*)big0, sink, r4); }, {}},
      {"write_only", [&] { hipLaunchKernelGGL(k_write, dim3((unsigned)((r4 + 255) / 256)), dim3(256), 0, 0, big0, r4); }, {}},
      {"efl_encode", [&] { CHECK_EFL(efl_fxp_encode(x, EFL_DT_FLOAT, (int64_t*)M, (int64_t*)E, n, 0, nullptr)); }, {}},
      {"efl_decode", [&] { CHECK_EFL(efl_fxp_decode((const int64_t*)M, (const int64_t*)E, y, EFL_DT_FLOAT, n, n, 0, nullptr)); }, {}},
  };
  time_all(ks, 10, 5);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  printf("{\"elements\": %lld, \"bytes_per_kernel\": %.0f, \"timing\": \"median of 10 interleaved rounds x 5\"", n, bytes);
  for (auto& k : ks) {
    const float ms = k.t[k.t.size() / 2];
    printf(", \"%s_ms\": %.4f, \"%s_GBs\": %.1f", k.name, ms, k.name, bytes / (ms * 1e-3) / 1e9);
  }
  printf("}\n");
  CHECK(hipFree(x));
  CHECK(hipFree(M));
  CHECK(hipFree(E));
  CHECK(hipFree(y));
  CHECK(hipFree(sink));
  CHECK(hipFree(big0));
  CHECK(hipFree(big1));
  return 0;
}
