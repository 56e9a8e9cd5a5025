// Exhaustive check of the DP noise kernel's float math on the GPU, for every uniform Box-Muller can
// draw (u = k 2^-23, k < 2^23):
// * the radius sqrt(-2 ln u1) through csrc/box_muller_math.h's log_unit / sqrt_normal (and the
//   folded clamp constant) against the device library's logf / sqrtf, as csrc/mask.hip computed it
//   before round 5;
// * the angle efl_box_muller_angle(u) (csrc/sincos_angle.h) against float(2 pi (double) u) in
//   double on the device;
// * the device's sin / cos of that angle against the same header run on the host, bit for bit
//   (so tests/test_sincos_angle.py, which checks the header on the host, speaks for the device).
// Prints one JSON line; exit status 1 on any bit difference.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I elastic-federated-learning-solution_amd/csrc \
//     tools/dp_fastmath_check.hip -o /tmp/dp_fastmath_check && /tmp/dp_fastmath_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

#include "box_muller_math.h"
#include "sincos_angle.h"

#pragma clang fp contract(off)

__global__ void k_angle(unsigned long long* diff, float* sn, float* cs) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << 23)) return;
  const float u = __uint_as_float(0x3f800000u | k) - 1.0f;
  const float v = efl_box_muller_angle(u);
  if (__float_as_uint(v) != __float_as_uint((float)(2.0 * 3.14159265358979323846 * (double)u))) atomicAdd(diff, 1ull);
  efl_sincos_angle(v, &sn[k], &cs[k]);
}

__global__ void k_check(unsigned long long* diff, uint32_t* first, uint32_t* clamp_bits) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (1u << 23)) return;
  const float u = __uint_as_float(0x3f800000u | k) - 1.0f;
  float u1 = u;
  if (u1 < 1.0e-7f) u1 = 1.0e-7f;
  const float ref = sqrtf(-2.0f * logf(u1));
  const float rr = sqrt_normal(-2.0f * log_unit(fmaxf(u, 1.0e-7f)));
  const float got = u < 1.0e-7f ? __uint_as_float(kRClampBits) : rr;
  if (k == 0) *clamp_bits = __float_as_uint(ref);
  // below the clamp the pre-round-5 kernel used the compiler's folded constant (kRClampBits, read
  // off its ISA), not a run-time logf; the run-time value is printed beside it
  if (u >= 1.0e-7f && __float_as_uint(ref) != __float_as_uint(got)) {
    atomicAdd(diff, 1ull);
    atomicMin(first, k);
  }
}

int main() {
  struct Out {
    unsigned long long diff, angle_diff;
    uint32_t first, clamp;
  } h = {0, 0, 0xffffffffu, 0};
  constexpr uint32_t N = 1u << 23;
  Out* d;
  float *sn, *cs;
  if (hipMalloc(&d, sizeof(Out)) != hipSuccess || hipMalloc(&sn, N * 4) != hipSuccess ||
      hipMalloc(&cs, N * 4) != hipSuccess || hipMemcpy(d, &h, sizeof(Out), hipMemcpyHostToDevice) != hipSuccess)
    return 2;
  hipLaunchKernelGGL(k_check, dim3(N / 256), dim3(256), 0, 0, &d->diff, &d->first, &d->clamp);
  hipLaunchKernelGGL(k_angle, dim3(N / 256), dim3(256), 0, 0, &d->angle_diff, sn, cs);
  static float hs[N], hc[N];
  if (hipMemcpy(&h, d, sizeof(Out), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hs, sn, N * 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hc, cs, N * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return 2;
  unsigned long long sc_diff = 0;
  for (uint32_t k = 0; k < N; ++k) {
    float u;
    const uint32_t b = 0x3f800000u | k;
    std::memcpy(&u, &b, 4);
    u -= 1.0f;
    float s, c;
    efl_sincos_angle(efl_box_muller_angle(u), &s, &c);
    if (std::memcmp(&s, &hs[k], 4) || std::memcmp(&c, &hc[k], 4)) ++sc_diff;
  }
  std::printf("{\"tool\": \"dp_fastmath_check\", \"inputs\": %u, \"radius_differ\": %llu, \"first_differing_k\": %d, "
              "\"clamp_runtime_bits\": \"0x%08x\", \"clamp_folded_bits\": \"0x%08x\", \"angle_differ\": %llu, "
              "\"sincos_device_vs_host_differ\": %llu}\n",
              N, h.diff, h.diff ? (int)h.first : -1, h.clamp, kRClampBits, h.angle_diff, sc_diff);
  return (h.diff || h.angle_diff || sc_diff) ? 1 : 0;
}
