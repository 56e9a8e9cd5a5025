// valu_probe — measured issue rates of the instructions a multi-precision Montgomery kernel is
// built from, on every CU of the MI355X at once. They set the Stage-P roofline:
// the Paillier kernels are VALU-bound, and the relevant peak is the rate of the 32x32->64
// multiply-accumulate (v_mad_u64_u32), not an HBM or MFMA number.
//
// Each kernel runs kChains independent dependency chains per lane for `iters` iterations; grid = 8
// workgroups of 256 lanes per CU. v_mad_u64_u32 is also run with 24 chains and a wave-uniform
// multiplier (the shape of a Montgomery row: one b limb times many a limbs into 64-bit
// accumulators), which is what saturates its issue. Reported per op: lane-ops/s and lane-ops per
// clock per CU at 2.4 GHz.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/valu_probe tools/valu_probe.hip && tools/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kChains = 8;

enum Op { MAD_U64_U32 = 0, MUL_LO_U32, MUL_HI_U32, ADD_CO_PAIR, FMA_F64, MAD_U32_U24, FMA_F32, LSHL_ADD_U64,
          MAD_ROW, kOps };
const char* kNames[kOps] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "add_co_u32+addc_co_u32",
                            "v_fma_f64", "v_mad_u32_u24", "v_fma_f32", "u64 add (v_lshl_add_u64)",
                            "v_mad_u64_u32 (24 accumulators, uniform multiplier)"};
constexpr int kRow = 24;

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint64_t* out, int iters, uint32_t seed, long long* clk) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  long long c0 = 0;
  if (threadIdx.x == 0) c0 = __builtin_amdgcn_s_memtime();
  uint64_t acc = 0;
  if constexpr (OP == MAD_ROW) {
    uint64_t T[kRow];
    uint32_t a[kRow];
#pragma unroll
    for (int j = 0; j < kRow; ++j) {
      T[j] = (uint64_t)t * (j + 5);
      a[j] = (t * 2654435761u + j) & 0x0FFFFFFFu;
    }
    uint32_t b = seed & 0x0FFFFFFFu;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < kRow; ++j) T[j] = (uint64_t)a[j] * b + T[j];
      b = (b * 1664525u + 1013904223u) & 0x0FFFFFFFu;   // uniform: stays in an SGPR
    }
#pragma unroll
    for (int j = 0; j < kRow; ++j) acc += T[j];
  } else if constexpr (OP == FMA_F64) {
    double d[kChains];
    const double m = 0.9999999, a = 1e-7 * (double)(t & 7);
#pragma unroll
    for (int j = 0; j < kChains; ++j) d[j] = 1.0 + j + (double)(t & 15);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < kChains; ++j) d[j] = __builtin_fma(d[j], m, a);
    }
#pragma unroll
    for (int j = 0; j < kChains; ++j) acc += (uint64_t)__double_as_longlong(d[j]);
  } else if constexpr (OP == FMA_F32) {
    float d[kChains];
    const float m = 0.9999f, a = 1e-5f * (float)(t & 7);
#pragma unroll
    for (int j = 0; j < kChains; ++j) d[j] = 1.0f + j + (float)(t & 15);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < kChains; ++j) d[j] = __builtin_fmaf(d[j], m, a);
    }
#pragma unroll
    for (int j = 0; j < kChains; ++j) acc += __float_as_uint(d[j]);
  } else {
    uint64_t v[kChains];
    uint32_t w[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) {
      v[j] = (uint64_t)t * (j + 3) + 0x9E3779B97F4A7C15ull;
      w[j] = t * 2654435761u + j;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < kChains; ++j) {
        if constexpr (OP == MAD_U64_U32) {
          v[j] = (uint64_t)w[j] * (uint32_t)v[j] + v[j];
        } else if constexpr (OP == MUL_LO_U32) {
          w[j] = w[j] * (w[j] | 1u);
        } else if constexpr (OP == MUL_HI_U32) {
          w[j] = __umulhi(w[j], w[j] | 0x80000001u) + 1u;
        } else if constexpr (OP == ADD_CO_PAIR) {
          unsigned int co;
          const uint32_t lo = __builtin_addc((uint32_t)v[j], w[j], 0u, &co);
          const uint32_t hi = __builtin_addc((uint32_t)(v[j] >> 32), 0u, co, &co);
          v[j] = ((uint64_t)hi << 32) | lo;
        } else if constexpr (OP == MAD_U32_U24) {
          w[j] = __umul24(w[j], w[j] | 1u) + w[j];
        } else if constexpr (OP == LSHL_ADD_U64) {
          v[j] = v[j] + (v[(j + 1) % kChains] << 1);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kChains; ++j) acc += v[j] + w[j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) *clk = __builtin_amdgcn_s_memtime() - c0;
}

template <int OP>
void run(int cus, int iters, uint64_t* out, long long* clk) {
  const int grid = cus * 8;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, out, 16, 1u, clk);   // warm
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, out, iters, 1u, clk);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  long long ticks = 0;
  CHECK(hipMemcpy(&ticks, clk, sizeof(ticks), hipMemcpyDeviceToHost));
  const double lane_ops = (double)grid * 256 * iters * (OP == MAD_ROW ? kRow : kChains);
  const double per_s = lane_ops / (ms * 1e-3);
  // s_memtime runs at a fixed 100 MHz reference on CDNA; report ops per CU per 2.4 GHz clock too
  const double per_clk_cu = per_s / cus / 2.4e9;
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"lane_ops_per_clk_per_cu_at_2.4GHz\": %.2f, "
         "\"wave64_cycles_per_op_per_simd\": %.2f}\n",
         kNames[OP], ms, per_s, per_clk_cu, 64.0 / (per_clk_cu / 4.0));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  uint64_t* out;
  long long* clk;
  CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(uint64_t)));
  CHECK(hipMalloc(&clk, sizeof(long long)));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, cus, p.clockRate);
  run<MAD_U64_U32>(cus, iters, out, clk);
  run<MUL_LO_U32>(cus, iters, out, clk);
  run<MUL_HI_U32>(cus, iters, out, clk);
  run<ADD_CO_PAIR>(cus, iters, out, clk);
  run<FMA_F64>(cus, iters, out, clk);
  run<MAD_U32_U24>(cus, iters, out, clk);
  run<FMA_F32>(cus, iters, out, clk);
  run<LSHL_ADD_U64>(cus, iters, out, clk);
  run<MAD_ROW>(cus, iters, out, clk);
  CHECK(hipFree(out));
  CHECK(hipFree(clk));
  return 0;
}
