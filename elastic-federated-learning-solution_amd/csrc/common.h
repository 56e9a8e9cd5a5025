// Shared helpers for the libefl_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "efl_hip.h"

#define EFL_API extern "C" __attribute__((visibility("default")))

namespace efl {

// 64-bit lane vectors as clang ext-vectors (so nontemporal builtins accept them).
typedef long long ll2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef signed char c2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;   // 4 waves of 64

void set_error(const char* fmt, ...);
int hip_status(hipError_t e, const char* what);

__host__ __device__ inline bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

}  // namespace efl
