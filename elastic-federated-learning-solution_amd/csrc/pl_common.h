// Pieces shared by the one-lane (paillier.hip) and the sliced (paillier_sliced.hip) Paillier kernels.
#pragma once

#include "common.h"

namespace efl {
namespace pl {

// key block (device, 32-bit limbs) + the descriptor of where each constant lives in it
struct Key {
  const uint32_t* base;
  efl_pl_key d;
  __device__ __forceinline__ const uint32_t* at(int64_t off) const { return base + off; }
};

// Philox4x32-10 (Salmon et al., SC'11): counter (ctr_lo, ctr_hi, block, 0), key = seed.
__device__ __forceinline__ void philox(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// Sliced kernels (paillier_sliced.hip): one number over L/C lanes of C limbs. L = limbs of the
// modulus the op works in (2*ln for n^2 ops, ln for decryption's p^2 / q^2).
bool sliced_available(int L, int C);
hipError_t sl_encrypt(const Key& k, int C, const long long* m, const uint32_t* hsa, uint32_t* out, long long N,
                      uint64_t seed, long long ctr0, hipStream_t s);
hipError_t sl_fbpowm(const Key& k, int C, const uint32_t* a, uint32_t* out, long long N, uint64_t seed,
                     long long ctr0, hipStream_t s);
hipError_t sl_add(const Key& k, int C, const uint32_t* x, const uint32_t* y, uint32_t* out, long long N,
                  hipStream_t s);
hipError_t sl_powm(const Key& k, int C, const uint32_t* x, const uint32_t* e, int ew, uint32_t* out, long long N,
                   hipStream_t s);
hipError_t sl_matmul(const Key& k, int C, const uint32_t* X, const long long* xe, const long long* ym,
                     const long long* ye, uint32_t* zpos, uint32_t* zneg, long long* ze, int u, int v, int w,
                     hipStream_t s);
hipError_t sl_decrypt(const Key& k, int C, const uint32_t* ct, uint32_t* mag, signed char* neg, long long N,
                      hipStream_t s);

}  // namespace pl
}  // namespace efl
