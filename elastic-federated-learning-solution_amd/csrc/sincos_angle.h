// sin and cos of Box-Muller's angle v1 = float(2 pi (double) u), u in [0, 1): a float in [0, 2 pi].
//
// OCML's sincosf serves any float, so it carries a Payne-Hanek reduction for huge arguments; the
// compiler flattens that path into selects (about 150 v_cndmask / v_alignbit / v_xor per lane of
// the DP noise kernel, which made it VALU-bound at 0.57-0.68 of 8 TB/s). On [0, 2 pi] one
// Cody-Waite step is exact enough: k = rint(v 2/pi) in 0..4, r = v - k pi/2 with pi/2 split into
// three floats (C1 + C2 + C3, 72 bits; every step one fma), then Cephes' single-precision minimax
// polynomials for sin and cos on [-pi/4, pi/4] and the quadrant's sign/swap. Round 3 reduced in
// double (pi/2 as a double-double); round 5 does it in float: the reduced r is the same float for
// every angle but one (float(pi/4) + 1 ulp, where v 2/pi rounds to 0.5 in float and k = 0 instead
// of 1; sin there is now the correctly rounded one, 1 ulp off before), and the f64 conversions,
// products and rint (4-cycle VALU on gfx950) go.
//
// efl_box_muller_angle(u) forms v1 = float(2 pi (double) u) without doubles: 2 pi (double) = A + B
// in floats, u A exactly as p + e (fma), then p + (u B + e). The same float as the double product
// for all 2^23 values of u (tests/test_sincos_angle.py checks them all).
//
// Accuracy is checked exhaustively on the host: tests/test_sincos_angle.py compiles this header
// with gcc (-ffp-contract=off, the kernel file's own `fp contract(off)`; every fused step is an
// explicit fma, so host and device round identically) and compares every reachable angle and every
// 61st float of [0, 2 pi] with the correctly rounded sin / cos (double libm, rounded to float).
#pragma once

#ifdef __HIPCC__
#define EFL_SC_FN __host__ __device__ __forceinline__
// every product and sum below rounds on its own wherever the header is included (hipcc contracts
// a * b + c by default; p + (u b + e) fused would not be the double product)
#define EFL_SC_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define EFL_SC_NOCONTRACT
#include <math.h>
#define EFL_SC_FN static inline
#endif

EFL_SC_FN float efl_box_muller_angle(float u) {
  EFL_SC_NOCONTRACT
  const float a = 0x1.921fb6p+2f, b = -0x1.777a5cp-23f;   // 2 pi (double) = a + b exactly
  const float p = u * a;
  const float e = fmaf(u, a, -p);                          // u a = p + e exactly
  return p + fmaf(u, b, e);
}

EFL_SC_FN void efl_sincos_angle(float v, float* s, float* c) {
  EFL_SC_NOCONTRACT
  const float k = rintf(v * 0x1.45f306p-1f);               // 2/pi
  float r = fmaf(-k, 0x1.921fb6p+0f, v);                   // pi/2 = C1 + C2 + C3
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  const float z = r * r;
  float ps = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(ps, z, -1.6666654611e-1f);
  const float sn = fmaf(ps * z, r, r);                     // r + r^3 P(r^2)
  float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(pc, z, 4.166664568298827e-2f);
  pc = fmaf(pc, z, -0.5f);
  const float cs = fmaf(pc, z, 1.0f);                      // 1 + r^2 (-1/2 + r^2 Q(r^2))
  const int q = (int)k & 3;
  const float ss = (q & 1) ? cs : sn;
  const float cc = (q & 1) ? sn : cs;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}
