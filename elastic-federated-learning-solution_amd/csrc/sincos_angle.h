// sin and cos of Box-Muller's angle v1 = float(2 pi (double) u), u in [0, 1): a float in [0, 2 pi].
//
// OCML's sincosf serves any float, so it carries a Payne-Hanek reduction for huge arguments; the
// compiler flattens that path into selects (about 150 v_cndmask / v_alignbit / v_xor per lane of
// the DP noise kernel, which made it VALU-bound at 0.57-0.68 of 8 TB/s). On [0, 2 pi] one
// Cody-Waite step is exact enough: k = rint(v 2/pi) in 0..4, r = v - k pi/2 in double with pi/2 as a
// double-double (an exact product in the FMA, |r| <= pi/4 + 2^-22, relative error < 2^-50 even for
// the floats nearest to pi and 2 pi), r rounded to float once, then Cephes' single-precision
// minimax polynomials for sin and cos on [-pi/4, pi/4] and the quadrant's sign/swap.
//
// Accuracy is checked exhaustively on the host: tests/test_sincos_angle.py compiles this header
// with gcc (-ffp-contract=off, the kernel file's own `fp contract(off)`; every fused step is an
// explicit fma, so host and device round identically) and compares all 1.08e9 floats in [0, 2 pi]
// with the correctly rounded sin / cos (double libm, rounded to float).
#pragma once

#ifdef __HIPCC__
#define EFL_SC_FN __host__ __device__ __forceinline__
#else
#include <math.h>
#define EFL_SC_FN static inline
#endif

EFL_SC_FN void efl_sincos_angle(float v, float* s, float* c) {
  const double vd = (double)v;
  const double k = rint(vd * 0.63661977236758134308);     // 2/pi
  double rd = fma(-k, 1.5707963267948965580, vd);          // pi/2 high part
  rd = fma(-k, 6.1232339957367658e-17, rd);                // pi/2 low part
  const float r = (float)rd;
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
