/*
 * efl_hip.h — C ABI of libefl_hip.so, the MI355X (gfx950) implementation of EFLS-train's
 * forward-encryption path.
 *
 * The reference binds this path as TensorFlow custom ops loaded with
 * `tf.load_op_library(libefl.so)` (efls-train/python/efl/lib.py:24-28) and called as
 * `fed_ops.<snake_case_op>` from efls-train/python/efl/privacy/paillier.py:56-155. This header is
 * what such an FFI binds instead: plain pointers, sizes and an opaque HIP stream, no framework
 * types. The Python drop-in (package `efl`, ctypes) and INTEGRATION.md show the binding.
 *
 * Conventions
 *  - Every payload pointer is DEVICE memory owned by the caller; the library never allocates
 *    payload memory and never synchronises: work is enqueued on `stream` (NULL = default stream).
 *  - Return value: 0 on success, otherwise the NEGATED TensorFlow error code
 *    (tensorflow/core/lib/core/error_codes.proto; the reference reports errors as TF Status):
 *      -3 INVALID_ARGUMENT, -8 RESOURCE_EXHAUSTED, -9 FAILED_PRECONDITION, -10 ABORTED,
 *      -12 UNIMPLEMENTED, -13 INTERNAL (a HIP runtime error).  efl_last_error() gives the text.
 *  - dtype codes are TensorFlow DataType numbers (tensorflow/core/framework/types.proto:19-27),
 *    the numbering the reference's wire format (TensorProto.dtype) carries.
 */
#ifndef EFL_HIP_H_
#define EFL_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TensorFlow DataType numbers. */
enum {
  EFL_DT_FLOAT = 1,
  EFL_DT_DOUBLE = 2,
  EFL_DT_INT32 = 3,
  EFL_DT_INT16 = 5,
  EFL_DT_INT8 = 6,
  EFL_DT_STRING = 7,
  EFL_DT_INT64 = 9
};

/* Negated TensorFlow error codes. */
enum {
  EFL_OK = 0,
  EFL_E_INVALID_ARGUMENT = -3,
  EFL_E_RESOURCE_EXHAUSTED = -8,
  EFL_E_FAILED_PRECONDITION = -9,
  EFL_E_ABORTED = -10,
  EFL_E_UNIMPLEMENTED = -12,
  EFL_E_INTERNAL = -13
};

/* efl_fxp_decode* flags */
enum {
  /* Flush float32 results below the normal range to signed zero, as the reference does when its
   * kernel runs on a TensorFlow threadpool thread (x86 MXCSR FTZ|DAZ; tininess after rounding). */
  EFL_FXP_FTZ = 1
};

/* ----------------------------------------------------------------------------------------- */
/* Library                                                                                    */
/* ----------------------------------------------------------------------------------------- */

const char* efl_version(void);
/* Text of the last error raised on the calling thread ("" if none). */
const char* efl_last_error(void);
/* Launch-shape knob of the fp32 Stage-F kernels (bench/profiling; results never change).
 * kind = 2*field + direction (direction 0 encode, 1 decode); fields: 0 layout (0 pair, 1 quad),
 * 1 units per lane per tile (1, 2), 2 nontemporal mask (bit0 loads, bit1 stores), 3 workgroup size
 * (128, 256, 512); kind 8 = grid cap (0 = one tile per workgroup). Returns the previous value or
 * EFL_E_INVALID_ARGUMENT. */
int efl_fxp_tune(int kind, int value);

/* ----------------------------------------------------------------------------------------- */
/* Stage F — fixed-point codec                                                                */
/* ----------------------------------------------------------------------------------------- */

/*
 * Replaces REGISTER_OP("ConvertToFixedPoint") / Convert2FixedPointOp<T>::Compute
 * (efls-train/cc/efl/math/fixed_point.cc:24-199), Python `fed_ops.convert_to_fixed_point`
 * (paillier.py:148-150).  x: n elements of `dtype` in {INT8, INT16, INT32, INT64, FLOAT, DOUBLE};
 * mantissa/exponent: n int64 each.  Bit-exact with the reference.
 */
int efl_fxp_encode(const void* x, int dtype, int64_t* mantissa, int64_t* exponent, int64_t n,
                   int decrease_precision, void* stream);

/*
 * Replaces REGISTER_OP("FixedPointToFloatPoint") / FixedPointToFloatPointOp<int64, Tout>
 * (fixed_point.cc:201-287), Python `fed_ops.fixed_point_to_float_point` (paillier.py:113-114,
 * 153-155).  y: n elements of `dtype` in {FLOAT, DOUBLE}.  n_mantissa != n_exponent ->
 * INVALID_ARGUMENT "mantissa and exponent should be the same size." (fixed_point.cc:230-232).
 * Result = GMP mpf_get_d(mantissa * 2^exponent) (truncating) then round-to-nearest to float.
 */
int efl_fxp_decode(const int64_t* mantissa, const int64_t* exponent, void* y, int dtype,
                   int64_t n_mantissa, int64_t n_exponent, int flags, void* stream);

/*
 * FixedPointToFloatPointOp<string, Tout> (fixed_point.cc:255-257, mpf_set_str base 16):
 * n hex mantissas ("[-]hexdigits", any case) packed back to back in `chars`, string i occupying
 * chars[offsets[i] .. offsets[i+1]).  `bad` (device, one int64) receives -1, or the smallest
 * index of a malformed string (the caller raises INVALID_ARGUMENT; the reference silently keeps
 * a stale value there — DESIGN.md).
 */
int efl_fxp_decode_hex(const char* chars, const int64_t* offsets, const int64_t* exponent,
                       void* y, int dtype, int64_t n, int flags, int64_t* bad, void* stream);

/*
 * Batched encode of `count` independent tensors in ONE launch (sparse-rec embedding slices,
 * BASELINE config 3). xs / mantissas / exponents / ns are DEVICE arrays of `count` entries;
 * max_n = max(ns) (host scalar, sizes the grid). Same semantics per tensor as efl_fxp_encode.
 */
int efl_fxp_encode_batched(const void* const* xs, int dtype, int64_t* const* mantissas,
                           int64_t* const* exponents, const int64_t* ns, int64_t count,
                           int64_t max_n, int decrease_precision, void* stream);

/* Batched decode, same layout conventions as efl_fxp_encode_batched. */
int efl_fxp_decode_batched(const int64_t* const* mantissas, const int64_t* const* exponents,
                           void* const* ys, int dtype, const int64_t* ns, int64_t count,
                           int64_t max_n, int flags, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* EFL_HIP_H_ */
