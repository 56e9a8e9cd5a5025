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
 *  - Every payload pointer is DEVICE memory owned by the caller; the library never synchronises:
 *    work is enqueued on `stream` (NULL = default stream). It allocates nothing except the
 *    stream-ordered scratch of efl_pl_matmul, of the sliced efl_pl_decrypt and of efl_pl_fxp_add
 *    in the kernel families without its fused kernel (see there).
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
 * 1 units per lane per tile (1, 2), 2 nontemporal mask (bit0 loads, bit1 stores; 7 = loads plus
 * `nt sc1` 16-B stores, the encode default), 3 workgroup size (128, 256, 512); kind 8 = grid cap
 * (0 = one tile per workgroup); kind 9 = nontemporal mask of the fp32 batched encode (1, 3 or 7);
 * kinds 10 / 11 = workgroup size (256, 512) / pairs per lane (1, 2, 4) of the fp32 batched encode,
 * 12 / 13 the same for the batched decode; kinds 14 / 15 = XCD-aware tile order (0 / 1; each of the
 * 8 XCDs streams one contiguous eighth) of the fp32 streaming encode / decode (default 0 / 1);
 * kind 16 = the streaming fp32 encode stores the exponent pair before the mantissa pair (0 / 1);
 * kinds 17 / 18 = tile order of the fp32 batched encode / decode (0 2-D grid, 1 one flat tensor-major
 * grid, 2 the flat grid in XCD-aware order, 3 a persistent walk of kind-19 workgroups that loads the
 * next tile while storing the current one); batched workgroup sizes 128, 256, 512; kind 20 =
 * Philox blocks per lane of efl_dp_noise (1, 2, 4; default 4); kinds 21-24 = the fp64 encode's
 * workgroup size (128, 256, 512, 1024), units per lane (1, 2), nontemporal mask (as kind 4) and
 * XCD-aware tile order (0 / 1).
 * kind 25 = lane groups (Philox blocks) per lane of efl_ss_noise / efl_ss_mask_cols /
 * efl_ss_mask_rows (1, 2, 4), kind 28 their store flavour (0 plain, 2 nontemporal, 7 `nt sc1`): each
 * has a per-kernel default; setting a value sets all kernels, -2 restores the defaults; kinds 26 / 27
 * = tiles per workgroup of the batched encode / decode (1, 2, 4, 8). Batched tile defaults (kinds 10-13): encode 512 lanes x 1 pair,
 * decode 512 x 2. Kind 29 = efl_ss_mask_rows with the row pair over the two halves of a wave (1,
 * default) or in one lane (0, round 5's kernel); kind 30 the same for the two outputs of
 * efl_ss_noise ops 1 and 2 (1 over the wave halves, default; 0 both in one lane). Value -1 on kinds
 * 10-13, 20, 25, 29 and 30 reads the current value without changing it.
 * Returns the previous value or EFL_E_INVALID_ARGUMENT. */
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


/* ----------------------------------------------------------------------------------------- */
/* Stage P — Paillier cipher                                                                  */
/* ----------------------------------------------------------------------------------------- */

/*
 * Key context. The reference keeps it in the PaillierKeypair TF resource (paillier.cc:50-331:
 * n, n^2, hs, max, fbpowm table; p, q, p^2, q^2, hp, hq, q^-1 mod p). Here the caller derives
 * the same quantities (plus Montgomery constants), packs them as little-endian 32-bit limbs into
 * ONE device buffer (the "key block") and describes it with this struct; the library never
 * allocates. All big-number offsets are in 32-bit words from the start of the key block.
 *   ln           limbs of n (16, 32, 64, 128 = 512..4096-bit n); n^2 has 2*ln limbs, p and q ln/2,
 *                p^2 and q^2 ln limbs.
 *   n2_minv      -n^2^-1 mod 2^32 (Montgomery), likewise p2_/q2_/p_/q_minv.
 *   off_n2_r2    R^2 mod n^2, R = 2^(32*2*ln);  off_n2_one  R mod n^2
 *   off_table    fbpowm table, table_rows x table_cols entries of 2*ln limbs, entry [i][j] =
 *                hs^((j+1) * 2^(W*i)) * R mod n^2, W = table_window (gmp_utils.cc:56-89 with its
 *                own window; Montgomery form)
 *   off_p2_r3    R'^3 mod p^2, R' = 2^(32*ln) (and q2)
 *   off_pm1      exponent p-1 (ln/2 limbs, pm1_bits significant bits), likewise q-1
 *   off_pinv_w   p^-1 mod 2^(32*ln/2) (exact division by p), likewise q
 *   off_hp       hp * R'' mod p with R'' = 2^(32*ln/2), hp = h-function (paillier.cc:28-37)
 *   off_qinvp    (q^-1 mod p) * R'' mod p
 *   off_max      ceil(2n/3) (paillier.cc:76-77), ln limbs
 */
typedef struct {
  int32_t ln;
  int32_t a_bits;
  int32_t group_size;
  int32_t table_rows;
  int32_t table_cols;
  int32_t has_private;
  int32_t pm1_bits;
  int32_t qm1_bits;
  uint32_t n2_minv, p2_minv, q2_minv, p_minv, q_minv;
  int64_t off_n, off_n2, off_n2_r2, off_n2_one, off_table, off_max;
  int64_t off_p, off_q, off_p2, off_q2, off_p2_r3, off_q2_r3, off_pm1, off_qm1;
  int64_t off_pinv_w, off_qinv_w, off_hp, off_hq, off_qinvp;
  /* Radix-2^28 constants of the decryption exponentiations (sliced kernels, csrc/sliced28.h):
   *   off_p2_28    p^2 as 28-bit limbs (one per 32-bit word), zero-padded to p2_28_len limbs
   *   p2_minv28    -p^2^-1 mod 2^28 (likewise q)
   *   off_p2_r2_28[k]  R28^2 mod p^2 as p2_28_len 28-bit limbs, R28 = 2^(28 L28) for the kernels
   *                that spread a number over G = 2^k lanes, L28 = G * ceil(ceil((32 ln + 2) / 28) / G)
   * has_private == 0 leaves them unused. */
  int32_t p2_28_len;
  uint32_t p2_minv28, q2_minv28;
  int64_t off_p2_28, off_q2_28;
  int64_t off_p2_r2_28[6], off_q2_r2_28[6];
  /* Radix-2^28 fixed-base table for the sliced n^2 kernels that spread n^2 over
   * G = 2^table28_log2g lanes (the family chosen when the key was set):
   *   n2_28_len     L28 = G * ceil(ceil((64 ln + 2) / 28) / G) limbs
   *   off_n2_28     n^2 as L28 28-bit limbs; n2_minv28 = -n^2^-1 mod 2^28
   *   off_n2_one28  R28 mod n^2, R28 = 2^(28 L28)
   *   off_table28   table_rows x table_cols entries of L28 limbs, entry [i][j] =
   *                 hs^((j+1) 2^(W i)) R28 mod n^2; -1 when absent (other families, or a
   *                 table too large to hold twice), and the 32-bit table serves; the powm and
   *                 matmul kernels of that family then also run in 32-bit limbs. */
  int32_t n2_28_len, table28_log2g;
  uint32_t n2_minv28;
  int64_t off_n2_28, off_n2_one28, off_table28;
  int64_t off_n2_r2_28;   /* R28^2 mod n^2 (same L28): powm and matmul of that family in radix 2^28 */
  /* Width W of the fixed-base table's windows (both layouts): table_rows = ceil(a_bits / W),
   * table_cols = 2^W - 1, entry [i][j] = hs^((j+1) 2^(W i)). The kernels bit-reverse a's
   * group_size-bit groups first (a -> a', as mpz_fbpowm's index order does) and then take a' in
   * plain W-bit windows, so W is the build's choice and does not change any result; 0 = W is
   * group_size (the reference's own table, gmp_utils.cc:56-89). */
  int32_t table_window;
  /* The key owner's CRT sub-keys only (key (x, hs mod x^2) for x = p or q, y the other prime; -1
   * elsewhere): radix-2^28 constants (n2_28_len limbs) with which the walk starts from
   * (y^2)^-1 g(m) mod x^2 for each element's plaintext m, so the CRT join of the two walks is the
   * ciphertext itself (efl_pl_ctx_encrypt; the g(m) product mod n^2 then disappears):
   *   off_gn28      (n mod x^2) 2^84 mod x^2: |m| (n mod x^2) by three Montgomery steps
   *   off_gstart28  (y^2)^-1 R28^2 mod x^2, R28 = 2^(28 n2_28_len): g R28 (y^2)^-1 by one product */
  int64_t off_gn28, off_gstart28;
} efl_pl_key;

/*
 * PaillierEncrypt (paillier.cc:443-503, Keypair::Encrypt :103-131): ciphertext[i] (2*ln limbs)
 * = (1 + |m| n)^(sign) * hsa mod n^2. hsa: [n][2*ln] limbs, or NULL for the reference's
 * hsa == "0" case: a fresh a of a_bits bits per element from Philox4x32-10(key = seed, counter =
 * counter_base + i) and hsa = hs^(a') through the fixed-base table (a' = a with every
 * group_size-bit group bit-reversed, as mpz_fbpowm does). n of up to 8192 bits (ln 16/32/64/128/256; a
 * smaller n runs in the smallest class that holds it, zero-padded).
 */
int efl_pl_encrypt(const void* key_block, const efl_pl_key* key, const int64_t* plaintext,
                   const uint32_t* hsa, uint32_t* ciphertext, int64_t n, uint64_t seed,
                   int64_t counter_base, void* stream);

/* FixedBasePowm::mpz_fbpowm (gmp_utils.cc:107-144): hsa[i] = hs^(a_i') mod n^2 for a given
 * [n][ceil(a_bits/32)] (or, a == NULL, the Philox draw of efl_pl_encrypt). */
int efl_pl_fbpowm(const void* key_block, const efl_pl_key* key, const uint32_t* a, uint32_t* hsa,
                  int64_t n, uint64_t seed, int64_t counter_base, void* stream);

/* The key owner's fixed-base exponentiation and encryption by CRT (no reference counterpart: the
 * reference's Encrypt, paillier.cc:103-131, always works mod n^2). v[i] = q^2 yp[i] + p^2 yq[i] mod
 * n^2 for yp[i] < p^2, yq[i] < q^2 ([n][ln] limbs each); with yp = x (q^2)^-1 mod p^2 and yq = x
 * (p^2)^-1 mod q^2, v = x mod n^2. plaintext NULL: z[i] = v[i] ([n][2*ln] limbs). plaintext given
 * (int64 m): v is taken as hsa R mod n^2 (R = 2^(64*ln), the n^2 Montgomery radix) and z[i] =
 * (1 + |m| n)^(sign) hsa mod n^2, the PaillierEncrypt ciphertext, with one Montgomery product. The
 * efl package gets yp and yq from efl_pl_fbpowm under the keys (p, hs mod p^2) and (q, hs mod q^2)
 * whose walks start from R (q^2)^-1 and R (p^2)^-1: the same ciphertexts, bit for bit, from
 * half-length products. ABORTED without the private key. */
int efl_pl_crt_join(const void* key_block, const efl_pl_key* key, const uint32_t* yp, const uint32_t* yq,
                    const int64_t* plaintext, uint32_t* z, int64_t n, void* stream);

/*
 * PaillierDecrypt (paillier.cc:505-561, _Decrypt :296-312): CRT decryption of [n][2*ln]
 * ciphertexts into |m| ([n][ln] limbs) and negative[i] = (m < 0) where m > ceil(2n/3) maps to
 * m - n. ABORTED "No private key." without p, q. n of up to 8192 bits. The sliced kernels take a
 * stream-ordered scratch slab for the sliding-window exponentiation (efl_pl_tune decrypt = 2); a
 * failed allocation returns the HIP error.
 */
int efl_pl_decrypt(const void* key_block, const efl_pl_key* key, const uint32_t* ciphertext,
                   uint32_t* magnitude, int8_t* negative, int64_t n, void* stream);

/* PaillierAdd (paillier.cc:157-178, :563-613): z = x * y mod n^2. */
int efl_pl_add(const void* key_block, const efl_pl_key* key, const uint32_t* x, const uint32_t* y,
               uint32_t* z, int64_t n, void* stream);

/* z = x^e mod n^2 with a per-element non-negative exponent of exp_words 32-bit words
 * (PaillierMulScalar / PaillierMulExp2, paillier.cc:180-265, 615-719). */
int efl_pl_powm(const void* key_block, const efl_pl_key* key, const uint32_t* x, const uint32_t* exps,
                int exp_words, uint32_t* z, int64_t n, void* stream);

/* PaillierMulExp2<int64> (paillier.cc:680-751; the int32 variant after widening): z = x^(2^y) mod
 * n^2, y squarings per element, no host-side exponent. y < 0 is the op's InvalidArgument "y should
 * be a positive tensor." (:724-726, :740-742). One launch squares at most 65536 times per element:
 * y > 65536 is reported like y < 0, and the caller cuts such shifts into launches of at most 65536
 * squarings, x^(2^(a+b)) = (x^(2^a))^(2^b) (efl.privacy.paillier_cipher _exp2_chunked).
 * bad (device, one int64) <- -1, or the smallest such index (its z is 0). */
int efl_pl_mul_exp2(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* y,
                    uint32_t* z, int64_t n, int64_t* bad, void* stream);

/* PaillierMulScalar<int64> (paillier.cc:197-237, :616-678; int32 after widening): z = x^|y| mod n^2,
 * then inverted mod n^2 where y < 0 — the element the reference computes as (x^-1)^|y|. One powm
 * launch plus one in-place inversion launch restricted to the negative scalars. bad <- -1, or the
 * smallest index with y < 0 whose x has no inverse mod n^2 (its z is 0). */
int efl_pl_mul_scalar(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* y,
                      uint32_t* z, int64_t n, int64_t* bad, void* stream);

/* PaillierMulScalar<string> (paillier.cc:239-248: mpz_init_set_str(op, y, 16), signed big-integer
 * scalars): |y| as y_words little-endian 32-bit words per element plus sign bytes (1 = negative),
 * as efl_hex_parse produces them from the hex text; y_negative NULL = all non-negative. Same
 * result and bad convention as efl_pl_mul_scalar. */
int efl_pl_mul_scalar_big(const void* key_block, const efl_pl_key* key, const uint32_t* x,
                          const uint32_t* y_magnitude, int y_words, const int8_t* y_negative, uint32_t* z,
                          int64_t n, int64_t* bad, void* stream);

/* FixedPointTensor.__add__ with encrypted mantissas (python/efl/privacy/paillier.py:116-133):
 * z = x^(2^(xe - m)) * y^(2^(ye - m)) mod n^2, m = min(xe, ye) (the caller keeps m as the exponent):
 * the reference's (x << dl) + (y << dr), i.e. two PaillierMulExp2 and one PaillierAdd, fused into
 * one launch. |xe - ye| > 65536 -> bad as in efl_pl_mul_exp2; the caller then runs the reference's
 * composition with chunked shifts. */
int efl_pl_fxp_add(const void* key_block, const efl_pl_key* key, const uint32_t* x, const int64_t* x_exponent,
                   const uint32_t* y, const int64_t* y_exponent, uint32_t* z, int64_t n, int64_t* bad,
                   void* stream);

/* PaillierInvert (paillier.cc:267-285, :721-797): z = x^-1 mod n^2 (Pornin's batched binary GCD,
 * "Optimized Binary GCD for Modular Inversion", 2020, on the GPU). bad <- -1, or
 * the first index without an inverse (its z is 0). */
int efl_pl_invert(const void* key_block, const efl_pl_key* key, const uint32_t* x, uint32_t* z,
                  int64_t n, int64_t* bad, void* stream);

/* PaillierMatmul (paillier.cc:915-1053) core: x_mantissa [u][v] ciphertexts, x_exponent [u][v],
 * y_mantissa / y_exponent [v][w] int64. For each output z_exponent = min_j(xe + ye) and the terms
 * (x^|y|)^(2^(xe + ye - min)) are multiplied into z_pos (y > 0) or z_neg (y < 0); the caller
 * finishes z = z_pos * z_neg^-1 (efl_pl_invert + efl_pl_add). With the radix-2^28 family the
 * kernels first write x R mod n^2 and its odd powers for every x (u*v*16 padded radix-2^28
 * numbers), then every output's multiply schedule (u*w*S lists of up to 5*ceil(v/S) 32-bit words,
 * S the term split) into scratch taken and released on `stream` (hipMallocAsync / hipFreeAsync);
 * a failed allocation returns the HIP error. An output squares its accumulator once per bit level,
 * up to the exponent spread (max - min of xe + ye over its terms) plus the top bit of |y|: the
 * Python host runs a product whose spread may pass 65536 term by term instead (PaillierMulScalar,
 * chunked PaillierMulExp2, PaillierAdd), so no launch loops that long. */
int efl_pl_matmul(const void* key_block, const efl_pl_key* key, const uint32_t* x_mantissa,
                  const int64_t* x_exponent, const int64_t* y_mantissa, const int64_t* y_exponent,
                  uint32_t* z_pos, uint32_t* z_neg, int64_t* z_exponent, int u, int v, int w,
                  void* stream);

/* Kernel family for keys of ln limbs (16/32/64/128/256): decrypt = 0 selects the n^2 ops (encrypt,
 * fbpowm, add, powm, matmul), 1 decryption. limbs_per_lane 0 = one lane per element (n^2 ops:
 * ln <= 64 only; decryption: ln <= 128), 8, 16 or 32 = one number spread over L/limbs_per_lane lanes
 * (L = 2 ln, or ln for decryption; ln = 256: n^2 ops 32 only); -1 queries; -2 restores the
 * default. Returns the previous choice, or a negative
 * error code. Results are identical across families; only speed differs. With the default
 * (never set, or restored by -2) a decryption of too few elements to give every SIMD a wave takes
 * more lanes per element; a family set explicitly is used for every size. decrypt = 2 selects the
 * sliced decryption's exponentiation instead: limbs_per_lane 1 = sliding 5-bit windows over odd
 * powers kept in a stream-ordered scratch slab (default; hipMallocAsync / hipFreeAsync on the
 * caller's stream, up to 2^18 elements x 16 entries per launch), 0 = binary square-and-multiply
 * (no scratch), -1 queries. decrypt = 3 sets efl_pl_matmul's term splits (radix-2^28 family):
 * limbs_per_lane 0 = chosen per launch (default), 1..16 = that many (rounded down to a power of two,
 * at most v), -1 queries. decrypt = 4 sets the row-split fixed-base walks of the radix-2^28 family
 * (encryption with fresh randomness, efl_pl_fbpowm): a launch of fewer than 4 waves per SIMD splits
 * every element's walk over 1..5 disjoint ranges of table rows and joins the parts in a second
 * launch (stream-ordered scratch), so the waves fill the SIMDs; 0 = parts chosen per launch
 * (default), 1 = never split, 2..5 = that many, -1 queries. decrypt = 5 sets how the key owner's
 * CRT encryption (efl_pl_ctx_encrypt / efl_pl_ctx_fbpowm) runs when one lane holds each of its
 * walks mod p^2 and mod q^2 (1024-bit n): 0 = chosen (default; the paired lanes whenever they
 * apply), 1 = a walk launch per sub-key and the CRT join launch, 2 = the paired lanes: an element's
 * two walks in one wave, its start made and its CRT join done in the same kernel, the waves past
 * the launch's whole rounds split over table rows; -1 queries. Results never change. */
int efl_pl_tune(int ln, int decrypt, int limbs_per_lane);

/* ---- Key context: the PaillierKeypair resource ----------------------------------------------
 * Replaces CreatePaillierKeypair / SetPaillierPublicKey / SetPaillierPrivateKey
 * (efls-train/cc/efl/math/paillier.cc:337-441; PaillierKeypair::SetPublicKey / SetPrivateKey
 * :70-101; the fixed-base table of gmp_utils.cc:56-89) and the Python binding's
 * Keypair.set_public_key / set_private_key (python/efl/privacy/paillier.py:62-73). An opaque
 * context holds the key block(s) above in device memory, derived by the library from the hex text
 * (csrc/keyset.hip): the caller packs nothing. A TF shim keeps one context per keypair resource.
 *
 * Device memory of the fixed-base tables is budgeted PROCESS-WIDE (efl_pl_table_budget; default
 * 4 GiB, EFL_PL_TABLE_BUDGET_MIB) and per context (efl_pl_ctx_options; default 4 GiB,
 * EFL_PL_TABLE_MAX_MIB): a key's table takes the widest window whose table fits what is left; when
 * not even the smallest (W = 1) does, or the reference's own guard trips (entries x bits of n^2 of
 * the table IT would build > 2^40, gmp_utils.h:20), setting the key returns RESOURCE_EXHAUSTED
 * "Memory usage exceeds a predefined threshold." (paillier.cc:399-401). A refused key leaves the
 * context's previous key in place. Setting a key synchronises `stream` (a one-off host op, like the
 * reference's synchronous SetPublicKey). */
typedef struct efl_pl_ctx efl_pl_ctx;

enum {
  EFL_PL_PREPARE_TABLE = 1,   /* efl_pl_ctx_prepare: build the n^2 fixed-base table now */
  EFL_PL_PREPARE_CRT = 2,     /* build the key owner's CRT sub-keys now */
  EFL_PL_PUBLIC_PATH = 1      /* efl_pl_ctx_encrypt / _fbpowm flag: walk the n^2 table even for the key owner */
};

typedef struct {
  int32_t has_public, has_private, n_bytes, ln, a_bits, group_size;
  int32_t table_window;           /* of the n^2 table (planned, if not built yet) */
  int32_t has_table;              /* the n^2 table is built (the key owner's is deferred) */
  int32_t crt_capable;            /* p q = n with half-length primes, CRT encryption enabled */
  int32_t crt;                    /* 1 sub-keys built, 0 not tried, -1 not available (budget) */
  int32_t crt_table_window[2];
  int64_t block_bytes, table_bytes, table_max_bytes;
  int64_t crt_block_bytes[2], crt_table_bytes[2];
  uint64_t generation;            /* changes whenever a pointer efl_pl_ctx_key gave may have */
} efl_pl_ctx_info;

/* CreatePaillierKeypair: an empty context. */
int efl_pl_ctx_create(efl_pl_ctx** ctx);
/* Frees every device block (hipFree: waits for work that still reads them). */
int efl_pl_ctx_destroy(efl_pl_ctx* ctx);
/* Options for the next key set on ctx: table_max_bytes (-1: EFL_PL_TABLE_MAX_MIB or 4 GiB, -2
 * unchanged), table_window (1..24 fixed, 0 chosen against the budget, -1 unchanged; results never
 * depend on it), crt_encrypt (1 on, 0 off, -1 EFL_PL_CRT_ENCRYPT (default on), -2 unchanged). */
int efl_pl_ctx_options(efl_pl_ctx* ctx, int64_t table_max_bytes, int table_window, int crt_encrypt);
/* SetPaillierPublicKey(n, n_bytes, hs, a_bytes, group_size): hex texts (NUL-terminated,
 * mpz_set_str base 16). Drops any private key (paillier.cc:79). The n^2 table is built now unless
 * the key is later made a key owner's. */
int efl_pl_set_public(efl_pl_ctx* ctx, const char* n_hex, int n_bytes, const char* hs_hex, int a_bytes,
                      int group_size, void* stream);
/* Both halves at once (GeneratePaillierKeypair's final step, paillier.cc:889-904): the key owner's
 * n^2 table is then deferred from the start (its encryptions go by CRT). */
int efl_pl_set_keypair(efl_pl_ctx* ctx, const char* n_hex, int n_bytes, const char* hs_hex, int a_bytes,
                       int group_size, const char* p_hex, const char* q_hex, void* stream);
/* SetPaillierPrivateKey(p, q): ignored without a public key (paillier.cc:88-91). p, q distinct odd
 * (INVALID_ARGUMENT otherwise, where the reference's mpz_invert would fail silently). */
int efl_pl_set_private(efl_pl_ctx* ctx, const char* p_hex, const char* q_hex, void* stream);
/* The key block and descriptor every efl_pl_* op above takes: which 0 = the key, 1 / 2 = the key
 * owner's CRT sub-keys (p, hs mod p^2) / (q, hs mod q^2) (after EFL_PL_PREPARE_CRT). ABORTED "No
 * public key." without one. Valid until the next set / prepare / destroy on ctx — and until the next
 * efl_pl_ctx_encrypt / efl_pl_ctx_fbpowm, which prepare implicitly: the first public-path call
 * builds the deferred n^2 table into a new allocation, and the first key-owner call builds the CRT
 * sub-keys and releases an n^2 table built before the private key arrived. Each such move bumps
 * efl_pl_ctx_info.generation: a caller holding a block across calls re-fetches it when that changes.
 * A failed table build leaves the previous table-less block in place (or no key at all), never a
 * freed one; every efl_pl_* op refuses a null block. */
int efl_pl_ctx_key(efl_pl_ctx* ctx, int which, const void** block, efl_pl_key* key);
/* Build what a path needs ahead of use: EFL_PL_PREPARE_TABLE -> 1 (or RESOURCE_EXHAUSTED);
 * EFL_PL_PREPARE_CRT -> 1 sub-keys ready, 0 this key cannot take them (no private key, p q != n, no
 * room in the budget, CRT off). */
int efl_pl_ctx_prepare(efl_pl_ctx* ctx, int what, void* stream);
int efl_pl_ctx_query(efl_pl_ctx* ctx, efl_pl_ctx_info* info);
/* Copy count 32-bit words of block `which` from word off_words into dst (device or host memory). */
int efl_pl_ctx_copy(efl_pl_ctx* ctx, int which, int64_t off_words, int64_t count, void* dst, void* stream);
/* PaillierEncrypt through the context: hsa given -> efl_pl_encrypt; otherwise the key owner's CRT
 * path (sub-keys' walks + efl_pl_crt_join) unless flags has EFL_PL_PUBLIC_PATH, else the n^2 table
 * (built on first use). Same ciphertexts, bit for bit, on every path. The CRT path takes
 * stream-ordered scratch (2 n ln words). */
int efl_pl_ctx_encrypt(efl_pl_ctx* ctx, const int64_t* plaintext, const uint32_t* hsa, uint32_t* ciphertext,
                       int64_t n, uint64_t seed, int64_t counter_base, int flags, void* stream);
/* FixedBasePowm through the context (hs^(a') mod n^2; a NULL = the Philox draw), routed as above. */
int efl_pl_ctx_fbpowm(efl_pl_ctx* ctx, const uint32_t* a, uint32_t* hsa, int64_t n, uint64_t seed,
                      int64_t counter_base, int flags, void* stream);
/* PaillierDecrypt through the context: ABORTED "No private key." without p, q. */
int efl_pl_ctx_decrypt(efl_pl_ctx* ctx, const uint32_t* ciphertext, uint32_t* magnitude, int8_t* negative,
                       int64_t n, void* stream);
/* Process-wide table budget in bytes: bytes >= 0 sets it, < 0 only queries; returns the previous
 * budget; in_use (optional) <- bytes the live contexts' tables hold. */
int64_t efl_pl_table_budget(int64_t bytes, int64_t* in_use);
/* The window rule: widest W <= 24 with ceil(a_bits / W) (2^W - 1) entry_bytes <= max_bytes, 0 if
 * none. */
int efl_pl_choose_window(int a_bits, int64_t entry_bytes, int64_t max_bytes);

/* The host half of setting a key, without the device (tests, inspection): the head words of the key
 * block (the constants, before any table) and its descriptor, for n, hs (and p, q; and a walk start
 * w: the fixed-base walk then starts from w R instead of R, as the CRT sub-keys do), with the table
 * plan (table_rows = rows it will have; off_table = -1). head NULL: *head_words <- the size only. */
int efl_pl_key_derive(const char* n_hex, const char* hs_hex, int a_bytes, int group_size, const char* p_hex,
                      const char* q_hex, const char* walk_hex, int table_window, int64_t allowance,
                      uint32_t* head, int64_t* head_words, efl_pl_key* desc);

/* mpz_get_str(..., 16) of n numbers ([n][limbs_per_elem], optional sign bytes): first the text
 * lengths (efl_hex_lengths), then, given offsets = exclusive prefix sum (n + 1 entries), the
 * characters (efl_hex_write). */
int efl_hex_lengths(const uint32_t* limbs, int limbs_per_elem, const int8_t* negative,
                    int64_t* lengths, int64_t n, void* stream);
int efl_hex_write(const uint32_t* limbs, int limbs_per_elem, const int8_t* negative,
                  const int64_t* offsets, char* chars, int64_t n, void* stream);
/* mpz_set_str(..., 16) of n texts "[-]hexdigits" into limbs; bad <- -1 or the first bad index. */
int efl_hex_parse(const char* chars, const int64_t* offsets, int limbs_per_elem, uint32_t* limbs,
                  int8_t* negative, int64_t n, int64_t* bad, void* stream);
/* PaillierDecrypt<int64> output: mpz_get_sll (gmp_utils.cc:38-45): low 64 bits of |m|, signed. */
int efl_pl_to_int64(const uint32_t* magnitude, int limbs_per_elem, const int8_t* negative,
                    int64_t* out, int64_t n, void* stream);

/* ---- Key generation, HOST memory (GeneratePaillierKeypairOp, paillier.cc:833-904) ------------
 * The reference's keygen is a CPU op over GMP (mpz_probab_prime_p in find_prime, :851-863;
 * mpz_powm for hs, :884-888). These two are its arithmetic, on host buffers of little-endian
 * 32-bit words; the caller draws and sieves the candidates (efl/privacy/paillier_cipher.py). */
/* out = base^exp mod mod, mod odd, base < mod; out has mod_words words. */
int efl_host_powm(const uint32_t* base, int base_words, const uint32_t* exp, int exp_words,
                  const uint32_t* mod, int mod_words, uint32_t* out);
/* Row bases of the fixed-base table (gmp_utils.cc:73-88): out[i] = base^(2^(k i)) mod mod for
 * i < steps ([steps][mod_words] words), mod odd, base < mod; KeyBlock builds every entry from them
 * on the device. */
int efl_host_sqr_chain(const uint32_t* base, int base_words, int k, int steps, const uint32_t* mod,
                       int mod_words, uint32_t* out);
/* Miller-Rabin of `count` odd candidates > 3 ([count][words]) with `reps` bases each
 * ([count][reps][words], in [2, c - 2]): out[i] = 1 probable prime, 0 composite; `threads` host
 * threads (<= 0: all). */
int efl_host_probable_primes(const uint32_t* cands, int words, int count, const uint32_t* bases, int reps,
                             int threads, int8_t* out);

/* ---- Secret-sharing masks -------------------------------------------------
 * Replace the per-element float work of efls-train/python/efl/privacy/secret_sharing.py, whose
 * noise is generate_suitable_noise(t) = tf.random.uniform(shape(t)) * t (:26-27). The uniform is
 * TF's construction (Philox4x32-10, Uint32ToFloat): element i of a call takes word i % 4 of Philox
 * block (ctr0 + i / 4) under key `seed`; a caller advances ctr0 by ceil(n / 4) per call. fp32 only
 * (tf.random.uniform's default dtype). Buffers are device memory, row-major, caller-allocated. */
/* n = U * x / divisor, and: op 0: out0 = n; op 1 (share(), :158-168): out0 = n (sent),
 * out1 = x - n (kept); op 2 (SecretSharingDense noise_divisor, :137-143): out0 = x - n (sent),
 * out1 = x + n (kept). 16-byte aligned buffers. */
int efl_ss_noise(const float* x, float* out0, float* out1, int64_t n, int op, uint64_t seed,
                 uint64_t ctr0, float divisor, void* stream);
/* _matmul mode A side (:30-41), a [rows, cols], cols even, e = U * a:
 * send [rows, 3*cols/2] = [a + e | e[:, ::2] + e[:, 1::2]], keep0 [rows, cols] = a - e,
 * keep1 [rows, cols/2] = e[:, 1::2] - e[:, ::2]. */
int efl_ss_mask_cols(const float* a, float* send, float* keep0, float* keep1, int64_t rows,
                     int64_t cols, uint64_t seed, uint64_t ctr0, void* stream);
/* _matmul mode B side (:42-53), b [rows, cols], rows even, f = U * b:
 * send [3*rows/2, cols] = [b/2 - f ; f[::2] - f[1::2]], keep0 [rows, cols] = b/2 + f,
 * keep1 [rows/2, cols] = f[1::2] + f[::2]. */
int efl_ss_mask_rows(const float* b, float* send, float* keep0, float* keep1, int64_t rows,
                     int64_t cols, uint64_t seed, uint64_t ctr0, void* stream);

/* ---- DP-SGD noise ---------------------------------------------------------
 * The noise step of efls-train/python/efl/privacy/dp_optimizer.py's DP optimisers over a summed
 * gradient x (n floats), then safe_normalize's division (:210-214), in one pass:
 * mode 0 (ElementWiseGaussianSumQuery, :70-71, no l2_norm_clip): out = (x + z * x * sigma) / divisor;
 * mode 1 (GaussianSumQuery, l2_norm_clip set; sigma = its stddev = clip * noise_multiplier):
 * out = (x + (z * sigma + 0)) / divisor. z = tf.random.normal's construction (Philox4x32-10, Box-Muller
 * on word pairs); element i takes normal i % 4 of block ctr0 + i / 4 under `seed`. 16-byte aligned
 * device buffers; out may equal x. */
int efl_dp_noise(const float* x, float* out, int64_t n, int mode, float sigma, float divisor, uint64_t seed,
                 uint64_t ctr0, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* EFL_HIP_H_ */
