/*
 * Sanitizer driver for libefl_hip.so's host side: the C-ABI argument checking and error text
 * that run before any HIP call (fxp.hip, version.cpp), built with -Xarch_host
 * -fsanitize=address,undefined and exercised without a GPU: every invalid-argument path of the
 * Stage-F entry points, efl_fxp_tune's ranges, efl_last_error's thread-local text. Driven by
 * tests/test_sanitizers.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "efl_hip.h"

static int fails = 0;
#define CHECK(c, msg)                                              \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, msg, efl_last_error()); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main(void) {
  void* p = (void*)(uintptr_t)16;
  CHECK(strstr(efl_version(), "gfx950") != NULL, "version");
  CHECK(efl_fxp_decode(NULL, NULL, NULL, EFL_DT_FLOAT, 3, 4, 0, NULL) == EFL_E_INVALID_ARGUMENT, "size mismatch");
  CHECK(strstr(efl_last_error(), "same size") != NULL, "size mismatch text");
  CHECK(efl_fxp_decode(NULL, NULL, NULL, EFL_DT_FLOAT, -1, -1, 0, NULL) == EFL_E_INVALID_ARGUMENT, "negative");
  CHECK(efl_fxp_decode(NULL, NULL, NULL, EFL_DT_FLOAT, 0, 0, 0, NULL) == EFL_OK, "empty decode");
  CHECK(efl_fxp_decode(NULL, NULL, NULL, EFL_DT_FLOAT, 5, 5, 0, NULL) == EFL_E_INVALID_ARGUMENT, "null decode");
  CHECK(efl_fxp_decode(p, p, p, EFL_DT_INT32, 5, 5, 0, NULL) == EFL_E_INVALID_ARGUMENT, "decode dtype");
  CHECK(strstr(efl_last_error(), "unsupported dtype") != NULL, "decode dtype text");
  CHECK(efl_fxp_encode(NULL, EFL_DT_FLOAT, NULL, NULL, 0, 0, NULL) == EFL_OK, "empty encode");
  CHECK(efl_fxp_encode(NULL, EFL_DT_FLOAT, NULL, NULL, 5, 0, NULL) == EFL_E_INVALID_ARGUMENT, "null encode");
  CHECK(efl_fxp_encode(p, EFL_DT_FLOAT, p, p, -5, 0, NULL) == EFL_E_INVALID_ARGUMENT, "negative encode");
  CHECK(efl_fxp_encode(p, EFL_DT_STRING, p, p, 5, 0, NULL) == EFL_E_INVALID_ARGUMENT, "encode dtype");
  CHECK(efl_fxp_decode_hex(NULL, NULL, NULL, NULL, EFL_DT_FLOAT, 1, 0, NULL, NULL) == EFL_E_INVALID_ARGUMENT,
        "hex null status");
  CHECK(efl_fxp_decode_hex(NULL, NULL, NULL, NULL, EFL_DT_FLOAT, -1, 0, p, NULL) == EFL_E_INVALID_ARGUMENT,
        "hex negative");
  CHECK(efl_fxp_encode_batched(NULL, EFL_DT_FLOAT, NULL, NULL, NULL, -1, 0, 0, NULL) == EFL_E_INVALID_ARGUMENT,
        "batched negative");
  CHECK(efl_fxp_encode_batched(NULL, EFL_DT_FLOAT, NULL, NULL, NULL, 0, 0, 0, NULL) == EFL_OK, "batched empty");
  CHECK(efl_fxp_decode_batched(NULL, NULL, NULL, EFL_DT_FLOAT, NULL, 3, -1, 0, NULL) == EFL_E_INVALID_ARGUMENT,
        "batched decode negative");
  for (int kind = -2; kind < 12; ++kind)
    for (int v = -1; v < 1100; v += 37) {
      const int prev = efl_fxp_tune(kind, v);
      if (prev >= 0) efl_fxp_tune(kind, prev);
    }
  /* a long error text is truncated, not overflowed */
  char big[2000];
  memset(big, 'a', sizeof big - 1);
  big[sizeof big - 1] = 0;
  CHECK(efl_fxp_decode(NULL, NULL, NULL, EFL_DT_FLOAT, 1, 2, 0, NULL) == EFL_E_INVALID_ARGUMENT, "again");
  if (fails) return 1;
  printf("abi sanitizer driver: ok\n");
  return 0;
}
