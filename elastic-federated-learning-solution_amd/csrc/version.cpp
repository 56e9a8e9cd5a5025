// efl_version(): names the sources libefl_hip.so was built from. The Makefile hashes every
// kernel source and header (sha256 of csrc/* in sorted order, then include/efl_hip.h) into
// EFL_SRC_HASH and rebuilds this file whenever one of them changes, so a run's log shows which
// kernels it used and tests/test_abi.py can check that the library matches the tree.
#include "efl_hip.h"

#ifndef EFL_SRC_HASH
#define EFL_SRC_HASH "unknown"
#endif

extern "C" __attribute__((visibility("default"))) const char* efl_version(void) {
  return "efl-hip 0.2.0 (gfx950) src " EFL_SRC_HASH;
}
