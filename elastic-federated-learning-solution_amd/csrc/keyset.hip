// Paillier key setup behind the C ABI: the PaillierKeypair resource of the reference
// (efls-train/cc/efl/math/paillier.cc:50-101 SetPublicKey / SetPrivateKey, :337-441 the
// CreatePaillierKeypair / SetPaillierPublicKey / SetPaillierPrivateKey ops; the fixed-base table of
// gmp_utils.cc:56-89) as an opaque context, efl_pl_ctx (include/efl_hip.h).
//
// Setting a key derives, on the host, every constant the gfx950 kernels read (the reference's n^2,
// ceil(2n/3), hp, hq, q^-1 mod p, plus the Montgomery and radix-2^28 constants of this build, the
// exact-division inverses and the Montgomery radices of the CRT decryption), packs them as one
// device "key block" (efl_pl_key) and builds the fixed-base table on the device: one host chain of
// squarings for the row bases (efl_host_sqr_chain), then W doubling passes of modular products
// (efl_pl_add), then the radix-2^28 copy. The key owner's encryptions go by CRT: two half-length
// sub-keys (p, hs mod p^2) and (q, hs mod q^2) whose walks start from R (q^2)^-1 and R (p^2)^-1, so
// efl_pl_crt_join gives the public-key path's ciphertexts bit for bit; its own n^2 table is built
// only if the public-key path is ever walked.
//
// Device memory of the tables is accounted process-wide (efl_pl_table_budget): a key's window is
// the widest whose table fits what the budget has left (and the context's own cap), and a key
// whose smallest table (W = 1) does not fit is refused with RESOURCE_EXHAUSTED, as the reference
// refuses a table past FBPOWM_MAX_TABLE_MEM (paillier.cc:399-401, gmp_utils.h:20).
#include <stdlib.h>

#include <memory>
#include <mutex>
#include <string>

#include "common.h"
#include "hostbig.h"
#include "pl_common.h"

using efl::hb::Big;
namespace hb = efl::hb;

namespace efl {
namespace {

constexpr int64_t kMaxTableBits = 1LL << 40;      // gmp_utils.h:20, entries x bits of n^2
constexpr int64_t kTable28MaxBytes = 1LL << 36;   // no radix-2^28 copy above this (explicit windows)
constexpr int kWindowMax = 24;
constexpr int64_t kDefaultBytes = 4LL << 30;      // per-context cap and process budget defaults
constexpr int64_t kChunkBytes = 64LL << 20;       // entries one table-build launch moves (at most)

int64_t env_mib(const char* name, int64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const long long x = strtoll(v, &end, 10);
  return (end && *end == 0 && x >= 0) ? (int64_t)x << 20 : dflt;
}

// ---- process-wide table budget ---------------------------------------------------------------
std::mutex g_budget_mu;
int64_t g_budget = -1;      // -1: not read from the environment yet
int64_t g_in_use = 0;

int64_t budget_locked() {
  if (g_budget < 0) g_budget = env_mib("EFL_PL_TABLE_BUDGET_MIB", kDefaultBytes);
  return g_budget;
}
int64_t budget_left() {
  std::lock_guard<std::mutex> g(g_budget_mu);
  const int64_t b = budget_locked();
  return b > g_in_use ? b - g_in_use : 0;
}
// reserve `bytes` only if they fit what is left, checked and taken under one lock: two contexts
// setting keys at once on different threads cannot both size against the same remaining bytes
bool budget_try_take(int64_t bytes) {
  std::lock_guard<std::mutex> g(g_budget_mu);
  if (bytes > 0 && g_in_use + bytes > budget_locked()) return false;
  g_in_use += bytes;
  return true;
}
void budget_give(int64_t bytes) {
  std::lock_guard<std::mutex> g(g_budget_mu);
  g_in_use -= bytes;
}

int64_t limbs28_total(int ln, int G) { return ((32LL * ln + 2 + 27) / 28 + G - 1) / G * G; }

int64_t table_bytes(int a_bits, int W, int64_t entry_bytes) {
  return (int64_t)((a_bits + W - 1) / W) * ((1LL << W) - 1) * entry_bytes;
}

// widest W <= kWindowMax whose table fits max_bytes; 0 when not even W = 1 does
int choose_window(int a_bits, int64_t entry_bytes, int64_t max_bytes) {
  int best = 0;
  for (int W = 1; W <= kWindowMax; ++W) {
    if (table_bytes(a_bits, W, entry_bytes) > max_bytes) break;
    best = W;
  }
  return best;
}

int limb_class(int bits) {
  for (int c : {16, 32, 64, 128, 256})
    if (32 * c >= bits) return c;
  return 0;
}

int hip_fail(hipError_t e, const char* what) {
  if (e == hipErrorOutOfMemory) {
    set_error("%s: out of device memory", what);
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  return hip_status(e, what);
}

// ---- table-build kernels (memory movement around the efl_pl_add products) --------------------

// pass k of the doubling build over entries e in [e0, e0 + count) of the flat (row, i) space of a
// pass with cnt columns: X[e] = T[r][i], Y[e] = P[r][k], r = e / cnt, i = e % cnt
__global__ void k_pass_gather(const uint32_t* __restrict__ T, const uint32_t* __restrict__ P,
                              uint32_t* __restrict__ X, uint32_t* __restrict__ Y, long long e0, long long count,
                              int cnt, int cols, int W, int k, int lc) {
  const long long total = count * lc;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = e0 + t / lc;
    const int w = (int)(t % lc);
    const long long r = e / cnt, i = e % cnt;
    X[t] = T[(r * cols + i) * lc + w];
    Y[t] = P[(r * W + k) * lc + w];
  }
}

// T[r][lo + i] = Z[e]
__global__ void k_pass_scatter(const uint32_t* __restrict__ Z, uint32_t* __restrict__ T, long long e0,
                               long long count, int cnt, int cols, int lo, int lc) {
  const long long total = count * lc;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = e0 + t / lc;
    const int w = (int)(t % lc);
    const long long r = e / cnt, i = e % cnt;
    T[(r * cols + lo + i) * lc + w] = Z[t];
  }
}

// Y[e] = v for e < count (v: lc words)
__global__ void k_bcast(const uint32_t* __restrict__ v, uint32_t* __restrict__ Y, long long count, int lc) {
  const long long total = count * lc;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x)
    Y[t] = v[t % lc];
}

// out[e] = X[e] as L28 radix-2^28 limbs (X[e] < 2^(32 lc); limbs past the value are 0)
__global__ void k_to28(const uint32_t* __restrict__ X, uint32_t* __restrict__ out, long long count, int lc,
                       int L28) {
  const long long total = count * L28;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = t / L28;
    const int j = (int)(t % L28);
    const int bit = 28 * j, q = bit >> 5, r = bit & 31;
    const uint32_t* x = X + e * lc;
    unsigned long long v = q < lc ? x[q] : 0u;
    if (q + 1 < lc) v |= (unsigned long long)x[q + 1] << 32;
    out[t] = (uint32_t)(v >> r) & 0xFFFFFFFu;
  }
}

unsigned grid_for(long long work) {
  long long g = (work + 255) / 256;
  if (g > 65536) g = 65536;
  return (unsigned)(g < 1 ? 1 : g);
}

// ---- one key block ---------------------------------------------------------------------------

struct Block {
  efl_pl_key d{};
  uint32_t* dev = nullptr;          // device key block: head (+ private reserve) (+ tables)
  int64_t dev_words = 0;
  int64_t table_bytes = 0;          // of the attached tables (accounted in the process budget)
  std::vector<uint32_t> head;       // host copy of the head words
  int64_t priv_off = 0, priv_words = 0;   // the private constants' reserved span of the head
  Big n, hs, n2, p, q, walk_start;
  bool has_walk = false, priv = false, has_table = false;
  std::vector<uint32_t> head0;      // head and descriptor before the table was attached (drop_table)
  efl_pl_key d0{};
  int a_bits = 0, g = 1, ln = 0, lc = 0, lh = 0;
  int W = 0, rows = 0, cols = 0, L28 = 0;   // the table's plan (L28 = 0: no radix-2^28 copy)

  ~Block() { release(); }
  void release() {
    if (dev) {
      (void)hipFree(dev);           // synchronises with work that still reads the block
      dev = nullptr;
    }
    if (table_bytes) budget_give(table_bytes);
    table_bytes = 0;
    has_table = false;
  }
};

int64_t put(std::vector<uint32_t>& h, const Big& x, int L) {
  const int64_t off = (int64_t)h.size();
  h.resize(h.size() + L);
  hb::put_words(x, L, h.data() + off);
  return off;
}
int64_t put28(std::vector<uint32_t>& h, const Big& x, int L) {
  const int64_t off = (int64_t)h.size();
  h.resize(h.size() + L);
  hb::put_limbs28(x, L, h.data() + off);
  return off;
}

int64_t private_words(int ln) {
  int64_t Lmax = 0;
  for (int k = 0; k < 6; ++k) Lmax = std::max(Lmax, limbs28_total(ln, 1 << k));
  return 9LL * (ln / 2) + 4LL * ln + 14 * Lmax;
}

// private constants into the head's reserved span (paillier.cc:88-99 plus this build's constants);
// p, q as the block orders them (q < 2p)
int write_private(Block& b, const Big& p, const Big& q) {
  const int ln = b.ln, lh = b.lh;
  efl_pl_key& d = b.d;
  std::vector<uint32_t> h;
  const Big p2 = hb::mul(p, p), q2 = hb::mul(q, q);
  const Big Rh = hb::pow2(32 * lh);
  const Big one(1);
  d.has_private = 1;
  const int64_t base = b.priv_off;
  auto at = [&](int64_t off) { return base + off; };
  d.off_p = at(put(h, p, lh));
  d.off_q = at(put(h, q, lh));
  d.off_p2 = at(put(h, p2, ln));
  d.off_q2 = at(put(h, q2, ln));
  d.p2_minv = hb::minv32(p2);
  d.q2_minv = hb::minv32(q2);
  d.p_minv = hb::minv32(p);
  d.q_minv = hb::minv32(q);
  d.off_p2_r3 = at(put(h, hb::mod(hb::pow2(3 * 32 * ln), p2), ln));
  d.off_q2_r3 = at(put(h, hb::mod(hb::pow2(3 * 32 * ln), q2), ln));
  const Big pm1 = hb::sub(p, one), qm1 = hb::sub(q, one);
  d.off_pm1 = at(put(h, pm1, lh));
  d.off_qm1 = at(put(h, qm1, lh));
  d.pm1_bits = pm1.bits();
  d.qm1_bits = qm1.bits();
  Big pinv, qinv, hp, hq, qinvp;
  if (!hb::modinv(p, Rh, &pinv) || !hb::modinv(q, Rh, &qinv)) {
    set_error("private key: p and q must be odd");
    return EFL_E_INVALID_ARGUMENT;
  }
  d.off_pinv_w = at(put(h, pinv, lh));
  d.off_qinv_w = at(put(h, qinv, lh));
  // h-function (paillier.cc:28-37): hp = L((n + 1)^(p - 1) mod p^2, p)^-1 mod p with L(u, p) =
  // (u - 1) / p. (1 + n)^(p - 1) = 1 + (p - 1) n mod p^2, as every higher binomial term holds n^2.
  for (int s = 0; s < 2; ++s) {
    const Big& x = s ? q : p;
    const Big& x2 = s ? q2 : p2;
    const Big u = hb::mod(hb::add(one, hb::mul(s ? qm1 : pm1, b.n)), x2);
    Big l;
    if (u.zero()) {
      set_error("private key does not fit the public key");
      return EFL_E_INVALID_ARGUMENT;
    }
    hb::divmod(hb::sub(u, one), x, &l, nullptr);
    Big inv;
    if (!hb::modinv(l, x, &inv)) {
      // mpz_invert fails and the reference keeps a stale hp; no decryption can be right then
      set_error("private key: L((n + 1)^(%c - 1) mod %c^2) has no inverse mod %c (p, q do not factor n?)",
                s ? 'q' : 'p', s ? 'q' : 'p', s ? 'q' : 'p');
      return EFL_E_INVALID_ARGUMENT;
    }
    (s ? hq : hp) = inv;
  }
  d.off_hp = at(put(h, hb::mod(hb::mul(hp, Rh), p), lh));
  d.off_hq = at(put(h, hb::mod(hb::mul(hq, Rh), q), lh));
  if (!hb::modinv(q, p, &qinvp)) {
    set_error("private key: q has no inverse mod p");
    return EFL_E_INVALID_ARGUMENT;
  }
  d.off_qinvp = at(put(h, hb::mod(hb::mul(qinvp, Rh), p), lh));
  // radix-2^28 constants of the sliced decryption (csrc/sliced28.h)
  int64_t Lmax = 0;
  for (int k = 0; k < 6; ++k) Lmax = std::max(Lmax, limbs28_total(ln, 1 << k));
  d.p2_28_len = (int32_t)Lmax;
  d.off_p2_28 = at(put28(h, p2, (int)Lmax));
  d.off_q2_28 = at(put28(h, q2, (int)Lmax));
  d.p2_minv28 = hb::minv28(p2);
  d.q2_minv28 = hb::minv28(q2);
  for (int k = 0; k < 6; ++k) {
    const int64_t L28 = limbs28_total(ln, 1 << k);
    const Big r2 = hb::pow2((int)(2 * 28 * L28));
    d.off_p2_r2_28[k] = at(put28(h, hb::mod(r2, p2), (int)Lmax));
    d.off_q2_r2_28[k] = at(put28(h, hb::mod(r2, q2), (int)Lmax));
  }
  if ((int64_t)h.size() != b.priv_words) {
    set_error("internal: private constants take %lld words, %lld reserved", (long long)h.size(),
              (long long)b.priv_words);
    return EFL_E_INTERNAL;
  }
  std::copy(h.begin(), h.end(), b.head.begin() + base);
  b.p = p;
  b.q = q;
  b.priv = true;
  return EFL_OK;
}

// Everything of a key block but its table (KeyBlock of round 4, efl/privacy/paillier_cipher.py):
// validation, the public constants, the private span (filled when p and q are given), the table
// plan. `allowance` bounds the table (0 with an explicit window: no bound but the budget's).
int plan_block(Block& b, const Big& n, const Big& hs, int a_bits, int g, const Big* p, const Big* q,
               int window, int64_t allowance, const Big* walk_start) {
  if (n.bits() < 128) {
    set_error("n of fewer than 128 bits is not supported on the GPU");
    return EFL_E_UNIMPLEMENTED;
  }
  if (!n.odd()) {
    set_error("n must be odd");
    return EFL_E_INVALID_ARGUMENT;
  }
  Big pp, qq;
  const bool priv = p && q;
  if (priv) {
    pp = *p;
    qq = *q;
    if (pp == qq) {
      // q^-1 mod p does not exist: the reference's mpz_invert fails silently there and its
      // decryption is wrong (paillier.cc:88-99); refuse the key instead
      set_error("private key: p and q must be distinct");
      return EFL_E_INVALID_ARGUMENT;
    }
    if (!pp.odd() || !qq.odd() || pp.bits() < 2 || qq.bits() < 2) {
      set_error("private key: p and q must be odd primes");
      return EFL_E_INVALID_ARGUMENT;
    }
    if (hb::cmp(qq, hb::shl(pp, 1)) >= 0) std::swap(pp, qq);   // the CRT reduces mq mod p once: q < 2p
  }
  const int need = std::max(n.bits(), priv ? 2 * std::max(pp.bits(), qq.bits()) : 0);
  const int ln = limb_class(need);
  if (!ln) {
    set_error("n of %d bits: at most 8192 supported", n.bits());
    return EFL_E_UNIMPLEMENTED;
  }
  if (a_bits <= 0 || a_bits > 8192) {
    set_error("a_bytes must be in [1, 1024]");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (g < 1 || g > 20) {
    set_error("group_size must be in [1, 20]");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (window && (window < 1 || window > kWindowMax)) {
    set_error("table_window must be in [1, %d]", kWindowMax);
    return EFL_E_INVALID_ARGUMENT;
  }
  b.n = n;
  b.n2 = hb::mul(n, n);
  b.hs = hb::mod(hs, b.n2);
  b.a_bits = a_bits;
  b.g = g;
  b.ln = ln;
  b.lc = 2 * ln;
  b.lh = ln / 2;
  b.has_walk = walk_start != nullptr;
  if (walk_start) b.walk_start = hb::mod(*walk_start, b.n2);
  // the reference's guard on the table IT would build (api group size g; gmp_utils.cc:66-71)
  const int64_t api_rows = (a_bits + g - 1) / g;
  if ((double)api_rows * (double)((1LL << g) - 1) * (double)b.n2.bits() > (double)kMaxTableBits) {
    set_error("Memory usage exceeds a predefined threshold.");
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  efl_pl_key& d = b.d;
  d = efl_pl_key{};
  std::vector<uint32_t>& h = b.head;
  h.clear();
  const int lc = b.lc;
  const Big Rc = hb::pow2(32 * lc);
  d.ln = ln;
  d.a_bits = a_bits;
  d.group_size = g;
  d.off_n = put(h, n, ln);
  d.off_n2 = put(h, b.n2, lc);
  d.off_n2_r2 = put(h, hb::mod(hb::pow2(2 * 32 * lc), b.n2), lc);
  d.off_n2_one = put(h, hb::mod(Rc, b.n2), lc);
  d.off_max = put(h, hb::cdiv(hb::shl(n, 1), Big(3)), ln);     // paillier.cc:76-77
  d.n2_minv = hb::minv32(b.n2);
  // the radix-2^28 table for the sliced family the n^2 kernels use
  const int fam = efl_pl_tune(ln, 0, -1);
  int64_t L28 = fam > 0 ? limbs28_total(2 * ln, 2 * ln / fam) : 0;
  int W = window;
  if (!W) {
    W = choose_window(a_bits, 4 * (lc + L28), allowance);
    if (!W) {
      set_error("Memory usage exceeds a predefined threshold. (the fixed-base table of the smallest window, "
                "%lld bytes, exceeds the %lld bytes left of the table budget; efl_pl_table_budget)",
                (long long)table_bytes(a_bits, 1, 4 * (lc + L28)), (long long)allowance);
      return EFL_E_RESOURCE_EXHAUSTED;
    }
  }
  const int cols = (1 << W) - 1, rows = (a_bits + W - 1) / W;
  d.table_cols = cols;
  d.table_window = W;
  d.off_table28 = -1;
  d.off_gn28 = d.off_gstart28 = -1;
  d.off_table = -1;
  d.table_rows = 0;                 // no table attached yet: the walks refuse (table_ok)
  if (fam > 0) {
    const int G = 2 * ln / fam;
    if ((int64_t)rows * cols * L28 * 4 <= kTable28MaxBytes) {
      const Big R28 = hb::pow2((int)(28 * L28));
      d.n2_28_len = (int32_t)L28;
      d.table28_log2g = 31 - __builtin_clz((unsigned)G);
      d.n2_minv28 = hb::minv28(b.n2);
      d.off_n2_28 = put28(h, b.n2, (int)L28);
      d.off_n2_one28 = put28(h, hb::mod(R28, b.n2), (int)L28);
      d.off_n2_r2_28 = put28(h, hb::mod(hb::mul(R28, R28), b.n2), (int)L28);
    } else {
      L28 = 0;
    }
  }
  b.W = W;
  b.rows = rows;
  b.cols = cols;
  b.L28 = (int)L28;
  // the private span, reserved whether or not p and q are known yet
  b.priv_off = (int64_t)h.size();
  b.priv_words = private_words(ln);
  h.resize(h.size() + b.priv_words, 0);
  b.priv = false;
  if (priv) return write_private(b, pp, qq);
  return EFL_OK;
}

int64_t planned_table_bytes(const Block& b) { return (int64_t)b.rows * b.cols * (b.lc + b.L28) * 4; }

// upload the head into a fresh device block, with room for the tables when `with_table`
int upload(Block& b, bool with_table, hipStream_t s) {
  const int64_t hw = (int64_t)b.head.size();
  const int64_t tw = with_table ? (int64_t)b.rows * b.cols * (b.lc + b.L28) : 0;
  uint32_t* dev = nullptr;
  hipError_t e = hipMalloc((void**)&dev, (size_t)(hw + tw) * 4);
  if (e != hipSuccess) return hip_fail(e, "key block");
  e = hipMemcpyAsync(dev, b.head.data(), (size_t)hw * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(dev);
    return hip_fail(e, "key block upload");
  }
  b.release();
  b.dev = dev;
  b.dev_words = hw + tw;
  return EFL_OK;
}

struct Scratch {   // stream-ordered device scratch, freed on the stream
  hipStream_t s;
  std::vector<void*> ptrs;
  explicit Scratch(hipStream_t st) : s(st) {}
  ~Scratch() {
    for (void* p : ptrs) (void)hipFreeAsync(p, s);
  }
  hipError_t get(void** p, size_t bytes) {
    hipError_t e = hipMallocAsync(p, bytes ? bytes : 4, s);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
};

#define KS_HIP(expr, what)                          \
  do {                                              \
    const hipError_t e_ = (expr);                   \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)
#define KS_RC(expr)                 \
  do {                              \
    const int rc_ = (expr);         \
    if (rc_ != EFL_OK) return rc_;  \
  } while (0)

// The fixed-base table into the block's table span (b.dev must have room): T[i][j - 1] =
// hs^(j 2^(W i)) R mod n^2 for j in 1 .. 2^W - 1 (gmp_utils.cc:73-88 fills its table with one
// mpz_mul per entry; here one device product per entry as well), plus its radix-2^28 copy.
// Row bases P[i][k] = hs^(2^(W i + k)) from one host chain of squarings (efl_host_sqr_chain);
// column 0 = P[i][0] R, then pass k fills columns 2^k .. 2^(k+1) - 1 of every row at once as
// column c times P[i][k] (efl_pl_add multiplies mod n^2: x R * y = x y R).
int build_table(Block& b, hipStream_t s) {
  // fault injection for the tests (tests/test_ctx_abi_gpu.py): a build that fails after upload()
  // has already let the block's previous allocation go, as a scratch hipMallocAsync OOM would
  const char* fail = getenv("EFL_PL_FAIL_TABLE_BUILD");
  if (fail && fail[0] == '1' && fail[1] == 0) {
    set_error("table build failed (EFL_PL_FAIL_TABLE_BUILD=1 fault injection)");
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  const int lc = b.lc, W = b.W, rows = b.rows, cols = b.cols, L28 = b.L28;
  const int64_t hw = (int64_t)b.head.size();
  uint32_t* T = b.dev + hw;
  uint32_t* T28 = T + (int64_t)rows * cols * lc;
  efl_pl_key d = b.d;               // the table-less descriptor runs the products
  const void* kb = b.dev;
  Scratch sc(s);
  // row bases on the host, uploaded
  std::vector<uint32_t> base((size_t)lc), mod((size_t)lc);
  hb::put_words(b.hs, lc, base.data());
  hb::put_words(b.n2, lc, mod.data());
  std::vector<uint32_t> P((size_t)rows * W * lc);
  KS_RC(efl_host_sqr_chain(base.data(), lc, 1, rows * W, mod.data(), lc, P.data()));
  uint32_t* Pd = nullptr;
  KS_HIP(sc.get((void**)&Pd, P.size() * 4), "table scratch");
  KS_HIP(hipMemcpyAsync(Pd, P.data(), P.size() * 4, hipMemcpyHostToDevice, s), "table upload");
  // entries per launch (EFL_PL_TABLE_CHUNK_BYTES lowers it: tests run the build in many launches)
  const char* cb = getenv("EFL_PL_TABLE_CHUNK_BYTES");
  const int64_t chunk = cb && *cb ? std::max<int64_t>(4 * lc, std::min<int64_t>(kChunkBytes, atoll(cb))) : kChunkBytes;
  const int64_t ce = std::max<int64_t>(1, chunk / (4 * lc));
  uint32_t *X = nullptr, *Y = nullptr, *Z = nullptr;
  const int64_t total_max = std::max<int64_t>(rows, std::min<int64_t>(ce, (int64_t)rows * ((cols + 1) / 2)));
  // (column 0 takes `rows` entries in one launch; every later launch at most total_max)
  KS_HIP(sc.get((void**)&X, (size_t)total_max * lc * 4), "table scratch");
  KS_HIP(sc.get((void**)&Y, (size_t)total_max * lc * 4), "table scratch");
  KS_HIP(sc.get((void**)&Z, (size_t)total_max * lc * 4), "table scratch");
  {
    // column 0: P[i][0] R: X[r] = P[r][0], Y[r] = R mod n^2 (the head's Montgomery one)
    hipLaunchKernelGGL(k_pass_gather, dim3(grid_for((long long)rows * lc)), dim3(256), 0, s, Pd, Pd, X, Y, 0ll,
                       (long long)rows, 1, W, W, 0, lc);
    hipLaunchKernelGGL(k_bcast, dim3(grid_for((long long)rows * lc)), dim3(256), 0, s, b.dev + d.off_n2_one, Y,
                       (long long)rows, lc);
    KS_HIP(hipGetLastError(), "table build");
    KS_RC(efl_pl_add(kb, &d, X, Y, Z, rows, s));
    hipLaunchKernelGGL(k_pass_scatter, dim3(grid_for((long long)rows * lc)), dim3(256), 0, s, Z, T, 0ll,
                       (long long)rows, 1, cols, 0, lc);
    KS_HIP(hipGetLastError(), "table build");
  }
  for (int k = 0; k < W; ++k) {
    const int lo = 1 << k;
    if (cols <= lo) break;
    const int cnt = std::min(lo, cols - lo);
    const int64_t total = (int64_t)rows * cnt;
    for (int64_t e0 = 0; e0 < total; e0 += total_max) {
      const int64_t c = std::min<int64_t>(total_max, total - e0);
      hipLaunchKernelGGL(k_pass_gather, dim3(grid_for((long long)c * lc)), dim3(256), 0, s, T, Pd, X, Y,
                         (long long)e0, (long long)c, cnt, cols, W, k, lc);
      KS_HIP(hipGetLastError(), "table build");
      KS_RC(efl_pl_add(kb, &d, X, Y, Z, c, s));
      hipLaunchKernelGGL(k_pass_scatter, dim3(grid_for((long long)c * lc)), dim3(256), 0, s, Z, T, (long long)e0,
                         (long long)c, cnt, cols, lo, lc);
      KS_HIP(hipGetLastError(), "table build");
    }
  }
  if (L28) {
    // x R -> x R28 = (x R) (R28 R^-1 mod n^2), then cut into 28-bit limbs
    const Big R = hb::pow2(32 * lc), R28 = hb::pow2(28 * L28);
    Big Rinv;
    if (!hb::modinv(R, b.n2, &Rinv)) {
      set_error("internal: R has no inverse mod n^2");
      return EFL_E_INTERNAL;
    }
    std::vector<uint32_t> c28((size_t)lc);
    hb::put_words(hb::mod(hb::mul(R28, Rinv), b.n2), lc, c28.data());
    uint32_t* c28d = nullptr;
    KS_HIP(sc.get((void**)&c28d, (size_t)lc * 4), "table scratch");
    KS_HIP(hipMemcpyAsync(c28d, c28.data(), (size_t)lc * 4, hipMemcpyHostToDevice, s), "table upload");
    hipLaunchKernelGGL(k_bcast, dim3(grid_for((long long)total_max * lc)), dim3(256), 0, s, c28d, Y,
                       (long long)total_max, lc);
    KS_HIP(hipGetLastError(), "table build");
    const int64_t total = (int64_t)rows * cols;
    for (int64_t e0 = 0; e0 < total; e0 += total_max) {
      const int64_t c = std::min<int64_t>(total_max, total - e0);
      KS_RC(efl_pl_add(kb, &d, T + e0 * lc, Y, Z, c, s));
      hipLaunchKernelGGL(k_to28, dim3(grid_for((long long)c * L28)), dim3(256), 0, s, Z, T28 + e0 * L28,
                         (long long)c, lc, L28);
      KS_HIP(hipGetLastError(), "table build");
    }
  }
  KS_HIP(hipStreamSynchronize(s), "table build");
  return EFL_OK;
}

// the walk start into the host head: the walk's initial value w R (and w R28) mod n^2
void apply_walk_host(Block& b) {
  const Big R = hb::pow2(32 * b.lc);
  hb::put_words(hb::mod(hb::mul(b.walk_start, R), b.n2), b.lc, b.head.data() + b.d.off_n2_one);
  if (b.L28) {
    const Big R28 = hb::pow2(28 * b.L28);
    hb::put_limbs28(hb::mod(hb::mul(b.walk_start, R28), b.n2), b.L28, b.head.data() + b.d.off_n2_one28);
  }
}

// attach the built table to the descriptor; a walk start replaces the walk's initial R mod n^2
// (after the build, which multiplies by the true R)
int attach(Block& b, hipStream_t s) {
  const int64_t hw = (int64_t)b.head.size();
  b.d.off_table = hw;
  b.d.table_rows = b.rows;
  b.d.off_table28 = b.L28 ? hw + (int64_t)b.rows * b.cols * b.lc : -1;
  if (b.has_walk) {
    apply_walk_host(b);
    KS_HIP(hipMemcpyAsync(b.dev + b.d.off_n2_one, b.head.data() + b.d.off_n2_one, (size_t)b.lc * 4,
                          hipMemcpyHostToDevice, s), "walk start");
    if (b.L28) {
      KS_HIP(hipMemcpyAsync(b.dev + b.d.off_n2_one28, b.head.data() + b.d.off_n2_one28, (size_t)b.L28 * 4,
                            hipMemcpyHostToDevice, s), "walk start");
    }
    KS_HIP(hipStreamSynchronize(s), "walk start");
  }
  b.has_table = true;
  return EFL_OK;
}

// head + table in one allocation, the table built now. The table's bytes are reserved in the
// process budget first (atomically); on any failure the block is left with no device allocation.
int realise_with_table(Block& b, hipStream_t s) {
  const int64_t tb = planned_table_bytes(b);
  if (!budget_try_take(tb)) {
    set_error("Memory usage exceeds a predefined threshold. (the %lld-byte fixed-base table no longer fits the "
              "table budget; efl_pl_table_budget)", (long long)tb);
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  b.head0 = b.head;
  b.d0 = b.d;
  const int rc0 = upload(b, true, s);
  if (rc0 != EFL_OK) {
    budget_give(tb);
    return rc0;
  }
  b.table_bytes = tb;
  int rc = build_table(b, s);
  if (rc == EFL_OK) rc = attach(b, s);
  if (rc != EFL_OK) b.release();
  return rc;
}

// back to the table-less head in a fresh allocation (the table's bytes go back to the budget):
// after a failed table build (whose upload had already let the old allocation go), or to hand a
// key owner's unused n^2 table to its CRT sub-tables. The previous error text is kept.
int drop_table(Block& b, hipStream_t s) {
  if (!b.head0.empty()) {
    b.head = b.head0;
    b.d = b.d0;
  }
  const std::string err = efl_last_error();
  const int rc = upload(b, false, s);
  if (rc == EFL_OK) set_error("%s", err.c_str());
  return rc;
}

}  // namespace
}  // namespace efl

using namespace efl;

// ---- the context ------------------------------------------------------------------------------

struct efl_pl_ctx {
  std::mutex mu;
  int64_t cap = -1;                  // per-context table cap (-1: EFL_PL_TABLE_MAX_MIB or 4 GiB)
  int window = 0;                    // explicit table window (0: chosen against the budget)
  int crt_mode = -1;                 // -1: EFL_PL_CRT_ENCRYPT (default on), 0 off, 1 on
  std::unique_ptr<Block> main;
  std::unique_ptr<Block> sub[2];
  int crt = 0;                       // 0 not tried, 1 sub-keys built, -1 not available
  int n_bytes = 0;
  uint64_t generation = 0;           // bumped whenever a pointer efl_pl_ctx_key handed out may change

  int64_t cap_bytes() const { return cap >= 0 ? cap : env_mib("EFL_PL_TABLE_MAX_MIB", kDefaultBytes); }
  int64_t held() const {
    int64_t t = main ? main->table_bytes : 0;
    for (auto& s : sub) t += s ? s->table_bytes : 0;
    return t;
  }
  // the cap bounds each of the context's two table sets (its n^2 table; the key owner's CRT pair),
  // the process-wide budget bounds them all
  int64_t allowance() const { return std::max<int64_t>(0, std::min(cap_bytes(), budget_left())); }
  bool crt_enabled() const {
    if (crt_mode >= 0) return crt_mode == 1;
    const char* v = getenv("EFL_PL_CRT_ENCRYPT");
    return !(v && v[0] == '0' && v[1] == 0);
  }
  // the key owner's encryption goes by CRT: p q = n, p != q, half-length primes of a limb class
  bool crt_capable() const {
    if (!main || !main->priv || !crt_enabled()) return false;
    const Block& b = *main;
    if (b.p == b.q || hb::mul(b.p, b.q) != b.n) return false;
    return 2 * limb_class(b.p.bits()) == b.ln && 2 * limb_class(b.q.bits()) == b.ln;
  }
  void drop_crt() {
    sub[0].reset();
    sub[1].reset();
    crt = 0;
  }
};

namespace {

int parse_hex(const char* s, const char* what, Big* out) {
  if (!s) {
    set_error("%s: null text", what);
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!hb::from_hex(s, strlen(s), out)) {
    set_error("%s is not a hex integer", what);
    return EFL_E_INVALID_ARGUMENT;
  }
  return EFL_OK;
}

// build the owner's CRT sub-keys if it can take them; false (not an error) when the key cannot, or
// when the budget holds no table for them
int ensure_crt(efl_pl_ctx* c, hipStream_t s, bool* ok) {
  *ok = false;
  if (c->crt == 1) {
    *ok = true;
    return EFL_OK;
  }
  if (c->crt == -1 || !c->crt_capable()) return EFL_OK;
  const Block& m = *c->main;
  const Big p2 = hb::mul(m.p, m.p), q2 = hb::mul(m.q, m.q);
  const Big R = hb::pow2(32 * m.lc);     // the n^2 Montgomery radix: the join yields hsa R
  Big ip, iq;
  if (!hb::modinv(q2, p2, &ip) || !hb::modinv(p2, q2, &iq)) {
    c->crt = -1;
    return EFL_OK;
  }
  // the two sub-tables take half each of what the context may hold (round 4's split: W = 18 for the
  // examples' 1024-bit key under the 4 GiB default); the owner's own n^2 table, built only if the
  // public-key path is walked, is sized against what the budget has left then
  int64_t each = c->allowance() / 2;
  std::unique_ptr<Block> sb[2];
  for (int i = 0; i < 2; ++i) {
    if (i == 0 && c->main->has_table && !c->window) {
      // A key that got its public half first (set_public, then set_private: the reference's usual
      // order) holds the n^2 table the owner's CRT encryption does not walk. When keeping it would
      // give the sub-tables a narrower window than releasing it (W 18 -> 12 under the
      // 4 GiB default), it is released and the sub-tables are sized as efl_pl_set_keypair sizes
      // them; with room for both (a larger budget) it stays. An explicit window keeps it too.
      Block probe;
      const Big R0 = hb::mul(R, ip);
      int rc = plan_block(probe, m.p, hb::mod(m.hs, p2), m.a_bits, m.g, nullptr, nullptr, 0, each, &R0);
      if ((rc == EFL_OK || rc == EFL_E_RESOURCE_EXHAUSTED) && probe.lc > 0) {
        const int64_t freed = std::max<int64_t>(0, std::min(c->cap_bytes(), budget_left() + c->main->table_bytes)) / 2;
        const int w_keep = rc == EFL_OK ? probe.W : 0;
        const int w_drop = choose_window(m.a_bits, 4LL * (probe.lc + probe.L28), freed);
        if (w_drop > w_keep) {
          KS_RC(drop_table(*c->main, s));
          ++c->generation;
          each = c->allowance() / 2;
        }
      }
    }
    const Big& x = i ? m.q : m.p;
    const Big x2 = i ? q2 : p2;
    const Big start = hb::mul(R, i ? iq : ip);    // walks give hs^(a') R (q^2)^-1 mod p^2, ...
    sb[i].reset(new Block());
    int rc = plan_block(*sb[i], x, hb::mod(m.hs, x2), m.a_bits, m.g, nullptr, nullptr, c->window, each, &start);
    if (rc == EFL_E_RESOURCE_EXHAUSTED) {
      c->crt = -1;                   // no room: the public-key path serves
      return EFL_OK;
    }
    if (rc != EFL_OK) return rc;
    if (sb[i]->L28) {
      // the per-element walk start (y^2)^-1 g(m) mod x^2 (efl_pl_key off_gn28 / off_gstart28)
      Block& b = *sb[i];
      const Big& y2 = i ? p2 : q2;
      Big y2inv;
      if (hb::modinv(y2, x2, &y2inv)) {
        const Big R28 = hb::pow2(28 * b.L28);
        b.d.off_gn28 = put28(b.head, hb::mod(hb::shl(hb::mod(m.n, x2), 84), x2), b.L28);
        b.d.off_gstart28 = put28(b.head, hb::mod(hb::mul(y2inv, hb::mod(hb::mul(R28, R28), x2)), x2), b.L28);
      }
    }
    if (c->window && planned_table_bytes(*sb[i]) > budget_left()) {
      c->crt = -1;
      return EFL_OK;
    }
    rc = realise_with_table(*sb[i], s);
    if (rc == EFL_E_RESOURCE_EXHAUSTED) {
      c->crt = -1;
      return EFL_OK;
    }
    if (rc != EFL_OK) return rc;
  }
  c->sub[0] = std::move(sb[0]);
  c->sub[1] = std::move(sb[1]);
  c->crt = 1;
  ++c->generation;
  *ok = true;
  return EFL_OK;
}

// the n^2 table of the main block (deferred for the key owner)
int ensure_table(efl_pl_ctx* c, hipStream_t s) {
  Block& b = *c->main;
  if (b.has_table) return EFL_OK;
  if (!c->window) {
    // re-plan the window against what the budget has left now (the owner's sub-tables hold part)
    const int64_t eb = 4LL * (b.lc + b.L28);
    const int W = choose_window(b.a_bits, eb, c->allowance());
    if (!W) {
      set_error("Memory usage exceeds a predefined threshold. (no room left in the table budget for the "
                "n^2 fixed-base table; efl_pl_table_budget)");
      return EFL_E_RESOURCE_EXHAUSTED;
    }
    if (W != b.W) {
      b.W = W;
      b.cols = (1 << W) - 1;
      b.rows = (b.a_bits + W - 1) / W;
      b.d.table_cols = b.cols;
      b.d.table_window = W;
      if (b.L28 && (int64_t)b.rows * b.cols * b.L28 * 4 > kTable28MaxBytes) {
        set_error("internal: radix-2^28 table over its cap after re-planning");
        return EFL_E_INTERNAL;
      }
    }
  } else if (planned_table_bytes(b) > budget_left()) {
    set_error("Memory usage exceeds a predefined threshold. (table_window %d needs %lld bytes, %lld left in "
              "the table budget)", c->window, (long long)planned_table_bytes(b), (long long)budget_left());
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  const int rc = realise_with_table(b, s);
  ++c->generation;
  if (rc != EFL_OK) {
    // the failed build had let the old allocation go: put the table-less head back, so every entry
    // point still finds a live key block; if not even that works, the context holds no
    // key ("No public key.") rather than a dangling block. The build's error is what is reported.
    const std::string err = efl_last_error();
    if (drop_table(b, s) != EFL_OK) {
      c->drop_crt();
      c->main.reset();
    }
    set_error("%s", err.c_str());
  }
  return rc;
}

int need_public(efl_pl_ctx* c) {
  if (!c) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!c->main) {
    set_error("No public key.");
    return EFL_E_ABORTED;
  }
  return EFL_OK;
}

}  // namespace

EFL_API int efl_pl_ctx_create(efl_pl_ctx** out) {
  if (!out) {
    set_error("efl_pl_ctx_create: null output");
    return EFL_E_INVALID_ARGUMENT;
  }
  *out = new efl_pl_ctx();
  return EFL_OK;
}

EFL_API int efl_pl_ctx_destroy(efl_pl_ctx* ctx) {
  delete ctx;                        // hipFree of every block synchronises with work still using it
  return EFL_OK;
}

EFL_API int efl_pl_ctx_options(efl_pl_ctx* ctx, int64_t table_max_bytes, int table_window, int crt_encrypt) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (table_window != -1 && (table_window < 0 || table_window > kWindowMax)) {
    set_error("table_window must be in [1, %d] (0: chosen, -1: unchanged)", kWindowMax);
    return EFL_E_INVALID_ARGUMENT;
  }
  if (crt_encrypt < -2 || crt_encrypt > 1) {
    set_error("crt_encrypt must be 0, 1, -1 (environment) or -2 (unchanged)");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  if (table_max_bytes != -2) ctx->cap = table_max_bytes < 0 ? -1 : table_max_bytes;
  if (table_window != -1) ctx->window = table_window;
  if (crt_encrypt != -2) ctx->crt_mode = crt_encrypt;
  return EFL_OK;
}

static int set_key(efl_pl_ctx* ctx, const Big& n, int n_bytes, const Big& hs, int a_bytes, int group_size,
                   const Big* p, const Big* q, hipStream_t s) {
  // everything that can be refused is checked on the host before the old key is let go of: a
  // refused key leaves the context as it was
  std::unique_ptr<Block> b(new Block());
  // the old key's tables are released first, so the new key's window is chosen against the budget
  // without them (the budget without this context's own holdings)
  const int64_t own = ctx->held();
  const int64_t allowance =
      std::max<int64_t>(0, std::min(ctx->cap_bytes(), budget_left() + own));
  int rc = plan_block(*b, n, hs, 8 * a_bytes, group_size, p, q, ctx->window, allowance, nullptr);
  if (rc != EFL_OK) return rc;
  if (ctx->window && planned_table_bytes(*b) > budget_left() + own) {
    set_error("Memory usage exceeds a predefined threshold. (table_window %d needs %lld bytes, %lld left in the "
              "table budget)", ctx->window, (long long)planned_table_bytes(*b), (long long)(budget_left() + own));
    return EFL_E_RESOURCE_EXHAUSTED;
  }
  ctx->drop_crt();
  ctx->main.reset();
  ++ctx->generation;
  // the key owner's own n^2 table is deferred: its encryptions go by CRT (ensure_table)
  ctx->main = std::move(b);
  const bool defer = ctx->crt_capable();
  rc = defer ? upload(*ctx->main, false, s) : realise_with_table(*ctx->main, s);
  if (rc != EFL_OK) {
    ctx->main.reset();
    return rc;
  }
  ctx->n_bytes = n_bytes;
  return EFL_OK;
}

EFL_API int efl_pl_set_public(efl_pl_ctx* ctx, const char* n_hex, int n_bytes, const char* hs_hex, int a_bytes,
                              int group_size, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  Big n, hs;
  int rc = parse_hex(n_hex, "n", &n);
  if (rc == EFL_OK) rc = parse_hex(hs_hex, "hs", &hs);
  if (rc != EFL_OK) return rc;
  std::lock_guard<std::mutex> g(ctx->mu);
  return set_key(ctx, n, n_bytes, hs, a_bytes, group_size, nullptr, nullptr, (hipStream_t)stream);
}

// GeneratePaillierKeypair's last step (paillier.cc:889-904 sets both halves of the resource): the
// public and the private key at once, so a key owner's n^2 table is deferred from the start
EFL_API int efl_pl_set_keypair(efl_pl_ctx* ctx, const char* n_hex, int n_bytes, const char* hs_hex, int a_bytes,
                               int group_size, const char* p_hex, const char* q_hex, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  Big n, hs, p, q;
  int rc = parse_hex(n_hex, "n", &n);
  if (rc == EFL_OK) rc = parse_hex(hs_hex, "hs", &hs);
  if (rc == EFL_OK) rc = parse_hex(p_hex, "p", &p);
  if (rc == EFL_OK) rc = parse_hex(q_hex, "q", &q);
  if (rc != EFL_OK) return rc;
  std::lock_guard<std::mutex> g(ctx->mu);
  return set_key(ctx, n, n_bytes, hs, a_bytes, group_size, &p, &q, (hipStream_t)stream);
}

EFL_API int efl_pl_set_private(efl_pl_ctx* ctx, const char* p_hex, const char* q_hex, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  Big p, q;
  int rc = parse_hex(p_hex, "p", &p);
  if (rc == EFL_OK) rc = parse_hex(q_hex, "q", &q);
  if (rc != EFL_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->main) return EFL_OK;     // ignored without a public key (paillier.cc:88-91)
  Block& b = *ctx->main;
  Big pp = p, qq = q;
  if (hb::cmp(qq, hb::shl(pp, 1)) >= 0) std::swap(pp, qq);
  if (b.priv && b.p == pp && b.q == qq) return EFL_OK;     // the same private key: nothing changes
  const int need = std::max(b.n.bits(), 2 * std::max(p.bits(), q.bits()));
  if (limb_class(need) != b.ln) {
    // the private key needs a wider limb class than the public key: a new block
    return set_key(ctx, b.n, ctx->n_bytes, b.hs, b.a_bits / 8, b.g, &p, &q, s);
  }
  if (p == q) {
    set_error("private key: p and q must be distinct");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (!p.odd() || !q.odd() || p.bits() < 2 || q.bits() < 2) {
    set_error("private key: p and q must be odd primes");
    return EFL_E_INVALID_ARGUMENT;
  }
  // into the reserved span, in place: the public part and its table do not change
  Block trial;
  trial.head = b.head;
  trial.d = b.d;
  trial.n = b.n;
  trial.ln = b.ln;
  trial.lh = b.lh;
  trial.priv_off = b.priv_off;
  trial.priv_words = b.priv_words;
  rc = write_private(trial, pp, qq);
  if (rc != EFL_OK) return rc;
  KS_HIP(hipMemcpyAsync(b.dev + b.priv_off, trial.head.data() + b.priv_off, (size_t)b.priv_words * 4,
                        hipMemcpyHostToDevice, s), "private key upload");
  KS_HIP(hipStreamSynchronize(s), "private key upload");
  b.head.swap(trial.head);
  b.d = trial.d;
  b.p = pp;
  b.q = qq;
  b.priv = true;
  ctx->drop_crt();
  ++ctx->generation;
  return EFL_OK;
}

EFL_API int efl_pl_ctx_key(efl_pl_ctx* ctx, int which, const void** block, efl_pl_key* key) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (which < 0 || which > 2 || !block || !key) {
    set_error("efl_pl_ctx_key: which must be 0 (the key), 1 or 2 (the CRT sub-keys), outputs non-null");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  const Block* b = which ? ctx->sub[which - 1].get() : ctx->main.get();
  if (!b) {
    set_error("efl_pl_ctx_key: no CRT sub-key (efl_pl_ctx_prepare(ctx, EFL_PL_PREPARE_CRT) first)");
    return EFL_E_FAILED_PRECONDITION;
  }
  *block = b->dev;
  *key = b->d;
  return EFL_OK;
}

EFL_API int efl_pl_ctx_prepare(efl_pl_ctx* ctx, int what, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (what == EFL_PL_PREPARE_TABLE) {
    rc = ensure_table(ctx, s);
    return rc == EFL_OK ? 1 : rc;
  }
  if (what == EFL_PL_PREPARE_CRT) {
    bool ok = false;
    rc = ensure_crt(ctx, s, &ok);
    return rc == EFL_OK ? (ok ? 1 : 0) : rc;
  }
  set_error("efl_pl_ctx_prepare: what must be EFL_PL_PREPARE_TABLE or EFL_PL_PREPARE_CRT");
  return EFL_E_INVALID_ARGUMENT;
}

EFL_API int efl_pl_ctx_query(efl_pl_ctx* ctx, efl_pl_ctx_info* info) {
  if (!ctx || !info) {
    set_error("null argument");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  *info = efl_pl_ctx_info{};
  info->generation = ctx->generation;
  info->table_max_bytes = ctx->cap_bytes();
  if (!ctx->main) return EFL_OK;
  const Block& b = *ctx->main;
  info->has_public = 1;
  info->has_private = b.priv ? 1 : 0;
  info->n_bytes = ctx->n_bytes;
  info->ln = b.ln;
  info->a_bits = b.a_bits;
  info->group_size = b.g;
  info->table_window = b.W;
  info->has_table = b.has_table ? 1 : 0;
  info->crt_capable = ctx->crt_capable() ? 1 : 0;
  info->crt = ctx->crt;
  info->block_bytes = b.dev_words * 4;
  info->table_bytes = b.table_bytes;
  for (int i = 0; i < 2; ++i)
    if (ctx->sub[i]) {
      info->crt_table_window[i] = ctx->sub[i]->W;
      info->crt_block_bytes[i] = ctx->sub[i]->dev_words * 4;
      info->crt_table_bytes[i] = ctx->sub[i]->table_bytes;
    }
  return EFL_OK;
}

EFL_API int efl_pl_ctx_copy(efl_pl_ctx* ctx, int which, int64_t off_words, int64_t count, void* dst,
                            void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  const Block* b = (which >= 1 && which <= 2) ? ctx->sub[which - 1].get() : which == 0 ? ctx->main.get() : nullptr;
  if (!b || !dst || off_words < 0 || count < 0 || off_words + count > b->dev_words) {
    set_error("efl_pl_ctx_copy: bad block, range or destination");
    return EFL_E_INVALID_ARGUMENT;
  }
  KS_HIP(hipMemcpyAsync(dst, b->dev + off_words, (size_t)count * 4, hipMemcpyDefault, (hipStream_t)stream),
         "efl_pl_ctx_copy");
  return EFL_OK;
}

// the CRT path: hs^(a') mod p^2 and mod q^2 through the sub-keys' tables, then the join (with the
// plaintext: g(m) hsa in one Montgomery product)
static int crt_run(efl_pl_ctx* c, const uint32_t* a, const int64_t* m, uint32_t* out, int64_t n, uint64_t seed,
                   int64_t ctr, hipStream_t s) {
  const Block& mb = *c->main;
  // round 5: each walk starts from the element's (y^2)^-1 g(m), so the join of the two walks is the
  // ciphertext and no product mod n^2 is left (k_fbpowm28g); otherwise the walks start from the
  // key's R (y^2)^-1 and the join multiplies by g(m) mod n^2 (efl_pl_crt_join with the plaintext)
  bool direct = c->sub[0]->d.off_gn28 >= 0 && c->sub[1]->d.off_gn28 >= 0;
  if (direct) {
    // an element's two walks in one wave, joined at the end (round 5): the ciphertext in one pass
    const Block& s0 = *c->sub[0];
    const Block& s1 = *c->sub[1];
    const int fam = efl_pl_tune(s0.ln, 0, -1);
    const hipError_t e = pl::sl_crt_encrypt_pair(pl::Key{s0.dev, s0.d}, pl::Key{s1.dev, s1.d}, fam > 0 ? fam : 0,
                                                 mb.dev + mb.d.off_n2, (const long long*)m, a, out, (long long)n, seed,
                                                 (long long)ctr, s);
    if (e == hipSuccess) return EFL_OK;
    if (e != hipErrorNotSupported) return hip_fail(e, "CRT encryption");
  }
  Scratch sc(s);
  uint32_t* y[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; ++i) KS_HIP(sc.get((void**)&y[i], (size_t)n * c->sub[i]->lc * 4), "CRT scratch");
  for (int i = 0; i < 2 && direct; ++i) {
    const Block& sb = *c->sub[i];
    const int fam = efl_pl_tune(sb.ln, 0, -1);
    const hipError_t e = pl::sl_fbpowm_g(pl::Key{sb.dev, sb.d}, fam > 0 ? fam : 0, (const long long*)m, a, y[i],
                                         (long long)n, seed, (long long)ctr, s);
    if (e == hipErrorNotSupported) direct = false;
    else if (e != hipSuccess) return hip_fail(e, "CRT walk");
  }
  if (direct) return efl_pl_crt_join(mb.dev, &mb.d, y[0], y[1], nullptr, out, n, s);
  for (int i = 0; i < 2; ++i) KS_RC(efl_pl_fbpowm(c->sub[i]->dev, &c->sub[i]->d, a, y[i], n, seed, ctr, s));
  const int64_t* mm = m;
  if (!mm) {                         // g(0) = 1: the join gives hs^(a') itself
    int64_t* z = nullptr;
    KS_HIP(sc.get((void**)&z, (size_t)n * 8), "CRT scratch");
    KS_HIP(hipMemsetAsync(z, 0, (size_t)n * 8, s), "CRT scratch");
    mm = z;
  }
  return efl_pl_crt_join(mb.dev, &mb.d, y[0], y[1], mm, out, n, s);
}

EFL_API int efl_pl_ctx_encrypt(efl_pl_ctx* ctx, const int64_t* plaintext, const uint32_t* hsa, uint32_t* ciphertext,
                               int64_t n, uint64_t seed, int64_t counter_base, int flags, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (n < 0) {
    set_error("negative count");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (n == 0) return EFL_OK;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  const Block& b = *ctx->main;
  if (hsa) return efl_pl_encrypt(b.dev, &b.d, plaintext, hsa, ciphertext, n, seed, counter_base, s);
  if (!(flags & EFL_PL_PUBLIC_PATH)) {
    bool ok = false;
    KS_RC(ensure_crt(ctx, s, &ok));
    if (ok) return crt_run(ctx, nullptr, plaintext, ciphertext, n, seed, counter_base, s);
  }
  KS_RC(ensure_table(ctx, s));
  const Block& bt = *ctx->main;
  return efl_pl_encrypt(bt.dev, &bt.d, plaintext, nullptr, ciphertext, n, seed, counter_base, s);
}

EFL_API int efl_pl_ctx_fbpowm(efl_pl_ctx* ctx, const uint32_t* a, uint32_t* hsa, int64_t n, uint64_t seed,
                              int64_t counter_base, int flags, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (n < 0) {
    set_error("negative count");
    return EFL_E_INVALID_ARGUMENT;
  }
  if (n == 0) return EFL_OK;
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  if (!(flags & EFL_PL_PUBLIC_PATH)) {
    bool ok = false;
    KS_RC(ensure_crt(ctx, s, &ok));
    if (ok) return crt_run(ctx, a, nullptr, hsa, n, seed, counter_base, s);
  }
  KS_RC(ensure_table(ctx, s));
  const Block& b = *ctx->main;
  return efl_pl_fbpowm(b.dev, &b.d, a, hsa, n, seed, counter_base, s);
}

EFL_API int efl_pl_ctx_decrypt(efl_pl_ctx* ctx, const uint32_t* ciphertext, uint32_t* magnitude, int8_t* negative,
                               int64_t n, void* stream) {
  if (!ctx) {
    set_error("null context");
    return EFL_E_INVALID_ARGUMENT;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = need_public(ctx);
  if (rc != EFL_OK) return rc;
  const Block& b = *ctx->main;
  if (!b.priv) {
    set_error("No private key.");
    return EFL_E_ABORTED;
  }
  return efl_pl_decrypt(b.dev, &b.d, ciphertext, magnitude, negative, n, (hipStream_t)stream);
}

EFL_API int64_t efl_pl_table_budget(int64_t bytes, int64_t* in_use) {
  std::lock_guard<std::mutex> g(g_budget_mu);
  const int64_t prev = budget_locked();
  if (bytes >= 0) g_budget = bytes;
  if (in_use) *in_use = g_in_use;
  return prev;
}

EFL_API int efl_pl_choose_window(int a_bits, int64_t entry_bytes, int64_t max_bytes) {
  if (a_bits <= 0 || entry_bytes <= 0) {
    set_error("efl_pl_choose_window: a_bits and entry_bytes must be positive");
    return EFL_E_INVALID_ARGUMENT;
  }
  return choose_window(a_bits, entry_bytes, max_bytes);
}

// The host half of setting a key, alone (no device): the head words and descriptor a key block
// would get (table not attached: table_rows 0, off_table -1). For tests and for callers that want
// to inspect the derivation; p_hex / q_hex / walk_hex may be NULL. head NULL: *head_words gets
// the size only.
EFL_API int efl_pl_key_derive(const char* n_hex, const char* hs_hex, int a_bytes, int group_size, const char* p_hex,
                              const char* q_hex, const char* walk_hex, int table_window, int64_t allowance,
                              uint32_t* head, int64_t* head_words, efl_pl_key* desc) {
  if (!head_words || !desc) {
    set_error("efl_pl_key_derive: null output");
    return EFL_E_INVALID_ARGUMENT;
  }
  Big n, hs, p, q, w;
  int rc = parse_hex(n_hex, "n", &n);
  if (rc == EFL_OK) rc = parse_hex(hs_hex, "hs", &hs);
  if (rc == EFL_OK && p_hex) rc = parse_hex(p_hex, "p", &p);
  if (rc == EFL_OK && q_hex) rc = parse_hex(q_hex, "q", &q);
  if (rc == EFL_OK && walk_hex) rc = parse_hex(walk_hex, "walk start", &w);
  if (rc != EFL_OK) return rc;
  Block b;
  rc = plan_block(b, n, hs, 8 * a_bytes, group_size, p_hex && q_hex ? &p : nullptr, p_hex && q_hex ? &q : nullptr,
                  table_window, allowance, walk_hex ? &w : nullptr);
  if (rc != EFL_OK) return rc;
  if (b.has_walk) apply_walk_host(b);
  if (head) {
    if (*head_words < (int64_t)b.head.size()) {
      set_error("efl_pl_key_derive: head needs %lld words", (long long)b.head.size());
      return EFL_E_INVALID_ARGUMENT;
    }
    std::copy(b.head.begin(), b.head.end(), head);
  }
  *head_words = (int64_t)b.head.size();
  *desc = b.d;
  desc->table_rows = b.rows;          // the plan (not attached)
  return EFL_OK;
}
