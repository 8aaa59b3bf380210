// Host side of the C ABI (include/hbbft_hip.h): device/stream/workspace management and batch
// orchestration of the HIP kernels in kernels.hpp.  No CPU fallback: every verdict comes from
// the GPU; without a usable device the calls fail with HBH_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hbbft_hip.h"
#include "kernels.hpp"

using namespace hb;

namespace {

thread_local std::string g_last_error = "";

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HBH_CHECK(expr)                                                                           \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return fail(HBH_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));            \
  } while (0)

// A growable device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 4096;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

inline int pad64(size_t n) { return (int)((n + 63) / 64 * 64); }

}  // namespace

struct hbh_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // workspaces
  DevBuf coef1, coef2, inf1, inf2;
  // staging for host-pointer entry points
  DevBuf in_p1, in_q1, in_i1, in_p2, in_q2, in_i2, out_v;
};

namespace {

size_t coef_bytes(size_t npts) { return (size_t)MILLER_STEPS * LINE_Q4 * pad64(npts) * sizeof(uint4); }

int launch_prepare(hbh_engine* e, hipStream_t s, const void* d_pts, size_t n, DevBuf& coef, DevBuf& inf) {
  if (n == 0) return HBH_OK;
  HBH_CHECK(coef.ensure(coef_bytes(n)));
  HBH_CHECK(inf.ensure(n));
  const int threads = 256;
  const int blocks = (int)((n + threads - 1) / threads);
  hipLaunchKernelGGL(k_g2_prepare, dim3(blocks), dim3(threads), 0, s, (int)n, (const uint32_t*)d_pts, pad64(n),
                     (uint4*)coef.p, (uint8_t*)inf.p);
  HBH_CHECK(hipGetLastError());
  return HBH_OK;
}

int run_pairing_eq_dev(hbh_engine* e, hipStream_t s, size_t n, const void* d_p1, const void* d_q1, size_t nq1,
                       const uint32_t* d_i1, const void* d_p2, const void* d_q2, size_t nq2, const uint32_t* d_i2,
                       uint8_t* d_v) {
  if (n == 0) return HBH_OK;
  if (n > (size_t)1 << 30 || nq1 > (size_t)1 << 30 || nq2 > (size_t)1 << 30) return fail(HBH_ERR_ARG, "batch too large");
  int rc = launch_prepare(e, s, d_q1, nq1, e->coef1, e->inf1);
  if (rc) return rc;
  rc = launch_prepare(e, s, d_q2, nq2, e->coef2, e->inf2);
  if (rc) return rc;
  const int threads = 256;
  const int blocks = (int)((n + threads - 1) / threads);
  hipLaunchKernelGGL(k_pairing_eq, dim3(blocks), dim3(threads), 0, s, (int)n, (const uint32_t*)d_p1,
                     (const uint4*)e->coef1.p, pad64(nq1), (const uint8_t*)e->inf1.p, d_i1, (const uint32_t*)d_p2,
                     (const uint4*)e->coef2.p, pad64(nq2), (const uint8_t*)e->inf2.p, d_i2, d_v);
  HBH_CHECK(hipGetLastError());
  return HBH_OK;
}

int check_idx(const uint32_t* idx, size_t n, size_t table) {
  if (!idx) return table == n ? HBH_OK : fail(HBH_ERR_ARG, "identity index map requires table size == n");
  for (size_t i = 0; i < n; i++)
    if (idx[i] >= table) return fail(HBH_ERR_ARG, "index out of range");
  return HBH_OK;
}

// Host-pointer pairing-eq: stage to device, run, copy verdicts back, synchronise.
int run_pairing_eq_host(hbh_engine* e, size_t n, const uint8_t* p1, const uint8_t* q1, size_t nq1, const uint32_t* i1,
                        const uint8_t* p2, const uint8_t* q2, size_t nq2, const uint32_t* i2, uint8_t* v) {
  if (n == 0) return HBH_OK;
  if (!p1 || !q1 || !p2 || !q2 || !v) return fail(HBH_ERR_ARG, "null pointer");
  int rc = check_idx(i1, n, nq1);
  if (rc) return rc;
  rc = check_idx(i2, n, nq2);
  if (rc) return rc;
  hipStream_t s = e->stream;
  HBH_CHECK(e->in_p1.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(e->in_p2.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(e->in_q1.ensure(nq1 * HBH_G2_BYTES));
  HBH_CHECK(e->in_q2.ensure(nq2 * HBH_G2_BYTES));
  HBH_CHECK(e->out_v.ensure(n));
  HBH_CHECK(hipMemcpyAsync(e->in_p1.p, p1, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_p2.p, p2, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_q1.p, q1, nq1 * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_q2.p, q2, nq2 * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  const uint32_t* d_i1 = nullptr;
  const uint32_t* d_i2 = nullptr;
  if (i1) {
    HBH_CHECK(e->in_i1.ensure(n * 4));
    HBH_CHECK(hipMemcpyAsync(e->in_i1.p, i1, n * 4, hipMemcpyHostToDevice, s));
    d_i1 = (const uint32_t*)e->in_i1.p;
  }
  if (i2) {
    HBH_CHECK(e->in_i2.ensure(n * 4));
    HBH_CHECK(hipMemcpyAsync(e->in_i2.p, i2, n * 4, hipMemcpyHostToDevice, s));
    d_i2 = (const uint32_t*)e->in_i2.p;
  }
  rc = run_pairing_eq_dev(e, s, n, e->in_p1.p, e->in_q1.p, nq1, d_i1, e->in_p2.p, e->in_q2.p, nq2, d_i2,
                          (uint8_t*)e->out_v.p);
  if (rc) return rc;
  HBH_CHECK(hipMemcpyAsync(v, e->out_v.p, n, hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

// G1 generator in the ABI format (canonical LE words), built once on the host.
const std::vector<uint8_t>& g1_generator_bytes() {
  static std::vector<uint8_t> g = [] {
    std::vector<uint8_t> b(HBH_G1_BYTES);
    Fp x = fp_from_mont(fp_const(G1X_M)), y = fp_from_mont(fp_const(G1Y_M));
    uint32_t w[24];
    fp_limbs_to_words(x, w);
    fp_limbs_to_words(y, w + 12);
    std::memcpy(b.data(), w, sizeof(w));
    return b;
  }();
  return g;
}

std::vector<uint8_t> repeat(const std::vector<uint8_t>& rec, size_t n) {
  std::vector<uint8_t> out(rec.size() * n);
  for (size_t i = 0; i < n; i++) std::memcpy(out.data() + i * rec.size(), rec.data(), rec.size());
  return out;
}

}  // namespace

extern "C" {

const char* hbh_last_error(void) { return g_last_error.c_str(); }

int hbh_device_count(int* out) {
  if (!out) return fail(HBH_ERR_ARG, "null pointer");
  int c = 0;
  hipError_t err = hipGetDeviceCount(&c);
  if (err != hipSuccess) {
    *out = 0;
    return fail(HBH_ERR_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(err));
  }
  *out = c;
  return HBH_OK;
}

int hbh_engine_create(int device, hbh_engine** out) {
  if (!out) return fail(HBH_ERR_ARG, "null pointer");
  *out = nullptr;
  int count = 0;
  HBH_CHECK(hipGetDeviceCount(&count));
  if (device < 0 || device >= count) return fail(HBH_ERR_ARG, "device ordinal out of range");
  HBH_CHECK(hipSetDevice(device));
  hbh_engine* e = new hbh_engine();
  e->device = device;
  hipError_t err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (err != hipSuccess) {
    delete e;
    return fail(HBH_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(err));
  }
  *out = e;
  return HBH_OK;
}

int hbh_engine_destroy(hbh_engine* e) {
  if (!e) return HBH_OK;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  for (DevBuf* b : {&e->coef1, &e->coef2, &e->inf1, &e->inf2, &e->in_p1, &e->in_q1, &e->in_i1, &e->in_p2, &e->in_q2,
                    &e->in_i2, &e->out_v})
    b->release();
  (void)hipStreamDestroy(e->stream);
  delete e;
  return HBH_OK;
}

int hbh_verify_pairing_eq(hbh_engine* e, size_t n, const uint8_t* p1, const uint8_t* q1, size_t nq1,
                          const uint32_t* i1, const uint8_t* p2, const uint8_t* q2, size_t nq2, const uint32_t* i2,
                          uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, p1, q1, nq1, i1, p2, q2, nq2, i2, v);
}

int hbh_verify_pairing_eq_dev(hbh_engine* e, void* stream, size_t n, const void* d_p1, const void* d_q1, size_t nq1,
                              const uint32_t* d_i1, const void* d_p2, const void* d_q2, size_t nq2,
                              const uint32_t* d_i2, uint8_t* d_v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n && (!d_p1 || !d_q1 || !d_p2 || !d_q2 || !d_v)) return fail(HBH_ERR_ARG, "null pointer");
  if ((!d_i1 && nq1 != n) || (!d_i2 && nq2 != n)) return fail(HBH_ERR_ARG, "identity index map requires table size == n");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  return run_pairing_eq_dev(e, s, n, d_p1, d_q1, nq1, d_i1, d_p2, d_q2, nq2, d_i2, d_v);
}

int hbh_verify_sig_shares(hbh_engine* e, size_t n, const uint8_t* pks, const uint8_t* sigs, const uint8_t* hashes,
                          size_t ndocs, const uint32_t* doc_idx, uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  std::vector<uint8_t> g1s = repeat(g1_generator_bytes(), n);
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, pks, hashes, ndocs, doc_idx, g1s.data(), sigs, n, nullptr, v);
}

int hbh_verify_dec_shares(hbh_engine* e, size_t n, const uint8_t* shares, const uint8_t* pks, const uint8_t* huv,
                          const uint8_t* w, size_t ncts, const uint32_t* ct_idx, uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, shares, huv, ncts, ct_idx, pks, w, ncts, ct_idx, v);
}

int hbh_verify_ciphertexts(hbh_engine* e, size_t n, const uint8_t* u, const uint8_t* w, const uint8_t* huv,
                           uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  std::vector<uint8_t> g1s = repeat(g1_generator_bytes(), n);
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, g1s.data(), w, n, nullptr, u, huv, n, nullptr, v);
}

int hbh_dbg_pairing(hbh_engine* e, size_t n, const uint8_t* p, const uint8_t* q, uint8_t* out) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!p || !q || !out) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  HBH_CHECK(e->in_p1.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(e->in_q1.ensure(n * HBH_G2_BYTES));
  HBH_CHECK(e->out_v.ensure(n * 576));
  HBH_CHECK(hipMemcpyAsync(e->in_p1.p, p, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_q1.p, q, n * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  int rc = launch_prepare(e, s, e->in_q1.p, n, e->coef1, e->inf1);
  if (rc) return rc;
  const int threads = 256;
  hipLaunchKernelGGL(k_dbg_pairing, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads), 0, s, (int)n,
                     (const uint32_t*)e->in_p1.p, (const uint4*)e->coef1.p, pad64(n), (const uint8_t*)e->inf1.p,
                     (uint32_t*)e->out_v.p);
  HBH_CHECK(hipGetLastError());
  HBH_CHECK(hipMemcpyAsync(out, e->out_v.p, n * 576, hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // extern "C"
