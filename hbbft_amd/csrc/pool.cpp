// Multi-device fan-out behind the C ABI (include/hbbft_hip.h, "engine pool").
//
// A pool owns one hbh_engine per shard (a device may carry several shards: each engine has its
// own HIP stream and workspaces).  A batched call is split by INSTANCE -- document, ciphertext,
// combine or SyncKeyGen part -- into contiguous instance ranges of about equal item counts, so the
// per-instance tables (H, W, H_uv line tables; 595-point commitments) live on one shard only.
// Each shard runs on its own host thread against its own engine; verdicts and points are
// scattered back into the caller's order.  No collective: the outputs are independent per item
// (SURVEY §8e).  The reference has one synchronous caller per node (src/traits.rs:297-336), which
// this keeps: a pool call returns when every shard is done.
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbbft_hip.h"

extern "C" void hbh__set_error(const char* msg);  // engine.hip: the calling thread's hbh_last_error

struct hbh_pool {
  std::vector<hbh_engine*> eng;
  std::vector<int> device;
};

namespace {

constexpr size_t G1B = HBH_G1_BYTES, G2B = HBH_G2_BYTES, FRB = HBH_FR_BYTES;

int pfail(int rc, const std::string& msg) {
  hbh__set_error(msg.c_str());
  return rc;
}

// Contiguous instance ranges [b[s], b[s+1]) with about total/S items each.
std::vector<size_t> split_instances(const std::vector<size_t>& count, size_t shards) {
  size_t total = 0;
  for (size_t c : count) total += c;
  std::vector<size_t> b(shards + 1, count.size());
  b[0] = 0;
  size_t acc = 0, s = 1;
  for (size_t i = 0; i < count.size() && s < shards; i++) {
    acc += count[i];
    while (s < shards && acc * shards >= total * s) b[s++] = i + 1;
  }
  for (size_t k = 1; k <= shards; k++)
    if (b[k] < b[k - 1]) b[k] = b[k - 1];
  return b;
}

// Run fn(shard) on one thread per shard; the first failure's code and message win.
template <class F>
int run_shards(size_t shards, F fn) {
  std::vector<int> rc(shards, HBH_OK);
  std::vector<std::string> err(shards);
  std::vector<std::thread> th;
  th.reserve(shards);
  for (size_t s = 0; s < shards; s++)
    th.emplace_back([&, s] {
      rc[s] = fn(s);
      if (rc[s] != HBH_OK) err[s] = hbh_last_error();
    });
  for (auto& t : th) t.join();
  for (size_t s = 0; s < shards; s++)
    if (rc[s] != HBH_OK) return pfail(rc[s], "shard " + std::to_string(s) + ": " + err[s]);
  return HBH_OK;
}

void gather(std::vector<uint8_t>& dst, const uint8_t* src, size_t i, size_t sz) {
  dst.insert(dst.end(), src + i * sz, src + (i + 1) * sz);
}

// Items grouped by instance: items[s] = original positions owned by shard s (in order), inst_lo[s]
// = first instance of shard s.
struct Plan {
  std::vector<std::vector<size_t>> items;
  std::vector<size_t> bounds;
};

int plan(size_t n, size_t ninst, const uint32_t* inst, size_t shards, Plan& p) {
  std::vector<size_t> count(ninst, 0);
  for (size_t i = 0; i < n; i++) {
    const size_t k = inst ? inst[i] : i;
    if (k >= ninst) return pfail(HBH_ERR_ARG, "instance index out of range");
    count[k]++;
  }
  p.bounds = split_instances(count, shards);
  std::vector<uint32_t> owner(ninst);
  for (size_t s = 0; s < shards; s++)
    for (size_t k = p.bounds[s]; k < p.bounds[s + 1]; k++) owner[k] = (uint32_t)s;
  p.items.assign(shards, {});
  for (size_t i = 0; i < n; i++) p.items[owner[inst ? inst[i] : i]].push_back(i);
  return HBH_OK;
}

}  // namespace

extern "C" {

int hbh_pool_create(const int* devices, int nshards, hbh_pool** out) {
  if (!out || !devices || nshards <= 0) return pfail(HBH_ERR_ARG, "bad pool arguments");
  *out = nullptr;
  auto* p = new hbh_pool();
  for (int s = 0; s < nshards; s++) {
    hbh_engine* e = nullptr;
    const int rc = hbh_engine_create(devices[s], &e);
    if (rc != HBH_OK) {
      const std::string msg = hbh_last_error();
      hbh_pool_destroy(p);
      return pfail(rc, "pool shard " + std::to_string(s) + " (device " + std::to_string(devices[s]) + "): " + msg);
    }
    p->eng.push_back(e);
    p->device.push_back(devices[s]);
  }
  *out = p;
  return HBH_OK;
}

int hbh_pool_destroy(hbh_pool* p) {
  if (!p) return HBH_OK;
  int rc = HBH_OK;
  for (auto* e : p->eng) {
    const int r = hbh_engine_destroy(e);
    if (r != HBH_OK && rc == HBH_OK) rc = r;
  }
  delete p;
  return rc;
}

int hbh_pool_shards(const hbh_pool* p, int* out) {
  if (!p || !out) return pfail(HBH_ERR_ARG, "null pool");
  *out = (int)p->eng.size();
  return HBH_OK;
}

int hbh_pool_engine(hbh_pool* p, int shard, hbh_engine** out) {
  if (!p || !out || shard < 0 || (size_t)shard >= p->eng.size()) return pfail(HBH_ERR_ARG, "bad shard");
  *out = p->eng[shard];
  return HBH_OK;
}

int hbh_pool_set_pairing_impl(hbh_pool* p, int impl) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  for (auto* e : p->eng) {
    const int rc = hbh_engine_set_pairing_impl(e, impl);
    if (rc != HBH_OK) return rc;
  }
  return HBH_OK;
}

int hbh_pool_verify_sig_shares(hbh_pool* p, size_t n, const uint8_t* pks, const uint8_t* sigs, const uint8_t* hashes,
                               size_t ndocs, const uint32_t* doc_idx, uint8_t* verdicts) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  if (n == 0) return HBH_OK;
  if (!pks || !sigs || !hashes || !verdicts) return pfail(HBH_ERR_ARG, "null pointer");
  if (!doc_idx && ndocs != n) return pfail(HBH_ERR_ARG, "doc_idx == NULL needs ndocs == n");
  Plan pl;
  const size_t S = p->eng.size();
  int rc = plan(n, ndocs, doc_idx, S, pl);
  if (rc) return rc;
  return run_shards(S, [&](size_t s) -> int {
    const auto& it = pl.items[s];
    if (it.empty()) return HBH_OK;
    const size_t lo = pl.bounds[s], nd = pl.bounds[s + 1] - lo;
    std::vector<uint8_t> pk, sg, v(it.size());
    std::vector<uint32_t> di;
    pk.reserve(it.size() * G1B);
    sg.reserve(it.size() * G2B);
    for (size_t i : it) {
      gather(pk, pks, i, G1B);
      gather(sg, sigs, i, G2B);
      di.push_back((uint32_t)((doc_idx ? doc_idx[i] : i) - lo));
    }
    const int r = hbh_verify_sig_shares(p->eng[s], it.size(), pk.data(), sg.data(), hashes + lo * G2B, nd, di.data(),
                                        v.data());
    if (r == HBH_OK)
      for (size_t k = 0; k < it.size(); k++) verdicts[it[k]] = v[k];
    return r;
  });
}

int hbh_pool_verify_dec_shares(hbh_pool* p, size_t n, const uint8_t* shares, const uint8_t* pks, const uint8_t* huv,
                               const uint8_t* w, size_t ncts, const uint32_t* ct_idx, uint8_t* verdicts) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  if (n == 0) return HBH_OK;
  if (!shares || !pks || !huv || !w || !verdicts) return pfail(HBH_ERR_ARG, "null pointer");
  if (!ct_idx && ncts != n) return pfail(HBH_ERR_ARG, "ct_idx == NULL needs ncts == n");
  Plan pl;
  const size_t S = p->eng.size();
  int rc = plan(n, ncts, ct_idx, S, pl);
  if (rc) return rc;
  return run_shards(S, [&](size_t s) -> int {
    const auto& it = pl.items[s];
    if (it.empty()) return HBH_OK;
    const size_t lo = pl.bounds[s], nc = pl.bounds[s + 1] - lo;
    std::vector<uint8_t> sh, pk, v(it.size());
    std::vector<uint32_t> ci;
    for (size_t i : it) {
      gather(sh, shares, i, G1B);
      gather(pk, pks, i, G1B);
      ci.push_back((uint32_t)((ct_idx ? ct_idx[i] : i) - lo));
    }
    const int r = hbh_verify_dec_shares(p->eng[s], it.size(), sh.data(), pk.data(), huv + lo * G2B, w + lo * G2B, nc,
                                        ci.data(), v.data());
    if (r == HBH_OK)
      for (size_t k = 0; k < it.size(); k++) verdicts[it[k]] = v[k];
    return r;
  });
}

int hbh_pool_combine_verify_g2(hbh_pool* p, size_t ncomb, int t, const uint32_t* idx, const uint8_t* shares,
                               const uint8_t* master_pk, const uint8_t* hashes, uint8_t* out, int* status,
                               uint8_t* verdicts) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  if (ncomb == 0) return HBH_OK;
  if (t < 0) return pfail(HBH_ERR_ARG, "negative threshold");
  const size_t S = p->eng.size(), k = (size_t)t + 1;
  return run_shards(S, [&](size_t s) -> int {
    const size_t lo = ncomb * s / S, hi = ncomb * (s + 1) / S;
    if (hi == lo) return HBH_OK;
    return hbh_combine_verify_g2(p->eng[s], hi - lo, t, idx ? idx + lo * k : nullptr, shares + lo * k * G2B,
                                 master_pk, hashes + lo * G2B, out + lo * G2B, status + lo, verdicts + lo);
  });
}

int hbh_pool_interpolate_g1(hbh_pool* p, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out,
                            int* status) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  if (ncomb == 0) return HBH_OK;
  if (t < 0) return pfail(HBH_ERR_ARG, "negative threshold");
  const size_t S = p->eng.size(), k = (size_t)t + 1;
  return run_shards(S, [&](size_t s) -> int {
    const size_t lo = ncomb * s / S, hi = ncomb * (s + 1) / S;
    if (hi == lo) return HBH_OK;
    return hbh_interpolate_g1(p->eng[s], hi - lo, t, idx ? idx + lo * k : nullptr, pts + lo * k * G1B,
                              out + lo * G1B, status + lo);
  });
}

int hbh_pool_bivar_ack_check(hbh_pool* p, size_t nack, int t, size_t nparts, const uint8_t* commits,
                             const uint32_t* part_idx, const uint32_t* xs, const uint32_t* ys, const uint8_t* vals,
                             uint8_t* verdicts) {
  if (!p) return pfail(HBH_ERR_ARG, "null pool");
  if (nack == 0) return HBH_OK;
  if (t < 0) return pfail(HBH_ERR_ARG, "negative threshold");
  if (!commits || !part_idx || !xs || !ys || !vals || !verdicts) return pfail(HBH_ERR_ARG, "null pointer");
  const size_t ncoef = ((size_t)t + 1) * ((size_t)t + 2) / 2;
  Plan pl;
  const size_t S = p->eng.size();
  int rc = plan(nack, nparts, part_idx, S, pl);
  if (rc) return rc;
  return run_shards(S, [&](size_t s) -> int {
    const auto& it = pl.items[s];
    if (it.empty()) return HBH_OK;
    const size_t lo = pl.bounds[s], np = pl.bounds[s + 1] - lo;
    std::vector<uint32_t> pi, x, y;
    std::vector<uint8_t> va, v(it.size());
    for (size_t a : it) {
      pi.push_back((uint32_t)(part_idx[a] - lo));
      x.push_back(xs[a]);
      y.push_back(ys[a]);
      gather(va, vals, a, FRB);
    }
    const int r = hbh_bivar_ack_check(p->eng[s], it.size(), t, np, commits + lo * ncoef * G1B, pi.data(), x.data(),
                                      y.data(), va.data(), v.data());
    if (r == HBH_OK)
      for (size_t k = 0; k < it.size(); k++) verdicts[it[k]] = v[k];
    return r;
  });
}

}  // extern "C"
