// Host side of the C ABI (include/hbbft_hip.h): device/stream/workspace management and batch
// orchestration of the HIP kernels behind launch.hpp.  No CPU fallback: every verdict comes from
// the GPU; without a usable device the calls fail with HBH_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/hbbft_hip.h"
#include "launch.hpp"
#include "interp_pair.hpp"
#include "wire.hpp"

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

}  // namespace

// Per-stage kernel timing (hbh_engine_set_profiling): HIP events recorded around each stage's
// launch on the stream it runs on, summed by hbh_engine_stage_time.
struct StageTimer {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[HBH_NUM_STAGES];
  hipEvent_t begin(hipStream_t s, int stage, bool on) {
    if (!on) return nullptr;
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return nullptr;
    if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return nullptr; }
    (void)hipEventRecord(a, s);
    ev[stage].push_back({a, b});
    return b;
  }
  void end(hipStream_t s, hipEvent_t b) {
    if (b) (void)hipEventRecord(b, s);
  }
  void clear() {
    for (auto& v : ev) {
      for (auto& p : v) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
      }
      v.clear();
    }
  }
};

// split master check when the call has at most split_waves_max(t) one-pair Miller waves
// (ncomb x (t + 2)).  Crossover against interpolate-then-verify, interpolated linearly between the
// measured batch sizes of profiles/r03/split_sweep_auto.jsonl: t = 21 at ~45 combines (~1,046 waves;
// 32 combines split 2.81 vs 3.60 ms, 48 combines 3.80 vs 3.70 ms), t = 33 at ~38 combines (~1,340
// waves; 33 combines 4.26 vs 4.66 ms, 40 combines 4.75 vs 4.59 ms).  One wave cap cannot fit both
// (ADVICE r3), so the cap grows with t through those two points: 540 + 24 t.
// HBH_SPLIT_MAX=<combines> in the environment replaces the rule by a plain combine count (A/B).
inline size_t split_waves_max(int t) { return 540 + 24 * (size_t)t; }
struct hbh_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  bool profiling = false;
  int impl = HBH_IMPL_AUTO;  // pairing implementation (hbh_engine_set_pairing_impl)
  int ack_impl = HBH_ACK_AUTO;  // Ack-check kernel of commitment sets (hbh_engine_set_ack_impl)
  StageTimer timer;
  // Completion of the last call's device work on whichever stream it ran.  Every call waits for it
  // on its own stream before touching the engine-owned workspaces, so a _dev call on a caller
  // stream can never overwrite tables another stream's kernels are still reading.
  hipEvent_t done = nullptr;
  // HBH_IMPL_PAIR device-pointer calls alternate between two table slots, each with its own
  // completion event: consecutive calls on different streams then overlap (one call's verify tail
  // with the next call's table walk and first waves) without sharing a workspace.  Every other
  // call waits for both slots and records both.
  hipEvent_t slot_done[2] = {nullptr, nullptr};
  int slot = 0;
  DevBuf ptab[2][2], pinf[2][2];
  // Device-pointer point decoding (hbh_g*_decompress_dev) alternates between two staging slots of
  // its own (wire words + flags), with its own completion events: a node's decode of one batch then
  // runs beside the previous batch's verify on another stream (the whole-node sign line, bench.py
  // --from-wire) instead of waiting for it.  It touches no other engine workspace.
  hipEvent_t wire_done[2] = {nullptr, nullptr};
  int wire_slot = 0;
  DevBuf wire_w[2], wire_f[2];
  // host staging of combine digits (kept alive until the call's stream synchronises)
  std::vector<uint64_t> h_digits;
  std::vector<int> h_status;
  // workspaces
  DevBuf work, status, fbtab, ipart;
  bool fbtab_ready = false;  // fixed-base comb table of g1 (built on first use)
  // staging for host-pointer entry points
  DevBuf in_p1, in_q1, in_i1, in_p2, in_q2, in_i2, out_v, in_a, in_b, in_c, in_d, out_x;
  // split master check (hbh_combine_verify_g2): a second stream runs the partial Miller loops while
  // the engine stream interpolates; partial Miller values in fval.  Created on the first split call:
  // HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues round-robin, and an idle extra stream
  // made at engine creation put the caller's two alternating verify streams on one queue
  // (sign bench: 23.3 instead of 21.1 ms per 65,536-check step)
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  DevBuf fval, split_in, split_out, tree_cnt;
  uint8_t* h_stage = nullptr;  // pinned host staging of the split check (one upload, one download)
  size_t h_stage_cap = 0;
  bool split_check = true;  // HBH_SPLIT_CHECK=0 in the environment: interpolate, then verify (A/B)
  bool split_tree = true;   // HBH_SPLIT_TREE=0: a separate product + FE launch (wave_prod_fe) (A/B)
  // Ack checks of dense y runs by finite differences (hbl::bivar_fd); HBH_ACK_FD=0: Horner only (A/B)
  bool ack_fd = true;
  DevBuf fd_e, fd_meta, fb16;
  bool fb16_ready = false;  // 16-bit comb of g1 (the FD ack check), built on first use
  size_t split_max = 0;  // HBH_SPLIT_MAX: most combines per call on the split check (0: the wave rule)
  // commitment sets created on this engine: hbh_engine_destroy frees their device memory and
  // detaches them, so a set destroyed after its engine never touches the freed engine
  std::unordered_set<hbh_commit_set*> sets;
};
void release_set_device(hbh_commit_set* cs);

namespace {

// Start of a call on stream s: order it after the engine's previous call.
int begin_call(hbh_engine* e, hipStream_t s) {
  HBH_CHECK(hipStreamWaitEvent(s, e->done, 0));
  HBH_CHECK(hipStreamWaitEvent(s, e->slot_done[0], 0));
  HBH_CHECK(hipStreamWaitEvent(s, e->slot_done[1], 0));
  return HBH_OK;
}
int end_call(hbh_engine* e, hipStream_t s) {
  HBH_CHECK(hipEventRecord(e->done, s));
  HBH_CHECK(hipEventRecord(e->slot_done[0], s));
  HBH_CHECK(hipEventRecord(e->slot_done[1], s));
  return HBH_OK;
}

int resolve_impl(const hbh_engine* e, size_t n) {
  if (e->impl != HBH_IMPL_AUTO) return e->impl;
  if (n <= HBH_AUTO_WAVE2_MAX) return HBH_IMPL_WAVE2;
  if (n <= HBH_AUTO_WAVE_MAX) return HBH_IMPL_WAVE;
  if (n <= HBH_AUTO_OCT_MAX) return HBH_IMPL_OCT;
  return n <= HBH_AUTO_QUAD_MAX ? HBH_IMPL_QUAD : HBH_IMPL_PAIR;
}

// the checks [off, n) of a side: per-check P and index map (or per-check Q when there is no map)
// advance by off; tables and shared Q tables stay
hbl::PairSideDesc offset_side(const hbl::PairSideDesc& d, size_t off) {
  hbl::PairSideDesc o = d;
  if (o.p) o.p = (const uint8_t*)o.p + off * HBH_G1_BYTES;
  if (o.idx) {
    o.idx += off;
  } else {  // identity map: Q is per check (nq == n, check_idx)
    o.q = (const uint8_t*)o.q + off * HBH_G2_BYTES;
    o.nq -= off;
  }
  return o;
}

#define HBH_WAVE_TT_MIN 1024  // WAVE calls that table two shared G2 sides (launch_pair)

// HBH_IMPL_WAVE2 (two waves per check) takes plain checks only; the split master check's modes
// (Miller-only, Jacobian P, one side) run on WAVE
hipError_t wave2_verify(hipStream_t s, int n, const hbl::PairSideDesc& a, const hbl::PairSideDesc& b, int flags,
                        uint8_t* v, uint32_t* val) {
  if (flags & ~(hbl::WAVE_NEG_P2 | hbl::WAVE_CONJ_VALUE)) return hbl::wave_verify(s, n, a, b, flags, v, val);
  return hbl::wave64_verify(s, n, a, b, flags, v, val);
}

// HBH_IMPL_AUTO's launches for n checks on one stream (profiles/r04/c8, c19, c20 sweeps): whole
// rounds of HBH_AUTO_PAIR_ROUND checks (two lane-pair waves per SIMD) on PAIR, then the remainder by
// size -- above HBH_AUTO_SPLIT_HI one more (partial) PAIR round; above HBH_AUTO_SPLIT_LO PAIR on
// HBH_AUTO_SPLIT_LO checks (one wave per SIMD) first; what is left runs on WAVE up to
// HBH_AUTO_WAVE_MAX, OCT up to HBH_AUTO_OCT_MAX, QUAD up to HBH_AUTO_QUAD_MAX, PAIR (one wave per
// SIMD) above.  A partial
// lane-pair round costs as much as a full one once any SIMD needs a second wave (40,960 checks:
// PAIR alone 20.5-20.7 ms, PAIR + QUAD 19.4 ms, profiles/r04/c20_auto_split.txt).
hipError_t verify_auto(hipStream_t s, size_t n, const hbl::PairSideDesc& s1, const hbl::PairSideDesc& s2, int flags,
                       uint8_t* d_v, uint32_t* d_value) {
  size_t off = 0;
  auto at = [&](size_t o, size_t cnt, int kind) -> hipError_t {
    const hbl::PairSideDesc a = o ? offset_side(s1, o) : s1, b = o ? offset_side(s2, o) : s2;
    uint8_t* v = d_v ? d_v + o : nullptr;
    uint32_t* val = d_value ? d_value + o * 144 : nullptr;
    if (kind == HBH_IMPL_WAVE2) return wave2_verify(s, (int)cnt, a, b, flags, v, val);
    if (kind == HBH_IMPL_WAVE) return hbl::wave_verify(s, (int)cnt, a, b, flags, v, val);
    if (kind == HBH_IMPL_QUAD) return hbl::quad_verify(s, (int)cnt, a, b, flags, v, val);
    if (kind == HBH_IMPL_OCT) return hbl::oct_verify(s, (int)cnt, a, b, flags, v, val);
    return hbl::pair_verify(s, (int)cnt, a, b, flags, v, val);
  };
  if (n > HBH_AUTO_SPLIT_HI) {  // whole two-wave lane-pair rounds
    off = (n / HBH_AUTO_PAIR_ROUND) * HBH_AUTO_PAIR_ROUND;
    if (off) {
      const hipError_t r = at(0, off, HBH_IMPL_PAIR);
      if (r != hipSuccess) return r;
    }
  }
  size_t rem = n - off;
  if (rem == 0) return hipSuccess;
  if (rem > HBH_AUTO_SPLIT_HI) return at(off, rem, HBH_IMPL_PAIR);  // one partial two-wave round
  if (rem > HBH_AUTO_SPLIT_LO) {  // one lane-pair wave per SIMD, then the rest by size
    const hipError_t r = at(off, HBH_AUTO_SPLIT_LO, HBH_IMPL_PAIR);
    if (r != hipSuccess) return r;
    off += HBH_AUTO_SPLIT_LO;
    rem -= HBH_AUTO_SPLIT_LO;
  }
  if (rem <= HBH_AUTO_WAVE2_MAX) return at(off, rem, HBH_IMPL_WAVE2);
  if (rem <= HBH_AUTO_WAVE_MAX) return at(off, rem, HBH_IMPL_WAVE);
  if (rem <= HBH_AUTO_OCT_MAX) return at(off, rem, HBH_IMPL_OCT);
  if (rem <= HBH_AUTO_QUAD_MAX) return at(off, rem, HBH_IMPL_QUAD);
  return at(off, rem, HBH_IMPL_PAIR);
}

// HBH_IMPL_PAIR: a G2 side shared through an index map by at least 4 checks per point gets a line
// table (k_oct_prep); every other side is walked inside the verify kernel.
int launch_pair(hbh_engine* e, hipStream_t s, int impl, size_t n, const void* d_p1, const void* d_q1, size_t nq1,
                const uint32_t* d_i1, const void* d_p2, const void* d_q2, size_t nq2, const uint32_t* d_i2, int flags,
                uint8_t* d_v, uint32_t* d_value, int slot) {
  hbl::PairSideDesc sd[2] = {{d_p1, d_q1, nullptr, nullptr, d_i1, nq1}, {d_p2, d_q2, nullptr, nullptr, d_i2, nq2}};
  DevBuf* tab[2] = {&e->ptab[slot][0], &e->ptab[slot][1]};
  DevBuf* inf[2] = {&e->pinf[slot][0], &e->pinf[slot][1]};
  const bool tab_ok[2] = {sd[0].idx && sd[0].nq * 4 <= n, sd[1].idx && sd[1].nq * 4 <= n};
  for (int k = 0; k < 2; k++) {
    // WAVE2 walks every side: a table costs a serial 68-step walk (k_oct_prep, ~0.5 ms) before the
    // first check.  WAVE tables both sides of a call of >= HBH_WAVE_TT_MIN checks when both are
    // shared (decryption shares: H_uv and W per ciphertext): its TT program takes 138 Miller stages
    // where walking both sides takes 211 (round 6); one walked side gains nothing (TW: 210).
    if (!tab_ok[k] || impl == HBH_IMPL_WAVE2) continue;
    if (impl == HBH_IMPL_WAVE && !(tab_ok[0] && tab_ok[1] && n >= HBH_WAVE_TT_MIN)) continue;
    HBH_CHECK(tab[k]->ensure(hbl::pair_table_bytes(sd[k].nq)));
    HBH_CHECK(inf[k]->ensure(sd[k].nq));
    hipEvent_t t = e->timer.begin(s, HBH_STAGE_PREPARE, e->profiling);
    HBH_CHECK(hbl::oct_prep(s, (int)sd[k].nq, sd[k].q, tab[k]->p, (uint8_t*)inf[k]->p));
    e->timer.end(s, t);
    sd[k].lines = tab[k]->p;
    sd[k].qinf = (const uint8_t*)inf[k]->p;
  }
  hipEvent_t t = e->timer.begin(s, HBH_STAGE_PAIRING, e->profiling);
  if (e->impl == HBH_IMPL_AUTO)
    HBH_CHECK(verify_auto(s, n, sd[0], sd[1], flags, d_v, d_value));
  else if (impl == HBH_IMPL_WAVE)
    HBH_CHECK(hbl::wave_verify(s, (int)n, sd[0], sd[1], flags, d_v, d_value));
  else if (impl == HBH_IMPL_WAVE2)
    HBH_CHECK(wave2_verify(s, (int)n, sd[0], sd[1], flags, d_v, d_value));
  else if (impl == HBH_IMPL_QUAD)
    HBH_CHECK(hbl::quad_verify(s, (int)n, sd[0], sd[1], flags, d_v, d_value));
  else if (impl == HBH_IMPL_OCT)
    HBH_CHECK(hbl::oct_verify(s, (int)n, sd[0], sd[1], flags, d_v, d_value));
  else
    HBH_CHECK(hbl::pair_verify(s, (int)n, sd[0], sd[1], flags, d_v, d_value));
  e->timer.end(s, t);
  return HBH_OK;
}

// e(P1_i, Q1[i1_i]) == e(P2_i, Q2[i2_i]) for device-resident inputs; d_p1 / d_p2 == nullptr means
// the G1 generator for every check.  flags as hbl::pair_verify.
int run_pairing_dev(hbh_engine* e, hipStream_t s, size_t n, const void* d_p1, const void* d_q1, size_t nq1,
                    const uint32_t* d_i1, const void* d_p2, const void* d_q2, size_t nq2, const uint32_t* d_i2,
                    int flags, uint8_t* d_v, uint32_t* d_value = nullptr, int slot = 0) {
  if (n == 0) return HBH_OK;
  if (n > (size_t)1 << 30 || nq1 > (size_t)1 << 30 || nq2 > (size_t)1 << 30) return fail(HBH_ERR_ARG, "batch too large");
  return launch_pair(e, s, resolve_impl(e, n), n, d_p1, d_q1, nq1, d_i1, d_p2, d_q2, nq2, d_i2, flags, d_v, d_value,
                     slot);
}

int check_idx(const uint32_t* idx, size_t n, size_t table) {
  if (!idx) return table == n ? HBH_OK : fail(HBH_ERR_ARG, "identity index map requires table size == n");
  for (size_t i = 0; i < n; i++)
    if (idx[i] >= table) return fail(HBH_ERR_ARG, "index out of range");
  return HBH_OK;
}

// Host-pointer pairing-eq: stage to device, run, copy verdicts back, synchronise.  p1 / p2 ==
// nullptr: the G1 generator (nothing is uploaded for it).
int run_pairing_eq_host(hbh_engine* e, size_t n, const uint8_t* p1, const uint8_t* q1, size_t nq1, const uint32_t* i1,
                        const uint8_t* p2, const uint8_t* q2, size_t nq2, const uint32_t* i2, uint8_t* v) {
  if (n == 0) return HBH_OK;
  if (!q1 || !q2 || !v) return fail(HBH_ERR_ARG, "null pointer");
  int rc = check_idx(i1, n, nq1);
  if (rc) return rc;
  rc = check_idx(i2, n, nq2);
  if (rc) return rc;
  hipStream_t s = e->stream;
  rc = begin_call(e, s);
  if (rc) return rc;
  if (p1) HBH_CHECK(e->in_p1.ensure(n * HBH_G1_BYTES));
  if (p2) HBH_CHECK(e->in_p2.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(e->in_q1.ensure(nq1 * HBH_G2_BYTES));
  HBH_CHECK(e->in_q2.ensure(nq2 * HBH_G2_BYTES));
  HBH_CHECK(e->out_v.ensure(n));
  if (p1) HBH_CHECK(hipMemcpyAsync(e->in_p1.p, p1, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  if (p2) HBH_CHECK(hipMemcpyAsync(e->in_p2.p, p2, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
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
  rc = run_pairing_dev(e, s, n, p1 ? e->in_p1.p : nullptr, e->in_q1.p, nq1, d_i1, p2 ? e->in_p2.p : nullptr,
                       e->in_q2.p, nq2, d_i2, 1, (uint8_t*)e->out_v.p);
  if (rc) return rc;
  HBH_CHECK(hipMemcpyAsync(v, e->out_v.p, n, hipMemcpyDeviceToHost, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // namespace

extern "C" {

const char* hbh_last_error(void) { return g_last_error.c_str(); }

// Not part of the public ABI: lets pool.cpp report a shard's failure on the calling thread.
extern "C" void hbh__set_error(const char* msg) { g_last_error = msg ? msg : ""; }

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
  if (const char* v = std::getenv("HBH_SPLIT_CHECK")) e->split_check = std::atoi(v) != 0;
  if (const char* v = std::getenv("HBH_SPLIT_TREE")) e->split_tree = std::atoi(v) != 0;
  if (const char* v = std::getenv("HBH_ACK_FD")) e->ack_fd = std::atoi(v) != 0;
  if (const char* v = std::getenv("HBH_SPLIT_MAX")) e->split_max = (size_t)std::max(0, std::atoi(v));
  hipError_t err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (err == hipSuccess) err = hipEventCreateWithFlags(&e->done, hipEventDisableTiming);
  if (err == hipSuccess) err = hipEventRecord(e->done, e->stream);
  for (int k = 0; k < 2 && err == hipSuccess; k++) {
    err = hipEventCreateWithFlags(&e->slot_done[k], hipEventDisableTiming);
    if (err == hipSuccess) err = hipEventRecord(e->slot_done[k], e->stream);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&e->wire_done[k], hipEventDisableTiming);
    if (err == hipSuccess) err = hipEventRecord(e->wire_done[k], e->stream);
  }
  if (err != hipSuccess) {
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return fail(HBH_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(err));
  }
  *out = e;
  return HBH_OK;
}

int hbh_engine_destroy(hbh_engine* e) {
  if (!e) return HBH_OK;
  (void)hipSetDevice(e->device);
  {
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipEventSynchronize(e->done);
    (void)hipStreamSynchronize(e->stream);
    for (hbh_commit_set* cs : e->sets) release_set_device(cs);  // detaches cs from e
    e->sets.clear();
  }
  (void)hipEventSynchronize(e->done);
  for (hipEvent_t ev : e->slot_done)
    if (ev) (void)hipEventSynchronize(ev);
  for (hipEvent_t ev : e->wire_done)
    if (ev) (void)hipEventSynchronize(ev);
  (void)hipStreamSynchronize(e->stream);
  if (e->side) (void)hipStreamSynchronize(e->side);
  e->timer.clear();
  for (DevBuf* b : {&e->work, &e->status, &e->fbtab, &e->ipart, &e->in_p1, &e->in_q1, &e->in_i1, &e->in_p2, &e->in_q2, &e->in_i2, &e->out_v,
                    &e->in_a, &e->in_b, &e->in_c, &e->in_d, &e->out_x, &e->ptab[0][0], &e->ptab[0][1], &e->ptab[1][0],
                    &e->ptab[1][1], &e->pinf[0][0], &e->pinf[0][1], &e->pinf[1][0], &e->pinf[1][1], &e->fval, &e->split_in,
                    &e->split_out, &e->tree_cnt, &e->fd_e, &e->fd_meta, &e->fb16, &e->wire_w[0], &e->wire_w[1],
                    &e->wire_f[0], &e->wire_f[1]})
    b->release();
  if (e->h_stage) (void)hipHostFree(e->h_stage);
  (void)hipEventDestroy(e->done);
  if (e->side) {
    (void)hipEventDestroy(e->fork);
    (void)hipEventDestroy(e->join);
    (void)hipStreamDestroy(e->side);
  }
  for (hipEvent_t ev : e->slot_done)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->wire_done)
    if (ev) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(e->stream);
  delete e;
  return HBH_OK;
}

int hbh_verify_pairing_eq(hbh_engine* e, size_t n, const uint8_t* p1, const uint8_t* q1, size_t nq1,
                          const uint32_t* i1, const uint8_t* p2, const uint8_t* q2, size_t nq2, const uint32_t* i2,
                          uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n && (!p1 || !p2)) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, p1, q1, nq1, i1, p2, q2, nq2, i2, v);
}

int hbh_verify_pairing_eq_dev(hbh_engine* e, void* stream, size_t n, const void* d_p1, const void* d_q1, size_t nq1,
                              const uint32_t* d_i1, const void* d_p2, const void* d_q2, size_t nq2,
                              const uint32_t* d_i2, uint8_t* d_v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n && (!d_q1 || !d_q2 || !d_v)) return fail(HBH_ERR_ARG, "null pointer");
  if ((!d_i1 && nq1 != n) || (!d_i2 && nq2 != n)) return fail(HBH_ERR_ARG, "identity index map requires table size == n");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  if (n == 0) return HBH_OK;
  // table slot of its own: wait for the last general call and for this slot's previous user only
  const int slot = e->slot;
  e->slot ^= 1;
  HBH_CHECK(hipStreamWaitEvent(s, e->done, 0));
  HBH_CHECK(hipStreamWaitEvent(s, e->slot_done[slot], 0));
  int rc = run_pairing_dev(e, s, n, d_p1, d_q1, nq1, d_i1, d_p2, d_q2, nq2, d_i2, 1, d_v, nullptr, slot);
  if (rc) return rc;
  HBH_CHECK(hipEventRecord(e->slot_done[slot], s));
  return HBH_OK;
}

int hbh_verify_sig_shares(hbh_engine* e, size_t n, const uint8_t* pks, const uint8_t* sigs, const uint8_t* hashes,
                          size_t ndocs, const uint32_t* doc_idx, uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!pks || !sigs) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, pks, hashes, ndocs, doc_idx, nullptr, sigs, n, nullptr, v);
}

int hbh_verify_dec_shares(hbh_engine* e, size_t n, const uint8_t* shares, const uint8_t* pks, const uint8_t* huv,
                          const uint8_t* w, size_t ncts, const uint32_t* ct_idx, uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n && (!shares || !pks)) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, shares, huv, ncts, ct_idx, pks, w, ncts, ct_idx, v);
}

int hbh_verify_ciphertexts(hbh_engine* e, size_t n, const uint8_t* u, const uint8_t* w, const uint8_t* huv,
                           uint8_t* v) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!u) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  return run_pairing_eq_host(e, n, nullptr, w, n, nullptr, u, huv, n, nullptr, v);
}

int hbh_dbg_pairing(hbh_engine* e, size_t n, const uint8_t* p, const uint8_t* q, uint8_t* out) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!p || !q || !out) return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  int rc = begin_call(e, s);
  if (rc) return rc;
  HBH_CHECK(e->in_p1.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(e->in_q1.ensure(n * HBH_G2_BYTES));
  HBH_CHECK(e->out_v.ensure(n * 576));
  HBH_CHECK(hipMemcpyAsync(e->in_p1.p, p, n * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_q1.p, q, n * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(e->in_p2.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(hipMemsetAsync(e->in_p2.p, 0, n * HBH_G1_BYTES, s));  // second pair inactive (P2 = O)
  rc = run_pairing_dev(e, s, n, e->in_p1.p, e->in_q1.p, n, nullptr, e->in_p2.p, e->in_q1.p, n, nullptr, 2, nullptr,
                       (uint32_t*)e->out_v.p);
  if (rc) return rc;
  HBH_CHECK(hipMemcpyAsync(out, e->out_v.p, n * 576, hipMemcpyDeviceToHost, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

int hbh_engine_set_pairing_impl(hbh_engine* e, int impl) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (impl != HBH_IMPL_PAIR && impl != HBH_IMPL_AUTO && impl != HBH_IMPL_WAVE && impl != HBH_IMPL_QUAD &&
      impl != HBH_IMPL_OCT && impl != HBH_IMPL_WAVE2)
    return fail(HBH_ERR_ARG, "unknown or retired pairing implementation");
  std::lock_guard<std::mutex> lk(e->mu);
  e->impl = impl;
  return HBH_OK;
}

int hbh_engine_set_ack_impl(hbh_engine* e, int impl) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (impl != HBH_ACK_AUTO && impl != HBH_ACK_QUAD && impl != HBH_ACK_LANE && impl != HBH_ACK_LANE_HORNER)
    return fail(HBH_ERR_ARG, "unknown Ack-check implementation");
  std::lock_guard<std::mutex> lk(e->mu);
  e->ack_impl = impl;
  return HBH_OK;
}

int hbh_engine_set_profiling(hbh_engine* e, int on) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  HBH_CHECK(hipStreamSynchronize(e->stream));
  e->timer.clear();
  e->profiling = on != 0;
  return HBH_OK;
}

int hbh_engine_stage_time(hbh_engine* e, int stage, double* total_ms, int* launches) {
  if (!e || !total_ms || !launches || stage < 0 || stage >= HBH_NUM_STAGES) return fail(HBH_ERR_ARG, "bad argument");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  double sum = 0;
  for (auto& p : e->timer.ev[stage]) {
    HBH_CHECK(hipEventSynchronize(p.second));
    float ms = 0;
    HBH_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
    sum += ms;
  }
  *total_ms = sum;
  *launches = (int)e->timer.ev[stage].size();
  return HBH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- curve entry points
namespace {
int check_t(int t) { return (t < 0 || t > 4096) ? fail(HBH_ERR_ARG, "threshold out of range") : HBH_OK; }

template <class Launch>
int run_mul(hbh_engine* e, size_t n, const uint8_t* pts, size_t pt_bytes, const uint8_t* scalars, uint8_t* out,
            Launch launch) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!pts || !scalars || !out) return fail(HBH_ERR_ARG, "null pointer");
  if (n > (size_t)1 << 28) return fail(HBH_ERR_ARG, "batch too large");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->in_a.ensure(n * pt_bytes));
  HBH_CHECK(e->in_b.ensure(n * HBH_FR_BYTES));
  HBH_CHECK(e->out_x.ensure(n * pt_bytes));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, pts, n * pt_bytes, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, scalars, n * HBH_FR_BYTES, hipMemcpyHostToDevice, s));
  hipEvent_t t = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(launch(s, (int)n, e->in_a.p, (const uint32_t*)e->in_b.p, e->out_x.p));
  e->timer.end(s, t);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, n * pt_bytes, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

// The g1 comb table, built on the engine stream the first time a call needs it.
int ensure_fbtab(hbh_engine* e, hipStream_t s) {
  if (e->fbtab_ready) return HBH_OK;
  HBH_CHECK(e->fbtab.ensure(hbl::fb_table_bytes()));
  HBH_CHECK(hbl::fb_table(s, e->fbtab.p));
  e->fbtab_ready = true;
  return HBH_OK;
}

int ensure_fb16(hbh_engine* e, hipStream_t s) {
  if (e->fb16_ready) return HBH_OK;
  HBH_CHECK(e->fb16.ensure(hbl::fb16_table_bytes()));
  DevBuf scratch;  // freed before return, also on failure
  hipError_t err = scratch.ensure(hbl::fb16_scratch_bytes());
  if (err == hipSuccess) err = hbl::fb16_table(s, e->fb16.p, scratch.p);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  scratch.release();
  HBH_CHECK(err);
  e->fb16_ready = true;
  return HBH_OK;
}

// ---- host Fr (4 x 64-bit Montgomery, R = 2^256) for the Lagrange digits of one or two combines:
// on the host they cost tens of microseconds, less than a kernel launch of k_interp_digits.
struct HFr {
  uint64_t l[4];
};
constexpr uint64_t HFR_P[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                               0x73eda753299d7d48ull};
constexpr uint64_t HFR_NP = 0xfffffffeffffffffull;  // -r^-1 mod 2^64
constexpr uint64_t HFR_R2[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                                0x0748d9d99f59ff11ull};
using u128 = unsigned __int128;

bool hfr_geq_p(const uint64_t* a) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != HFR_P[i]) return a[i] > HFR_P[i];
  return true;
}
void hfr_sub_p(uint64_t* a) {
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a[i] - HFR_P[i] - br;
    a[i] = (uint64_t)d;
    br = (d >> 64) ? 1 : 0;
  }
}
HFr hfr_mul(const HFr& a, const HFr& b) {  // CIOS
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.l[j] * b.l[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    const uint64_t m = t[0] * HFR_NP;
    c = (u128)m * HFR_P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * HFR_P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  HFr r{{t[0], t[1], t[2], t[3]}};
  if (t[4] || hfr_geq_p(r.l)) hfr_sub_p(r.l);
  return r;
}
HFr hfr_from_u64(uint64_t v) { return hfr_mul(HFr{{v, 0, 0, 0}}, HFr{{HFR_R2[0], HFR_R2[1], HFR_R2[2], HFR_R2[3]}}); }
HFr hfr_sub(const HFr& a, const HFr& b) {
  HFr r;
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (uint64_t)d;
    br = (d >> 64) ? 1 : 0;
  }
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)r.l[i] + HFR_P[i];
      r.l[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}
bool hfr_is_zero(const HFr& a) { return !(a.l[0] | a.l[1] | a.l[2] | a.l[3]); }
HFr hfr_inv(const HFr& a) {  // a^(r-2)
  uint64_t e[4] = {HFR_P[0] - 2, HFR_P[1], HFR_P[2], HFR_P[3]};
  HFr r = hfr_from_u64(1);
  for (int i = 255; i >= 0; i--) {
    r = hfr_mul(r, r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = hfr_mul(r, a);
  }
  return r;
}
void hfr_to_canon(const HFr& a, uint64_t* out) {
  const HFr c = hfr_mul(a, HFr{{1, 0, 0, 0}});
  for (int i = 0; i < 4; i++) out[i] = c.l[i];
}

// k_interp_digits on the host: the four GLS digits (base |x|) of every lambda_k(0) of each combine;
// status[c] = HBH_ERR_DUPLICATE_ENTRY and zero digits on a repeated x
// q (4 x u64) <- q / x^2, rem <- q mod x^2 (bit-serial, the host twin of k_curve.hip div_x2)
void host_div_x2(uint64_t q[4], uint64_t rem[2]) {
  constexpr uint64_t X2_LO = 0x0000000100000000ull, X2_HI = 0xac45a4010001a402ull;
  uint64_t r0 = 0, r1 = 0;
  for (int w = 3; w >= 0; w--) {
    uint64_t qw = 0;
    for (int b = 63; b >= 0; b--) {
      const bool top = (r1 >> 63) != 0;
      r1 = (r1 << 1) | (r0 >> 63);
      r0 = (r0 << 1) | ((q[w] >> b) & 1);
      const bool ge = top || r1 > X2_HI || (r1 == X2_HI && r0 >= X2_LO);
      if (ge) {
        const uint64_t nr0 = r0 - X2_LO;
        r1 = r1 - X2_HI - (r0 < X2_LO ? 1 : 0);
        r0 = nr0;
      }
      qw |= (uint64_t)ge << b;
    }
    q[w] = qw;
  }
  rem[0] = r0;
  rem[1] = r1;
}

// lambda_k(0) = prod_{j != k} x_j / (x_j - x_k) of every sample of each combine, canonical (4 x u64
// LE per sample); status[c] = HBH_ERR_DUPLICATE_ENTRY and zero lambdas on a repeated x
void host_lagrange(const uint32_t* xs, size_t ncomb, size_t m, uint64_t* lam, int* status) {
  std::vector<HFr> x(m), num(m), den(m), pre(m);
  for (size_t c = 0; c < ncomb; c++) {
    const uint32_t* cx = xs + c * m;
    for (size_t k = 0; k < m; k++) x[k] = hfr_from_u64(cx[k]);
    bool dup = false;
    for (size_t k = 0; k < m; k++) {
      HFr n = hfr_from_u64(1), d = hfr_from_u64(1);
      for (size_t j = 0; j < m; j++) {
        if (j == k) continue;
        n = hfr_mul(n, x[j]);
        d = hfr_mul(d, hfr_sub(x[j], x[k]));
      }
      dup = dup || hfr_is_zero(d);
      num[k] = n;
      den[k] = d;
    }
    status[c] = dup ? HBH_ERR_DUPLICATE_ENTRY : HBH_OK;
    uint64_t* lc = lam + c * m * 4;
    if (dup) {
      std::memset(lc, 0, m * 4 * sizeof(uint64_t));
      continue;
    }
    pre[0] = den[0];
    for (size_t k = 1; k < m; k++) pre[k] = hfr_mul(pre[k - 1], den[k]);
    HFr inv = hfr_inv(pre[m - 1]);
    for (size_t k = m; k-- > 0;) {
      const HFr ik = k ? hfr_mul(inv, pre[k - 1]) : inv;
      if (k) inv = hfr_mul(inv, den[k]);
      hfr_to_canon(hfr_mul(num[k], ik), lc + k * 4);
    }
  }
}

// the four GLS digits (base |x|) of n canonical scalars (4 x u64 each): q <- q / |x| three times, digit j
// = remainder, digit 3 = the last quotient
void host_gls_digits(const uint64_t* lam, size_t n, uint64_t* dg) {
  constexpr uint64_t XA = 0xd201000000010000ull;
  for (size_t k = 0; k < n; k++) {
    uint64_t q[4] = {lam[k * 4], lam[k * 4 + 1], lam[k * 4 + 2], lam[k * 4 + 3]};
    for (int j = 0; j < 3; j++) {
      u128 rem = 0;
      for (int w = 3; w >= 0; w--) {
        const u128 cur = (rem << 64) | q[w];
        q[w] = (uint64_t)(cur / XA);
        rem = cur % XA;
      }
      dg[k * 4 + j] = (uint64_t)rem;
    }
    dg[k * 4 + 3] = q[0];
  }
}

void host_interp_digits(const uint32_t* xs, size_t ncomb, size_t m, uint64_t* digits, int* status, bool g1 = false) {
  constexpr uint64_t XA = 0xd201000000010000ull;
  host_lagrange(xs, ncomb, m, digits, status);  // in place: lambda_k's 4 words become its 4 digits
  for (size_t c = 0; c < ncomb; c++) {
    uint64_t* dg = digits + c * m * 4;
    if (status[c] != HBH_OK) continue;
    for (size_t k = 0; k < m; k++) {
      uint64_t q[4] = {dg[k * 4], dg[k * 4 + 1], dg[k * 4 + 2], dg[k * 4 + 3]};
      if (g1) {  // lambda = d0 + d1 x^2
        uint64_t rem[2];
        host_div_x2(q, rem);
        dg[k * 4 + 0] = rem[0];
        dg[k * 4 + 1] = rem[1];
        dg[k * 4 + 2] = q[0];
        dg[k * 4 + 3] = q[1];
        continue;
      }
      for (int j = 0; j < 3; j++) {  // q <- q / |x|, digit j = remainder
        u128 rem = 0;
        for (int w = 3; w >= 0; w--) {
          const u128 cur = (rem << 64) | q[w];
          q[w] = (uint64_t)(cur / XA);
          rem = cur % XA;
        }
        dg[k * 4 + j] = (uint64_t)rem;
      }
      dg[k * 4 + 3] = q[0];
    }
  }
}

// G2 combines: few combines (latency-bound: the chip is idle but for the serial chains) take the
// lane-pair form (digits + k_interp_pair); many take k_interp_endo (throughput form).  With the x
// values on the host and at most HOST_DIGITS_MAX combines, the digits are computed on the host and
// uploaded (status too) instead of running k_interp_digits.
#ifndef HBH_INTERP_PAIR_MAX
#define HBH_INTERP_PAIR_MAX 384  // measured crossover with k_interp_endo<Fp2>: 100 combines 5.25 -> 2.46 ms, 1,024: 11.9 vs 15.8 ms
#endif
constexpr size_t INTERP_PAIR_MAX = HBH_INTERP_PAIR_MAX;
constexpr size_t HOST_DIGITS_MAX = 2;
int launch_combine_g2(hbh_engine* e, hipStream_t s, size_t ncomb, size_t m, const uint32_t* d_xs, const void* d_pts,
                      void* d_out, int* d_status, const uint32_t* h_xs = nullptr) {
  if (ncomb <= INTERP_PAIR_MAX && hbl::interp_g2_pair_fits((int)m)) {
    HBH_CHECK(e->in_d.ensure(ncomb * m * 4 * sizeof(uint64_t)));
    if (h_xs && ncomb <= HOST_DIGITS_MAX) {
      e->h_digits.resize(ncomb * m * 4);
      e->h_status.resize(ncomb);
      host_interp_digits(h_xs, ncomb, m, e->h_digits.data(), e->h_status.data());
      HBH_CHECK(hipMemcpyAsync(e->in_d.p, e->h_digits.data(), ncomb * m * 32, hipMemcpyHostToDevice, s));
      HBH_CHECK(hipMemcpyAsync(d_status, e->h_status.data(), ncomb * sizeof(int), hipMemcpyHostToDevice, s));
    } else {
      HBH_CHECK(hbl::interp_digits(s, (int)ncomb, (int)m, d_xs, (uint64_t*)e->in_d.p, d_status));
    }
    HBH_CHECK(e->ipart.ensure(hbl::interp_g2_pair_part_bytes((int)ncomb)));
    HBH_CHECK(hbl::interp_g2_pair(s, (int)ncomb, (int)m, (const uint64_t*)e->in_d.p, d_pts, e->ipart.p, d_out));
    return HBH_OK;
  }
  HBH_CHECK(hbl::combine_g2(s, (int)ncomb, (int)m, d_xs, d_pts, d_out, d_status));
  return HBH_OK;
}

// G1 combines: few combines take the lane-quad latency form (digits + k_interp_g1q + join), many
// k_interp_endo<Fp> (throughput form).
#ifndef HBH_INTERP_G1Q_MAX
#define HBH_INTERP_G1Q_MAX 256  // quad form: 1 combine 0.91 ms, 100 1.74 ms (k_interp_endo<Fp>: 3.2 ms), 256 3.0 ms; 1,024 endo 4.1 ms
#endif
int launch_combine_g1(hbh_engine* e, hipStream_t s, size_t ncomb, size_t m, const uint32_t* d_xs, const void* d_pts,
                      void* d_out, int* d_status, const uint32_t* h_xs = nullptr) {
  if (ncomb <= HBH_INTERP_G1Q_MAX && m <= 4096) {
    HBH_CHECK(e->in_d.ensure(ncomb * m * 4 * sizeof(uint64_t)));
    if (h_xs && ncomb <= HOST_DIGITS_MAX) {
      e->h_digits.resize(ncomb * m * 4);
      e->h_status.resize(ncomb);
      host_interp_digits(h_xs, ncomb, m, e->h_digits.data(), e->h_status.data(), true);
      HBH_CHECK(hipMemcpyAsync(e->in_d.p, e->h_digits.data(), ncomb * m * 32, hipMemcpyHostToDevice, s));
      HBH_CHECK(hipMemcpyAsync(d_status, e->h_status.data(), ncomb * sizeof(int), hipMemcpyHostToDevice, s));
    } else {
      HBH_CHECK(hbl::interp_digits(s, (int)ncomb, (int)m, d_xs, (uint64_t*)e->in_d.p, d_status, true));
    }
    HBH_CHECK(e->ipart.ensure(hbl::interp_g1_quad_part_bytes((int)ncomb)));
    HBH_CHECK(hbl::interp_g1_quad(s, (int)ncomb, (int)m, (const uint64_t*)e->in_d.p, d_pts, e->ipart.p, d_out));
    return HBH_OK;
  }
  HBH_CHECK(hbl::combine_g1(s, (int)ncomb, (int)m, d_xs, d_pts, d_out, d_status));
  return HBH_OK;
}

int run_interp(hbh_engine* e, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out, int* status,
               bool g2) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (ncomb == 0) return HBH_OK;
  if (!idx || !pts || !out || !status) return fail(HBH_ERR_ARG, "null pointer");
  const size_t m = (size_t)t + 1, pb = g2 ? HBH_G2_BYTES : HBH_G1_BYTES;
  if (ncomb * m > (size_t)1 << 26) return fail(HBH_ERR_ARG, "batch too large");
  // x_k = idx_k + 1 as a small Fr integer (threshold_crypto into_fr_plus_1)
  std::vector<uint32_t> xs(ncomb * m);
  for (size_t k = 0; k < ncomb * m; k++) {
    if (idx[k] == 0xffffffffu) return fail(HBH_ERR_ARG, "node index out of range");
    xs[k] = idx[k] + 1;
  }
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->in_a.ensure(ncomb * m * 4));
  HBH_CHECK(e->in_b.ensure(ncomb * m * pb));
  HBH_CHECK(e->out_x.ensure(ncomb * pb));
  HBH_CHECK(e->status.ensure(ncomb * sizeof(int)));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, xs.data(), ncomb * m * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, pts, ncomb * m * pb, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemsetAsync(e->status.p, 0, ncomb * sizeof(int), s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  if (g2) {
    rc = launch_combine_g2(e, s, ncomb, m, (const uint32_t*)e->in_a.p, e->in_b.p, e->out_x.p, (int*)e->status.p,
                           xs.data());
    if (rc) return rc;
  } else {
    rc = launch_combine_g1(e, s, ncomb, m, (const uint32_t*)e->in_a.p, e->in_b.p, e->out_x.p, (int*)e->status.p,
                           xs.data());
    if (rc) return rc;
  }
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, ncomb * pb, hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipMemcpyAsync(status, e->status.p, ncomb * sizeof(int), hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

// ThresholdSign::combine_and_verify_sig's master check split off the interpolation (few combines, the
// latency case).  e(g1, sigma) == e(mpk, H) with sigma = sum_k lambda_k sigma_k is, by bilinearity,
//   prod_k e(lambda_k g1, sigma_k) * e(-mpk, H) == 1,
// which needs no sigma: its m + 1 Miller loops (two pairs per wave, k_wave's Miller-only mode) run on a
// second stream WHILE the engine stream interpolates sigma (one pair per wave, homogeneous walk: mode
// W1J of tools/gen_wave_prog.py); in the same launch the partial values are multiplied up a binary tree
// (the later of two sibling waves multiplies: log2(m + 1) products on the critical path instead of m)
// and the wave holding a combine's product runs the single final exponentiation (wave_miller_tree;
// HBH_SPLIT_TREE=0: a second launch multiplies the m + 1 values in order, wave_prod_fe).  The verdict is the same
// boolean for every input (an exact identity, no randomisation); lambda_k g1 comes from the device comb
// table summed in a 5-level tree on lane quads (k_g1_gen_quad) on the side stream, left in Jacobian
// form: the Miller kernel scales each line by Z^3 instead of inverting Z (WAVE_JAC_P).  A repeated index gives zero
// lambdas (status DuplicateEntry), as in the interpolation.
#ifndef HBH_SPLIT_PAIRS
#define HBH_SPLIT_PAIRS 1
#endif
}  // namespace
extern "C" int hbh__host_g1_neg(const uint8_t* pk, uint8_t* neg_out);
namespace {

int combine_verify_split(hbh_engine* e, size_t ncomb, size_t m, const std::vector<uint32_t>& xs,
                         const uint8_t* shares, const uint8_t* master_pk, const uint8_t* hashes, uint8_t* out,
                         int* status, uint8_t* verdicts) {
  // SPLIT_PAIRS pairs per wave: 1 = the homogeneous-walk program (two stages per Miller step),
  // 2 = the two-sided Jacobian program (WWJ, three stages per step, half the waves)
  constexpr int pairs = HBH_SPLIT_PAIRS;
  const size_t np = m + 1, nw = (np + pairs - 1) / pairs, nchk = ncomb * nw, nq = ncomb * np;
  constexpr size_t JB = 3 * 48;  // Jacobian P: X || Y || Z canonical
  uint8_t negpk[HBH_G1_BYTES];
  if (hbh__host_g1_neg(master_pk, negpk)) return fail(HBH_ERR_ARG, "master key coordinate >= p");  // checked by the caller too
  bool pk_inf = true;
  for (int b = 0; b < HBH_G1_BYTES; b++) pk_inf = pk_inf && negpk[b] == 0;
  // one upload: Q table (shares, then one H per combine) | GLS digits | lambdas | P sides | Q indices
  const size_t o_q = 0, o_dg = o_q + nq * HBH_G2_BYTES, o_lam = o_dg + ncomb * m * 32, o_p0 = o_lam + ncomb * m * 32,
               o_p1 = o_p0 + nchk * JB, o_i0 = o_p1 + nchk * JB, o_i1 = o_i0 + nchk * 4, in_bytes = o_i1 + nchk * 4;
  // one download: signatures | verdicts
  const size_t o_v = ncomb * HBH_G2_BYTES, out_bytes = o_v + ncomb;
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  if (!e->side) {
    HBH_CHECK(hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
    HBH_CHECK(hipEventCreateWithFlags(&e->fork, hipEventDisableTiming));
    HBH_CHECK(hipEventCreateWithFlags(&e->join, hipEventDisableTiming));
  }
  const size_t stage_bytes = std::max(in_bytes, out_bytes);
  if (stage_bytes > e->h_stage_cap) {
    if (e->h_stage) HBH_CHECK(hipHostFree(e->h_stage));
    e->h_stage = nullptr;
    e->h_stage_cap = 0;
    HBH_CHECK(hipHostMalloc((void**)&e->h_stage, stage_bytes + stage_bytes / 4 + 4096, hipHostMallocDefault));
    e->h_stage_cap = stage_bytes + stage_bytes / 4 + 4096;
  }
  uint8_t* hs = e->h_stage;
  std::memcpy(hs + o_q, shares, ncomb * m * HBH_G2_BYTES);
  std::memcpy(hs + o_q + ncomb * m * HBH_G2_BYTES, hashes, ncomb * HBH_G2_BYTES);
  std::vector<int> lst(ncomb);
  host_lagrange(xs.data(), ncomb, m, (uint64_t*)(hs + o_lam), lst.data());
  host_gls_digits((const uint64_t*)(hs + o_lam), ncomb * m, (uint64_t*)(hs + o_dg));
  std::memset(hs + o_p0, 0, 2 * nchk * JB);
  uint32_t* i0 = (uint32_t*)(hs + o_i0);
  uint32_t* i1 = (uint32_t*)(hs + o_i1);
  for (size_t c = 0; c < ncomb; c++)
    for (size_t w = 0; w < nw; w++)
      for (int sd = 0; sd < pairs; sd++) {
        const size_t k = pairs * w + sd, j = c * nw + w;
        uint32_t* qi = sd ? &i1[j] : &i0[j];
        if (k < m) {
          *qi = (uint32_t)(c * m + k);  // (lambda_k g1, sigma_k): P written by k_g1_gen_quad
        } else {
          if (k == m) {  // (-mpk, H_c) with Z = 1 (Z = 0: mpk at infinity, an inactive pair)
            uint8_t* d = hs + (sd ? o_p1 : o_p0) + j * JB;
            std::memcpy(d, negpk, HBH_G1_BYTES);
            d[96] = pk_inf ? 0 : 1;
          }
          *qi = (uint32_t)(ncomb * m + c);  // then an inactive pad (P = O)
        }
      }
  hipStream_t s = e->stream, s2 = e->side;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->split_in.ensure(in_bytes));
  HBH_CHECK(e->split_out.ensure(out_bytes));
  HBH_CHECK(e->fval.ensure(nchk * 144 * 4));
  HBH_CHECK(e->ipart.ensure(hbl::interp_g2_pair_part_bytes((int)ncomb)));
  uint8_t* din = (uint8_t*)e->split_in.p;
  uint8_t* dout = (uint8_t*)e->split_out.p;
  HBH_CHECK(hipMemcpyAsync(din, hs, in_bytes, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipEventRecord(e->fork, s));
  HBH_CHECK(hipStreamWaitEvent(s2, e->fork, 0));
  // From here on both streams hold queued work: every exit joins the side stream into s and closes the
  // call on s, so e->done covers the side stream's kernels even when a launch fails.
  auto launch = [&]() -> int {
    // side stream: lambda_k g1 (Jacobian, over the zero P entries), the m + 1 Miller loops, the product
    // and the final exponentiation
    int rc = ensure_fbtab(e, s2);
    if (rc) return rc;
    HBH_CHECK(hbl::g1_gen_tree(s2, (int)(ncomb * m), (int)m, (int)nw, pairs, e->fbtab.p,
                               (const uint32_t*)(din + o_lam), din + o_p0, din + o_p1));
    hbl::PairSideDesc sd0 = {din + o_p0, din + o_q, nullptr, nullptr, (const uint32_t*)(din + o_i0), nq};
    hbl::PairSideDesc sd1 = {din + o_p1, din + o_q, nullptr, nullptr, (const uint32_t*)(din + o_i1), nq};
    hipEvent_t tp = e->timer.begin(s2, HBH_STAGE_PAIRING, e->profiling);
    const int wflags = hbl::WAVE_MILLER_ONLY | hbl::WAVE_JAC_P | (pairs == 1 ? hbl::WAVE_ONE_SIDE : 0);
    if (e->split_tree) {  // product up a tree and the final exponentiation inside the Miller launch
      HBH_CHECK(e->tree_cnt.ensure(hbl::wave_tree_counter_bytes((int)ncomb, (int)nw)));
      HBH_CHECK(hbl::wave_miller_tree(s2, (int)ncomb, (int)nw, sd0, sd1, wflags, (uint32_t*)e->fval.p,
                                      (uint32_t*)e->tree_cnt.p, dout + o_v));
    } else {
      HBH_CHECK(hbl::wave_verify(s2, (int)nchk, sd0, sd1, wflags, nullptr, (uint32_t*)e->fval.p));
      HBH_CHECK(hbl::wave_prod_fe(s2, (int)ncomb, (int)nw, (const uint32_t*)e->fval.p, dout + o_v));
    }
    e->timer.end(s2, tp);
    // engine stream, concurrently: the interpolation (lane-quad latency form, host digits)
    hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
    HBH_CHECK(hbl::interp_g2_pair(s, (int)ncomb, (int)m, (const uint64_t*)(din + o_dg), din + o_q, e->ipart.p, dout));
    e->timer.end(s, tm);
    return HBH_OK;
  };
  const int lrc = launch();
  const hipError_t jerr = hipEventRecord(e->join, s2);
  const hipError_t werr = jerr == hipSuccess ? hipStreamWaitEvent(s, e->join, 0) : jerr;
  if (werr != hipSuccess) {  // cannot order s after s2: drain both before the workspaces are reused
    (void)hipStreamSynchronize(s2);
    (void)hipStreamSynchronize(s);
  }
  if (!lrc && werr == hipSuccess) HBH_CHECK(hipMemcpyAsync(hs, dout, out_bytes, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (lrc) return lrc;
    if (werr != hipSuccess) return fail(HBH_ERR_DEVICE, std::string("split check join: ") + hipGetErrorString(werr));
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  std::memcpy(out, hs, ncomb * HBH_G2_BYTES);
  std::memcpy(verdicts, hs + o_v, ncomb);
  for (size_t c = 0; c < ncomb; c++) status[c] = lst[c];
  return HBH_OK;
}
}  // namespace

extern "C" {

int hbh_g1_mul(hbh_engine* e, size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out) {
  return run_mul(e, n, pts, HBH_G1_BYTES, scalars, out, hbl::g1_mul);
}
int hbh_g2_mul(hbh_engine* e, size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out) {
  return run_mul(e, n, pts, HBH_G2_BYTES, scalars, out, hbl::g2_mul);
}
int hbh_interpolate_g2(hbh_engine* e, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out,
                       int* status) {
  return run_interp(e, ncomb, t, idx, pts, out, status, true);
}
int hbh_interpolate_g1(hbh_engine* e, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out,
                       int* status) {
  return run_interp(e, ncomb, t, idx, pts, out, status, false);
}

// ThresholdSign::combine_and_verify_sig (src/threshold_sign.rs:249-270) as one device pass: the
// interpolated signature stays in HBM and feeds the master check e(pk, H_c) == e(g1, sig_c) on the
// same stream -- no host round trip between combine and verify.
int hbh_combine_verify_g2(hbh_engine* e, size_t ncomb, int t, const uint32_t* idx, const uint8_t* shares,
                          const uint8_t* master_pk, const uint8_t* hashes, uint8_t* out, int* status,
                          uint8_t* verdicts) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (ncomb == 0) return HBH_OK;
  if (!idx || !shares || !master_pk || !hashes || !out || !status || !verdicts) return fail(HBH_ERR_ARG, "null pointer");
  const size_t m = (size_t)t + 1;
  if (ncomb * m > (size_t)1 << 26) return fail(HBH_ERR_ARG, "batch too large");
  std::vector<uint32_t> xs(ncomb * m);
  for (size_t k = 0; k < ncomb * m; k++) {
    if (idx[k] == 0xffffffffu) return fail(HBH_ERR_ARG, "node index out of range");
    xs[k] = idx[k] + 1;
  }
  {
    // one contract for both forms of the check: a master key coordinate >= p is an argument error
    // (the split form rejected it, interpolate-then-verify returned verdicts)
    uint8_t negpk[HBH_G1_BYTES];
    if (hbh__host_g1_neg(master_pk, negpk)) return fail(HBH_ERR_ARG, "master key coordinate >= p");
  }
  if (e->split_check && (e->split_max ? ncomb <= e->split_max : ncomb * (m + 1) <= split_waves_max(t)) &&
      ncomb <= INTERP_PAIR_MAX && hbl::interp_g2_pair_fits((int)m))
    return combine_verify_split(e, ncomb, m, xs, shares, master_pk, hashes, out, status, verdicts);
  // P1 = master pk (one record per combine), P2 = the G1 generator (a flag, nothing uploaded)
  std::vector<uint8_t> p12(ncomb * HBH_G1_BYTES);
  for (size_t c = 0; c < ncomb; c++) std::memcpy(p12.data() + c * HBH_G1_BYTES, master_pk, HBH_G1_BYTES);
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->in_a.ensure(ncomb * m * 4));
  HBH_CHECK(e->in_b.ensure(ncomb * m * HBH_G2_BYTES));
  HBH_CHECK(e->in_q1.ensure(ncomb * HBH_G2_BYTES));
  HBH_CHECK(e->in_p1.ensure(p12.size()));
  HBH_CHECK(e->out_x.ensure(ncomb * HBH_G2_BYTES));
  HBH_CHECK(e->status.ensure(ncomb * sizeof(int)));
  HBH_CHECK(e->out_v.ensure(ncomb));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, xs.data(), ncomb * m * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, shares, ncomb * m * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_q1.p, hashes, ncomb * HBH_G2_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_p1.p, p12.data(), p12.size(), hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemsetAsync(e->status.p, 0, ncomb * sizeof(int), s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  rc = launch_combine_g2(e, s, ncomb, m, (const uint32_t*)e->in_a.p, e->in_b.p, e->out_x.p, (int*)e->status.p,
                         xs.data());
  if (rc) return rc;
  e->timer.end(s, tm);
  rc = run_pairing_dev(e, s, ncomb, e->in_p1.p, e->in_q1.p, ncomb, nullptr, nullptr, e->out_x.p, ncomb, nullptr, 1,
                       (uint8_t*)e->out_v.p);
  if (rc) return rc;
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, ncomb * HBH_G2_BYTES, hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipMemcpyAsync(status, e->status.p, ncomb * sizeof(int), hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipMemcpyAsync(verdicts, e->out_v.p, ncomb, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

int hbh_bivar_row(hbh_engine* e, size_t nrow, int t, size_t nparts, const uint8_t* commits, const uint32_t* part_idx,
                  const uint32_t* xs, uint8_t* out) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (nrow == 0) return HBH_OK;
  if (!commits || !part_idx || !xs || !out) return fail(HBH_ERR_ARG, "null pointer");
  const size_t ncoef = (size_t)(t + 1) * (t + 2) / 2;
  for (size_t r = 0; r < nrow; r++)
    if (part_idx[r] >= nparts) return fail(HBH_ERR_ARG, "part index out of range");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  const size_t nout = nrow * (t + 1);
  HBH_CHECK(e->in_a.ensure(nparts * ncoef * HBH_G1_BYTES));
  HBH_CHECK(e->in_b.ensure(nrow * 4));
  HBH_CHECK(e->in_c.ensure(nrow * 4));
  HBH_CHECK(e->out_x.ensure(nout * HBH_G1_BYTES));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, commits, nparts * ncoef * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, part_idx, nrow * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_c.p, xs, nrow * 4, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::bivar_row(s, (int)nrow, t, e->in_a.p, (const uint32_t*)e->in_b.p, (const uint32_t*)e->in_c.p,
                           e->out_x.p));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, nout * HBH_G1_BYTES, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // extern "C"

namespace {
// Byte-level half of pairing 0.14's compressed decoding: flags (0x80 compressed, 0x40 infinity --
// then 0xc0 || 0...0 exactly --, 0x20 larger y) and the big-endian -> little-endian word reversal.
// The encoding holds nfe 48-byte field elements, highest Fp2 coefficient first (G2: x.c1 || x.c0);
// words come out as coefficient 0 first (12 words each).
void parse_compressed(const uint8_t* b, int nfe, uint32_t* words, uint8_t& f) {
  f = 0;
  if (!(b[0] & 0x80)) {
    f = hbl::WIRE_REJECT;
  } else if (b[0] & 0x40) {
    bool zero = (b[0] & 0x3f) == 0;
    for (int k = 1; k < 48 * nfe && zero; k++) zero = b[k] == 0;
    f = zero ? hbl::WIRE_INFINITY : hbl::WIRE_REJECT;
  } else if (b[0] & 0x20) {
    f = hbl::WIRE_GREATEST;
  }
  for (int c = 0; c < nfe; c++) {
    const uint8_t* e = b + 48 * (nfe - 1 - c);
    for (int w = 0; w < 12; w++) {
      uint32_t v = 0;
      for (int k = 0; k < 4; k++) {
        const int pos = 47 - (w * 4 + k);  // little-endian byte w*4+k of the element
        const uint8_t byte = (e == b && pos == 0) ? (uint8_t)(b[0] & 0x1f) : e[pos];
        v |= (uint32_t)byte << (8 * k);
      }
      words[c * 12 + w] = v;
    }
  }
}

int run_decompress(hbh_engine* e, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok, bool g2) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!in || !out || !ok) return fail(HBH_ERR_ARG, "null pointer");
  if (n > (size_t)1 << 28) return fail(HBH_ERR_ARG, "batch too large");
  const int nfe = g2 ? 2 : 1;
  const size_t pb = g2 ? HBH_G2_BYTES : HBH_G1_BYTES;
  std::vector<uint32_t> xw(n * 12 * nfe);
  std::vector<uint8_t> fl(n);
  for (size_t i = 0; i < n; i++) parse_compressed(in + i * 48 * nfe, nfe, xw.data() + i * 12 * nfe, fl[i]);
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->in_a.ensure(xw.size() * 4));
  HBH_CHECK(e->in_b.ensure(n));
  HBH_CHECK(e->out_x.ensure(n * pb));
  HBH_CHECK(e->out_v.ensure(n));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, xw.data(), xw.size() * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, fl.data(), n, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  if (g2)
    HBH_CHECK(hbl::g2_decompress(s, (int)n, (const uint32_t*)e->in_a.p, (const uint8_t*)e->in_b.p, e->out_x.p,
                                 (uint8_t*)e->out_v.p));
  else
    HBH_CHECK(hbl::g1_decompress(s, (int)n, (const uint32_t*)e->in_a.p, (const uint8_t*)e->in_b.p, e->out_x.p,
                                 (uint8_t*)e->out_v.p));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, n * pb, hipMemcpyDeviceToHost, s));
  HBH_CHECK(hipMemcpyAsync(ok, e->out_v.p, n, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}
}  // namespace

extern "C" {

int hbh_g1_decompress(hbh_engine* e, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok) {
  return run_decompress(e, n, in, out, ok, false);
}
int hbh_g2_decompress(hbh_engine* e, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok) {
  return run_decompress(e, n, in, out, ok, true);
}

int hbh_commitment_eval(hbh_engine* e, size_t n, int t, size_t ncommits, const uint8_t* commits,
                        const uint32_t* commit_idx, const uint32_t* xs, uint8_t* out) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (n == 0) return HBH_OK;
  if (!commits || !commit_idx || !xs || !out) return fail(HBH_ERR_ARG, "null pointer");
  if (n > (size_t)1 << 28) return fail(HBH_ERR_ARG, "batch too large");
  for (size_t r = 0; r < n; r++)
    if (commit_idx[r] >= ncommits) return fail(HBH_ERR_ARG, "commitment index out of range");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  const size_t cbytes = ncommits * (size_t)(t + 1) * HBH_G1_BYTES;
  HBH_CHECK(e->in_a.ensure(cbytes));
  HBH_CHECK(e->in_b.ensure(n * 4));
  HBH_CHECK(e->in_c.ensure(n * 4));
  HBH_CHECK(e->out_x.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, commits, cbytes, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_b.p, commit_idx, n * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_c.p, xs, n * 4, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::commit_eval(s, (int)n, t, e->in_a.p, (const uint32_t*)e->in_b.p, (const uint32_t*)e->in_c.p,
                             e->out_x.p));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, n * HBH_G1_BYTES, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

int hbh_bivar_ack_check(hbh_engine* e, size_t nack, int t, size_t nparts, const uint8_t* commits,
                        const uint32_t* part_idx, const uint32_t* xs, const uint32_t* ys, const uint8_t* vals,
                        uint8_t* verdicts) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (nack == 0) return HBH_OK;
  if (!commits || !part_idx || !xs || !ys || !vals || !verdicts) return fail(HBH_ERR_ARG, "null pointer");
  const size_t ncoef = (size_t)(t + 1) * (t + 2) / 2;
  // one row(x) per distinct (part, x): evaluate(x, y) = sum_j row(x)_j y^j
  std::vector<uint32_t> row_part, row_x, row_of(nack);
  {
    std::unordered_map<uint64_t, uint32_t> seen;
    seen.reserve(nack < 4096 ? nack : 4096);
    for (size_t a = 0; a < nack; a++) {
      if (part_idx[a] >= nparts) return fail(HBH_ERR_ARG, "part index out of range");
      const uint64_t key = ((uint64_t)part_idx[a] << 32) | xs[a];
      auto it = seen.emplace(key, (uint32_t)row_part.size());
      if (it.second) {
        row_part.push_back(part_idx[a]);
        row_x.push_back(xs[a]);
      }
      row_of[a] = it.first->second;
    }
  }
  const size_t nrow = row_part.size();
  // acks in order of y: the lanes of a wave then run the same small-scalar double-and-add
  std::vector<uint32_t> order(nack);
  for (size_t a = 0; a < nack; a++) order[a] = (uint32_t)a;
  std::stable_sort(order.begin(), order.end(), [ys](uint32_t i, uint32_t j) { return ys[i] < ys[j]; });
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  {
    const int rc_ = begin_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(e->in_a.ensure(nparts * ncoef * HBH_G1_BYTES));
  HBH_CHECK(e->in_b.ensure(nrow * 8 + nack * 12));
  HBH_CHECK(e->in_c.ensure(nack * HBH_FR_BYTES));
  HBH_CHECK(e->work.ensure(hbl::bivar_rows_quad_bytes((int)nrow, t)));
  HBH_CHECK(e->out_v.ensure(nack));
  uint32_t* d_rp = (uint32_t*)e->in_b.p;
  uint32_t* d_rx = d_rp + nrow;
  uint32_t* d_ro = d_rx + nrow;
  uint32_t* d_y = d_ro + nack;
  uint32_t* d_ord = d_y + nack;
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, commits, nparts * ncoef * HBH_G1_BYTES, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_rp, row_part.data(), nrow * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_rx, row_x.data(), nrow * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_ro, row_of.data(), nack * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_y, ys, nack * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_ord, order.data(), nack * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_c.p, vals, nack * HBH_FR_BYTES, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::bivar_row_quad(s, (int)nrow, t, e->in_a.p, d_rp, d_rx, e->work.p));
  rc = ensure_fbtab(e, s);
  if (rc) return rc;
  HBH_CHECK(hbl::bivar_check_quad(s, (int)nack, t, e->work.p, d_ro, d_y, (const uint32_t*)e->in_c.p, e->fbtab.p,
                                  (uint8_t*)e->out_v.p, d_ord));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(verdicts, e->out_v.p, nack, hipMemcpyDeviceToHost, s));
  {
    const int rc_ = end_call(e, s);
    if (rc_) return rc_;
  }
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device-resident variants
// Inputs and outputs in device memory, asynchronous on `stream` (NULL = engine stream), ordered
// after the engine's previous call like hbh_verify_pairing_eq_dev.
namespace {
hipStream_t dev_stream(hbh_engine* e, void* stream) { return stream ? (hipStream_t)stream : e->stream; }

int run_interp_dev(hbh_engine* e, void* stream, size_t ncomb, int t, const uint32_t* d_idx, const void* d_pts,
                   void* d_out, int* d_status, bool g2) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (ncomb == 0) return HBH_OK;
  if (!d_idx || !d_pts || !d_out || !d_status) return fail(HBH_ERR_ARG, "null pointer");
  const size_t m = (size_t)t + 1;
  if (ncomb * m > (size_t)1 << 26) return fail(HBH_ERR_ARG, "batch too large");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = dev_stream(e, stream);
  rc = begin_call(e, s);
  if (rc) return rc;
  HBH_CHECK(e->in_a.ensure(ncomb * m * 4));
  HBH_CHECK(hipMemsetAsync(d_status, 0, ncomb * sizeof(int), s));
  HBH_CHECK(hbl::index_plus_one(s, (int)(ncomb * m), (int)m, d_idx, (uint32_t*)e->in_a.p, d_status));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  if (g2) {
    rc = launch_combine_g2(e, s, ncomb, m, (const uint32_t*)e->in_a.p, d_pts, d_out, d_status);
    if (rc) return rc;
  } else {
    rc = launch_combine_g1(e, s, ncomb, m, (const uint32_t*)e->in_a.p, d_pts, d_out, d_status);
    if (rc) return rc;
  }
  e->timer.end(s, tm);
  return end_call(e, s);
}

int run_decompress_dev(hbh_engine* e, void* stream, size_t n, const uint8_t* d_in, void* d_out, uint8_t* d_ok,
                       bool g2) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!d_in || !d_out || !d_ok) return fail(HBH_ERR_ARG, "null pointer");
  if (n > (size_t)1 << 28) return fail(HBH_ERR_ARG, "batch too large");
  const int nfe = g2 ? 2 : 1;
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = dev_stream(e, stream);
  // a staging slot of its own: wait for the last general call and this slot's previous user only
  const int slot = e->wire_slot;
  e->wire_slot ^= 1;
  HBH_CHECK(hipStreamWaitEvent(s, e->done, 0));
  HBH_CHECK(hipStreamWaitEvent(s, e->wire_done[slot], 0));
  HBH_CHECK(e->wire_w[slot].ensure(n * 12 * nfe * 4));
  HBH_CHECK(e->wire_f[slot].ensure(n));
  uint32_t* xw = (uint32_t*)e->wire_w[slot].p;
  uint8_t* fl = (uint8_t*)e->wire_f[slot].p;
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::wire_parse(s, (int)n, nfe, d_in, xw, fl));
  if (g2)
    HBH_CHECK(hbl::g2_decompress(s, (int)n, xw, fl, d_out, d_ok));
  else
    HBH_CHECK(hbl::g1_decompress(s, (int)n, xw, fl, d_out, d_ok));
  e->timer.end(s, tm);
  HBH_CHECK(hipEventRecord(e->wire_done[slot], s));
  return HBH_OK;
}
}  // namespace

extern "C" {

int hbh_interpolate_g1_dev(hbh_engine* e, void* stream, size_t ncomb, int t, const uint32_t* d_idx, const void* d_pts,
                           void* d_out, int* d_status) {
  return run_interp_dev(e, stream, ncomb, t, d_idx, d_pts, d_out, d_status, false);
}
int hbh_interpolate_g2_dev(hbh_engine* e, void* stream, size_t ncomb, int t, const uint32_t* d_idx, const void* d_pts,
                           void* d_out, int* d_status) {
  return run_interp_dev(e, stream, ncomb, t, d_idx, d_pts, d_out, d_status, true);
}
int hbh_g1_decompress_dev(hbh_engine* e, void* stream, size_t n, const uint8_t* d_in, void* d_out, uint8_t* d_ok) {
  return run_decompress_dev(e, stream, n, d_in, d_out, d_ok, false);
}
int hbh_g2_decompress_dev(hbh_engine* e, void* stream, size_t n, const uint8_t* d_in, void* d_out, uint8_t* d_ok) {
  return run_decompress_dev(e, stream, n, d_in, d_out, d_ok, true);
}

int hbh_bivar_ack_check_dev(hbh_engine* e, void* stream, size_t nack, int t, const void* d_commits, size_t nrow,
                            const uint32_t* d_row_part, const uint32_t* d_row_x, const uint32_t* d_row_of,
                            const uint32_t* d_ys, const void* d_vals, uint8_t* d_verdicts) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  int rc = check_t(t);
  if (rc) return rc;
  if (nack == 0) return HBH_OK;
  if (!d_commits || !d_row_part || !d_row_x || !d_row_of || !d_ys || !d_vals || !d_verdicts || nrow == 0)
    return fail(HBH_ERR_ARG, "null pointer");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = dev_stream(e, stream);
  rc = begin_call(e, s);
  if (rc) return rc;
  HBH_CHECK(e->work.ensure(hbl::bivar_rows_quad_bytes((int)nrow, t)));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::bivar_row_quad(s, (int)nrow, t, d_commits, d_row_part, d_row_x, e->work.p));
  rc = ensure_fbtab(e, s);
  if (rc) return rc;
  HBH_CHECK(hbl::bivar_check_quad(s, (int)nack, t, e->work.p, d_row_of, d_ys, (const uint32_t*)d_vals, e->fbtab.p,
                                  d_verdicts, nullptr));
  e->timer.end(s, tm);
  return end_call(e, s);
}

}  // extern "C"

extern "C" {

// out[i] = g1 * k_i from the comb table: Poly::commitment / BivarPoly::commitment and public-key
// derivation (src/sync_key_gen.rs:346-357, 508; network_info.rs:59-62).
int hbh_g1_mul_gen(hbh_engine* e, size_t n, const uint8_t* scalars, uint8_t* out) {
  if (!e) return fail(HBH_ERR_ARG, "null engine");
  if (n == 0) return HBH_OK;
  if (!scalars || !out) return fail(HBH_ERR_ARG, "null pointer");
  if (n > (size_t)1 << 28) return fail(HBH_ERR_ARG, "batch too large");
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  int rc = begin_call(e, s);
  if (rc) return rc;
  rc = ensure_fbtab(e, s);
  if (rc) return rc;
  HBH_CHECK(e->in_a.ensure(n * 32));
  HBH_CHECK(e->out_x.ensure(n * HBH_G1_BYTES));
  HBH_CHECK(hipMemcpyAsync(e->in_a.p, scalars, n * 32, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::g1_mul_gen(s, (int)n, e->fbtab.p, (const uint32_t*)e->in_a.p, e->out_x.p));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, n * HBH_G1_BYTES, hipMemcpyDeviceToHost, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device-resident commitment sets
// ProposalState::commit (src/sync_key_gen.rs:254-262) lives as long as the SyncKeyGen instance and
// is read by every row check (:496) and every Ack check (:542): a set keeps such commitments in HBM
// (uploaded once) together with the Jacobian rows row(x) computed so far, so an Ack drain uploads
// only its indices and values.
struct hbh_commit_set {
  hbh_engine* e = nullptr;
  int t = 0;
  size_t ncoef = 0;
  size_t nparts = 0;
  void* commits = nullptr;  // nparts * ncoef ABI G1 points
  size_t commits_cap = 0;   // bytes
  // cached rows row(x), two layouts: [0] Jacobian signed-limb rows of the lane-quad check
  // (hbl::bivar_rows_quad_bytes(1, t) each), [1] affine ABI rows of the one-lane check
  // ((t + 1) G1 points each)
  struct Rows {
    std::unordered_map<uint64_t, uint32_t> slot;  // (part << 32 | x) -> row
    size_t n = 0;
    void* p = nullptr;
    size_t cap = 0;  // bytes
  } rows[2];
  DevBuf stage;      // indices of rows computed by a call
};

// Frees a set's device memory and detaches it from its engine (cs->e = nullptr): every later call on
// the set fails with HBH_ERR_ARG, and hbh_commit_set_destroy only deletes the host object.  Caller
// holds the engine lock with the engine's streams drained.
void release_set_device(hbh_commit_set* cs) {
  if (cs->commits) (void)hipFree(cs->commits);
  cs->commits = nullptr;
  cs->commits_cap = 0;
  cs->nparts = 0;
  for (auto& R : cs->rows) {
    if (R.p) (void)hipFree(R.p);
    R.p = nullptr;
    R.cap = 0;
    R.n = 0;
    R.slot.clear();
  }
  cs->stage.release();
  cs->e = nullptr;
}

namespace {
// Grow a device allocation to at least `want` bytes, keeping its first `used` bytes.
int grow_keep(hipStream_t s, void** p, size_t* cap, size_t used, size_t want) {
  if (want <= *cap) return HBH_OK;
  const size_t nc = std::max(want, *cap * 2);
  void* q = nullptr;
  HBH_CHECK(hipMalloc(&q, nc));
  if (used) HBH_CHECK(hipMemcpyAsync(q, *p, used, hipMemcpyDeviceToDevice, s));
  HBH_CHECK(hipStreamSynchronize(s));
  if (*p) HBH_CHECK(hipFree(*p));
  *p = q;
  *cap = nc;
  return HBH_OK;
}

// Row slots for n (part, x) requests; rows not cached yet are computed on stream s (k_bivar_row_quad
// into the set's row buffer).  Caller holds the engine lock.
int set_rows(hbh_commit_set* cs, hipStream_t s, bool affine, size_t n, const uint32_t* part_idx, const uint32_t* xs,
             std::vector<uint32_t>& slot) {
  hbh_commit_set::Rows& R = cs->rows[affine ? 1 : 0];
  std::vector<uint32_t> np, nx;
  slot.resize(n);
  uint64_t last_key = ~(uint64_t)0;
  uint32_t last_slot = 0;
  for (size_t a = 0; a < n; a++) {
    const uint64_t key = ((uint64_t)part_idx[a] << 32) | xs[a];
    if (key != last_key) {  // consecutive acks of one (part, x) skip the map
      auto it = R.slot.emplace(key, (uint32_t)(R.n + np.size()));
      if (it.second) {
        np.push_back(part_idx[a]);
        nx.push_back(xs[a]);
      }
      last_key = key;
      last_slot = it.first->second;
    }
    slot[a] = last_slot;
  }
  if (np.empty()) return HBH_OK;
  const size_t row_bytes = affine ? (size_t)(cs->t + 1) * HBH_G1_BYTES : hbl::bivar_rows_quad_bytes(1, cs->t);
  const size_t first = R.n;
  auto compute = [&]() -> int {
    int rc = grow_keep(s, &R.p, &R.cap, first * row_bytes, (first + np.size()) * row_bytes);
    if (rc) return rc;
    HBH_CHECK(cs->stage.ensure(np.size() * 8));
    uint32_t* d_p = (uint32_t*)cs->stage.p;
    HBH_CHECK(hipMemcpyAsync(d_p, np.data(), np.size() * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_p + np.size(), nx.data(), nx.size() * 4, hipMemcpyHostToDevice, s));
    hipEvent_t tm = cs->e->timer.begin(s, HBH_STAGE_CURVE, cs->e->profiling);
    void* dst = (uint8_t*)R.p + first * row_bytes;
    if (affine)
      HBH_CHECK(hbl::bivar_row(s, (int)np.size(), cs->t, cs->commits, d_p, d_p + np.size(), dst));
    else
      HBH_CHECK(hbl::bivar_row_quad(s, (int)np.size(), cs->t, cs->commits, d_p, d_p + np.size(), dst));
    cs->e->timer.end(s, tm);
    // the staged indices are read by the kernel: the host vectors die at return
    HBH_CHECK(hipStreamSynchronize(s));
    return HBH_OK;
  };
  const int rc = compute();
  if (rc) {  // the new slots were never filled: forget them, so no later ack reads an empty row
    for (size_t k = 0; k < np.size(); k++) R.slot.erase(((uint64_t)np[k] << 32) | nx[k]);
    return rc;
  }
  R.n = first + np.size();
  return HBH_OK;
}

// Finite-difference plan of an Ack drain (hbl::bivar_fd): a row slot whose acks form a dense run of y
// -- at least 2 (t + 1) acks spanning at most twice as many consecutive y, as a node's drain has (one
// Ack per sender per Part) -- is evaluated at every y of its span from the difference table at y0 (the
// seed levels: (t+1)(t+2)/2 small products) and t additions per further y; its acks then compare
// against those points (epos).  y0 = 0 when the run starts at y <= t + 1 (the seed's products are then
// one per entry, worth the few extra steps), else the run's first y.  Every other ack takes the Horner
// kernel (other, in order of y).  FD rows are sorted by span length (the run kernel's workgroups step
// their rows together); a span is at least 2 (t + 1) points (the seed's two tables live in it).
struct FdPlan {
  std::vector<uint32_t> slot, y0, off, len;  // per FD row
  std::vector<uint32_t> epos;                // per ack (FD acks only)
  std::vector<uint32_t> fd_acks, other;      // ack lists
  size_t npts = 0;                           // E points of all FD rows
};
void plan_fd(size_t n, const std::vector<uint32_t>& slot, const uint32_t* ys, int t, FdPlan& P) {
  const uint64_t T1 = (uint64_t)t + 1;
  uint32_t nslot = 0;
  for (size_t a = 0; a < n; a++) nslot = std::max(nslot, slot[a] + 1);
  std::vector<uint32_t> cnt(nslot, 0), ymin(nslot, 0xffffffffu), ymax(nslot, 0);
  for (size_t a = 0; a < n; a++) {
    const uint32_t s = slot[a];
    cnt[s]++;
    ymin[s] = std::min(ymin[s], ys[a]);
    ymax[s] = std::max(ymax[s], ys[a]);
  }
  std::vector<uint32_t> cand;
  for (uint32_t s = 0; s < nslot; s++) {
    if (!cnt[s] || T1 > 128) continue;
    if (ymin[s] <= T1) ymin[s] = 0;  // seed at y0 = 0
    const uint64_t span = (uint64_t)ymax[s] - ymin[s] + 1;
    if (cnt[s] >= 2 * T1 && span >= 2 * T1 && span <= 2 * (uint64_t)cnt[s] && span < ((uint64_t)1 << 20))
      cand.push_back(s);
  }
  std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) {
    const uint32_t la = ymax[a] - ymin[a], lb = ymax[b] - ymin[b];
    return la != lb ? la > lb : ymin[a] < ymin[b];
  });
  std::vector<int32_t> fd_of(nslot, -1);
  for (uint32_t s : cand) {
    fd_of[s] = (int32_t)P.slot.size();
    P.slot.push_back(s);
    P.y0.push_back(ymin[s]);
    P.off.push_back((uint32_t)P.npts);
    P.len.push_back(ymax[s] - ymin[s] + 1);  // >= 2 (t + 1)
    P.npts += ymax[s] - ymin[s] + 1;
  }
  P.epos.assign(n, 0);
  for (size_t a = 0; a < n; a++) {
    const int32_t f = fd_of[slot[a]];
    if (f < 0) {
      P.other.push_back((uint32_t)a);
    } else {
      P.epos[a] = P.off[f] + (ys[a] - P.y0[f]);
      P.fd_acks.push_back((uint32_t)a);
    }
  }
}

// Acks in order of y (stable): the lanes of a wave then run the same small-scalar double-and-add.
// y is a node index + 1, so a counting sort does it in O(n) (10^6 acks of a network-wide check).
// Round 4 measured (row tile, y) orders, whose waves re-read one tile's rows while they sit in L2:
// HBM traffic per 10^6 acks falls from 4.68 GB (this order) to 0.74 GB (tiles of 256 row slots) and
// 0.24 GB (1,024), but the launch is SLOWER at every tile size -- 54.2 ms here, 57.5 (64), 61.8-62.2
// (256), 60.6-60.8 (1,024), 57.4 (4,096) (profiles/r04/c11_ack_tile_traffic.txt; with an XCD-
// contiguous workgroup map as well: 57.5-58.2 ms, c3_ab.txt).  The kernel is VALU-bound at two
// waves per SIMD (255 VGPRs) and its row fetches overlap the Horner arithmetic, so this order stays.
void order_by_y(size_t n, const uint32_t* ys, std::vector<uint32_t>& order) {
  order.resize(n);
  uint32_t ymax = 0;
  for (size_t a = 0; a < n; a++) ymax = std::max(ymax, ys[a]);
  if (ymax < (1u << 20)) {
    std::vector<uint32_t> start((size_t)ymax + 2, 0);
    for (size_t a = 0; a < n; a++) start[(size_t)ys[a] + 1]++;
    for (size_t y = 1; y < start.size(); y++) start[y] += start[y - 1];
    for (size_t a = 0; a < n; a++) order[start[ys[a]]++] = (uint32_t)a;
    return;
  }
  for (size_t a = 0; a < n; a++) order[a] = (uint32_t)a;
  std::stable_sort(order.begin(), order.end(), [ys](uint32_t i, uint32_t j) { return ys[i] < ys[j]; });
}

int check_parts(const hbh_commit_set* cs, size_t n, const uint32_t* part_idx) {
  for (size_t a = 0; a < n; a++)
    if (part_idx[a] >= cs->nparts) return fail(HBH_ERR_ARG, "part index out of range");
  return HBH_OK;
}
}  // namespace

extern "C" {

int hbh_commit_set_create(hbh_engine* e, int t, hbh_commit_set** out) {
  if (!e || !out) return fail(HBH_ERR_ARG, "null pointer");
  *out = nullptr;
  int rc = check_t(t);
  if (rc) return rc;
  hbh_commit_set* cs = new hbh_commit_set();
  cs->e = e;
  cs->t = t;
  cs->ncoef = (size_t)(t + 1) * (t + 2) / 2;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    e->sets.insert(cs);
  }
  *out = cs;
  return HBH_OK;
}

int hbh_commit_set_destroy(hbh_commit_set* cs) {
  if (!cs) return HBH_OK;
  if (hbh_engine* e = cs->e) {  // else: detached by hbh_engine_destroy, device memory already freed
    std::lock_guard<std::mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    (void)hipEventSynchronize(e->done);
    (void)hipStreamSynchronize(e->stream);
    e->sets.erase(cs);
    release_set_device(cs);
  }
  delete cs;
  return HBH_OK;
}

int hbh_commit_set_add(hbh_commit_set* cs, size_t nparts, const uint8_t* commits, size_t* first) {
  if (!cs) return fail(HBH_ERR_ARG, "null commitment set");
  if (!cs->e) return fail(HBH_ERR_ARG, "commitment set detached: its engine was destroyed");
  if (first) *first = cs->nparts;
  if (nparts == 0) return HBH_OK;
  if (!commits) return fail(HBH_ERR_ARG, "null pointer");
  if (cs->nparts + nparts > ((size_t)1 << 24)) return fail(HBH_ERR_ARG, "too many commitments");
  hbh_engine* e = cs->e;
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  int rc = begin_call(e, s);
  if (rc) return rc;
  const size_t cb = cs->ncoef * HBH_G1_BYTES;
  rc = grow_keep(s, &cs->commits, &cs->commits_cap, cs->nparts * cb, (cs->nparts + nparts) * cb);
  if (rc) return rc;
  HBH_CHECK(hipMemcpyAsync((uint8_t*)cs->commits + cs->nparts * cb, commits, nparts * cb, hipMemcpyHostToDevice, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  cs->nparts += nparts;
  return HBH_OK;
}

int hbh_commit_set_size(const hbh_commit_set* cs, size_t* nparts, size_t* nrows) {
  if (!cs) return fail(HBH_ERR_ARG, "null commitment set");
  if (nparts) *nparts = cs->nparts;
  if (nrows) *nrows = cs->rows[0].n + cs->rows[1].n;
  return HBH_OK;
}

int hbh_bivar_row_set(hbh_commit_set* cs, size_t nrow, const uint32_t* part_idx, const uint32_t* xs, uint8_t* out) {
  if (!cs) return fail(HBH_ERR_ARG, "null commitment set");
  if (!cs->e) return fail(HBH_ERR_ARG, "commitment set detached: its engine was destroyed");
  if (nrow == 0) return HBH_OK;
  if (!part_idx || !xs || !out) return fail(HBH_ERR_ARG, "null pointer");
  int rc = check_parts(cs, nrow, part_idx);
  if (rc) return rc;
  hbh_engine* e = cs->e;
  const int t = cs->t;
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  rc = begin_call(e, s);
  if (rc) return rc;
  const size_t nout = nrow * (t + 1);
  HBH_CHECK(e->in_b.ensure(nrow * 8));
  HBH_CHECK(e->out_x.ensure(nout * HBH_G1_BYTES));
  uint32_t* d_p = (uint32_t*)e->in_b.p;
  HBH_CHECK(hipMemcpyAsync(d_p, part_idx, nrow * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_p + nrow, xs, nrow * 4, hipMemcpyHostToDevice, s));
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  HBH_CHECK(hbl::bivar_row(s, (int)nrow, t, cs->commits, d_p, d_p + nrow, e->out_x.p));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(out, e->out_x.p, nout * HBH_G1_BYTES, hipMemcpyDeviceToHost, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

int hbh_bivar_ack_check_set(hbh_commit_set* cs, size_t nack, const uint32_t* part_idx, const uint32_t* xs,
                            const uint32_t* ys, const uint8_t* vals, uint8_t* verdicts) {
  if (!cs) return fail(HBH_ERR_ARG, "null commitment set");
  if (!cs->e) return fail(HBH_ERR_ARG, "commitment set detached: its engine was destroyed");
  if (nack == 0) return HBH_OK;
  if (!part_idx || !xs || !ys || !vals || !verdicts) return fail(HBH_ERR_ARG, "null pointer");
  if (nack > ((size_t)1 << 28)) return fail(HBH_ERR_ARG, "batch too large");
  int rc = check_parts(cs, nack, part_idx);
  if (rc) return rc;
  std::vector<uint32_t> order;
  hbh_engine* e = cs->e;
  const int t = cs->t;
  std::lock_guard<std::mutex> lk(e->mu);
  HBH_CHECK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  rc = begin_call(e, s);
  if (rc) return rc;
  // lane quads (four lanes per ack, one wave per SIMD) for latency; one lane per ack on affine
  // rows (two waves per SIMD, mixed additions) for throughput
  const bool lane = e->ack_impl == HBH_ACK_LANE || e->ack_impl == HBH_ACK_LANE_HORNER ||
                    (e->ack_impl == HBH_ACK_AUTO && nack >= HBH_ACK_LANE_MIN);
  std::vector<uint32_t> slot;
  rc = set_rows(cs, s, lane, nack, part_idx, xs, slot);
  if (rc) return rc;
  FdPlan fd;
  if (lane && e->ack_fd && e->ack_impl != HBH_ACK_LANE_HORNER) {
    plan_fd(nack, slot, ys, t, fd);
    // the Horner kernel's acks in order of y
    std::vector<uint32_t> oy(fd.other.size());
    for (size_t k = 0; k < fd.other.size(); k++) oy[k] = ys[fd.other[k]];
    order_by_y(fd.other.size(), oy.data(), order);
    for (auto& o : order) o = fd.other[o];
  } else {
    order_by_y(nack, ys, order);
  }
  HBH_CHECK(e->in_b.ensure(nack * 12));
  HBH_CHECK(e->in_c.ensure(nack * HBH_FR_BYTES));
  HBH_CHECK(e->out_v.ensure(nack));
  uint32_t* d_ro = (uint32_t*)e->in_b.p;
  uint32_t* d_y = d_ro + nack;
  uint32_t* d_ord = d_y + nack;
  HBH_CHECK(hipMemcpyAsync(d_ro, slot.data(), nack * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(d_y, ys, nack * 4, hipMemcpyHostToDevice, s));
  if (!order.empty()) HBH_CHECK(hipMemcpyAsync(d_ord, order.data(), order.size() * 4, hipMemcpyHostToDevice, s));
  HBH_CHECK(hipMemcpyAsync(e->in_c.p, vals, nack * HBH_FR_BYTES, hipMemcpyHostToDevice, s));
  rc = ensure_fbtab(e, s);
  if (rc) return rc;
  if (!fd.slot.empty() && ensure_fb16(e, s) != HBH_OK) {
    // the 16-bit comb (96 MiB + ~192 MiB of build scratch) could not be built: the Horner kernel
    // checks every ack (same verdicts), and this engine stops planning FD runs
    e->fb16.release();
    e->ack_fd = false;
    static std::once_flag warned;
    std::call_once(warned, [] { fprintf(stderr, "hbbft_hip: no memory for the FD ack comb; Horner ack checks\n"); });
    fd = FdPlan();
    order_by_y(nack, ys, order);
  }
  const size_t nfd = fd.slot.size();
  uint32_t* d_fd = nullptr;
  if (nfd) {
    const size_t words = 4 * nfd + 2 * nack;
    HBH_CHECK(e->fd_meta.ensure(words * 4));
    HBH_CHECK(e->fd_e.ensure(fd.npts * hbl::fd_point_bytes()));
    d_fd = (uint32_t*)e->fd_meta.p;
    HBH_CHECK(hipMemcpyAsync(d_fd, fd.slot.data(), nfd * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_fd + nfd, fd.y0.data(), nfd * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_fd + 2 * nfd, fd.off.data(), nfd * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_fd + 3 * nfd, fd.len.data(), nfd * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_fd + 4 * nfd, fd.epos.data(), nack * 4, hipMemcpyHostToDevice, s));
    HBH_CHECK(hipMemcpyAsync(d_fd + 4 * nfd + nack, fd.fd_acks.data(), fd.fd_acks.size() * 4, hipMemcpyHostToDevice, s));
  }
  hipEvent_t tm = e->timer.begin(s, HBH_STAGE_CURVE, e->profiling);
  if (lane && nfd) {
    HBH_CHECK(hbl::bivar_fd(s, (int)nfd, t, cs->rows[1].p, d_fd, d_fd + nfd, d_fd + 2 * nfd, d_fd + 3 * nfd,
                            e->fd_e.p));
    HBH_CHECK(hbl::bivar_fd_check(s, (int)fd.fd_acks.size(), e->fd_e.p, d_fd + 4 * nfd, (const uint32_t*)e->in_c.p,
                                  e->fb16.p, d_fd + 4 * nfd + nack, (uint8_t*)e->out_v.p));
    HBH_CHECK(hbl::bivar_check(s, (int)order.size(), t, cs->rows[1].p, d_ro, d_y, (const uint32_t*)e->in_c.p,
                               e->fbtab.p, (uint8_t*)e->out_v.p, d_ord));
  } else if (lane)
    HBH_CHECK(hbl::bivar_check(s, (int)order.size(), t, cs->rows[1].p, d_ro, d_y, (const uint32_t*)e->in_c.p,
                               e->fbtab.p, (uint8_t*)e->out_v.p, d_ord));
  else
    HBH_CHECK(hbl::bivar_check_quad(s, (int)nack, t, cs->rows[0].p, d_ro, d_y, (const uint32_t*)e->in_c.p,
                                    e->fbtab.p, (uint8_t*)e->out_v.p, d_ord));
  e->timer.end(s, tm);
  HBH_CHECK(hipMemcpyAsync(verdicts, e->out_v.p, nack, hipMemcpyDeviceToHost, s));
  rc = end_call(e, s);
  if (rc) return rc;
  HBH_CHECK(hipStreamSynchronize(s));
  return HBH_OK;
}

}  // extern "C"
