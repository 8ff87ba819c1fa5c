// Collective transport of the multi-GPU owner-partitioned reconciliation, and the protocol itself
// (DESIGN.md §6.1), behind the C ABI: a Kernel host with no collective library of its own (a JVM
// GpuScan: Engine has no collective hook, KA/engine/Engine.java:30-64) hands libdkgpu the 128-byte
// unique id of an RCCL communicator and calls dk_replay_owner_run once per scan.
//
// delta-spark resolves a snapshot by repartitioning every action by path
// (spark/src/main/scala/org/apache/spark/sql/delta/Snapshot.scala:476-485); here the key
// (URI(path), dvUniqueId) with hash h is owned by rank h mod world and three exchanges resolve every
// action exactly (tail key records, checkpoint row hashes, candidate keys). One run is 11 collectives:
//   tail:  counts+vote, records+keys, collision/error vote, answers back
//   ckpt:  counts+vote, row hashes, answers back
//   cand:  counts+vote, records+keys, answers back, final vote
// Each "counts+vote" is one all-to-all of [error flag, sizes...] per peer, so a rank that failed in the
// local part of a step is seen by every peer at that step (every rank then returns an error instead
// of waiting in a collective for it).
//
// Transports (dk_comm):
//   RCCL    ncclSend / ncclRecv groups over xGMI on the communicator's own stream (librccl resolved at
//           run time, so N = 1 never loads it);
//   callbacks  the caller's all-to-all / all-reduce over host memory (tests over gloo; a JVM with its
//           own transport);
//   local   `world` communicators of one process, exchanged through shared memory between threads
//           (one-GPU rehearsals and tests of every rank).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/dkgpu.h"

namespace dk {
int dk_fail(const std::string& m);
hipStream_t replay_stream(dk_replay* r);
}
using dk::dk_fail;

#define CHIP(x)                                                                                   \
  do {                                                                                            \
    hipError_t _e = (x);                                                                          \
    if (_e != hipSuccess) return dk_fail(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #x); \
  } while (0)

namespace {

constexpr int kRecBytes = 32;               // OwnerKeyRec
constexpr int64_t kErrBit = 1 << 20;        // vote bit: a rank failed at this step
constexpr int64_t kCollision = 4;           // E_COLLISION: a 64-bit key-hash collision at an owner

// ---- RCCL, resolved at run time -------------------------------------------------------------
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string error;
};

const Rccl& rccl() {
  static Rccl* R = [] {
    auto* r = new Rccl();
    // the process's RCCL if one is loaded already (torch's), else the ROCm one
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { r->error = std::string("cannot load librccl.so.1: ") + dlerror(); return r; }
#define SYM(f, n) r->f = (decltype(r->f))dlsym(h, n); if (!r->f) { r->error = "librccl lacks " n; return r; }
    SYM(get_unique_id, "ncclGetUniqueId")
    SYM(init_rank, "ncclCommInitRank")
    SYM(destroy, "ncclCommDestroy")
    SYM(abort, "ncclCommAbort")
    SYM(group_start, "ncclGroupStart")
    SYM(group_end, "ncclGroupEnd")
    SYM(send, "ncclSend")
    SYM(recv, "ncclRecv")
    SYM(all_reduce, "ncclAllReduce")
    SYM(error_string, "ncclGetErrorString")
#undef SYM
    return r;
  }();
  return *R;
}

#define CNCCL(x)                                                                                  \
  do {                                                                                            \
    ncclResult_t _r = (x);                                                                        \
    if (_r != ncclSuccess) return dk_fail(std::string("RCCL error: ") + rccl().error_string(_r) + " at " #x); \
  } while (0)

// ---- grow-only scratch in host or device memory -----------------------------------------------
struct Scratch {
  void* p = nullptr;
  size_t cap = 0;
  bool device = false;
  Scratch() = default;
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  ~Scratch() { release(); }
  void release() {
    if (p) { if (device) hipFree(p); else free(p); }
    p = nullptr; cap = 0;
  }
  // at least n bytes (never a null pointer: collectives and kernels get a valid address for 0 bytes)
  int get(size_t n, bool dev, void** out) {
    if (n == 0) n = 1;
    if (p && dev == device && cap >= n) { *out = p; return 0; }
    release();
    device = dev;
    size_t c = 256;
    while (c < n) c <<= 1;
    if (dev) {
      if (hipMalloc(&p, c) != hipSuccess) { p = nullptr; return dk_fail("dk_comm: hipMalloc failed for " + std::to_string(c) + " bytes"); }
    } else if (!(p = malloc(c))) {
      return dk_fail("dk_comm: out of host memory");
    }
    cap = c;
    *out = p;
    return 0;
  }
};

// ---- the in-process hub of local communicators ----------------------------------------------
struct Hub {
  int world;
  std::mutex side_mu;                         // DK_LOCAL_SERIAL=1: one rank's local step at a time
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  // what each rank posted for the current collective
  struct Post { const uint8_t* send; const int64_t* sbytes; uint8_t* recv; const int64_t* rbytes; int64_t* vals; };
  std::vector<Post> post;
  explicit Hub(int w) : world(w), post(w) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const long g = gen;
    if (++arrived == world) { arrived = 0; gen++; cv.notify_all(); return; }
    cv.wait(lk, [&] { return gen != g; });
  }
};

}  // namespace

struct dk_comm {
  enum Kind { RCCL = 0, CALLBACKS = 1, LOCAL = 2 } kind;
  int world = 1, rank = 0, device = -1;
  // RCCL
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  // callbacks
  dk_comm_callbacks cb{};
  // local
  std::shared_ptr<Hub> hub;
  bool local_device = false;
  // staging between the protocol's buffers and the transport's memory
  Scratch stage_send, stage_recv, small;
  // the protocol's buffers (side memory), kept between runs
  Scratch b_recs, b_keys, b_rrecs, b_rkeys, b_ans, b_back, b_cksend, b_ckrecv, b_flags, b_ckback;
  // the last run: phase wall times, local-step times per phase, time inside collectives (ms), the
  // payload bytes sent and the number of collectives
  double ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double step_ms[16] = {0};                   // per local step, in dk_owner_side member order
  int64_t bytes_sent = 0, n_coll = 0;
  bool transport_on_device() const { return kind == RCCL || (kind == LOCAL && local_device); }
};

namespace {

// One plane of an all-to-all: send[soff..] of sbytes[p] bytes to each rank p (owner-major runs), the
// runs received from every rank laid out by rbytes in rank order.
struct Plane {
  const void* send;
  const int64_t* sbytes;
  void* recv;
  const int64_t* rbytes;
};

int64_t total(const int64_t* v, int n) { int64_t s = 0; for (int i = 0; i < n; i++) s += v[i]; return s; }

int rccl_a2a(dk_comm* c, const Plane* P, int np) {
  const Rccl& R = rccl();
  const int W = c->world;
  CNCCL(R.group_start());
  for (int k = 0; k < np; k++) {
    int64_t so = 0, ro = 0;
    for (int q = 0; q < W; q++) {
      const int64_t sb = P[k].sbytes[q], rb = P[k].rbytes[q];
      if (q == c->rank) {
        if (sb != rb) { R.group_end(); return dk_fail("dk_comm: self send / receive sizes differ"); }
        if (sb) {
          hipError_t e = hipMemcpyAsync((uint8_t*)P[k].recv + ro, (const uint8_t*)P[k].send + so, sb, hipMemcpyDeviceToDevice, c->stream);
          if (e != hipSuccess) { R.group_end(); return dk_fail(std::string("HIP error: ") + hipGetErrorString(e)); }
        }
      } else {
        if (sb) {
          ncclResult_t r = R.send((const uint8_t*)P[k].send + so, sb, ncclUint8, q, c->nccl, c->stream);
          if (r != ncclSuccess) { R.group_end(); return dk_fail(std::string("RCCL error: ") + R.error_string(r) + " in ncclSend"); }
        }
        if (rb) {
          ncclResult_t r = R.recv((uint8_t*)P[k].recv + ro, rb, ncclUint8, q, c->nccl, c->stream);
          if (r != ncclSuccess) { R.group_end(); return dk_fail(std::string("RCCL error: ") + R.error_string(r) + " in ncclRecv"); }
        }
      }
      so += sb;
      ro += rb;
    }
  }
  CNCCL(R.group_end());
  CHIP(hipStreamSynchronize(c->stream));
  return 0;
}

int local_a2a(dk_comm* c, const Plane* P, int np, bool device) {
  Hub& H = *c->hub;
  const int W = c->world;
  for (int k = 0; k < np; k++) {
    H.post[c->rank] = Hub::Post{(const uint8_t*)P[k].send, P[k].sbytes, (uint8_t*)P[k].recv, P[k].rbytes, nullptr};
    H.barrier();
    // pull this rank's run from every source
    int err = 0;
    int64_t ro = 0;
    for (int s = 0; s < W; s++) {
      const Hub::Post& src = H.post[s];
      int64_t so = 0;
      for (int q = 0; q < c->rank; q++) so += src.sbytes[q];
      const int64_t n = src.sbytes[c->rank];
      if (n != P[k].rbytes[s]) err = dk_fail("dk_comm: send / receive sizes disagree between ranks");
      else if (n) {
        if (device) {                          // on this rank's copy stream (a hipMemcpy between device
                                               // buffers may return before the copy has landed)
          if (hipMemcpyAsync((uint8_t*)P[k].recv + ro, src.send + so, n, hipMemcpyDefault, c->stream) != hipSuccess)
            err = dk_fail("dk_comm: local all-to-all copy failed");
        } else {
          memcpy((uint8_t*)P[k].recv + ro, src.send + so, n);
        }
      }
      ro += P[k].rbytes[s];
    }
    if (device && hipStreamSynchronize(c->stream) != hipSuccess && !err) err = dk_fail("dk_comm: local copy failed");
    H.barrier();                              // every source buffer stays valid until all have pulled
    if (err) return err;
  }
  return 0;
}

// the communicator's own stream for its device copies (created on first use)
int comm_stream(dk_comm* c) {
  if (c->stream) return 0;
  CHIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  return 0;
}

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

int comm_a2a_(dk_comm* c, const Plane* P, int np, bool device);
// all-to-all of the planes; `device`: where the caller's buffers live
int comm_a2a(dk_comm* c, const Plane* P, int np, bool device) {
  const auto t = Clock::now();
  const int rc = comm_a2a_(c, P, np, device);
  c->ms[7] += ms_since(t);
  c->n_coll++;
  return rc;
}
int comm_a2a_(dk_comm* c, const Plane* P, int np, bool device) {
  const int W = c->world;
  for (int k = 0; k < np; k++) c->bytes_sent += total(P[k].sbytes, W) - P[k].sbytes[c->rank];
  if (c->kind == dk_comm::LOCAL) return (device && comm_stream(c)) ? 1 : local_a2a(c, P, np, device);
  const bool tdev = c->transport_on_device();
  std::vector<Plane> T(P, P + np);
  std::vector<int64_t> soff(np + 1, 0), roff(np + 1, 0);
  if (device != tdev) {                        // stage every plane through the transport's memory
    for (int k = 0; k < np; k++) {
      soff[k + 1] = soff[k] + total(P[k].sbytes, W);
      roff[k + 1] = roff[k] + total(P[k].rbytes, W);
    }
    void *ss, *rs;
    if (c->stage_send.get(soff[np], tdev, &ss) || c->stage_recv.get(roff[np], tdev, &rs)) return 1;
    if (comm_stream(c)) return 1;
    for (int k = 0; k < np; k++) {
      const int64_t n = soff[k + 1] - soff[k];
      if (n) CHIP(hipMemcpyAsync((uint8_t*)ss + soff[k], P[k].send, n, tdev ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost,
                                 c->stream));
      T[k].send = (uint8_t*)ss + soff[k];
      T[k].recv = (uint8_t*)rs + roff[k];
    }
    CHIP(hipStreamSynchronize(c->stream));
  }
  int rc = 0;
  if (c->kind == dk_comm::RCCL) {
    rc = rccl_a2a(c, T.data(), np);
  } else {
    for (int k = 0; k < np && !rc; k++)
      if (c->cb.alltoallv(c->cb.user, T[k].send, T[k].sbytes, T[k].recv, T[k].rbytes))
        rc = dk_fail("dk_comm: the all-to-all callback failed");
  }
  if (rc) return rc;
  if (device != tdev) {
    for (int k = 0; k < np; k++) {
      const int64_t n = roff[k + 1] - roff[k];
      if (n) CHIP(hipMemcpyAsync(P[k].recv, T[k].recv, n, tdev ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice, c->stream));
    }
    CHIP(hipStreamSynchronize(c->stream));
  }
  return 0;
}

// every rank sends k int64 to every peer (host memory): send[p * k + j] -> recv[p * k + j] from rank p
int comm_a2a_small(dk_comm* c, const int64_t* send, int64_t* recv, int k) {
  const int W = c->world;
  std::vector<int64_t> b(W, 8 * (int64_t)k);
  Plane P{send, b.data(), recv, b.data()};
  const int64_t before = c->bytes_sent;
  int rc = comm_a2a(c, &P, 1, false);
  c->bytes_sent = before;                      // (control traffic is not counted)
  return rc;
}

int comm_allreduce_(dk_comm* c, int64_t* vals, int n, int op);
int comm_allreduce(dk_comm* c, int64_t* vals, int n, int op) {
  const auto t = Clock::now();
  const int rc = comm_allreduce_(c, vals, n, op);
  c->ms[7] += ms_since(t);
  c->n_coll++;
  return rc;
}
int comm_allreduce_(dk_comm* c, int64_t* vals, int n, int op) {
  if (n <= 0) return 0;
  if (op != 0 && op != 1) return dk_fail("dk_comm_allreduce_i64: op must be 0 (sum) or 1 (max)");
  switch (c->kind) {
    case dk_comm::CALLBACKS:
      return c->cb.allreduce_i64(c->cb.user, vals, n, op) ? dk_fail("dk_comm: the all-reduce callback failed") : 0;
    case dk_comm::LOCAL: {
      Hub& H = *c->hub;
      std::vector<int64_t> mine(vals, vals + n);
      H.post[c->rank] = Hub::Post{nullptr, nullptr, nullptr, nullptr, mine.data()};
      H.barrier();
      for (int i = 0; i < n; i++) {
        int64_t v = H.post[0].vals[i];
        for (int s = 1; s < c->world; s++) v = op == 0 ? v + H.post[s].vals[i] : std::max(v, H.post[s].vals[i]);
        vals[i] = v;
      }
      H.barrier();
      return 0;
    }
    case dk_comm::RCCL: {
      void* d;
      if (c->small.get((size_t)n * 8, true, &d)) return 1;
      CHIP(hipMemcpyAsync(d, vals, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
      CNCCL(rccl().all_reduce(d, d, n, ncclInt64, op == 0 ? ncclSum : ncclMax, c->nccl, c->stream));
      CHIP(hipMemcpyAsync(vals, d, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
      CHIP(hipStreamSynchronize(c->stream));
      return 0;
    }
  }
  return dk_fail("dk_comm: bad communicator");
}

// ---- the protocol's side: the device replay, or a caller's stand-in (dk_owner_side) -----------
struct Side {
  const dk_owner_side* cs = nullptr;
  dk_replay* r = nullptr;
  double* acc = nullptr;                        // the phase's local-step time (ms)
  double* steps = nullptr;                      // per-step times (dk_owner_side member order)
  std::mutex* serial = nullptr;                 // one rank's local step at a time (local transport)
  bool device() const { return r != nullptr || (cs && cs->device_buffers); }
  // every local step timed (and, with a serial lock, run alone on the device)
  struct Timed {
    const Side& s;
    int k;
    Clock::time_point t;
    std::unique_lock<std::mutex> lk;
    // serial (rehearsals: every rank in one process on one GPU): the step runs alone -- the device
    // drained of the other ranks' work before it, its own work finished inside its time
    // (the step's own stream is drained inside its time; work it queued on other streams -- the
    // add.size mirror, which overlaps the exchanges on a rank's own GPU -- before the next step)
    Timed(const Side& s_, int k_) : s(s_), k(k_) {
      if (s.serial) { lk = std::unique_lock<std::mutex>(*s.serial); hipDeviceSynchronize(); }
      t = Clock::now();
    }
    ~Timed() {
      if (s.serial && s.r) hipStreamSynchronize(dk::replay_stream(s.r));
      const double d = ms_since(t);
      if (s.acc) *s.acc += d;
      if (s.steps) s.steps[k] += d;
    }
  };
  enum { S_BEGIN, S_TAIL_COUNTS, S_TAIL_PACK, S_TAIL_RESOLVE, S_RESEED, S_TAIL_FINISH, S_RUN, S_CKPT_COUNTS,
         S_CKPT_PACK, S_CKPT_LOOKUP, S_CKPT_APPLY, S_CAND_COUNTS, S_CAND_PACK, S_CAND_VERIFY, S_CAND_FINISH };
#define CALL(name, K, ...) (Timed(*this, K), r ? dk_replay_owner_##name(r, ##__VA_ARGS__) : cs->name(cs->user, ##__VA_ARGS__))
  int begin() { Timed tm(*this, S_BEGIN); return r ? dk_replay_owner_begin(r) : cs->begin(cs->user); }
  int tail_counts(int64_t* recs, int64_t* bytes) { return CALL(tail_counts, S_TAIL_COUNTS, recs, bytes); }
  int tail_pack(void* recs, void* keys) { return CALL(tail_pack, S_TAIL_PACK, recs, keys); }
  int tail_resolve(const void* recs, int64_t n, const void* keys, int64_t nb, uint8_t* ans, int32_t* flags) {
    return CALL(tail_resolve, S_TAIL_RESOLVE, recs, n, keys, nb, ans, flags);
  }
  int reseed() { Timed tm(*this, S_RESEED); return r ? dk_replay_owner_reseed(r) : cs->reseed(cs->user); }
  int tail_finish(const uint8_t* back) { return CALL(tail_finish, S_TAIL_FINISH, back); }
  int run() { Timed tm(*this, S_RUN); return r ? dk_replay_run(r) : cs->run(cs->user); }
  int ckpt_counts(int64_t* c) { return CALL(ckpt_counts, S_CKPT_COUNTS, c); }
  int ckpt_pack(uint64_t* send) { return CALL(ckpt_pack, S_CKPT_PACK, send); }
  int ckpt_lookup(const uint64_t* recv, int64_t n, uint8_t* flags) { return CALL(ckpt_lookup, S_CKPT_LOOKUP, recv, n, flags); }
  int ckpt_apply(const uint8_t* back) { return CALL(ckpt_apply, S_CKPT_APPLY, back); }
  int cand_counts(int64_t* recs, int64_t* bytes) { return CALL(cand_counts, S_CAND_COUNTS, recs, bytes); }
  int cand_pack(void* recs, void* keys) { return CALL(cand_pack, S_CAND_PACK, recs, keys); }
  int cand_verify(const void* recs, int64_t n, const void* keys, int64_t nb, uint8_t* ans) {
    return CALL(cand_verify, S_CAND_VERIFY, recs, n, keys, nb, ans);
  }
  int cand_finish(const uint8_t* back) { return CALL(cand_finish, S_CAND_FINISH, back); }
#undef CALL
};

// A step's local error: its message is kept (the collectives after it may overwrite the thread's
// error text) and reported once every rank has voted.
struct StepErr {
  bool set = false;
  std::string msg;
  void take(int rc) {
    if (rc && !set) { set = true; msg = dk_last_error(); if (msg.empty()) msg = "owner exchange: local step failed"; }
  }
};

// after a vote: 0 = go on; else the status to return (1 local error, DK_STATUS_PEER a peer's)
int vote_outcome(const StepErr& e, int64_t votes) {
  if (!(votes & kErrBit)) return 0;
  if (e.set) return dk_fail(e.msg);
  dk_fail("owner exchange: another rank failed");
  return DK_STATUS_PEER;
}

int run_protocol(Side& S, dk_comm* c) {
  const int W = c->world;
  const bool dev = S.device();
  if (c->device >= 0) CHIP(hipSetDevice(c->device));
  c->bytes_sent = 0;
  c->n_coll = 0;
  for (double& m : c->ms) m = 0;
  for (double& m : c->step_ms) m = 0;
  S.steps = c->step_ms;
  static const bool serial = getenv("DK_LOCAL_SERIAL") && atoi(getenv("DK_LOCAL_SERIAL")) != 0;
  if (c->kind == dk_comm::LOCAL && serial) S.serial = &c->hub->side_mu;
  S.acc = &c->ms[4];
  const auto t0 = Clock::now();
  std::vector<int64_t> sv(3 * W), rv(3 * W);
  std::vector<int64_t> rc(W), bc(W), rrc(W), rbc(W), zero(W, 0), ones(W);
  void *recs = nullptr, *keys = nullptr, *rrecs = nullptr, *rkeys = nullptr, *ans = nullptr, *back = nullptr;
  auto peers_failed = [&](int k) {                 // a vote carried by a counts exchange
    int64_t v = 0;
    for (int p = 0; p < W; p++) v |= rv[p * k];
    return v;
  };

  // ---- 1. commit-tail key records to their owners, resolved there, answers back
  bool first = true;
  StepErr carry;                                   // a failed reseed: voted at the next round's counts
  for (;;) {
    StepErr e = carry;
    carry = StepErr();
    if (first) { e.take(S.begin()); first = false; }
    if (!e.set) e.take(S.tail_counts(rc.data(), bc.data()));
    if (!e.set) {
      int64_t nr = 0, nb = 0;
      for (int p = 0; p < W; p++) { nr += rc[p]; nb += bc[p]; }
      if (c->b_recs.get(nr * kRecBytes, dev, &recs) || c->b_keys.get(nb, dev, &keys)) e.take(1);
      else e.take(S.tail_pack(recs, keys));
    }
    for (int p = 0; p < W; p++) {
      sv[3 * p] = e.set ? kErrBit : 0;
      sv[3 * p + 1] = e.set ? 0 : rc[p] * kRecBytes;
      sv[3 * p + 2] = e.set ? 0 : bc[p];
    }
    if (comm_a2a_small(c, sv.data(), rv.data(), 3)) return 1;
    if (int st = vote_outcome(e, peers_failed(3))) return st;
    std::vector<int64_t> sr(W), rr(W);
    for (int p = 0; p < W; p++) { sr[p] = rc[p] * kRecBytes; rr[p] = rv[3 * p + 1]; rrc[p] = rv[3 * p + 1]; rbc[p] = rv[3 * p + 2]; }
    const int64_t nrr = total(rrc.data(), W), nrb = total(rbc.data(), W);
    if (c->b_rrecs.get(nrr, dev, &rrecs) || c->b_rkeys.get(nrb, dev, &rkeys)) return 1;
    Plane P[2] = {{recs, sr.data(), rrecs, rrc.data()}, {keys, bc.data(), rkeys, rbc.data()}};
    if (comm_a2a(c, P, 2, dev)) return 1;
    StepErr e2;
    int32_t flag = 0;
    const int64_t n_in = nrr / kRecBytes;
    if (c->b_ans.get(n_in, dev, &ans)) e2.take(1);
    else e2.take(S.tail_resolve(rrecs, n_in, rkeys, nrb, (uint8_t*)ans, &flag));
    int64_t vote = e2.set ? kErrBit : (int64_t)(flag & kCollision);
    if (comm_allreduce(c, &vote, 1, 1)) return 1;
    if (int st = vote_outcome(e2, vote)) return st;
    if (vote & kCollision) {                        // a collision at some owner: every rank reseeds
      carry.take(S.reseed());
      continue;
    }
    std::vector<int64_t> a_s(W), a_r(W);
    for (int p = 0; p < W; p++) { a_s[p] = rrc[p] / kRecBytes; a_r[p] = rc[p]; }
    if (c->b_back.get(total(a_r.data(), W), dev, &back)) return 1;
    Plane A{ans, a_s.data(), back, a_r.data()};
    if (comm_a2a(c, &A, 1, dev)) return 1;
    break;
  }
  c->ms[0] = ms_since(t0);
  const auto t1 = Clock::now();
  S.acc = &c->ms[5];

  // ---- 2. every checkpoint row's key hash to its owner; rows no owned tail key hashes to decide there
  void *cks = nullptr, *ckr = nullptr, *flags = nullptr, *ckb = nullptr;
  std::vector<int64_t> cc(W), ccb(W), rcb(W);
  StepErr e;
  e.take(S.tail_finish((const uint8_t*)back));
  if (!e.set) e.take(S.run());
  if (!e.set) e.take(S.ckpt_counts(cc.data()));
  if (!e.set) {
    if (c->b_cksend.get(total(cc.data(), W) * 8, dev, &cks)) e.take(1);
    else e.take(S.ckpt_pack((uint64_t*)cks));
  }
  c->ms[1] = ms_since(t1);
  const auto t2 = Clock::now();
  S.acc = &c->ms[6];
  for (int p = 0; p < W; p++) {
    sv[2 * p] = e.set ? kErrBit : 0;
    sv[2 * p + 1] = e.set ? 0 : cc[p] * 8;
  }
  if (comm_a2a_small(c, sv.data(), rv.data(), 2)) return 1;
  if (int st = vote_outcome(e, peers_failed(2))) return st;
  for (int p = 0; p < W; p++) { ccb[p] = cc[p] * 8; rcb[p] = rv[2 * p + 1]; }
  const int64_t n_rows_in = total(rcb.data(), W) / 8;
  if (c->b_ckrecv.get(n_rows_in * 8, dev, &ckr)) return 1;
  {
    Plane P{cks, ccb.data(), ckr, rcb.data()};
    if (comm_a2a(c, &P, 1, dev)) return 1;
  }
  // the owner's lookup; a failure here is voted with the candidate counts below (the answers it
  // sends back are then never used: every rank returns the error)
  StepErr el;
  if (c->b_flags.get(n_rows_in, dev, &flags)) el.take(1);
  else el.take(S.ckpt_lookup((const uint64_t*)ckr, n_rows_in, (uint8_t*)flags));
  {
    std::vector<int64_t> f_s(W), f_r(W);
    for (int p = 0; p < W; p++) { f_s[p] = rcb[p] / 8; f_r[p] = cc[p]; }
    if (c->b_ckback.get(total(f_r.data(), W), dev, &ckb)) return 1;
    Plane P{flags, f_s.data(), ckb, f_r.data()};
    if (comm_a2a(c, &P, 1, dev)) return 1;
  }

  // ---- 3. candidates (rows whose hash some owned tail key has) verified byte-exactly by the owner
  StepErr e3 = el;
  if (!e3.set) e3.take(S.ckpt_apply((const uint8_t*)ckb));
  std::vector<int64_t> cr(W), cb(W), crr(W), cbr(W);
  if (!e3.set) e3.take(S.cand_counts(cr.data(), cb.data()));
  if (!e3.set) {
    if (c->b_recs.get(total(cr.data(), W) * kRecBytes, dev, &recs) || c->b_keys.get(total(cb.data(), W), dev, &keys)) e3.take(1);
    else e3.take(S.cand_pack(recs, keys));
  }
  for (int p = 0; p < W; p++) {
    sv[3 * p] = e3.set ? kErrBit : 0;
    sv[3 * p + 1] = e3.set ? 0 : cr[p] * kRecBytes;
    sv[3 * p + 2] = e3.set ? 0 : cb[p];
  }
  if (comm_a2a_small(c, sv.data(), rv.data(), 3)) return 1;
  if (int st = vote_outcome(e3, peers_failed(3))) return st;
  std::vector<int64_t> crb(W);
  for (int p = 0; p < W; p++) { crb[p] = cr[p] * kRecBytes; crr[p] = rv[3 * p + 1]; cbr[p] = rv[3 * p + 2]; }
  const int64_t n_cand_in = total(crr.data(), W) / kRecBytes, n_cand_bytes = total(cbr.data(), W);
  if (c->b_rrecs.get(n_cand_in * kRecBytes, dev, &rrecs) || c->b_rkeys.get(n_cand_bytes, dev, &rkeys)) return 1;
  {
    Plane P[2] = {{recs, crb.data(), rrecs, crr.data()}, {keys, cb.data(), rkeys, cbr.data()}};
    if (comm_a2a(c, P, 2, dev)) return 1;
  }
  StepErr e4;
  if (c->b_ans.get(n_cand_in, dev, &ans)) e4.take(1);
  else e4.take(S.cand_verify(rrecs, n_cand_in, rkeys, n_cand_bytes, (uint8_t*)ans));
  {
    std::vector<int64_t> v_s(W), v_r(W);
    for (int p = 0; p < W; p++) { v_s[p] = crr[p] / kRecBytes; v_r[p] = cr[p]; }
    if (c->b_back.get(total(v_r.data(), W), dev, &back)) return 1;
    Plane P{ans, v_s.data(), back, v_r.data()};
    if (comm_a2a(c, &P, 1, dev)) return 1;
  }
  if (!e4.set) e4.take(S.cand_finish((const uint8_t*)back));
  int64_t vote = e4.set ? kErrBit : 0;
  if (comm_allreduce(c, &vote, 1, 1)) return 1;
  if (int st = vote_outcome(e4, vote)) return st;
  c->ms[2] = ms_since(t2);
  c->ms[3] = ms_since(t0);
  return 0;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" int dk_comm_unique_id(uint8_t id[DK_COMM_ID_BYTES]) {
  const Rccl& R = rccl();
  if (!R.error.empty()) return dk_fail("dk_comm_unique_id: " + R.error);
  ncclUniqueId u;
  CNCCL(R.get_unique_id(&u));
  static_assert(sizeof(u) == DK_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof u);
  return 0;
}

extern "C" int dk_comm_create(const uint8_t id[DK_COMM_ID_BYTES], int32_t world, int32_t rank, int32_t device,
                              dk_comm** out) {
  if (!out) return dk_fail("dk_comm_create: null out");
  *out = nullptr;
  if (world < 1 || world > 64 || rank < 0 || rank >= world) return dk_fail("dk_comm_create: bad world / rank");
  const Rccl& R = rccl();
  if (!R.error.empty()) return dk_fail("dk_comm_create: " + R.error);
  CHIP(hipSetDevice(device));
  std::unique_ptr<dk_comm> c(new dk_comm());
  c->kind = dk_comm::RCCL;
  c->world = world; c->rank = rank; c->device = device;
  CHIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclResult_t r = R.init_rank(&c->nccl, world, u, rank);
  if (r != ncclSuccess) {
    hipStreamDestroy(c->stream);
    return dk_fail(std::string("dk_comm_create: ncclCommInitRank: ") + R.error_string(r));
  }
  *out = c.release();
  return 0;
}

extern "C" int dk_comm_create_callbacks(const dk_comm_callbacks* cb, int32_t world, int32_t rank, dk_comm** out) {
  if (!out) return dk_fail("dk_comm_create_callbacks: null out");
  *out = nullptr;
  if (!cb || !cb->alltoallv || !cb->allreduce_i64) return dk_fail("dk_comm_create_callbacks: missing callback");
  if (world < 1 || world > 64 || rank < 0 || rank >= world) return dk_fail("dk_comm_create_callbacks: bad world / rank");
  auto* c = new dk_comm();
  c->kind = dk_comm::CALLBACKS;
  c->world = world; c->rank = rank;
  c->cb = *cb;
  *out = c;
  return 0;
}

extern "C" int dk_comm_create_local(int32_t world, int32_t on_device, dk_comm** comms) {
  if (!comms) return dk_fail("dk_comm_create_local: null out");
  if (world < 1 || world > 64) return dk_fail("dk_comm_create_local: bad world");
  int dev = -1;
  if (on_device) CHIP(hipGetDevice(&dev));
  auto hub = std::make_shared<Hub>(world);
  for (int r = 0; r < world; r++) {
    auto* c = new dk_comm();
    c->kind = dk_comm::LOCAL;
    c->world = world; c->rank = r; c->device = dev;
    c->hub = hub;
    c->local_device = on_device != 0;
    comms[r] = c;
  }
  return 0;
}

extern "C" int32_t dk_comm_world(const dk_comm* c) { return c ? c->world : -1; }
extern "C" int32_t dk_comm_rank(const dk_comm* c) { return c ? c->rank : -1; }

extern "C" int dk_comm_allreduce_i64(dk_comm* c, int64_t* vals, int32_t n, int32_t op) {
  if (!c) return dk_fail("dk_comm_allreduce_i64: null communicator");
  if (c->device >= 0) CHIP(hipSetDevice(c->device));
  return comm_allreduce(c, vals, n, op);
}

extern "C" int dk_comm_alltoallv(dk_comm* c, const void* send, const int64_t* send_bytes, void* recv,
                                 const int64_t* recv_bytes, int32_t on_device) {
  if (!c) return dk_fail("dk_comm_alltoallv: null communicator");
  if (c->device >= 0) CHIP(hipSetDevice(c->device));
  for (int p = 0; p < c->world; p++)
    if (send_bytes[p] < 0 || recv_bytes[p] < 0) return dk_fail("dk_comm_alltoallv: negative size");
  Plane P{send, send_bytes, recv, recv_bytes};
  return comm_a2a(c, &P, 1, on_device != 0);
}

extern "C" int dk_comm_abort(dk_comm* c) {
  // the failing rank's answer to the owner run's first vote (its tail counts exchange)
  if (!c) return dk_fail("dk_comm_abort: null communicator");
  if (c->device >= 0) CHIP(hipSetDevice(c->device));
  std::vector<int64_t> sv(3 * c->world, 0), rv(3 * c->world);
  for (int p = 0; p < c->world; p++) sv[3 * p] = kErrBit;
  return comm_a2a_small(c, sv.data(), rv.data(), 3);
}

extern "C" int dk_comm_last_run(const dk_comm* c, double ms[8], int64_t* bytes_sent, int64_t* collectives) {
  if (!c) return dk_fail("dk_comm_last_run: null communicator");
  if (ms) for (int i = 0; i < 8; i++) ms[i] = c->ms[i];
  if (bytes_sent) *bytes_sent = c->bytes_sent;
  if (collectives) *collectives = c->n_coll;
  return 0;
}

extern "C" int dk_comm_last_steps(const dk_comm* c, double ms[16]) {
  if (!c) return dk_fail("dk_comm_last_steps: null communicator");
  for (int i = 0; i < 16; i++) ms[i] = c->step_ms[i];
  return 0;
}

extern "C" void dk_comm_destroy(dk_comm* c) {
  if (!c) return;
  if (c->device >= 0) hipSetDevice(c->device);
  if (c->kind == dk_comm::RCCL && c->nccl) rccl().destroy(c->nccl);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

extern "C" int dk_owner_protocol_run(const dk_owner_side* side, dk_comm* c) {
  if (!side || !c) return dk_fail("dk_owner_protocol_run: null argument");
  Side S;
  S.cs = side;
  return run_protocol(S, c);
}

extern "C" int dk_replay_owner_run(dk_replay* r, dk_comm* c) {
  if (!r || !c) return dk_fail("dk_replay_owner_run: null argument");
  Side S;
  S.r = r;
  return run_protocol(S, c);
}
