// Host side of libdkgpu: file open (footer + offset index), page enumeration, device buffers,
// kernel orchestration on one HIP stream, commit-tail JSON parsing, C ABI (include/dkgpu.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <thread>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <string>
#include <string_view>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "../../include/dkgpu.h"
#include "dk_device.h"
#include "dk_thrift.h"
#include "dk_uri.h"
#include "dk_expr.h"

namespace dk {
void launch_page_headers(const DChunk*, DPage*, int, hipStream_t);
void launch_snappy(const SnapCtx&, int, int, const int2*, int, hipStream_t);
void snap_stats(unsigned long long*);
void launch_pack_bits(const uint8_t*, long long, uint8_t*, hipStream_t);
void launch_expand(const int64_t*, const int32_t*, int, int, void*, hipStream_t);
void launch_copy_zc(void*, const void*, long long, hipStream_t);
void launch_arrow_window(const ArrowWin&, hipStream_t);
void launch_dv_expand(const DvCont*, int, const uint8_t*, unsigned long long*, hipStream_t);
void launch_dv_select(const unsigned long long*, long long, const long long*, long long, uint8_t*, hipStream_t);
void launch_positions(const DChunk*, DPage*, int, int, const uint8_t*, int32_t*, DPosChunk*, int, int, int16_t*, hipStream_t);
void launch_page_runs(const DChunk*, DPage*, int, const uint8_t*, Seg*, hipStream_t);
void launch_tile_count(const DChunk*, DPage*, const uint8_t*, const Seg*, DTile*, int, int, hipStream_t);
void launch_tile_scan1(DColumn*, int, DPage*, DTile*, DState*, hipStream_t);
void launch_tile_chars(const DChunk*, DPage*, const uint8_t*, const int32_t*, const Seg*, DTile*, int, int, hipStream_t);
void launch_tile_scan2(DColumn*, int, DPage*, DTile*, DState*, hipStream_t);
void launch_tile_decode(const DChunk*, DPage*, const DColumn*, const uint8_t*, const int32_t*, const long long*, const Seg*, const DTile*, int, int, DState*, hipStream_t);
void launch_delta_decode(const DChunk*, DPage*, int, const uint8_t*, long long*, hipStream_t);
void launch_string_copy(const DChunk*, const DPage*, int, const DColumn*, const uint8_t*, const int32_t*, const int2*, hipStream_t,
                        int, int);
void launch_json_canon(DJsonAction*, int, const uint8_t*, uint8_t*, uint32_t, DState*, hipStream_t);
void launch_slots_init(Slot*, uint64_t, hipStream_t);
void launch_table_insert(const DJsonAction*, int, Slot*, uint64_t, hipStream_t);
void launch_first_row(const uint8_t*, long long, int, unsigned long long*, hipStream_t);
void launch_table_update(DJsonAction*, int, Slot*, uint64_t, const uint8_t*, DState*, hipStream_t);
void launch_json_select(const DJsonAction*, int, const Slot*, uint64_t, const uint8_t*, uint8_t*, DState*, hipStream_t);
void launch_stats_eval(const StatsRows&, const DSkipProg&, const SkScratch&, uint8_t*, DState*, hipStream_t);
void launch_stats_parsed(const StatsParsedRows&, const DSkipProg&, const SkScratch&, uint8_t*, DState*, hipStream_t);
void launch_part_eval(const MapRows&, const DPartProg&, uint8_t*, DState*, hipStream_t);
void launch_table_fp(const Slot*, uint32_t*, uint64_t, hipStream_t);
void launch_probe_all(const ProbeSet&, const Slot*, const uint32_t*, uint64_t, const DJsonAction*, const uint8_t*, uint32_t, uint64_t,
                      int32_t*, unsigned int*, DState*, hipStream_t);
int a2a_blocks(long long, long long*);
void launch_a2a_count(const ProbeSet&, int, unsigned long long*, unsigned long long*, hipStream_t);
void launch_a2a_pack(const ProbeSet&, int, const unsigned long long*, uint64_t*, int32_t*, int32_t*, unsigned int*, DState*,
                     hipStream_t);
void launch_a2a_filter(const uint64_t*, long long, const uint64_t*, long long, uint8_t*, hipStream_t);
void launch_a2a_apply(const ProbeSet&, const int32_t*, const uint8_t*, long long, const Slot*, uint64_t, const DJsonAction*,
                      const uint8_t*, uint32_t, int32_t*, unsigned int*, DState*, hipStream_t);
void launch_probe(const ProbeCols&, const Slot*, const uint32_t*, uint64_t, const DJsonAction*, const uint8_t*, uint32_t, uint64_t,
                  uint8_t*, int32_t*, unsigned int*, DState*, hipStream_t);
void launch_own_rowhash(const ProbeSet&, uint64_t*, uint32_t, uint64_t, DState*, hipStream_t);
void launch_own_count(const ProbeSet&, const uint64_t*, int, unsigned long long*, unsigned long long*, hipStream_t);
void launch_own_pack(const ProbeSet&, const uint64_t*, int, const unsigned long long*, uint64_t*, int32_t*, hipStream_t);
void launch_own_lookup(const uint64_t*, long long, const Slot*, const uint32_t*, uint64_t, uint8_t*, hipStream_t);
void launch_own_tail_count(const DJsonAction*, int, int, unsigned long long*, hipStream_t);
void launch_own_tail_pack(const DJsonAction*, int, int, const unsigned long long*, const uint8_t*, OwnerKeyRec*, uint8_t*,
                          int32_t*, hipStream_t);
void launch_own_tail_finish(const int32_t*, const uint8_t*, long long, uint8_t*, hipStream_t);
int own_recs_blocks(long long, long long*);
void launch_own_recs_acts(const OwnerKeyRec*, long long, long long, unsigned long long*, int*, unsigned long long*,
                          DJsonAction*, hipStream_t);
void launch_own_apply(const ProbeSet&, const int32_t*, const uint8_t*, long long, int32_t*, unsigned int*, DState*, hipStream_t);
void launch_own_cand_len(const ProbeSet&, const int32_t*, long long, const uint64_t*, int, int32_t*, int32_t*, int32_t*,
                         hipStream_t);
void launch_own_cand_keys(const ProbeSet&, const int32_t*, long long, const uint64_t*, const int64_t*, const int64_t*,
                          const int32_t*, const int32_t*, OwnerKeyRec*, uint8_t*, hipStream_t);
void launch_own_verify(const OwnerKeyRec*, long long, const int64_t*, const uint8_t*, const Slot*, uint64_t,
                       const DJsonAction*, const uint8_t*, uint8_t*, hipStream_t);
void launch_own_cand_finish(const ProbeSet&, const int32_t*, const uint8_t*, long long, DState*, hipStream_t);
int warm_kernels();
void launch_json_parse_stats(const uint8_t*, const int64_t*, const uint8_t*, const uint8_t*, long long, const DSkipProg&,
                             const SkScratch&, long long*, uint32_t*, DState*, hipStream_t);
void launch_parsed_eval(const uint8_t*, const int64_t*, long long, const DSkipProg&, long long*, uint32_t*,
                        uint8_t*, hipStream_t);
}  // namespace dk

using namespace dk;

static thread_local std::string g_err;
static int fail(const std::string& m) { g_err = m; return 1; }
namespace dk { int dk_fail(const std::string& m) { return fail(m); } }

#define HIPOK(x)                                                                              \
  do {                                                                                        \
    hipError_t _e = (x);                                                                      \
    if (_e != hipSuccess) return fail(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #x); \
  } while (0)

extern "C" const char* dk_last_error(void) { return g_err.c_str(); }
extern "C" const char* dk_version(void) { return "libdkgpu 0.2 (gfx950)"; }
// debug: k_snap_frag counters (non-zero only in DK_SNAP_STATS builds; tools/snap_stats.py)
extern "C" int dk_debug_snap_stats(int64_t out[24]) { snap_stats((unsigned long long*)out); return 0; }

// ------------------------------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------------------------------
// The engine holds configuration only; every call object owns its stream, so one engine can be used
// from several threads at once (each reader / replay stays single-threaded, like Kernel iterators).
struct dk_engine {
  dk_config cfg;
};

static int engine_warm(int device);
extern "C" int dk_engine_create(const dk_config* cfg, dk_engine** out) {
  dk_config c = cfg ? *cfg : dk_config{1024, 1024, 0, 0};
  if (c.parquet_batch_size <= 0) c.parquet_batch_size = 1024;
  if (c.json_batch_size <= 0) return fail("invalid JSON reader batch size: " + std::to_string(c.json_batch_size));
  {  // the compile-time fast-path character set must agree with the URI character classes
    for (uint32_t ch = 0; ch < 256; ch++)
      if (simple8(0x6161616161616100ull | ch) != (ch > 0 && ch < 128 && (uri_class((uint8_t)ch) & CC_SIMPLE) != 0))
        return fail("libdkgpu: internal error: SimpleSet disagrees with uri_class");
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail("libdkgpu: no HIP device available (the GPU engine has no CPU fallback)");
  if (c.device < 0 || c.device >= ndev) return fail("libdkgpu: bad device ordinal");
  HIPOK(hipSetDevice(c.device));
  if (engine_warm(c.device)) return 1;
  auto* e = new dk_engine();
  e->cfg = c;
  *out = e;
  return 0;
}

static void reaper_drain_all();
extern "C" void dk_engine_destroy(dk_engine* e) {
  if (!e) return;
  reaper_drain_all();
  hipSetDevice(e->cfg.device);
  delete e;
}

// ------------------------------------------------------------------------------------------------
// device buffer helper
// ------------------------------------------------------------------------------------------------
// Process-wide block caches for device memory (hipMalloc) and pinned host memory (hipHostMalloc),
// per device. A getScanFiles allocates tens of GB (decoded-column arena, snappy arena, file images,
// pinned host staging); the next scan on the same table asks for the same sizes, so released blocks
// are kept and handed out again instead of being unmapped and re-mapped (hipHostMalloc pins page by
// page: ~90 ms for a 90 MB file image; hipFree synchronises the device). Sizes are rounded to a
// geometric grid (8 classes per doubling, <= 12.5 % slack) so near sizes share blocks.
//
// A released block may still be read or written by work queued on its owner's stream. Owners
// release inside a SyncedRelease scope once their stream is drained (object close / free), and
// those blocks are reusable at once; any other release parks the block, and parked blocks are only
// reused after the cache itself drains the device (when trimming).
// Deferred release: a closed call object (dk_parquet_close, dk_json_tail_free) is deleted on a
// background thread -- host tables, events, blocks back to the caches -- so that close returns at
// once. A cache lookup that misses waits for pending releases before allocating afresh (the next
// scan's blocks are usually the ones being released), and dk_engine_destroy / process exit wait for
// all of them. Jobs are numbered: the threads of an open wait only for the jobs submitted before the
// open started (a later job may be the close that joins this very open; older ones never wait for
// it), so no wait needs a time limit.
struct Reaper {
  std::mutex mu;
  std::condition_variable cv;
  int pending = 0;
  uint64_t next_id = 0;
  std::vector<uint64_t> live;          // ids of the jobs still running
  void run(std::function<void()> f) {
    uint64_t id;
    {
      std::lock_guard<std::mutex> g(mu);
      if (pending++ == 0 && !registered) { registered = true; std::atexit([] { reaper_drain(); }); }
      id = next_id++;
      live.push_back(id);
    }
    std::thread([this, f, id] {
      f();
      std::lock_guard<std::mutex> g(mu);
      live.erase(std::find(live.begin(), live.end(), id));
      if (--pending == 0) cv.notify_all();
      else cv.notify_all();
    }).detach();
  }
  uint64_t ticket() { std::lock_guard<std::mutex> g(mu); return next_id; }
  bool oldest_below(uint64_t t) {      // (mu held) a job submitted before ticket t is still running
    for (uint64_t id : live) if (id < t) return true;
    return false;
  }
  bool busy_before(uint64_t t) { std::lock_guard<std::mutex> g(mu); return oldest_below(t); }
  void drain_before(uint64_t t) { std::unique_lock<std::mutex> lk(mu); cv.wait(lk, [&] { return !oldest_below(t); }); }
  void drain() { std::unique_lock<std::mutex> lk(mu); cv.wait(lk, [&] { return pending == 0; }); }
  bool registered = false;
  static void reaper_drain();
};
static Reaper& reaper() { static Reaper* r = new Reaper(); return *r; }
void Reaper::reaper_drain() { reaper().drain(); }
static void reaper_drain_all() { reaper().drain(); }

static thread_local int t_synced = 0;
// The reaper ticket of the open a thread works for (the opener, its image reader and their
// parallel_for workers): a cache miss there waits only for releases submitted before that open
// started. Other threads wait for every pending release (UINT64_MAX).
static thread_local uint64_t t_open_ticket = UINT64_MAX;
struct SyncedRelease {
  SyncedRelease() { t_synced++; }
  ~SyncedRelease() { t_synced--; }
};
struct MemCache {
  struct Blk { void* p; size_t n; int dev; };
  std::mutex mu;
  std::vector<Blk> idle, parked;
  size_t held = 0;                 // bytes in idle + parked
  const bool pinned;
  const size_t cap;
  const bool pageable;             // plain host memory (header images): malloc / free
  MemCache(bool pinned_, size_t cap_, bool pageable_ = false) : pinned(pinned_), cap(cap_), pageable(pageable_) {}
  static size_t round(size_t n) {
    if (n < ((size_t)1 << 20)) return (n + 4095) & ~(size_t)4095;
    int e = 63 - __builtin_clzll((unsigned long long)n);       // 2^e <= n < 2^(e+1)
    const size_t step = (size_t)1 << (e - 3);                   // 8 classes per doubling
    return (n + step - 1) & ~(step - 1);
  }
  int raw_alloc(void** p, size_t n) {
    if (pageable) return (*p = malloc(n)) ? 0 : 1;
    return pinned ? (hipHostMalloc(p, n, hipHostMallocDefault) == hipSuccess ? 0 : 1)
                  : (hipMalloc(p, n) == hipSuccess ? 0 : 1);
  }
  void raw_free(void* p) { if (pageable) free(p); else if (pinned) hipHostFree(p); else hipFree(p); }
  void* get(size_t want, size_t* got) {
    int dev = 0;
    hipGetDevice(&dev);
    const size_t n = round(want);
    {
      std::lock_guard<std::mutex> lk(mu);
      int best = -1;
      for (size_t i = 0; i < idle.size(); i++) {   // the smallest idle block of this class or up to 2 above
        const Blk& b = idle[i];
        if (b.dev == dev && b.n >= n && b.n <= n + n / 4 && (best < 0 || b.n < idle[best].n)) best = (int)i;
      }
      if (best >= 0) {
        Blk b = idle[best];
        idle[best] = idle.back();
        idle.pop_back();
        held -= b.n;
        *got = b.n;
        return b.p;
      }
    }
    static const bool verbose = getenv("DK_VERBOSE") != nullptr;
    // A deferred release may be returning just such a block (the previous scan's close); an open's
    // threads wait only for releases older than the open (its own close may be among the newer)
    if (reaper().busy_before(t_open_ticket)) {
      const auto t0 = std::chrono::steady_clock::now();
      reaper().drain_before(t_open_ticket);
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (verbose && ms > 2) fprintf(stderr, "[dk] cache %s: waited %.1f ms for pending releases\n", pinned ? "pinned" : "device", ms);
      return get(want, got);
    }
    void* p = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if (raw_alloc(&p, n)) {        // out of memory: give back every cached block of this device, retry
      trim(dev, 0);
      if (raw_alloc(&p, n)) return nullptr;
    }
    if (verbose) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms > 2) fprintf(stderr, "[dk] cache %s miss: %.1f MB allocated in %.1f ms (held %.2f GB)\n", pinned ? "pinned" : "device",
                          n / 1e6, ms, held / 1e9);
    }
    *got = n;
    return p;
  }
  void put(void* p, size_t n) {
    if (!p) return;
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    (t_synced || pageable ? idle : parked).push_back({p, n, dev});   // (no device work reads host images)
    held += n;
    if (held > cap) trim_locked(-1, cap / 2);
  }
  void trim(int dev, size_t keep) { std::lock_guard<std::mutex> lk(mu); trim_locked(dev, keep); }
  void trim_locked(int dev, size_t keep) {
    if (getenv("DK_VERBOSE"))
      fprintf(stderr, "[dk] cache %s trim: %.2f GB held, keeping %.2f GB\n", pinned ? "pinned" : "device", held / 1e9, keep / 1e9);
    hipDeviceSynchronize();
    idle.insert(idle.end(), parked.begin(), parked.end());
    parked.clear();
    // free the largest blocks first until at most `keep` bytes stay cached
    std::sort(idle.begin(), idle.end(), [](const Blk& a, const Blk& b) { return a.n > b.n; });
    for (size_t i = 0; i < idle.size() && held > keep;) {
      if (dev >= 0 && idle[i].dev != dev) { i++; continue; }
      int cur = 0;
      hipGetDevice(&cur);
      hipSetDevice(idle[i].dev);
      raw_free(idle[i].p);
      hipSetDevice(cur);
      held -= idle[i].n;
      idle.erase(idle.begin() + i);
    }
  }
};
static MemCache& dev_cache() { static MemCache* c = new MemCache(false, (size_t)96 << 30); return *c; }
static MemCache& pinned_cache() { static MemCache* c = new MemCache(true, (size_t)24 << 30); return *c; }
// header images (HostImg): kept between scans so that the page-header blocks read into them land on
// pages already faulted in (fresh pages cost ~50 ms of faults per C3 open); only touched pages are
// resident
static MemCache& pageable_cache() { static MemCache* c = new MemCache(false, (size_t)64 << 30, true); return *c; }

// Non-blocking streams are pooled per device (creating one costs milliseconds): a call object takes
// one when it is created and gives it back, drained, when it is freed.
// Three classes, each its own pool: HIP maps each stream priority to its own set of hardware queues
// (GPU_MAX_HW_QUEUES of them, 4 by default), and work on one hardware queue runs in queue order.
//  - normal: the open's sizing / decode passes, mirrors, readers;
//  - high: the replay's (commit-tail uploads and kernels, probes) and the per-slice decode, so that
//    they do not queue behind the passes an asynchronous open keeps feeding to the normal queues;
//  - copy: the H2D image copies of an open, at the lowest priority. On a queue they shared with
//    compute streams, a kernel would wait behind every image copy queued there before it (the first
//    sizing pass of an open started 23 ms after its files had landed, profiles/r04/hwq/).
enum StreamClass { kStreamNormal = 0, kStreamHigh = 1, kStreamCopy = 2 };
static bool copy_class_on() {         // DK_COPY_PRIORITY=0: image copies on normal streams (A/B)
  static const bool on = !(getenv("DK_COPY_PRIORITY") && atoi(getenv("DK_COPY_PRIORITY")) == 0);
  return on;
}
struct StreamPool {
  std::mutex mu;
  std::vector<std::pair<int, hipStream_t>> free_[3];
  hipStream_t get(int cls = kStreamNormal) {
    int dev = 0;
    hipGetDevice(&dev);
    {
      std::lock_guard<std::mutex> lk(mu);
      auto& F = free_[cls];
      for (size_t i = 0; i < F.size(); i++)
        if (F[i].first == dev) { hipStream_t s = F[i].second; F.erase(F.begin() + i); return s; }
    }
    hipStream_t s = nullptr;
    if (cls != kStreamNormal) {
      int least = 0, greatest = 0;
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
      return hipStreamCreateWithPriority(&s, hipStreamNonBlocking, cls == kStreamHigh ? greatest : least) == hipSuccess ? s : nullptr;
    }
    return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? s : nullptr;
  }
  void put(hipStream_t s, int cls = kStreamNormal) {
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    free_[cls].push_back({dev, s});
  }
};
static StreamPool& stream_pool() { static StreamPool* p = new StreamPool(); return *p; }

struct DBuf {
  void* p = nullptr;
  size_t n = 0;       // bytes asked for
  size_t cap = 0;     // bytes of the cached block
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  ~DBuf() { release(); }
  void release() { if (p) dev_cache().put(p, cap); p = nullptr; n = cap = 0; }
  int alloc(size_t bytes) {
    release();
    n = bytes;
    if (bytes == 0) return 0;
    p = dev_cache().get(bytes, &cap);
    if (!p) { n = 0; return fail("hipMalloc failed for " + std::to_string(bytes) + " bytes"); }
    return 0;
  }
  template <class T> T* as() const { return (T*)p; }
};

// A file's packed image layout in pageable host memory: the open reads only the page-header blocks
// into it (the host builds the page tables from them); the column chunks themselves go to HBM
// through the pinned staging ring (PinRing), never through here. Untouched pages cost nothing.
struct HostImg {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  HostImg() = default;
  HostImg(const HostImg&) = delete;
  HostImg& operator=(const HostImg&) = delete;
  HostImg(HostImg&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  HostImg& operator=(HostImg&& o) noexcept { if (this != &o) { release(); p = o.p; n = o.n; cap = o.cap; o.p = nullptr; o.n = o.cap = 0; } return *this; }
  ~HostImg() { release(); }
  void release() { if (p) pageable_cache().put(p, cap); p = nullptr; n = cap = 0; }
  int alloc(size_t bytes) {
    release();
    n = bytes;
    p = (uint8_t*)pageable_cache().get(bytes ? bytes : 1, &cap);
    return p ? 0 : fail("host allocation failed for " + std::to_string(bytes) + " bytes");
  }
  uint8_t* data() const { return p; }
  size_t size() const { return n; }
};

// Pinned host memory from the process-wide cache (selections and column mirrors on their way back,
// small staged uploads): DMA at full PCIe rate, no page faults on reuse.
struct HBuf {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  HBuf() = default;
  HBuf(const HBuf&) = delete;
  HBuf& operator=(const HBuf&) = delete;
  HBuf(HBuf&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  HBuf& operator=(HBuf&& o) noexcept { if (this != &o) { release(); p = o.p; n = o.n; cap = o.cap; o.p = nullptr; o.n = o.cap = 0; } return *this; }
  ~HBuf() { release(); }
  void release() { if (p) pinned_cache().put(p, cap); p = nullptr; n = cap = 0; }
  int alloc(size_t bytes) {
    release();
    n = bytes;
    if (!bytes) return 0;
    p = (uint8_t*)pinned_cache().get(bytes, &cap);
    if (!p) { n = 0; return fail("hipHostMalloc failed for " + std::to_string(bytes) + " bytes"); }
    return 0;
  }
  uint8_t* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
};

// A HIP stream owned by one call object (dk_parquet, dk_replay, dk_reader): Kernel calls
// readParquetFiles from several connector threads at once (MultiThreadedTableReader.java:244), so
// nothing of a call runs on a stream shared through the engine.
struct StreamH {
  hipStream_t s = nullptr;
  int cls = kStreamNormal;
  ~StreamH() { if (s) { hipStreamSynchronize(s); stream_pool().put(s, cls); } }
  int create(bool high_priority = false) { return create_class(high_priority ? kStreamHigh : kStreamNormal); }
  int create_class(int c) {
    cls = c;
    s = stream_pool().get(cls);
    return s ? 0 : fail("hipStreamCreate failed");
  }
};

// the replay's stream is high-priority unless DK_REPLAY_PRIORITY=0 (A/B)
static bool replay_high_priority() {
  static const bool on = !(getenv("DK_REPLAY_PRIORITY") && atoi(getenv("DK_REPLAY_PRIORITY")) == 0);
  return on;
}

// The pinned staging ring of the file images' way to HBM: DK_PINNED_MB (default 1024) MiB per device
// in slots of one H2D piece (DK_PIECE_MB, default 8 MiB), allocated once. A reader thread preads a
// piece into a free slot, queues its DMA copy to HBM and records the slot's event; the slot is reused
// once that event has fired. Pinned memory no longer grows with the table (a scan used to pin its
// whole projected image, 5.8 GB at C3) and an open never waits for the previous scan's release of it.
static int64_t piece_bytes() {
  static const int64_t piece = (int64_t)(getenv("DK_PIECE_MB") ? std::max(1, atoi(getenv("DK_PIECE_MB"))) : 8) << 20;
  return piece;
}
struct PinRing {
  struct Slot { uint8_t* p = nullptr; hipEvent_t ev = nullptr; bool used = false; };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Slot> slots;
  std::deque<int> free_;
  std::string err;
  explicit PinRing(int dev) {
    int64_t mb = getenv("DK_PINNED_MB") ? std::max(16, atoi(getenv("DK_PINNED_MB"))) : 1024;
    const int64_t sb = piece_bytes();
    int n = (int)std::max<int64_t>(4, (mb << 20) / sb);
    int cur = 0;
    hipGetDevice(&cur);
    hipSetDevice(dev);
    uint8_t* base = nullptr;
    if (hipHostMalloc((void**)&base, (size_t)n * sb, hipHostMallocDefault) != hipSuccess) {
      err = "hipHostMalloc failed for the pinned staging ring";
    } else {
      for (int i = 0; i < n; i++) {
        Slot s;
        s.p = base + (size_t)i * sb;
        if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) { err = "hipEventCreate failed"; break; }
        slots.push_back(s);
        free_.push_back(i);
      }
    }
    hipSetDevice(cur);
  }
  // a slot whose previous copy has finished (blocks while every slot is in flight)
  int acquire() {
    int i;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return !free_.empty(); });
      i = free_.front();
      free_.pop_front();
    }
    if (slots[i].used && hipEventSynchronize(slots[i].ev) != hipSuccess) { release(i, nullptr); return -1; }
    return i;
  }
  // back to the ring; its copy (queued on s) must finish before the next user writes it
  void release(int i, hipStream_t s) {
    if (s) slots[i].used = hipEventRecord(slots[i].ev, s) == hipSuccess;
    std::lock_guard<std::mutex> g(mu);
    free_.push_back(i);
    cv.notify_one();
  }
};
static PinRing* pin_ring(int dev) {
  static std::mutex mu;
  static std::vector<std::pair<int, PinRing*>> rings;
  std::lock_guard<std::mutex> g(mu);
  for (auto& r : rings) if (r.first == dev) return r.second;
  auto* r = new PinRing(dev);
  rings.push_back({dev, r});
  return r;
}

// Warm-up at engine creation (once per device and process): the code objects' lazy load, a pooled
// stream, a first launch on it, the first device / pinned blocks -- costs the first
// getLatestSnapshot would otherwise pay.
static int engine_warm(int device) {
  static std::mutex warm_mu;
  static std::vector<int> warmed;
  std::lock_guard<std::mutex> lk(warm_mu);
  if (std::find(warmed.begin(), warmed.end(), device) != warmed.end()) return 0;
  warmed.push_back(device);
  warm_kernels();
  if (!pin_ring(device)->err.empty()) return fail(pin_ring(device)->err);   // (the staging ring, once)
  // the pooled streams a checkpoint open and a replay take (own, aux, copy, side, decode; the replay's
  // two high-priority ones), each with a first launch; the DMA engines' first copies both ways
  constexpr int kWarmStreams = 12, kWarmHigh = 3;
  StreamH cp[4], sh[kWarmStreams], hi[kWarmHigh];
  for (auto& x : cp) if (x.create_class(copy_class_on() ? kStreamCopy : kStreamNormal)) return 1;
  for (auto& x : sh) if (x.create()) return 1;
  for (auto& x : hi) if (x.create(replay_high_priority())) return 1;
  DBuf d;
  HBuf h;
  if (d.alloc(1 << 20) || h.alloc(1 << 20)) return 1;
  memset(h.data(), 0, 1 << 20);
  for (auto& x : sh) launch_copy_zc(d.p, h.data(), 256, x.s);
  for (auto& x : hi) launch_copy_zc(d.p, h.data(), 256, x.s);
  for (int k = 0; k < 4; k++) {
    HIPOK(hipMemcpyAsync(d.p, h.data(), 1 << 20, hipMemcpyHostToDevice, cp[k].s));
    HIPOK(hipMemcpyAsync(h.data(), d.p, 1 << 20, hipMemcpyDeviceToHost, sh[k].s));
  }
  for (auto& x : cp) HIPOK(hipStreamSynchronize(x.s));
  for (auto& x : sh) HIPOK(hipStreamSynchronize(x.s));
  for (auto& x : hi) HIPOK(hipStreamSynchronize(x.s));
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Parquet footer (FileMetaData) + offset index
// ------------------------------------------------------------------------------------------------
// logical annotation of a leaf as parquet-mr derives it (LogicalType union, else ConvertedType)
enum : int { LT_NONE = 0, LT_STRING = 1, LT_INT = 2, LT_DATE = 3, LT_OTHER = 4 };
struct SchemaEl {
  std::string name;
  int type = -1, type_length = 0, repetition = 0, num_children = 0;
  int conv = -1, logical = -1, int_bits = 0, int_signed = 1;
  int ts_unit = 0;                      // TIMESTAMP logical type unit: 1 millis, 2 micros, 3 nanos
  int scale = -1, precision = -1;       // DECIMAL (SchemaElement 7 / 8, or the logical type's)
  int field_id = -1;                    // SchemaElement.field_id (9), -1 when absent
  std::vector<int> kids;                // children (schema element indices), in file order
  int leaf = -1;                        // leaf index of a primitive element
};
// Statistics (parquet.thrift): deprecated max(1) / min(2), null_count(3), max_value(5) / min_value(6)
struct StatsM {
  bool has_min = false, has_max = false, has_min_value = false, has_max_value = false, has_nulls = false;
  std::string min, max, min_value, max_value;
  int64_t null_count = 0;
};
struct ColMeta {
  int type = -1, codec = 0;
  int64_t num_values = 0, total_compressed = 0, data_page_offset = 0, dict_page_offset = -1;
  int64_t oi_off = -1; int32_t oi_len = 0;
  bool has_stats = false;
  StatsM st;
};
struct RowGroupM { int64_t num_rows = 0; std::vector<ColMeta> cols; };
struct LeafM {
  std::string path; int phys, type_length, max_def, max_rep, rep_def;
  int leaf_rep = 0, lt = LT_NONE, int_bits = 0, int_signed = 1;   // own repetition, logical type
  int ts_unit = 0, dec_scale = -1;      // timestamp unit (1 ms, 2 us, 3 ns; INT96 = 4), decimal scale
};
// A checkpoint file as the decoder sees it: the footer, plus only the byte ranges of the
// projected column chunks (and their offset indexes), read with pread -- parquet-mr's column
// projection (ParquetFileReader reads the chunks of the requested schema only). `bytes` holds the
// packed chunks; `spans` maps file offsets to positions in it.
struct Span { int64_t file_off, len, packed_off; };
struct FileM {
  std::string path;
  int64_t size = 0;
  std::vector<uint8_t> footer;            // the FileMetaData bytes
  HostImg bytes;                          // packed column-chunk / offset-index layout (pageable; only
                                          // the page-header blocks are read into it, on the host)
  std::vector<Span> spans;
  int64_t num_rows = 0;                   // rows of the selected row groups
  std::vector<int32_t> sel;               // selected row groups, ascending
  int64_t row0 = 0;                       // file row index of the first selected row
  std::string created_by;
  std::vector<int> col_order;             // per leaf: 1 TYPE_DEFINED_ORDER, 0 unset
  std::vector<SchemaEl> schema;
  std::vector<LeafM> leaves;
  std::vector<RowGroupM> rgs;
};

static std::string read_string(TReader& t) {
  uint64_t n = t.varint();
  if (t.bad || n > (uint64_t)(t.e - t.p)) { t.bad = 1; return {}; }
  std::string s((const char*)t.p, n);
  t.p += n;
  return s;
}

static void parse_stats(TReader& t, StatsM& st) {
  int last = 0, ty, id;
  while ((id = t.field(&last, &ty))) {
    if (id == 1 && ty == 8) { st.max = read_string(t); st.has_max = true; }
    else if (id == 2 && ty == 8) { st.min = read_string(t); st.has_min = true; }
    else if (id == 3) { st.null_count = t.zigzag(); st.has_nulls = true; }
    else if (id == 5 && ty == 8) { st.max_value = read_string(t); st.has_max_value = true; }
    else if (id == 6 && ty == 8) { st.min_value = read_string(t); st.has_min_value = true; }
    else t.skip(ty);
    if (t.bad) return;
  }
}

static void parse_col_meta(TReader& t, ColMeta& m) {
  int last = 0, ty, id;
  while ((id = t.field(&last, &ty))) {
    switch (id) {
      case 1: m.type = (int)t.zigzag(); break;
      case 4: m.codec = (int)t.zigzag(); break;
      case 5: m.num_values = t.zigzag(); break;
      case 7: m.total_compressed = t.zigzag(); break;
      case 9: m.data_page_offset = t.zigzag(); break;
      case 11: m.dict_page_offset = t.zigzag(); break;
      case 12: if (ty == 12) { m.has_stats = true; parse_stats(t, m.st); } else t.skip(ty); break;
      default: t.skip(ty);
    }
    if (t.bad) return;
  }
}

// bytes [off, off+len) of the file, when they were read (a projected chunk or offset index)
static const uint8_t* span_ptr(const FileM& f, int64_t off, int64_t len) {
  for (const Span& sp : f.spans)
    if (off >= sp.file_off && off + len <= sp.file_off + sp.len) return f.bytes.data() + sp.packed_off + (off - sp.file_off);
  return nullptr;
}

static int read_footer(FileM& f) {
  FILE* fp = fopen(f.path.c_str(), "rb");
  if (!fp) return fail("Error reading Parquet file: " + f.path + " (cannot open)");
  fseek(fp, 0, SEEK_END);
  f.size = ftell(fp);
  uint8_t head[4] = {0}, tail[8] = {0};
  bool ok = f.size >= 12 && fseek(fp, 0, SEEK_SET) == 0 && fread(head, 1, 4, fp) == 4 &&
            fseek(fp, f.size - 8, SEEK_SET) == 0 && fread(tail, 1, 8, fp) == 8;
  if (!ok || memcmp(head, "PAR1", 4) || memcmp(tail + 4, "PAR1", 4)) {
    fclose(fp);
    return fail("Error reading Parquet file: " + f.path + " (not a Parquet file)");
  }
  uint32_t flen;
  memcpy(&flen, tail, 4);
  if ((int64_t)flen > f.size - 12) { fclose(fp); return fail("Error reading Parquet file: " + f.path + " (bad footer)"); }
  f.footer.resize(flen);
  ok = fseek(fp, f.size - 8 - (int64_t)flen, SEEK_SET) == 0 && fread(f.footer.data(), 1, flen, fp) == flen;
  fclose(fp);
  if (!ok) return fail("Error reading Parquet file: " + f.path + " (short read)");
  return 0;
}

// Read the projected spans (file order) into f.bytes. Each span keeps its file offset modulo 64 so
// that the kernels see the same alignment as in a whole-file image.
static int read_spans(FileM& f, std::vector<Span> want) {
  std::sort(want.begin(), want.end(), [](const Span& a, const Span& b) { return a.file_off < b.file_off; });
  f.spans.clear();
  for (const Span& w : want) {   // merge overlapping / adjacent ranges
    if (w.len <= 0) continue;
    if (w.file_off < 0 || w.file_off + w.len > f.size) return fail("Error reading Parquet file: " + f.path + " (chunk out of range)");
    if (!f.spans.empty() && w.file_off <= f.spans.back().file_off + f.spans.back().len) {
      Span& b = f.spans.back();
      b.len = std::max(b.len, w.file_off + w.len - b.file_off);
    } else f.spans.push_back({w.file_off, w.len, 0});
  }
  int64_t cur = 0;
  for (Span& sp : f.spans) {
    cur = (cur + 63) / 64 * 64 + (sp.file_off % 64);
    sp.packed_off = cur;
    cur += sp.len;
  }
  if (f.bytes.alloc(cur)) return 1;
  return 0;
}

static int parse_footer(FileM& f) {
  const std::vector<uint8_t>& b = f.footer;
  TReader t{b.data(), b.data() + b.size(), 0};
  int last = 0, ty, id;
  while ((id = t.field(&last, &ty))) {
    if (id == 2 && ty == 9) {
      int et;
      int n = t.list_header(&et);
      f.schema.resize(n);
      for (int i = 0; i < n && !t.bad; i++) {
        SchemaEl& s = f.schema[i];
        int l2 = 0, t2, i2;
        while ((i2 = t.field(&l2, &t2))) {
          if (i2 == 1) s.type = (int)t.zigzag();
          else if (i2 == 2) s.type_length = (int)t.zigzag();
          else if (i2 == 3) s.repetition = (int)t.zigzag();
          else if (i2 == 4) s.name = read_string(t);
          else if (i2 == 5) s.num_children = (int)t.zigzag();
          else if (i2 == 6) s.conv = (int)t.zigzag();
          else if (i2 == 7) s.scale = (int)t.zigzag();
          else if (i2 == 8) s.precision = (int)t.zigzag();
          else if (i2 == 9) s.field_id = (int)t.zigzag();
          else if (i2 == 10 && t2 == 12) {        // LogicalType union: the set member's field id
            int l3 = 0, t3, i3;
            while ((i3 = t.field(&l3, &t3))) {
              s.logical = i3;
              if (i3 == 10 && t3 == 12) {         // IntType {bitWidth: byte, isSigned: bool}
                int l4 = 0, t4, i4;
                while ((i4 = t.field(&l4, &t4))) {
                  if (i4 == 1 && t4 == 3) s.int_bits = (int8_t)t.byte();
                  else if (i4 == 2 && (t4 == 1 || t4 == 2)) s.int_signed = t4 == 1;
                  else t.skip(t4);
                  if (t.bad) break;
                }
              } else if (i3 == 8 && t3 == 12) {   // TimestampType {isAdjustedToUTC, unit: TimeUnit union}
                int l4 = 0, t4, i4;
                while ((i4 = t.field(&l4, &t4))) {
                  if (i4 == 2 && t4 == 12) {
                    int l5 = 0, t5, i5;
                    while ((i5 = t.field(&l5, &t5))) { s.ts_unit = i5; t.skip(t5); if (t.bad) break; }
                  } else t.skip(t4);
                  if (t.bad) break;
                }
              } else if (i3 == 5 && t3 == 12) {   // DecimalType {scale, precision}
                int l4 = 0, t4, i4;
                while ((i4 = t.field(&l4, &t4))) {
                  if (i4 == 1) s.scale = (int)t.zigzag();
                  else if (i4 == 2) s.precision = (int)t.zigzag();
                  else t.skip(t4);
                  if (t.bad) break;
                }
              } else t.skip(t3);
              if (t.bad) break;
            }
          }
          else t.skip(t2);
          if (t.bad) break;
        }
      }
    } else if (id == 3) {
      f.num_rows = t.zigzag();
    } else if (id == 6 && ty == 8) {
      f.created_by = read_string(t);
    } else if (id == 7 && ty == 9) {              // column_orders: list<ColumnOrder union>
      int et;
      int n = t.list_header(&et);
      for (int i = 0; i < n && !t.bad; i++) {
        int l2 = 0, t2, i2, kind = 0;
        while ((i2 = t.field(&l2, &t2))) { kind = i2 == 1 ? 1 : 0; t.skip(t2); if (t.bad) break; }
        f.col_order.push_back(kind);
      }
    } else if (id == 4 && ty == 9) {
      int et;
      int n = t.list_header(&et);
      f.rgs.resize(n);
      for (int g = 0; g < n && !t.bad; g++) {
        RowGroupM& rg = f.rgs[g];
        int l2 = 0, t2, i2;
        while ((i2 = t.field(&l2, &t2))) {
          if (i2 == 1 && t2 == 9) {
            int et2;
            int nc = t.list_header(&et2);
            rg.cols.resize(nc);
            for (int c = 0; c < nc && !t.bad; c++) {
              ColMeta& m = rg.cols[c];
              int l3 = 0, t3, i3;
              while ((i3 = t.field(&l3, &t3))) {
                if (i3 == 3 && t3 == 12) parse_col_meta(t, m);
                else if (i3 == 4) m.oi_off = t.zigzag();
                else if (i3 == 5) m.oi_len = (int32_t)t.zigzag();
                else t.skip(t3);
                if (t.bad) break;
              }
            }
          } else if (i2 == 3) {
            rg.num_rows = t.zigzag();
          } else t.skip(t2);
          if (t.bad) break;
        }
      }
    } else t.skip(ty);
    if (t.bad) break;
  }
  if (t.bad || f.schema.empty()) return fail("Error reading Parquet file: " + f.path + " (corrupt footer)");
  // leaves (DFS over the flattened schema)
  struct Fr { int remaining, def, rep, rep_def; std::string path; int el; };
  std::vector<Fr> st;
  st.push_back({f.schema[0].num_children, 0, 0, 0, "", 0});
  size_t pos = 1;
  while (!st.empty()) {
    if (st.back().remaining == 0) { st.pop_back(); continue; }
    st.back().remaining--;
    if (pos >= f.schema.size()) return fail("Error reading Parquet file: " + f.path + " (bad schema)");
    f.schema[st.back().el].kids.push_back((int)pos);
    SchemaEl& e = f.schema[pos++];
    if (e.num_children <= 0) e.leaf = (int)f.leaves.size();
    Fr& top = st.back();
    int def = top.def + (e.repetition != 0 ? 1 : 0);
    int rep = top.rep + (e.repetition == 2 ? 1 : 0);
    int rep_def = e.repetition == 2 ? def : top.rep_def;
    std::string path = top.path.empty() ? e.name : top.path + "." + e.name;
    if (e.num_children > 0) st.push_back({e.num_children, def, rep, rep_def, path, (int)pos - 1});
    else {
      LeafM L{path, e.type, e.type_length, def, rep, rep_def};
      L.leaf_rep = e.repetition;
      // parquet-mr: the LogicalType when set, else the ConvertedType (UTF8 0, DATE 6, INT_8..INT_64
      // 15..18, UINT_8..UINT_64 11..14)
      if (e.logical == 1) L.lt = LT_STRING;
      else if (e.logical == 6) L.lt = LT_DATE;
      else if (e.logical == 10) { L.lt = LT_INT; L.int_bits = e.int_bits; L.int_signed = e.int_signed; }
      else if (e.logical > 0) L.lt = LT_OTHER;
      else if (e.conv == 0) L.lt = LT_STRING;
      else if (e.conv == 6) L.lt = LT_DATE;
      else if (e.conv >= 15 && e.conv <= 18) { L.lt = LT_INT; L.int_bits = 8 << (e.conv - 15); }
      else if (e.conv >= 11 && e.conv <= 14) { L.lt = LT_INT; L.int_bits = 8 << (e.conv - 11); L.int_signed = 0; }
      else if (e.conv >= 0) L.lt = LT_OTHER;
      // timestamp unit (typed add.stats_parsed): the logical type's, else TIMESTAMP_MILLIS (9) /
      // TIMESTAMP_MICROS (10), else an INT96 leaf (Spark's default timestamp encoding)
      if (e.logical == 8) L.ts_unit = e.ts_unit;
      else if (e.logical <= 0 && e.conv == 9) L.ts_unit = 1;
      else if (e.logical <= 0 && e.conv == 10) L.ts_unit = 2;
      else if (e.type == PT_INT96) L.ts_unit = 4;
      if (e.logical == 5 || (e.logical <= 0 && e.conv == 5)) L.dec_scale = e.scale >= 0 ? e.scale : 0;
      f.leaves.push_back(L);
    }
  }
  for (auto& rg : f.rgs)
    if (rg.cols.size() != f.leaves.size()) return fail("Error reading Parquet file: " + f.path + " (column count)");
  return 0;
}

// page offsets of one chunk: from the OffsetIndex when present, otherwise a host walk of headers
struct PageRef { int64_t hdr_off; bool dict; };
static int64_t chunk_start(const ColMeta& m) {
  int64_t start = m.data_page_offset;
  if (m.dict_page_offset > 0 && m.dict_page_offset < start) start = m.dict_page_offset;
  return start;
}

static int pread_full(int fd, uint8_t* dst, int64_t len, int64_t off) {
  for (int64_t done = 0; done < len;) {
    const ssize_t k = pread(fd, dst + done, (size_t)(len - done), off + done);
    if (k <= 0) return 1;
    done += k;
  }
  return 0;
}

// Header pre-read (parquet_open's first phase): the file bytes [lo, hi) are valid in the image; more
// are pread on demand, in blocks of at least 16 KiB (many small pages' headers per read), so the page
// tables can be built before the column chunks themselves are read.
struct HdrWin {
  int fd = -1;
  const FileM* f = nullptr;
  int64_t lo = 0, hi = 0;
  // make the file bytes [off, min(off + want, lim)) valid; returns the end of the valid range, -1 on error
  int64_t ensure(int64_t off, int64_t want, int64_t lim) {
    const int64_t e = std::min(off + want, lim);
    if (off >= lo && e <= hi) return hi;
    const int64_t n = std::max(e - off, std::min<int64_t>(16384, lim - off));
    uint8_t* dst = n > 0 ? (uint8_t*)span_ptr(*f, off, n) : nullptr;
    if (!dst || pread_full(fd, dst, n, off)) return -1;
    lo = off;
    hi = off + n;
    return hi;
  }
  // a complete page header at file offset p (chunk end `end`) in the image
  int header(int64_t p, int64_t end) {
    for (int64_t want = 256;; want *= 8) {
      const int64_t h = ensure(p, want, end);
      if (h < 0) return fail("Error reading Parquet file: " + f->path + " (short read)");
      const uint8_t* b = span_ptr(*f, p, h - p);
      if (b && parse_page_header(b, b + (h - p)).ok) return 0;
      if (h >= end || want > (int64_t)1 << 26) return 0;   // malformed: the table build reports it
    }
  }
};

static int enumerate_pages(const FileM& f, const ColMeta& m, std::vector<PageRef>& out, HdrWin* w = nullptr) {
  const int64_t N = f.size;
  int64_t start = chunk_start(m);
  const int64_t cend = start + m.total_compressed;
  if (w && m.oi_off > 0 && m.oi_len > 0 && m.oi_off + m.oi_len <= N && w->ensure(m.oi_off, m.oi_len, m.oi_off + m.oi_len) < 0)
    return fail("Error reading Parquet file: " + f.path + " (short read)");
  const uint8_t* oi = (m.oi_off > 0 && m.oi_len > 0 && m.oi_off + m.oi_len <= N) ? span_ptr(f, m.oi_off, m.oi_len) : nullptr;
  if (oi) {
    TReader t{oi, oi + m.oi_len, 0};
    std::vector<int64_t> offs;
    int last = 0, ty, id;
    while ((id = t.field(&last, &ty))) {
      if (id == 1 && ty == 9) {
        int et;
        int n = t.list_header(&et);
        for (int i = 0; i < n && !t.bad; i++) {
          int l2 = 0, t2, i2;
          int64_t off = -1;
          while ((i2 = t.field(&l2, &t2))) {
            if (i2 == 1) off = t.zigzag(); else t.skip(t2);
            if (t.bad) break;
          }
          offs.push_back(off);
        }
      } else t.skip(ty);
      if (t.bad) break;
    }
    if (!t.bad && !offs.empty()) {
      if (offs[0] > start) out.push_back({start, true});   // dictionary page precedes the first data page
      for (int64_t o : offs) out.push_back({o, false});
      if (w)
        for (const PageRef& r : out)
          if (r.hdr_off >= start && r.hdr_off < cend && w->header(r.hdr_off, cend)) return 1;
      return 0;
    }
    out.clear();
  }
  // host walk (no offset index)
  int64_t p = start, end = cend;
  const uint8_t* cb = end <= N ? span_ptr(f, start, m.total_compressed) : nullptr;
  if (!cb) return fail("Error reading Parquet file: " + f.path + " (chunk out of range)");
  const uint8_t* b = cb - start;   // file-offset view of the chunk
  while (p < end) {
    if (w && w->header(p, end)) return 1;
    PageHeader h = parse_page_header(b + p, b + (w ? std::min(w->hi, end) : end));
    if (!h.ok || h.csize < 0) return fail("Error reading Parquet file: " + f.path + " (bad page header)");
    if (h.type != PAGE_INDEX) out.push_back({p, h.type == PAGE_DICT});
    p += h.hdr_len + h.csize;
  }
  return 0;
}

// The file leaf of a projected column, resolved one schema level at a time as
// ParquetSchemaUtils.findSubFieldType does (ParquetSchemaUtils.java:92-119): by the Kernel field's
// parquet.field.id when it has one and a child carries that id, then by exact name, then by the first
// case-insensitive name. Every struct group descended into builds its id -> child map first, so a
// group with two children of the same id fails (getParquetFieldToTypeMap, :122-138). Inside a map the
// key_value / key / value levels are structural (the repeated child, its first and second field).
// ids: one entry per dotted component (-1 = no id), or null. Returns the leaf index, -1 when the
// column is absent (read as all-null), -2 on error (g_err set).
static constexpr int kMaxLeafDepth = 8;
static int leaf_index(const FileM& f, const std::string& want, const int32_t* ids = nullptr) {
  std::vector<std::string> comps;
  for (size_t a = 0;;) {
    const size_t b = want.find('.', a);
    comps.push_back(want.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  auto low = [](std::string x) { for (auto& c : x) c = (char)tolower((unsigned char)c); return x; };
  int g = 0;
  int map_level = 0;                        // 1: g is a MAP group, 2: g is a map's key_value group
  for (size_t ci = 0; ci < comps.size(); ci++) {
    const SchemaEl& G = f.schema[g];
    if (G.kids.empty()) return -1;          // a primitive where the projection expects a group
    const std::string& name = comps[ci];
    int hit = -1;
    if (map_level == 0 && (G.conv == 1 || G.logical == 2)) map_level = 1;   // MAP annotation
    if (map_level == 1) {
      if (G.kids.size() == 1 && f.schema[G.kids[0]].repetition == 2) hit = G.kids[0];
      map_level = hit >= 0 ? 2 : 0;
    } else if (map_level == 2) {
      if (G.kids.size() == 2 && (name == "key" || name == "value")) hit = G.kids[name == "key" ? 0 : 1];
      map_level = 0;
    }
    if (hit < 0) {
      // a struct group: id map first (duplicate ids fail even when the read schema has none)
      std::vector<std::pair<int, int>> by_id;
      for (int k : G.kids)
        if (f.schema[k].field_id >= 0) {
          for (auto& q : by_id)
            if (q.first == f.schema[k].field_id) {
              fail("java.lang.IllegalStateException: Parquet file contains multiple columns (" +
                   f.schema[q.second].name + ", " + f.schema[k].name + ") with the same field id");
              return -2;
            }
          by_id.push_back({f.schema[k].field_id, k});
        }
      const int id = ids && ci < (size_t)kMaxLeafDepth ? ids[ci] : -1;
      if (id >= 0)
        for (auto& q : by_id) if (q.first == id) { hit = q.second; break; }
      if (hit < 0) for (int k : G.kids) if (f.schema[k].name == name) { hit = k; break; }
      if (hit < 0) {
        const std::string w = low(name);
        for (int k : G.kids) if (low(f.schema[k].name) == w) { hit = k; break; }
      }
    }
    if (hit < 0) return -1;
    g = hit;
  }
  return f.schema[g].leaf;                  // -1 when the path ends on a group
}

static int phys_width(int phys, int tl) {
  switch (phys) { case PT_BOOLEAN: return 1; case PT_INT32: case PT_FLOAT: return 4; case PT_INT64: case PT_DOUBLE: return 8;
    case PT_INT96: return 12; case PT_FIXED: return tl; default: return 0; }
}

// ------------------------------------------------------------------------------------------------
// kernel timing (HIP events on the engine stream)
// ------------------------------------------------------------------------------------------------
struct KTimer {
  static constexpr int K = 24;
  const char* names[K] = {"k_page_headers", "unused", "k_tile_count", "k_tile_scan",
                          "k_string_positions", "k_tile_decode", "k_string_copy", "k_json_canon",
                          "k_table_insert", "k_table_update", "k_json_select", "k_probe", "step_total",
                          "k_snap_walk_link", "k_delta_decode", "k_page_runs", "k_tile_chars", "k_stats_eval", "k_part_eval",
                          "k_snap_fix", "k_snap_frag", "k_snappy_serial", "k_owner_route", "k_owner_resolve"};
  double sum_ms[K] = {0};
  int64_t cnt[K] = {0};
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  bool on = false;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e; hipEventCreate(&e); return e;
  }
  struct Scope {
    KTimer* t; int k; hipStream_t s; hipEvent_t a = nullptr, b = nullptr;
    Scope(KTimer* t_, int k_, hipStream_t s_) : t(t_), k(k_), s(s_) { if (t->on) { a = t->get(); b = t->get(); hipEventRecord(a, s); } }
    ~Scope() { if (t->on) { hipEventRecord(b, s); t->pending.push_back({k, {a, b}}); } }
  };
  void collect() {
    for (auto& p : pending) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, p.second.first, p.second.second) == hipSuccess) { sum_ms[p.first] += ms; cnt[p.first]++; }
      pool.push_back(p.second.first); pool.push_back(p.second.second);
    }
    pending.clear();
  }
  ~KTimer() { for (auto& p : pending) { hipEventDestroy(p.second.first); hipEventDestroy(p.second.second); }
              for (auto e : pool) hipEventDestroy(e); }
};

// ------------------------------------------------------------------------------------------------
// dk_parquet: a set of files x projected leaves, decoded on the GPU
// ------------------------------------------------------------------------------------------------
struct HostCol {           // host copy of a row range of one decoded column (dk_parquet_column_rows)
  bool ready = false;
  std::vector<uint8_t> row_def, entry_def, fixed, chars;
  std::vector<int64_t> row_offs, offs;
};
// Host mirror of one decoded column in pinned memory (dk_parquet_column). The first request for a
// leaf queues the D2H copies of that leaf for EVERY file of the set at once (a scan consumer reads
// the same leaves of every batch), each with its own event; a request waits only for its file.
struct HostMirror {
  int state = 0;            // 0 empty, 1 copy queued (wait on ev), 2 ready
  hipEvent_t ev = nullptr;
  HBuf row_def, row_offs, entry_def, fixed, offs, chars;
  HostMirror() = default;
  HostMirror(const HostMirror&) = delete;
  HostMirror(HostMirror&& o) noexcept : state(o.state), ev(o.ev), row_def(std::move(o.row_def)), row_offs(std::move(o.row_offs)),
      entry_def(std::move(o.entry_def)), fixed(std::move(o.fixed)), offs(std::move(o.offs)), chars(std::move(o.chars)) { o.ev = nullptr; }
  ~HostMirror() { if (ev) hipEventDestroy(ev); }
};

static constexpr int kCopyStreams = 8;   // H2D streams of a file open (the SDMA engines work in parallel)
static int copy_streams() {
  static const int n = getenv("DK_COPY_STREAMS") ? std::max(1, std::min(kCopyStreams, atoi(getenv("DK_COPY_STREAMS")))) : 4;
  return n;
}
struct EventH {
  hipEvent_t e = nullptr;
  EventH() = default;
  EventH(const EventH&) = delete;
  EventH& operator=(const EventH&) = delete;
  EventH(EventH&& o) noexcept : e(o.e) { o.e = nullptr; }
  ~EventH() { if (e) hipEventDestroy(e); }
  operator hipEvent_t() const { return e; }
};
struct dk_parquet {
  StreamH own;                      // first members: destroyed after every buffer below
  StreamH copy[kCopyStreams];
  StreamH aux;                      // table uploads while `stream` waits for the H2D copies
  StreamH side[2];                  // sizing slices rotate over stream, side[0], side[1] (created on demand)
  StreamH dec;                      // per-slice value decode (high priority): never queued behind a later
                                    // slice's sizing passes and their waits on its files' H2D copies
  EventH copy_done[kCopyStreams];
  hipStream_t stream = nullptr;
  dk_engine* eng = nullptr;
  std::vector<FileM> files;
  std::vector<std::string> leaves;
  // per (file, leaf): column index or -1 (missing leaf)
  std::vector<std::vector<int>> colmap;
  std::vector<std::vector<int>> leafidx;  // file leaf index for (file, leaf)
  std::vector<DBuf> dfile;
  std::vector<DChunk> h_chunks;
  std::vector<DPage> h_pages;
  std::vector<DColumn> h_cols;
  std::vector<int> col_file;
  DBuf d_chunks, d_pages, d_cols, d_pos, d_arena, d_state, d_dbp, d_tiles;
  // snappy: compressed pages, their 64 KiB fragment bases / work items / starts, serial flags
  DBuf d_cpage, d_fbase, d_fwork, d_fstart, d_serial, d_snap_ob, d_fseg;
  DBuf d_sbase, d_spage, d_snapws;   // speculative-walk segments: page bases, owner page, workspace
  DBuf d_tbits;                      // page mode: tag-start bitmap (DK_SNAP_SEG / 64 words per segment)
  DBuf d_pwork;                      // page-mode work items (page, -1)
  int n_cpages = 0, n_frags = 0, n_segs = 0;
  DBuf d_ltiles, d_runs;     // level tiles (DTile) and hybrid-stream run tables (Seg)
  int n_ltiles = 0;
  DBuf d_pchunks;            // string-position chunks (DPosChunk)
  DBuf d_pos_scratch;        // k_pos_count's candidates, DK_POS_CAP int16 offsets per chunk
  int n_pchunks = 0;
  // string-copy tile table: (page, first value) per 256-value tile of every PLAIN BYTE_ARRAY data
  // page, grouped by column (col_tile0[c] = first tile of column c; col_tile0[n_cols] = total)
  std::vector<int> col_tile0;
  int copy_cb = 16384;       // k_string_copy staging buffer bytes (sized to the data in prepare)
  std::vector<std::unique_ptr<DBuf>> outbufs;
  std::vector<HostMirror> host;
  std::vector<HostCol> slice;   // dk_parquet_column_rows: one row range per column, offsets rebased
  DBuf d_first;                 // dk_parquet_first_row result
  DBuf d_expand;                // k_expand inputs (group prefix + ids)
  // slices for the pipelined prepare: per file its first page / column (n_files + 1 entries), the
  // compressed-page list and its segment / fragment prefixes, and an event after each file's copies
  std::vector<int> file_page0, file_col0;
  // grouped replay runs (dk_replay_run_grouped): per file, the event after which its decoded columns
  // are final (set and cleared by the replay; empty: the stream order is enough)
  std::vector<hipEvent_t> file_done;
  std::vector<int32_t> h_cpage, h_sbase, h_fbase;
  std::vector<EventH> file_ev;
  // the images are read while prepare runs: per file 0 = its H2D copies not queued yet, 1 = queued
  // (file_ev recorded), 2 = its read failed (null: every image was queued before prepare)
  std::unique_ptr<std::atomic<int>[]> queued;
  std::chrono::steady_clock::time_point t_open0;   // DK_VERBOSE timeline origin
  std::vector<HBuf> staging;        // pinned sources of zero-copy uploads, released when prepare ends
  int n_pages = 0, n_cols = 0;
  bool has_compressed = false, has_dbp = false;
  int64_t bytes_read = 0, bytes_written = 0, bytes_arena = 0;
  KTimer timer;
  // host read + H2D issue, page metadata, prepare passes; inside prepare: H2D wait + headers,
  // host page tables, device sizing passes, host tiles + output arena
  double open_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool prepared = false;
  // the prepare pass ran every stage up to the tile scans on the current inputs: the next full
  // pipeline run only re-runs the scans (sentinels into the freshly allocated outputs), the string
  // copy and the value decode (a getScanFiles that runs once decodes each page once)
  bool fresh = false;
  // the prepare pass also decoded every column, slice by slice as the files landed: the next full
  // run skips the decode pipeline (value decode included) once; skip_decode: that run is under way
  // (a grouped replay's per-group decode_cols calls are no-ops)
  bool decoded_fresh = false, skip_decode = false;
  // asynchronous open (dk_parquet_open_async): the opening thread keeps reading, sizing and decoding
  // after the handle is returned; files [0, files_ready) have final columns and a decode event
  // (file_dec) by then. open_state: 0 running, 1 done, 2 failed (open_err).
  std::thread opener;
  std::atomic<bool> abort_open{false};   // dk_parquet_close before the open finished: stop reading
  std::atomic<int> open_state{1};
  std::string open_err;
  std::mutex rmu;
  std::condition_variable rcv;
  int files_ready = INT_MAX;
  std::vector<hipEvent_t> file_dec;  // per file (events owned by dec_events)
  std::vector<hipEvent_t> dec_events;
  StreamH mir;                       // host-mirror copies (not behind the open's passes on `stream`)
  hipEvent_t mir_ev = nullptr;
  bool async_open = false;
  ~dk_parquet() {
    if (opener.joinable()) opener.join();
    for (hipEvent_t e : dec_events) hipEventDestroy(e);
    if (mir_ev) hipEventDestroy(mir_ev);
  }
};

static int upload(DBuf& d, const void* src, size_t n, hipStream_t s) {
  if (d.n < n || !d.p) if (d.alloc(n ? n : 16)) return 1;
  if (n) HIPOK(hipMemcpyAsync(d.p, src, n, hipMemcpyHostToDevice, s));
  return 0;
}


// Snappy page mode (DK_SNAPPY_MODE=page): one wave decodes a whole page in order.
static bool snap_page_mode(const dk_parquet* p) {
  static const char* env = getenv("DK_SNAPPY_MODE");
  (void)p;
  return env && !strcmp(env, "page");
}
// Default (hybrid): 64 KiB fragments (k_snap_fix finds their starts from the verified segment
// entries) decoded with page mode's tag-start bitmap: page mode's discovery with frag mode's load
// balance -- one wave per 1 MB page left the largest pages as two serial rounds of ~20 ms each on
// C3. DK_SNAPPY_MODE=page | frag forces the other two.
static bool snap_hybrid(const dk_parquet* p) {
  static const char* env = getenv("DK_SNAPPY_MODE");
  (void)p;
  return !env || !strcmp(env, "hybrid");
}

// A contiguous slice of the decode work: files [f0, f1) own pages [pa, pb), compressed pages
// [ca, cb) with their segments [s0, s1) and fragments [fr0, fr1), columns [col0, col1), level tiles
// [t0, t1) and string-position chunks [pc0, pc1). The prepare pass runs one slice per group of files
// as soon as those files' H2D copies have landed.
struct PRange { int pa = 0, pb = 0, ca = 0, cb = 0, s0 = 0, s1 = 0, fr0 = 0, fr1 = 0, col0 = 0, col1 = 0, t0 = 0, t1 = 0, pc0 = 0, pc1 = 0; };

static PRange file_range(const dk_parquet* p, int f0, int f1) {
  PRange R;
  R.pa = p->file_page0[f0]; R.pb = p->file_page0[f1];
  R.col0 = p->file_col0[f0]; R.col1 = p->file_col0[f1];
  R.ca = (int)(std::lower_bound(p->h_cpage.begin(), p->h_cpage.end(), R.pa) - p->h_cpage.begin());
  R.cb = (int)(std::lower_bound(p->h_cpage.begin(), p->h_cpage.end(), R.pb) - p->h_cpage.begin());
  if (!p->h_sbase.empty()) { R.s0 = p->h_sbase[R.ca]; R.s1 = p->h_sbase[R.cb]; R.fr0 = p->h_fbase[R.ca]; R.fr1 = p->h_fbase[R.cb]; }
  R.t0 = R.col0 < p->n_cols ? p->h_cols[R.col0].first_tile : p->n_ltiles;
  R.t1 = R.col1 < p->n_cols ? p->h_cols[R.col1].first_tile : p->n_ltiles;
  R.pc0 = R.pa < p->n_pages ? p->h_pages[R.pa].pchunk0 : p->n_pchunks;
  R.pc1 = R.pb < p->n_pages ? p->h_pages[R.pb].pchunk0 : p->n_pchunks;
  return R;
}

// headers, snappy, runs, counts, positions, chars and the scans over one slice
static void sizing_stages(dk_parquet* p, hipStream_t s, const PRange& R) {
  KTimer& T = p->timer;
  const DChunk* C = p->d_chunks.as<DChunk>();
  DPage* P = p->d_pages.as<DPage>();
  int32_t* pos = p->d_pos.as<int32_t>();
  const uint8_t* arena = p->d_arena.as<uint8_t>();
  DState* st = p->d_state.as<DState>();
  DColumn* cols = p->d_cols.as<DColumn>();
  DTile* LT = p->d_ltiles.as<DTile>();
  Seg* runs = p->d_runs.as<Seg>();
  const int np = R.pb - R.pa;
  if (p->has_compressed && R.cb > R.ca) {
    SnapCtx X{};
    X.chunks = C; X.pages = P; X.arena = p->d_arena.as<uint8_t>();
    X.cpage = p->d_cpage.as<int32_t>(); X.sbase = p->d_sbase.as<int32_t>(); X.spage = p->d_spage.as<int32_t>();
    X.nseg = p->n_segs;
    int32_t* ws = p->d_snapws.as<int32_t>();
    const int64_t ns = p->n_segs;
    X.w_exit = ws; X.w_out = ws + ns; X.w_npos = ws + 2 * ns; X.t_entry = ws + 3 * ns; X.t_out = ws + 4 * ns;
    X.t_exit = ws + 5 * ns; X.w_pos = ws + 6 * ns; X.w_cum = ws + (6 + DK_SNAP_REC) * ns;
    X.relink = ws + (6 + 2 * DK_SNAP_REC) * ns; X.relink_n = ws + (7 + 2 * DK_SNAP_REC) * ns;
    X.fbase = p->d_fbase.as<int32_t>(); X.fstart = p->d_fstart.as<int64_t>(); X.serial = p->d_serial.as<int32_t>();
    X.t_ob = p->d_snap_ob.as<int64_t>(); X.fseg = p->d_fseg.as<int32_t>();
    X.k0 = R.s0; X.k1 = R.s1; X.c0 = R.ca;
    // page mode (one wave decodes a whole page in order, no walk; never sliced) or the speculative
    // walk that splits pages into 64 KiB fragments
    const bool page_mode = snap_page_mode(p);
    const int ncp = R.cb - R.ca;
    const int nfr = page_mode ? -1 : R.fr1 - R.fr0;
    X.page_mode = page_mode ? 1 : 0;
    X.tbits = (page_mode || snap_hybrid(p)) ? p->d_tbits.as<uint64_t>() : nullptr;
    const int2* wk = page_mode ? p->d_pwork.as<int2>() : p->d_fwork.as<int2>() + R.fr0;
    { KTimer::Scope s0(&T, 13, s); launch_snappy(X, ncp, nfr, wk, 0, s); }
    { KTimer::Scope s1(&T, 19, s); launch_snappy(X, ncp, nfr, wk, 1, s); }
    { KTimer::Scope s2(&T, 20, s); launch_snappy(X, ncp, nfr, wk, 2, s); }
    { KTimer::Scope s3(&T, 21, s); launch_snappy(X, ncp, nfr, wk, 3, s); }
  }
  { KTimer::Scope sc(&T, 15, s); launch_page_runs(C, P + R.pa, np, arena, runs, s); }
  { KTimer::Scope sc(&T, 2, s); launch_tile_count(C, P, arena, runs, LT, R.t1 - R.t0, R.t0, s); }
  { KTimer::Scope sc(&T, 3, s); launch_tile_scan1(cols + R.col0, R.col1 - R.col0, P, LT, st, s); }
  { KTimer::Scope sc(&T, 4, s); launch_positions(C, P, R.pa, np, arena, pos, p->d_pchunks.as<DPosChunk>(), R.pc0, R.pc1 - R.pc0,
                                                    p->d_pos_scratch.as<int16_t>(), s); }
  if (p->has_dbp) { KTimer::Scope sc(&T, 14, s); launch_delta_decode(C, P + R.pa, np, arena, p->d_dbp.as<long long>(), s); }
  { KTimer::Scope sc(&T, 16, s); launch_tile_chars(C, P, arena, pos, runs, LT, R.t1 - R.t0, R.t0, s); }
  { KTimer::Scope sc(&T, 3, s); launch_tile_scan2(cols + R.col0, R.col1 - R.col0, P, LT, st, s); }
}

// the value decode of columns [c0, c1) (every column of a run of files): string copies first -- they
// fill the key column's per-value hashes that k_tile_decode forwards -- then the level / value tiles
static void decode_cols(dk_parquet* p, hipStream_t s, int c0, int c1) {
  if (c1 <= c0 || p->skip_decode) return;
  KTimer& T = p->timer;
  const DChunk* C = p->d_chunks.as<DChunk>();
  DPage* P = p->d_pages.as<DPage>();
  int32_t* pos = p->d_pos.as<int32_t>();
  const uint8_t* arena = p->d_arena.as<uint8_t>();
  DState* st = p->d_state.as<DState>();
  DColumn* cols = p->d_cols.as<DColumn>();
  const long long* dbp = p->d_dbp.as<long long>();
  DTile* LT = p->d_ltiles.as<DTile>();
  Seg* runs = p->d_runs.as<Seg>();
  {
    KTimer::Scope sc(&T, 6, s);
    const int2* tiles = p->d_tiles.as<int2>();
    const int t0 = p->col_tile0[c0], t1 = p->col_tile0[c1];
    if (t1 > t0) launch_string_copy(C, P, t1 - t0, cols, arena, pos, tiles, s, t0, p->copy_cb);
  }
  {
    KTimer::Scope sc(&T, 5, s);
    const int a = p->h_cols[c0].first_tile;
    const int b = c1 < p->n_cols ? p->h_cols[c1].first_tile : p->n_ltiles;
    if (b > a) launch_tile_decode(C, P, cols, arena, pos, dbp, runs, LT, b - a, a, st, s);
  }
}

// the decode pipeline over every file (mode: -1 = headers only; 0 = through the scans, which size the
// outputs; 1 = full step; front_only: mode 1 without the value decode, which the caller runs per file
// group with decode_cols)
static int run_pipeline(dk_parquet* p, int mode, hipStream_t s = nullptr, bool front_only = false) {
  if (!s) s = p->stream;
  KTimer& T = p->timer;
  const DChunk* C = p->d_chunks.as<DChunk>();
  DPage* P = p->d_pages.as<DPage>();
  DState* st = p->d_state.as<DState>();
  DColumn* cols = p->d_cols.as<DColumn>();
  DTile* LT = p->d_ltiles.as<DTile>();
  p->skip_decode = false;
  if (mode == 1 && p->decoded_fresh) {   // prepare decoded everything already (per slice)
    p->decoded_fresh = false;
    p->fresh = false;
    p->skip_decode = true;
    return 0;
  }
  const bool reuse = mode == 1 && p->fresh;
  p->fresh = false;
  if (reuse) {                         // headers, snappy, runs, counts, positions, chars: done by prepare
    { KTimer::Scope sc(&T, 3, s); launch_tile_scan1(cols, p->n_cols, P, LT, st, s); }
    { KTimer::Scope sc(&T, 3, s); launch_tile_scan2(cols, p->n_cols, P, LT, st, s); }
  } else {
    { KTimer::Scope sc(&T, 0, s); launch_page_headers(C, P, p->n_pages, s); }
    if (mode == -1) return 0;
    sizing_stages(p, s, file_range(p, 0, (int)p->files.size()));
    if (mode == 0) return 0;
  }
  if (!front_only) decode_cols(p, s, 0, p->n_cols);
  return 0;
}

static int64_t file_offset(const FileM& f, int64_t packed) {
  for (const Span& sp : f.spans)
    if (packed >= sp.packed_off && packed < sp.packed_off + sp.len) return sp.file_off + (packed - sp.packed_off);
  return packed;
}

static std::string page_status_msg(const dk_parquet* p, const std::vector<DPage>& pages) {
  for (const DPage& pg : pages)
    if (pg.status != PS_OK) {
      const DChunk& ck = p->h_chunks[pg.chunk];
      int fi = p->col_file[ck.col];
      static const char* why[] = {"ok", "bad page header", "bad levels", "bad values", "unsupported encoding/codec",
                                  "bad dictionary", "bad snappy block"};
      return "Error reading Parquet file: " + p->files[fi].path + " (" + why[pg.status < 7 ? pg.status : 4] +
             " at offset " + std::to_string(file_offset(p->files[fi], pg.hdr_off)) + ")";
    }
  return "";
}

// dst = the work items of `groups` (item i of group g: k_expand's record kind over gid[g] or g and
// the item's index within its group), base = the groups' item prefix (n + 1 entries)
static int expand(dk_parquet* p, hipStream_t us, DBuf& dst, const std::vector<int32_t>& gid,
                  const std::vector<int64_t>& base, int kind, size_t item_bytes) {
  const int n = (int)base.size() - 1;
  const int64_t total = base.back();
  if (dst.alloc((size_t)std::max<int64_t>(total, 1) * item_bytes)) return 1;
  if (!total) return 0;
  // the kernel reads the prefix / ids straight from pinned host memory (kept until prepare ends):
  // no DMA behind the file images, no synchronisation
  HBuf hb;
  if (hb.alloc((size_t)(n + 1) * 8 + (size_t)n * 4 + 64)) return 1;
  memcpy(hb.data(), base.data(), (size_t)(n + 1) * 8);
  if (!gid.empty()) memcpy(hb.data() + (size_t)(n + 1) * 8, gid.data(), (size_t)n * 4);
  launch_expand((const int64_t*)hb.data(), gid.empty() ? nullptr : (const int32_t*)(hb.data() + (size_t)(n + 1) * 8),
                n, kind, dst.p, us);
  p->staging.push_back(std::move(hb));
  return 0;
}

// upload through pinned staging copied by a kernel (launch_copy_zc): never queues behind, nor
// blocks on, the H2D copies of the file images
static int upload_zc(dk_parquet* p, DBuf& d, const void* src, size_t n, hipStream_t s) {
  if (d.n < n || !d.p) if (d.alloc(n ? n : 16)) return 1;
  if (!n) return 0;
  HBuf hb;
  if (hb.alloc(n)) return 1;
  memcpy(hb.data(), src, n);
  launch_copy_zc(d.p, hb.data(), (long long)n, s);
  p->staging.push_back(std::move(hb));
  return 0;
}

// String-copy tiles of columns [c0, c1) (appended; col_tile0 gets one entry per column) and the
// staging size they need (p->copy_cb: the running max over calls; page counts must be final)
static void build_tiles(dk_parquet* p, int c0, int c1, std::vector<int2>& tiles) {
  const int base = p->col_tile0.back() - (int)tiles.size();   // tiles of earlier calls already counted
  // staging buffer: the busiest PLAIN page's mean span of DK_COPY_TILE values (+5%), so a typical
  // tile is one pass while the two buffers stay small enough for high occupancy
  double span = 0;
  for (int ci = c0; ci < c1; ci++) {
    const DColumn& c = p->h_cols[ci];
    if (c.phys != PT_BYTE_ARRAY) continue;
    for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) {
      const DPage& pg = p->h_pages[pi];
      if ((pg.flags & PF_DICT) || pg.enc != ENC_PLAIN || pg.n_values <= 0) continue;
      span = std::max(span, (double)pg.vbytes / pg.n_values * DK_COPY_TILE * 1.05 + 64);
    }
  }
  p->copy_cb = std::max(p->copy_cb, span > 0 ? (int)span : 16384);
  for (int ci = c0; ci < c1; ci++) {
    const DColumn& c = p->h_cols[ci];
    for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) {
      const DPage& pg = p->h_pages[pi];
      if (c.phys != PT_BYTE_ARRAY || (pg.flags & PF_DICT) || pg.enc != ENC_PLAIN) continue;
      for (int v0 = 0; v0 < pg.n_values; v0 += DK_COPY_TILE) tiles.push_back(make_int2(pi, v0));
    }
    // key column: its dictionary pages are hashed entry by entry (hash-only tiles)
    if (c.key_hash && c.phys == PT_BYTE_ARRAY && c.max_rep == 0)
      for (const DChunk& ck : p->h_chunks)
        if (ck.col == ci && ck.dict_page >= 0)
          for (int v0 = 0; v0 < p->h_pages[ck.dict_page].num_values; v0 += DK_COPY_TILE)
            tiles.push_back(make_int2(ck.dict_page, v0));
    p->col_tile0.push_back(base + (int)tiles.size());
  }
}

// Output buffers of columns [c0, c1) carved from one new device arena (one hipMalloc instead of ~3
// per (file, leaf) -- thousands at C3's 64 files x 21 leaves); pass 0 sizes the arena, pass 1 hands
// out the pointers. got[ci]: the device column after the sizing scans (entry / char totals).
static int alloc_outputs(dk_parquet* p, int c0, int c1, const std::vector<DColumn>& got) {
  size_t arena_bytes = 0;
  for (int pass = 0; pass < 2; pass++) {
  if (pass == 1) {
    p->outbufs.emplace_back(new DBuf());
    if (p->outbufs.back()->alloc(arena_bytes + 256)) return 1;
  }
  uint8_t* const arena_base = pass == 1 ? p->outbufs.back()->as<uint8_t>() : nullptr;
  size_t arena_at = 0;
  for (int i = c0; i < c1; i++) {
    DColumn& c = p->h_cols[i];
    c.n_entries = got[i].n_entries;
    c.n_chars = got[i].n_chars;
    c.cap_entries = c.n_entries;
    c.cap_chars = c.n_chars;
    int64_t nv = c.max_rep > 0 ? c.n_entries : c.n_rows;
    auto mk = [&](size_t bytes) -> void* {
      const size_t at = arena_at;
      arena_at += (bytes + 16 + 255) & ~(size_t)255;     // 256-byte aligned, 16 bytes of slack each
      if (pass == 1) p->bytes_written += bytes;
      return pass == 1 ? (void*)(arena_base + at) : (void*)(uintptr_t)(at + 256);   // pass 0: non-null
    };
    int64_t n_values = 0;
    for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) n_values += p->h_pages[pi].n_values;
    c.null_only = (n_values == 0 && (c.max_rep == 0 || c.n_entries == 0)) ? 1 : 0;
    c.row_def = (uint8_t*)mk(c.n_rows);
    c.vhash = c.hash = c.dhash = nullptr;
    if (c.key_hash && !c.null_only && c.phys == PT_BYTE_ARRAY && c.max_rep == 0) {
      int64_t dn = 0;        // dictionary entries of the column's chunks
      for (DChunk& ck : p->h_chunks)
        if (ck.col == i && ck.dict_page >= 0) { ck.dict_hash_off = dn; dn += p->h_pages[ck.dict_page].num_values; }
      if (dn) {
        c.dhash = (uint64_t*)mk(dn * 8);
        if (pass == 1) p->bytes_written -= dn * 8;               // scratch
        if (!c.dhash) return 1;
      }
      c.vhash = (uint64_t*)mk((n_values + 1) * 8);
      if (pass == 1) p->bytes_written -= (n_values + 1) * 8;     // scratch, not an output (written + re-read once)
      c.hash = (uint64_t*)mk(c.n_rows * 8);
      if (!c.vhash || !c.hash) return 1;
    }
    c.row_offs = (c.max_rep > 0 && !c.null_only) ? (int64_t*)mk((c.n_rows + 1) * 8) : nullptr;
    c.entry_def = (c.max_rep > 0 && !c.null_only) ? (uint8_t*)mk(nv) : nullptr;
    c.fixed = nullptr; c.offs = nullptr; c.chars = nullptr;
    if (!c.null_only) {
      if (c.phys == PT_BYTE_ARRAY) {
        c.offs = (int64_t*)mk((nv + 1) * 8);
        c.chars = (uint8_t*)mk(c.n_chars);
      } else {
        c.fixed = (uint8_t*)mk(nv * c.width);
      }
    }
    if (!c.row_def) return 1;
  }
  arena_bytes = arena_at;
  }
  return 0;
}

// hipEventQuery: 1 complete, 0 not yet, -1 an error (reported through fail): a sticky device fault
// must end the open's polling loops with that error instead of polling forever
static int ev_done(hipEvent_t e) {
  const hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return 1;
  if (q == hipErrorNotReady) return 0;
  fail(std::string("HIP error: ") + hipGetErrorString(q) + " (an event of the checkpoint open)");
  return -1;
}

// Wait until file f's image copies are queued (file_ev recorded: a stream may wait for it; an event
// that was never recorded would let it through at once). False: the file's read failed.
static bool wait_queued(const dk_parquet* p, int f) {
  if (!p->queued) return true;
  int v;
  while ((v = p->queued[f].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
  return v == 1;
}
static bool is_queued(const dk_parquet* p, int f) { return !p->queued || p->queued[f].load(std::memory_order_acquire) == 1; }

static int check_state(dk_parquet* p);

// upload_zc to dst (device memory of any buffer, any offset)
static int upload_zc_to(dk_parquet* p, void* dst, const void* src, size_t n, hipStream_t s) {
  if (!n) return 0;
  HBuf hb;
  if (hb.alloc(n)) return 1;
  memcpy(hb.data(), src, n);
  launch_copy_zc(dst, hb.data(), (long long)n, s);
  p->staging.push_back(std::move(hb));
  return 0;
}

// A sized slice whose outputs are still to be allocated: its columns and pages come back to pinned
// memory through a copy kernel (a D2H copy would wait behind the H2D copies of the later files).
struct SizedSlice {
  PRange R;
  int f0 = 0, f1 = 0;
  hipStream_t cs = nullptr;
  hipEvent_t ev = nullptr;
  HBuf cols, pages;
};

// After a slice's sizing passes: page status, string-copy tiles, output arena, the scans again (the
// sentinels into the new outputs) and the value decode of its columns, on its stream.
static int finish_slice(dk_parquet* p, SizedSlice& S, std::vector<DColumn>& got) {
  const PRange& R = S.R;
  HIPOK(hipEventSynchronize(S.ev));                // the sizing passes are complete
  const hipStream_t ds = p->dec.s ? p->dec.s : S.cs;
  hipEventDestroy(S.ev);
  S.ev = nullptr;
  memcpy(got.data() + R.col0, S.cols.data(), (size_t)(R.col1 - R.col0) * sizeof(DColumn));
  memcpy(p->h_pages.data() + R.pa, S.pages.data(), (size_t)(R.pb - R.pa) * sizeof(DPage));
  for (int pi = R.pa; pi < R.pb; pi++)
    if (p->h_pages[pi].status != PS_OK) {
      std::vector<DPage> one(1, p->h_pages[pi]);
      return fail(page_status_msg(p, one));
    }
  std::vector<int2> tiles;
  const int t0 = p->col_tile0.back();
  build_tiles(p, R.col0, R.col1, tiles);
  if ((size_t)(t0 + tiles.size()) * sizeof(int2) > p->d_tiles.n) return fail("internal: string-copy tile bound exceeded");
  if (upload_zc_to(p, p->d_tiles.as<int2>() + t0, tiles.data(), tiles.size() * sizeof(int2), ds)) return 1;
  if (alloc_outputs(p, R.col0, R.col1, got)) return 1;
  if (upload_zc_to(p, p->d_cols.as<DColumn>() + R.col0, p->h_cols.data() + R.col0, (size_t)(R.col1 - R.col0) * sizeof(DColumn), ds))
    return 1;
  int k0 = (int)p->h_chunks.size(), k1 = 0;        // the slice's chunks (dict_hash_off)
  for (int k = 0; k < (int)p->h_chunks.size(); k++)
    if (p->h_chunks[k].col >= R.col0 && p->h_chunks[k].col < R.col1) { k0 = std::min(k0, k); k1 = k + 1; }
  if (k1 > k0 && upload_zc_to(p, p->d_chunks.as<DChunk>() + k0, p->h_chunks.data() + k0, (size_t)(k1 - k0) * sizeof(DChunk), ds))
    return 1;
  KTimer& T = p->timer;
  DColumn* cols = p->d_cols.as<DColumn>();
  { KTimer::Scope sc(&T, 3, ds); launch_tile_scan1(cols + R.col0, R.col1 - R.col0, p->d_pages.as<DPage>(), p->d_ltiles.as<DTile>(), p->d_state.as<DState>(), ds); }
  { KTimer::Scope sc(&T, 3, ds); launch_tile_scan2(cols + R.col0, R.col1 - R.col0, p->d_pages.as<DPage>(), p->d_ltiles.as<DTile>(), p->d_state.as<DState>(), ds); }
  decode_cols(p, ds, R.col0, R.col1);
  hipEvent_t dev = nullptr;                       // the slice's files are decoded after this
  HIPOK(hipEventCreateWithFlags(&dev, hipEventDisableTiming));
  HIPOK(hipEventRecord(dev, ds));
  p->dec_events.push_back(dev);
  {
    std::lock_guard<std::mutex> g(p->rmu);
    if (p->file_dec.size() < p->files.size()) p->file_dec.resize(p->files.size(), nullptr);
    for (int f = S.f0; f < S.f1; f++) p->file_dec[f] = dev;
    if (p->files_ready != INT_MAX) p->files_ready = S.f1;
  }
  if (getenv("DK_VERBOSE"))
    fprintf(stderr, "[dk] decode of files [%d, %d) queued at %.1f ms\n", S.f0, S.f1,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p->t_open0).count());
  p->rcv.notify_all();
  return 0;
}

// Asynchronous opens: wait until files [0, f1) are decoded (their columns final, file_dec recorded)
static int wait_files(dk_parquet* p, int f1) {
  std::unique_lock<std::mutex> lk(p->rmu);
  p->rcv.wait(lk, [&] { return p->files_ready >= f1 || p->open_state.load() != 0; });
  if (p->files_ready >= f1 || p->open_state.load() == 1) return 0;
  return fail(p->open_err);
}
// ... without waiting: are files [0, f1) decoded already?
static bool files_ready_now(dk_parquet* p, int f1) {
  std::lock_guard<std::mutex> lk(p->rmu);
  return p->files_ready >= f1 || p->open_state.load() != 0;
}
// ... until the whole open has finished (joined); its error, if any
static int ensure_open(dk_parquet* p) {
  if (p->opener.joinable() && p->opener.get_id() != std::this_thread::get_id()) p->opener.join();
  if (p->open_state.load() == 2) return fail(p->open_err);
  return 0;
}

static int prepare(dk_parquet* p) {
  hipStream_t s = p->stream;
  // the decode stream waits for the file images' H2D copies: table uploads and work-list expansion
  // go on the aux stream meanwhile (a pageable upload on a waiting stream would block the host)
  hipStream_t us = p->aux.s;
  using clk = std::chrono::steady_clock;
  auto since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  const auto t0 = clk::now();
  // 1. page headers were parsed on the host while the images were read (build_file_meta): size the
  // scratch areas from them right away, while the H2D copies still run
  DState st0{};
  st0.err_row = LLONG_MAX;
  if (upload_zc(p, p->d_state, &st0, sizeof st0, us)) return 1;
  p->open_ms[3] = since(t0);
  const auto t1 = clk::now();
  // header errors
  for (DPage& pg : p->h_pages) if (pg.status != PS_OK && pg.status != PS_UNSUPPORTED) return fail(page_status_msg(p, p->h_pages));
  for (const DPage& pg : p->h_pages) {   // every page body must lie inside the bytes that were read
    const FileM& f = p->files[p->col_file[p->h_chunks[pg.chunk].col]];
    if (pg.csize < 0 || pg.data_off + (int64_t)pg.csize > (int64_t)f.bytes.size())
      return fail("Error reading Parquet file: " + f.path + " (bad page header at offset " +
                  std::to_string(file_offset(f, pg.hdr_off)) + ")");
  }
  int64_t posn = 0, arena_n = 0, dbp_n = 0;
  // per-page work lists (fragments, segments, level tiles, position chunks) are expanded on the device
  // from per-group counts (k_expand): the host only builds the prefix arrays (one entry per page)
  std::vector<int32_t> cpage, fbase(1, 0), sbase(1, 0);
  for (size_t i = 0; i < p->h_pages.size(); i++) {
    DPage& pg = p->h_pages[i];
    DChunk& ck = p->h_chunks[pg.chunk];
    pg.unc_off = -1;
    if (ck.codec != CODEC_NONE) {
      if (ck.codec != CODEC_SNAPPY)
        return fail("Error reading Parquet file: " + p->files[p->col_file[ck.col]].path +
                    " (unsupported compression codec " + std::to_string(ck.codec) + ")");
      if (!(pg.ptype == PAGE_DATA_V2 && !pg.is_comp)) {
        const int64_t lv = pg.ptype == PAGE_DATA_V2 ? (int64_t)pg.rl_len + pg.dl_len : 0;
        // the decompressed body (after v2's uncompressed levels) starts 16-byte aligned, and the
        // page's region is padded to 16 bytes (k_snap_frag stores whole dwordx4 granules)
        pg.unc_off = ((arena_n + lv + 15) & ~(int64_t)15) - lv;
        arena_n = (pg.unc_off + (int64_t)pg.usize + 15) & ~(int64_t)15;
        p->has_compressed = true;
        const int64_t body = pg.usize > lv ? pg.usize - lv : 0;
        const int nf = body > 0 ? (int)((body + 65535) / 65536) : 1;   // k_snap_frag fragments (64 KiB)
        const int64_t cbody = pg.csize > lv ? pg.csize - lv : 0;
        const int ns = cbody > 0 ? (int)((cbody + DK_SNAP_SEG - 1) / DK_SNAP_SEG) : 1;
        sbase.push_back(sbase.back() + ns);
        cpage.push_back((int32_t)i);
        fbase.push_back(fbase.back() + nf);
      }
      pg.status = PS_OK;
    }
    if ((ck.phys == PT_INT32 || ck.phys == PT_INT64) && !(pg.flags & PF_DICT) && pg.enc == ENC_DELTA_BP) {
      pg.pos_base = dbp_n;
      dbp_n += (int64_t)pg.num_values + 1;
      p->has_dbp = true;
    }
    if (ck.phys == PT_BYTE_ARRAY) {
      if (pg.flags & PF_DICT) { ck.dict_pos = posn; }
      else pg.pos_base = posn;
      posn += (int64_t)pg.num_values + 1;
    }
  }
  // level tiles and run-table scratch (standard writers emit >= 8 values per hybrid run; a stream
  // with more than num_values / 4 + 64 runs is reported as unsupported)
  {
    std::vector<int32_t> tpage;              // tile groups: data pages with levels, in column order
    std::vector<int64_t> tbase(1, 0);
    int64_t runs_n = 0;
    for (DColumn& c : p->h_cols) {
      c.first_tile = (int)tbase.back();
      for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) {
        DPage& pg = p->h_pages[pi];
        const DChunk& ck = p->h_chunks[pg.chunk];
        const int nv = pg.num_values > 0 ? pg.num_values : 0;
        const int cap = nv / 4 + 64;
        const bool idx = pg.enc == ENC_PLAIN_DICT || pg.enc == ENC_RLE_DICT || (ck.phys == PT_BOOLEAN && pg.enc == ENC_RLE);
        pg.run_cap = cap;
        pg.run_r = pg.run_d = pg.run_i = 0;
        if (ck.max_rep > 0) { pg.run_r = runs_n; runs_n += cap; }
        if (ck.max_def > 0) { pg.run_d = runs_n; runs_n += cap; }
        if (idx) { pg.run_i = runs_n; runs_n += cap; }
        pg.first_tile = (int)tbase.back();
        pg.n_tiles = (nv + DK_LEVEL_TILE - 1) / DK_LEVEL_TILE;
        if (pg.n_tiles) { tpage.push_back(pi); tbase.push_back(tbase.back() + pg.n_tiles); }
      }
      c.n_tiles = (int)tbase.back() - c.first_tile;
    }
    p->n_ltiles = (int)tbase.back();
    // string-position chunks of every BYTE_ARRAY PLAIN data page and dictionary page (the region
    // is at most the page body; chunks past the region's end find nothing)
    std::vector<int32_t> ppage;
    std::vector<int64_t> pbase(1, 0);
    for (size_t pi = 0; pi < p->h_pages.size(); pi++) {
      DPage& pg = p->h_pages[pi];
      const DChunk& ck = p->h_chunks[pg.chunk];
      pg.pchunk0 = (int)pbase.back();
      pg.npchunk = 0;
      pg.pos_fail = 0;
      if (ck.phys != PT_BYTE_ARRAY || (!(pg.flags & PF_DICT) && pg.enc != ENC_PLAIN)) continue;
      const int64_t body = (pg.unc_off >= 0 ? pg.usize : pg.csize) + 16;
      pg.npchunk = (int)((body + DK_POS_CHUNK - 1) / DK_POS_CHUNK);
      ppage.push_back((int32_t)pi);
      pbase.push_back(pbase.back() + pg.npchunk);
    }
    p->n_pchunks = (int)pbase.back();
    if (p->d_pos_scratch.alloc(((size_t)p->n_pchunks * DK_POS_CAP + 8) * 2)) return 1;
    if (expand(p, us, p->d_pchunks, ppage, pbase, EX_POSCHUNK, sizeof(DPosChunk)) ||
        expand(p, us, p->d_ltiles, tpage, tbase, EX_TILE, sizeof(DTile)))
      return 1;
    if (p->d_runs.alloc((size_t)(runs_n + 1) * sizeof(Seg))) return 1;
  }
  if (p->d_pos.alloc((size_t)(posn + 16) * 4)) return 1;
  if (p->d_arena.alloc((size_t)arena_n + 256)) return 1;
  p->n_cpages = (int)cpage.size();
  p->n_frags = fbase.back();
  p->h_cpage = cpage; p->h_sbase = sbase; p->h_fbase = fbase;
  if (p->n_cpages) {
    std::vector<int64_t> fb(fbase.begin(), fbase.end()), sb(sbase.begin(), sbase.end());
    std::vector<int32_t> none;
    if (upload_zc(p, p->d_cpage, cpage.data(), cpage.size() * 4, us) || upload_zc(p, p->d_fbase, fbase.data(), fbase.size() * 4, us) ||
        expand(p, us, p->d_fwork, none, fb, EX_FRAG, sizeof(int2)) || p->d_fstart.alloc((size_t)p->n_frags * 8) ||
        p->d_serial.alloc(cpage.size() * 4) || upload_zc(p, p->d_sbase, sbase.data(), sbase.size() * 4, us) ||
        expand(p, us, p->d_spage, none, sb, EX_SEG, 4) ||
        p->d_snapws.alloc((size_t)sbase.back() * 4 * (8 + 2 * DK_SNAP_REC) + 64) ||
        p->d_snap_ob.alloc((size_t)sbase.back() * 8 + 8) || p->d_fseg.alloc((size_t)p->n_frags * 4 + 4))
      return 1;
    p->n_segs = sbase.back();
    if (snap_page_mode(p)) {
      // page mode: largest pages first (workgroups are dispatched in order; the long serial decodes
      // start early and the short ones fill in behind them)
      std::vector<int2> pwork(cpage.size());
      for (size_t i = 0; i < cpage.size(); i++) pwork[i] = make_int2((int)i, -1);
      std::stable_sort(pwork.begin(), pwork.end(), [&](const int2& a, const int2& b) {
        return p->h_pages[cpage[a.x]].usize > p->h_pages[cpage[b.x]].usize;
      });
      if (upload_zc(p, p->d_pwork, pwork.data(), pwork.size() * sizeof(int2), us)) return 1;
    }
    // page and hybrid modes find tags through a bitmap built by the speculative walk
    if ((snap_page_mode(p) || snap_hybrid(p)) && p->d_tbits.alloc(((size_t)p->n_segs * (DK_SNAP_SEG / 64) + 4) * 8)) return 1;
  }
  if (p->d_dbp.alloc((size_t)(dbp_n + 16) * 8)) return 1;
  p->bytes_arena = arena_n;
  if (upload_zc(p, p->d_chunks, p->h_chunks.data(), p->h_chunks.size() * sizeof(DChunk), us)) return 1;
  if (upload_zc(p, p->d_pages, p->h_pages.data(), p->h_pages.size() * sizeof(DPage), us)) return 1;
  // 2. count + scan to size the outputs (entries / chars are data dependent)
  for (DColumn& c : p->h_cols) { c.cap_entries = LLONG_MAX; c.cap_chars = LLONG_MAX; c.offs = nullptr; c.row_offs = nullptr; }
  if (upload_zc(p, p->d_cols, p->h_cols.data(), p->h_cols.size() * sizeof(DColumn), us)) return 1;
  {
    hipEvent_t ev = nullptr;
    HIPOK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPOK(hipEventRecord(ev, us));
    HIPOK(hipStreamWaitEvent(s, ev, 0));
    hipEventDestroy(ev);
  }
  p->open_ms[4] = since(t1);            // host: page tables, scratch sizing and allocation
  const auto t2 = clk::now();
  bool per_slice = false;                // outputs allocated and values decoded slice by slice
  std::vector<DColumn> got(p->h_cols.size());
  // the sizing passes, one slice of files at a time, each as soon as its files' images have landed
  // (the later files' H2D copies overlap the earlier slices' snappy / level passes); page mode is
  // never sliced. Adaptive (default): a slice is every file whose image has landed by the time the
  // previous slice is queued, at least 1/DK_OPEN_SLICES of the bytes (the host waits for more
  // files until it has that much, or the rest) -- each slice's passes have a fixed latency cost
  // (k_snap_fix's per-page chains), so fewer, larger slices once the reads have run ahead.
  // Asynchronous opens also allocate the outputs and decode the values slice by slice.
  {
    const int nf = (int)p->files.size();
    int64_t total = 0;
    for (const FileM& f : p->files) total += (int64_t)f.bytes.size();
    static const int want = getenv("DK_OPEN_SLICES") ? std::max(1, atoi(getenv("DK_OPEN_SLICES"))) : 8;
    const int slices = snap_page_mode(p) ? 1 : want;
    const int64_t target = std::max<int64_t>(1, total / slices);
    int f0 = 0;
    int64_t acc = 0;
    per_slice = slices > 1 && p->async_open;
    std::vector<SizedSlice> sized;
    if (per_slice) {
      // string-copy tiles: a bound from the headers (PLAIN byte-array data pages and key-column
      // dictionary pages, num_values >= the values the count pass finds)
      int64_t nt = 0;
      for (const DColumn& c : p->h_cols) {
        if (c.phys != PT_BYTE_ARRAY) continue;
        for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) {
          const DPage& pg = p->h_pages[pi];
          if (!(pg.flags & PF_DICT) && pg.enc == ENC_PLAIN) nt += (std::max(pg.num_values, 0) + DK_COPY_TILE - 1) / DK_COPY_TILE;
        }
      }
      for (const DChunk& ck : p->h_chunks)
        if (ck.dict_page >= 0 && p->h_cols[ck.col].key_hash && p->h_cols[ck.col].phys == PT_BYTE_ARRAY && p->h_cols[ck.col].max_rep == 0)
          nt += (std::max(p->h_pages[ck.dict_page].num_values, 0) + DK_COPY_TILE - 1) / DK_COPY_TILE;
      if (p->d_tiles.alloc((size_t)(nt + 1) * sizeof(int2))) return 1;
      p->col_tile0.assign(1, 0);
      p->copy_cb = 0;
      p->bytes_written = 0;
    }
    if (slices > 1) {
      // slices touch disjoint pages / segments / tiles / columns: they rotate over up to three
      // streams (DK_OPEN_STREAMS), so one slice's latency tail (k_snap_fix / k_snap_frag's longest
      // pages) overlaps the next slice's passes; `s` joins them all at the end
      static const int nss = getenv("DK_OPEN_STREAMS") ? std::max(1, std::min(3, atoi(getenv("DK_OPEN_STREAMS")))) : 3;
      hipStream_t ss[3] = {s, nullptr, nullptr};
      hipEvent_t tables = nullptr;
      if (nss > 1) {
        HIPOK(hipEventCreateWithFlags(&tables, hipEventDisableTiming));
        HIPOK(hipEventRecord(tables, s));          // the table uploads (s already waits for them)
        for (int k = 1; k < nss; k++) {
          if (!p->side[k - 1].s && p->side[k - 1].create()) return 1;
          ss[k] = p->side[k - 1].s;
          HIPOK(hipStreamWaitEvent(ss[k], tables, 0));
        }
      }
      if (per_slice && !p->dec.s && p->dec.create(true)) { if (tables) hipEventDestroy(tables); return 1; }
      // on any error return: drain the streams the loop queued work on, then free its events (the
      // remaining slices' and `tables`)
      struct LoopGuard {
        hipEvent_t& tables; std::vector<SizedSlice>& sized; hipStream_t* ss; int nss; hipStream_t dec; bool armed = true;
        ~LoopGuard() {
          if (!armed) return;
          for (int k = 0; k < nss; k++) if (ss[k]) hipStreamSynchronize(ss[k]);
          if (dec) hipStreamSynchronize(dec);
          for (SizedSlice& S : sized) if (S.ev) { hipEventDestroy(S.ev); S.ev = nullptr; }
          if (tables) { hipEventDestroy(tables); tables = nullptr; }
        }
      } guard{tables, sized, ss, nss, p->dec.s};
      int slice = 0;
      while (f0 < nf) {
        int f1 = f0;
        acc = 0;
        // at least `target` bytes (or the rest), then every file already landed
        for (;;) {
          if (f1 >= nf) break;
          if (acc >= target) {
            const int landed = is_queued(p, f1) ? ev_done(p->file_ev[f1]) : 0;
            if (landed < 0) return 1;
            if (!landed) break;
          }
          // while the next file lands, finish the sized slices whose passes are done (never block
          // the loop on them: the next slice is queued as soon as its files are in)
          while (per_slice) {
            const int landed = is_queued(p, f1) ? ev_done(p->file_ev[f1]) : 0;
            if (landed < 0) return 1;
            if (landed) break;
            const int sdone = sized.empty() ? 0 : ev_done(sized.front().ev);
            if (sdone < 0) return 1;
            if (sdone) {
              if (finish_slice(p, sized.front(), got)) return 1;
              sized.erase(sized.begin());
            } else if (p->queued && p->queued[f1].load() == 2) {
              break;
            } else {
              std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
          }
          if (!wait_queued(p, f1)) return 1;     // parquet_open reports the read error
          HIPOK(hipEventSynchronize(p->file_ev[f1]));
          acc += (int64_t)p->files[f1].bytes.size();
          f1++;
        }
        hipStream_t cs = ss[slice++ % nss];
        static const bool verbose = getenv("DK_VERBOSE") != nullptr;
        if (verbose) fprintf(stderr, "[dk] sizing slice %d: files [%d, %d) %.1f MB queued at %.1f ms\n", slice - 1, f0, f1,
                             acc / 1e6, since(p->t_open0));
        for (int f = f0; f < f1; f++) HIPOK(hipStreamWaitEvent(cs, p->file_ev[f], 0));
        // test hook (tests/test_async_open.py): an error in the middle of the sliced loop
        static const int inject = getenv("DK_INJECT_SLICE_FAULT") ? atoi(getenv("DK_INJECT_SLICE_FAULT")) : -1;
        if (slice - 1 == inject) return fail("injected fault in checkpoint open slice " + std::to_string(inject));
        const PRange R = file_range(p, f0, f1);
        sizing_stages(p, cs, R);
        if (per_slice) {
          // the slice's columns / pages back to pinned memory, then (one slice later, when its passes
          // have had the next files' landing time to run) its outputs and value decode
          SizedSlice S;
          S.R = R; S.cs = cs; S.f0 = f0; S.f1 = f1;
          if (S.cols.alloc((size_t)(R.col1 - R.col0) * sizeof(DColumn) + 16) || S.pages.alloc((size_t)(R.pb - R.pa) * sizeof(DPage) + 16))
            return 1;
          launch_copy_zc(S.cols.data(), p->d_cols.as<DColumn>() + R.col0, (long long)(R.col1 - R.col0) * sizeof(DColumn), cs);
          launch_copy_zc(S.pages.data(), p->d_pages.as<DPage>() + R.pa, (long long)(R.pb - R.pa) * sizeof(DPage), cs);
          HIPOK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
          sized.push_back(std::move(S));
          HIPOK(hipEventRecord(sized.back().ev, cs));
          for (;;) {
            const int sdone = sized.empty() ? 0 : ev_done(sized.front().ev);
            if (sdone < 0) return 1;
            if (!sdone) break;
            if (finish_slice(p, sized.front(), got)) return 1;
            sized.erase(sized.begin());
          }
        }
        f0 = f1;
      }
      while (!sized.empty()) {
        if (finish_slice(p, sized.front(), got)) return 1;
        sized.erase(sized.begin());
      }
      for (int k = 1; k < nss; k++) {               // `s` waits for the side streams' slices
        HIPOK(hipEventRecord(tables, ss[k]));
        HIPOK(hipStreamWaitEvent(s, tables, 0));
      }
      if (per_slice && p->dec.s) {                  // ... and for the slices' decode
        if (!tables) HIPOK(hipEventCreateWithFlags(&tables, hipEventDisableTiming));
        HIPOK(hipEventRecord(tables, p->dec.s));
        HIPOK(hipStreamWaitEvent(s, tables, 0));
      }
      guard.armed = false;
      if (tables) hipEventDestroy(tables);
    } else {
      for (int f = 0; f < nf; f++) {
        acc += (int64_t)p->files[f].bytes.size();
        if (!wait_queued(p, f)) return 1;
        HIPOK(hipStreamWaitEvent(s, p->file_ev[f], 0));
        if (f + 1 == nf || acc >= target) {
          sizing_stages(p, s, file_range(p, f0, f + 1));
          f0 = f + 1;
          acc = 0;
        }
      }
    }
  }
  if (!per_slice) {
    HIPOK(hipMemcpyAsync(got.data(), p->d_cols.p, got.size() * sizeof(DColumn), hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(p->h_pages.data(), p->d_pages.p, p->h_pages.size() * sizeof(DPage), hipMemcpyDeviceToHost, s));
  }
  HIPOK(hipStreamSynchronize(s));
  std::string m = page_status_msg(p, p->h_pages);
  if (!m.empty()) return fail(m);
  p->open_ms[5] = since(t2);            // sizing passes on the device (snappy, runs, counts, positions)
  if (getenv("DK_VERBOSE")) fprintf(stderr, "[dk] sizing done at %.1f ms\n", since(p->t_open0));
  const auto t3 = clk::now();
  // 3. string-copy tile table (page counts are final after the count pass), 4. output arena
  if (!per_slice) {
    std::vector<int2> tiles;
    p->col_tile0.assign(1, 0);
    p->copy_cb = 0;
    p->bytes_written = 0;
    build_tiles(p, 0, (int)p->h_cols.size(), tiles);
    if (upload(p->d_tiles, tiles.data(), tiles.size() * sizeof(int2), s)) return 1;
    if (alloc_outputs(p, 0, (int)p->h_cols.size(), got)) return 1;
  }
  if (!per_slice) {
    if (upload(p->d_cols, p->h_cols.data(), p->h_cols.size() * sizeof(DColumn), s)) return 1;
    if (upload(p->d_chunks, p->h_chunks.data(), p->h_chunks.size() * sizeof(DChunk), s)) return 1;   // dict_hash_off
  }
  HIPOK(hipStreamSynchronize(s));
  if (per_slice && check_state(p)) return 1;   // decode errors of the per-slice value decode
  {
    SyncedRelease drained;              // the zero-copy sources have been read
    p->staging.clear();
  }
  p->open_ms[6] = since(t3);            // host: tile tables + output arena
  if (!p->async_open) {                 // (an asynchronous open's mirrors are in use already)
    p->host.clear();
    p->host.resize(p->h_cols.size());
  }
  p->slice.assign(p->h_cols.size(), HostCol());
  p->prepared = true;
  p->fresh = true;
  p->decoded_fresh = per_slice;
  return 0;
}

// Select row groups [lo, hi) of a parsed file (hi < 0: to the end): the file then reads as just
// those rows (num_rows, row0) -- a shard of a checkpoint part, or row-group pruning.
static int select_row_groups(FileM& f, const std::vector<int32_t>& groups) {
  const int32_t n = (int32_t)f.rgs.size();
  for (size_t i = 0; i < groups.size(); i++)
    if (groups[i] < 0 || groups[i] >= n || (i && groups[i] <= groups[i - 1]))
      return fail("Error reading Parquet file: " + f.path + " (row groups out of range)");
  f.sel = groups;
  f.row0 = 0; f.num_rows = 0;
  for (int32_t g = 0; g < (groups.empty() ? n : groups[0]); g++) f.row0 += f.rgs[g].num_rows;
  for (int32_t g : groups) f.num_rows += f.rgs[g].num_rows;
  return 0;
}

static int select_row_groups(FileM& f, int32_t lo, int32_t hi) {
  const int32_t n = (int32_t)f.rgs.size();
  if (hi < 0) hi = n;
  if (lo < 0 || lo > hi || hi > n) return fail("Error reading Parquet file: " + f.path + " (row groups out of range)");
  std::vector<int32_t> g;
  for (int32_t i = lo; i < hi; i++) g.push_back(i);
  return select_row_groups(f, g);
}

// ------------------------------------------------------------------------------------------------
// Row-group pruning of checkpoint parts and sidecars (the checkpoint predicate, ActionsIterator.java:
// 336-351, handed to DefaultParquetHandler -> ParquetFileReader.java:111-132). The Kernel predicate
// is converted as ParquetFilterUtils.toParquetFilter does (KD/internal/parquet/ParquetFilterUtils.java:
// 63-440: comparators need a column and a non-null literal of a compatible type -- a literal on the
// left is swapped without flipping the operator --, AND keeps a convertible side, OR needs both,
// NOT wraps, IS_NULL / IS_NOT_NULL become eq / notEq(null); predicates on missing or repeated
// columns and anything else are dropped), then evaluated per row group by parquet-mr 1.12.3's
// StatisticsFilter (after LogicalInverseRewriter pushes NOT down) over the footer statistics as
// ParquetMetadataConverter.fromParquetStatisticsInternal reads them (min_value / max_value when the
// column has TYPE_DEFINED_ORDER or they are equal; the deprecated min / max only for signed sort
// orders and uncorrupted writers; float / double stats with a NaN carry no min / max, a +0.0 min
// reads as -0.0 and a -0.0 max as +0.0).
// ------------------------------------------------------------------------------------------------
namespace {
enum : int { RF_COL = 0, RF_LIT = 1, RF_NULL = 2, RF_EQ = 3, RF_LT = 4, RF_LE = 5, RF_GT = 6, RF_GE = 7, RF_AND = 8,
             RF_OR = 9, RF_NOT = 10, RF_ISNULL = 11, RF_ISNOTNULL = 12, RF_UNSUPPORTED = 13 };
// literal types (Kernel DataType of the literal)
enum : int { RL_LONG = 0, RL_INT = 1, RL_SHORT = 2, RL_BYTE = 3, RL_DATE = 4, RL_FLOAT = 5, RL_DOUBLE = 6, RL_BOOL = 7,
             RL_STRING = 8, RL_OTHER = 9 };
// parquet-mr filter node (after conversion); op: RF_EQ..RF_GE, RF_AND/OR/NOT, 20 = notEq
constexpr int PF_NOTEQ = 20;
struct PNode {
  int op = 0, leaf = -1, a = -1, b = -1;
  bool null_value = false;
  int64_t iv = 0; double dv = 0; std::string bv;   // the value in the column's primitive type
};
struct PItem { int kind = 0; int col = -1; int lt = 0; int64_t lit = 0; std::string str; int node = -1; };  // kind 0 col, 1 lit, 2 null lit, 3 filter (node -1: none)

int cmp_signed(int64_t a, int64_t b) { return a < b ? -1 : a > b ? 1 : 0; }
int cmp_unsigned(uint64_t a, uint64_t b) { return a < b ? -1 : a > b ? 1 : 0; }
int cmp_float(double a, double b) {                 // Float.compare / Double.compare
  const bool an = a != a, bn = b != b;
  if (an || bn) return an && bn ? 0 : an ? 1 : -1;
  if (a < b) return -1;
  if (a > b) return 1;
  if (a == 0 && b == 0) { const bool sa = std::signbit(a), sb = std::signbit(b); return sa == sb ? 0 : sa ? -1 : 1; }
  return 0;
}
int cmp_binary(const std::string& a, const std::string& b) {   // unsigned lexicographic, then length
  const size_t n = a.size() < b.size() ? a.size() : b.size();
  for (size_t i = 0; i < n; i++)
    if ((uint8_t)a[i] != (uint8_t)b[i]) return (uint8_t)a[i] < (uint8_t)b[i] ? -1 : 1;
  return a.size() < b.size() ? -1 : a.size() > b.size() ? 1 : 0;
}

// VersionParser + SemanticVersion for CorruptStatistics.shouldIgnoreStatistics (binary columns):
// ignore stats written by parquet-mr before 1.8.0 (except CDH 5.5-5.x backports), or when created_by
// is missing / unparseable
bool ignore_binary_stats(const std::string& created_by) {
  if (created_by.empty()) return true;
  // "<application> version <semver> (build <hash>)"
  const size_t sp = created_by.find(" version ");
  if (sp == std::string::npos) return true;
  const std::string app = created_by.substr(0, sp);
  if (app != "parquet-mr") return false;
  std::string ver = created_by.substr(sp + 9);
  const size_t end = ver.find(' ');
  if (end != std::string::npos) ver = ver.substr(0, end);
  int v[3] = {0, 0, 0};
  size_t i = 0;
  for (int k = 0; k < 3; k++) {
    if (i >= ver.size() || !isdigit((unsigned char)ver[i])) return true;
    while (i < ver.size() && isdigit((unsigned char)ver[i])) v[k] = v[k] * 10 + (ver[i++] - '0');
    if (k < 2) { if (i >= ver.size() || ver[i] != '.') return true; i++; }
  }
  const long sem = v[0] * 1000000L + v[1] * 1000L + v[2];
  return sem < 1008000L;
}

struct RGStats {          // parquet-mr Statistics of one column chunk
  bool has_minmax = false, nulls_set = false;
  int64_t nulls = 0, value_count = 0;
  int64_t imin = 0, imax = 0; double dmin = 0, dmax = 0; std::string bmin, bmax;
  bool empty() const { return !has_minmax && !nulls_set; }
};

bool decode_stat(const std::string& raw, int phys, int64_t* iv, double* dv, std::string* bv) {
  if (phys == PT_INT32) { if (raw.size() != 4) return false; int32_t x; memcpy(&x, raw.data(), 4); *iv = x; return true; }
  if (phys == PT_INT64) { if (raw.size() != 8) return false; int64_t x; memcpy(&x, raw.data(), 8); *iv = x; return true; }
  if (phys == PT_BOOLEAN) { if (raw.size() != 1) return false; *iv = raw[0] != 0; return true; }
  if (phys == PT_FLOAT) { if (raw.size() != 4) return false; float x; memcpy(&x, raw.data(), 4); *dv = x; return true; }
  if (phys == PT_DOUBLE) { if (raw.size() != 8) return false; double x; memcpy(&x, raw.data(), 8); *dv = x; return true; }
  *bv = raw;
  return true;
}

RGStats chunk_stats(const FileM& f, int leaf, const ColMeta& m) {
  RGStats r;
  r.value_count = m.num_values;
  if (!m.has_stats) return r;
  const LeafM& L = f.leaves[leaf];
  const StatsM& st = m.st;
  const bool typed_order = leaf < (int)f.col_order.size() && f.col_order[leaf] == 1;
  const bool is_bin = L.phys == PT_BYTE_ARRAY || L.phys == PT_FIXED;
  const bool signed_order = !(is_bin || (L.lt == LT_INT && !L.int_signed));
  const std::string *mn = nullptr, *mx = nullptr;
  if (st.has_min_value && st.has_max_value) {
    if (typed_order || st.min_value == st.max_value) { mn = &st.min_value; mx = &st.max_value; }
  } else if (st.has_min && st.has_max) {
    const bool ignore = is_bin && ignore_binary_stats(f.created_by);
    if (!ignore && (signed_order || st.min == st.max)) { mn = &st.min; mx = &st.max; }
  }
  if (mn && mx) {
    r.has_minmax = decode_stat(*mn, L.phys, &r.imin, &r.dmin, &r.bmin) && decode_stat(*mx, L.phys, &r.imax, &r.dmax, &r.bmax);
    if (r.has_minmax && (L.phys == PT_FLOAT || L.phys == PT_DOUBLE)) {
      if (r.dmin != r.dmin || r.dmax != r.dmax) r.has_minmax = false;   // NaN: no usable min / max
      else {
        if (cmp_float(r.dmin, 0.0) == 0) r.dmin = -0.0;
        if (cmp_float(r.dmax, -0.0) == 0) r.dmax = 0.0;
      }
    }
  }
  if (st.has_nulls) { r.nulls_set = true; r.nulls = st.null_count; }
  return r;
}

struct RGFilter {
  const FileM& f;
  std::vector<PNode> nodes;
  int cmp_min(const PNode& n, const RGStats& s) const {   // comparator().compare(min, value)
    const LeafM& L = f.leaves[n.leaf];
    if (L.phys == PT_FLOAT || L.phys == PT_DOUBLE) return cmp_float(s.dmin, n.dv);
    if (L.phys == PT_BYTE_ARRAY) return cmp_binary(s.bmin, n.bv);
    if (L.lt == LT_INT && !L.int_signed) return L.phys == PT_INT32 ? cmp_unsigned((uint32_t)s.imin, (uint32_t)n.iv) : cmp_unsigned((uint64_t)s.imin, (uint64_t)n.iv);
    return cmp_signed(s.imin, n.iv);
  }
  int cmp_max(const PNode& n, const RGStats& s) const {
    const LeafM& L = f.leaves[n.leaf];
    if (L.phys == PT_FLOAT || L.phys == PT_DOUBLE) return cmp_float(s.dmax, n.dv);
    if (L.phys == PT_BYTE_ARRAY) return cmp_binary(s.bmax, n.bv);
    if (L.lt == LT_INT && !L.int_signed) return L.phys == PT_INT32 ? cmp_unsigned((uint32_t)s.imax, (uint32_t)n.iv) : cmp_unsigned((uint64_t)s.imax, (uint64_t)n.iv);
    return cmp_signed(s.imax, n.iv);
  }
  // StatisticsFilter.canDrop with LogicalInverseRewriter's NOT push-down (neg)
  bool can_drop(int id, int g, bool neg) const {
    const PNode& n = nodes[id];
    if (n.op == RF_NOT) return can_drop(n.a, g, !neg);
    if (n.op == RF_AND || n.op == RF_OR) {
      const bool is_and = (n.op == RF_AND) != neg;            // not(and) = or(not, not)
      const bool l = can_drop(n.a, g, neg), r = can_drop(n.b, g, neg);
      return is_and ? (l || r) : (l && r);
    }
    int op = n.op;
    if (neg) op = op == RF_EQ ? PF_NOTEQ : op == PF_NOTEQ ? RF_EQ : op == RF_LT ? RF_GE : op == RF_LE ? RF_GT
                : op == RF_GT ? RF_LE : RF_LT;
    const RGStats s = chunk_stats(f, n.leaf, f.rgs[g].cols[n.leaf]);
    if (s.empty()) return false;
    const bool all_nulls = s.nulls_set && s.nulls == s.value_count;
    if (op == RF_EQ) {
      if (n.null_value) return s.nulls_set ? s.nulls == 0 : false;
      if (all_nulls) return true;
      if (!s.has_minmax) return false;
      return cmp_min(n, s) > 0 || cmp_max(n, s) < 0;
    }
    if (op == PF_NOTEQ) {
      if (n.null_value) return all_nulls;
      if (s.nulls_set && s.nulls > 0) return false;
      if (!s.has_minmax) return false;
      return cmp_min(n, s) == 0 && cmp_max(n, s) == 0;
    }
    if (all_nulls) return true;
    if (!s.has_minmax) return false;
    if (op == RF_LT) return cmp_min(n, s) >= 0;
    if (op == RF_LE) return cmp_min(n, s) > 0;
    if (op == RF_GT) return cmp_max(n, s) <= 0;
    return cmp_max(n, s) < 0;                                  // RF_GE
  }
};

// ParquetFilterUtils.canUseLiteral
bool can_use_literal(int lt, int64_t v, const LeafM& L) {
  const bool integer = lt == RL_BYTE || lt == RL_SHORT || lt == RL_INT || lt == RL_DATE ||
                       (lt == RL_LONG && (int64_t)(int32_t)v == v);
  const bool lng = lt == RL_LONG || lt == RL_BYTE || lt == RL_SHORT || lt == RL_INT || lt == RL_DATE;
  switch (L.phys) {
    case PT_BOOLEAN: return lt == RL_BOOL;
    case PT_INT32: return integer && (L.lt == LT_NONE || (L.lt == LT_INT && L.int_bits <= 32) || L.lt == LT_DATE);
    case PT_INT64: return lng && (L.lt == LT_NONE || (L.lt == LT_INT && L.int_bits <= 64));
    case PT_FLOAT: return lt == RL_FLOAT;
    case PT_DOUBLE: return lt == RL_DOUBLE;
    case PT_BYTE_ARRAY: return lt == RL_STRING && (L.lt == LT_NONE || L.lt == LT_STRING);
    default: return false;
  }
}
}  // namespace

extern "C" int dk_parquet_prune_row_groups(const char* path, const dk_rg_filter* flt, uint8_t* keep, int32_t cap,
                                           int32_t* n) {
  FileM f;
  f.path = path ? path : "";
  if (read_footer(f) || parse_footer(f)) return 1;
  *n = (int32_t)f.rgs.size();
  for (int32_t g = 0; g < *n && g < cap; g++) keep[g] = 1;
  if (!flt) return 0;
  if (flt->n_cols < 0 || flt->n_ops < 0 || flt->pool_len < 0 || (flt->n_cols && (!flt->col_off || !flt->col_len)) ||
      (flt->n_ops && (!flt->op || !flt->arg || !flt->lit)) || (flt->pool_len && !flt->pool))
    return fail("dk_parquet_prune_row_groups: bad filter");
  std::vector<int> col_leaf(flt->n_cols, -1);       // filter column -> non-repeated leaf of this file
  for (int c = 0; c < flt->n_cols; c++) {
    if (flt->col_off[c] < 0 || flt->col_len[c] < 0 || (int64_t)flt->col_off[c] + flt->col_len[c] > flt->pool_len)
      return fail("dk_parquet_prune_row_groups: bad column");
    const std::string name(flt->pool + flt->col_off[c], flt->col_len[c]);
    for (size_t li = 0; li < f.leaves.size(); li++)
      if (f.leaves[li].path == name && f.leaves[li].leaf_rep != 2) col_leaf[c] = (int)li;
  }
  RGFilter F{f, {}};
  std::vector<PItem> st;
  auto filt = [&](int node) { PItem it; it.kind = 3; it.node = node; return it; };
  for (int k = 0; k < flt->n_ops; k++) {
    const int op = flt->op[k];
    if (op == RF_COL) {
      if (flt->arg[k] < 0 || flt->arg[k] >= flt->n_cols) return fail("dk_parquet_prune_row_groups: bad column ref");
      PItem it; it.kind = 0; it.col = col_leaf[flt->arg[k]]; st.push_back(it);
    } else if (op == RF_LIT) {
      PItem it; it.kind = 1; it.lt = flt->arg[k]; it.lit = flt->lit[k];
      if (it.lt == RL_STRING) {
        const int64_t off = flt->lit[k] & 0xffffffffll, len = flt->lit[k] >> 32;
        if (off < 0 || len < 0 || off + len > flt->pool_len) return fail("dk_parquet_prune_row_groups: bad literal");
        it.str.assign(flt->pool + off, (size_t)len);
      }
      st.push_back(it);
    } else if (op == RF_NULL) {
      PItem it; it.kind = 2; st.push_back(it);
    } else if (op == RF_UNSUPPORTED) {
      st.push_back(filt(-1));
    } else if (op >= RF_EQ && op <= RF_GE) {
      if (st.size() < 2) return fail("dk_parquet_prune_row_groups: stack underflow");
      PItem b = st.back(); st.pop_back();
      PItem a = st.back(); st.pop_back();
      if (a.kind != 0 && b.kind == 0) std::swap(a, b);            // literal first: swapped, operator kept
      int node = -1;
      if (a.kind == 0 && b.kind == 1 && a.col >= 0) {
        const LeafM& L = f.leaves[a.col];
        if (can_use_literal(b.lt, b.lit, L) && (L.phys != PT_BOOLEAN || op == RF_EQ)) {
          PNode pn; pn.op = op; pn.leaf = a.col;
          if (L.phys == PT_FLOAT) { double d; memcpy(&d, &b.lit, 8); pn.dv = (float)d; }
          else if (L.phys == PT_DOUBLE) memcpy(&pn.dv, &b.lit, 8);
          else if (L.phys == PT_BYTE_ARRAY) pn.bv = b.str;
          else pn.iv = L.phys == PT_INT32 ? (int64_t)(int32_t)b.lit : b.lit;
          F.nodes.push_back(pn);
          node = (int)F.nodes.size() - 1;
        }
      }
      st.push_back(filt(node));
    } else if (op == RF_ISNULL || op == RF_ISNOTNULL) {
      if (st.empty()) return fail("dk_parquet_prune_row_groups: stack underflow");
      PItem a = st.back(); st.pop_back();
      int node = -1;
      if (a.kind == 0 && a.col >= 0) {
        const int ph = f.leaves[a.col].phys;
        if (ph == PT_BOOLEAN || ph == PT_INT32 || ph == PT_INT64 || ph == PT_FLOAT || ph == PT_DOUBLE || ph == PT_BYTE_ARRAY) {
          PNode pn; pn.op = op == RF_ISNULL ? RF_EQ : PF_NOTEQ; pn.leaf = a.col; pn.null_value = true;
          F.nodes.push_back(pn);
          node = (int)F.nodes.size() - 1;
        }
      }
      st.push_back(filt(node));
    } else if (op == RF_AND || op == RF_OR) {
      if (st.size() < 2) return fail("dk_parquet_prune_row_groups: stack underflow");
      const PItem b = st.back(); st.pop_back();
      const PItem a = st.back(); st.pop_back();
      const int l = a.kind == 3 ? a.node : -1, r = b.kind == 3 ? b.node : -1;
      int node = -1;
      if (l >= 0 && r >= 0) { PNode pn; pn.op = op; pn.a = l; pn.b = r; F.nodes.push_back(pn); node = (int)F.nodes.size() - 1; }
      else if (op == RF_AND) node = l >= 0 ? l : r;
      st.push_back(filt(node));
    } else if (op == RF_NOT) {
      if (st.empty()) return fail("dk_parquet_prune_row_groups: stack underflow");
      const PItem a = st.back(); st.pop_back();
      int node = -1;
      if (a.kind == 3 && a.node >= 0) { PNode pn; pn.op = RF_NOT; pn.a = a.node; F.nodes.push_back(pn); node = (int)F.nodes.size() - 1; }
      st.push_back(filt(node));
    } else {
      return fail("dk_parquet_prune_row_groups: bad opcode");
    }
  }
  if (st.size() != 1) return fail("dk_parquet_prune_row_groups: program must leave one value");
  const int root = st[0].kind == 3 ? st[0].node : -1;
  if (root < 0) return 0;                                      // nothing convertible: read everything
  for (int32_t g = 0; g < *n && g < cap; g++) keep[g] = F.can_drop(root, g, false) ? 0 : 1;
  return 0;
}

// Row groups of `path` whose leaf may hold a non-null value: those without statistics, or whose
// null_count is below the chunk's value count. The snapshot-load P&M pass only decodes these (the
// first non-null protocol / metaData row cannot lie in an all-null row group).
extern "C" int dk_parquet_nonnull_row_groups(const char* path, const char* leaf, uint8_t* keep, int32_t cap,
                                             int32_t* n) {
  FileM f;
  f.path = path ? path : "";
  if (read_footer(f) || parse_footer(f)) return 1;
  *n = (int32_t)f.rgs.size();
  const int idx = leaf ? leaf_index(f, leaf) : -1;
  if (idx == -2) return 1;
  for (int32_t g = 0; g < *n && g < cap; g++) {
    if (idx < 0) { keep[g] = 0; continue; }                 // a missing leaf is null everywhere
    const ColMeta& m = f.rgs[g].cols[idx];
    keep[g] = !(m.has_stats && m.st.has_nulls && m.st.null_count >= m.num_values);
  }
  return 0;
}

extern "C" int dk_parquet_row_groups(const char* path, int64_t* rows, int32_t cap, int32_t* n) {
  FileM f;
  f.path = path ? path : "";
  if (read_footer(f) || parse_footer(f)) return 1;
  *n = (int32_t)f.rgs.size();
  for (int32_t g = 0; g < *n && g < cap; g++) rows[g] = f.rgs[g].num_rows;
  return 0;
}

extern "C" int dk_parquet_open(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                               int32_t n_leaves, dk_parquet** out) {
  return dk_parquet_open_rg(e, paths, n_files, leaves, n_leaves, nullptr, nullptr, out);
}

static int parquet_open(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                        int32_t n_leaves, const std::vector<std::vector<int32_t>>* groups, dk_parquet** out,
                        const int32_t* field_ids = nullptr, const std::function<void(dk_parquet*)>* publish = nullptr);

// fn(i) for i in [0, n) on up to DK_IO_THREADS (default 16) host threads. (A persistent pool with
// prioritised jobs was measured against these per-call threads and lost: 188-193 / 192-206 ms with
// per-call threads against 206-209 / 206-207 ms pooled, async / default open, same box,
// profiles/r04/pool_ab.)
template <class F>
static void parallel_for(int n, F fn) {
  int nt = 16;
  if (const char* v = getenv("DK_IO_THREADS")) nt = atoi(v) > 0 ? atoi(v) : 1;
  if (nt > n) nt = n;
  if (nt <= 1) { for (int i = 0; i < n; i++) fn(i); return; }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  const uint64_t ticket = t_open_ticket;         // workers of an open wait only for older releases
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, ticket] { t_open_ticket = ticket; for (int i; (i = next.fetch_add(1)) < n;) fn(i); });
  for (auto& x : th) x.join();
}

// Many small host -> device uploads gathered into one pinned block and copied by kernels
// (launch_copy_zc): nothing waits on the DMA engines, which a concurrent checkpoint open keeps
// busy with file images. add() allocates the destination at once; flush() stages and launches.
struct ZcStage {
  struct Item { void* dst; const void* src; size_t n; };
  std::vector<Item> items;
  size_t total = 0;
  HBuf hb;
  int add(DBuf& d, const void* src, size_t n) {
    if (d.n < n || !d.p) if (d.alloc(n ? n : 16)) return 1;
    add_raw(d.p, src, n);
    return 0;
  }
  void add_raw(void* dst, const void* src, size_t n) {
    if (n) { items.push_back({dst, src, n}); total += (n + 15) & ~size_t(15); }
  }
  // the staging block must outlive the copies: the caller synchronizes the stream before `this` dies
  int flush(hipStream_t s) {
    if (!total) return 0;
    if (hb.alloc(total)) return 1;
    // staging copies in 1 MiB pieces over the host threads, then one copy kernel per item
    struct Piece { uint8_t* d; const uint8_t* s; size_t n; };
    std::vector<Piece> pieces;
    std::vector<size_t> at(items.size());
    size_t o = 0;
    for (size_t i = 0; i < items.size(); i++) {
      at[i] = o;
      for (size_t q = 0; q < items[i].n; q += (1 << 20))
        pieces.push_back({hb.data() + o + q, (const uint8_t*)items[i].src + q, std::min<size_t>(1 << 20, items[i].n - q)});
      o += (items[i].n + 15) & ~size_t(15);
    }
    parallel_for((int)pieces.size(), [&](int k) { memcpy(pieces[k].d, pieces[k].s, pieces[k].n); });
    for (size_t i = 0; i < items.size(); i++) launch_copy_zc(items[i].dst, hb.data() + at[i], (long long)items[i].n, s);
    items.clear();
    total = 0;
    return 0;
  }
};


extern "C" int dk_parquet_open_rg(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                                  int32_t n_leaves, const int32_t* rg_lo, const int32_t* rg_hi, dk_parquet** out) {
  if (!rg_lo && !rg_hi) return parquet_open(e, paths, n_files, leaves, n_leaves, nullptr, out);
  std::vector<std::vector<int32_t>> groups(n_files > 0 ? n_files : 0);
  for (int32_t fi = 0; fi < n_files; fi++) {
    FileM f;
    f.path = paths[fi];
    if (read_footer(f) || parse_footer(f)) return 1;
    const int32_t n = (int32_t)f.rgs.size();
    const int32_t lo = rg_lo ? rg_lo[fi] : 0, hi = rg_hi && rg_hi[fi] >= 0 ? rg_hi[fi] : n;
    if (lo < 0 || lo > hi || hi > n) return fail("Error reading Parquet file: " + f.path + " (row groups out of range)");
    for (int32_t g = lo; g < hi; g++) groups[fi].push_back(g);
  }
  return parquet_open(e, paths, n_files, leaves, n_leaves, &groups, out);
}

extern "C" int dk_parquet_open_sel(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                                   int32_t n_leaves, const int32_t* rg_count, const int32_t* rg_list, dk_parquet** out) {
  if (!rg_count) return parquet_open(e, paths, n_files, leaves, n_leaves, nullptr, out);
  std::vector<std::vector<int32_t>> groups(n_files > 0 ? n_files : 0);
  bool all = true;
  for (int32_t fi = 0, at = 0; fi < n_files; fi++) {
    if (rg_count[fi] < 0) {                       // every row group of this file
      FileM f;
      f.path = paths[fi];
      if (read_footer(f) || parse_footer(f)) return 1;
      for (int32_t g = 0; g < (int32_t)f.rgs.size(); g++) groups[fi].push_back(g);
      continue;
    }
    all = false;
    for (int32_t k = 0; k < rg_count[fi]; k++) groups[fi].push_back(rg_list[at + k]);
    at += rg_count[fi];
  }
  return parquet_open(e, paths, n_files, leaves, n_leaves, all ? nullptr : &groups, out);
}

// One file's share of the page / chunk / column tables, built (and its page headers parsed) on the
// host thread that read the file, with file-local indices; parquet_open concatenates them in file
// order. Page headers are parsed from the pinned image with the same code the device uses
// (apply_page_header, dk_thrift.h), so the sizing pass needs no device round trip first.
struct FileMeta {
  std::vector<DColumn> cols;
  std::vector<int> col_leaf;        // projected leaf of each local column
  std::vector<DChunk> chunks;       // .col: local column; .dict_page: local page
  std::vector<DPage> pages;         // .chunk: local chunk
  int64_t bytes_read = 0;
};

static int build_file_meta(const dk_parquet* p, int fi, const FileM& f, const std::vector<int>& leafidx, FileMeta& M) {
  const int n_leaves = (int)p->leaves.size();
  const uint8_t* img = f.bytes.data();
  const uint8_t* img_end = img + f.bytes.size();
  for (int li = 0; li < n_leaves; li++) {
    const int idx = leafidx[li];
    if (idx < 0) continue;
    const LeafM& L = f.leaves[idx];
    if (L.max_rep > 1) return fail("Error reading Parquet file: " + f.path + " (nested repetition not supported: " + L.path + ")");
    DColumn c{};
    c.phys = L.phys; c.width = L.phys == PT_BYTE_ARRAY ? 0 : phys_width(L.phys, L.type_length);
    c.max_def = L.max_def; c.max_rep = L.max_rep; c.rep_def = L.rep_def; c.present = 1;
    c.key_hash = p->leaves[li] == "add.path";   // the reconciliation key (ActiveAddFilesIterator)
    c.n_rows = 0;
    c.first_page = (int)M.pages.size();
    const int colid = (int)M.cols.size();
    const int chunk0 = (int)M.chunks.size();
    // chunks and pages in row-group order; data pages of a column stay contiguous
    std::vector<DPage> dicts;
    for (int32_t g : f.sel) {
      const ColMeta& m = f.rgs[g].cols[idx];
      c.n_rows += f.rgs[g].num_rows;
      DChunk ck{};
      ck.file = p->dfile[fi].as<uint8_t>();
      ck.col = colid;
      ck.phys = L.phys; ck.width = c.width; ck.max_def = L.max_def; ck.max_rep = L.max_rep; ck.rep_def = L.rep_def;
      ck.codec = m.codec; ck.dict_page = -1; ck.dict_pos = 0;
      const int chunk_id = (int)M.chunks.size();
      std::vector<PageRef> refs;
      if (enumerate_pages(f, m, refs)) return 1;
      M.bytes_read += m.total_compressed;
      for (const PageRef& r : refs) {
        DPage pg{};
        const uint8_t* hp = span_ptr(f, r.hdr_off, 1);
        if (!hp) return fail("Error reading Parquet file: " + f.path + " (page outside its column chunk)");
        pg.hdr_off = hp - img; pg.chunk = chunk_id; pg.flags = r.dict ? PF_DICT : 0; pg.unc_off = -1;
        apply_page_header(pg, ck, img, img_end);
        if (r.dict) { ck.dict_page = -2 - (int)dicts.size(); dicts.push_back(pg); }
        else M.pages.push_back(pg);
      }
      M.chunks.push_back(ck);
    }
    c.n_pages = (int)M.pages.size() - c.first_page;
    // dictionary pages go after the data pages (they are not part of the column's page range)
    for (size_t d = 0; d < dicts.size(); d++) {
      const int at = (int)M.pages.size();
      for (size_t k = chunk0; k < M.chunks.size(); k++) if (M.chunks[k].dict_page == -2 - (int)d) M.chunks[k].dict_page = at;
      M.pages.push_back(dicts[d]);
    }
    M.cols.push_back(c);
    M.col_leaf.push_back(li);
  }
  return 0;
}

static int parquet_open(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                        int32_t n_leaves, const std::vector<std::vector<int32_t>>* groups, dk_parquet** out,
                        const int32_t* field_ids, const std::function<void(dk_parquet*)>* publish) {
  if (!e) return fail("null engine");
  // this open's threads wait only for releases submitted before it started (a synchronous open on a
  // caller's thread takes its ticket here; the asynchronous opener brought its own)
  struct TicketScope {
    uint64_t saved;
    TicketScope() : saved(t_open_ticket) { if (t_open_ticket == UINT64_MAX) t_open_ticket = reaper().ticket(); }
    ~TicketScope() { t_open_ticket = saved; }
  } ticket_scope;
  hipSetDevice(e->cfg.device);
  std::unique_ptr<dk_parquet> p(new dk_parquet());
  p->eng = e;
  if (p->own.create()) return 1;
  p->stream = p->own.s;
  if (p->aux.create()) return 1;
  for (int k = 0; k < copy_streams(); k++) {
    if (p->copy[k].create_class(copy_class_on() ? kStreamCopy : kStreamNormal)) return 1;
    HIPOK(hipEventCreateWithFlags(&p->copy_done[k].e, hipEventDisableTiming));
  }
  p->timer.on = (e->cfg.flags & DK_FLAG_TIMING) != 0;
  for (int i = 0; i < n_leaves; i++) p->leaves.push_back(leaves[i]);
  p->files.resize(n_files);
  p->colmap.assign(n_files, std::vector<int>(n_leaves, -1));
  p->leafidx.assign(n_files, std::vector<int>(n_leaves, -1));
  p->dfile.resize(n_files);
  // host I/O in parallel over files (footer, row-group selection, projected column chunks):
  // DefaultParquetHandler reads files one after another; here every file of the call is in flight
  std::vector<std::string> errs(n_files > 0 ? n_files : 0);
  std::vector<FileMeta> metas(n_files > 0 ? n_files : 0);
  p->file_ev.resize(n_files > 0 ? n_files : 0);
  for (auto& ev : p->file_ev) HIPOK(hipEventCreateWithFlags(&ev.e, hipEventDisableTiming));
  const auto t_io0 = std::chrono::steady_clock::now();
  p->t_open0 = t_io0;
  if (getenv("DK_VERBOSE"))     // the timeline's origin on CLOCK_MONOTONIC (Python's time.monotonic)
    fprintf(stderr, "[dk] open of %d files starts at monotonic %.3f ms\n", n_files,
            std::chrono::duration<double, std::milli>(t_io0.time_since_epoch()).count());
  parallel_for(n_files, [&](int fi) {
    FileM& f = p->files[fi];
    f.path = paths[fi];
    if (read_footer(f) || parse_footer(f) ||
        (groups ? select_row_groups(f, (*groups)[fi]) : select_row_groups(f, 0, -1))) { errs[fi] = g_err; return; }
    // projection: only the chunks (and offset indexes) of the requested leaves travel to HBM
    std::vector<Span> want;
    for (int li = 0; li < n_leaves; li++) {
      const int idx = leaf_index(f, p->leaves[li], field_ids ? field_ids + (size_t)li * kMaxLeafDepth : nullptr);
      if (idx == -2) { errs[fi] = g_err; return; }
      p->leafidx[fi][li] = idx;
      if (idx < 0) continue;
      for (int32_t g : f.sel) {
        const ColMeta& m = f.rgs[g].cols[idx];
        want.push_back({chunk_start(m), m.total_compressed, 0});
        if (m.oi_off > 0 && m.oi_len > 0 && m.oi_off + m.oi_len <= f.size) want.push_back({m.oi_off, m.oi_len, 0});
      }
    }
    if (read_spans(f, want)) { errs[fi] = g_err; return; }
    hipSetDevice(e->cfg.device);
    if (p->dfile[fi].alloc(f.bytes.size() + 256)) { errs[fi] = g_err; return; }
  });
  for (int fi = 0; fi < n_files; fi++)
    if (!errs[fi].empty()) return fail(errs[fi]);
  if (getenv("DK_VERBOSE")) fprintf(stderr, "[dk] footers read at %.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_io0).count());
  // then only the offset indexes and page headers (pread in blocks): the page tables, and with them
  // the whole host half of prepare, are built before the column chunks are read (reading the headers
  // beside the image reads was no faster: both are CPU-bound on the box's share of cores)
  parallel_for(n_files, [&](int fi) {
    FileM& f = p->files[fi];
    HdrWin w;
    w.f = &f;
    w.fd = open(f.path.c_str(), O_RDONLY);
    if (w.fd < 0) { errs[fi] = "Error reading Parquet file: " + f.path + " (cannot open)"; return; }
    std::vector<PageRef> refs;
    for (int li = 0; li < n_leaves && errs[fi].empty(); li++) {
      const int idx = p->leafidx[fi][li];
      if (idx < 0) continue;
      for (int32_t g : f.sel) {
        refs.clear();
        if (enumerate_pages(f, f.rgs[g].cols[idx], refs, &w)) { errs[fi] = g_err; break; }
      }
    }
    close(w.fd);
    if (!errs[fi].empty()) return;
    if (build_file_meta(p.get(), fi, f, p->leafidx[fi], metas[fi])) errs[fi] = g_err;
  });
  for (int fi = 0; fi < n_files; fi++)
    if (!errs[fi].empty()) return fail(errs[fi]);
  if (getenv("DK_VERBOSE")) fprintf(stderr, "[dk] page headers read at %.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_io0).count());
  std::vector<std::string> rerrs(n_files > 0 ? n_files : 0);   // the reader's errors
  // then the images: read into pinned memory, each going to HBM in 8 MiB pieces on a copy stream while
  // the rest of it (and the other files) are still being read -- on background threads, while prepare
  // runs the sizing passes over the files whose copies have landed
  p->queued.reset(new std::atomic<int>[n_files > 0 ? n_files : 1]);
  for (int fi = 0; fi < n_files; fi++) p->queued[fi].store(0);
  // Pieces: every image cut into 8 MiB pieces, all threads working through them in file order, so
  // files land one after another from the first milliseconds on (one file per thread would land the
  // first file only after a sixteenth of the whole read); the thread that finishes a file's last
  // piece records its event.
  struct Piece { int fi; int64_t packed_off, len; };
  std::vector<Piece> pieces;
  const int64_t piece = piece_bytes();
  PinRing* ring = pin_ring(e->cfg.device);
  if (!ring->err.empty()) return fail(ring->err);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[n_files > 0 ? n_files : 1]);
  std::unique_ptr<int[]> fds(new int[n_files > 0 ? n_files : 1]);
  // A piece is a `piece`-byte window of the packed image, whatever spans it cuts; the window's spans
  // are read into it, then the whole window (padding between spans included) goes to HBM in one
  // copy. Cutting by span instead gave every small column chunk a copy of its own, which HIP runs as
  // a blit kernel on the copy stream between the DMA transfers (160 per stream per C3 step, ~20 ms
  // of each stream's time).
  for (int fi = 0; fi < n_files; fi++) {
    int n = 0;
    fds[fi] = -1;
    const FileM& f = p->files[fi];
    const int64_t size = f.spans.empty() ? 0 : f.spans.back().packed_off + f.spans.back().len;
    for (int64_t o = 0; o < size; o += piece, n++) pieces.push_back({fi, o, std::min<int64_t>(piece, size - o)});
    left[fi].store(n);
  }
  const uint64_t ticket = t_open_ticket;
  std::mutex rerr_mu;                             // every write of rerrs[] by the reader's threads
  std::thread reader([&, ticket] {
    t_open_ticket = ticket;
    {
      for (int fi = 0; fi < n_files; fi++) {
        fds[fi] = open(p->files[fi].path.c_str(), O_RDONLY);
        if (fds[fi] < 0) { rerrs[fi] = "Error reading Parquet file: " + p->files[fi].path + " (cannot open)"; p->queued[fi].store(2); }
        else if (left[fi].load() == 0) {              // nothing projected to read
          const bool rec = hipEventRecord(p->file_ev[fi], p->copy[fi % copy_streams()].s) == hipSuccess;
          if (!rec) { std::lock_guard<std::mutex> g(rerr_mu); rerrs[fi] = "hipEventRecord failed"; }
          p->queued[fi].store(rec ? 1 : 2, std::memory_order_release);
        }
      }
      parallel_for((int)pieces.size(), [&](int k) {
        const Piece& pc = pieces[k];
        FileM& f = p->files[pc.fi];
        if (p->queued[pc.fi].load(std::memory_order_acquire) == 2) return;
        if (p->abort_open.load(std::memory_order_relaxed)) {   // closed while opening: stop reading
          std::lock_guard<std::mutex> g(rerr_mu);
          if (rerrs[pc.fi].empty()) rerrs[pc.fi] = "Error reading Parquet file: " + f.path + " (reader closed)";
          p->queued[pc.fi].store(2, std::memory_order_release);
          return;
        }
        hipSetDevice(e->cfg.device);
        // a file's pieces share one copy stream (round-robin pieces over the streams were measured
        // slower: 171-176 against 153-181 ms at C3, the file's readiness then waits for every
        // stream, profiles/r06/ring_ab)
        hipStream_t cs = p->copy[pc.fi % copy_streams()].s;
        const int slot = ring->acquire();             // a pinned slot whose previous copy has landed
        bool ok = slot >= 0;
        uint8_t* buf = ok ? ring->slots[slot].p : nullptr;
        const int64_t w0 = pc.packed_off, w1 = w0 + pc.len;   // the parts of every span inside the window
        for (const Span& sp : f.spans) {
          if (!ok) break;
          const int64_t a = std::max(w0, sp.packed_off), b = std::min(w1, sp.packed_off + sp.len);
          if (a < b && pread_full(fds[pc.fi], buf + (a - w0), b - a, sp.file_off + (a - sp.packed_off))) ok = false;
        }
        const bool copied = ok && hipMemcpyAsync(p->dfile[pc.fi].as<uint8_t>() + pc.packed_off, buf, (size_t)pc.len,
                                                 hipMemcpyHostToDevice, cs) == hipSuccess;
        if (slot >= 0) ring->release(slot, copied ? cs : nullptr);
        ok = copied;
        if (!ok) {
          std::lock_guard<std::mutex> g(rerr_mu);
          if (rerrs[pc.fi].empty()) rerrs[pc.fi] = "Error reading Parquet file: " + f.path + " (short read)";
          p->queued[pc.fi].store(2, std::memory_order_release);
          return;
        }
        if (left[pc.fi].fetch_sub(1) == 1) {          // the file's last piece: its copies are all queued
          const bool rec = hipEventRecord(p->file_ev[pc.fi], cs) == hipSuccess;
          if (!rec) { std::lock_guard<std::mutex> g(rerr_mu); if (rerrs[pc.fi].empty()) rerrs[pc.fi] = "hipEventRecord failed"; }
          int expect = 0;
          p->queued[pc.fi].compare_exchange_strong(expect, rec ? 1 : 2, std::memory_order_acq_rel);
        }
      });
      if (getenv("DK_VERBOSE"))
        fprintf(stderr, "[dk] images read and queued at %.1f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p->t_open0).count());
      for (int fi = 0; fi < n_files; fi++) {
        if (fds[fi] >= 0) close(fds[fi]);
        int expect = 0;                               // (every file is settled by now)
        p->queued[fi].compare_exchange_strong(expect, 2);
        if (expect == 0 && rerrs[fi].empty()) rerrs[fi] = "Error reading Parquet file: " + p->files[fi].path + " (short read)";
      }
    }
  });
  struct Joiner { std::thread& t; ~Joiner() { if (t.joinable()) t.join(); } } joiner{reader};
  auto read_errors = [&]() -> int {
    if (reader.joinable()) reader.join();
    for (int fi = 0; fi < n_files; fi++)
      if (!rerrs[fi].empty()) return fail(rerrs[fi]);
    return 0;
  };
  const auto t_io1 = std::chrono::steady_clock::now();
  for (int fi = 0; fi < n_files; fi++) {             // concatenate the files' tables in file order
    FileMeta& M = metas[fi];
    const int col0 = (int)p->h_cols.size(), chunk0 = (int)p->h_chunks.size(), page0 = (int)p->h_pages.size();
    p->file_page0.push_back(page0);
    p->file_col0.push_back(col0);
    for (size_t k = 0; k < M.cols.size(); k++) {
      DColumn c = M.cols[k];
      c.first_page += page0;
      p->colmap[fi][M.col_leaf[k]] = col0 + (int)k;
      p->h_cols.push_back(c);
      p->col_file.push_back(fi);
    }
    for (DChunk ck : M.chunks) {
      ck.col += col0;
      if (ck.dict_page >= 0) ck.dict_page += page0;
      p->h_chunks.push_back(ck);
    }
    for (DPage pg : M.pages) {
      pg.chunk += chunk0;
      p->h_pages.push_back(pg);
    }
    p->bytes_read += M.bytes_read;
    M = FileMeta();
  }
  p->file_page0.push_back((int)p->h_pages.size());
  p->file_col0.push_back((int)p->h_cols.size());
  p->n_pages = (int)p->h_pages.size();
  p->n_cols = (int)p->h_cols.size();
  const auto t_h2d = std::chrono::steady_clock::now();
  // asynchronous open: the caller gets the handle now (the tables are final); reads, sizing and the
  // per-slice decode go on here, files becoming ready slice by slice (wait_files)
  bool published = false;
  auto failed = [&](int rc) -> int {
    if (!published) return rc;
    {
      std::lock_guard<std::mutex> g(p->rmu);
      p->open_err = g_err;
      p->open_state.store(2);
    }
    p->rcv.notify_all();
    p.release();                                  // the caller owns it
    return rc;
  };
  if (publish) {
    p->async_open = true;
    p->host.resize(p->h_cols.size());            // column mirrors (queued per file as files get ready)
    p->files_ready = 0;
    p->open_state.store(0);
    (*publish)(p.get());
    published = true;
  }
  if (prepare(p.get())) {
    const std::string perr = g_err;
    if (read_errors()) return failed(1);         // a failed read is the error to report
    return failed(fail(perr));
  }
  if (reader.joinable() && read_errors()) return failed(1);
  p->queued.reset();
  {
    const auto t_end = std::chrono::steady_clock::now();
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count(); };
    p->open_ms[0] = ms(t_io0, t_io1); p->open_ms[1] = ms(t_io1, t_h2d); p->open_ms[2] = ms(t_h2d, t_end);
    if (getenv("DK_VERBOSE")) {
      int64_t nb = 0;
      for (const FileM& f : p->files) nb += (int64_t)f.bytes.size();
      fprintf(stderr, "[dk] parquet_open %d files %.1f MB: io+h2d %.1f ms, metadata %.1f ms, prepare %.1f ms\n",
              n_files, nb / 1e6, p->open_ms[0], p->open_ms[1], p->open_ms[2]);
    }
  }
  if (published) {
    {
      std::lock_guard<std::mutex> g(p->rmu);
      p->files_ready = INT_MAX;
      p->open_state.store(1);
    }
    p->rcv.notify_all();
    p.release();
    return 0;
  }
  *out = p.release();
  return 0;
}

// The asynchronous form of dk_parquet_open_sel: returns once the footers, page headers and tables
// are read (num_rows / row_offset answer at once); the chunk reads, sizing passes and value decode
// continue on a thread of the handle, files becoming ready slice by slice. Every other call on the
// handle waits for what it needs (dk_parquet_column: its file; the rest: the whole open).
extern "C" int dk_parquet_open_async(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                                     int32_t n_leaves, const int32_t* rg_count, const int32_t* rg_list, dk_parquet** out) {
  *out = nullptr;
  const bool slice_decode = !(getenv("DK_SNAPPY_MODE") && !strcmp(getenv("DK_SNAPPY_MODE"), "page")) &&
                            !(getenv("DK_ASYNC_OPEN") && atoi(getenv("DK_ASYNC_OPEN")) == 0) &&
                            !(getenv("DK_OPEN_SLICES") && atoi(getenv("DK_OPEN_SLICES")) <= 1);
  if (!slice_decode) return dk_parquet_open_sel(e, paths, n_files, leaves, n_leaves, rg_count, rg_list, out);
  std::vector<std::vector<int32_t>> groups(n_files > 0 ? n_files : 0);
  bool all = true;
  if (rg_count) {
    for (int32_t fi = 0, at = 0; fi < n_files; fi++) {
      if (rg_count[fi] < 0) {
        FileM f;
        f.path = paths[fi];
        if (read_footer(f) || parse_footer(f)) return 1;
        for (int32_t g = 0; g < (int32_t)f.rgs.size(); g++) groups[fi].push_back(g);
        continue;
      }
      all = false;
      for (int32_t k = 0; k < rg_count[fi]; k++) groups[fi].push_back(rg_list[at + k]);
      at += rg_count[fi];
    }
  }
  std::promise<dk_parquet*> handed;
  std::future<dk_parquet*> got = handed.get_future();
  std::string early_err;
  std::function<void(dk_parquet*)> publish = [&](dk_parquet* q) { handed.set_value(q); };
  const std::vector<std::vector<int32_t>>* gp = (rg_count && !all) ? &groups : nullptr;
  const uint64_t ticket = reaper().ticket();     // releases older than this open
  std::thread t([&, gp, ticket] {
    t_open_ticket = ticket;
    dk_parquet* q = nullptr;
    bool pub = false;
    std::function<void(dk_parquet*)> pub_fn = [&](dk_parquet* x) { pub = true; publish(x); };
    if (parquet_open(e, paths, n_files, leaves, n_leaves, gp, &q, nullptr, &pub_fn) && !pub) {
      early_err = g_err;
      handed.set_value(nullptr);
    }
  });
  dk_parquet* p = got.get();
  if (!p) {
    t.join();
    return fail(early_err);
  }
  p->opener = std::move(t);
  *out = p;
  return 0;
}

static int invalidate_mirrors(dk_parquet* p);
extern "C" int dk_parquet_decode(dk_parquet* p) {
  if (ensure_open(p)) return 1;
  hipSetDevice(p->eng->cfg.device);
  DState st0{};
  st0.err_row = LLONG_MAX;
  HIPOK(hipMemcpyAsync(p->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, p->stream));
  KTimer::Scope sc(&p->timer, 12, p->stream);
  if (invalidate_mirrors(p)) return 1;
  return run_pipeline(p, 1);
}

static int check_state(dk_parquet* p) {
  DState st;
  HIPOK(hipMemcpy(&st, p->d_state.p, sizeof st, hipMemcpyDeviceToHost));
  if (st.err_flags & E_PAGE) {
    std::vector<DPage> pages(p->h_pages.size());
    HIPOK(hipMemcpy(pages.data(), p->d_pages.p, pages.size() * sizeof(DPage), hipMemcpyDeviceToHost));
    std::string m = page_status_msg(p, pages);
    return fail(m.empty() ? std::string("Error reading Parquet file: decode size mismatch") : m);
  }
  return 0;
}

extern "C" int dk_parquet_sync(dk_parquet* p) {
  if (ensure_open(p)) return 1;
  hipSetDevice(p->eng->cfg.device);   // this thread may not have used the device yet
  HIPOK(hipStreamSynchronize(p->stream));
  p->timer.collect();
  return check_state(p);
}

extern "C" int64_t dk_parquet_num_rows(dk_parquet* p, int32_t file) {
  if (!p || file < 0 || file >= (int)p->files.size()) return -1;
  return p->files[file].num_rows;
}

extern "C" int64_t dk_parquet_row_offset(dk_parquet* p, int32_t file) {
  if (!p || file < 0 || file >= (int)p->files.size()) return -1;
  return p->files[file].row0;
}

extern "C" int dk_parquet_open_ms(dk_parquet* p, double out[7]) {
  if (ensure_open(p)) return 1;
  for (int i = 0; i < 7; i++) out[i] = p->open_ms[i];
  return 0;
}

extern "C" int dk_parquet_traffic(dk_parquet* p, int64_t* r, int64_t* w) {
  if (ensure_open(p)) return 1;
  *r = p->bytes_read; *w = p->bytes_written; return 0;
}

// Algorithmic bytes of one launch of a decode kernel ("Roofline"): what the kernel must
// read and write at minimum, from the page / column metadata of the last prepare.
extern "C" int dk_parquet_kernel_traffic(dk_parquet* p, const char* kernel, int64_t* r, int64_t* w) {
  if (ensure_open(p)) return 1;
  if (!p || !kernel || !p->prepared) return fail("dk_parquet_kernel_traffic: not prepared");
  const std::string k = kernel;
  int64_t rd = 0, wr = 0;
  if (k == "k_probe") {
    // k_probe_fast_all (+ k_probe_cand_all): per add row the path definition level and decode-time
    // hash, a 4-byte fingerprint slot (at least), the selection byte; DV rows also read the DV leaves
    // (storageType / offset definition levels, the two string offsets and chars, the offset value)
    auto col = [&](size_t fi, const char* leaf) -> const DColumn* {
      for (size_t li = 0; li < p->leaves.size(); li++)
        if (p->leaves[li] == leaf) { const int ci = p->colmap[fi][li]; return ci >= 0 ? &p->h_cols[ci] : nullptr; }
      return nullptr;
    };
    for (size_t fi = 0; fi < p->files.size(); fi++) {
      const DColumn* path = col(fi, "add.path");
      if (!path) continue;
      const int64_t n = path->n_rows;
      rd += n * (1 + 8 + 4);
      wr += n;
      const DColumn* st = col(fi, "add.deletionVector.storageType");
      const DColumn* pid = col(fi, "add.deletionVector.pathOrInlineDv");
      if (st && pid && !st->null_only) {
        rd += n * (1 + 8 + 8 + 1 + 4) + st->n_chars + pid->n_chars;
      }
    }
    *r = rd; *w = wr;
    return 0;
  }
  for (size_t ci = 0; ci < p->h_cols.size(); ci++) {
    const DColumn& c = p->h_cols[ci];
    const bool key = c.hash != nullptr;
    for (int pi = c.first_page; pi < c.first_page + c.n_pages; pi++) {
      const DPage& pg = p->h_pages[pi];
      const int64_t body = pg.unc_off >= 0 ? pg.usize : pg.csize;
      const bool plain_str = c.phys == PT_BYTE_ARRAY && pg.enc == ENC_PLAIN;
      if (k == "k_string_copy") {
        if (plain_str) { rd += pg.vbytes; wr += pg.n_chars + (key ? 8ll * pg.n_values : 0); }
      } else if (k == "k_snap_frag") {
        // snappy pages: compressed body read, decompressed body written (v2 levels excluded)
        if (pg.unc_off >= 0) {
          const int64_t lv = pg.ptype == PAGE_DATA_V2 ? (int64_t)pg.rl_len + pg.dl_len : 0;
          rd += pg.csize - lv; wr += pg.usize - lv;
        }
      } else if (k == "k_tile_decode") {
        rd += body - pg.vbytes;                                   // level streams
        if (!plain_str) rd += pg.vbytes;                          // values / dictionary indices
        else rd += 4ll * pg.n_values + (key ? 8ll * pg.n_values : 0);   // positions (+ value hashes)
        wr += pg.n_rows;                                          // row_def
        if (c.max_rep > 0) wr += 8ll * pg.n_rows + pg.n_entries;  // row_offs, entry_def
        if (!c.null_only) {
          const int64_t nv = c.max_rep > 0 ? pg.n_entries : pg.n_rows;
          if (c.phys == PT_BYTE_ARRAY) wr += 8ll * nv + (plain_str ? 0 : pg.n_chars);   // offs (+ dict chars)
          else wr += (int64_t)c.width * nv;
        }
        if (key) wr += 8ll * pg.n_rows;                           // key hash per row
      } else {
        return fail("dk_parquet_kernel_traffic: no byte model for " + k);
      }
    }
    if (k == "k_snap_frag")                                       // snappy dictionary pages
      for (const DChunk& ck : p->h_chunks)
        if (ck.col == (int)ci && ck.dict_page >= 0) {
          const DPage& d = p->h_pages[ck.dict_page];
          if (d.unc_off >= 0) { rd += d.csize; wr += d.usize; }
        }
    if (k == "k_tile_decode")                                     // dictionary pages (read once)
      for (const DChunk& ck : p->h_chunks)
        if (ck.col == (int)ci && ck.dict_page >= 0) {
          const DPage& d = p->h_pages[ck.dict_page];
          rd += d.unc_off >= 0 ? d.usize : d.csize;
        }
  }
  *r = rd; *w = wr;
  return 0;
}

// an asynchronous open's mirrors are k_copy_zc kernels on a normal stream: DMA copies on a copy-class
// stream were no faster (profiles/r05/mirror_dma_ab)
static int create_mirror_stream(dk_parquet* p) { return p->mir.create(); }

// queue the D2H copy of decoded column ci into its pinned mirror (on the parquet stream, so it
// follows the decode that produced the column)
static int queue_mirror(dk_parquet* p, int ci) {
  const DColumn& c = p->h_cols[ci];
  HostMirror& h = p->host[ci];
  if (h.state) return 0;
  // own stream (an asynchronous open keeps queueing its passes on `stream`); while the open's H2D
  // copies are in flight the copies are made by a kernel into the pinned mirror (a DMA copy would
  // queue behind them)
  if (p->async_open && !p->mir.s && create_mirror_stream(p)) return 1;
  hipStream_t s = p->async_open ? p->mir.s : p->stream;
  if (p->async_open && p->open_state.load() != 0) {   // after the decode queued on `stream`
    if (!p->mir_ev) HIPOK(hipEventCreateWithFlags(&p->mir_ev, hipEventDisableTiming));
    HIPOK(hipEventRecord(p->mir_ev, p->stream));
    HIPOK(hipStreamWaitEvent(s, p->mir_ev, 0));
  }
  const int cf = p->col_file[ci];
  if (cf < (int)p->file_done.size() && p->file_done[cf]) HIPOK(hipStreamWaitEvent(s, p->file_done[cf], 0));
  if (cf < (int)p->file_dec.size() && p->file_dec[cf]) HIPOK(hipStreamWaitEvent(s, p->file_dec[cf], 0));
  const bool zc = p->async_open;
  auto d2h = [&](void* dst, const void* src, size_t n) -> int {
    if (!n) return 0;
    if (zc) { launch_copy_zc(dst, src, (long long)n, s); return 0; }
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s) == hipSuccess ? 0 : fail("hipMemcpyAsync failed");
  };
  const int64_t nv = c.max_rep > 0 ? c.n_entries : c.n_rows;
  if (h.row_def.alloc(c.n_rows + 1)) return 1;
  if (c.n_rows && d2h(h.row_def.data(), c.row_def, c.n_rows)) return 1;
  if (c.max_rep > 0) {
    if (h.row_offs.alloc((c.n_rows + 1) * 8) || h.entry_def.alloc(nv + 1)) return 1;
    if (c.null_only) { memset(h.row_offs.data(), 0, (c.n_rows + 1) * 8); memset(h.entry_def.data(), 0, nv + 1); }
    else {
      if (d2h(h.row_offs.data(), c.row_offs, (c.n_rows + 1) * 8)) return 1;
      if (nv && d2h(h.entry_def.data(), c.entry_def, nv)) return 1;
    }
  }
  if (c.phys == PT_BYTE_ARRAY) {
    if (h.offs.alloc((nv + 1) * 8) || h.chars.alloc(c.n_chars + 1)) return 1;
    if (c.null_only) memset(h.offs.data(), 0, (nv + 1) * 8);
    else {
      if (d2h(h.offs.data(), c.offs, (nv + 1) * 8)) return 1;
      if (c.n_chars && d2h(h.chars.data(), c.chars, c.n_chars)) return 1;
    }
  } else {
    if (h.fixed.alloc(nv * c.width + 1)) return 1;
    if (c.null_only) memset(h.fixed.data(), 0, nv * c.width + 1);
    else if (nv && d2h(h.fixed.data(), c.fixed, nv * c.width)) return 1;
  }
  if (!h.ev) HIPOK(hipEventCreateWithFlags(&h.ev, hipEventDisableTiming));
  HIPOK(hipEventRecord(h.ev, s));
  h.state = 1;
  return 0;
}

// a new decode overwrites the device columns: wait for copies in flight, then forget the mirrors
static int invalidate_mirrors(dk_parquet* p) {
  for (auto& h : p->host) {
    if (h.state == 1) HIPOK(hipEventSynchronize(h.ev));
    h.state = 0;
  }
  return 0;
}

extern "C" int dk_parquet_column(dk_parquet* p, int32_t file, int32_t leaf, dk_column* out) {
  hipSetDevice(p->eng->cfg.device);   // this thread may not have used the device yet
  memset(out, 0, sizeof *out);
  if (file < 0 || file >= (int)p->files.size() || leaf < 0 || leaf >= (int)p->leaves.size()) return fail("bad column index");
  int ci = p->colmap[file][leaf];
  out->n_rows = p->files[file].num_rows;
  if (ci < 0) { out->present = 0; return 0; }
  const DColumn& c = p->h_cols[ci];
  HostMirror& h = p->host[ci];
  if (wait_files(p, file + 1)) return 1;   // asynchronous open: this file's columns are final
  int ready;
  {
    std::lock_guard<std::mutex> g(p->rmu);
    ready = std::min(p->files_ready, (int)p->files.size());
  }
  if (h.state == 0)                    // first touch of this leaf: queue it for this and every later (ready) file
    for (int f = file; f < ready; f++)
      if (p->colmap[f][leaf] >= 0 && queue_mirror(p, p->colmap[f][leaf])) return 1;
  if (h.state == 1) { HIPOK(hipEventSynchronize(h.ev)); h.state = 2; }
  int64_t nv = c.max_rep > 0 ? c.n_entries : c.n_rows;
  out->n_entries = nv; out->n_chars = c.n_chars;
  out->phys = c.phys; out->width = c.width; out->max_def = c.max_def; out->max_rep = c.max_rep;
  out->rep_def = c.rep_def; out->present = 1;
  out->row_def = h.row_def.data();
  out->row_offs = c.max_rep > 0 ? (const int64_t*)h.row_offs.data() : nullptr;
  out->entry_def = c.max_rep > 0 ? h.entry_def.data() : nullptr;
  out->fixed = c.phys == PT_BYTE_ARRAY ? nullptr : h.fixed.data();
  out->offs = c.phys == PT_BYTE_ARRAY ? (const int64_t*)h.offs.data() : nullptr;
  out->chars = c.phys == PT_BYTE_ARRAY ? h.chars.data() : nullptr;
  return 0;
}

extern "C" int dk_parquet_first_row(dk_parquet* p, int32_t file, int32_t leaf, int32_t min_def, int64_t* row) {
  if (ensure_open(p)) return 1;
  *row = -1;
  if (file < 0 || file >= (int)p->files.size() || leaf < 0 || leaf >= (int)p->leaves.size()) return fail("bad column index");
  int ci = p->colmap[file][leaf];
  if (ci < 0) return 0;
  const DColumn& c = p->h_cols[ci];
  if (!c.n_rows) return 0;
  hipSetDevice(p->eng->cfg.device);
  hipStream_t s = p->stream;
  if (!p->d_first.p && p->d_first.alloc(8)) return 1;
  const unsigned long long none = ~0ull;
  HIPOK(hipMemcpyAsync(p->d_first.p, &none, 8, hipMemcpyHostToDevice, s));
  launch_first_row(c.row_def, c.n_rows, min_def, p->d_first.as<unsigned long long>(), s);
  unsigned long long got = none;
  HIPOK(hipMemcpyAsync(&got, p->d_first.p, 8, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  if (check_state(p)) return 1;
  *row = got == none ? -1 : (int64_t)got;
  return 0;
}

extern "C" int dk_parquet_column_rows(dk_parquet* p, int32_t file, int32_t leaf, int64_t row0, int64_t n,
                                      dk_column* out) {
  if (ensure_open(p)) return 1;
  hipSetDevice(p->eng->cfg.device);   // this thread may not have used the device yet
  memset(out, 0, sizeof *out);
  HIPOK(hipStreamSynchronize(p->stream));
  if (file < 0 || file >= (int)p->files.size() || leaf < 0 || leaf >= (int)p->leaves.size()) return fail("bad column index");
  if (row0 < 0 || n < 0 || row0 + n > p->files[file].num_rows) return fail("bad row range");
  int ci = p->colmap[file][leaf];
  out->n_rows = n;
  if (ci < 0) { out->present = 0; return 0; }
  const DColumn& c = p->h_cols[ci];
  HostCol& h = p->slice[ci];
  h = HostCol();
  h.row_def.resize(n);
  if (n) HIPOK(hipMemcpy(h.row_def.data(), c.row_def + row0, n, hipMemcpyDeviceToHost));
  int64_t v0 = row0, v1 = row0 + n;   // value range
  if (c.max_rep > 0) {
    h.row_offs.resize(n + 1);
    if (c.null_only) std::fill(h.row_offs.begin(), h.row_offs.end(), 0);
    else HIPOK(hipMemcpy(h.row_offs.data(), c.row_offs + row0, (n + 1) * 8, hipMemcpyDeviceToHost));
    v0 = h.row_offs[0]; v1 = h.row_offs[n];
    for (auto& o : h.row_offs) o -= v0;
    h.entry_def.resize(v1 - v0);
    if (v1 > v0) HIPOK(hipMemcpy(h.entry_def.data(), c.entry_def + v0, v1 - v0, hipMemcpyDeviceToHost));
  }
  const int64_t nv = v1 - v0;
  if (c.phys == PT_BYTE_ARRAY) {
    h.offs.assign(nv + 1, 0);
    if (!c.null_only) HIPOK(hipMemcpy(h.offs.data(), c.offs + v0, (nv + 1) * 8, hipMemcpyDeviceToHost));
    const int64_t c0 = h.offs[0];
    for (auto& o : h.offs) o -= c0;
    h.chars.resize(h.offs[nv]);
    if (!h.chars.empty()) HIPOK(hipMemcpy(h.chars.data(), c.chars + c0, h.chars.size(), hipMemcpyDeviceToHost));
  } else {
    h.fixed.assign(nv * c.width, 0);
    if (!c.null_only && nv) HIPOK(hipMemcpy(h.fixed.data(), c.fixed + v0 * c.width, nv * c.width, hipMemcpyDeviceToHost));
  }
  out->n_entries = nv; out->n_chars = (int64_t)h.chars.size();
  out->phys = c.phys; out->width = c.width; out->max_def = c.max_def; out->max_rep = c.max_rep;
  out->rep_def = c.rep_def; out->present = 1;
  out->row_def = h.row_def.data();
  out->row_offs = c.max_rep > 0 ? h.row_offs.data() : nullptr;
  out->entry_def = c.max_rep > 0 ? h.entry_def.data() : nullptr;
  out->fixed = c.phys == PT_BYTE_ARRAY ? nullptr : h.fixed.data();
  out->offs = c.phys == PT_BYTE_ARRAY ? h.offs.data() : nullptr;
  out->chars = c.phys == PT_BYTE_ARRAY ? h.chars.data() : nullptr;
  return 0;
}

extern "C" void dk_parquet_close(dk_parquet* p) {
  if (!p) return;
  p->abort_open.store(true);            // an open still reading stops at its next piece
  reaper().run([p] {
    ensure_open(p);
    hipSetDevice(p->eng->cfg.device);
    hipStreamSynchronize(p->stream);
    for (int k = 0; k < kCopyStreams; k++) if (p->copy[k].s) hipStreamSynchronize(p->copy[k].s);
    SyncedRelease drained;               // every buffer below is idle: back to the caches for reuse
    delete p;
  });
}

// ------------------------------------------------------------------------------------------------
// JSON commit tail (DefaultJsonHandler.readJsonFiles + DefaultJsonRow semantics, host side)
// ------------------------------------------------------------------------------------------------
namespace {

// Java UTF-8 decoding with replacement (InputStreamReader(UTF_8)): each maximal ill-formed
// subsequence becomes U+FFFD.
std::string java_utf8(const uint8_t* s, size_t n) {
  // valid runs are copied in bulk (ASCII eight bytes at a time); each maximal ill-formed subpart
  // becomes U+FFFD, as StandardCharsets.UTF_8.decode does
  std::string o;
  o.reserve(n);
  size_t i = 0, run = 0;                       // [run, i): valid, not yet appended
  while (i < n) {
    while (i + 8 <= n) {
      uint64_t w;
      memcpy(&w, s + i, 8);
      if (w & 0x8080808080808080ull) break;
      i += 8;
    }
    if (i >= n) break;
    if (s[i] < 0x80) { i++; continue; }
    uint32_t cp;
    int l = utf8_len_valid(s, (int64_t)i, (int64_t)n, &cp);
    if (l) { i += l; continue; }
    o.append((const char*)s + run, i - run);
    // maximal subpart length
    uint8_t b = s[i];
    int need = 0; uint8_t lo = 0x80, hi = 0xBF;
    if (b >= 0xC2 && b <= 0xDF) need = 1;
    else if (b >= 0xE0 && b <= 0xEF) { need = 2; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
    else if (b >= 0xF0 && b <= 0xF4) { need = 3; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
    size_t j = i + 1;
    for (int k = 0; k < need && j < n; k++, j++) {
      uint8_t c = s[j];
      uint8_t l2 = k == 0 ? lo : 0x80, h2 = k == 0 ? hi : 0xBF;
      if (c < l2 || c > h2) break;
    }
    o.append("\xEF\xBF\xBD");
    i = j;
    run = j;
  }
  o.append((const char*)s + run, n - run);
  return o;
}

enum JT { J_NULL, J_BOOL, J_NUM, J_STR, J_ARR, J_OBJ };
struct JNode {
  JT t = J_NULL;
  bool b = false;
  bool integral = false;
  std::string s;                                   // string value or raw number text
  std::vector<std::pair<std::string, int>> kv;      // object members (child node index)
  std::vector<int> arr;
};

// A parser over one JSON text whose nodes live in `nodes` from index 0. The nodes of an earlier
// parse are reused in place (their strings and vectors keep their capacity), so parsing one commit
// line after another allocates almost nothing once warm.
struct JParser {
  const char* p; const char* e;
  std::vector<JNode>& nodes;
  std::string err;
  size_t used = 0;
  std::vector<std::string>& keys;        // per nesting depth: the key being parsed (thread's buffers)
  static std::vector<std::string>& key_bufs() { static thread_local std::vector<std::string> k; return k; }
  JParser(const char* b, const char* en, std::vector<JNode>& n) : p(b), e(en), nodes(n), keys(key_bufs()) {}
  int alloc() {
    if (used < nodes.size()) {
      JNode& n = nodes[used];
      n.t = J_NULL; n.b = false; n.integral = false;
      n.s.clear(); n.kv.clear(); n.arr.clear();
    } else {
      nodes.emplace_back();
    }
    return (int)used++;
  }
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
  bool str(std::string& out) {
    if (p >= e || *p != '"') return false;
    p++;
    out.clear();
    while (p < e && *p != '"') {
      const char* q = p;                         // a run without escapes / control characters
      while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) q++;
      if (q > p) { out.append(p, q - p); p = q; continue; }
      unsigned char c = (unsigned char)*p;
      if (c < 0x20) return false;
      p++;
      if (p >= e) return false;
      char x = *p++;
      switch (x) {
        case '"': out.push_back('"'); break; case '\\': out.push_back('\\'); break; case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break; case 'f': out.push_back('\f'); break; case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break; case 't': out.push_back('\t'); break;
        case 'u': {
          auto hex4 = [&](uint32_t* v) {
            if (e - p < 4) return false;
            uint32_t r = 0;
            for (int k = 0; k < 4; k++) {
              char h = p[k]; r <<= 4;
              if (h >= '0' && h <= '9') r |= h - '0'; else if (h >= 'a' && h <= 'f') r |= h - 'a' + 10;
              else if (h >= 'A' && h <= 'F') r |= h - 'A' + 10; else return false;
            }
            p += 4; *v = r; return true;
          };
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else p = save;
          }
          // lone surrogates are encoded as 3 bytes (invalid UTF-8); key builders report them
          if (cp < 0x80) out.push_back((char)cp);
          else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 63))); }
          else if (cp < 0x10000) { out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 63))); out.push_back((char)(0x80 | (cp & 63))); }
          else { out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 63))); out.push_back((char)(0x80 | ((cp >> 6) & 63))); out.push_back((char)(0x80 | (cp & 63))); }
          break;
        }
        default: return false;
      }
    }
    if (p >= e) return false;
    p++;
    return true;
  }
  int value(int depth) {
    if (depth > 200) { err = "nesting too deep"; return -1; }
    ws();
    if (p >= e) { err = "unexpected end"; return -1; }
    int id = alloc();
    char c = *p;
    if (c == '{') {
      p++;
      nodes[id].t = J_OBJ;
      ws();
      if (p < e && *p == '}') { p++; return id; }
      if ((int)keys.size() <= depth) keys.resize(depth + 1);
      for (;;) {
        ws();
        std::string& k = keys[depth];
        if (!str(k)) { err = "bad object key"; return -1; }
        ws();
        if (p >= e || *p != ':') { err = "expected ':'"; return -1; }
        p++;
        int dup = -1;                             // ObjectNode.set: last wins, first position
        for (size_t m = 0; m < nodes[id].kv.size(); m++) if (nodes[id].kv[m].first == k) { dup = (int)m; break; }
        if (dup < 0) nodes[id].kv.push_back({k, -1});
        const int slot = dup < 0 ? (int)nodes[id].kv.size() - 1 : dup;
        int v = value(depth + 1);
        if (v < 0) return -1;
        nodes[id].kv[slot].second = v;
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') { p++; return id; }
        err = "expected ',' or '}'"; return -1;
      }
    }
    if (c == '[') {
      p++;
      nodes[id].t = J_ARR;
      ws();
      if (p < e && *p == ']') { p++; return id; }
      for (;;) {
        int v = value(depth + 1);
        if (v < 0) return -1;
        nodes[id].arr.push_back(v);
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; return id; }
        err = "expected ',' or ']'"; return -1;
      }
    }
    if (c == '"') {
      if (!str(nodes[id].s)) { err = "bad string"; return -1; }
      nodes[id].t = J_STR;
      return id;
    }
    if (e - p >= 4 && !memcmp(p, "null", 4)) { p += 4; nodes[id].t = J_NULL; return id; }
    if (e - p >= 4 && !memcmp(p, "true", 4)) { p += 4; nodes[id].t = J_BOOL; nodes[id].b = true; return id; }
    if (e - p >= 5 && !memcmp(p, "false", 5)) { p += 5; nodes[id].t = J_BOOL; nodes[id].b = false; return id; }
    if (c == '-' || (c >= '0' && c <= '9')) {
      const char* b = p;
      if (*p == '-') p++;
      if (p >= e || !(*p >= '0' && *p <= '9')) { err = "bad number"; return -1; }
      if (*p == '0' && p + 1 < e && p[1] >= '0' && p[1] <= '9') { err = "leading zero"; return -1; }
      while (p < e && *p >= '0' && *p <= '9') p++;
      bool integral = true;
      if (p < e && *p == '.') { integral = false; p++; if (p >= e || !(*p >= '0' && *p <= '9')) { err = "bad number"; return -1; } while (p < e && *p >= '0' && *p <= '9') p++; }
      if (p < e && (*p == 'e' || *p == 'E')) { integral = false; p++; if (p < e && (*p == '+' || *p == '-')) p++; if (p >= e || !(*p >= '0' && *p <= '9')) { err = "bad number"; return -1; } while (p < e && *p >= '0' && *p <= '9') p++; }
      nodes[id].t = J_NUM; nodes[id].integral = integral; nodes[id].s.assign(b, p - b);
      return id;
    }
    err = "unexpected character";
    return -1;
  }
};

bool parse_i64(const std::string& s, int64_t lo, int64_t hi, int64_t* out) {
  // integral text -> value if within [lo, hi]
  size_t i = 0; bool neg = false;
  if (s[0] == '-') { neg = true; i = 1; }
  __int128 v = 0;
  for (; i < s.size(); i++) { v = v * 10 + (s[i] - '0'); if (v > ((__int128)1 << 64)) return false; }
  if (neg) v = -v;
  if (v < lo || v > hi) return false;
  *out = (int64_t)v;
  return true;
}

// vectors whose resize leaves new elements uninitialized: the tail concatenation sizes its columns
// once and fills them from many threads, so the first touch of each page is spread over them too
template <class T>
struct NoInitAlloc : std::allocator<T> {
  using value_type = T;
  NoInitAlloc() = default;
  template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U> struct rebind { using other = NoInitAlloc<U>; };
  template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T> using RawVec = std::vector<T, NoInitAlloc<T>>;

// column builder in the dk_column layout
struct CB {
  int phys, width, max_def, max_rep, rep_def;
  RawVec<uint8_t> row_def, entry_def, fixed, chars;
  RawVec<int64_t> row_offs, offs;
  void init(int ph, int w, int md, int mr, int rd) { phys = ph; width = w; max_def = md; max_rep = mr; rep_def = rd; if (mr) row_offs.push_back(0); if (ph == PT_BYTE_ARRAY) offs.push_back(0); }
  // non-repeated
  void null_row(int def) { row_def.push_back((uint8_t)def); if (phys == PT_BYTE_ARRAY) offs.push_back((int64_t)chars.size()); else fixed.insert(fixed.end(), width, 0); }
  void str_row(const std::string& s) { row_def.push_back((uint8_t)max_def); chars.insert(chars.end(), s.begin(), s.end()); offs.push_back((int64_t)chars.size()); }
  void fix_row(const void* v) { row_def.push_back((uint8_t)max_def); fixed.insert(fixed.end(), (const uint8_t*)v, (const uint8_t*)v + width); }
  // repeated (map leaves): row begin / entry
  void map_row(int def) { row_def.push_back((uint8_t)def); }
  void map_end() { row_offs.push_back((int64_t)entry_def.size()); }
  void entry_str(const std::string* s) {
    if (s) { entry_def.push_back((uint8_t)max_def); chars.insert(chars.end(), s->begin(), s->end()); }
    else entry_def.push_back((uint8_t)(max_def - 1));
    offs.push_back((int64_t)chars.size());
  }
};

}  // namespace

static const char* JSON_LEAVES[] = {
    "add.path", "add.partitionValues.key_value.key", "add.partitionValues.key_value.value", "add.size",
    "add.modificationTime", "add.dataChange", "add.deletionVector.storageType", "add.deletionVector.pathOrInlineDv",
    "add.deletionVector.offset", "add.deletionVector.sizeInBytes", "add.deletionVector.cardinality",
    "add.tags.key_value.key", "add.tags.key_value.value", "add.baseRowId", "add.defaultRowCommitVersion", "add.stats",
    "remove.path", "remove.deletionVector.storageType", "remove.deletionVector.pathOrInlineDv",
    "remove.deletionVector.offset", "remove.deletionVector.sizeInBytes", "remove.deletionVector.cardinality"};
enum { JL_PATH, JL_PVK, JL_PVV, JL_SIZE, JL_MTIME, JL_DC, JL_DVST, JL_DVPID, JL_DVOFF, JL_DVSIZE, JL_DVCARD,
       JL_TGK, JL_TGV, JL_BRID, JL_DRCV, JL_STATS, JL_RPATH, JL_RDVST, JL_RDVPID, JL_RDVOFF, JL_RDVSIZE, JL_RDVCARD,
       JL_N };

struct dk_json_tail {
  int64_t rows = 0;
  int64_t ckpt_row0 = -1;             // rows from here on come from JSON checkpoint parts (-1: none)
  bool with_stats = false;
  CB col[JL_N];
  std::vector<int32_t> step, rowin;   // per row: batch step and row within batch
  int32_t n_steps = 0;
  // per parsed file: first row, first step and batches (dk_json_tail_file_steps / _rebase_steps)
  std::vector<int64_t> file_row0;
  std::vector<int32_t> file_step0, file_nsteps;
};

namespace {
struct JErr { std::string msg; };

const JNode* member(const std::vector<JNode>& N, const JNode& o, const char* k) {
  for (auto& m : o.kv) if (m.first == k) return &N[m.second];
  return nullptr;
}
std::string node_text(const std::vector<JNode>& N, const JNode& n);
std::string node_text(const std::vector<JNode>& N, const JNode& n) {
  switch (n.t) {
    case J_NULL: return "null";
    case J_BOOL: return n.b ? "true" : "false";
    case J_NUM: return n.s;
    case J_STR: return "\"" + n.s + "\"";
    case J_ARR: { std::string r = "["; for (size_t i = 0; i < n.arr.size(); i++) { if (i) r += ","; r += node_text(N, N[n.arr[i]]); } return r + "]"; }
    default: { std::string r = "{"; for (size_t i = 0; i < n.kv.size(); i++) { if (i) r += ","; r += "\"" + n.kv[i].first + "\":" + node_text(N, N[n.kv[i].second]); } return r + "}"; }
  }
}
[[noreturn]] void mismatch(const std::vector<JNode>& N, const JNode& n, const char* what) {
  throw JErr{"Couldn't decode " + node_text(N, n) + ", expected a " + what};
}
const JNode* field(const std::vector<JNode>& N, const JNode& o, const char* name, bool nullable) {
  const JNode* v = member(N, o, name);
  if (!v || v->t == J_NULL) {
    if (nullable) return nullptr;
    throw JErr{std::string("Root node at key ") + name + " is null but field isn't nullable. Root node: " + node_text(N, o)};
  }
  return v;
}
const std::string& as_str(const std::vector<JNode>& N, const JNode& n) { if (n.t != J_STR) mismatch(N, n, "string"); return n.s; }
int64_t as_long(const std::vector<JNode>& N, const JNode& n) {
  int64_t v;
  if (n.t != J_NUM || !n.integral || !parse_i64(n.s, LLONG_MIN, LLONG_MAX, &v)) mismatch(N, n, "long");
  return v;
}
int32_t as_int(const std::vector<JNode>& N, const JNode& n) {
  int64_t v;
  if (n.t != J_NUM || !n.integral || !parse_i64(n.s, INT_MIN, INT_MAX, &v)) mismatch(N, n, "integer");
  return (int32_t)v;
}
bool as_bool(const std::vector<JNode>& N, const JNode& n) { if (n.t != J_BOOL) mismatch(N, n, "boolean"); return n.b; }

void put_map(CB& k, CB& v, const std::vector<JNode>& N, const JNode* m, int null_def) {
  if (!m) { k.map_row(null_def); v.map_row(null_def); k.map_end(); v.map_end(); return; }
  if (m->t != J_OBJ) mismatch(N, *m, "map");
  int present = k.rep_def - 1;   // map defined
  k.map_row(m->kv.empty() ? present : k.rep_def);
  v.map_row(m->kv.empty() ? present : v.rep_def);
  for (auto& kv : m->kv) {
    const JNode& val = N[kv.second];
    k.entry_str(&kv.first);
    if (val.t == J_NULL) v.entry_str(nullptr);
    else v.entry_str(&as_str(N, val));
  }
  k.map_end(); v.map_end();
}

void put_dv(CB* c, const std::vector<JNode>& N, const JNode* dv, int add_def) {
  // c[0..4] = storageType, pathOrInlineDv, offset, sizeInBytes, cardinality (leaf max_def 3)
  if (!dv) { for (int i = 0; i < 5; i++) c[i].null_row(add_def); return; }
  if (dv->t != J_OBJ) mismatch(N, *dv, "object");
  const JNode* st = field(N, *dv, "storageType", false);
  const JNode* pid = field(N, *dv, "pathOrInlineDv", false);
  const JNode* off = field(N, *dv, "offset", true);
  const JNode* sz = field(N, *dv, "sizeInBytes", false);
  const JNode* card = field(N, *dv, "cardinality", false);
  c[0].str_row(as_str(N, *st));
  c[1].str_row(as_str(N, *pid));
  if (off) { int32_t v = as_int(N, *off); c[2].fix_row(&v); } else c[2].null_row(2);
  int32_t s = as_int(N, *sz); c[3].fix_row(&s);
  int64_t cd = as_long(N, *card); c[4].fix_row(&cd);
}
}  // namespace

// One commit file's rows in the tail layout (the files parse in parallel, then concatenate).
struct TailPart {
  int64_t rows = 0;
  CB col[JL_N];
  std::vector<int32_t> step, rowin;     // step local to the file
  int32_t n_steps = 0;
};

static void init_tail_cols(CB* c) {
  c[JL_PATH].init(PT_BYTE_ARRAY, 0, 2, 0, 0);
  c[JL_PVK].init(PT_BYTE_ARRAY, 0, 3, 1, 3);
  c[JL_PVV].init(PT_BYTE_ARRAY, 0, 4, 1, 3);
  c[JL_SIZE].init(PT_INT64, 8, 2, 0, 0);
  c[JL_MTIME].init(PT_INT64, 8, 2, 0, 0);
  c[JL_DC].init(PT_BOOLEAN, 1, 2, 0, 0);
  c[JL_DVST].init(PT_BYTE_ARRAY, 0, 3, 0, 0);
  c[JL_DVPID].init(PT_BYTE_ARRAY, 0, 3, 0, 0);
  c[JL_DVOFF].init(PT_INT32, 4, 3, 0, 0);
  c[JL_DVSIZE].init(PT_INT32, 4, 3, 0, 0);
  c[JL_DVCARD].init(PT_INT64, 8, 3, 0, 0);
  c[JL_TGK].init(PT_BYTE_ARRAY, 0, 3, 1, 3);
  c[JL_TGV].init(PT_BYTE_ARRAY, 0, 4, 1, 3);
  c[JL_BRID].init(PT_INT64, 8, 2, 0, 0);
  c[JL_DRCV].init(PT_INT64, 8, 2, 0, 0);
  c[JL_STATS].init(PT_BYTE_ARRAY, 0, 2, 0, 0);
  c[JL_RPATH].init(PT_BYTE_ARRAY, 0, 2, 0, 0);
  c[JL_RDVST].init(PT_BYTE_ARRAY, 0, 3, 0, 0);
  c[JL_RDVPID].init(PT_BYTE_ARRAY, 0, 3, 0, 0);
  c[JL_RDVOFF].init(PT_INT32, 4, 3, 0, 0);
  c[JL_RDVSIZE].init(PT_INT32, 4, 3, 0, 0);
  c[JL_RDVCARD].init(PT_INT64, 8, 3, 0, 0);
}

// DefaultJsonHandler.readJsonFiles over one commit: lines (BufferedReader.readLine: \n, \r or \r\n),
// each a JSON object decoded with DefaultJsonRow's rules for the add / remove read schema, in
// batches of J lines. Returns an error message or "".
static std::string parse_commit_file(const char* path, int J, bool with_stats, TailPart& P) {
  CB* c = P.col;
  init_tail_cols(c);
  std::vector<uint8_t> raw;
  FILE* fp = fopen(path, "rb");
  if (!fp) return std::string("Error reading JSON file: ") + path;
  fseek(fp, 0, SEEK_END); long n = ftell(fp); fseek(fp, 0, SEEK_SET);
  raw.resize(n > 0 ? n : 0);
  size_t got = n > 0 ? fread(raw.data(), 1, n, fp) : 0;
  fclose(fp);
  if ((long)got != n) return std::string("Error reading JSON file: ") + path;
  std::string text = java_utf8(raw.data(), raw.size());
  std::vector<JNode> N;
  size_t i = 0;
  int in_batch = 0;
  bool any = false;
  while (i < text.size()) {
    size_t j = i;
    while (j < text.size() && text[j] != '\n' && text[j] != '\r') j++;
    const char* lb = text.data() + i;
    const char* le = text.data() + j;
    if (j < text.size() && text[j] == '\r' && j + 1 < text.size() && text[j + 1] == '\n') j++;
    i = j + 1;
    JParser jp(lb, le, N);                      // N's nodes are reused line after line
    int root = jp.value(0);
    if (root >= 0) { jp.ws(); if (jp.p != jp.e) { root = -1; jp.err = "trailing characters"; } }
    if (root < 0) return std::string("Error reading JSON file: ") + path + " (" + jp.err + ")";
    if (in_batch == J) { P.n_steps++; in_batch = 0; }
    P.step.push_back(P.n_steps);
    P.rowin.push_back(in_batch++);
    any = true;
    try {
      const JNode& R = N[root];
      if (R.t != J_OBJ) mismatch(N, R, "object");
      const JNode* add = field(N, R, "add", true);
      const JNode* rm = field(N, R, "remove", true);
      if (add) {
        if (add->t != J_OBJ) mismatch(N, *add, "object");
        const JNode& A = *add;
        c[JL_PATH].str_row(as_str(N, *field(N, A, "path", false)));
        put_map(c[JL_PVK], c[JL_PVV], N, field(N, A, "partitionValues", false), 1);
        int64_t v = as_long(N, *field(N, A, "size", false)); c[JL_SIZE].fix_row(&v);
        v = as_long(N, *field(N, A, "modificationTime", false)); c[JL_MTIME].fix_row(&v);
        uint8_t b = as_bool(N, *field(N, A, "dataChange", false)); c[JL_DC].fix_row(&b);
        put_dv(&c[JL_DVST], N, field(N, A, "deletionVector", true), 1);
        put_map(c[JL_TGK], c[JL_TGV], N, field(N, A, "tags", true), 1);
        const JNode* x = field(N, A, "baseRowId", true);
        if (x) { v = as_long(N, *x); c[JL_BRID].fix_row(&v); } else c[JL_BRID].null_row(1);
        x = field(N, A, "defaultRowCommitVersion", true);
        if (x) { v = as_long(N, *x); c[JL_DRCV].fix_row(&v); } else c[JL_DRCV].null_row(1);
        if (with_stats) { x = field(N, A, "stats", true); if (x) c[JL_STATS].str_row(as_str(N, *x)); else c[JL_STATS].null_row(1); }
        else c[JL_STATS].null_row(1);
      } else {
        for (int k : {JL_PATH, JL_SIZE, JL_MTIME, JL_DC, JL_DVST, JL_DVPID, JL_DVOFF, JL_DVSIZE, JL_DVCARD, JL_BRID, JL_DRCV, JL_STATS})
          c[k].null_row(0);
        put_map(c[JL_PVK], c[JL_PVV], N, nullptr, 0);
        put_map(c[JL_TGK], c[JL_TGV], N, nullptr, 0);
      }
      if (rm) {
        if (rm->t != J_OBJ) mismatch(N, *rm, "object");
        c[JL_RPATH].str_row(as_str(N, *field(N, *rm, "path", false)));
        put_dv(&c[JL_RDVST], N, field(N, *rm, "deletionVector", true), 1);
      } else {
        for (int k : {JL_RPATH, JL_RDVST, JL_RDVPID, JL_RDVOFF, JL_RDVSIZE, JL_RDVCARD}) c[k].null_row(0);
      }
    } catch (const JErr& je) {
      return je.msg;
    }
    P.rows++;
  }
  if (any) P.n_steps++;
  return "";
}

// Concatenates the files' parts in file order: every destination is sized once, then the files
// copy (offsets rebased) into their slices in parallel and free their parts.
static void concat_tail(dk_json_tail* t, std::vector<TailPart>& parts, int n_checkpoint_files) {
  const int nf = (int)parts.size();
  struct Base { int64_t row_def, entry_def, fixed, chars, row_offs, offs; };
  std::vector<Base> base((size_t)(nf + 1) * JL_N);
  std::vector<int64_t> row0(nf + 1, 0);
  std::vector<int32_t> step0(nf + 1, 0);
  for (int k = 0; k < JL_N; k++) base[k] = Base{0, 0, 0, 0, 1, 1};
  for (int fi = 0; fi < nf; fi++) {
    const TailPart& P = parts[fi];
    for (int k = 0; k < JL_N; k++) {
      const CB& c = P.col[k];
      const Base& b = base[(size_t)fi * JL_N + k];
      base[(size_t)(fi + 1) * JL_N + k] = Base{b.row_def + (int64_t)c.row_def.size(), b.entry_def + (int64_t)c.entry_def.size(),
                                               b.fixed + (int64_t)c.fixed.size(), b.chars + (int64_t)c.chars.size(),
                                               b.row_offs + (int64_t)c.row_offs.size() - 1, b.offs + (int64_t)c.offs.size() - 1};
    }
    row0[fi + 1] = row0[fi] + P.rows;
    step0[fi + 1] = step0[fi] + P.n_steps;
  }
  for (int k = 0; k < JL_N; k++) {
    CB& d = t->col[k];
    const Base& e = base[(size_t)nf * JL_N + k];
    d.row_def.resize(e.row_def); d.entry_def.resize(e.entry_def); d.fixed.resize(e.fixed); d.chars.resize(e.chars);
    d.row_offs.resize(d.max_rep ? e.row_offs : 0); d.offs.resize(d.phys == PT_BYTE_ARRAY ? e.offs : 0);
  }
  t->rows = row0[nf];
  t->n_steps = step0[nf];
  t->step.resize(t->rows);
  t->rowin.resize(t->rows);
  t->file_row0.assign(row0.begin(), row0.end());
  t->file_step0.assign(step0.begin(), step0.begin() + nf);
  t->file_nsteps.resize(nf);
  if (n_checkpoint_files > 0) t->ckpt_row0 = row0[nf - n_checkpoint_files];
  parallel_for(nf, [&](int fi) {
    TailPart& P = parts[fi];
    for (int k = 0; k < JL_N; k++) {
      CB& d = t->col[k];
      const CB& c = P.col[k];
      const Base& b = base[(size_t)fi * JL_N + k];
      if (!c.row_def.empty()) memcpy(d.row_def.data() + b.row_def, c.row_def.data(), c.row_def.size());
      if (!c.entry_def.empty()) memcpy(d.entry_def.data() + b.entry_def, c.entry_def.data(), c.entry_def.size());
      if (!c.fixed.empty()) memcpy(d.fixed.data() + b.fixed, c.fixed.data(), c.fixed.size());
      if (!c.chars.empty()) memcpy(d.chars.data() + b.chars, c.chars.data(), c.chars.size());
      const int64_t ebase = d.max_rep ? b.entry_def : 0;
      for (size_t i = 1; i < c.row_offs.size(); i++) d.row_offs[b.row_offs + i - 1] = c.row_offs[i] + ebase;
      for (size_t i = 1; i < c.offs.size(); i++) d.offs[b.offs + i - 1] = c.offs[i] + b.chars;
    }
    for (int64_t i = 0; i < P.rows; i++) {
      t->step[row0[fi] + i] = step0[fi] + P.step[i];
      t->rowin[row0[fi] + i] = P.rowin[i];
    }
    t->file_nsteps[fi] = P.n_steps;
    P = TailPart();
  });
}

extern "C" int dk_json_tail_parse(dk_engine* e, const char* const* paths, const int64_t* versions, int32_t n_files,
                                  int32_t with_stats, dk_json_tail** out) {
  return dk_json_tail_parse_parts(e, paths, versions, n_files, 0, with_stats, out);
}

extern "C" int dk_json_tail_parse_parts(dk_engine* e, const char* const* paths, const int64_t* versions, int32_t n_files,
                                        int32_t n_checkpoint_files, int32_t with_stats, dk_json_tail** out) {
  (void)versions;
  if (!e) return fail("null engine");
  if (n_checkpoint_files < 0 || n_checkpoint_files > n_files) return fail("dk_json_tail_parse_parts: bad file counts");
  std::unique_ptr<dk_json_tail> t(new dk_json_tail());
  t->with_stats = with_stats != 0;
  init_tail_cols(t->col);
  const int J = e->cfg.json_batch_size;
  // commits parse in parallel (each starts its own batches); the first failing file in replay
  // order reports, as the sequential reader would
  std::vector<TailPart> parts(n_files > 0 ? n_files : 0);
  std::vector<std::string> errs(parts.size());
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  parallel_for(n_files, [&](int fi) { errs[fi] = parse_commit_file(paths[fi], J, t->with_stats, parts[fi]); });
  const auto t1 = clk::now();
  for (int fi = 0; fi < n_files; fi++)
    if (!errs[fi].empty()) return fail(errs[fi]);
  concat_tail(t.get(), parts, n_checkpoint_files);
  if (getenv("DK_VERBOSE"))
    fprintf(stderr, "[dk] commit tail: %d files, %lld rows: parse %.1f ms, concatenate %.1f ms\n", n_files,
            (long long)t->rows, std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(clk::now() - t1).count());
  *out = t.release();
  return 0;
}

// batches of each parsed file (a file's lines in batches of json_batch_size; an empty file has none)
extern "C" int dk_json_tail_file_steps(dk_json_tail* t, int32_t* steps) {
  if (!t || !steps) return fail("dk_json_tail_file_steps: null argument");
  for (size_t f = 0; f < t->file_nsteps.size(); f++) steps[f] = t->file_nsteps[f];
  return 0;
}

// first row of each parsed file, and the row count at the end (n_files + 1 entries)
extern "C" int dk_json_tail_file_row0(dk_json_tail* t, int64_t* row0) {
  if (!t || !row0) return fail("dk_json_tail_file_row0: null argument");
  for (size_t f = 0; f < t->file_row0.size(); f++) row0[f] = t->file_row0[f];
  return 0;
}

// Renumber the batch steps so that file f's first batch is step0[f]: a rank that parsed only its
// share of the commit files places its batches in the global replay order (ActionsIterator visits
// the commit files newest first, LogSegment.java:166-178), which the owner-partitioned
// reconciliation compares across ranks (R2 / R5: a remove tombstones adds of its own and later
// batches).
extern "C" int dk_json_tail_rebase_steps(dk_json_tail* t, const int32_t* step0) {
  if (!t || !step0) return fail("dk_json_tail_rebase_steps: null argument");
  const size_t nf = t->file_nsteps.size();
  for (size_t f = 0; f < nf; f++) {
    if (step0[f] < 0 || (int64_t)step0[f] + t->file_nsteps[f] > INT32_MAX - 1)
      return fail("dk_json_tail_rebase_steps: step out of range");
    const int32_t delta = step0[f] - t->file_step0[f];
    for (int64_t row = t->file_row0[f]; row < t->file_row0[f + 1]; row++) t->step[row] += delta;
    t->file_step0[f] = step0[f];
  }
  int32_t mx = 0;
  for (size_t f = 0; f < nf; f++) mx = std::max(mx, t->file_step0[f] + t->file_nsteps[f]);
  t->n_steps = mx;
  return 0;
}

extern "C" int64_t dk_json_tail_rows(dk_json_tail* t) { return t ? t->rows : -1; }
extern "C" int64_t dk_json_tail_checkpoint_row0(dk_json_tail* t) {
  return t ? (t->ckpt_row0 >= 0 ? t->ckpt_row0 : t->rows) : -1;
}

extern "C" int dk_json_tail_column(dk_json_tail* t, const char* leaf, dk_column* out) {
  memset(out, 0, sizeof *out);
  out->n_rows = t->rows;
  int k = -1;
  for (int i = 0; i < JL_N; i++) if (!strcmp(JSON_LEAVES[i], leaf)) k = i;
  if (k < 0 || (k == JL_STATS && !t->with_stats)) { out->present = 0; return 0; }
  CB& c = t->col[k];
  out->present = 1;
  out->phys = c.phys; out->width = c.width; out->max_def = c.max_def; out->max_rep = c.max_rep; out->rep_def = c.rep_def;
  out->n_entries = c.max_rep ? (int64_t)c.entry_def.size() : t->rows;
  out->n_chars = (int64_t)c.chars.size();
  out->row_def = c.row_def.data();
  out->row_offs = c.max_rep ? c.row_offs.data() : nullptr;
  out->entry_def = c.max_rep ? c.entry_def.data() : nullptr;
  out->fixed = c.phys == PT_BYTE_ARRAY ? nullptr : c.fixed.data();
  out->offs = c.phys == PT_BYTE_ARRAY ? c.offs.data() : nullptr;
  out->chars = c.phys == PT_BYTE_ARRAY ? c.chars.data() : nullptr;
  return 0;
}

extern "C" void dk_json_tail_free(dk_json_tail* t) {
  if (t) reaper().run([t] { delete t; });
}

// One commit line's protocol / metaData action decoded with DefaultJsonRow's rules for
// Protocol.FULL_SCHEMA / Metadata.FULL_SCHEMA (kernel-defaults/.../internal/data/DefaultJsonRow.java:
// 136-357; actions/Protocol.java:49-54, Metadata.java:57-72, Format.java:42-48): required fields
// missing or null fail ("Root node at key .. is null but field isn't nullable"), ints need an
// integral JSON number in int range, longs an integral number in long range, strings JSON strings,
// arrays JSON arrays without null elements, maps JSON objects without null values. The result is
// the action re-serialised with exactly the schema's fields (null where absent), for the host.
namespace {
void json_esc(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += (char)c;
  }
  o += '"';
}
void pm_str(std::string& o, const std::vector<JNode>& N, const JNode& obj, const char* k, bool nullable) {
  const JNode* v = field(N, obj, k, nullable);
  if (!v) { o += "null"; return; }
  json_esc(o, as_str(N, *v));
}
void pm_str_array(std::string& o, const std::vector<JNode>& N, const JNode& obj, const char* k, bool nullable) {
  const JNode* v = field(N, obj, k, nullable);
  if (!v) { o += "null"; return; }
  if (v->t != J_ARR) mismatch(N, *v, "array");
  o += '[';
  for (size_t i = 0; i < v->arr.size(); i++) {
    const JNode& e = N[v->arr[i]];
    if (e.t == J_NULL) throw JErr{"Array type expects no nulls as elements, but received `null` as array element"};
    if (i) o += ',';
    json_esc(o, as_str(N, e));
  }
  o += ']';
}
void pm_str_map(std::string& o, const std::vector<JNode>& N, const JNode& obj, const char* k, bool nullable) {
  const JNode* v = field(N, obj, k, nullable);
  if (!v) { o += "null"; return; }
  if (v->t != J_OBJ) mismatch(N, *v, "map");
  o += '{';
  for (size_t i = 0; i < v->kv.size(); i++) {
    const JNode& e = N[v->kv[i].second];
    if (e.t == J_NULL) throw JErr{"Map type expects no nulls in values, but received `null` as value"};
    if (i) o += ',';
    json_esc(o, v->kv[i].first);
    o += ':';
    json_esc(o, as_str(N, e));
  }
  o += '}';
}
}  // namespace

extern "C" int dk_json_pm_decode(const char* path, int64_t off, int64_t len, int32_t which, char* out, int64_t cap,
                                 int64_t* out_len) {
  FILE* fp = fopen(path, "rb");
  if (!fp) return fail(std::string("Error reading JSON file: ") + path);
  std::vector<uint8_t> raw(len > 0 ? len : 0);
  const bool ok = fseek(fp, (long)off, SEEK_SET) == 0 && (len <= 0 || fread(raw.data(), 1, len, fp) == (size_t)len);
  fclose(fp);
  if (!ok) return fail(std::string("Error reading JSON file: ") + path);
  const std::string text = java_utf8(raw.data(), raw.size());
  std::vector<JNode> N;
  JParser jp(text.data(), text.data() + text.size(), N);
  int root = jp.value(0);
  if (root >= 0) { jp.ws(); if (jp.p != jp.e) { root = -1; jp.err = "trailing characters"; } }
  if (root < 0) return fail(std::string("Error reading JSON file: ") + path + " (" + jp.err + ")");
  std::string o;
  try {
    const JNode& R = N[root];
    if (R.t != J_OBJ) mismatch(N, R, "object");
    const JNode* a = field(N, R, which == 0 ? "protocol" : "metaData", false);
    if (a->t != J_OBJ) mismatch(N, *a, "object");
    const JNode& A = *a;
    if (which == 0) {
      o += "{\"minReaderVersion\":" + std::to_string(as_int(N, *field(N, A, "minReaderVersion", false)));
      o += ",\"minWriterVersion\":" + std::to_string(as_int(N, *field(N, A, "minWriterVersion", false)));
      o += ",\"readerFeatures\":"; pm_str_array(o, N, A, "readerFeatures", true);
      o += ",\"writerFeatures\":"; pm_str_array(o, N, A, "writerFeatures", true);
      o += '}';
    } else {
      o += "{\"id\":"; pm_str(o, N, A, "id", false);
      o += ",\"name\":"; pm_str(o, N, A, "name", true);
      o += ",\"description\":"; pm_str(o, N, A, "description", true);
      const JNode* f = field(N, A, "format", false);
      if (f->t != J_OBJ) mismatch(N, *f, "object");
      o += ",\"format\":{\"provider\":"; pm_str(o, N, *f, "provider", false);
      o += ",\"options\":"; pm_str_map(o, N, *f, "options", true);
      o += "},\"schemaString\":"; pm_str(o, N, A, "schemaString", false);
      o += ",\"partitionColumns\":"; pm_str_array(o, N, A, "partitionColumns", false);
      const JNode* ct = field(N, A, "createdTime", true);
      o += ",\"createdTime\":" + (ct ? std::to_string(as_long(N, *ct)) : std::string("null"));
      o += ",\"configuration\":"; pm_str_map(o, N, A, "configuration", false);
      o += '}';
    }
  } catch (const JErr& je) {
    return fail(je.msg);
  }
  *out_len = (int64_t)o.size();
  if ((int64_t)o.size() > cap) return 2;                   // caller retries with *out_len bytes
  memcpy(out, o.data(), o.size());
  return 0;
}

// Snapshot-load P&M scan over the commit files (LogReplay.loadTableProtocolAndMetadata,
// internal/replay/LogReplay.java:220-314, reading PROTOCOL_METADATA_READ_SCHEMA through
// DefaultJsonHandler): files newest first, read 16 at a time on host threads, stopping after the
// block in which both actions have been seen. Per file: the first line whose top-level object has a
// non-null "protocol" / "metaData" (its line index and byte range), or -1. Only lines that contain
// one of the two key names (or a \u escape, the one other way to spell a key) are parsed.
extern "C" int dk_log_pm_scan(const char* const* paths, int32_t n, int64_t* p_line, int64_t* p_off, int64_t* p_len,
                              int64_t* m_line, int64_t* m_off, int64_t* m_len, int32_t* n_scanned) {
  for (int32_t i = 0; i < n; i++) { p_line[i] = m_line[i] = -1; p_off[i] = p_len[i] = m_off[i] = m_len[i] = 0; }
  *n_scanned = 0;
  std::vector<std::string> errs(n > 0 ? n : 0);
  auto scan = [&](int i) {
    FILE* fp = fopen(paths[i], "rb");
    if (!fp) { errs[i] = std::string("Error reading JSON file: ") + paths[i]; return; }
    fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET);
    std::vector<char> raw(sz > 0 ? sz : 0);
    const size_t got = sz > 0 ? fread(raw.data(), 1, sz, fp) : 0;
    fclose(fp);
    if ((long)got != sz) { errs[i] = std::string("Error reading JSON file: ") + paths[i]; return; }
    const char* b = raw.data();
    const size_t N = raw.size();
    std::vector<JNode> nodes;
    size_t at = 0;
    for (int64_t line = 0; at < N && (p_line[i] < 0 || m_line[i] < 0); line++) {
      size_t j = at;
      while (j < N && b[j] != '\n' && b[j] != '\r') j++;
      const std::string_view v(b + at, j - at);
      const size_t next = (j < N && b[j] == '\r' && j + 1 < N && b[j + 1] == '\n') ? j + 2 : j + 1;
      if (v.find("\"protocol\"") != std::string_view::npos || v.find("\"metaData\"") != std::string_view::npos ||
          v.find("\\u") != std::string_view::npos) {
        const std::string text = java_utf8((const uint8_t*)v.data(), v.size());
        nodes.clear();
        JParser jp(text.data(), text.data() + text.size(), nodes);
        const int root = jp.value(0);
        if (root < 0) { errs[i] = std::string("Error reading JSON file: ") + paths[i] + " (" + jp.err + ")"; return; }
        if (nodes[root].t == J_OBJ)
          for (auto& kv : nodes[root].kv) {
            if (nodes[kv.second].t == J_NULL) continue;
            if (kv.first == "protocol" && p_line[i] < 0) { p_line[i] = line; p_off[i] = (int64_t)at; p_len[i] = (int64_t)v.size(); }
            if (kv.first == "metaData" && m_line[i] < 0) { m_line[i] = line; m_off[i] = (int64_t)at; m_len[i] = (int64_t)v.size(); }
          }
      }
      at = next;
    }
  };
  // newest first, in batches of 16, 32, 64, ... files (a few thread launches for a long log; files
  // past the batch where both turn up are never looked at, as the sequential reader would not)
  bool hp = false, hm = false;
  for (int32_t b0 = 0, bs = 16; b0 < n; b0 += bs, bs = std::min(bs * 2, 512)) {
    const int32_t b1 = std::min<int32_t>(n, b0 + bs);
    parallel_for(b1 - b0, [&](int k) { scan(b0 + k); });
    for (int32_t i = b0; i < b1; i++) {             // in replay order: an error counts only before both are found
      if (!errs[i].empty()) return fail(errs[i]);
      hp = hp || p_line[i] >= 0;
      hm = hm || m_line[i] >= 0;
      *n_scanned = i + 1;
      if (hp && hm) return 0;
    }
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// replay
// ------------------------------------------------------------------------------------------------
// A compiled program (dk_skip_compile / dk_part_compile) installed in device memory: its image
// (dk_expr.h program_image) in one buffer and the kernel-argument struct of pointers into it. Wide
// skipping programs (> SK_NARROW paths) also own the per-lane scratch their kernels keep the values
// in (SkScratch: lanes x paths, sized to <= 256 MiB; grids are cut to the lanes).
struct DevSkip {
  dk_program prog;                      // host copy (paths: the stats_parsed leaves, the parsed schema)
  DBuf img, scratch;
  DSkipProg P{};
  SkScratch S{};
};
struct DevPart {
  dk_program prog;
  DBuf img;
  DPartProg P{};
};
static int install_skip(DevSkip& d, const dk_program& src) {
  if (src.kind != DK_PROGRAM_SKIPPING) return fail("not a data-skipping program");
  d.prog = src;
  int64_t offs[8];
  const std::string img = program_image(src, offs);
  if (d.img.alloc(img.size())) return 1;
  HIPOK(hipMemcpy(d.img.p, img.data(), img.size(), hipMemcpyHostToDevice));
  const char* b = d.img.as<char>();
  DSkipProg P{};
  P.n_paths = (int32_t)src.path_type.size();
  P.n_ops = (int32_t)src.op.size();
  for (auto& p : src.paths) P.max_comps = std::max<int32_t>(P.max_comps, (int32_t)p.size());
  P.path_type = (const int32_t*)(b + offs[0]);
  P.path_comp = (const int32_t*)(b + offs[1]);
  P.comp_off = (const int32_t*)(b + offs[2]);
  P.comp_len = (const int32_t*)(b + offs[3]);
  P.op = (const int32_t*)(b + offs[4]);
  P.arg = (const int32_t*)(b + offs[5]);
  P.lit = (const int64_t*)(b + offs[6]);
  P.names = b + offs[7];
  d.P = P;
  d.S = SkScratch{};
  if (P.n_paths > SK_NARROW) {
    const long long nw = (P.n_paths + 31) / 32;
    const long long per_lane = (long long)P.n_paths * 24 + nw * 4;
    long long lanes = ((256ll << 20) / per_lane) / 256 * 256;
    lanes = std::max(256ll, std::min(lanes, 65536ll));
    const size_t v = (size_t)lanes * P.n_paths * 8, w = (size_t)lanes * nw * 4, k = (size_t)lanes * P.n_paths * 4;
    if (d.scratch.alloc(v + w + 2 * k + v + 64)) return 1;
    char* q = d.scratch.as<char>();
    d.S.val = (long long*)q;
    d.S.ptr = (const uint8_t**)(q + v);
    d.S.setw = (uint32_t*)(q + 2 * v);
    d.S.kind = (int32_t*)(q + 2 * v + w);
    d.S.scale = (int32_t*)(q + 2 * v + w + k);
    d.S.lanes = lanes;
  }
  return 0;
}
static int install_part(DevPart& d, const dk_program& src) {
  if (src.kind != DK_PROGRAM_PARTITION) return fail("not a partition-pruning program");
  d.prog = src;
  int64_t offs[8];
  const std::string img = program_image(src, offs);
  if (d.img.alloc(img.size())) return 1;
  HIPOK(hipMemcpy(d.img.p, img.data(), img.size(), hipMemcpyHostToDevice));
  const char* b = d.img.as<char>();
  DPartProg P{};
  P.n_fields = (int32_t)src.field_type.size();
  P.n_ops = (int32_t)src.op.size();
  P.field_type = (const int32_t*)(b + offs[0]);
  P.name_off = (const int32_t*)(b + offs[1]);
  P.name_len = (const int32_t*)(b + offs[2]);
  P.op = (const int32_t*)(b + offs[4]);
  P.arg = (const int32_t*)(b + offs[5]);
  P.lit = (const int64_t*)(b + offs[6]);
  P.pool = b + offs[7];
  for (int32_t o : src.op) P.wide |= o == PO_FCMP2;
  d.P = P;
  return 0;
}

struct dk_replay {
  StreamH own;                          // the replay's stream (the checkpoint decode runs on it too)
  hipStream_t stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;   // ordering against the checkpoint's own stream
  hipEvent_t ev_pf = nullptr;                      // owner mode: the prefetched mirrors follow the decode
  dk_engine* eng = nullptr;
  dk_json_tail* tail = nullptr;
  dk_parquet* ck = nullptr;
  std::vector<DJsonAction> acts;
  std::vector<int64_t> act_row;        // tail row of each action
  DBuf d_acts, d_jchars, d_canon, d_slots, d_state, d_jsel;
  DBuf d_fp;                  // slot fingerprints for k_probe_fast (k_table_fp)
  DBuf d_cand, d_cand_n;      // probe candidates (rows needing the full key path)
  // data skipping (dk_replay_set_skipping): program + the tail's stats strings per action
  bool has_skip = false;
  DevSkip skip;                         // the program in device memory
  DevPart part;
  DBuf typed_buf;                       // TypedPath tables of the stats_parsed files
  std::vector<int> typed_paths;
  DBuf d_tstats_chars, d_tstats_off, d_tstats_len;
  std::vector<StatsRows> ck_stats;      // per checkpoint file (n = 0: no stats column)
  std::vector<StatsParsedRows> ck_parsed;   // per checkpoint file: stats_parsed columns (n = 0: JSON)
  // partition pruning (dk_replay_set_partition_filter): program + partitionValues maps
  bool has_part = false;
  MapRows tail_maps{};
  std::vector<MapRows> ck_maps;         // per checkpoint file (n = 0: no partitionValues leaves)
  std::vector<std::unique_ptr<DBuf>> map_bufs;
  std::vector<std::unique_ptr<DBuf>> d_csel;   // per checkpoint file
  std::vector<ProbeCols> probe;
  // one-launch probe over every checkpoint file (ProbeSet): per-file columns / row prefix / selection
  std::vector<ProbeCols> probe_run;      // the columns as launched (path hashes dropped on a reseed)
  std::vector<int64_t> probe_row0;
  std::vector<uint8_t*> probe_sel;
  DBuf d_probe_cols, d_probe_row0, d_probe_sel;
  bool probe_all = false;
  // hash(path)-owner exchange (dk_replay_set_exchange): this rank's share of the commit-tail path
  // hashes (sorted), per-chunk owner offsets, the send rows, and where the run stopped
  int32_t xw = 0, xr = 0;                 // world, rank (xw = 0: the local probe)
  DBuf d_owned, d_xbc, d_xtot, d_xg;
  int64_t n_owned = 0, n_send = 0;
  std::vector<unsigned long long> xtot;
  int32_t xphase = 0;                     // 1: counted (run), 2: packed, 3: finished
  // owner-partitioned reconciliation (dk_replay_set_owner, "owner" mode): this rank's commit-tail
  // actions are routed to the owners of their keys; this rank owns the keys with h mod ow == orank,
  // builds their table from the records routed to it (oacts / ocanon / oslots) and answers every
  // rank's checkpoint rows for them
  int32_t ow = 0, orank = 0;              // ow = 0: off
  int32_t ophase = 0;                     // OP_* below
  DBuf d_otot;                            // tail records / key bytes per owner (k_own_tail_count)
  DBuf d_osrc;                            // own action of each tail record, in send order
  DBuf d_orsum;                           // owner: key bytes per record chunk, then chunk offsets (+ total, bad)
  int64_t n_osend = 0;                    // tail records this rank sends
  DBuf d_oacts, d_ocanon, d_oslots, d_ofp, d_osel;
  int64_t n_oacts = 0;
  uint64_t omask = 0;
  DBuf d_rowh;                            // key hash per checkpoint row (global row order)
  int64_t n_ocand = 0;                    // checkpoint candidates (found by hash at their owner)
  DBuf d_oc_plen, d_oc_dlen, d_oc_own, d_oc_rpos, d_oc_koff, d_oc_sendg, d_ov_koff;
  uint64_t mask = 0;
  uint32_t seed = 0;
  KTimer timer;
  std::vector<uint8_t> h_jsel;
  DState h_state{};
  bool have_result = false;
  // every checkpoint file's selection bytes in one pinned block (dk_replay_ckpt_selection_host)
  HBuf h_csel;
  // grouped runs: the error states (replay, checkpoint) after the tail and after each group, and the
  // tail's selection bytes, written into pinned memory by a copy kernel before the event (a small
  // hipMemcpy would queue on the DMA engines behind the groups' selection / mirror copies)
  HBuf h_zstate, h_zjsel;
  std::vector<int64_t> h_csel_off;
  bool h_csel_ready = false;
  // grouped run (dk_replay_run_grouped): the checkpoint files in n_groups runs, each decoded, probed,
  // filtered and its selections copied to h_csel before the next; grp_ev[g] after group g's copies
  int32_t n_groups = 0;
  std::vector<int32_t> grp_f0;            // first file of each group (n_groups + 1 entries)
  std::vector<int> prefetch;              // leaves mirrored to the host per group (dk_replay_prefetch_leaf)
  // attached to a checkpoint whose open is still running (dk_parquet_open_async): per-file probe
  // columns, maps and stats rows are filled as the files get ready (attach_upto), and a grouped run
  // issues each group when the consumer first waits on one of its files (issue_group)
  bool lazy = false;
  bool run_lazy = false;                  // this run overlaps the open (the open decodes the values)
  std::vector<uint8_t> attached;
  int grp_issued = 0;
  uint64_t h_nodv = 0;
  HBuf h_probe_cols, h_st0;
  std::vector<hipEvent_t> grp_ev;
  hipEvent_t ev_tail = nullptr;           // after the commit-tail half (its selection is final)
  std::vector<int64_t> grp_row0;          // per group: its files' row prefix, rebased (probe_all)
  DBuf d_grp_row0;
  std::vector<uint8_t> file_ready;        // dk_replay_wait_file passed for the file
  bool tail_ready = false;
  StreamH aux;                            // error-state reads while a grouped run is in flight
};

static const DColumn* find_col(dk_parquet* p, int fi, const char* leaf) {
  for (size_t li = 0; li < p->leaves.size(); li++)
    if (p->leaves[li] == leaf) { int ci = p->colmap[fi][li]; return ci >= 0 ? &p->h_cols[ci] : nullptr; }
  return nullptr;
}
// the file's schema leaf behind a projected leaf (logical type, timestamp unit, decimal scale)
static const LeafM* find_leafm(dk_parquet* p, int fi, const char* leaf) {
  for (size_t li = 0; li < p->leaves.size(); li++)
    if (p->leaves[li] == leaf) { int x = p->leafidx[fi][li]; return x >= 0 ? &p->files[fi].leaves[x] : nullptr; }
  return nullptr;
}

// The checkpoint half of a replay: selection buffers, probe columns, partition maps and stats rows
// of every checkpoint file. Separate from the commit-tail half so that the tail's action table and
// key table are built while the checkpoint files are still being read (dk_replay_attach_checkpoint).
// one checkpoint file's probe columns, partition map and stats rows (its columns are final)
static void attach_file(dk_replay* r, dk_parquet* ckpt, size_t fi) {
  ProbeCols pc{};
  const DColumn* path = find_col(ckpt, (int)fi, "add.path");
  pc.n_rows = ckpt->files[fi].num_rows;
  if (!path) pc.n_rows = 0;
  else {
    pc.path_def = path->row_def; pc.path_offs = path->offs; pc.path_chars = path->chars;
    pc.path_hash = path->hash;
    const DColumn* st = find_col(ckpt, (int)fi, "add.deletionVector.storageType");
    const DColumn* pid = find_col(ckpt, (int)fi, "add.deletionVector.pathOrInlineDv");
    const DColumn* off = find_col(ckpt, (int)fi, "add.deletionVector.offset");
    if (st && pid) {
      pc.has_dv = 1;
      pc.st_def = st->row_def; pc.st_offs = st->offs; pc.st_chars = st->chars;
      pc.pid_offs = pid->offs; pc.pid_chars = pid->chars;
      if (off) { pc.off_def = off->row_def; pc.off_vals = (const int32_t*)off->fixed; pc.off_maxdef = off->max_def; }
    }
  }
  r->probe[fi] = pc;
  MapRows M{};
  const DColumn* kc = find_col(ckpt, (int)fi, "add.partitionValues.key_value.key");
  const DColumn* vc = find_col(ckpt, (int)fi, "add.partitionValues.key_value.value");
  M.n = ckpt->files[fi].num_rows;
  if (kc && vc && kc->row_offs && kc->offs && vc->entry_def && vc->offs) {
    M.row_def = kc->row_def; M.rep_def = kc->rep_def; M.v_max_def = vc->max_def;
    M.row_offs = kc->row_offs; M.k_offs = kc->offs; M.k_chars = kc->chars;
    M.v_def = vc->entry_def; M.v_offs = vc->offs; M.v_chars = vc->chars;
  }                            // else no map entry anywhere (or no map leaf): every field is null
  r->ck_maps[fi] = M;
  StatsRows R{};
  const DColumn* sc = find_col(ckpt, (int)fi, "add.stats");
  if (sc && !sc->null_only && sc->offs) {
    R.n = ckpt->files[fi].num_rows;
    R.row_def = sc->row_def; R.max_def = sc->max_def;
    R.offs = sc->offs; R.chars = sc->chars;
  }
  r->ck_stats[fi] = R;
  r->attached[fi] = 1;
}

// attach files [0, f1) (waiting for an asynchronous open to make them ready)
static int attach_upto(dk_replay* r, int f1) {
  if (!r->ck) return 0;
  f1 = std::min(f1, (int)r->ck->files.size());
  if (wait_files(r->ck, f1)) return 1;
  for (int f = 0; f < f1; f++) if (!r->attached[f]) attach_file(r, r->ck, (size_t)f);
  return 0;
}

// The checkpoint half of a replay: selection buffers, probe columns, partition maps and stats rows
// of every checkpoint file. Separate from the commit-tail half so that the tail's action table and
// key table are built while the checkpoint files are still being read (dk_replay_attach_checkpoint).
// With the checkpoint's open still running, the per-file parts wait for their files (attach_upto).
static int replay_attach(dk_replay* r, dk_parquet* ckpt) {
  r->ck = ckpt;
  if (hipEventCreateWithFlags(&r->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&r->ev_out, hipEventDisableTiming) != hipSuccess)
    return fail("hipEventCreate failed");
  if (ckpt) {
    const size_t nf = ckpt->files.size();
    int64_t max_rows = 1, total = 0;
    for (size_t fi = 0; fi < nf; fi++) {
      max_rows = std::max<int64_t>(max_rows, ckpt->files[fi].num_rows);
      total += ckpt->files[fi].num_rows;
    }
    // every file in one probe launch while global row numbers fit the int32 candidate list
    r->probe_all = nf > 1 && total < (1ll << 31) - 1;
    if (r->d_cand.alloc((size_t)(r->probe_all ? total : max_rows) * 4 + 64)) return 1;
    if (r->d_cand_n.alloc(64)) return 1;
    for (size_t fi = 0; fi < nf; fi++) {
      r->d_csel.emplace_back(new DBuf());
      if (r->d_csel.back()->alloc(ckpt->files[fi].num_rows + 16)) return 1;
    }
    r->probe.assign(nf, ProbeCols{});
    r->ck_maps.assign(nf, MapRows{});
    r->ck_stats.assign(nf, StatsRows{});
    r->attached.assign(nf, 0);
    r->lazy = ckpt->open_state.load() == 0;
    if (!r->lazy) for (size_t fi = 0; fi < nf; fi++) attach_file(r, ckpt, fi);
  }
  return 0;
}

extern "C" int dk_replay_create(dk_engine* e, dk_json_tail* tail, dk_parquet* ckpt, dk_replay** out) {
  if (!e) return fail("null engine");
  const auto t_create0 = std::chrono::steady_clock::now();
  hipSetDevice(e->cfg.device);
  ZcStage zs;   // declared before r: r's stream is synchronized before the staging block is freed
  std::unique_ptr<dk_replay> r(new dk_replay());
  r->eng = e; r->tail = tail;
  if (r->own.create(replay_high_priority())) return 1;
  r->stream = r->own.s;
  r->timer.on = (e->cfg.flags & DK_FLAG_TIMING) != 0;
  hipStream_t s = r->stream;
  // actions: removes and adds of each tail row (a row may carry both), built in parallel over row
  // blocks. Their strings stay in the tail's columns: d_jchars holds the character buffers of the
  // six key columns back to back and each action points into it.
  static const int kKeyCols[6] = {JL_PATH, JL_RPATH, JL_DVST, JL_DVPID, JL_RDVST, JL_RDVPID};
  int64_t jbase[JL_N] = {};
  int64_t jchars_n = 0;
  if (tail) for (int k : kKeyCols) { jbase[k] = jchars_n; jchars_n += (int64_t)tail->col[k].chars.size(); }
  int64_t canon_n = 0;
  std::vector<int64_t> arow, soff;
  std::vector<int32_t> slen;
  if (tail) {
    const CB* c = tail->col;
    const int64_t R = tail->rows;
    const int nb = (int)std::min<int64_t>(64, std::max<int64_t>(1, R / 2048));
    std::vector<int64_t> b_na(nb + 1, 0), b_canon(nb + 1, 0);
    // rows of a JSON checkpoint part: adds are checkpoint adds, removes are ignored
    // (ActiveAddFilesIterator.java:163-183 reads tombstones only from commit files)
    auto each = [&](int bi, bool fill) {
      const int64_t r0 = R * bi / nb, r1 = R * (bi + 1) / nb;
      int64_t ai = fill ? b_na[bi] : 0, co = fill ? b_canon[bi] : 0;   // (counting: this block's own)
      for (int64_t row = r0; row < r1; row++) {
        const bool ck = tail->ckpt_row0 >= 0 && row >= tail->ckpt_row0;
        for (int kind : {JA_REMOVE, JA_ADD}) {
          if (ck && kind == JA_REMOVE) continue;
          const int pk = kind == JA_ADD ? JL_PATH : JL_RPATH;
          const CB& pc = c[pk];
          if (pc.row_def[row] < 1) continue;
          const int sk = kind == JA_ADD ? JL_DVST : JL_RDVST, ik = kind == JA_ADD ? JL_DVPID : JL_RDVPID;
          const CB& st = c[sk];
          const bool has_dv = st.row_def[row] >= 2;
          const int32_t path_len = (int32_t)(pc.offs[row + 1] - pc.offs[row]);
          const int32_t st_len = has_dv ? (int32_t)(st.offs[row + 1] - st.offs[row]) : 0;
          const int32_t pid_len = has_dv ? (int32_t)(c[ik].offs[row + 1] - c[ik].offs[row]) : 0;
          if (fill) {
            DJsonAction a{};
            a.kind = ck ? JA_CKADD : kind; a.step = tail->step[row]; a.row = tail->rowin[row];
            a.path_off = jbase[pk] + pc.offs[row]; a.path_len = path_len;
            a.has_dv = has_dv;
            if (has_dv) {
              const CB& off = c[kind == JA_ADD ? JL_DVOFF : JL_RDVOFF];
              a.st_off = jbase[sk] + st.offs[row]; a.st_len = st_len;
              a.pid_off = jbase[ik] + c[ik].offs[row]; a.pid_len = pid_len;
              a.has_off = off.row_def[row] == 3;
              if (a.has_off) memcpy(&a.dv_off, off.fixed.data() + row * 4, 4);
            }
            a.canon_off = co;
            r->acts[ai] = a;
            r->act_row[ai] = row;
          }
          ai++;
          co += path_len + 64 + st_len + pid_len + 32;
        }
      }
      if (!fill) { b_na[bi + 1] = ai; b_canon[bi + 1] = co; }
    };
    parallel_for(nb, [&](int bi) { each(bi, false); });     // per block: actions, canonical bytes
    for (int bi = 0; bi < nb; bi++) { b_na[bi + 1] += b_na[bi]; b_canon[bi + 1] += b_canon[bi]; }
    r->acts.resize(b_na[nb]);
    r->act_row.resize(b_na[nb]);
    parallel_for(nb, [&](int bi) { each(bi, true); });
    canon_n = b_canon[nb];
  }
  size_t na = r->acts.size();
  const auto t_built = std::chrono::steady_clock::now();
  uint64_t cap = 1024;
  while (cap < 2 * na + 16) cap <<= 1;
  r->mask = cap - 1;
  if (zs.add(r->d_acts, r->acts.data(), na * sizeof(DJsonAction))) return 1;
  if (r->d_jchars.alloc(jchars_n + 16)) return 1;
  if (tail)
    for (int k : kKeyCols) zs.add_raw(r->d_jchars.as<uint8_t>() + jbase[k], tail->col[k].chars.data(), tail->col[k].chars.size());
  if (r->d_canon.alloc(canon_n + 64)) return 1;
  if (r->d_slots.alloc(cap * sizeof(Slot))) return 1;
  if (r->d_fp.alloc(cap * sizeof(uint32_t))) return 1;
  if (r->d_state.alloc(sizeof(DState))) return 1;
  if (r->d_jsel.alloc(na + 16)) return 1;
  // partitionValues maps for partition pruning: the tail's (rows mapped from add actions) and the
  // checkpoint's decoded key / value leaves
  auto up = [&](const void* src, size_t n) -> void* {
    r->map_bufs.emplace_back(new DBuf());
    if (zs.add(*r->map_bufs.back(), src, n)) return nullptr;
    return r->map_bufs.back()->p;
  };
  if (tail) {
    const CB& kc = tail->col[JL_PVK];
    const CB& vc = tail->col[JL_PVV];
    arow.assign(na, 0);
    for (size_t i = 0; i < na; i++) arow[i] = r->acts[i].kind != JA_REMOVE ? r->act_row[i] : -1;
    MapRows M{};
    M.n = (int64_t)na;
    M.act_row = (const int64_t*)up(arow.data(), arow.size() * 8);
    M.row_def = (const uint8_t*)up(kc.row_def.data(), kc.row_def.size());
    M.rep_def = kc.rep_def; M.v_max_def = vc.max_def;
    M.row_offs = (const int64_t*)up(kc.row_offs.data(), kc.row_offs.size() * 8);
    M.k_offs = (const int64_t*)up(kc.offs.data(), kc.offs.size() * 8);
    M.k_chars = (const uint8_t*)up(kc.chars.data(), kc.chars.size());
    M.v_def = (const uint8_t*)up(vc.entry_def.data(), vc.entry_def.size());
    M.v_offs = (const int64_t*)up(vc.offs.data(), vc.offs.size() * 8);
    M.v_chars = (const uint8_t*)up(vc.chars.data(), vc.chars.size());
    M.row_tag = -1000000000000ll;
    if (!M.act_row || !M.row_def || !M.row_offs || !M.k_offs || !M.k_chars || !M.v_def || !M.v_offs || !M.v_chars)
      return 1;
    r->tail_maps = M;
  }
  // stats strings for data skipping: the tail's per action (adds only), the checkpoint's column
  if (tail && tail->with_stats) {
    const CB& sc = tail->col[JL_STATS];
    soff.assign(na + 1, 0);
    slen.assign(na + 1, -1);
    for (size_t i = 0; i < na; i++) {
      const int64_t row = r->act_row[i];
      if (r->acts[i].kind == JA_REMOVE || sc.row_def[row] < 2) continue;
      soff[i] = sc.offs[row];
      slen[i] = (int32_t)(sc.offs[row + 1] - sc.offs[row]);
    }
    if (zs.add(r->d_tstats_chars, sc.chars.data(), sc.chars.size())) return 1;
    if (zs.add(r->d_tstats_off, soff.data(), soff.size() * 8)) return 1;
    if (zs.add(r->d_tstats_len, slen.data(), slen.size() * 4)) return 1;
  }
  if (zs.flush(s)) return 1;
  const auto t_queued = std::chrono::steady_clock::now();
  HIPOK(hipStreamSynchronize(s));
  if (getenv("DK_VERBOSE")) {
    using ms = std::chrono::duration<double, std::milli>;
    const auto t_end = std::chrono::steady_clock::now();
    fprintf(stderr, "[dk] replay create: %zu actions: build %.1f ms, uploads queued %.1f ms, waited %.1f ms\n", na,
            ms(t_built - t_create0).count(), ms(t_queued - t_built).count(), ms(t_end - t_queued).count());
  }
  if (ckpt && replay_attach(r.get(), ckpt)) return 1;
  *out = r.release();
  return 0;
}

extern "C" int dk_replay_attach_checkpoint(dk_replay* r, dk_parquet* ckpt) {
  if (!r || !ckpt) return fail("dk_replay_attach_checkpoint: null argument");
  if (r->ck) return fail("dk_replay_attach_checkpoint: a checkpoint is already attached");
  hipSetDevice(r->eng->cfg.device);
  return replay_attach(r, ckpt);
}


// validate a data-skipping program (layout dk_skip_program); `who` prefixes the error
// ---- Engine plugin point 1: JsonHandler.parseJson over stats strings, and the data-skipping
// PredicateEvaluator over the parsed result (KA/engine/JsonHandler.java:68-71,
// KA/engine/ExpressionHandler.java:58, as ScanImpl.applyDataSkipping drives them,
// KA/internal/ScanImpl.java:304-352) ----
struct dk_parsed {
  StreamH own;
  int device = 0;
  int64_t n = 0;
  dk_program schema;                       // one path per schema leaf, no ops
  DevSkip prog;                            // the schema as a device program (extraction only)
  DBuf d_chars, d_offs, d_isnull, d_sel, d_vals, d_set, d_state, d_out;
  bool dev_input = false;
  const uint8_t* chars = nullptr;          // device views of the input
  const int64_t* offs = nullptr;
  std::vector<int64_t> h_offs;             // host copies of the input (for the typed columns)
  std::vector<uint8_t> h_chars;
  bool host_ready = false;
  std::vector<int64_t> h_vals;             // [leaf][n]
  std::vector<uint32_t> h_set;             // [word][n]
  // the typed columns handed out (dk_parsed_column_get), per leaf
  struct Col { std::vector<uint8_t> valid; std::vector<int64_t> values, hi; std::vector<int32_t> offs, scale;
               std::vector<uint8_t> chars, wide; bool built = false; };
  std::vector<Col> cols;
  std::vector<std::string> path_json;
};

namespace dk { int schema_program(const char* schema_json, dk_program* out); }

extern "C" int dk_json_parse(dk_engine* e, const char* schema_json, int64_t n, const int64_t* offs,
                             const uint8_t* chars, const uint8_t* isnull, const uint8_t* selection,
                             int32_t on_device, dk_parsed** out) {
  if (!e || !schema_json || !out || n < 0 || (n && (!offs || !chars))) return fail("dk_json_parse: bad arguments");
  *out = nullptr;
  hipSetDevice(e->cfg.device);
  std::unique_ptr<dk_parsed> ps(new dk_parsed());
  ps->device = e->cfg.device;
  if (dk::schema_program(schema_json, &ps->schema)) return 1;
  if (install_skip(ps->prog, ps->schema)) return 1;
  const int np = (int)ps->schema.paths.size();
  const int nw = (np + 31) / 32;
  ps->cols.resize(np);
  if (ps->own.create()) return 1;
  hipStream_t s = ps->own.s;
  ps->n = n;
  ps->dev_input = on_device != 0;
  if (ps->dev_input) {
    ps->chars = chars; ps->offs = offs;
  } else {
    const int64_t nchars = n ? offs[n] - offs[0] : 0;
    ps->h_offs.assign(offs, offs + n + 1);
    for (auto& o : ps->h_offs) o -= offs[0];
    ps->h_chars.assign(nchars + 16, 0);
    if (nchars) memcpy(ps->h_chars.data(), chars + offs[0], (size_t)nchars);
    if (upload(ps->d_chars, ps->h_chars.data(), ps->h_chars.size(), s) ||
        upload(ps->d_offs, ps->h_offs.data(), (size_t)(n + 1) * 8, s)) return 1;
    ps->chars = ps->d_chars.as<uint8_t>(); ps->offs = ps->d_offs.as<int64_t>();
  }
  const uint8_t* dnull = isnull;
  const uint8_t* dsel = selection;
  if (!ps->dev_input) {                    // exactly n bytes each (the caller's arrays are not padded)
    if (isnull) { if (upload(ps->d_isnull, isnull, (size_t)n, s)) return 1; dnull = ps->d_isnull.as<uint8_t>(); }
    if (selection) { if (upload(ps->d_sel, selection, (size_t)n, s)) return 1; dsel = ps->d_sel.as<uint8_t>(); }
  }
  if (ps->d_vals.alloc((size_t)std::max(np, 1) * n * 8 + 64) || ps->d_set.alloc((size_t)std::max(nw, 1) * n * 4 + 64) ||
      ps->d_state.alloc(sizeof(DState)))
    return 1;
  DState st0{};
  st0.err_row = LLONG_MAX;
  HIPOK(hipMemcpyAsync(ps->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, s));
  launch_json_parse_stats(ps->chars, ps->offs, dnull, dsel, n, ps->prog.P, ps->prog.S, ps->d_vals.as<long long>(),
                          ps->d_set.as<uint32_t>(), ps->d_state.as<DState>(), s);
  HIPOK(hipStreamSynchronize(s));
  DState h{};
  HIPOK(hipMemcpy(&h, ps->d_state.p, sizeof h, hipMemcpyDeviceToHost));
  if (h.err_flags & E_STATS)
    return fail("Parsing the JSON statistics: couldn't decode the stats of row " + std::to_string(h.err_row));
  for (auto& p : ps->schema.paths) {
    std::string j = "[";
    for (size_t k = 0; k < p.size(); k++) {
      j += k ? ",\"" : "\"";
      for (unsigned char c : p[k]) {
        if (c == '"' || c == '\\') { j += '\\'; j += (char)c; }
        else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); j += b; }
        else j += (char)c;
      }
      j += "\"";
    }
    ps->path_json.push_back(j + "]");
  }
  *out = ps.release();
  return 0;
}

extern "C" int32_t dk_parsed_num_leaves(const dk_parsed* ps) { return ps ? (int32_t)ps->schema.paths.size() : -1; }

extern "C" int64_t dk_parsed_leaf_path(const dk_parsed* ps, int32_t leaf, char* buf, int64_t cap) {
  if (!ps || leaf < 0 || leaf >= (int32_t)ps->path_json.size()) return -1;
  const std::string& j = ps->path_json[leaf];
  if (buf && cap > 0) {
    const int64_t m = std::min<int64_t>((int64_t)j.size(), cap - 1);
    memcpy(buf, j.data(), (size_t)m);
    buf[m] = 0;
  }
  return (int64_t)j.size();
}

// JSON string body s[a, b) (escapes decoded as Jackson does; a lone surrogate becomes '?', as
// String.getBytes(UTF_8) writes it) appended as UTF-8
static void json_unescape(const uint8_t* s, int64_t a, int64_t b, std::vector<uint8_t>& o) {
  auto put = [&](uint32_t cp) {
    if (cp >= 0xD800 && cp <= 0xDFFF) { o.push_back('?'); return; }
    if (cp < 0x80) o.push_back((uint8_t)cp);
    else if (cp < 0x800) { o.push_back(0xC0 | (cp >> 6)); o.push_back(0x80 | (cp & 63)); }
    else if (cp < 0x10000) { o.push_back(0xE0 | (cp >> 12)); o.push_back(0x80 | ((cp >> 6) & 63)); o.push_back(0x80 | (cp & 63)); }
    else { o.push_back(0xF0 | (cp >> 18)); o.push_back(0x80 | ((cp >> 12) & 63)); o.push_back(0x80 | ((cp >> 6) & 63)); o.push_back(0x80 | (cp & 63)); }
  };
  auto hex4 = [&](int64_t i, uint32_t* v) {
    if (i + 4 > b) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) {
      const uint8_t c = s[i + k];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= c - '0'; else if ((c | 0x20) >= 'a' && (c | 0x20) <= 'f') x |= (c | 0x20) - 'a' + 10; else return false;
    }
    *v = x;
    return true;
  };
  for (int64_t i = a; i < b;) {
    if (s[i] != '\\') { o.push_back(s[i++]); continue; }
    const uint8_t c = s[i + 1];
    i += 2;
    if (c == 'u') {
      uint32_t cp = 0;
      hex4(i, &cp);
      i += 4;
      if (cp >= 0xD800 && cp <= 0xDBFF && i + 6 <= b && s[i] == '\\' && s[i + 1] == 'u') {
        uint32_t lo;
        if (hex4(i + 2, &lo) && lo >= 0xDC00 && lo <= 0xDFFF) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); i += 6; }
      }
      put(cp);
    } else {
      o.push_back(c == 'b' ? '\b' : c == 'f' ? '\f' : c == 'n' ? '\n' : c == 'r' ? '\r' : c == 't' ? '\t' : c);
    }
  }
}

// The typed column of one leaf (host memory, valid until dk_parsed_free), as DefaultJsonRow decodes
// it (KD/internal/data/DefaultJsonRow.java:136-357): integral / date (epoch days) / timestamp(_ntz)
// (micros) values; strings after JSON unescaping (int32 offsets + chars); decimals as the BigDecimal
// of the number token (unscaled 128-bit value + scale, and the token text); float / double as the
// IEEE bits of DecimalNode.floatValue / doubleValue (correctly rounded; "-0.0" is +0.0, as BigDecimal
// has no negative zero; NaN / +-Infinity from their string forms).
extern "C" int dk_parsed_column_get(dk_parsed* ps, int32_t leaf, dk_parsed_column* out) {
  if (!ps || !out || leaf < 0 || leaf >= (int32_t)ps->schema.paths.size()) return fail("dk_parsed_column_get: bad leaf");
  hipSetDevice(ps->device);
  const int64_t n = ps->n;
  const int np = (int)ps->schema.paths.size();
  const int nw = (np + 31) / 32;
  if (!ps->host_ready) {
    ps->h_vals.resize((size_t)np * n);
    ps->h_set.resize((size_t)nw * n);
    if (n) {
      HIPOK(hipMemcpy(ps->h_vals.data(), ps->d_vals.p, (size_t)np * n * 8, hipMemcpyDeviceToHost));
      HIPOK(hipMemcpy(ps->h_set.data(), ps->d_set.p, (size_t)nw * n * 4, hipMemcpyDeviceToHost));
    }
    if (ps->dev_input && n) {               // the rows' strings, for the spans
      ps->h_offs.resize(n + 1);
      HIPOK(hipMemcpy(ps->h_offs.data(), ps->offs, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost));
      const int64_t base = ps->h_offs[0];
      ps->h_chars.assign(ps->h_offs[n] - base + 16, 0);
      HIPOK(hipMemcpy(ps->h_chars.data(), ps->chars + base, (size_t)(ps->h_offs[n] - base), hipMemcpyDeviceToHost));
      for (auto& o : ps->h_offs) o -= base;
    }
    ps->host_ready = true;
  }
  dk_parsed::Col& C = ps->cols[leaf];
  const int t = ps->schema.path_type[leaf];
  if (!C.built) {
    C.valid.assign(n, 0);
    C.values.assign(n, 0);
    const bool strings = t == SK_STRING || t == SK_DECIMAL;
    if (strings) C.offs.assign(n + 1, 0);
    if (t == SK_DECIMAL) { C.hi.assign(n, 0); C.scale.assign(n, 0); C.wide.assign(n, 0); }
    for (int64_t r = 0; r < n; r++) {
      const bool present = (ps->h_set[(size_t)(leaf >> 5) * n + r] >> (leaf & 31)) & 1;
      C.valid[r] = present;
      const int64_t v = ps->h_vals[(size_t)leaf * n + r];
      const uint8_t* row = ps->h_chars.data() + (n ? ps->h_offs[r] : 0);
      if (present) {
        if (t == SK_STRING) {
          const int64_t a = v & 0x7fffffff, len = (v >> 32) & 0x3fffffff;
          if ((v >> 62) & 1) json_unescape(row, a, a + len, C.chars);
          else C.chars.insert(C.chars.end(), row + a, row + a + len);
        } else if (t == SK_DECIMAL) {
          const int64_t a = v & 0x7fffffff, len = v >> 32;
          C.chars.insert(C.chars.end(), row + a, row + a + len);
          // new BigDecimal(token): unscaled = the mantissa digits, scale = fraction digits - exponent
          unsigned __int128 u = 0;
          const unsigned __int128 lim = ((unsigned __int128)1 << 127) / 10;
          bool neg = false, wide = false;
          int64_t i = a, frac = 0, exp = 0;
          bool dot = false;
          if (row[i] == '-') { neg = true; i++; }
          for (; i < a + len && row[i] != 'e' && row[i] != 'E'; i++) {
            if (row[i] == '.') { dot = true; continue; }
            if (u > lim) wide = true;
            u = u * 10 + (row[i] - '0');
            if (dot) frac++;
          }
          if (i < a + len) exp = strtoll(std::string((const char*)row + i + 1, (size_t)(a + len - i - 1)).c_str(), nullptr, 10);
          const __int128 sv = neg ? -(__int128)u : (__int128)u;
          C.values[r] = (int64_t)(uint64_t)sv;
          C.hi[r] = (int64_t)(sv >> 64);
          C.scale[r] = (int32_t)(frac - exp);
          C.wide[r] = wide;
        } else if (t == SK_FLOAT || t == SK_DOUBLE) {
          uint64_t bits;
          if ((v >> 62) & 1) {                    // NaN / +Infinity / -Infinity
            const int code = (int)(v & 3);
            bits = t == SK_FLOAT ? (code == 1 ? 0x7fc00000ull : code == 2 ? 0x7f800000ull : 0xff800000ull)
                                 : (code == 1 ? 0x7ff8000000000000ull : code == 2 ? 0x7ff0000000000000ull : 0xfff0000000000000ull);
          } else {
            const int64_t a = v & 0x7fffffff, len = v >> 32;
            const std::string tok((const char*)row + a, (size_t)len);
            bool zero = true;                       // an exact zero (BigDecimal: no sign) -> +0.0
            for (size_t k = 0; k < tok.size() && tok[k] != 'e' && tok[k] != 'E'; k++) zero = zero && !(tok[k] >= '1' && tok[k] <= '9');
            if (t == SK_FLOAT) { float f = zero ? 0.0f : strtof(tok.c_str(), nullptr); uint32_t b; memcpy(&b, &f, 4); bits = b; }
            else { double d = zero ? 0.0 : strtod(tok.c_str(), nullptr); memcpy(&bits, &d, 8); }
          }
          C.values[r] = (int64_t)bits;
        } else {
          C.values[r] = v;
        }
      }
      if (strings) C.offs[r + 1] = (int32_t)C.chars.size();
    }
    if (C.chars.size() > (size_t)INT32_MAX) return fail("dk_parsed_column_get: strings exceed 2 GiB");
    C.chars.push_back(0);
    C.built = true;
  }
  memset(out, 0, sizeof *out);
  out->type = t;
  out->n = n;
  out->validity = C.valid.data();
  out->values = C.values.data();
  if (t == SK_STRING || t == SK_DECIMAL) { out->offs = C.offs.data(); out->chars = C.chars.data(); }
  if (t == SK_DECIMAL) { out->values_hi = C.hi.data(); out->scale = C.scale.data(); out->wide = C.wide.data(); }
  return 0;
}

// PredicateEvaluator.eval(parsed stats, selection) for COALESCE(prog, true): every stats path of the
// program must be a leaf of the parsed schema with the same type (the program is re-indexed onto the
// schema's leaves); selection is updated in place (host memory, or device memory when the stats were
// parsed from device input)
extern "C" int dk_parsed_eval(dk_parsed* ps, const dk_program* prog, uint8_t* selection) {
  if (!ps || !prog || (ps->n && !selection)) return fail("dk_parsed_eval: bad arguments");
  if (prog->kind != DK_PROGRAM_SKIPPING) return fail("dk_parsed_eval: not a data-skipping program");
  dk_program P = ps->schema;               // the schema's path table, the program's ops re-indexed
  std::vector<int32_t> map(prog->paths.size(), -1);
  for (size_t i = 0; i < prog->paths.size(); i++) {
    for (size_t j = 0; j < ps->schema.paths.size(); j++)
      if (ps->schema.paths[j] == prog->paths[i]) { map[i] = (int32_t)j; break; }
    if (map[i] < 0 || ps->schema.path_type[map[i]] != prog->path_type[i])
      return fail("dk_parsed_eval: the predicate's stats paths are not in the parsed schema");
  }
  // the program's pool starts with its own path names: literal offsets move by the size difference
  int64_t names0 = 0;
  for (auto& p : prog->paths) for (auto& c : p) names0 += (int64_t)c.size();
  const int64_t base = (int64_t)P.pool.size();
  P.pool += prog->pool.substr((size_t)names0);
  P.op = prog->op; P.arg = prog->arg; P.lit = prog->lit;
  for (size_t k = 0; k < P.op.size(); k++) {
    const int op = P.op[k];
    if (op == OP_STAT) P.arg[k] = map[P.arg[k]];
    else if (op == OP_LIT_STR || op == OP_LIT_DEC) P.lit[k] += base - names0;
    else if (op == OP_FCMP) P.lit[k] += base - names0;        // offset in the low 32 bits
  }
  P.stack = prog->stack;
  hipSetDevice(ps->device);
  hipStream_t s = ps->own.s;
  if (!ps->n) return 0;
  DevSkip d;
  if (install_skip(d, P)) return 1;
  uint8_t* dsel = selection;
  if (!ps->dev_input) {
    if (upload(ps->d_out, selection, (size_t)ps->n, s)) return 1;
    dsel = ps->d_out.as<uint8_t>();
  }
  launch_parsed_eval(ps->chars, ps->offs, ps->n, d.P, ps->d_vals.as<long long>(), ps->d_set.as<uint32_t>(), dsel, s);
  if (!ps->dev_input) HIPOK(hipMemcpyAsync(selection, dsel, (size_t)ps->n, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

extern "C" void dk_parsed_free(dk_parsed* ps) {
  if (!ps) return;
  hipSetDevice(ps->device);
  hipStreamSynchronize(ps->own.s);
  delete ps;
}

extern "C" int dk_replay_set_skipping(dk_replay* r, const dk_program* prog) {
  if (!r) return fail("null replay");
  if (!prog) { r->has_skip = false; return 0; }
  if (prog->kind != DK_PROGRAM_SKIPPING) return fail("dk_replay_set_skipping: not a data-skipping program");
  if (!r->tail || !r->tail->with_stats) return fail("dk_replay_set_skipping: the commit tail was parsed without stats");
  if (r->lazy && attach_upto(r, INT_MAX)) return 1;   // the typed stats columns of every file
  if (install_skip(r->skip, *prog)) return 1;
  const dk_program& P = r->skip.prog;
  const int np = (int)P.paths.size();
  // add.stats_parsed fast path, per checkpoint file: every program path's typed leaf
  // add.stats_parsed.<path> was projected and decoded with a physical / logical type that holds the
  // stat's Kernel type (long: INT64; int / short / byte / date: INT32; timestamp(_ntz): INT64 micros /
  // millis or INT96; string: BYTE_ARRAY; decimal: INT32 / INT64 with a scale; float: FLOAT; double:
  // DOUBLE), and the file's add.stats JSON column is there for the rows the typed values cannot
  // stand for (k_stats_parsed)
  r->ck_parsed.assign(r->ck ? r->ck->files.size() : 0, StatsParsedRows{});
  r->typed_paths.clear();
  std::vector<TypedPath> all;
  std::vector<size_t> at(r->ck_parsed.size(), SIZE_MAX);
  for (size_t fi = 0; fi < r->ck_parsed.size(); fi++) {
    StatsParsedRows R{};
    R.n_paths = np;
    R.struct_def = 2;                     // add (1) . stats_parsed (2)
    R.js = fi < r->ck_stats.size() ? r->ck_stats[fi] : StatsRows{};
    bool ok = np > 0 && R.js.n > 0 && R.js.offs;
    std::vector<TypedPath> tp(np);
    for (int q = 0; q < np && ok; q++) {
      const int t = P.path_type[q];
      std::string leaf = "add.stats_parsed";
      for (auto& c : P.paths[q]) leaf += "." + c;
      const DColumn* c = find_col(r->ck, (int)fi, leaf.c_str());
      const LeafM* L = find_leafm(r->ck, (int)fi, leaf.c_str());
      ok = c && L && c->present && !c->max_rep && c->max_def >= 3;
      if (!ok) break;
      int kind = -1;
      switch (t) {
        case SK_LONG: if (c->phys == PT_INT64 && L->dec_scale < 0 && !L->ts_unit) kind = TP_INT; break;
        case SK_INT: case SK_SHORT: case SK_BYTE: case SK_DATE:
          if (c->phys == PT_INT32 && L->dec_scale < 0) kind = TP_INT; break;
        case SK_TIMESTAMP: case SK_TIMESTAMP_NTZ:
          if (c->phys == PT_INT64 && L->ts_unit == 2) kind = TP_INT;
          else if (c->phys == PT_INT64 && L->ts_unit == 1) kind = TP_MILLIS;
          else if (c->phys == PT_INT96) kind = TP_INT96;
          break;
        case SK_STRING: if (c->phys == PT_BYTE_ARRAY) kind = TP_STR; break;
        case SK_DECIMAL:
          if ((c->phys == PT_INT32 || c->phys == PT_INT64) && L->dec_scale >= 0 && L->dec_scale <= 38) kind = TP_DEC; break;
        case SK_FLOAT: if (c->phys == PT_FLOAT) kind = TP_F32; break;
        case SK_DOUBLE: if (c->phys == PT_DOUBLE) kind = TP_F64; break;
      }
      ok = kind >= 0 && (kind == TP_STR ? (c->null_only || c->offs) : (c->null_only || c->fixed));
      if (!ok) break;
      TypedPath& T = tp[q];
      T.kind = kind; T.scale = kind == TP_DEC ? L->dec_scale : 0;
      T.def = c->row_def; T.max_def = c->max_def;
      T.vals = c->null_only || kind == TP_STR ? nullptr : c->fixed; T.width = c->width;
      T.offs = kind == TP_STR && !c->null_only ? c->offs : nullptr;
      T.chars = kind == TP_STR && !c->null_only ? c->chars : nullptr;
      if (c->null_only) T.max_def = 1 << 30;          // no value anywhere: always null
    }
    if (ok) {
      R.n = r->ck->files[fi].num_rows;
      r->ck_parsed[fi] = R;
      at[fi] = all.size();
      all.insert(all.end(), tp.begin(), tp.end());
    }
  }
  if (!all.empty()) {                      // every file's TypedPath table in one device buffer
    if (r->typed_buf.alloc(all.size() * sizeof(TypedPath))) return 1;
    HIPOK(hipMemcpy(r->typed_buf.p, all.data(), all.size() * sizeof(TypedPath), hipMemcpyHostToDevice));
    for (size_t fi = 0; fi < at.size(); fi++)
      if (at[fi] != SIZE_MAX) r->ck_parsed[fi].paths = r->typed_buf.as<TypedPath>() + at[fi];
  }
  r->has_skip = true;
  return 0;
}

extern "C" int dk_replay_set_partition_filter(dk_replay* r, const dk_program* prog) {
  if (!r) return fail("null replay");
  if (!prog) { r->has_part = false; return 0; }
  if (install_part(r->part, *prog)) return 1;
  r->has_part = true;
  return 0;
}

static int replay_ckpt_filters(dk_replay* r);
static int replay_grouped(dk_replay* r, uint64_t h_nodv);
static int issue_group(dk_replay* r);
static int replay_launch(dk_replay* r) {
  hipStream_t s = r->stream;
  KTimer& T = r->timer;
  KTimer::Scope total(&T, 12, s);
  r->xphase = 0;
  if (r->xw > 0) HIPOK(hipMemsetAsync(r->d_xtot.p, 0, (size_t)r->xw * 8, s));
  DState st0{};
  st0.err_row = LLONG_MAX;
  if (r->lazy && r->ck && r->ck->open_state.load() == 0) {
    // the checkpoint's H2D copies are in flight: a small DMA copy would queue behind them
    if (r->h_st0.size() < sizeof st0 && r->h_st0.alloc(sizeof st0 + 16)) return 1;
    memcpy(r->h_st0.data(), &st0, sizeof st0);
    launch_copy_zc(r->d_state.p, r->h_st0.data(), sizeof st0, s);
  } else HIPOK(hipMemcpyAsync(r->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, s));
  // probe table: h = 0 (empty), first_add = ~0, min_rm_step = INT32_MAX
  launch_slots_init(r->d_slots.as<Slot>(), r->mask + 1, s);
  int na = (int)r->acts.size();
  DState* st = r->d_state.as<DState>();
  DJsonAction* A = r->d_acts.as<DJsonAction>();
  Slot* S = r->d_slots.as<Slot>();
  { KTimer::Scope sc(&T, 7, s); launch_json_canon(A, na, r->d_jchars.as<uint8_t>(), r->d_canon.as<uint8_t>(), r->seed, st, s); }
  { KTimer::Scope sc(&T, 8, s); launch_table_insert(A, na, S, r->mask, s); }
  { KTimer::Scope sc(&T, 9, s); launch_table_update(A, na, S, r->mask, r->d_canon.as<uint8_t>(), st, s); }
  { KTimer::Scope sc(&T, 10, s); launch_json_select(A, na, S, r->mask, r->d_canon.as<uint8_t>(), r->d_jsel.as<uint8_t>(), st, s); }
  if (r->has_part && na) {                 // partition pruning on the tail's adds (before skipping)
    KTimer::Scope sc(&T, 18, s);
    launch_part_eval(r->tail_maps, r->part.P, r->d_jsel.as<uint8_t>(), st, s);
  }
  if (r->has_skip && na) {                 // data skipping on the tail's selected adds
    KTimer::Scope sc(&T, 17, s);
    StatsRows R{};
    R.n = na; R.soff = r->d_tstats_off.as<int64_t>(); R.slen = r->d_tstats_len.as<int32_t>();
    R.chars = r->d_tstats_chars.as<uint8_t>(); R.row_tag = -1000000000000ll;
    launch_stats_eval(R, r->skip.P, r->skip.S, r->d_jsel.as<uint8_t>(), st, s);
  }
  if (r->n_groups > 0 && r->xw == 0 && r->ck) {
    const int ng = std::max(1, std::min(r->n_groups, (int)r->ck->files.size()));
    if (r->h_zstate.size() < (size_t)(ng + 1) * 2 * sizeof(DState) && r->h_zstate.alloc((size_t)(ng + 1) * 2 * sizeof(DState))) return 1;
    if (r->h_zjsel.size() < (size_t)na + 16 && r->h_zjsel.alloc((size_t)na + 16)) return 1;
    memset(r->h_zstate.data(), 0, 2 * sizeof(DState));
    launch_copy_zc(r->h_zstate.data(), r->d_state.p, sizeof(DState), s);
    launch_copy_zc(r->h_zjsel.data(), r->d_jsel.p, na, s);
  }
  if (!r->ev_tail) HIPOK(hipEventCreateWithFlags(&r->ev_tail, hipEventDisableTiming));
  HIPOK(hipEventRecord(r->ev_tail, s));
  if (r->ck) r->ck->file_done.clear();
  if (r->ck) {
    dk_parquet* p = r->ck;
    const bool grouped = r->n_groups > 0 && r->xw == 0;
    // a checkpoint still being opened (and decoded, slice by slice): only a grouped run overlaps
    // it; anything else waits for the whole open first
    const bool lazy_run = r->lazy && grouped && p->open_state.load() == 0;
    r->run_lazy = lazy_run;
    if (r->lazy && !lazy_run) {
      if (ensure_open(p) || attach_upto(r, INT_MAX)) return 1;
    }
    if (!lazy_run) {
      // the decode runs on the replay's stream, after anything queued on the checkpoint's own
      HIPOK(hipEventRecord(r->ev_in, p->stream));
      HIPOK(hipStreamWaitEvent(s, r->ev_in, 0));
      // decode errors are collected into the replay state too
      HIPOK(hipMemcpyAsync(p->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, s));
      if (run_pipeline(p, 1, s, grouped)) return 1;
    }
    launch_table_fp(S, r->d_fp.as<uint32_t>(), r->mask + 1, s);
    HashSink kd; kd.hs.init(kHashSeed(r->seed)); kd.n = 0;       // dvUniqueId stream of "no DV"
    dv_emit(false, nullptr, 0, nullptr, 0, false, 0, kd);
    const uint64_t h_nodv = kd.hs.final_(kd.n);
    if (grouped) return replay_grouped(r, h_nodv);
    if (r->probe_all || r->xw > 0) {
      KTimer::Scope sc(&T, 11, s);
      const size_t nf = r->probe.size();
      r->probe_run = r->probe;
      r->probe_row0.assign(nf + 1, 0);
      r->probe_sel.resize(nf);
      for (size_t fi = 0; fi < nf; fi++) {
        if (r->seed != kDecodeSeed) r->probe_run[fi].path_hash = nullptr;   // collision retry
        r->probe_row0[fi + 1] = r->probe_row0[fi] + r->probe_run[fi].n_rows;
        r->probe_sel[fi] = r->d_csel[fi]->as<uint8_t>();
      }
      if (upload(r->d_probe_cols, r->probe_run.data(), nf * sizeof(ProbeCols), s) ||
          upload(r->d_probe_row0, r->probe_row0.data(), (nf + 1) * 8, s) ||
          upload(r->d_probe_sel, r->probe_sel.data(), nf * sizeof(uint8_t*), s)) return 1;
      ProbeSet PS{r->d_probe_cols.as<ProbeCols>(), r->d_probe_row0.as<int64_t>(), r->d_probe_sel.as<uint8_t* const>(),
                  (int32_t)nf, r->probe_row0[nf]};
      if (r->xw > 0) {
        // exchange mode: route counts only; dk_replay_exchange_pack / _filter / _finish do the rest
        long long chunk;
        const int nb = a2a_blocks(PS.total, &chunk);
        if (r->d_xbc.alloc((size_t)nb * r->xw * 8 + 64)) return 1;
        launch_a2a_count(PS, r->xw, r->d_xbc.as<unsigned long long>(), r->d_xtot.as<unsigned long long>(), s);
        r->xphase = 1;
        return 0;
      }
      launch_probe_all(PS, S, r->d_fp.as<uint32_t>(), r->mask, A, r->d_canon.as<uint8_t>(), r->seed, h_nodv, r->d_cand.as<int32_t>(),
                       r->d_cand_n.as<unsigned int>(), st, s);
    } else {
      for (size_t fi = 0; fi < r->probe.size(); fi++) {
        KTimer::Scope sc(&T, 11, s);
        ProbeCols pc = r->probe[fi];
        if (r->seed != kDecodeSeed) pc.path_hash = nullptr;   // collision retry: rehash from the chars
        launch_probe(pc, S, r->d_fp.as<uint32_t>(), r->mask, A, r->d_canon.as<uint8_t>(), r->seed, h_nodv,
                     r->d_csel[fi]->as<uint8_t>(), r->d_cand.as<int32_t>(), r->d_cand_n.as<unsigned int>(), st, s);
      }
    }
    if (replay_ckpt_filters(r)) return 1;
  }
  return 0;
}

// partition pruning and data skipping on checkpoint file fi's rows (after its probe)
static void replay_file_filters(dk_replay* r, size_t fi) {
  hipStream_t s = r->stream;
  KTimer& T = r->timer;
  DState* st = r->d_state.as<DState>();
  if (r->has_part && fi < r->ck_maps.size()) {
    KTimer::Scope sc(&T, 18, s);
    launch_part_eval(r->ck_maps[fi], r->part.P, r->d_csel[fi]->as<uint8_t>(), st, s);
  }
  if (r->has_skip && fi < r->ck_stats.size()) {
    KTimer::Scope sc(&T, 17, s);
    if (fi < r->ck_parsed.size() && r->ck_parsed[fi].n > 0)
      launch_stats_parsed(r->ck_parsed[fi], r->skip.P, r->skip.S, r->d_csel[fi]->as<uint8_t>(), st, s);
    else
      launch_stats_eval(r->ck_stats[fi], r->skip.P, r->skip.S, r->d_csel[fi]->as<uint8_t>(), st, s);
  }
}

// the grouped form of the checkpoint half (after the front of the decode pipeline and the table
// fingerprints): per group of files, value decode, probe, filters and the D2H of the selections,
// then an event the host waits on before handing out those files' batches
static int replay_grouped(dk_replay* r, uint64_t h_nodv) {
  hipStream_t s = r->stream;
  dk_parquet* p = r->ck;
  const int nf = (int)p->files.size();
  const int ng = std::max(1, std::min(r->n_groups, nf));
  r->grp_f0.assign(ng + 1, 0);
  for (int g = 0; g <= ng; g++) r->grp_f0[g] = (int)((int64_t)nf * g / ng);
  while ((int)r->grp_ev.size() < ng) {
    hipEvent_t e = nullptr;
    HIPOK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    r->grp_ev.push_back(e);
  }
  p->file_done.assign(nf, nullptr);
  r->file_ready.assign(nf, 0);
  // the host block every selection lands in
  r->h_csel_off.assign(nf + 1, 0);
  for (int f = 0; f < nf; f++) r->h_csel_off[f + 1] = r->h_csel_off[f] + ((p->files[f].num_rows + 63) & ~(int64_t)63);
  // (kept across reruns of the same scan: batches already handed out point into it)
  if (r->h_csel.size() != (size_t)(r->h_csel_off[nf] + 64) && r->h_csel.alloc(r->h_csel_off[nf] + 64)) return 1;
  // probe sets: per-file columns and selections as in the one-launch probe, row prefixes per group
  r->probe_run = r->probe;
  r->probe_sel.resize(nf);
  r->grp_row0.assign(nf + ng, 0);
  for (int f = 0; f < nf; f++) {
    if (r->seed != kDecodeSeed) r->probe_run[f].path_hash = nullptr;   // collision retry
    r->probe_sel[f] = r->d_csel[f]->as<uint8_t>();
  }
  for (int g = 0; g < ng; g++) {
    int64_t* row0 = r->grp_row0.data() + r->grp_f0[g] + g;
    for (int f = r->grp_f0[g]; f < r->grp_f0[g + 1]; f++) row0[f - r->grp_f0[g] + 1] = row0[f - r->grp_f0[g]] + r->probe_run[f].n_rows;
  }
  // (row counts come from the footers: the prefixes are final before any file is attached)
  for (int g = 0; g < ng; g++) {
    int64_t* row0 = r->grp_row0.data() + r->grp_f0[g] + g;
    for (int f = r->grp_f0[g]; f < r->grp_f0[g + 1]; f++) row0[f - r->grp_f0[g] + 1] = row0[f - r->grp_f0[g]] + (find_col(p, f, "add.path") ? p->files[f].num_rows : 0);
  }
  if (r->lazy) {
    // tables through pinned memory and a copy kernel: the open's H2D copies are still in flight
    if (r->d_probe_cols.alloc(nf * sizeof(ProbeCols) + 16) || r->d_grp_row0.alloc(r->grp_row0.size() * 8 + 16) ||
        r->d_probe_sel.alloc(nf * sizeof(uint8_t*) + 16) || r->h_probe_cols.alloc(nf * sizeof(ProbeCols) + 16))
      return 1;
    HBuf a, b;
    if (a.alloc(r->grp_row0.size() * 8 + 16) || b.alloc(nf * sizeof(uint8_t*) + 16)) return 1;
    memcpy(a.data(), r->grp_row0.data(), r->grp_row0.size() * 8);
    memcpy(b.data(), r->probe_sel.data(), nf * sizeof(uint8_t*));
    launch_copy_zc(r->d_grp_row0.p, a.data(), (long long)(r->grp_row0.size() * 8), s);
    launch_copy_zc(r->d_probe_sel.p, b.data(), (long long)(nf * sizeof(uint8_t*)), s);
    HIPOK(hipStreamSynchronize(s));                // (the staging goes back to the cache)
  } else if (upload(r->d_probe_cols, r->probe_run.data(), nf * sizeof(ProbeCols), s) ||
             upload(r->d_grp_row0, r->grp_row0.data(), r->grp_row0.size() * 8, s) ||
             upload(r->d_probe_sel, r->probe_sel.data(), nf * sizeof(uint8_t*), s)) return 1;
  r->h_nodv = h_nodv;
  r->grp_issued = 0;
  r->h_csel_ready = true;   // the block every group's selections land in (file f's after wait_file(f))
  if (!r->run_lazy)
    while (r->grp_issued < ng) if (issue_group(r)) return 1;
  return 0;
}

// The next group of a grouped run: value decode (unless the open decoded it), probe, filters, the
// selections and error states to pinned memory, its event, the prefetched mirrors. Lazy runs (the
// checkpoint's open still running) attach the group's files first, waiting for them to be ready.
static int issue_group(dk_replay* r) {
  hipStream_t s = r->stream;
  KTimer& T = r->timer;
  dk_parquet* p = r->ck;
  DState* st = r->d_state.as<DState>();
  DJsonAction* A = r->d_acts.as<DJsonAction>();
  Slot* S = r->d_slots.as<Slot>();
  const int ng = (int)r->grp_f0.size() - 1;
  const int g = r->grp_issued;
  if (g >= ng) return 0;
  const uint64_t h_nodv = r->h_nodv;
  {
    const int f0 = r->grp_f0[g], f1 = r->grp_f0[g + 1];
    if (r->lazy) {
      if (attach_upto(r, f1)) return 1;
      for (int f = f0; f < f1; f++) {
        r->probe_run[f] = r->probe[f];
        if (r->seed != kDecodeSeed) r->probe_run[f].path_hash = nullptr;   // collision retry
      }
      memcpy(r->h_probe_cols.data() + (size_t)f0 * sizeof(ProbeCols), r->probe_run.data() + f0, (size_t)(f1 - f0) * sizeof(ProbeCols));
      launch_copy_zc(r->d_probe_cols.as<ProbeCols>() + f0, r->h_probe_cols.data() + (size_t)f0 * sizeof(ProbeCols),
                     (long long)((f1 - f0) * sizeof(ProbeCols)), s);
    }
    if (r->run_lazy) {
      for (int f = f0; f < f1; f++)                // the files' value decode (the open's slice streams)
        if (f < (int)p->file_dec.size() && p->file_dec[f]) HIPOK(hipStreamWaitEvent(s, p->file_dec[f], 0));
    } else {
      decode_cols(p, s, p->file_col0[f0], p->file_col0[f1]);
    }
    {
      KTimer::Scope sc(&T, 11, s);
      const int64_t* row0 = r->grp_row0.data() + f0 + g;
      ProbeSet PS{r->d_probe_cols.as<ProbeCols>() + f0, r->d_grp_row0.as<int64_t>() + f0 + g,
                  r->d_probe_sel.as<uint8_t* const>() + f0, (int32_t)(f1 - f0), row0[f1 - f0]};
      launch_probe_all(PS, S, r->d_fp.as<uint32_t>(), r->mask, A, r->d_canon.as<uint8_t>(), r->seed, h_nodv,
                       r->d_cand.as<int32_t>(), r->d_cand_n.as<unsigned int>(), st, s);
    }
    for (int f = f0; f < f1; f++) replay_file_filters(r, (size_t)f);
    for (int f = f0; f < f1; f++) {
      const int64_t n = p->files[f].num_rows;
      if (r->probe[f].n_rows == 0) memset(r->h_csel.data() + r->h_csel_off[f], 0, n);
      else if (n && r->lazy) launch_copy_zc(r->h_csel.data() + r->h_csel_off[f], r->d_csel[f]->p, n, s);
      else if (n) HIPOK(hipMemcpyAsync(r->h_csel.data() + r->h_csel_off[f], r->d_csel[f]->p, n, hipMemcpyDeviceToHost, s));
    }
    {
      uint8_t* z = r->h_zstate.data() + (size_t)(g + 1) * 2 * sizeof(DState);
      launch_copy_zc(z, r->d_state.p, sizeof(DState), s);
      launch_copy_zc(z + sizeof(DState), p->d_state.p, sizeof(DState), s);
    }
    HIPOK(hipEventRecord(r->grp_ev[g], s));
    for (int f = f0; f < f1; f++) p->file_done[f] = r->grp_ev[g];
    for (int leaf : r->prefetch)
      for (int f = f0; f < f1; f++)
        if (p->colmap[f][leaf] >= 0 && queue_mirror(p, p->colmap[f][leaf])) return 1;
  }
  r->grp_issued = g + 1;
  if (getenv("DK_VERBOSE"))
    fprintf(stderr, "[dk] group %d (files [%d, %d)) issued at %.1f ms\n", g, r->grp_f0[g], r->grp_f0[g + 1],
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p->t_open0).count());
  if (r->grp_issued == ng) HIPOK(hipEventRecord(r->ev_out, s));   // the checkpoint stream waits for it at dk_replay_sync
  return 0;
}

// the checkpoint rows' partition pruning and data skipping after the probe, then the hand-back to
// the checkpoint's own stream
static int replay_ckpt_filters(dk_replay* r) {
  hipStream_t s = r->stream;
  if (r->has_part || r->has_skip)         // partition pruning, then data skipping, per file
    for (size_t fi = 0; fi < r->d_csel.size(); fi++) replay_file_filters(r, fi);
  // later work on the checkpoint's stream (column reads) sees the decoded columns
  HIPOK(hipEventRecord(r->ev_out, s));
  HIPOK(hipStreamWaitEvent(r->ck->stream, r->ev_out, 0));
  return 0;
}

static int owner_launch(dk_replay* r);
extern "C" int dk_replay_run(dk_replay* r) {
  hipSetDevice(r->eng->cfg.device);
  r->have_result = false;
  r->h_csel_ready = false;
  if (r->ck && invalidate_mirrors(r->ck)) return 1;
  r->n_groups = 0;
  if (r->ow > 0) return owner_launch(r);
  return replay_launch(r);
}

// The run with the checkpoint files in n_groups groups (1 <= n_groups; at most one group per file),
// so that a consumer can take the first files' batches while the later groups are still decoding:
// dk_replay_wait_file(r, -1) before the commit-tail selection, dk_replay_wait_file(r, f) before
// file f's selection / columns, dk_replay_sync at the end (counters). Exchange mode runs ungrouped.
extern "C" int dk_replay_run_grouped(dk_replay* r, int32_t n_groups) {
  if (!r) return fail("null replay");
  if (n_groups < 1) return fail("dk_replay_run_grouped: n_groups must be >= 1");
  if (r->ow > 0) return fail("dk_replay_run_grouped: owner mode runs ungrouped (dk_replay_run)");
  hipSetDevice(r->eng->cfg.device);
  r->have_result = false;
  r->h_csel_ready = false;
  r->tail_ready = false;
  r->file_ready.clear();
  if (r->ck && invalidate_mirrors(r->ck)) return 1;
  r->n_groups = n_groups;
  if (!r->aux.s && r->aux.create(replay_high_priority())) return 1;
  return replay_launch(r);
}

// Wait until file f's selection (f = -1: the commit tail's) of a grouped run is on the host; a device
// error seen by then (flags only grow) is reported the way dk_replay_sync reports it, after the whole
// run (a key-hash collision reruns it). After dk_replay_sync, or for an ungrouped run: the sync.
extern "C" int dk_replay_prefetch_leaf(dk_replay* r, const char* leaf) {
  if (!r || !leaf) return fail("dk_replay_prefetch_leaf: null argument");
  if (!r->ck) return fail("dk_replay_prefetch_leaf: no checkpoint attached");
  for (size_t li = 0; li < r->ck->leaves.size(); li++)
    if (r->ck->leaves[li] == leaf) {
      if (std::find(r->prefetch.begin(), r->prefetch.end(), (int)li) == r->prefetch.end()) r->prefetch.push_back((int)li);
      return 0;
    }
  return fail(std::string("dk_replay_prefetch_leaf: leaf not projected: ") + leaf);
}

extern "C" int dk_replay_wait_file(dk_replay* r, int32_t file) {
  if (!r) return fail("null replay");
  hipSetDevice(r->eng->cfg.device);
  if (r->have_result) return 0;
  const bool grouped = r->n_groups > 0 && r->xw == 0 && r->ck && !r->grp_f0.empty() && r->ev_tail;
  if (!grouped) return dk_replay_sync(r);      // no checkpoint, an ungrouped run, or exchange mode
  if (file >= (int)r->file_ready.size()) return fail("dk_replay_wait_file: bad checkpoint file index");
  // every later group whose files the open has decoded already is issued now, so that its probe,
  // selection copies and mirrors run while the consumer works on the files before it (also on the
  // calls for files of a group that is ready: those return at once below)
  auto issue_ready = [&]() -> int {
    if (!r->run_lazy) return 0;
    const int ng = (int)r->grp_f0.size() - 1;
    while (r->grp_issued > 0 && r->grp_issued < ng && files_ready_now(r->ck, r->grp_f0[r->grp_issued + 1]))
      if (issue_group(r)) return 1;
    return 0;
  };
  if (file >= 0 && r->file_ready[file]) return issue_ready();
  if (file < 0 && r->tail_ready) return 0;
  hipEvent_t ev = r->ev_tail;
  if (file >= 0) {
    int g = 0;
    while (r->grp_f0[g + 1] <= file) g++;
    while (r->grp_issued <= g) if (issue_group(r)) return 1;   // lazy runs issue groups on demand
    ev = r->grp_ev[g];
  }
  if (r->run_lazy) {
    const int ng = (int)r->grp_f0.size() - 1;
    while (r->grp_issued < ng && files_ready_now(r->ck, r->grp_f0[r->grp_issued + 1]))
      if (issue_group(r)) return 1;
  }
  int slot = 0;
  if (file >= 0) {
    int g = 0;
    while (r->grp_f0[g + 1] <= file) g++;
    slot = g + 1;
  }
  HIPOK(hipEventSynchronize(ev));
  if (getenv("DK_VERBOSE") && file >= 0 && r->ck)
    fprintf(stderr, "[dk] file %d ready at %.1f ms\n", file,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r->ck->t_open0).count());
  DState st{}, ps{};
  memcpy(&st, r->h_zstate.data() + (size_t)slot * 2 * sizeof(DState), sizeof st);
  memcpy(&ps, r->h_zstate.data() + (size_t)slot * 2 * sizeof(DState) + sizeof(DState), sizeof ps);
  if (st.err_flags || ps.err_flags) return dk_replay_sync(r);
  if (file < 0) r->tail_ready = true;
  else {
    int g = 0;
    while (r->grp_f0[g + 1] <= file) g++;
    for (int f = r->grp_f0[g]; f < r->grp_f0[g + 1]; f++) r->file_ready[f] = 1;
  }
  return 0;
}

// ---- hash(path)-owner exchange ("alltoall" mode) ----
extern "C" int dk_replay_set_exchange(dk_replay* r, int32_t world, int32_t rank) {
  if (!r) return fail("null replay");
  hipSetDevice(r->eng->cfg.device);
  if (world <= 1) { r->xw = 0; return 0; }
  if (world > 64 || rank < 0 || rank >= world) return fail("dk_replay_set_exchange: bad world / rank");
  if (!r->tail) return fail("dk_replay_set_exchange: no commit tail");
  // this rank's share of the commit tail's keys, by path hash (seed kDecodeSeed, the checkpoint
  // columns' decode-time hash): simple paths only -- a simple checkpoint path never equals a
  // non-simple tail path, and non-simple checkpoint paths stay local candidates
  std::vector<uint64_t> own;
  for (size_t i = 0; i < r->acts.size(); i++) {
    const DJsonAction& a = r->acts[i];
    if (a.kind != JA_ADD && a.kind != JA_REMOVE) continue;
    const CB& pc = r->tail->col[a.kind == JA_ADD ? JL_PATH : JL_RPATH];
    const int64_t row = r->act_row[i];
    const uint8_t* p = pc.chars.data() + pc.offs[row];
    const int32_t n = (int32_t)(pc.offs[row + 1] - pc.offs[row]);
    auto load8 = [&](int32_t j) -> uint64_t {
      uint64_t w = 0;
      for (int b = 0; b < 8 && 8 * j + b < n; b++) w |= (uint64_t)p[8 * j + b] << (8 * b);
      return w;
    };
    uint64_t hp = 0;
    if (simple_path_hash(n, load8, kDecodeSeed, &hp) && hp % (uint64_t)world == (uint64_t)rank) own.push_back(hp);
  }
  std::sort(own.begin(), own.end());
  own.erase(std::unique(own.begin(), own.end()), own.end());
  r->n_owned = (int64_t)own.size();
  if (upload(r->d_owned, own.data(), own.size() * 8, r->stream)) return 1;
  if (r->d_xtot.alloc((size_t)world * 8 + 64)) return 1;
  int64_t total = 0;
  if (r->ck) for (auto& f : r->ck->files) total += f.num_rows;
  if (r->d_cand.n < (size_t)total * 4 + 64 && r->d_cand.alloc((size_t)total * 4 + 64)) return 1;
  if (r->d_xg.alloc((size_t)total * 4 + 64)) return 1;
  HIPOK(hipStreamSynchronize(r->stream));
  r->xw = world; r->xr = rank;
  r->xtot.assign(world, 0);
  return 0;
}

extern "C" int dk_replay_exchange_counts(dk_replay* r, int64_t* counts) {
  hipSetDevice(r->eng->cfg.device);
  if (r->xw <= 0 || r->xphase != 1) return fail("dk_replay_exchange_counts: no exchange-mode run");
  HIPOK(hipStreamSynchronize(r->stream));
  HIPOK(hipMemcpy(r->xtot.data(), r->d_xtot.p, (size_t)r->xw * 8, hipMemcpyDeviceToHost));
  r->n_send = 0;
  for (int o = 0; o < r->xw; o++) { counts[o] = (int64_t)r->xtot[o]; r->n_send += counts[o]; }
  return 0;
}

extern "C" int dk_replay_exchange_pack(dk_replay* r, uint64_t* send) {
  hipSetDevice(r->eng->cfg.device);
  if (r->xw <= 0 || r->xphase != 1) return fail("dk_replay_exchange_pack: counts first");
  hipStream_t s = r->stream;
  if (r->ck && !r->probe_row0.empty() && r->probe_row0.back() > 0) {
    ProbeSet PS{r->d_probe_cols.as<ProbeCols>(), r->d_probe_row0.as<int64_t>(), r->d_probe_sel.as<uint8_t* const>(),
                (int32_t)r->probe.size(), r->probe_row0.back()};
    KTimer::Scope sc(&r->timer, 11, s);
    launch_a2a_pack(PS, r->xw, r->d_xbc.as<unsigned long long>(), send, r->d_xg.as<int32_t>(), r->d_cand.as<int32_t>(),
                    r->d_cand_n.as<unsigned int>(), r->d_state.as<DState>(), s);
  }
  HIPOK(hipStreamSynchronize(s));
  r->xphase = 2;
  return 0;
}

extern "C" int dk_replay_exchange_filter(dk_replay* r, const uint64_t* recv, int64_t n, uint8_t* flags) {
  hipSetDevice(r->eng->cfg.device);
  if (r->xw <= 0) return fail("dk_replay_exchange_filter: not in exchange mode");
  KTimer::Scope sc(&r->timer, 11, r->stream);
  launch_a2a_filter(recv, n, r->d_owned.as<uint64_t>(), r->n_owned, flags, r->stream);
  HIPOK(hipStreamSynchronize(r->stream));
  return 0;
}

extern "C" int dk_replay_exchange_finish(dk_replay* r, const uint8_t* back) {
  hipSetDevice(r->eng->cfg.device);
  if (r->xw <= 0 || r->xphase != 2) return fail("dk_replay_exchange_finish: pack first");
  hipStream_t s = r->stream;
  if (r->ck) {
    if (!r->probe_row0.empty() && r->probe_row0.back() > 0) {
      ProbeSet PS{r->d_probe_cols.as<ProbeCols>(), r->d_probe_row0.as<int64_t>(), r->d_probe_sel.as<uint8_t* const>(),
                  (int32_t)r->probe.size(), r->probe_row0.back()};
      KTimer::Scope sc(&r->timer, 11, s);
      launch_a2a_apply(PS, r->d_xg.as<int32_t>(), back, r->n_send, r->d_slots.as<Slot>(), r->mask, r->d_acts.as<DJsonAction>(),
                       r->d_canon.as<uint8_t>(), r->seed, r->d_cand.as<int32_t>(), r->d_cand_n.as<unsigned int>(),
                       r->d_state.as<DState>(), s);
    }
    if (replay_ckpt_filters(r)) return 1;
  }
  r->xphase = 3;
  return 0;
}

// ---- owner-partitioned reconciliation ("owner" mode) ----
// Every rank parses only its share of the commit files (their batch steps rebased to the global
// replay order, dk_json_tail_rebase_steps) and decodes only its share of the checkpoint. Each key
// (URI(path), dvUniqueId) is owned by rank h mod world. One run, driven by the caller's collectives:
//   begin; tail_counts / tail_pack -> (all-to-all) -> tail_resolve on the owner (the table of its
//   keys, R2-R5 selection of the actions routed to it, counters) -> (reverse all-to-all) ->
//   tail_finish (the origin's tail selection, then its partition / skipping filters);
//   dk_replay_run (decode + key hash of every checkpoint row + routing counts); ckpt_counts /
//   ckpt_pack -> (all-to-all of 8-byte hashes) -> ckpt_lookup -> (reverse) -> ckpt_apply (rows
//   whose hash no tail key has are selected; the rest are candidates); cand_counts / cand_pack ->
//   (all-to-all of candidate keys) -> cand_verify (byte-exact) -> (reverse) -> cand_finish;
//   then dk_replay_sync.
// A key-hash collision among an owner's tail keys is reported by tail_resolve; the caller reduces
// the flag over the ranks and, if any is set, every rank calls dk_replay_owner_reseed and repeats the
// tail exchange with the next seed.
enum : int32_t { OP_IDLE = 0, OP_BEGUN, OP_TAIL_COUNTED, OP_TAIL_PACKED, OP_TAIL_RESOLVED, OP_TAIL_DONE, OP_DECODED,
                 OP_CK_COUNTED, OP_CK_PACKED, OP_CK_APPLIED, OP_CAND_COUNTED, OP_CAND_PACKED, OP_DONE };

static int owner_phase(dk_replay* r, int want, const char* who) {
  if (!r) return fail(std::string(who) + ": null replay");
  hipSetDevice(r->eng->cfg.device);
  if (r->ow <= 0) return fail(std::string(who) + ": not in owner mode (dk_replay_set_owner)");
  if (want >= 0 && r->ophase != want) return fail(std::string(who) + ": called out of order");
  return 0;
}

extern "C" int dk_replay_set_owner(dk_replay* r, int32_t world, int32_t rank) {
  if (!r) return fail("null replay");
  if (world == 0) { r->ow = 0; return 0; }        // (owner mode off)
  // world 1 is a real owner run (one rank through a communicator, e.g. a one-GPU RCCL world)
  if (world < 0 || world > 64 || rank < 0 || rank >= world) return fail("dk_replay_set_owner: bad world / rank");
  if (r->xw > 0) return fail("dk_replay_set_owner: the replay is in hash-exchange mode");
  r->ow = world; r->orank = rank;
  r->ophase = OP_IDLE;
  return 0;
}

namespace dk { hipStream_t replay_stream(dk_replay* r) { return r ? r->stream : nullptr; } }

extern "C" int dk_replay_owner_begin(dk_replay* r) {
  if (owner_phase(r, -1, "dk_replay_owner_begin")) return 1;
  r->have_result = false;
  r->h_csel_ready = false;
  r->n_groups = 0;
  DState st0{};
  st0.err_row = LLONG_MAX;
  // (on the replay's stream, synchronised: a pageable hipMemcpy may return before its DMA lands)
  HIPOK(hipMemcpyAsync(r->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, r->stream));
  HIPOK(hipStreamSynchronize(r->stream));
  r->ophase = OP_BEGUN;
  return 0;
}

extern "C" int dk_replay_owner_tail_counts(dk_replay* r, int64_t* recs, int64_t* bytes) {
  if (owner_phase(r, OP_BEGUN, "dk_replay_owner_tail_counts")) return 1;
  hipStream_t s = r->stream;
  const int na = (int)r->acts.size();
  {
    KTimer::Scope sc(&r->timer, 7, s);
    launch_json_canon(r->d_acts.as<DJsonAction>(), na, r->d_jchars.as<uint8_t>(), r->d_canon.as<uint8_t>(), r->seed,
                      r->d_state.as<DState>(), s);
  }
  // records / key bytes per owner, counted on the device (k_own_tail_count): only 2 x world counts
  // come back
  if (r->d_otot.n < (size_t)r->ow * 16 + 64 && r->d_otot.alloc((size_t)r->ow * 16 + 64)) return 1;
  launch_own_tail_count(r->d_acts.as<DJsonAction>(), na, r->ow, r->d_otot.as<unsigned long long>(), s);
  std::vector<unsigned long long> tot(2 * (size_t)r->ow);
  HIPOK(hipMemcpyAsync(tot.data(), r->d_otot.p, tot.size() * 8, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  r->n_osend = 0;
  for (int o = 0; o < r->ow; o++) {
    recs[o] = (int64_t)tot[o];
    bytes[o] = (int64_t)tot[r->ow + o];
    r->n_osend += recs[o];
  }
  r->ophase = OP_TAIL_COUNTED;
  return 0;
}

// the records and key bytes, owner-major, written by the device (k_own_tail_pack) straight into the
// caller's send buffers
extern "C" int dk_replay_owner_tail_pack(dk_replay* r, void* recs, void* keys) {
  if (owner_phase(r, OP_TAIL_COUNTED, "dk_replay_owner_tail_pack")) return 1;
  hipStream_t s = r->stream;
  if (r->d_osrc.n < (size_t)r->n_osend * 4 + 64 && r->d_osrc.alloc((size_t)r->n_osend * 4 + 64)) return 1;
  if (r->n_osend > 0)
    launch_own_tail_pack(r->d_acts.as<DJsonAction>(), (int)r->acts.size(), r->ow, r->d_otot.as<unsigned long long>(),
                         r->d_canon.as<uint8_t>(), (OwnerKeyRec*)recs, (uint8_t*)keys, r->d_osrc.as<int32_t>(), s);
  HIPOK(hipStreamSynchronize(s));                 // the records leave through the caller's collective
  r->ophase = OP_TAIL_PACKED;
  return 0;
}

extern "C" int dk_replay_owner_tail_resolve(dk_replay* r, const void* recs, int64_t n, const void* keys, int64_t nbytes,
                                            uint8_t* answers, int32_t* flags) {
  if (owner_phase(r, OP_TAIL_PACKED, "dk_replay_owner_tail_resolve")) return 1;
  if (n < 0 || nbytes < 0 || n > INT32_MAX / 2) return fail("dk_replay_owner_tail_resolve: bad sizes");
  hipStream_t s = r->stream;
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n + 16) cap <<= 1;
  r->omask = cap - 1;
  r->n_oacts = n;
  // the received records -> the owner's action table, on the device (k_own_recs_count / _acts)
  long long chunk;
  const int nb = own_recs_blocks(n, &chunk);
  if (r->d_oacts.n < (size_t)n * sizeof(DJsonAction) + 64 && r->d_oacts.alloc((size_t)n * sizeof(DJsonAction) + 64)) return 1;
  if (r->d_orsum.n < (size_t)nb * 8 + 64 && r->d_orsum.alloc((size_t)nb * 8 + 64)) return 1;
  unsigned long long* bsum = r->d_orsum.as<unsigned long long>();
  unsigned long long* total = bsum + nb;
  int* bad = (int*)(bsum + nb + 1);
  HIPOK(hipMemsetAsync(bsum + nb, 0, 16, s));
  launch_own_recs_acts((const OwnerKeyRec*)recs, n, nbytes, bsum, bad, total, r->d_oacts.as<DJsonAction>(), s);
  if (r->d_ocanon.alloc(nbytes + 64)) return 1;
  if (nbytes) HIPOK(hipMemcpyAsync(r->d_ocanon.p, keys, nbytes, hipMemcpyDeviceToDevice, s));
  if (r->d_oslots.alloc(cap * sizeof(Slot)) || r->d_ofp.alloc(cap * sizeof(uint32_t)) || r->d_osel.alloc(n + 16)) return 1;
  DJsonAction* OA = r->d_oacts.as<DJsonAction>();
  Slot* S = r->d_oslots.as<Slot>();
  DState* st = r->d_state.as<DState>();
  launch_slots_init(S, cap, s);
  { KTimer::Scope sc(&r->timer, 8, s); launch_table_insert(OA, (int)n, S, r->omask, s); }
  { KTimer::Scope sc(&r->timer, 9, s); launch_table_update(OA, (int)n, S, r->omask, r->d_ocanon.as<uint8_t>(), st, s); }
  { KTimer::Scope sc(&r->timer, 10, s);
    launch_json_select(OA, (int)n, S, r->omask, r->d_ocanon.as<uint8_t>(), r->d_osel.as<uint8_t>(), st, s); }
  launch_table_fp(S, r->d_ofp.as<uint32_t>(), cap, s);
  if (n) HIPOK(hipMemcpyAsync(answers, r->d_osel.p, n, hipMemcpyDeviceToDevice, s));
  struct { unsigned long long total; int bad, pad; } chk{0, 0, 0};
  DState h{};
  HIPOK(hipMemcpyAsync(&chk, total, 16, hipMemcpyDeviceToHost, s));
  HIPOK(hipMemcpyAsync(&h, r->d_state.p, sizeof h, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  if (n && chk.bad) return fail("dk_replay_owner_tail_resolve: malformed key record");
  if ((int64_t)(n ? chk.total : 0) != nbytes) return fail("dk_replay_owner_tail_resolve: key bytes do not match the records");
  *flags = h.err_flags & E_COLLISION;
  r->ophase = OP_TAIL_RESOLVED;
  return 0;
}

// after a collision anywhere: the next seed, the commit-tail counters cleared, the tail exchange again
extern "C" int dk_replay_owner_reseed(dk_replay* r) {
  if (owner_phase(r, -1, "dk_replay_owner_reseed")) return 1;
  if (r->ophase != OP_TAIL_RESOLVED) return fail("dk_replay_owner_reseed: called out of order");
  DState h{};
  HIPOK(hipStreamSynchronize(r->stream));
  HIPOK(hipMemcpy(&h, r->d_state.p, sizeof h, hipMemcpyDeviceToHost));
  for (int i = 0; i < 5; i++) h.counters[i] = 0;
  h.err_flags &= ~E_COLLISION;
  HIPOK(hipMemcpyAsync(r->d_state.p, &h, sizeof h, hipMemcpyHostToDevice, r->stream));
  HIPOK(hipStreamSynchronize(r->stream));
  if (++r->seed > 64) return fail("replay: repeated key-hash collisions");
  r->ophase = OP_BEGUN;
  return 0;
}

extern "C" int dk_replay_owner_tail_finish(dk_replay* r, const uint8_t* back) {
  if (owner_phase(r, OP_TAIL_RESOLVED, "dk_replay_owner_tail_finish")) return 1;
  hipStream_t s = r->stream;
  const size_t na = r->acts.size();
  if (r->d_jsel.n < na + 16 && r->d_jsel.alloc(na + 16)) return 1;
  HIPOK(hipMemsetAsync(r->d_jsel.p, 0, na + 16, s));
  launch_own_tail_finish(r->d_osrc.as<int32_t>(), (const uint8_t*)back, r->n_osend, r->d_jsel.as<uint8_t>(), s);
  DState* st = r->d_state.as<DState>();
  if (r->has_part && na) {                 // partition pruning on this rank's tail adds (before skipping)
    KTimer::Scope sc(&r->timer, 18, s);
    launch_part_eval(r->tail_maps, r->part.P, r->d_jsel.as<uint8_t>(), st, s);
  }
  if (r->has_skip && na) {                 // data skipping on this rank's selected tail adds
    KTimer::Scope sc(&r->timer, 17, s);
    StatsRows R{};
    R.n = (int64_t)na; R.soff = r->d_tstats_off.as<int64_t>(); R.slen = r->d_tstats_len.as<int32_t>();
    R.chars = r->d_tstats_chars.as<uint8_t>(); R.row_tag = -1000000000000ll;
    launch_stats_eval(R, r->skip.P, r->skip.S, r->d_jsel.as<uint8_t>(), st, s);
  }
  r->ophase = OP_TAIL_DONE;
  return 0;
}

static ProbeSet owner_probe_set(dk_replay* r) {
  return ProbeSet{r->d_probe_cols.as<ProbeCols>(), r->d_probe_row0.as<int64_t>(), r->d_probe_sel.as<uint8_t* const>(),
                  (int32_t)r->probe.size(), r->probe_row0.empty() ? 0 : r->probe_row0.back()};
}

// dk_replay_run in owner mode: the checkpoint decode, every row's key hash, the routing counts
static int owner_launch(dk_replay* r) {
  if (r->ophase != OP_TAIL_DONE) return fail("dk_replay_run (owner mode): finish the commit-tail exchange first");
  hipStream_t s = r->stream;
  r->probe_row0.assign(1, 0);
  if (r->ck) {
    dk_parquet* p = r->ck;
    if (r->lazy && (ensure_open(p) || attach_upto(r, INT_MAX))) return 1;
    HIPOK(hipEventRecord(r->ev_in, p->stream));
    HIPOK(hipStreamWaitEvent(s, r->ev_in, 0));
    DState st0{};
    st0.err_row = LLONG_MAX;
    HIPOK(hipMemcpyAsync(p->d_state.p, &st0, sizeof st0, hipMemcpyHostToDevice, s));
    if (run_pipeline(p, 1, s, false)) return 1;
    if (!r->prefetch.empty()) {
      // the prefetched leaves (add.size) go to host memory now, on the mirror stream, while the
      // row exchanges run: the consumer then finds them there
      if (p->async_open && !p->mir.s && create_mirror_stream(p)) return 1;
      hipStream_t ms = p->async_open ? p->mir.s : p->stream;
      if (!r->ev_pf) HIPOK(hipEventCreateWithFlags(&r->ev_pf, hipEventDisableTiming));
      HIPOK(hipEventRecord(r->ev_pf, s));
      HIPOK(hipStreamWaitEvent(ms, r->ev_pf, 0));
      for (int leaf : r->prefetch)
        for (size_t f = 0; f < p->files.size(); f++)
          if (p->colmap[f][leaf] >= 0 && queue_mirror(p, p->colmap[f][leaf])) return 1;
    }
    const size_t nf = r->probe.size();
    r->probe_run = r->probe;
    r->probe_row0.assign(nf + 1, 0);
    r->probe_sel.resize(nf);
    for (size_t fi = 0; fi < nf; fi++) {
      if (r->seed != kDecodeSeed) r->probe_run[fi].path_hash = nullptr;   // the decode-time hashes use seed 0
      r->probe_row0[fi + 1] = r->probe_row0[fi] + r->probe_run[fi].n_rows;
      r->probe_sel[fi] = r->d_csel[fi]->as<uint8_t>();
    }
    const int64_t total = r->probe_row0[nf];
    if (total >= (1ll << 31) - 1) return fail("owner mode: more than 2^31 checkpoint rows on one rank");
    if (upload(r->d_probe_cols, r->probe_run.data(), nf * sizeof(ProbeCols), s) ||
        upload(r->d_probe_row0, r->probe_row0.data(), (nf + 1) * 8, s) ||
        upload(r->d_probe_sel, r->probe_sel.data(), nf * sizeof(uint8_t*), s)) return 1;
    if (r->d_rowh.n < (size_t)total * 8 + 64 && r->d_rowh.alloc((size_t)total * 8 + 64)) return 1;
    if (r->d_cand.n < (size_t)total * 4 + 64 && r->d_cand.alloc((size_t)total * 4 + 64)) return 1;
    if (r->d_xg.n < (size_t)total * 4 + 64 && r->d_xg.alloc((size_t)total * 4 + 64)) return 1;
    long long chunk;
    const int nb = a2a_blocks(total, &chunk);
    if (r->d_xbc.n < (size_t)nb * r->ow * 8 + 64 && r->d_xbc.alloc((size_t)nb * r->ow * 8 + 64)) return 1;
    if (r->d_xtot.n < (size_t)r->ow * 8 + 64 && r->d_xtot.alloc((size_t)r->ow * 8 + 64)) return 1;
    HIPOK(hipMemsetAsync(r->d_xtot.p, 0, (size_t)r->ow * 8, s));
    HashSink kd; kd.hs.init(kHashSeed(r->seed)); kd.n = 0;       // dvUniqueId stream of "no DV"
    dv_emit(false, nullptr, 0, nullptr, 0, false, 0, kd);
    const uint64_t h_nodv = kd.hs.final_(kd.n);
    const ProbeSet PS = owner_probe_set(r);
    KTimer::Scope sc(&r->timer, 22, s);
    launch_own_rowhash(PS, r->d_rowh.as<uint64_t>(), r->seed, h_nodv, r->d_state.as<DState>(), s);
    if (total > 0)
      launch_own_count(PS, r->d_rowh.as<uint64_t>(), r->ow, r->d_xbc.as<unsigned long long>(),
                       r->d_xtot.as<unsigned long long>(), s);
  }
  r->ophase = OP_DECODED;
  return 0;
}

extern "C" int dk_replay_owner_ckpt_counts(dk_replay* r, int64_t* counts) {
  if (owner_phase(r, OP_DECODED, "dk_replay_owner_ckpt_counts")) return 1;
  HIPOK(hipStreamSynchronize(r->stream));
  r->n_send = 0;
  for (int o = 0; o < r->ow; o++) counts[o] = 0;
  if (r->ck && r->probe_row0.back() > 0) {
    r->xtot.assign(r->ow, 0);
    HIPOK(hipMemcpy(r->xtot.data(), r->d_xtot.p, (size_t)r->ow * 8, hipMemcpyDeviceToHost));
    for (int o = 0; o < r->ow; o++) { counts[o] = (int64_t)r->xtot[o]; r->n_send += counts[o]; }
  }
  r->ophase = OP_CK_COUNTED;
  return 0;
}

extern "C" int dk_replay_owner_ckpt_pack(dk_replay* r, uint64_t* send) {
  if (owner_phase(r, OP_CK_COUNTED, "dk_replay_owner_ckpt_pack")) return 1;
  hipStream_t s = r->stream;
  if (r->n_send > 0) {
    KTimer::Scope sc(&r->timer, 22, s);
    launch_own_pack(owner_probe_set(r), r->d_rowh.as<uint64_t>(), r->ow, r->d_xbc.as<unsigned long long>(), send,
                    r->d_xg.as<int32_t>(), s);
  }
  HIPOK(hipStreamSynchronize(s));
  r->ophase = OP_CK_PACKED;
  return 0;
}

extern "C" int dk_replay_owner_ckpt_lookup(dk_replay* r, const uint64_t* recv, int64_t n, uint8_t* flags) {
  if (owner_phase(r, -1, "dk_replay_owner_ckpt_lookup")) return 1;
  if (r->ophase < OP_TAIL_RESOLVED) return fail("dk_replay_owner_ckpt_lookup: the owner's key table is not built");
  hipStream_t s = r->stream;
  {
    KTimer::Scope sc(&r->timer, 23, s);
    launch_own_lookup(recv, n, r->d_oslots.as<Slot>(), r->d_ofp.as<uint32_t>(), r->omask, flags, s);
  }
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int dk_replay_owner_ckpt_apply(dk_replay* r, const uint8_t* back) {
  if (owner_phase(r, OP_CK_PACKED, "dk_replay_owner_ckpt_apply")) return 1;
  hipStream_t s = r->stream;
  if (r->ck) {
    KTimer::Scope sc(&r->timer, 22, s);
    launch_own_apply(owner_probe_set(r), r->d_xg.as<int32_t>(), back, r->n_send, r->d_cand.as<int32_t>(),
                     r->d_cand_n.as<unsigned int>(), r->d_state.as<DState>(), s);
  }
  HIPOK(hipStreamSynchronize(s));
  r->ophase = OP_CK_APPLIED;
  return 0;
}

extern "C" int dk_replay_owner_cand_counts(dk_replay* r, int64_t* recs, int64_t* bytes) {
  if (owner_phase(r, OP_CK_APPLIED, "dk_replay_owner_cand_counts")) return 1;
  hipStream_t s = r->stream;
  for (int o = 0; o < r->ow; o++) recs[o] = bytes[o] = 0;
  unsigned int nc = 0;
  if (r->ck) HIPOK(hipMemcpy(&nc, r->d_cand_n.p, sizeof nc, hipMemcpyDeviceToHost));
  r->n_ocand = nc;
  if (nc) {
    if (r->d_oc_plen.alloc(nc * 4 + 16) || r->d_oc_dlen.alloc(nc * 4 + 16) || r->d_oc_own.alloc(nc * 4 + 16)) return 1;
    const ProbeSet PS = owner_probe_set(r);
    {
      KTimer::Scope sc(&r->timer, 22, s);
      launch_own_cand_len(PS, r->d_cand.as<int32_t>(), nc, r->d_rowh.as<uint64_t>(), r->ow, r->d_oc_plen.as<int32_t>(),
                          r->d_oc_dlen.as<int32_t>(), r->d_oc_own.as<int32_t>(), s);
    }
    HIPOK(hipStreamSynchronize(s));
    std::vector<int32_t> plen(nc), dlen(nc), own(nc), cand(nc);
    HIPOK(hipMemcpy(plen.data(), r->d_oc_plen.p, nc * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(dlen.data(), r->d_oc_dlen.p, nc * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(own.data(), r->d_oc_own.p, nc * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(cand.data(), r->d_cand.p, nc * 4, hipMemcpyDeviceToHost));
    // owner-major send order (stable): record position and key offset of each candidate
    std::vector<int64_t> start(r->ow + 1, 0), kstart(r->ow + 1, 0);
    for (unsigned i = 0; i < nc; i++) {
      if (own[i] < 0 || own[i] >= r->ow) return fail("owner mode: bad candidate owner");
      recs[own[i]]++;
      bytes[own[i]] += plen[i] + dlen[i];
    }
    for (int o = 0; o < r->ow; o++) { start[o + 1] = start[o] + recs[o]; kstart[o + 1] = kstart[o] + bytes[o]; }
    std::vector<int64_t> rpos(nc), koff(nc);
    std::vector<int32_t> sendg(nc);
    for (unsigned i = 0; i < nc; i++) {
      const int o = own[i];
      rpos[i] = start[o]++;
      koff[i] = kstart[o];
      kstart[o] += plen[i] + dlen[i];
      sendg[rpos[i]] = cand[i];
    }
    if (upload(r->d_oc_rpos, rpos.data(), nc * 8, s) || upload(r->d_oc_koff, koff.data(), nc * 8, s) ||
        upload(r->d_oc_sendg, sendg.data(), nc * 4, s)) return 1;
    HIPOK(hipStreamSynchronize(s));
  }
  r->ophase = OP_CAND_COUNTED;
  return 0;
}

extern "C" int dk_replay_owner_cand_pack(dk_replay* r, void* recs, void* keys) {
  if (owner_phase(r, OP_CAND_COUNTED, "dk_replay_owner_cand_pack")) return 1;
  hipStream_t s = r->stream;
  if (r->n_ocand) {
    KTimer::Scope sc(&r->timer, 22, s);
    launch_own_cand_keys(owner_probe_set(r), r->d_cand.as<int32_t>(), r->n_ocand, r->d_rowh.as<uint64_t>(),
                         r->d_oc_rpos.as<int64_t>(), r->d_oc_koff.as<int64_t>(), r->d_oc_plen.as<int32_t>(),
                         r->d_oc_dlen.as<int32_t>(), (OwnerKeyRec*)recs, (uint8_t*)keys, s);
  }
  HIPOK(hipStreamSynchronize(s));
  r->ophase = OP_CAND_PACKED;
  return 0;
}

extern "C" int dk_replay_owner_cand_verify(dk_replay* r, const void* recs, int64_t n, const void* keys, int64_t nbytes,
                                           uint8_t* answers) {
  if (owner_phase(r, -1, "dk_replay_owner_cand_verify")) return 1;
  if (r->ophase < OP_TAIL_RESOLVED) return fail("dk_replay_owner_cand_verify: the owner's key table is not built");
  if (n < 0 || nbytes < 0) return fail("dk_replay_owner_cand_verify: bad sizes");
  hipStream_t s = r->stream;
  if (n) {
    std::vector<OwnerKeyRec> R(n);
    HIPOK(hipMemcpy(R.data(), recs, n * sizeof(OwnerKeyRec), hipMemcpyDeviceToHost));
    std::vector<int64_t> koff(n);
    int64_t k = 0;
    for (int64_t i = 0; i < n; i++) {
      if (R[i].key_len < 0 || R[i].canon_len < 0 || R[i].canon_len > R[i].key_len)
        return fail("dk_replay_owner_cand_verify: malformed key record");
      koff[i] = k;
      k += R[i].key_len;
    }
    if (k != nbytes) return fail("dk_replay_owner_cand_verify: key bytes do not match the records");
    if (upload(r->d_ov_koff, koff.data(), n * 8, s)) return 1;
    KTimer::Scope sc(&r->timer, 23, s);
    launch_own_verify((const OwnerKeyRec*)recs, n, r->d_ov_koff.as<int64_t>(), (const uint8_t*)keys, r->d_oslots.as<Slot>(),
                      r->omask, r->d_oacts.as<DJsonAction>(), r->d_ocanon.as<uint8_t>(), answers, s);
  }
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int dk_replay_owner_cand_finish(dk_replay* r, const uint8_t* back) {
  if (owner_phase(r, OP_CAND_PACKED, "dk_replay_owner_cand_finish")) return 1;
  hipStream_t s = r->stream;
  if (r->ck) {
    if (r->n_ocand) {
      KTimer::Scope sc(&r->timer, 22, s);
      launch_own_cand_finish(owner_probe_set(r), r->d_oc_sendg.as<int32_t>(), back, r->n_ocand, r->d_state.as<DState>(), s);
    }
    if (replay_ckpt_filters(r)) return 1;
  }
  r->ophase = OP_DONE;
  return 0;
}

extern "C" int dk_replay_sync(dk_replay* r) {
  hipSetDevice(r->eng->cfg.device);   // this thread may not have used the device yet
  hipStream_t s = r->stream;
  if (r->xw > 0 && r->xphase != 3) return fail("dk_replay_sync: the exchange-mode run has not finished its exchange");
  if (r->ow > 0 && r->ophase != OP_DONE) return fail("dk_replay_sync: the owner-mode run has not finished its exchanges");
  if (r->ck && r->n_groups > 0 && r->xw == 0)      // a lazy grouped run: the groups not issued yet
    while (r->grp_issued + 1 < (int)r->grp_f0.size()) if (issue_group(r)) return 1;
  if (r->ck && ensure_open(r->ck)) return 1;        // (an asynchronous open has finished by now)
  for (int attempt = 0; attempt < 8; attempt++) {
    HIPOK(hipStreamSynchronize(s));
    if (r->ck && r->n_groups > 0) HIPOK(hipStreamWaitEvent(r->ck->stream, r->ev_out, 0));
    r->timer.collect();
    if (r->ck) { r->ck->timer.collect(); if (check_state(r->ck)) return 1; }
    HIPOK(hipMemcpy(&r->h_state, r->d_state.p, sizeof(DState), hipMemcpyDeviceToHost));
    if (r->h_state.err_flags & E_COLLISION) {     // 64-bit key-hash collision: rebuild with a new seed
      if (r->ow > 0) return fail("replay (owner mode): a key-hash collision was not resolved by the tail exchange");
      r->seed++;
      const int32_t xw = r->xw;                   // (exchange mode: the rebuilt run probes locally)
      r->xw = 0;
      const int rc = replay_launch(r);
      r->xw = xw;
      if (rc) return 1;
      continue;
    }
    if (r->h_state.err_flags & E_PART) {
      const long long row = r->h_state.err_row;
      return fail(std::string("Evaluating the partition expression: java.lang.NumberFormatException for a partition "
                              "value of ") +
                  (row < 0 ? "commit-tail action " + std::to_string(row + 1000000000000ll)
                           : "checkpoint row " + std::to_string(row)));
    }
    if (r->h_state.err_flags & E_STATS) {
      const long long row = r->h_state.err_row;
      return fail(std::string("Evaluating the data skipping filter: couldn't decode add.stats of ") +
                  (row < 0 ? "commit-tail action " + std::to_string(row + 1000000000000ll)
                           : "checkpoint row " + std::to_string(row)));
    }
    if (r->h_state.err_flags & (E_URI | E_UTF8)) {
      std::vector<DJsonAction> acts(r->acts.size());
      if (!acts.empty()) HIPOK(hipMemcpy(acts.data(), r->d_acts.p, acts.size() * sizeof(DJsonAction), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < acts.size(); i++)
        if (acts[i].status) {
          const CB& pc = r->tail->col[acts[i].kind != JA_REMOVE ? JL_PATH : JL_RPATH];
          int64_t row = r->act_row[i];
          std::string path(pc.chars.begin() + pc.offs[row], pc.chars.begin() + pc.offs[row + 1]);
          return fail((acts[i].status == -1 ? "java.net.URISyntaxException: Illegal character in path: "
                                            : "malformed UTF-8 in action key (unsupported): ") + path);
        }
      return fail(std::string(r->h_state.err_flags & E_URI ? "java.net.URISyntaxException" : "malformed UTF-8 key") +
                  " in checkpoint row " + std::to_string(r->h_state.err_row));
    }
    r->have_result = true;
    return 0;
  }
  return fail("replay: repeated key-hash collisions");
}

extern "C" int dk_replay_counters(dk_replay* r, int64_t out[5]) {
  if (!r->have_result) return fail("replay has no result (call dk_replay_sync)");
  for (int i = 0; i < 5; i++) out[i] = (int64_t)(r->h_state.counters[i] + r->h_state.ckpt_counters[i]);
  return 0;
}

extern "C" int dk_replay_counters_split(dk_replay* r, int64_t tail[5], int64_t ckpt[5]) {
  if (!r->have_result) return fail("replay has no result (call dk_replay_sync)");
  for (int i = 0; i < 5; i++) { tail[i] = (int64_t)r->h_state.counters[i]; ckpt[i] = (int64_t)r->h_state.ckpt_counters[i]; }
  return 0;
}

extern "C" int dk_replay_json_selection(dk_replay* r, uint8_t* out, int64_t n) {
  hipSetDevice(r->eng->cfg.device);   // this thread may not have used the device yet
  if (!r->have_result && !r->tail_ready) return fail("replay has no result");
  if (!r->tail || n != r->tail->rows) return fail("bad selection size");
  memset(out, 0, n);
  std::vector<uint8_t> sel(r->acts.size());
  if (!r->have_result && r->tail_ready && r->h_zjsel.size() >= sel.size()) {
    if (!sel.empty()) memcpy(sel.data(), r->h_zjsel.data(), sel.size());   // grouped run: copied before ev_tail
  } else if (!sel.empty()) HIPOK(hipMemcpy(sel.data(), r->d_jsel.p, sel.size(), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < sel.size(); i++) if (r->acts[i].kind != JA_REMOVE && sel[i]) out[r->act_row[i]] = 1;
  return 0;
}

extern "C" int dk_replay_ckpt_selection(dk_replay* r, int32_t file, uint8_t* out, int64_t n) {
  hipSetDevice(r->eng->cfg.device);   // this thread may not have used the device yet
  if (!r->have_result) return fail("replay has no result");
  if (!r->ck || file < 0 || file >= (int)r->d_csel.size()) return fail("bad checkpoint file index");
  if (n != r->ck->files[file].num_rows) return fail("bad selection size");
  if (r->probe[file].n_rows == 0) { memset(out, 0, n); return 0; }
  HIPOK(hipMemcpy(out, r->d_csel[file]->p, n, hipMemcpyDeviceToHost));
  return 0;
}

// Zero-copy view of checkpoint file `file`'s selection (one byte per row, valid until the next run
// or free). The first call after a sync moves every file's selection to one pinned block in one
// round of async copies and one synchronisation.
extern "C" int dk_replay_ckpt_selection_host(dk_replay* r, int32_t file, const uint8_t** out) {
  hipSetDevice(r->eng->cfg.device);
  *out = nullptr;
  if (!r->ck || file < 0 || file >= (int)r->d_csel.size()) return fail("bad checkpoint file index");
  if (!r->have_result && !(file < (int)r->file_ready.size() && r->file_ready[file]))
    return fail("replay has no result");
  if (!r->h_csel_ready) {
    const int nf = (int)r->d_csel.size();
    r->h_csel_off.assign(nf + 1, 0);
    for (int f = 0; f < nf; f++) r->h_csel_off[f + 1] = r->h_csel_off[f] + ((r->ck->files[f].num_rows + 63) & ~(int64_t)63);
    if (r->h_csel.alloc(r->h_csel_off[nf] + 64)) return 1;
    for (int f = 0; f < nf; f++) {
      const int64_t n = r->ck->files[f].num_rows;
      if (r->probe[f].n_rows == 0) memset(r->h_csel.data() + r->h_csel_off[f], 0, n);
      else if (n) HIPOK(hipMemcpyAsync(r->h_csel.data() + r->h_csel_off[f], r->d_csel[f]->p, n, hipMemcpyDeviceToHost, r->stream));
    }
    HIPOK(hipStreamSynchronize(r->stream));
    r->h_csel_ready = true;
  }
  *out = r->h_csel.data() + r->h_csel_off[file];
  return 0;
}

extern "C" int dk_replay_ckpt_selection_bits(dk_replay* r, int32_t file, void* dst, int64_t n, int32_t dst_on_device) {
  hipSetDevice(r->eng->cfg.device);   // this thread may not have used the device yet
  if (!r->have_result) return fail("dk_replay_ckpt_selection_bits: no result (run + sync first)");
  if (!r->ck || file < 0 || file >= (int)r->d_csel.size()) return fail("bad checkpoint file index");
  if (n != r->ck->files[file].num_rows) return fail("bad selection size");
  const int64_t nb = (n + 7) / 8;
  hipStream_t s = r->stream;
  if (dst_on_device) {
    launch_pack_bits(r->d_csel[file]->as<uint8_t>(), n, (uint8_t*)dst, s);
    HIPOK(hipStreamSynchronize(s));
    return 0;
  }
  DBuf tmp;
  if (tmp.alloc(nb + 16)) return 1;
  launch_pack_bits(r->d_csel[file]->as<uint8_t>(), n, tmp.as<uint8_t>(), s);
  HIPOK(hipMemcpyAsync(dst, tmp.p, nb, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

// every checkpoint file's packed selection at dst + offsets[file] (one pack launch per file, one
// synchronisation for all): the multi-GPU exchange fills its collective buffer with this
extern "C" int dk_replay_ckpt_selection_bits_all(dk_replay* r, void* dst, const int64_t* offsets, int32_t dst_on_device) {
  hipSetDevice(r->eng->cfg.device);
  if (!r->have_result) return fail("dk_replay_ckpt_selection_bits_all: no result (run + sync first)");
  if (!r->ck) return 0;
  hipStream_t s = r->stream;
  const int nf = (int)r->d_csel.size();
  int64_t total = 0;
  for (int f = 0; f < nf; f++) total = std::max(total, offsets[f] + (r->ck->files[f].num_rows + 7) / 8);
  DBuf tmp;
  uint8_t* base = (uint8_t*)dst;
  if (!dst_on_device) { if (tmp.alloc(total + 16)) return 1; base = tmp.as<uint8_t>(); }
  for (int f = 0; f < nf; f++)
    launch_pack_bits(r->d_csel[f]->as<uint8_t>(), r->ck->files[f].num_rows, base + offsets[f], s);
  if (!dst_on_device && total) HIPOK(hipMemcpyAsync(dst, tmp.p, total, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

// checkpoint files whose data skipping reads add.stats_parsed (after dk_replay_set_skipping)
extern "C" int dk_replay_stats_parsed_files(dk_replay* r) {
  int n = 0;
  if (r && r->has_skip) for (const auto& R : r->ck_parsed) n += R.n > 0;
  return n;
}

extern "C" int dk_replay_kernel_stats(dk_replay* r, int32_t i, const char** name, double* avg_us, int64_t* count) {
  if (i < 0 || i >= KTimer::K) return 1;
  // decode kernels are timed by the parquet object's timer, the rest by the replay's
  const KTimer* t = (r->ck && (i <= 6 || (i >= 13 && i <= 16) || (i >= 19 && i <= 21))) ? &r->ck->timer : &r->timer;
  *name = t->names[i];
  if (!*name) return 1;
  *count = t->cnt[i];
  *avg_us = t->cnt[i] ? 1000.0 * t->sum_ms[i] / (double)t->cnt[i] : 0.0;
  return 0;
}

extern "C" void dk_replay_free(dk_replay* r) {
  if (!r) return;
  hipSetDevice(r->eng->cfg.device);
  // the attached checkpoint set forgets this run's group events now (it may be closed next); the
  // rest -- events, blocks back to the caches, the streams -- is released in the background, like a
  // closed checkpoint set (close 3 -> 0.1 ms at C3)
  // (its streams drain first: their kernels may read the checkpoint's and the tail's buffers)
  hipStreamSynchronize(r->stream);
  if (r->aux.s) hipStreamSynchronize(r->aux.s);
  if (r->ck) { hipStreamSynchronize(r->ck->stream); r->ck->file_done.clear(); r->ck = nullptr; }
  reaper().run([r] {
    hipSetDevice(r->eng->cfg.device);
    if (r->ev_in) hipEventDestroy(r->ev_in);
    if (r->ev_out) hipEventDestroy(r->ev_out);
    if (r->ev_pf) hipEventDestroy(r->ev_pf);
    if (r->ev_tail) hipEventDestroy(r->ev_tail);
    for (hipEvent_t e : r->grp_ev) hipEventDestroy(e);
    SyncedRelease drained;
    delete r;
  });
}

// ------------------------------------------------------------------------------------------------
// Streaming ParquetHandler reader (dk_reader_*): ParquetHandler.readParquetFiles as Kernel consumes
// it -- a CloseableIterator<ColumnarBatch> of at most parquet.reader.batch-size rows per batch, in
// input-file order then row order (ParquetHandler.java:59-68, ParquetFileReader.java:54-147), safe to
// close early (ScanImpl.java:376-392). The files are decoded on the GPU when the reader opens; batches
// are then shipped to pinned host memory one window (about 1M rows) at a time: validity bits and
// int32 offsets are built on the device (k_arrow_window), the other buffers are slices of the
// decoded columns.
// ------------------------------------------------------------------------------------------------
namespace {

struct PinnedBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  ~PinnedBuf() { if (p) hipHostFree(p); }
  int reserve(size_t n) {
    if (n <= cap) return 0;
    if (p) { hipHostFree(p); p = nullptr; cap = 0; }
    if (hipHostMalloc((void**)&p, n, hipHostMallocDefault) != hipSuccess) { p = nullptr; return fail("hipHostMalloc failed"); }
    cap = n;
    return 0;
  }
};

struct WinLeaf {                 // one leaf's buffers inside a window (offsets into the host buffer)
  int present = 0, null_only = 0;
  int64_t nv = 0, nchars = 0;
  size_t o_rowdef = 0, o_entdef = 0, o_fixed = 0, o_chars = 0, o_bits = 0, o_offs = 0, o_rowoffs = 0;
};

struct RWin {                    // rows [r0, r0 + nr) of one file in pinned host memory
  int file = -1;
  int64_t r0 = 0, nr = 0;
  PinnedBuf buf;
  std::vector<WinLeaf> leaf;
  size_t o_rowidx = 0;
  int refs = 0;                  // outstanding batches (+1 while it is the reader's current window)
};

}  // namespace

struct dk_reader {
  StreamH own;
  dk_engine* eng = nullptr;
  dk_parquet* p = nullptr;
  std::vector<std::string> leaves;
  int B = 1024;
  int64_t W = 1 << 20;
  bool row_index = false;
  int file = 0;
  int64_t next = 0;              // next row of `file`
  RWin* cur = nullptr;
  std::vector<RWin*> pool;       // windows no batch refers to any more
  std::mutex mu;                 // batches may be released from other threads
  int outstanding = 0;           // live batches
  bool closed = false;
  DBuf d_stage, d_ovf;
  // row-index map per file: (first selected row, file row) of every selected row group
  std::vector<std::vector<std::pair<int64_t, int64_t>>> rgmap;
  ~dk_reader() {
    delete cur;
    for (RWin* w : pool) delete w;
    if (p) dk_parquet_close(p);
  }
};

struct dk_batch_impl {
  dk_batch pub;
  std::vector<dk_batch_column> cols;
  dk_reader* rd;
  RWin* win;
};

static void reader_maybe_free(dk_reader* r, std::unique_lock<std::mutex>& lk) {
  if (r->closed && r->outstanding == 0) { lk.unlock(); delete r; }
}

extern "C" int dk_reader_open(dk_engine* e, const char* const* paths, int32_t n_files, const char* const* leaves,
                              int32_t n_leaves, const dk_read_options* opt, dk_reader** out) {
  *out = nullptr;
  if (!e) return fail("null engine");
  hipSetDevice(e->cfg.device);
  std::unique_ptr<dk_reader> r(new dk_reader());
  r->eng = e;
  r->B = e->cfg.parquet_batch_size > 0 ? e->cfg.parquet_batch_size : 1024;
  if (opt && opt->window_rows > 0) r->W = opt->window_rows;
  r->W = std::max<int64_t>(r->B, r->W / r->B * r->B);
  r->row_index = opt && opt->row_index;
  for (int i = 0; i < n_leaves; i++) r->leaves.push_back(leaves[i]);
  if (r->own.create()) return 1;
  // the predicate prunes row groups (best effort, like parquet-mr's StatisticsFilter: never rows)
  std::vector<std::vector<int32_t>> groups(n_files > 0 ? n_files : 0);
  for (int32_t fi = 0; fi < n_files; fi++) {
    FileM f;
    f.path = paths[fi];
    if (read_footer(f) || parse_footer(f)) return 1;
    std::vector<uint8_t> keep(f.rgs.size() + 1, 1);
    int32_t ng = 0;
    if (opt && opt->predicate &&
        dk_parquet_prune_row_groups(paths[fi], opt->predicate, keep.data(), (int32_t)keep.size(), &ng)) return 1;
    int64_t at = 0, sel = 0;
    std::vector<std::pair<int64_t, int64_t>> m;
    for (int32_t g = 0; g < (int32_t)f.rgs.size(); g++) {
      if (keep[g]) { groups[fi].push_back(g); m.push_back({sel, at}); sel += f.rgs[g].num_rows; }
      at += f.rgs[g].num_rows;
    }
    r->rgmap.push_back(m);
  }
  if (parquet_open(e, paths, n_files, leaves, n_leaves, &groups, &r->p, opt ? opt->field_ids : nullptr)) return 1;
  if (dk_parquet_decode(r->p) || dk_parquet_sync(r->p)) return 1;
  if (r->d_ovf.alloc(16)) return 1;
  *out = r.release();
  return 0;
}

// file rows [r0, r0 + nr) of the reader's current file into a window
static int load_window(dk_reader* r, RWin* w, int64_t r0, int64_t nr) {
  dk_parquet* p = r->p;
  const int fi = r->file;
  const hipStream_t s = r->own.s;
  const size_t nl = r->leaves.size();
  w->file = fi; w->r0 = r0; w->leaf.assign(nl, WinLeaf());
  // value / char ranges of the window (two int64 per leaf and level from HBM)
  struct Rng { int64_t v0 = 0, v1 = 0, c0 = 0, c1 = 0; };
  std::vector<Rng> rg(nl);
  for (;;) {
    bool fits = true;
    for (size_t li = 0; li < nl; li++) {
      const int ci = p->colmap[fi][li];
      if (ci < 0) continue;
      const DColumn& c = p->h_cols[ci];
      Rng& q = rg[li];
      q = Rng();
      if (c.null_only) { q.v0 = c.max_rep > 0 ? 0 : r0; q.v1 = c.max_rep > 0 ? 0 : r0 + nr; continue; }
      if (c.max_rep > 0) {
        HIPOK(hipMemcpy(&q.v0, c.row_offs + r0, 8, hipMemcpyDeviceToHost));
        HIPOK(hipMemcpy(&q.v1, c.row_offs + r0 + nr, 8, hipMemcpyDeviceToHost));
      } else { q.v0 = r0; q.v1 = r0 + nr; }
      if (c.phys == PT_BYTE_ARRAY) {
        HIPOK(hipMemcpy(&q.c0, c.offs + q.v0, 8, hipMemcpyDeviceToHost));
        HIPOK(hipMemcpy(&q.c1, c.offs + q.v1, 8, hipMemcpyDeviceToHost));
      }
      if (q.c1 - q.c0 >= (1ll << 31) - 1 || q.v1 - q.v0 >= (1ll << 31) - 1) fits = false;
    }
    if (fits) break;
    if (nr <= r->B) return fail("Error reading Parquet file: " + p->files[fi].path + " (a batch exceeds 2 GiB)");
    nr = std::max<int64_t>(r->B, nr / 2 / r->B * r->B);           // int32 offsets: a smaller window
  }
  w->nr = nr;
  // host layout, 64-byte aligned pieces; device staging for bits + int32 offsets
  size_t hsz = 0, dsz = 0;
  auto take = [](size_t& at, size_t n) { at = (at + 63) & ~(size_t)63; const size_t o = at; at += n; return o; };
  std::vector<size_t> d_bits(nl), d_offs(nl), d_roffs(nl);
  for (size_t li = 0; li < nl; li++) {
    const int ci = p->colmap[fi][li];
    WinLeaf& L = w->leaf[li];
    L.o_rowdef = take(hsz, nr);
    if (ci < 0) continue;
    const DColumn& c = p->h_cols[ci];
    L.present = 1; L.null_only = c.null_only;
    L.nv = rg[li].v1 - rg[li].v0;
    L.nchars = rg[li].c1 - rg[li].c0;
    if (c.max_rep > 0) { L.o_entdef = take(hsz, L.nv); L.o_rowoffs = take(hsz, 4 * (nr + 1)); d_roffs[li] = take(dsz, 4 * (nr + 1)); }
    L.o_bits = take(hsz, 8 * ((L.nv + 63) / 64)); d_bits[li] = take(dsz, 8 * ((L.nv + 63) / 64));
    if (c.phys == PT_BYTE_ARRAY) {
      L.o_offs = take(hsz, 4 * (L.nv + 1)); d_offs[li] = take(dsz, 4 * (L.nv + 1));
      L.o_chars = take(hsz, L.nchars);
    } else {
      L.o_fixed = take(hsz, (size_t)L.nv * c.width);
    }
  }
  if (r->row_index) w->o_rowidx = take(hsz, 8 * nr);
  if (w->buf.reserve(hsz + 64)) return 1;
  if (dsz > r->d_stage.n && r->d_stage.alloc(dsz + 64)) return 1;
  uint8_t* H = w->buf.p;
  uint8_t* D = r->d_stage.as<uint8_t>();
  HIPOK(hipMemsetAsync(r->d_ovf.p, 0, 4, s));
  for (size_t li = 0; li < nl; li++) {
    const int ci = p->colmap[fi][li];
    WinLeaf& L = w->leaf[li];
    if (ci < 0) { memset(H + L.o_rowdef, 0, nr); continue; }
    const DColumn& c = p->h_cols[ci];
    HIPOK(hipMemcpyAsync(H + L.o_rowdef, c.row_def + r0, nr, hipMemcpyDeviceToHost, s));
    if (c.null_only) {          // no value anywhere: all-null values, empty maps
      memset(H + L.o_bits, 0, 8 * ((L.nv + 63) / 64));
      if (c.max_rep > 0) { memset(H + L.o_rowoffs, 0, 4 * (nr + 1)); }
      if (c.phys == PT_BYTE_ARRAY) memset(H + L.o_offs, 0, 4 * (L.nv + 1));
      else memset(H + L.o_fixed, 0, (size_t)L.nv * c.width);
      continue;
    }
    const int64_t v0 = rg[li].v0;
    ArrowWin A{};
    A.def = c.max_rep > 0 ? c.entry_def + v0 : c.row_def + r0;
    A.offs = c.phys == PT_BYTE_ARRAY ? c.offs + v0 : nullptr;
    A.row_offs = c.max_rep > 0 ? c.row_offs + r0 : nullptr;
    A.nv = L.nv; A.nr = c.max_rep > 0 ? nr : 0; A.max_def = c.max_def;
    A.bits = (uint64_t*)(D + d_bits[li]);
    A.offs32 = (int32_t*)(D + d_offs[li]);
    A.row_offs32 = (int32_t*)(D + d_roffs[li]);
    A.overflow = r->d_ovf.as<int32_t>();
    launch_arrow_window(A, s);
    HIPOK(hipMemcpyAsync(H + L.o_bits, D + d_bits[li], 8 * ((L.nv + 63) / 64), hipMemcpyDeviceToHost, s));
    if (c.max_rep > 0) {
      HIPOK(hipMemcpyAsync(H + L.o_rowoffs, D + d_roffs[li], 4 * (nr + 1), hipMemcpyDeviceToHost, s));
      if (L.nv) HIPOK(hipMemcpyAsync(H + L.o_entdef, c.entry_def + v0, L.nv, hipMemcpyDeviceToHost, s));
    }
    if (c.phys == PT_BYTE_ARRAY) {
      HIPOK(hipMemcpyAsync(H + L.o_offs, D + d_offs[li], 4 * (L.nv + 1), hipMemcpyDeviceToHost, s));
      if (L.nchars) HIPOK(hipMemcpyAsync(H + L.o_chars, c.chars + rg[li].c0, L.nchars, hipMemcpyDeviceToHost, s));
    } else if (L.nv) {
      HIPOK(hipMemcpyAsync(H + L.o_fixed, c.fixed + v0 * c.width, (size_t)L.nv * c.width, hipMemcpyDeviceToHost, s));
    }
  }
  // row index: the file row of each selected row (row groups pruned by the predicate are skipped,
  // as parquet-mr's getCurrentRowIndex counts them)
  if (r->row_index) {
    int64_t* ri = (int64_t*)(H + w->o_rowidx);
    const auto& m = r->rgmap[fi];
    size_t k = 0;
    for (int64_t i = 0; i < nr; i++) {
      const int64_t row = r0 + i;
      while (k + 1 < m.size() && m[k + 1].first <= row) k++;
      ri[i] = m.empty() ? row : m[k].second + (row - m[k].first);
    }
  }
  int32_t ovf = 0;
  HIPOK(hipMemcpyAsync(&ovf, r->d_ovf.p, 4, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  if (ovf) return fail("Error reading Parquet file: " + p->files[fi].path + " (int32 offset overflow)");
  return 0;
}

extern "C" int dk_reader_next(dk_reader* r, dk_batch** out) {
  *out = nullptr;
  if (!r) return fail("null reader");
  hipSetDevice(r->eng->cfg.device);
  dk_parquet* p = r->p;
  for (;;) {
    if (r->file >= (int)p->files.size()) return 0;
    const int64_t n = p->files[r->file].num_rows;
    if (r->next >= n) { r->file++; r->next = 0; continue; }
    if (!r->cur || r->cur->file != r->file || r->next >= r->cur->r0 + r->cur->nr) {
      RWin* w = nullptr;
      {
        std::lock_guard<std::mutex> g(r->mu);
        if (r->cur) { if (--r->cur->refs == 0) r->pool.push_back(r->cur); r->cur = nullptr; }
        if (!r->pool.empty()) { w = r->pool.back(); r->pool.pop_back(); }
      }
      if (!w) w = new RWin();
      if (load_window(r, w, r->next, std::min<int64_t>(r->W, n - r->next))) {
        std::lock_guard<std::mutex> g(r->mu);
        r->pool.push_back(w);
        return 1;
      }
      w->refs = 1;
      r->cur = w;
    }
    break;
  }
  RWin* w = r->cur;
  const int64_t b0 = r->next, b1 = std::min<int64_t>(b0 + r->B, w->r0 + w->nr);
  const int64_t rb = b0 - w->r0, nb = b1 - b0;
  auto* b = new dk_batch_impl();
  b->rd = r; b->win = w;
  b->cols.resize(r->leaves.size());
  uint8_t* H = w->buf.p;
  for (size_t li = 0; li < r->leaves.size(); li++) {
    const WinLeaf& L = w->leaf[li];
    dk_batch_column& c = b->cols[li];
    memset(&c, 0, sizeof c);
    c.row_def = H + L.o_rowdef + rb;
    if (!L.present) { c.present = 0; c.n_values = nb; continue; }
    const DColumn& d = p->h_cols[p->colmap[w->file][li]];
    c.present = 1; c.phys = d.phys; c.width = d.width; c.max_def = d.max_def; c.max_rep = d.max_rep; c.rep_def = d.rep_def;
    c.validity = H + L.o_bits;
    if (d.max_rep > 0) {
      c.row_offs = (const int32_t*)(H + L.o_rowoffs) + rb;
      c.entry_def = H + L.o_entdef;
      c.value_offset = c.row_offs[0];
      c.n_values = c.row_offs[nb] - c.row_offs[0];
    } else {
      c.value_offset = rb;
      c.n_values = nb;
    }
    if (d.phys == PT_BYTE_ARRAY) { c.offs = (const int32_t*)(H + L.o_offs); c.chars = H + L.o_chars; }
    else c.fixed = H + L.o_fixed;
  }
  b->pub.file = w->file;
  b->pub.n_rows = nb;
  b->pub.n_cols = (int32_t)b->cols.size();
  b->pub.cols = b->cols.data();
  b->pub.row_index = r->row_index ? (const int64_t*)(H + w->o_rowidx) + rb : nullptr;
  {
    std::lock_guard<std::mutex> g(r->mu);
    w->refs++;
    r->outstanding++;
  }
  r->next = b1;
  *out = &b->pub;
  return 0;
}

extern "C" void dk_batch_release(dk_batch* pub) {
  if (!pub) return;
  dk_batch_impl* b = reinterpret_cast<dk_batch_impl*>(pub);   // pub is the first member
  dk_reader* r = b->rd;
  std::unique_lock<std::mutex> lk(r->mu);
  if (--b->win->refs == 0) r->pool.push_back(b->win);
  r->outstanding--;
  delete b;
  reader_maybe_free(r, lk);
}

extern "C" void dk_reader_close(dk_reader* r) {
  if (!r) return;
  hipSetDevice(r->eng->cfg.device);
  std::unique_lock<std::mutex> lk(r->mu);
  if (r->closed) return;
  r->closed = true;
  if (r->cur) { if (--r->cur->refs == 0) r->pool.push_back(r->cur); r->cur = nullptr; }
  reader_maybe_free(r, lk);
}

extern "C" int64_t dk_reader_num_rows(dk_reader* r, int32_t file) {
  return r ? dk_parquet_num_rows(r->p, file) : -1;
}

// ------------------------------------------------------------------------------------------------
// Deletion vectors (dk_dv_*): DeletionVectorUtils.loadNewDvAndBitmap for every DV of a scan
// (internal/deletionvectors/DeletionVectorUtils.java:27-37, DeletionVectorStoredBitmap.java:50-129,
// RoaringBitmapArray.java:100-229, Base85Codec.java, DeletionVectorDescriptor.java:176-231).
// Host: descriptor -> bytes (Z85 inline payload or the file range), size and CRC-32 checks, the
// RoaringBitmapArray / portable-roaring headers; device: container expansion (dk_dv.hip).
// ------------------------------------------------------------------------------------------------
namespace {

// Base85Codec.decodeBlocks (Z85 alphabet); false when the text is not 5-aligned or not valid Z85
bool z85_decode(const std::string& in, std::vector<uint8_t>& out) {
  static const char* enc = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";
  int8_t dec[128];
  memset(dec, -1, sizeof dec);
  for (int i = 0; i < 85; i++) dec[(uint8_t)enc[i]] = (int8_t)i;
  if (in.size() % 5) return false;
  out.clear();
  for (size_t i = 0; i < in.size(); i += 5) {
    uint64_t sum = 0;
    for (int k = 0; k < 5; k++) {
      const uint8_t c = (uint8_t)in[i + k];
      if (c >= 128 || dec[c] < 0) return false;
      sum = sum * 85 + (uint64_t)dec[c];
    }
    const uint32_t v = (uint32_t)sum;                   // (int) sum: the low 32 bits, big-endian
    out.push_back(v >> 24); out.push_back(v >> 16); out.push_back(v >> 8); out.push_back(v);
  }
  return true;
}

uint32_t crc32_ieee(const uint8_t* p, size_t n) {       // java.util.zip.CRC32
  static uint32_t tab[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
  });
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// Hadoop Path.toString of a local path: "file:/x/y" -> "/x/y" for reading
std::string local_path(const std::string& p) {
  if (p.compare(0, 7, "file://") == 0 && p.size() > 7 && p[7] == '/') return p.substr(7);
  if (p.compare(0, 5, "file:") == 0) return p.substr(5);
  return p;
}

std::string join_path(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  return a.back() == '/' ? a + b : a + "/" + b;
}

// LE reader over one serialized RoaringBitmapArray (BufferUnderflowException past the end)
struct LeBuf {
  const uint8_t* p; size_t n, at = 0; bool bad = false;
  bool need(size_t k) { if (bad || at + k > n) { bad = true; return false; } return true; }
  uint32_t u16() { if (!need(2)) return 0; uint32_t v = p[at] | (p[at + 1] << 8); at += 2; return v; }
  uint32_t u32() { if (!need(4)) return 0; uint32_t v; memcpy(&v, p + at, 4); at += 4; return v; }
  uint64_t u64() { if (!need(8)) return 0; uint64_t v; memcpy(&v, p + at, 8); at += 8; return v; }
};

// org.roaringbitmap 0.9.25 RoaringArray.deserialize (portable format) of one 32-bit bitmap at b.at:
// appends its containers (values high << 32 | key << 16 | low) and returns its serialized size
bool roaring32(LeBuf& b, size_t base_off, uint64_t high, std::vector<DvCont>& out, uint64_t* maxv, std::string* err) {
  const size_t start = b.at;
  const uint32_t cookie = b.u32();
  const bool hasrun = (cookie & 0xFFFF) == 12347;
  if (!hasrun && cookie != 12346) { *err = "org.roaringbitmap.InvalidRoaringFormat: I failed to find one of the right cookies."; return false; }
  const uint32_t size = hasrun ? (cookie >> 16) + 1 : b.u32();
  if (size > (1u << 16)) { *err = "org.roaringbitmap.InvalidRoaringFormat: Size too large"; return false; }
  std::vector<uint8_t> runbits;
  if (hasrun) { const size_t nb = (size + 7) / 8; if (!b.need(nb)) return false; runbits.assign(b.p + b.at, b.p + b.at + nb); b.at += nb; }
  std::vector<uint32_t> key(size), card(size);
  for (uint32_t k = 0; k < size; k++) { key[k] = b.u16(); card[k] = b.u16() + 1; }
  if (!hasrun || size >= 4) { if (!b.need(4ull * size)) return false; b.at += 4ull * size; }   // offset header
  for (uint32_t k = 0; k < size; k++) {
    const bool run = hasrun && (runbits[k / 8] >> (k % 8) & 1);
    DvCont c{};
    c.word0 = (int64_t)((high << 32 | (uint64_t)key[k] << 16) >> 6);
    if (run) {
      c.type = DV_RUN;
      c.src = (int64_t)(base_off + b.at);
      const uint32_t nr = b.u16();
      c.n = (int32_t)nr;
      if (!b.need(4ull * nr)) return false;
      uint32_t last = 0;
      for (uint32_t r = 0; r < nr; r++) {
        const uint32_t st = b.p[b.at + 4 * r] | (b.p[b.at + 4 * r + 1] << 8);
        const uint32_t ln = b.p[b.at + 4 * r + 2] | (b.p[b.at + 4 * r + 3] << 8);
        if (st + ln > 0xFFFF) { *err = "org.roaringbitmap.InvalidRoaringFormat: run past the container"; return false; }
        last = std::max(last, st + ln);
      }
      b.at += 4ull * nr;
      if (nr) *maxv = std::max<uint64_t>(*maxv, high << 32 | (uint64_t)key[k] << 16 | last);
    } else if (card[k] > 4096) {
      c.type = DV_BITMAP;
      c.src = (int64_t)(base_off + b.at);
      if (!b.need(8192)) return false;
      for (int w = 1023; w >= 0; w--) {
        uint64_t v; memcpy(&v, b.p + b.at + 8 * w, 8);
        if (v) { *maxv = std::max<uint64_t>(*maxv, high << 32 | (uint64_t)key[k] << 16 | (uint64_t)(64 * w + 63 - __builtin_clzll(v))); break; }
      }
      b.at += 8192;
    } else {
      c.type = DV_ARRAY;
      c.src = (int64_t)(base_off + b.at);
      c.n = (int32_t)card[k];
      if (!b.need(2ull * card[k])) return false;
      const uint32_t lastv = b.p[b.at + 2 * (card[k] - 1)] | (b.p[b.at + 2 * (card[k] - 1) + 1] << 8);
      *maxv = std::max<uint64_t>(*maxv, high << 32 | (uint64_t)key[k] << 16 | lastv);
      b.at += 2ull * card[k];
    }
    out.push_back(c);
  }
  (void)start;
  return true;
}

}  // namespace

struct dk_dv_set {
  StreamH own;
  dk_engine* eng = nullptr;
  DBuf d_bits;
  std::vector<int64_t> word0, nbits;    // per DV: first word, bits (max deleted row + 1; 0 = empty)
};

extern "C" int dk_dv_load(dk_engine* e, const char* table_root, const dk_dv_descriptor* dvs, int32_t n,
                          dk_dv_set** out) {
  *out = nullptr;
  if (!e) return fail("null engine");
  hipSetDevice(e->cfg.device);
  std::unique_ptr<dk_dv_set> S(new dk_dv_set());
  S->eng = e;
  if (S->own.create()) return 1;
  const std::string root = table_root ? table_root : "";
  std::vector<uint8_t> blob;
  std::vector<DvCont> conts;
  std::vector<std::vector<DvCont>> per(n);
  S->nbits.assign(n, 0);
  S->word0.assign(n, 0);
  for (int32_t i = 0; i < n; i++) {
    const dk_dv_descriptor& d = dvs[i];
    const std::string st = d.storage_type ? d.storage_type : "", pd = d.path_or_inline ? d.path_or_inline : "";
    if (d.cardinality == 0) continue;                          // isEmpty: no read
    // isInline() compares the storage type by reference (`storageType == INLINE_DV_MARKER`,
    // DeletionVectorDescriptor.java:176-178): a descriptor read from the log never is, so every DV
    // takes the on-disk branch, and an "i" DV fails in getAbsolutePath (:190-216)
    std::string path;
    if (st == "u") {
      if (pd.size() < 20) return fail("java.lang.StringIndexOutOfBoundsException: deletion vector path " + pd);
      std::vector<uint8_t> u;
      if (!z85_decode(pd.substr(pd.size() - 20), u) || u.size() < 16)
        return fail("java.lang.IllegalArgumentException: Input is not valid Z85: " + pd.substr(pd.size() - 20));
      char id[40];
      snprintf(id, sizeof id, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", u[0], u[1], u[2],
               u[3], u[4], u[5], u[6], u[7], u[8], u[9], u[10], u[11], u[12], u[13], u[14], u[15]);
      const std::string prefix = pd.substr(0, pd.size() - 20);
      path = join_path(prefix.empty() ? root : join_path(root, prefix), std::string("deletion_vector_") + id + ".bin");
    } else if (st == "p") {
      if (pd.find(':') == std::string::npos) return fail("java.lang.IllegalArgumentException: Relative URIs are not supported for DVs");
      path = pd;
    } else {
      return fail("A uri " + pd + " which cannot be turned into a relative path as found in the transaction log");
    }
    // FileReadRequest(offset, sizeInBytes + 8): 4-byte big-endian size, the bitmap, 4-byte CRC-32
    const std::string lp = local_path(path);
    FILE* fp = fopen(lp.c_str(), "rb");
    if (!fp) return fail("Couldn't load dv: java.io.FileNotFoundException: " + path);
    const int64_t off = d.has_offset ? d.offset : 0;
    std::vector<uint8_t> raw((size_t)std::max(0, d.size_in_bytes) + 8);
    const bool ok = fseek(fp, off, SEEK_SET) == 0 && fread(raw.data(), 1, raw.size(), fp) == raw.size();
    fclose(fp);
    if (!ok) return fail("Couldn't load dv: java.io.EOFException: " + path);
    const uint32_t size_file = (uint32_t)raw[0] << 24 | raw[1] << 16 | raw[2] << 8 | raw[3];
    if ((int32_t)size_file != d.size_in_bytes) return fail("DV size mismatch");
    const uint8_t* body = raw.data() + 4;
    const size_t nb = (size_t)d.size_in_bytes;
    const uint32_t want = (uint32_t)body[nb] << 24 | body[nb + 1] << 16 | body[nb + 2] << 8 | body[nb + 3];
    if (crc32_ieee(body, nb) != want) return fail("DV checksum mismatch");
    // RoaringBitmapArray.readFrom: magic, then the native or portable array of 32-bit bitmaps
    const size_t base = blob.size();
    blob.insert(blob.end(), body, body + nb);
    LeBuf b{blob.data() + base, nb};
    std::string err;
    uint64_t maxv = 0;
    bool any = false;
    const uint32_t magic = b.u32();
    if (magic == 1681511377u) {                                 // portable
      const uint64_t nbm = b.u64();
      if ((int64_t)nbm < 0) return fail("Couldn't load dv: java.io.IOException: Invalid RoaringBitmapArray length (" + std::to_string((int64_t)nbm) + " < 0)");
      if (nbm > 0x7fffffffull) return fail("Couldn't load dv: java.io.IOException: Invalid RoaringBitmapArray length (" + std::to_string(nbm) + " > 2147483647)");
      for (uint64_t k = 0; k < nbm && !b.bad; k++) {
        const int32_t key = (int32_t)b.u32();
        if (key < 0) return fail("Couldn't load dv: java.io.IOException: Invalid unsigned entry in RoaringBitmapArray (" + std::to_string(key) + ")");
        const size_t before = per[i].size();
        if (!roaring32(b, base, (uint64_t)key, per[i], &maxv, &err)) break;
        any = any || per[i].size() > before;
      }
    } else if (magic == 1681511376u) {                          // native
      const int32_t nbm = (int32_t)b.u32();
      if (nbm < 0) return fail("Couldn't load dv: java.io.IOException: Invalid RoaringBitmapArray length (" + std::to_string(nbm) + " < 0)");
      for (int32_t k = 0; k < nbm && !b.bad; k++) {
        const uint32_t bsize = b.u32();
        const size_t at0 = b.at;
        const size_t before = per[i].size();
        if (!roaring32(b, base, (uint64_t)k, per[i], &maxv, &err)) break;
        any = any || per[i].size() > before;
        b.at = at0 + bsize;
      }
    } else {
      return fail("Couldn't load dv: java.io.IOException: Unexpected RoaringBitmapArray magic number " + std::to_string((int32_t)magic));
    }
    if (!err.empty()) return fail("Couldn't load dv: " + err);
    if (b.bad || b.at > nb) return fail("Couldn't load dv: java.nio.BufferUnderflowException");
    if (any) {
      if (maxv >= (1ull << 36)) return fail("deletion vector row index too large for a dense bitmap");
      S->nbits[i] = (int64_t)maxv + 1;
    }
  }
  // one zeroed word array for all DVs; containers carry their DV's word base
  int64_t words = 0;
  for (int32_t i = 0; i < n; i++) {
    S->word0[i] = words;
    const int64_t nw = (S->nbits[i] + 63) / 64;
    for (DvCont c : per[i]) { c.out_word = words; c.nwords = nw; conts.push_back(c); }
    words += nw;
  }
  const hipStream_t s = S->own.s;
  if (S->d_bits.alloc((size_t)std::max<int64_t>(words, 1) * 8)) return 1;
  HIPOK(hipMemsetAsync(S->d_bits.p, 0, (size_t)std::max<int64_t>(words, 1) * 8, s));
  if (!conts.empty()) {
    DBuf d_blob, d_conts;
    if (upload(d_blob, blob.data(), blob.size(), s) || upload(d_conts, conts.data(), conts.size() * sizeof(DvCont), s)) return 1;
    launch_dv_expand(d_conts.as<DvCont>(), (int)conts.size(), d_blob.as<uint8_t>(), S->d_bits.as<unsigned long long>(), s);
    HIPOK(hipStreamSynchronize(s));
  }
  HIPOK(hipStreamSynchronize(s));
  *out = S.release();
  return 0;
}

extern "C" int64_t dk_dv_num_bits(dk_dv_set* S, int32_t i) {
  return S && i >= 0 && i < (int32_t)S->nbits.size() ? S->nbits[i] : -1;
}

extern "C" int dk_dv_bitmap(dk_dv_set* S, int32_t i, void* dst, int64_t nbytes, int32_t dst_on_device) {
  if (!S || i < 0 || i >= (int32_t)S->nbits.size()) return fail("bad deletion vector index");
  hipSetDevice(S->eng->cfg.device);
  const int64_t need = (S->nbits[i] + 7) / 8;
  if (nbytes < need) return fail("dk_dv_bitmap: destination too small");
  if (need) HIPOK(hipMemcpyAsync(dst, S->d_bits.as<uint8_t>() + S->word0[i] * 8, need,
                                 dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, S->own.s));
  HIPOK(hipStreamSynchronize(S->own.s));
  return 0;
}

extern "C" int dk_dv_selection(dk_dv_set* S, int32_t i, const int64_t* row_index, int64_t n, uint8_t* sel) {
  if (!S || i < 0 || i >= (int32_t)S->nbits.size()) return fail("bad deletion vector index");
  hipSetDevice(S->eng->cfg.device);
  for (int64_t k = 0; k < n; k++)       // RoaringBitmapArray.contains: checkArgument(value >= 0 && <= max)
    if (row_index[k] < 0) return fail("java.lang.IllegalArgumentException: row index " + std::to_string(row_index[k]));
  DBuf d_rows, d_sel;
  const hipStream_t s = S->own.s;
  if (upload(d_rows, row_index, (size_t)n * 8, s) || d_sel.alloc((size_t)n + 1)) return 1;
  launch_dv_select(S->d_bits.as<unsigned long long>() + S->word0[i], S->nbits[i], d_rows.as<long long>(), n,
                   d_sel.as<uint8_t>(), s);
  if (n) HIPOK(hipMemcpyAsync(sel, d_sel.p, n, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  return 0;
}

extern "C" void dk_dv_free(dk_dv_set* S) {
  if (!S) return;
  hipSetDevice(S->eng->cfg.device);
  delete S;
}

// ------------------------------------------------------------------------------------------------
// Checkpoint Parquet writer (Table.checkpoint -> ParquetHandler.writeParquetFileAtomically,
// kernel-defaults/.../engine/DefaultParquetHandler.java:110-163 over parquet-mr's writer): the
// CHECKPOINT_SCHEMA file (SingleAction.java:30-37 with each action's FULL_SCHEMA), encoded on the
// device (dk_encode.hip). Row group 0 holds the rows built on the host (JSON action lines shredded
// here with DefaultJsonRow's type rules); each later row group holds the surviving add rows of one
// old checkpoint file, gathered on the device from its decoded columns by the replay's selection.
// v1 data pages of <= 262144 rows: levels as RLE/bit-packed hybrid (one bit-packed run), PLAIN
// values, snappy (or uncompressed); Thrift compact page headers and footer written here.
// ------------------------------------------------------------------------------------------------
namespace dk {
struct EncSrc {
  const uint8_t* row_def; const int64_t* row_offs; const uint8_t* entry_def;
  const uint8_t* fixed; const int64_t* offs; const uint8_t* chars;
  int32_t width, is_str, repeated, max_def_new;
  int32_t entry_def_old;
  uint8_t defmap[16], emap[16];
};
struct SzBlock { long long src; int32_t n; int32_t pad; };
void enc_exscan(const long long*, long long, long long*, long long*, long long*, hipStream_t);
long long enc_scan_blocks(long long);
void enc_sel_rows(const uint8_t*, long long, long long*, long long*, long long*, long long*, int32_t*, hipStream_t);
void enc_count(const EncSrc&, const int32_t*, long long, long long*, long long*, long long*, int*, hipStream_t);
void enc_fill(const EncSrc&, const int32_t*, long long, const long long*, const long long*, const long long*, uint8_t*,
              uint8_t*, uint8_t*, int32_t*, uint8_t*, long long*, hipStream_t);
void enc_bitpack(const uint8_t*, long long, int, uint8_t*, hipStream_t);
void enc_plain_str(const int32_t*, const long long*, const uint8_t*, long long, long long, long long, uint8_t*, hipStream_t);
void enc_snappy(const uint8_t*, const SzBlock*, int, long long, uint8_t*, int32_t*, hipStream_t);
}  // namespace dk

namespace {
enum { W_REQ = 0, W_OPT = 1, W_REP = 2 };
enum { WC_NONE = -1, WC_UTF8 = 0, WC_MAP = 1, WC_LIST = 3 };
struct WNode {
  std::string name; int rep; int phys; int conv;
  std::vector<int> kids; int leaf = -1; int def = 0, replv = 0;   // levels at this node (inclusive)
};
struct WLeaf {
  std::string path; int node; int phys, width, max_def, max_rep;
  std::vector<std::string> comps;
  std::vector<int> chain;                 // node indices root-child .. leaf
  // host-built rows (row group 0)
  std::vector<uint8_t> def, rep, fixed, chars;
  std::vector<int32_t> lens;
};
struct WSchema {
  std::vector<WNode> nodes;               // preorder, nodes[0] = root
  std::vector<WLeaf> leaves;
  int add(int parent, const char* name, int rep, int phys = -1, int conv = WC_NONE) {
    WNode n; n.name = name; n.rep = rep; n.phys = phys; n.conv = conv;
    nodes.push_back(n);
    const int id = (int)nodes.size() - 1;
    if (parent >= 0) nodes[parent].kids.push_back(id);
    return id;
  }
  int str(int p, const char* n, int rep) { return add(p, n, rep, PT_BYTE_ARRAY, WC_UTF8); }
  int map(int p, const char* n, int rep, int value_rep) {
    const int m = add(p, n, rep, -1, WC_MAP);
    const int kv = add(m, "key_value", W_REP);
    str(kv, "key", W_REQ); str(kv, "value", value_rep);
    return m;
  }
  int list(int p, const char* n, int rep) {
    const int l = add(p, n, rep, -1, WC_LIST);
    const int g = add(l, "list", W_REP);
    str(g, "element", W_REQ);
    return l;
  }
  void dv(int p) {
    const int d = add(p, "deletionVector", W_OPT);
    str(d, "storageType", W_REQ); str(d, "pathOrInlineDv", W_REQ); add(d, "offset", W_OPT, PT_INT32);
    add(d, "sizeInBytes", W_REQ, PT_INT32); add(d, "cardinality", W_REQ, PT_INT64);
  }
  void build() {
    const int root = add(-1, "schema", W_REQ);
    int t = add(root, "txn", W_OPT);
    str(t, "appId", W_REQ); add(t, "version", W_REQ, PT_INT64); add(t, "lastUpdated", W_OPT, PT_INT64);
    int a = add(root, "add", W_OPT);
    str(a, "path", W_REQ); map(a, "partitionValues", W_REQ, W_OPT); add(a, "size", W_REQ, PT_INT64);
    add(a, "modificationTime", W_REQ, PT_INT64); add(a, "dataChange", W_REQ, PT_BOOLEAN); dv(a);
    map(a, "tags", W_OPT, W_OPT); add(a, "baseRowId", W_OPT, PT_INT64); add(a, "defaultRowCommitVersion", W_OPT, PT_INT64);
    str(a, "stats", W_OPT);
    int r = add(root, "remove", W_OPT);
    str(r, "path", W_REQ); add(r, "deletionTimestamp", W_OPT, PT_INT64); add(r, "dataChange", W_REQ, PT_BOOLEAN);
    add(r, "extendedFileMetadata", W_OPT, PT_BOOLEAN); map(r, "partitionValues", W_OPT, W_OPT); add(r, "size", W_OPT, PT_INT64);
    str(r, "stats", W_OPT); map(r, "tags", W_OPT, W_OPT); dv(r); add(r, "baseRowId", W_OPT, PT_INT64);
    add(r, "defaultRowCommitVersion", W_OPT, PT_INT64);
    int m = add(root, "metaData", W_OPT);
    str(m, "id", W_REQ); str(m, "name", W_OPT); str(m, "description", W_OPT);
    int f = add(m, "format", W_REQ); str(f, "provider", W_REQ); map(f, "options", W_OPT, W_REQ);
    str(m, "schemaString", W_REQ); list(m, "partitionColumns", W_REQ); add(m, "createdTime", W_OPT, PT_INT64);
    map(m, "configuration", W_REQ, W_REQ);
    int pr = add(root, "protocol", W_OPT);
    add(pr, "minReaderVersion", W_REQ, PT_INT32); add(pr, "minWriterVersion", W_REQ, PT_INT32);
    list(pr, "readerFeatures", W_OPT); list(pr, "writerFeatures", W_OPT);
    int dm = add(root, "domainMetadata", W_OPT);
    str(dm, "domain", W_REQ); str(dm, "configuration", W_REQ); add(dm, "removed", W_REQ, PT_BOOLEAN);
    // levels and leaves (preorder = the footer's schema list order = column order)
    std::vector<int> stack;
    walk(0, 0, 0, stack);
  }
  void walk(int id, int def, int rep, std::vector<int>& chain) {
    WNode& n = nodes[id];
    if (id != 0) {
      if (n.rep != W_REQ) def++;
      if (n.rep == W_REP) rep++;
      chain.push_back(id);
    }
    n.def = def; n.replv = rep;
    if (n.phys >= 0) {
      WLeaf L;
      L.node = id; L.phys = n.phys; L.max_def = def; L.max_rep = rep; L.chain = chain;
      L.width = n.phys == PT_INT64 ? 8 : n.phys == PT_INT32 ? 4 : n.phys == PT_BOOLEAN ? 1 : 0;
      for (int c : chain) { L.comps.push_back(nodes[c].name); L.path += (L.path.empty() ? "" : ".") + nodes[c].name; }
      n.leaf = (int)leaves.size();
      leaves.push_back(std::move(L));
    }
    for (int k : std::vector<int>(n.kids)) walk(k, def, rep, chain);
    if (id != 0) chain.pop_back();
  }
};

// Dremel shredding of one JSON value (DefaultJsonRow's type rules: strings must be JSON strings,
// ints / longs integral in range, booleans JSON booleans; a required field missing or null and a
// null array element or required map value are errors)
struct Shredder {
  WSchema& S;
  const std::vector<JNode>& N;
  void push(WLeaf& L, int r, int d, const JNode* v) {
    L.def.push_back((uint8_t)d);
    if (L.max_rep) L.rep.push_back((uint8_t)r);
    if (d < L.max_def) return;
    if (L.phys == PT_BYTE_ARRAY) {
      const std::string& s = as_str(N, *v);
      L.lens.push_back((int32_t)s.size());
      L.chars.insert(L.chars.end(), s.begin(), s.end());
    } else if (L.phys == PT_INT64) {
      const int64_t x = as_long(N, *v);
      L.fixed.insert(L.fixed.end(), (const uint8_t*)&x, (const uint8_t*)&x + 8);
    } else if (L.phys == PT_INT32) {
      const int32_t x = as_int(N, *v);
      L.fixed.insert(L.fixed.end(), (const uint8_t*)&x, (const uint8_t*)&x + 4);
    } else {
      L.fixed.push_back(as_bool(N, *v) ? 1 : 0);
    }
  }
  void nulls(int id, int r, int d) {
    const WNode& n = S.nodes[id];
    if (n.leaf >= 0) { push(S.leaves[n.leaf], r, d, nullptr); return; }
    for (int k : n.kids) nulls(k, r, d);
  }
  void value(int id, const JNode* v, int r, int d) {       // d: def of the parent
    const WNode& n = S.nodes[id];
    if (!v || v->t == J_NULL) {
      if (n.rep == W_REQ) throw JErr{"Field `" + n.name + "` is not nullable, but it is missing or null"};
      nulls(id, r, d);
      return;
    }
    const int dd = n.rep == W_OPT ? d + 1 : d;
    if (n.leaf >= 0) { push(S.leaves[n.leaf], r, dd, v); return; }
    if (n.conv == WC_MAP) {
      if (v->t != J_OBJ) mismatch(N, *v, "map");
      const WNode& kv = S.nodes[n.kids[0]];
      const int key = kv.kids[0], val = kv.kids[1];
      if (v->kv.empty()) { nulls(n.kids[0], r, dd); return; }
      for (size_t i = 0; i < v->kv.size(); i++) {
        const int ri = i ? kv.replv : r;
        WLeaf& KL = S.leaves[S.nodes[key].leaf];
        KL.def.push_back((uint8_t)(dd + 1)); KL.rep.push_back((uint8_t)ri);
        KL.lens.push_back((int32_t)v->kv[i].first.size());
        KL.chars.insert(KL.chars.end(), v->kv[i].first.begin(), v->kv[i].first.end());
        const JNode& x = N[v->kv[i].second];
        if (x.t == J_NULL && S.nodes[val].rep == W_REQ)
          throw JErr{"Map type expects no nulls in values, but received `null` as value"};
        value(val, &x, ri, dd + 1);
      }
      return;
    }
    if (n.conv == WC_LIST) {
      if (v->t != J_ARR) mismatch(N, *v, "array");
      const WNode& g = S.nodes[n.kids[0]];
      if (v->arr.empty()) { nulls(n.kids[0], r, dd); return; }
      for (size_t i = 0; i < v->arr.size(); i++) {
        const JNode& x = N[v->arr[i]];
        if (x.t == J_NULL) throw JErr{"Array type expects no nulls as elements, but received `null` as array element"};
        value(g.kids[0], &x, i ? g.replv : r, dd + 1);
      }
      return;
    }
    if (v->t != J_OBJ) mismatch(N, *v, "object");
    for (int k : n.kids) value(k, member(N, *v, S.nodes[k].name.c_str()), r, dd);
  }
};

// Thrift compact protocol writer (the footer and page headers)
struct TWriter {
  std::vector<uint8_t> b;
  std::vector<int> last{0};
  void varint(uint64_t v) { while (v >= 0x80) { b.push_back((uint8_t)(v | 0x80)); v >>= 7; } b.push_back((uint8_t)v); }
  void zz(int64_t v) { varint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void field(int id, int type) {
    const int d = id - last.back();
    if (d > 0 && d <= 15) b.push_back((uint8_t)((d << 4) | type));
    else { b.push_back((uint8_t)type); zz(id); }
    last.back() = id;
  }
  void i32(int id, int64_t v) { field(id, 5); zz(v); }
  void i64(int id, int64_t v) { field(id, 6); zz(v); }
  void str(int id, const std::string& s) { field(id, 8); varint(s.size()); b.insert(b.end(), s.begin(), s.end()); }
  void begin(int id) { field(id, 12); last.push_back(0); }
  void end() { b.push_back(0); last.pop_back(); }
  void list(int id, int etype, size_t n) {
    field(id, 9);
    if (n < 15) b.push_back((uint8_t)((n << 4) | etype)); else { b.push_back((uint8_t)(0xf0 | etype)); varint(n); }
  }
  void lbegin() { last.push_back(0); }             // a struct element of a list
  void lend() { b.push_back(0); last.pop_back(); }
};

struct WChunk { int64_t offset = 0, comp = 0, unc = 0, nlev = 0; };
}  // namespace

struct dk_ckpt_writer {
  dk_engine* eng = nullptr;
  StreamH own;
  hipStream_t s = nullptr;
  std::string path;
  FILE* fp = nullptr;
  int codec = 1;                          // 1 SNAPPY, 0 UNCOMPRESSED
  WSchema S;
  int64_t host_rows = 0, off = 4, total_rows = 0;
  std::vector<std::vector<WChunk>> rgs;   // per row group, per leaf
  std::vector<int64_t> rg_rows;
  DBuf d_def, d_rep, d_vals, d_lens, d_chars, d_coff, d_tmp, d_sums, d_total, d_ubuf, d_cbuf, d_clens, d_blocks;
  DBuf d_rows, d_rowpos, d_lv, d_vv, d_cc, d_lb, d_vb, d_cb, d_err;
};

namespace {
// one leaf's level / value arrays, already in device memory (d_def, d_rep, d_vals | d_lens + d_chars
// + d_coff), over `nrows` rows whose level / value / char boundaries at page starts are in pb
// (3 x (np + 1): level, value, char): encode, compress, append to the file
int write_chunk(dk_ckpt_writer* w, WLeaf& L, int64_t nlev, const std::vector<int64_t>& lb, const std::vector<int64_t>& vb,
                const std::vector<int64_t>& cb, WChunk& out) {
  hipStream_t s = w->s;
  const int np = (int)lb.size() - 1;
  auto bw_of = [](int m) { int b = 0; while ((1 << b) <= m) b++; return m == 0 ? 0 : b; };
  const int bwd = bw_of(L.max_def), bwr = bw_of(L.max_rep);
  auto hyb = [](int64_t n, int bw) -> int64_t {           // 4-byte length + varint header + groups
    const int64_t g = (n + 7) / 8;
    uint64_t h = ((uint64_t)g << 1) | 1; int hb = 1; while (h >= 0x80) { h >>= 7; hb++; }
    return 4 + hb + g * bw;
  };
  std::vector<int64_t> poff(np + 1, 0), psz(np);
  for (int p = 0; p < np; p++) {
    const int64_t nl = lb[p + 1] - lb[p], nv = vb[p + 1] - vb[p];
    int64_t z = (L.max_rep ? hyb(nl, bwr) : 0) + (L.max_def ? hyb(nl, bwd) : 0);
    z += L.phys == PT_BYTE_ARRAY ? 4 * nv + (cb[p + 1] - cb[p]) : L.phys == PT_BOOLEAN ? (nv + 7) / 8 : nv * L.width;
    psz[p] = z; poff[p + 1] = poff[p] + z;
  }
  if (poff[np] > (int64_t)w->d_ubuf.n && w->d_ubuf.alloc((size_t)poff[np] + 64)) return 1;
  uint8_t* U = w->d_ubuf.as<uint8_t>();
  // page bodies: [rep levels][def levels][values]; the 4-byte lengths and varint headers from the host
  std::vector<uint8_t> head(16);
  for (int p = 0; p < np; p++) {
    int64_t at = poff[p];
    const int64_t nl = lb[p + 1] - lb[p], nv = vb[p + 1] - vb[p];
    auto levels = [&](const DBuf& lv, int bw) -> int {
      const int64_t g = (nl + 7) / 8, tot = hyb(nl, bw);
      int n = 0;
      uint32_t len = (uint32_t)(tot - 4);
      for (int k = 0; k < 4; k++) head[n++] = (uint8_t)(len >> (8 * k));
      uint64_t h = ((uint64_t)g << 1) | 1;
      while (h >= 0x80) { head[n++] = (uint8_t)(h | 0x80); h >>= 7; }
      head[n++] = (uint8_t)h;
      HIPOK(hipMemcpyAsync(U + at, head.data(), n, hipMemcpyHostToDevice, s));
      HIPOK(hipStreamSynchronize(s));
      enc_bitpack(lv.as<uint8_t>() + lb[p], nl, bw, U + at + n, s);
      at += tot;
      return 0;
    };
    if (L.max_rep && levels(w->d_rep, bwr)) return 1;
    if (L.max_def && levels(w->d_def, bwd)) return 1;
    if (L.phys == PT_BYTE_ARRAY) {
      enc_plain_str(w->d_lens.as<int32_t>(), w->d_coff.as<long long>(), w->d_chars.as<uint8_t>(), vb[p], nv, cb[p], U + at, s);
    } else if (L.phys == PT_BOOLEAN) {
      enc_bitpack(w->d_vals.as<uint8_t>() + vb[p], nv, 1, U + at, s);
    } else if (nv > 0) {
      HIPOK(hipMemcpyAsync(U + at, w->d_vals.as<uint8_t>() + vb[p] * L.width, (size_t)(nv * L.width), hipMemcpyDeviceToDevice, s));
    }
  }
  // compression: snappy in 64 KiB blocks per page (one stream per page: varint length + blocks)
  std::vector<std::vector<uint8_t>> pages(np);
  if (w->codec == 1) {
    std::vector<SzBlock> blk;
    std::vector<int> bpage;
    for (int p = 0; p < np; p++)
      for (int64_t a = 0; a < psz[p]; a += 65536) {
        SzBlock b{}; b.src = poff[p] + a; b.n = (int32_t)std::min<int64_t>(65536, psz[p] - a);
        blk.push_back(b); bpage.push_back(p);
      }
    const long long cap = 65536 + 65536 / 6 + 64;
    if (!blk.empty()) {
      if (upload(w->d_blocks, blk.data(), blk.size() * sizeof(SzBlock), s)) return 1;
      if ((size_t)(blk.size() * cap) > w->d_cbuf.n && w->d_cbuf.alloc(blk.size() * cap)) return 1;
      if (blk.size() * 4 > w->d_clens.n && w->d_clens.alloc(blk.size() * 4 + 16)) return 1;
      enc_snappy(U, w->d_blocks.as<SzBlock>(), (int)blk.size(), cap, w->d_cbuf.as<uint8_t>(), w->d_clens.as<int32_t>(), s);
      std::vector<int32_t> cl(blk.size());
      HIPOK(hipMemcpyAsync(cl.data(), w->d_clens.p, cl.size() * 4, hipMemcpyDeviceToHost, s));
      HIPOK(hipStreamSynchronize(s));
      std::vector<uint8_t> tmp;
      for (size_t i = 0; i < blk.size(); i++) {
        std::vector<uint8_t>& pg = pages[bpage[i]];
        if (pg.empty()) {                                  // preamble: varint of the page's bytes
          uint64_t v = (uint64_t)psz[bpage[i]];
          while (v >= 0x80) { pg.push_back((uint8_t)(v | 0x80)); v >>= 7; }
          pg.push_back((uint8_t)v);
        }
        const size_t at = pg.size();
        pg.resize(at + cl[i]);
        HIPOK(hipMemcpyAsync(pg.data() + at, w->d_cbuf.as<uint8_t>() + i * cap, cl[i], hipMemcpyDeviceToHost, s));
      }
      HIPOK(hipStreamSynchronize(s));
    }
    for (int p = 0; p < np; p++)
      if (pages[p].empty()) pages[p].push_back(0);       // an empty page: varint 0, no tags
  } else {
    for (int p = 0; p < np; p++) {
      pages[p].resize(psz[p]);
      if (psz[p]) HIPOK(hipMemcpyAsync(pages[p].data(), U + poff[p], psz[p], hipMemcpyDeviceToHost, s));
    }
    HIPOK(hipStreamSynchronize(s));
  }
  out.offset = w->off; out.nlev = nlev; out.unc = 0; out.comp = 0;
  for (int p = 0; p < np; p++) {
    TWriter t;
    t.i32(1, 0);                                  // DATA_PAGE
    t.i32(2, psz[p]);
    t.i32(3, (int64_t)pages[p].size());
    t.begin(5);                                   // DataPageHeader
    t.i32(1, lb[p + 1] - lb[p]); t.i32(2, 0); t.i32(3, 3); t.i32(4, 3);
    t.end();
    t.b.push_back(0);
    if (fwrite(t.b.data(), 1, t.b.size(), w->fp) != t.b.size() ||
        (!pages[p].empty() && fwrite(pages[p].data(), 1, pages[p].size(), w->fp) != pages[p].size()))
      return fail("checkpoint write failed: " + w->path);
    w->off += (int64_t)(t.b.size() + pages[p].size());
    out.unc += (int64_t)t.b.size() + psz[p];
    out.comp += (int64_t)(t.b.size() + pages[p].size());
  }
  return 0;
}

std::vector<int64_t> page_rows(int64_t nrows) {
  const int64_t PR = 262144;
  std::vector<int64_t> b;
  for (int64_t r = 0; r < nrows; r += PR) b.push_back(r);
  b.push_back(nrows);
  if (nrows == 0) b = {0, 0};
  return b;
}
}  // namespace

extern "C" int dk_ckpt_writer_open(dk_engine* e, const char* path, int32_t codec, dk_ckpt_writer** out) {
  if (!e) return fail("null engine");
  hipSetDevice(e->cfg.device);
  std::unique_ptr<dk_ckpt_writer> w(new dk_ckpt_writer());
  w->eng = e; w->path = path; w->codec = codec ? 1 : 0;
  if (w->own.create()) return 1;
  w->s = w->own.s;
  w->S.build();
  w->fp = fopen(path, "wb");
  if (!w->fp) return fail(std::string("cannot create ") + path);
  if (fwrite("PAR1", 1, 4, w->fp) != 4) return fail("checkpoint write failed");
  *out = w.release();
  return 0;
}

// row group 0: action rows as JSON lines ({"add": {...}} / {"remove": ...} / {"metaData": ...} /
// {"protocol": ...} / {"txn": ...} / {"domainMetadata": ...}, one action per line), in order
extern "C" int dk_ckpt_writer_add_json(dk_ckpt_writer* w, const char* text, int64_t len) {
  hipSetDevice(w->eng->cfg.device);
  std::vector<JNode> N;
  int64_t i = 0, nrows = 0;
  try {
    while (i < len) {
      int64_t j = i;
      while (j < len && text[j] != '\n') j++;
      if (j > i) {
        N.clear();
        JParser jp(text + i, text + j, N);
        int root = jp.value(0);
        if (root >= 0) { jp.ws(); if (jp.p != jp.e) root = -1; }
        if (root < 0 || N[root].t != J_OBJ) return fail("dk_ckpt_writer_add_json: bad action line");
        Shredder sh{w->S, N};
        for (int k : w->S.nodes[0].kids) sh.value(k, member(N, N[root], w->S.nodes[k].name.c_str()), 0, 0);
        nrows++;
      }
      i = j + 1;
    }
  } catch (const JErr& je) {
    return fail("checkpoint row: " + je.msg);
  }
  w->host_rows += nrows;
  return 0;
}

// flush row group 0 (the host rows)
static int flush_host_rows(dk_ckpt_writer* w) {
  hipStream_t s = w->s;
  const int64_t nrows = w->host_rows;
  std::vector<WChunk> chunks(w->S.leaves.size());
  const std::vector<int64_t> prow = page_rows(nrows);
  for (size_t li = 0; li < w->S.leaves.size(); li++) {
    WLeaf& L = w->S.leaves[li];
    const int64_t nlev = (int64_t)L.def.size(), nv = L.phys == PT_BYTE_ARRAY ? (int64_t)L.lens.size() : (int64_t)(L.width ? L.fixed.size() / L.width : 0);
    // page boundaries at row starts: level / value / char indices
    std::vector<int64_t> lb, vb, cb;
    int64_t row = -1, v = 0, c = 0;
    size_t pi = 0;
    for (int64_t l = 0; l < nlev; l++) {
      const bool start = !L.max_rep || L.rep[l] == 0;
      if (start) {
        row++;
        if (pi < prow.size() - 1 && row == prow[pi]) { lb.push_back(l); vb.push_back(v); cb.push_back(c); pi++; }
      }
      if (L.def[l] == L.max_def) { if (L.phys == PT_BYTE_ARRAY) c += L.lens[v]; v++; }
    }
    while (lb.size() < prow.size()) { lb.push_back(nlev); vb.push_back(v); cb.push_back(c); }
    if (nv != v) return fail("checkpoint writer: value count mismatch in " + L.path);
    if (upload(w->d_def, L.def.data(), L.def.size(), s) || upload(w->d_rep, L.rep.data(), L.rep.size(), s)) return 1;
    if (L.phys == PT_BYTE_ARRAY) {
      std::vector<long long> coff(L.lens.size() + 1, 0);
      for (size_t k = 0; k < L.lens.size(); k++) coff[k + 1] = coff[k] + L.lens[k];
      if (upload(w->d_lens, L.lens.data(), L.lens.size() * 4, s) || upload(w->d_chars, L.chars.data(), L.chars.size(), s) ||
          upload(w->d_coff, coff.data(), coff.size() * 8, s)) return 1;
    } else if (upload(w->d_vals, L.fixed.data(), L.fixed.size(), s)) return 1;
    HIPOK(hipStreamSynchronize(s));
    if (write_chunk(w, L, nlev, lb, vb, cb, chunks[li])) return 1;
    L.def.clear(); L.rep.clear(); L.fixed.clear(); L.chars.clear(); L.lens.clear();
  }
  w->rgs.push_back(chunks);
  w->rg_rows.push_back(nrows);
  w->total_rows += nrows;
  w->host_rows = 0;
  return 0;
}

// The old checkpoint's column for a new-schema leaf path (add.* only), with the repetition of every
// node along the path in the old file's schema
static const DColumn* old_leaf(dk_parquet* p, int fi, const WLeaf& L, std::vector<int>* reps) {
  const DColumn* c = find_col(p, fi, L.path.c_str());
  if (!c) return nullptr;
  const FileM& f = p->files[fi];
  // walk the old schema along the components as leaf_index resolves them (a MAP group's repeated
  // child and its key / value by position, struct fields by name)
  int g = 0, map_level = 0;
  for (size_t ci = 0; ci < L.comps.size(); ci++) {
    const SchemaEl& G = f.schema[g];
    if (G.kids.empty()) return nullptr;
    int hit = -1;
    if (map_level == 0 && (G.conv == 1 || G.logical == 2)) map_level = 1;
    if (map_level == 1) {
      if (G.kids.size() == 1 && f.schema[G.kids[0]].repetition == 2) hit = G.kids[0];
      map_level = hit >= 0 ? 2 : 0;
    } else if (map_level == 2) {
      if (G.kids.size() == 2 && (L.comps[ci] == "key" || L.comps[ci] == "value")) hit = G.kids[L.comps[ci] == "key" ? 0 : 1];
      map_level = 0;
    }
    if (hit < 0) for (int k : G.kids) if (f.schema[k].name == L.comps[ci]) { hit = k; break; }
    if (hit < 0) return nullptr;
    reps->push_back(f.schema[hit].repetition);
    g = hit;
  }
  return c;
}

// row group: the surviving add rows among rows [row0, row1) of checkpoint file `file` of the replay
// (selection on the device); host rows added before it are flushed as their own row group first
extern "C" int dk_ckpt_writer_add_checkpoint_adds(dk_ckpt_writer* w, dk_replay* r, int32_t file, int64_t row0,
                                                  int64_t row1, int64_t* n_rows) {
  hipSetDevice(w->eng->cfg.device);
  if (w->host_rows > 0 && flush_host_rows(w)) return 1;
  if (!r || !r->ck || file < 0 || file >= (int32_t)r->ck->files.size()) return fail("dk_ckpt_writer_add_checkpoint_adds: bad file");
  if (!r->have_result && !(file < (int32_t)r->file_ready.size() && r->file_ready[file]))
    return fail("dk_ckpt_writer_add_checkpoint_adds: the replay has no result");
  if (row0 < 0 || row1 < row0 || row1 > r->ck->files[file].num_rows) return fail("dk_ckpt_writer_add_checkpoint_adds: bad rows");
  hipStream_t s = w->s;
  HIPOK(hipStreamSynchronize(r->stream));
  dk_parquet* p = r->ck;
  const int64_t n = row1 - row0;
  const uint8_t* sel = r->d_csel[file]->as<uint8_t>() + row0;
  const long long nsb = enc_scan_blocks(n + 1);
  if (w->d_tmp.alloc((size_t)(n + 1) * 8 + 64) || w->d_rowpos.alloc((size_t)(n + 1) * 8 + 64) ||
      w->d_sums.alloc((size_t)nsb * 8 + 64) || w->d_total.alloc(64) || w->d_rows.alloc((size_t)(n + 1) * 4 + 64) ||
      w->d_err.alloc(64)) return 1;
  enc_sel_rows(sel, n, w->d_tmp.as<long long>(), w->d_rowpos.as<long long>(), w->d_sums.as<long long>(),
               w->d_total.as<long long>(), w->d_rows.as<int32_t>(), s);
  long long ns = 0;
  HIPOK(hipMemcpyAsync(&ns, w->d_total.p, 8, hipMemcpyDeviceToHost, s));
  HIPOK(hipStreamSynchronize(s));
  std::vector<WChunk> chunks(w->S.leaves.size());
  const std::vector<int64_t> prow = page_rows(ns);
  if (w->d_lv.alloc((size_t)(ns + 1) * 8 + 64) || w->d_vv.alloc((size_t)(ns + 1) * 8 + 64) ||
      w->d_cc.alloc((size_t)(ns + 1) * 8 + 64) || w->d_lb.alloc((size_t)(ns + 2) * 8 + 64) ||
      w->d_vb.alloc((size_t)(ns + 2) * 8 + 64) || w->d_cb.alloc((size_t)(ns + 2) * 8 + 64)) return 1;
  for (size_t li = 0; li < w->S.leaves.size(); li++) {
    WLeaf& L = w->S.leaves[li];
    std::vector<int> reps;
    const DColumn* c = L.comps[0] == "add" ? old_leaf(p, file, L, &reps) : nullptr;
    int64_t nlev = ns, nv = 0, nc = 0;
    std::vector<int64_t> lb, vb(prow.size(), 0), cb(prow.size(), 0);
    if (!c || !c->present) {
      // every row of this group is an add: a leaf of another action, or an add leaf with no value
      // in the old file, is null at the deepest level its ancestors reach
      int d = 0;
      if (L.comps[0] == "add") {
        d = w->S.nodes[L.chain[0]].def;      // add defined
        for (size_t k = 1; k < L.chain.size(); k++) {
          const WNode& nd = w->S.nodes[L.chain[k]];
          if (nd.rep != W_REQ) break;
          return fail("checkpoint writer: required field " + L.path + " is missing in " + p->files[file].path);
        }
      }
      std::vector<uint8_t> lv(ns, (uint8_t)d);
      if (upload(w->d_def, lv.data(), lv.size(), s)) return 1;
      if (L.max_rep) { std::vector<uint8_t> rp(ns, 0); if (upload(w->d_rep, rp.data(), rp.size(), s)) return 1; }
      HIPOK(hipStreamSynchronize(s));
      for (int64_t rr : prow) lb.push_back(rr);
    } else {
      // definition levels: old -> new through the nodes each old level defines
      if (reps.size() != L.chain.size()) return fail("checkpoint writer: schema mismatch for " + L.path);
      EncSrc E{};
      // row-indexed arrays start at row0 (entry-indexed ones are reached through row_offs)
      const bool rep_old = c->max_rep > 0;
      E.row_def = c->row_def + row0; E.row_offs = c->row_offs ? c->row_offs + row0 : nullptr; E.entry_def = c->entry_def;
      E.fixed = c->fixed ? (rep_old ? c->fixed : c->fixed + row0 * c->width) : nullptr;
      E.offs = c->offs ? (rep_old ? c->offs : c->offs + row0) : nullptr;
      E.chars = c->chars;
      E.width = c->width; E.is_str = L.phys == PT_BYTE_ARRAY; E.repeated = L.max_rep > 0 && c->max_rep > 0 && c->row_offs;
      E.max_def_new = L.max_def; E.entry_def_old = c->rep_def;
      if ((L.max_rep > 0) != (c->max_rep > 0) || c->phys != L.phys || (L.phys != PT_BYTE_ARRAY && !c->null_only && c->width != L.width))
        return fail("checkpoint writer: type mismatch for " + L.path);
      for (int dold = 0; dold < 16; dold++) {
        int cnt = 0, J = -1;
        for (size_t k = 0; k < reps.size(); k++) {
          cnt += reps[k] != W_REQ;
          if (cnt > dold) break;
          J = (int)k;
        }
        int dnew = 0;
        for (int k = 0; k <= J; k++) dnew += w->S.nodes[L.chain[k]].rep != W_REQ;
        const bool bad = J + 1 < (int)L.chain.size() && w->S.nodes[L.chain[J + 1]].rep == W_REQ;
        E.defmap[dold] = bad ? 0xff : (uint8_t)dnew;
        E.emap[dold] = E.defmap[dold];
      }
      HIPOK(hipMemsetAsync(w->d_err.p, 0, 4, s));
      enc_count(E, w->d_rows.as<int32_t>(), ns, w->d_lv.as<long long>(), w->d_vv.as<long long>(),
                E.is_str ? w->d_cc.as<long long>() : nullptr, w->d_err.as<int>(), s);
      auto scan = [&](DBuf& in, DBuf& outb, long long* tot) -> int {
        if (ns > 0) {
          enc_exscan(in.as<long long>(), ns, outb.as<long long>(), w->d_sums.as<long long>(), w->d_total.as<long long>(), s);
          HIPOK(hipMemcpyAsync(tot, w->d_total.p, 8, hipMemcpyDeviceToHost, s));
        } else *tot = 0;
        return 0;
      };
      long long tl = 0, tv = 0, tc = 0;
      if (scan(w->d_lv, w->d_lb, &tl) || scan(w->d_vv, w->d_vb, &tv) || (E.is_str && scan(w->d_cc, w->d_cb, &tc))) return 1;
      int err = 0;
      HIPOK(hipMemcpyAsync(&err, w->d_err.p, 4, hipMemcpyDeviceToHost, s));
      HIPOK(hipStreamSynchronize(s));
      if (err) return fail("checkpoint writer: a required field of " + L.path + " is null in " + p->files[file].path);
      nlev = tl; nv = tv; nc = tc;
      if (w->d_def.alloc((size_t)nlev + 64) || w->d_rep.alloc((size_t)nlev + 64)) return 1;
      if (E.is_str) {
        if (w->d_lens.alloc((size_t)nv * 4 + 64) || w->d_chars.alloc((size_t)nc + 64) || w->d_coff.alloc((size_t)(nv + 1) * 8 + 64)) return 1;
      } else if (w->d_vals.alloc((size_t)nv * std::max(1, L.width) + 64)) return 1;
      enc_fill(E, w->d_rows.as<int32_t>(), ns, w->d_lb.as<long long>(), w->d_vb.as<long long>(),
               E.is_str ? w->d_cb.as<long long>() : nullptr, w->d_def.as<uint8_t>(), L.max_rep ? w->d_rep.as<uint8_t>() : nullptr,
               w->d_vals.as<uint8_t>(), w->d_lens.as<int32_t>(), w->d_chars.as<uint8_t>(),
               E.is_str ? w->d_coff.as<long long>() : nullptr, s);
      if (E.is_str) HIPOK(hipMemcpyAsync(w->d_coff.as<long long>() + nv, &tc, 8, hipMemcpyHostToDevice, s));
      // page boundaries (rows prow) -> level / value / char indices
      std::vector<long long> hb(3 * prow.size());
      for (size_t k = 0; k < prow.size(); k++) {
        const int64_t rr = prow[k];
        if (rr >= ns) { hb[3 * k] = tl; hb[3 * k + 1] = tv; hb[3 * k + 2] = tc; continue; }
        HIPOK(hipMemcpyAsync(&hb[3 * k], w->d_lb.as<long long>() + rr, 8, hipMemcpyDeviceToHost, s));
        HIPOK(hipMemcpyAsync(&hb[3 * k + 1], w->d_vb.as<long long>() + rr, 8, hipMemcpyDeviceToHost, s));
        if (E.is_str) HIPOK(hipMemcpyAsync(&hb[3 * k + 2], w->d_cb.as<long long>() + rr, 8, hipMemcpyDeviceToHost, s));
      }
      HIPOK(hipStreamSynchronize(s));
      for (size_t k = 0; k < prow.size(); k++) { lb.push_back(hb[3 * k]); vb[k] = hb[3 * k + 1]; cb[k] = E.is_str ? hb[3 * k + 2] : 0; }
    }
    if (write_chunk(w, L, nlev, lb, vb, cb, chunks[li])) return 1;
  }
  w->rgs.push_back(chunks);
  w->rg_rows.push_back(ns);
  w->total_rows += ns;
  if (n_rows) *n_rows = ns;
  return 0;
}

extern "C" int dk_ckpt_writer_close(dk_ckpt_writer* w, int64_t* n_rows, int64_t* file_size) {
  if (!w) return fail("null writer");
  hipSetDevice(w->eng->cfg.device);
  int rc = 0;
  if (w->host_rows > 0) rc = flush_host_rows(w);
  if (!rc) {
    TWriter t;
    t.i32(1, 1);
    t.list(2, 12, w->S.nodes.size());
    for (const WNode& n : w->S.nodes) {
      t.lbegin();
      if (n.phys >= 0) t.i32(1, n.phys);
      if (&n != &w->S.nodes[0]) t.i32(3, n.rep);
      t.str(4, n.name);
      if (n.phys < 0) t.i32(5, (int64_t)n.kids.size());
      if (n.conv >= 0) t.i32(6, n.conv);
      t.lend();
    }
    t.i64(3, w->total_rows);
    t.list(4, 12, w->rgs.size());
    for (size_t g = 0; g < w->rgs.size(); g++) {
      t.lbegin();
      t.list(1, 12, w->S.leaves.size());
      int64_t tot = 0;
      for (size_t li = 0; li < w->S.leaves.size(); li++) {
        const WLeaf& L = w->S.leaves[li];
        const WChunk& c = w->rgs[g][li];
        tot += c.unc;
        t.lbegin();
        t.i64(2, c.offset);
        t.begin(3);
        t.i32(1, L.phys);
        t.list(2, 5, 2); t.zz(0); t.zz(3);              // PLAIN, RLE
        t.list(3, 8, L.comps.size());
        for (const std::string& x : L.comps) { t.varint(x.size()); t.b.insert(t.b.end(), x.begin(), x.end()); }
        t.i32(4, w->codec);
        t.i64(5, c.nlev);
        t.i64(6, c.unc);
        t.i64(7, c.comp);
        t.i64(9, c.offset);
        t.end();
        t.lend();
      }
      t.i64(2, tot);
      t.i64(3, w->rg_rows[g]);
      t.lend();
    }
    t.str(6, "delta_amd dk_ckpt_writer (gfx950 encoder)");
    t.b.push_back(0);
    const uint32_t fl = (uint32_t)t.b.size();
    if (fwrite(t.b.data(), 1, t.b.size(), w->fp) != t.b.size() || fwrite(&fl, 1, 4, w->fp) != 4 ||
        fwrite("PAR1", 1, 4, w->fp) != 4)
      rc = fail("checkpoint write failed: " + w->path);
    w->off += (int64_t)t.b.size() + 8;
  }
  if (fclose(w->fp) != 0 && !rc) rc = fail("checkpoint write failed: " + w->path);
  if (n_rows) *n_rows = w->total_rows;
  if (file_size) *file_size = w->off;
  HIPOK(hipStreamSynchronize(w->s));
  delete w;
  return rc;
}
