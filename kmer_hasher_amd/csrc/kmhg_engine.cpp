// kmhg_engine.cpp -- host orchestrator of the MI355X k-mer position index + the C-ABI.
//
// Runtime pieces (native, as the reference's C core is native):
//   * DevicePool   caching device allocator (size-classed free lists per device)
//   * Timing       per-kernel HIP-event pairs on the launch stream (kmhg_timing_*)
//   * Index/Query  build -> query -> readout pipelines over kmhg_kernels.hip
// Reference entry points each C function replaces are listed in include/kmhgpu.h.
#include <atomic>
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kmhg_common.h"
#include "kmhg_kernels.h"
#include "kmhg_fastx.h"
#include "kmhg_khash.h"
#include "kmhg_sh.h"

// Environment knobs.  The product library reads four: KMHG_TIMING (per-kernel events),
// KMHG_DEVICES (multi-device query), KMHG_ROW_ORDER and KMHG_D2H_THREADS.  Everything else exists
// only in the test build (-DKMHG_TEST_BUILD: libkmhgpu_test.so, which the GPU suite loads for the
// tests that force a path, tests/conftest.py `test_lib`): the path selectors that force each
// build / query / counts path against the oracle (KMHG_BUILD, KMHG_BUILD_BID, KMHG_MAXR,
// KMHG_FUSE_BOUNDS, KMHG_TEST_BALLOT, KMHG_QUERY_TAGS, KMHG_QUERY_DIAG, KMHG_DIAG_CODES,
// KMHG_COUNT_TABLE, KMHG_COUNT_WALK, KMHG_CO_SPREAD, KMHG_CO_GLOBAL, KMHG_PART_COMPACT,
// KMHG_ROW_ORDER_SORT, KMHG_PACK8, KMHG_NB_ROUND, KMHG_SLICE_POISON, KMHG_TEST_REPLICA,
// KMHG_DIGIT_STREAM, KMHG_DS_BID, KMHG_DS_U8, KMHG_DS_PACK, KMHG_BUILD_TAGS), which choose
// between equivalent paths and change no result; fault injection (KMHG_TEST_DISORDER); and the
// A/B-only switches (KMHG_D2H, KMHG_D2H_HUGE, KMHG_HOST_RUNS, KMHG_HOST_PAIRS, KMHG_HOST_POOL,
// KMHG_COUNT_BID, KMHG_RK_CAP, KMHG_POOL_DEPTH, KMHG_POOL_BESTFIT, KMHG_POOL_TRACE).
namespace kmhg {
inline const char* test_build_knob(const char* name) {
#ifdef KMHG_TEST_BUILD
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
}  // namespace kmhg
#include "../../include/kmhgpu.h"

using namespace kmhg;

// ============================================================================ errors
static thread_local std::string g_err;

namespace {

struct Error {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    if (e == hipErrorOutOfMemory) fail(KMHG_ENOMEM, std::string(what) + ": out of device memory");
    fail(KMHG_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
  }
}
#define HIPC(x) hip_check((x), #x)

template <class F>
int guarded(F&& f) {
  try {
    f();
    return KMHG_OK;
  } catch (const Error& e) {
    g_err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return KMHG_ENOMEM;
  }
}

// ============================================================================ device pool
// Caching allocator: blocks are kept per (device, rounded size) and reused, so repeated builds
// and queries (bench steps, many queries against one index) pay hipMalloc once.
// Stream-ordered releases inside one host call (one build, query, ...) share ONE event: every
// ordered release on the group's stream is deferred to the group's end, where a single event is
// recorded for all of them.  (Each event record is a marker packet the command processor
// drains the stream for; a build used to record ~14 of them back to back.)
struct ReleaseGroup;
thread_local ReleaseGroup* tl_release_group = nullptr;

class DevicePool {
 public:
  static DevicePool& get() {
    static DevicePool p;
    return p;
  }
  void* alloc(size_t bytes) {
    if (bytes == 0) bytes = 256;
    size_t sz = round(bytes);
    int dev = 0;
    HIPC(hipGetDevice(&dev));
    {
      std::unique_lock<std::mutex> g(mu_);
      poll_pending();
      auto& fl = free_[{dev, sz}];
      if (!fl.empty()) {
        void* p = fl.back();
        fl.pop_back();
        cached_ -= sz;
        live_[p] = {dev, sz};
        return p;
      }
      // a block of this size still in use by queued work: wait for it rather than grow the
      // pool -- the back-pressure that bounds how far asynchronous builds run ahead.  Up to
      // DEPTH blocks of a size class exist before a request waits.  (Depth 2, so that the host
      // enqueues build i + 1 while build i runs, measured no faster at 10 / 100 / 500 Mbp:
      // the gaps between a build's kernels are the device's, not the host's enqueue.)
      static const size_t depth = [] {            // KMHG_POOL_DEPTH (test build): 1..8
        const char* e = test_build_knob("KMHG_POOL_DEPTH");
        return e ? (size_t)std::max(1, std::min(8, std::atoi(e))) : POOL_DEPTH;
      }();
      for (size_t i = 0; i < pending_.size() && count_[{dev, sz}] >= depth; ++i) {
        if (pending_[i].key != std::make_pair(dev, sz)) continue;
        Pending pd = pending_[i];
        pending_.erase(pending_.begin() + (long)i);
        g.unlock();
        (void)hipEventSynchronize(pd.ev);
        g.lock();
        if (pd.owns_ev) events_.push_back(pd.ev);
        live_[pd.p] = pd.key;
        return pd.p;
      }
      // a large request with no block of its own size: the smallest idle cached block of at
      // most 1.5x its size serves it (it keeps its own size class and returns to it).  A
      // hipMalloc of GBs costs ~0.1 ms per GB: the first 500 Mbp query of a process reuses the
      // build's freed 6 GB stream buffers for its records and rows (2 of its 3 GB-sized
      // buffers) instead of allocating 10 GB.
      static const bool best_fit = [] {           // KMHG_POOL_BESTFIT=0 (test build): off
        const char* e = test_build_knob("KMHG_POOL_BESTFIT");
        return !(e && e[0] == '0');
      }();
      if (best_fit && sz >= BEST_FIT_MIN) {
        auto it = free_.lower_bound({dev, sz});
        for (; it != free_.end() && it->first.first == dev && it->first.second <= sz + sz / 2;
             ++it) {
          if (it->second.empty()) continue;
          void* p = it->second.back();
          it->second.pop_back();
          cached_ -= it->first.second;
          live_[p] = it->first;
          return p;
        }
      }
    }
    void* p = nullptr;
    static const bool trace = test_build_knob("KMHG_POOL_TRACE") != nullptr;   // test build
    if (trace) std::fprintf(stderr, "kmhg pool: hipMalloc %zu B on device %d\n", sz, dev);
    hipError_t e = hipMalloc(&p, sz);
    if (e == hipErrorOutOfMemory) {   // release the cache and retry once
      (void)hipGetLastError();
      trim();
      e = hipMalloc(&p, sz);
    }
    hip_check(e, "hipMalloc");
    std::lock_guard<std::mutex> g(mu_);
    live_[p] = {dev, sz};
    ++count_[{dev, sz}];
    return p;
  }
  // Stream-ordered release: the block returns to the free list once the work queued on
  // `stream` up to now has completed (an event is recorded and polled on later allocations).
  void release(void* p, hipStream_t stream = nullptr, bool ordered = false);
  // the group's blocks: one event recorded on `stream` for all of them
  void release_batch(const std::vector<void*>& ps, hipStream_t stream) {
    if (ps.empty()) return;
    hipEvent_t ev = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!events_.empty()) { ev = events_.back(); events_.pop_back(); }
    }
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
    if (!ev || hipEventRecord(ev, stream) != hipSuccess) {
      (void)hipStreamSynchronize(stream);
      if (ev) { std::lock_guard<std::mutex> g(mu_); events_.push_back(ev); }
      ev = nullptr;
    }
    std::lock_guard<std::mutex> g(mu_);
    size_t owner = SIZE_MAX;            // the last entry actually queued recycles the event
    for (size_t i = 0; i < ps.size(); ++i) {
      auto it = live_.find(ps[i]);
      if (it == live_.end()) continue;
      if (ev) {
        owner = pending_.size();
        pending_.push_back({ps[i], it->second, ev, false});
      } else {
        free_[it->second].push_back(ps[i]);
        cached_ += it->second.second;
      }
      live_.erase(it);
    }
    if (ev) {
      if (owner != SIZE_MAX) pending_[owner].owns_ev = true;
      else events_.push_back(ev);       // nothing queued: the event goes straight back
    }
  }
  // blocks no queued work uses any more (their stream was synchronized)
  void release_now(const std::vector<void*>& ps) {
    std::lock_guard<std::mutex> g(mu_);
    for (void* p : ps) {
      auto it = live_.find(p);
      if (it == live_.end()) continue;
      free_[it->second].push_back(p);
      cached_ += it->second.second;
      live_.erase(it);
    }
  }
  void release_one(void* p, hipStream_t stream, bool ordered) {
    if (!p) return;
    hipEvent_t ev = nullptr;
    if (ordered) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!events_.empty()) { ev = events_.back(); events_.pop_back(); }
      }
      if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
      if (!ev || hipEventRecord(ev, stream) != hipSuccess) {
        (void)hipStreamSynchronize(stream);
        if (ev) { std::lock_guard<std::mutex> g(mu_); events_.push_back(ev); }
        ev = nullptr;
      }
    }
    std::lock_guard<std::mutex> g(mu_);
    auto it = live_.find(p);
    if (it == live_.end()) return;
    if (ev) {
      pending_.push_back({p, it->second, ev, true});
    } else {
      free_[it->second].push_back(p);
      cached_ += it->second.second;
    }
    live_.erase(it);
  }
  void trim() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& pd : pending_) {
      (void)hipEventSynchronize(pd.ev);
      if (pd.owns_ev) events_.push_back(pd.ev);
      free_[pd.key].push_back(pd.p);
    }
    pending_.clear();
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto& kv : free_) {
      (void)hipSetDevice(kv.first.first);
      for (void* p : kv.second) (void)hipFree(p);
      count_[kv.first] -= std::min(count_[kv.first], kv.second.size());
      kv.second.clear();
    }
    (void)hipSetDevice(cur);
    cached_ = 0;
  }
  int64_t cached() {
    std::lock_guard<std::mutex> g(mu_);
    return (int64_t)cached_;
  }

 private:
  // owns_ev: the one entry of a batch that recycles the shared event.  An entry polled after
  // its batch's event was recycled and recorded again only waits for later work (safe).
  struct Pending { void* p; std::pair<int, size_t> key; hipEvent_t ev; bool owns_ev; };
  void poll_pending() {
    for (size_t i = 0; i < pending_.size();) {
      if (hipEventQuery(pending_[i].ev) == hipSuccess) {
        if (pending_[i].owns_ev)
          events_.push_back(pending_[i].ev);        // recycled: no create/destroy per release
        free_[pending_[i].key].push_back(pending_[i].p);
        cached_ += pending_[i].key.second;
        pending_[i] = pending_.back();
        pending_.pop_back();
      } else {
        ++i;
      }
    }
  }
  static constexpr size_t BEST_FIT_MIN = (size_t)256 << 20;
  static constexpr size_t POOL_DEPTH = 1;   // depth 2 measured: no gain
  static size_t round(size_t b) {
    if (b <= (1u << 20)) {           // small: power of two >= 256 B
      size_t r = 256;
      while (r < b) r <<= 1;
      return r;
    }
    const size_t g = 2u << 20;       // large: 2 MiB granules
    return (b + g - 1) / g * g;
  }
  std::mutex mu_;
  std::map<std::pair<int, size_t>, std::vector<void*>> free_;
  std::map<std::pair<int, size_t>, size_t> count_;   // blocks of each size class (any state)
  std::map<void*, std::pair<int, size_t>> live_;
  std::vector<Pending> pending_;
  std::vector<hipEvent_t> events_;
  size_t cached_ = 0;
};

struct ReleaseGroup {
  hipStream_t s;
  std::vector<void*> ps;
  ReleaseGroup* prev;
  // set after a synchronize of `s` with no launch behind it: the blocks go straight back to the
  // pool, no event (a synchronous call's last step)
  bool synced = false;
  explicit ReleaseGroup(hipStream_t stream) : s(stream), prev(tl_release_group) {
    tl_release_group = this;
  }
  ~ReleaseGroup() {
    tl_release_group = prev;
    if (synced) DevicePool::get().release_now(ps);
    else DevicePool::get().release_batch(ps, s);
  }
  ReleaseGroup(const ReleaseGroup&) = delete;
  ReleaseGroup& operator=(const ReleaseGroup&) = delete;
};

void DevicePool::release(void* p, hipStream_t stream, bool ordered) {
  if (!p) return;
  if (ordered && tl_release_group && tl_release_group->s == stream) {
    tl_release_group->ps.push_back(p);          // deferred to the group's one event
    return;
  }
  release_one(p, stream, ordered);
}

// RAII device buffer from the pool.  A buffer bound to a stream is released stream-ordered
// (kernels still queued on that stream may use it after the C++ object dies).
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipStream_t s = nullptr;
  bool ordered = false;
  DBuf() = default;
  explicit DBuf(size_t count) { reset(count); }
  DBuf(size_t count, hipStream_t stream) { reset(count); bind(stream); }
  ~DBuf() { free(); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  void bind(hipStream_t stream) { s = stream; ordered = true; }
  void reset(size_t count) {
    free();
    n = count;
    p = static_cast<T*>(DevicePool::get().alloc(std::max<size_t>(count, 1) * sizeof(T)));
  }
  void free() {
    if (p) DevicePool::get().release(p, s, ordered);
    p = nullptr; n = 0;
  }
  size_t bytes() const { return n * sizeof(T); }
  void swap_with(DBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(s, o.s);
    std::swap(ordered, o.ordered);
  }
};

// Pinned, device-visible host records for the build totals: V_stats writes one directly, so the
// host reads U / N / P with no copy launch.  Each record carries an event recorded after the
// build's last kernel; a record given back while its build is still in flight (an index freed
// before it was ever used) is reused only once that event has completed.
struct PinnedRec {
  BuildMeta* meta = nullptr;
  hipEvent_t ev = nullptr;
};
class PinnedPool {
 public:
  static PinnedPool& get() {
    static PinnedPool p;
    return p;
  }
  PinnedRec take() {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < pending_.size();) {
      if (hipEventQuery(pending_[i].ev) == hipSuccess) {
        free_.push_back(pending_[i]);
        pending_[i] = pending_.back();
        pending_.pop_back();
      } else {
        ++i;
      }
    }
    if (free_.empty()) {
      constexpr int kSlots = 64;
      BuildMeta* blk = nullptr;
      HIPC(hipHostMalloc(reinterpret_cast<void**>(&blk), sizeof(BuildMeta) * kSlots,
                         hipHostMallocCoherent));
      for (int i = 0; i < kSlots; ++i) {
        PinnedRec r;
        r.meta = blk + i;
        HIPC(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
        free_.push_back(r);
      }
    }
    PinnedRec r = free_.back();
    free_.pop_back();
    std::memset(r.meta, 0, sizeof(*r.meta));
    return r;
  }
  void give(PinnedRec r, bool in_flight) {
    if (!r.meta) return;
    std::lock_guard<std::mutex> g(mu_);
    (in_flight ? pending_ : free_).push_back(r);
  }

 private:
  std::mutex mu_;
  std::vector<PinnedRec> free_, pending_;
};
// returns a record taken for a host round trip that the scope waited for (any exit path)
// On an exception path the device may still write into the record (a queued scan's total), so
// the stream is drained first: a record back in the free list is never a DMA target.
struct GiveBack {
  PinnedRec& r;
  hipStream_t s;
  ~GiveBack() {
    if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(s);
    PinnedPool::get().give(r, false);
  }
};

// ============================================================================ timing
struct Timing {
  static Timing& get() {
    static Timing t;
    return t;
  }
  bool on = false;
  std::string only;                   // record just this kernel (empty = every kernel)
  struct Rec { std::string name; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::map<std::string, std::pair<int64_t, double>> acc;
  std::mutex mu;

  Timing() {
    const char* e = std::getenv("KMHG_TIMING");
    on = e && e[0] == '1';
  }
  std::vector<hipEvent_t> pool;       // recycled events: no create/destroy per launch
  hipEvent_t take() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e;
    // timing-only events: no system-scope fence (a default event writes back / invalidates the
    // caches at every record, ~10 us of dead time between the kernels it brackets)
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
      (void)hipGetLastError();
      HIPC(hipEventCreate(&e));
    }
    return e;
  }
  template <class F>
  void run(const char* name, hipStream_t s, F&& launch) {
    if (!on || (!only.empty() && only != name)) { launch(); HIPC(hipGetLastError()); return; }
    hipEvent_t a, b;
    {
      std::lock_guard<std::mutex> g(mu);
      a = take();
      b = take();
    }
    HIPC(hipEventRecord(a, s));
    launch();
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(b, s));
    std::lock_guard<std::mutex> g(mu);
    recs.push_back({name, a, b});
  }
  void collect() {   // resolve recorded events (synchronises on them)
    std::lock_guard<std::mutex> g(mu);
    for (auto& r : recs) {
      (void)hipEventSynchronize(r.b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, r.a, r.b);
      auto& x = acc[r.name];
      x.first += 1;
      x.second += ms;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
  }
};
#define LAUNCH(name, stream, ...) Timing::get().run(name, stream, [&] { __VA_ARGS__; })

// One library stream per device for host-pointer entry points.
hipStream_t lib_stream() {
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  hipStream_t s;
  HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  streams[dev] = s;
  return s;
}

// Host worker pool for the host-side copies: HOST_WORKERS threads made on first use and kept,
// so a call that splits a few MB over threads does not pay their creation and join (8 threads:
// ~0.1-0.35 ms a round -- per 16-MB chunk of a staged copy before).  run(n, fn) runs fn(0) ..
// fn(n - 1), the calling thread taking tasks too, and returns when all are done; calls from
// several threads at once (a multi-device query's parts) share the workers.  No task may call
// run() itself.  big = true (GB-scale writes: the expansions) starts fresh threads instead: the
// kernel spreads new threads over the machine's memory controllers, while woken pool workers
// crowd near their waker (A/B in one run, profiles/r6al_pool_ab/: config 5's run expansion
// 18-21 ms fresh, 30-54 pooled; config 4's pair rows 108-112 fresh, 99-164 pooled).
constexpr uint64_t HOST_BIG_BYTES = 512u << 20;   // (config 2's 80 MB of rows: pooled 0.84-0.91
                                                  // ms, fresh 1.19-1.41; profiles/r6ak*, r6al*)
class HostPool {
 public:
  static constexpr int HOST_WORKERS = 15;        // + the calling thread = 16
  static HostPool& get() {
    static HostPool p;
    return p;
  }
  void run(int n, const std::function<void(int)>& fn, bool big = false) {
    if (n <= 1) {
      if (n == 1) fn(0);
      return;
    }
    const char* pe = test_build_knob("KMHG_HOST_POOL");   // "0": a thread per task (A/B)
    if (big || (pe && pe[0] == '0')) {
      std::vector<std::thread> th;
      for (int i = 1; i < n; ++i) th.emplace_back(fn, i);
      fn(0);
      for (auto& t : th) t.join();
      return;
    }
    Job job{&fn, n};
    {
      std::lock_guard<std::mutex> g(mu_);
      if (workers_.empty()) start();
      jobs_.push_back(&job);
    }
    cv_.notify_all();
    work_on(job, false);                         // until every task is handed out
    {
      std::lock_guard<std::mutex> g(mu_);        // no worker takes the job from here on
      for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
        if (*it == &job) {
          jobs_.erase(it);
          break;
        }
    }
    std::unique_lock<std::mutex> g(job.m);       // the job lives until its last worker is out
    job.cv.wait(g, [&] { return job.done == job.n && job.refs == 0; });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  struct Job {
    const std::function<void(int)>* fn;
    int n;
    std::atomic<int> next{0};
    int done = 0, refs = 0;                      // guarded by m (refs: workers inside)
    std::mutex m;
    std::condition_variable cv;
    Job(const std::function<void(int)>* f, int count) : fn(f), n(count) {}
  };
  void work_on(Job& job, bool worker) {
    int ran = 0;
    for (int i; (i = job.next.fetch_add(1)) < job.n; ++ran) (*job.fn)(i);
    std::lock_guard<std::mutex> g(job.m);
    job.done += ran;
    if (worker) --job.refs;
    if (job.done == job.n && job.refs == 0) job.cv.notify_all();
  }
  void start() {
    for (int w = 0; w < HOST_WORKERS; ++w)
      workers_.emplace_back([this] {
        for (;;) {
          Job* job = nullptr;
          {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] {
              while (!jobs_.empty() && jobs_.front()->next.load() >= jobs_.front()->n)
                jobs_.pop_front();                 // handed out completely
              return stop_ || !jobs_.empty();
            });
            if (stop_) return;
            job = jobs_.front();
            std::lock_guard<std::mutex> gj(job->m);
            ++job->refs;                           // (the caller waits for it)
          }
          work_on(*job, true);
        }
      });
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job*> jobs_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
};

// Device -> pageable host copy for the host-pointer entry points (R matrices, numpy arrays):
// results above D2H_STAGE_MIN go through two pinned chunks, the DMA of chunk i + 1 overlapping
// the host copy of chunk i, which d2h_threads() threads split (they also take the destination's
// first-touch page faults in parallel).  Synchronous: returns once dst holds the bytes.
constexpr size_t D2H_CHUNK = 16u << 20;
constexpr size_t D2H_STAGE_MIN = 4u << 20;
// KMHG_D2H_THREADS (A/B), default 8: A/B in one run (`profiles/rd4n_ab_d2h.log`, config 2
// host-boundary query, 10 M rows into a fresh array): 4 threads 7.9 / 8.4 ms, 8 threads 7.0 /
// 6.7 ms, 16 threads 7.7 / 10.1 ms
static int d2h_threads() {
  static const int n = [] {
    const char* e = std::getenv("KMHG_D2H_THREADS");
    return e ? std::max(1, std::min(16, std::atoi(e))) : 8;
  }();
  return n;
}

static void host_copy_par(char* dst, const char* src, size_t n) {
  const int T = d2h_threads();
  const size_t stripe = ((n + T - 1) / T + 4095) & ~(size_t)4095;
  HostPool::get().run(T, [=](int t) {
    const size_t a = std::min(n, t * stripe), b = std::min(n, a + stripe);
    if (a < b) std::memcpy(dst + a, src + a, b - a);
  });
}

struct PinStage {
  std::mutex mu;
  char* pin[2] = {nullptr, nullptr};
};
static PinStage& pin_stage() {           // the device's two pinned D2H_CHUNK buffers
  static std::mutex map_mu;
  static std::map<int, PinStage> stages;
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(map_mu);
  return stages[dev];
}

// A result matrix is usually fresh memory of the caller's allocator (R's allocMatrix: malloc,
// 4-KB pages), so the copy below takes one page fault per 4 KB.  Asking for transparent huge
// pages on the destination's whole 2-MB spans first (madvise(MADV_HUGEPAGE): a hint on the
// mapping, no change to its contents or ownership) makes that one fault per 2 MB.  Measured on
// the box (tools/host_thp_probe.py, profiles/r6r_thp.json, 10 M rows = 80 MB into a fresh
// array): 7.49 ms with 4-KB pages, 2.82 ms with huge pages (numpy asks for them itself).
// KMHG_D2H_HUGE=0 (test build) leaves the destination alone (A/B).
constexpr size_t HUGE_SPAN = 2u << 20;
static void hint_huge_pages(void* dst, size_t bytes) {
  static const bool on = [] {
    const char* e = test_build_knob("KMHG_D2H_HUGE");
    return !(e && e[0] == '0');
  }();
  if (!on || bytes < 2 * HUGE_SPAN) return;
  const uintptr_t m = ~(uintptr_t)(HUGE_SPAN - 1), d = reinterpret_cast<uintptr_t>(dst);
  const uintptr_t a = (d + HUGE_SPAN - 1) & m, b = (d + bytes) & m;
  if (b > a) (void)madvise(reinterpret_cast<void*>(a), b - a, MADV_HUGEPAGE);   // a hint only
}

void d2h_host(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return;
  static const bool staged = [] {
    const char* e = test_build_knob("KMHG_D2H");      // A/B knob: "direct" = one hipMemcpy
    return !(e && std::string(e) == "direct");
  }();
  hint_huge_pages(dst, bytes);
  if (!staged || bytes < D2H_STAGE_MIN) {
    HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return;
  }
  // two pinned chunks per device, so the parts of a multi-device query copy out concurrently
  PinStage& st = pin_stage();
  std::lock_guard<std::mutex> g(st.mu);
  char** pin = st.pin;
  if (!pin[0])
    for (int i = 0; i < 2; ++i)
      HIPC(hipHostMalloc(reinterpret_cast<void**>(&pin[i]), D2H_CHUNK, hipHostMallocPortable));
  // the two events, destroyed on every exit; on an exception the stream is drained first so no
  // DMA into the static pinned chunks is still in flight when the next caller takes them
  struct Ev2 {
    hipEvent_t e[2] = {nullptr, nullptr};
    hipStream_t s;
    ~Ev2() {
      if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(s);
      for (auto x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } evs{{nullptr, nullptr}, s};
  hipEvent_t* ev = evs.e;
  for (int i = 0; i < 2; ++i) HIPC(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  const size_t nch = (bytes + D2H_CHUNK - 1) / D2H_CHUNK;
  auto issue = [&](size_t i) {
    const size_t off = i * D2H_CHUNK, n = std::min(D2H_CHUNK, bytes - off);
    HIPC(hipMemcpyAsync(pin[i & 1], static_cast<const char*>(src) + off, n,
                        hipMemcpyDeviceToHost, s));
    HIPC(hipEventRecord(ev[i & 1], s));
  };
  issue(0);
  if (nch > 1) issue(1);
  for (size_t i = 0; i < nch; ++i) {
    HIPC(hipEventSynchronize(ev[i & 1]));
    const size_t off = i * D2H_CHUNK, n = std::min(D2H_CHUNK, bytes - off);
    host_copy_par(static_cast<char*>(dst) + off, pin[i & 1], n);
    if (i + 2 < nch) issue(i + 2);
  }
}

// Query rows into a host matrix (kmhg_query_fill, the R matrix of seq.kmer.pos).  A dot plot's
// rows are diagonal runs -- (i, j), (i + 1, j + 1), ... (config 5: 133 rows per run) -- so from
// RUNS_HOST_MIN rows on, the device writes the runs (R_count, scan, R_emit: the sharded
// query's gather format), 12 B per run cross PCIe into a pinned buffer, and host threads
// expand them into dst: the link carries ~1/90 of the bytes and the host's memory bandwidth
// writes the rows.  Rows that do not shrink RUNS_HOST_GAIN-fold (multi-hit windows) take
// d2h_host.  KMHG_HOST_RUNS=0 (test build): always d2h_host (A/B).
constexpr uint64_t RUNS_HOST_MIN = 1u << 19;           // rows (4 MB)
constexpr uint64_t RUNS_HOST_GAIN = 4;
struct PinRuns {
  std::mutex mu;
  int32_t* p = nullptr;
  size_t cap = 0;                                       // int32 words
};
static PinRuns& pin_runs() {                            // the device's pinned run buffer
  static std::mutex map_mu;
  static std::map<int, PinRuns> bufs;
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(map_mu);
  return bufs[dev];
}

// Host threads for the expansion: it is bound by the host's write bandwidth, which more threads
// reach (box, 16 CPUs, config 5's 376 M rows: 4 threads 51 ms, 8 30 ms, 16 16.5 ms;
// profiles/r6y_runs_probe*.json): every CPU this process may run on, at most 16.
// (The host's later unmapping of the matrix grows with the threads that wrote it -- 80 MB: 2.5
// ms written by one thread, 5.2 by 16, profiles/r6af_release_probe.json -- but giving each thread
// 16 MB instead (5 threads at 80 MB) traded 0.85 ms of fill for 0.9 of release,
// profiles/r6ag_release.json: every thread is used from 1 MB of output per thread on.)
constexpr uint64_t EXPAND_MIN_BYTES = 1u << 20;
static int expand_threads(uint64_t out_bytes) {
  static const int n = [] {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    const int c = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? CPU_COUNT(&cs) : 8;
    return std::max(1, std::min(16, c));
  }();
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(n, out_bytes / EXPAND_MIN_BYTES));
}

static void expand_runs_host(const int32_t* runs, uint64_t n, uint64_t H, int32_t* dst) {
  const int T = expand_threads(H * 8);
  const uint64_t stripe = (((H + T - 1) / T) + 511) & ~(uint64_t)511;
  auto work = [=](uint64_t r0, uint64_t r1) {
    uint64_t lo = 0, hi = n;                            // the run covering r0
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((uint64_t)(uint32_t)runs[3 * mid] <= r0) lo = mid; else hi = mid;
    }
    uint64_t r = r0;
    for (uint64_t q = lo; r < r1; ++q) {
      const uint64_t st = (uint32_t)runs[3 * q];
      const uint32_t i0 = (uint32_t)runs[3 * q + 1], j0 = (uint32_t)runs[3 * q + 2];
      const uint64_t e = std::min(r1, q + 1 < n ? (uint64_t)(uint32_t)runs[3 * q + 3] : H);
      uint32_t* o = reinterpret_cast<uint32_t*>(dst) + 2 * r;
      for (uint32_t d = (uint32_t)(r - st); r < e; ++r, ++d, o += 2) {
        o[0] = i0 + d;
        o[1] = j0 + d;
      }
    }
  };
  HostPool::get().run(T, [&](int t) {
    const uint64_t a = std::min(H, t * stripe), b = std::min(H, a + stripe);
    if (a < b) work(a, b);
  }, H * 8 >= HOST_BIG_BYTES);
}

void rows_to_host(const int2* d_rows, uint64_t H, int32_t* dst, hipStream_t s) {
  if (!H) return;
  const char* hre = test_build_knob("KMHG_HOST_RUNS");    // (read per call: tests flip it)
  const bool runs_on = !(hre && hre[0] == '0');
  if (!runs_on || H < RUNS_HOST_MIN || H > INT32_MAX) {
    d2h_host(dst, d_rows, H * 8, s);
    return;
  }
  ReleaseGroup rg(s);
  const uint64_t nt = (H + TILE - 1) / TILE;
  DBuf<uint64_t> tiles(nt + scan_u64_scratch(nt), s);
  PinnedRec hrec = PinnedPool::get().take();
  GiveBack give_back{hrec, s};
  uint64_t* total = &hrec.meta->n_kmers;
  LAUNCH("k_runs_count", s, launch_runs_count(d_rows, H, tiles.p, s));
  LAUNCH("k_scan_tiles_u64", s, launch_scan_u64(tiles.p, nt, total, tiles.p + nt, s));
  HIPC(hipStreamSynchronize(s));
  const uint64_t n = __atomic_load_n(total, __ATOMIC_ACQUIRE);
  if (n * 12 * RUNS_HOST_GAIN > H * 8) {                // runs would not pay: the rows
    d2h_host(dst, d_rows, H * 8, s);
    return;
  }
  DBuf<int32_t> druns(3 * n, s);
  LAUNCH("k_runs_emit", s, launch_runs_emit(d_rows, H, tiles.p, druns.p, s));
  PinRuns& pr = pin_runs();
  std::lock_guard<std::mutex> g(pr.mu);
  if (pr.cap < 3 * n) {
    if (pr.p) HIPC(hipHostFree(pr.p));                  // (no copy into it is in flight)
    pr.p = nullptr;
    pr.cap = 0;
    const size_t cap = std::max<size_t>(3 * n, 3u << 20);
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&pr.p), cap * 4, hipHostMallocPortable));
    pr.cap = cap;
  }
  HIPC(hipMemcpyAsync(pr.p, druns.p, 3 * n * 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  hint_huge_pages(dst, H * 8);
  expand_runs_host(pr.p, n, H, dst);
}

// Pageable host -> device copy for the host-pointer entry points (the R string of make.kmer.hash
// / seq.kmer.pos), ordered on `s`.
void h2d_host(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return;
  // pageable: the runtime stages it at the link's rate (10 MB in 0.194 ms, 54 GB/s,
  // tools/h2d_probe.hip).  Measured and removed: two pinned chunks filled by host threads while
  // the previous chunk's DMA runs (round 3: 0.81-0.92 ms against 0.63 for the config-2 host
  // build), and pinning the caller's pages in place (hipHostRegister: the same 0.194 ms).
  HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
}

// The hash table is sized from the number of windows (an upper bound on distinct k-mers) for a
// load factor <= 0.7; capacity is not a power of two (slot = mulhi(hash, cap)).
uint64_t table_capacity(int64_t Nw) {
  uint64_t cap = (uint64_t)((double)Nw / 0.7) + 16;
  return (cap + 7) & ~7ull;
}

// KMHG_ROW_ORDER=khash makes new indices label kmer.pos rows in the reference's khash order.
int default_row_order() {
  const char* e = std::getenv("KMHG_ROW_ORDER");
  return (e && std::string(e) == "khash") ? KMHG_ORDER_KHASH : KMHG_ORDER_FIRST;
}

struct Canon {              // readout order arrays (first occurrence or khash), built on use
  bool ready = false;
  int order = KMHG_ORDER_FIRST;   // which order the arrays below hold
  DBuf<uint32_t> perm, canon_off, pkeys;
  DBuf<uint64_t> pair_off;
  DBuf<uint2> rinfo;        // {count, aux} of each row's slot (readout kernels read rows in order)
  uint64_t n_multi = 0;
};

}  // namespace

// ============================================================================ objects
struct kmhg_index {
  int k = 0;
  int device = 0;
  hipStream_t stream = nullptr;   // last stream the index was used on (ordered release)
  int64_t L = 0;
  Geom geom{1, 1};             // nb buckets x capb slots (+1 side slot)
  uint64_t U = 0, N = 0, P = 0;
  uint64_t slots() const { return (uint64_t)geom.nb * geom.capb + 1; }
  uint32_t max_n = 0;
  DBuf<Slot> table;
  DBuf<int32_t> positions;
  Canon canon;
  int row_order = default_row_order();   // kmer.pos k-mer order (KMHG_ORDER_*)
  // asynchronous build (kmhg_build_device returns before the kernels finish): the totals land
  // in `rec`; `src` is kept for the overflow fallback until finish_build()
  bool pending = false;
  PinnedRec rec;
  const uint8_t* src = nullptr;
  // counts index (count.kmers, kmhg_count.hip): sources > 0.  `positions` then holds the
  // U x sources count matrix (row-major, rows_cap allocated), `ckeys` the keys of the rows,
  // slot_row / row_slot the table <-> row maps.  count.kmers rows are appended in slot order with
  // their insertion-order keys `rord`; before a readout, `rorder` (first-insertion rank -> row)
  // is derived from them (ensure_row_order; order_ready) -- the rows themselves never move.  A
  // suffix hash's rows are order-free (no rord, no rorder).
  uint32_t sources = 0;
  bool canonical = false;         // suffix hash (count.kmers.fq.sh.rp): canonical k-mer counts
  uint64_t rows_cap = 0, kmer_count = 0;
  bool u_upper = false;           // U is only an upper bound (batch table of the global fallback)
  // last read batch (kmhg_sh_last_batch): HLL distinct estimate, bucket spread, build path
  double co_est = 0;
  int co_spread = 0, co_path = 0;
  DBuf<uint64_t> ckeys, rord;
  DBuf<uint32_t> rorder;
  bool order_ready = true;
  // per-bucket statistics of a partitioned build (bstats_nb buckets, 0 for other builds): a
  // batch index adopted by a counts index takes its row offsets from them (k_count_walk_b)
  DBuf<BucketStats> bstats;
  uint32_t bstats_nb = 0;
  DBuf<uint32_t> slot_row, row_slot;
  // seq.kmer.pos diagonal path (DiagIdx, kmhg_kernels.h): the index sequence's 2-bit code words
  // and window bits, written by the build (V_hist0); the bits of repeated keys' windows are
  // cleared and the slot tags built on the first eligible query (V_diag_prep)
  DBuf<uint64_t> dcodes;
  DBuf<uint8_t> ptag;             // one tag byte per table slot (0 = empty)
  // part of an owner-computes build (kmhg_build_device_part): holds buckets
  // [geom.b0, geom.b0 + geom.nb) of a table of geom.nbh buckets; exported for an assembly, or
  // queried in place by the owner-routed query (kmhg_query_run_device_part)
  bool is_part = false;
  // ps_ready: published (release) after the preparing query's synchronize; read (acquire) by
  // later queries, possibly on other threads, before they use ptag / the uniq bits
  std::atomic<bool> ps_ready{false};
  // how the index was built (kmhg_info.build / .fallback): KMHG_BUILD_* and whether
  // finish_build() had to rebuild it with the global-atomic build
  int build_kind = 0;
  int fallback = 0;
  // copies of this index on other devices for multi-device queries (KMHG_DEVICES), keyed by
  // device (one per device); made on first use by peer copies over xGMI, freed with the index
  std::map<int, kmhg_index*> replicas;
  std::mutex rep_mu;
  bool ps_failed = false;                 // guarded by ps_mu
  // the build wrote ptag and the repeated keys' window bits (build_device_v2, build-time tags):
  // the first diagonal query derives uniq alone (V_diag_valid)
  bool tags_built = false;
  std::mutex ps_mu;
  DiagBlock diag_block_of() const { return diag_block(dcodes.p, L - k + 1); }
  DiagIdx diag_view() const {
    const DiagBlock b = diag_block_of();
    return DiagIdx{b.code, b.uniq, L - k + 1};
  }
  // stream-ordered release of everything the index holds (work queued on `s` may still read it)
  void bind_all(hipStream_t s) {
    table.bind(s); positions.bind(s); ckeys.bind(s); rord.bind(s); rorder.bind(s); bstats.bind(s);
    slot_row.bind(s);
    row_slot.bind(s); dcodes.bind(s); ptag.bind(s);
    canon.perm.bind(s); canon.canon_off.bind(s); canon.pkeys.bind(s); canon.pair_off.bind(s);
    canon.rinfo.bind(s);
  }
};

struct kmhg_query {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t H = 0;
  DBuf<int2> rows;
  // multi-device query (KMHG_DEVICES): one part per device, each holding the rows of its
  // contiguous window range in its own HBM; part i's rows start at row part_off[i].  `rows`
  // then stays empty until a device-side reader asks for them on `device` (gathered once).
  std::vector<kmhg_query*> parts;
  std::vector<int64_t> part_off;
  bool gathered = false;
  // a query over a part of an owner-computes build (kmhg_query_run_device_part): the first row
  // of each query tile (TILE windows from w0), for the root's merge of the parts' rows
  DBuf<uint64_t> tile_off;
  int64_t n_tiles = 0;
  // a range query run for the sharded gather (kmhg_query_run_device_range_runs): its rows as
  // n_runs diagonal runs {first row, i, j} instead of `rows` (n_runs = -1: it holds rows)
  DBuf<int32_t> runs;
  int64_t n_runs = -1;
};

namespace {

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    HIPC(hipGetDevice(&prev));
    if (dev != prev) HIPC(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

inline bool LCN(char c) { return (c | 0x20) == 'n'; }   // LC(c) == 'n', src/kmer_util.h:10

size_t effective_len(const char* seq, size_t L) {   // a C string ends at its first NUL
  const void* z = memchr(seq, 0, L);
  return z ? (size_t)((const char*)z - seq) : L;
}

// A host string to the device, returning its C length (its first NUL, else L).  From
// H2D_SCAN_MIN bytes on, a second thread issues the copy of all L bytes while this one scans
// for the NUL (10 MB: 0.07 ms; 500 MB: ~3.5 ms), so the scan costs nothing beside the copy;
// bytes past a NUL are copied and never read.  d_dst holds at least L bytes.
constexpr size_t H2D_SCAN_MIN = 4u << 20;
size_t h2d_cstring(void* d_dst, const char* seq, size_t L, hipStream_t s) {
  if (L < H2D_SCAN_MIN) {
    const size_t n = effective_len(seq, L);
    h2d_host(d_dst, seq, n, s);
    return n;
  }
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  Error err{KMHG_OK, ""};
  std::thread copy([&] {
    try {
      DeviceGuard g(dev);                    // (the current device is per thread)
      h2d_host(d_dst, seq, L, s);
    } catch (const Error& e) {
      err = e;
    }
  });
  const size_t n = effective_len(seq, L);
  copy.join();
  if (err.code != KMHG_OK) fail(err.code, err.msg);
  return n;
}

void check_build_args(size_t L, int k) {
  // make_kmer_h_index, src/kmer_hash.c:514-520
  if (k < 1 || k > 32) fail(KMHG_EINVAL, "k must be a positive integer less than 1+MAX_K");
  if ((int64_t)L <= k) fail(KMHG_EINVAL, "the length of the sequence must be at least k");
  if (L >= (size_t)INT32_MAX) fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1 (int positions)");
}

void check_query_args(size_t L, int k) {
  // sequence_kmer_positions, src/kmer_hash.c:1163-1164
  if ((int64_t)L <= k || k > 31 || k < 1)
    fail(KMHG_EINVAL,
         "the sequence should be longer than k and k should not be longer than 31");
  if (L >= (size_t)INT32_MAX) fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1 (int positions)");
}

// ---------------------------------------------------------------------------- build
kmhg_index* build_device_v1(const uint8_t* d_seq, int64_t L, int k, hipStream_t s) {
  ReleaseGroup rg(s);
  auto idx = std::make_unique<kmhg_index>();
  idx->stream = s;
  idx->build_kind = KMHG_BUILD_GLOBAL;
  HIPC(hipGetDevice(&idx->device));
  idx->k = k;
  idx->L = L;
  const int64_t Nw = L - k + 1;
  const bool aligned = (reinterpret_cast<uintptr_t>(d_seq) & 15) == 0;
  idx->geom = Geom{1u, (uint32_t)table_capacity(Nw)};
  const uint64_t nslots = idx->slots();
  idx->table.reset(nslots);
  DBuf<uint32_t> win_slot(Nw, s);
  LAUNCH("k_table_init", s, launch_table_init(idx->table.p, nslots, s));
  LAUNCH("k_build_insert", s,
         launch_build_insert(d_seq, L, k, idx->table.p, idx->geom, win_slot.p, Nw, aligned, s));
  // compaction scratch: look-back status + ticket + meta in one zeroed block
  const uint32_t nt = tiles_for(nslots);
  const size_t scratch_bytes = (size_t)nt * 8 + 64 + sizeof(BuildMeta);
  DBuf<uint8_t> scratch(scratch_bytes, s);
  HIPC(hipMemsetAsync(scratch.p, 0, scratch_bytes, s));
  uint64_t* status = reinterpret_cast<uint64_t*>(scratch.p);
  uint32_t* ticket = reinterpret_cast<uint32_t*>(scratch.p + (size_t)nt * 8);
  BuildMeta* meta = reinterpret_cast<BuildMeta*>(scratch.p + (size_t)nt * 8 + 64);
  DBuf<uint64_t> ukeys(Nw, s);            // dense CSR arrays: sort bookkeeping only
  DBuf<uint32_t> counts(Nw, s), offsets(Nw + 1, s);
  DBuf<uint32_t> small_ids(Nw / 2 + 1, s), large_ids(Nw / LARGE_MIN + 1, s);
  LAUNCH("k_build_compact", s,
         launch_build_compact(idx->table.p, nslots, status, ticket, ukeys.p, counts.p,
                              offsets.p, small_ids.p, large_ids.p, meta, s));
  idx->positions.reset(Nw);
  LAUNCH("k_build_scatter", s, launch_build_scatter(win_slot.p, Nw, idx->table.p,
                                                    idx->positions.p, s));
  LAUNCH("k_sort_small", s, launch_sort_small(small_ids.p, meta, counts.p, offsets.p,
                                              idx->positions.p, s));
  LAUNCH("k_sort_large", s,
         launch_sort_large(large_ids.p, meta, counts.p, offsets.p, idx->positions.p,
                           reinterpret_cast<int32_t*>(win_slot.p), s));
  LAUNCH("k_inline_singles", s, launch_inline_singles(idx->table.p, nslots, idx->positions.p, s));
  BuildMeta hm;
  HIPC(hipMemcpyAsync(&hm, meta, sizeof(hm), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  idx->U = hm.n_kmers;
  idx->N = hm.n_positions;
  idx->P = hm.n_pairs;
  idx->max_n = hm.max_count;
  return idx.release();
}

// Bucket-id radix streams (position builds that keep their code words) up to this many windows
// (build_device_v2); KMHG_BUILD_BID=0 / 1 forces key / bucket-id streams.
constexpr int64_t BID_MAX_WINDOWS = 12 << 20;
bool bid_streams_for(int64_t Nw) {
  const char* bide = test_build_knob("KMHG_BUILD_BID");
  return bide ? bide[0] == '1' : Nw <= BID_MAX_WINDOWS;
}

// One round of the bucket kernel on the current device: its CUs x the workgroups one CU holds
// (cached per device; 0 if the device cannot be queried).
uint32_t bucket_round_of_current_device() {
  static std::atomic<uint32_t> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  if (dev < 64) {
    if (uint32_t v = cache[dev].load(std::memory_order_relaxed)) return v;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 0;
  const uint32_t v = (uint32_t)std::max(cus, 0) * (uint32_t)KMHG_BUCKET_WGS;
  if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

constexpr double CO_FILL = 0.6;                  // target mean occupancy of a count-only bucket

// Stream entries per group bucket (in units of V2_BW_WG) for a batch of `total` keys with
// ~`distinct` distinct ones: mean distinct keys per bucket ~CO_FILL x V2_CAPW, at most 4x.
// KMHG_CO_SPREAD (tests) forces one, rounded down to a divisor of 12 (build_device_v2).
int co_spread_for(double distinct, uint64_t total) {
  if (const char* e = test_build_knob("KMHG_CO_SPREAD")) {
    int f = std::max(1, std::min(12, std::atoi(e)));
    while (12 % f) --f;
    return f;
  }
  const double ratio = std::max(std::min(distinct / std::max<double>((double)total, 1.0), 1.0), 1e-3);
  const int f = (int)(CO_FILL * V2_CAPW / (V2_BW_WG * ratio));
  return std::max(1, std::min(4, f));
}

// Partitioned build (kmhg_build_v2.hip): LSD radix partition of the windows by hash bucket,
// then one wave per bucket builds its sub-table in LDS.  Falls back to v1 if a bucket's LDS
// sub-table overflows (position builds: never observed -- distinct keys per bucket ~ Binomial,
// mean <= V2_BW; count-only builds retry at spread 1 instead, sh_count_reads_device).
// Partitioned build over the windows of a sequence (d_seq), or over a stream of n_keys
// distinct keys (d_keys, d_seq == nullptr; the counts index's table rebuild): key r is stored
// with count 1 and aux = r + 1.
// count_only (a key stream whose positions nobody reads: read counting): the group bucket kernel
// skips its position pass and no positions array is kept.
// count_only with co_spread = 0: the spread is chosen from the key stream's own HLL estimate
// (co_spread_for), read back while the radix passes run.
// skip_empty (count-only key streams of k <= 31): EMPTY_KEY entries are padding, not keys --
// the first pass drops them, and the valid count comes from its scan.
kmhg_index* build_device_v2(const uint8_t* d_seq, int64_t L, int k, hipStream_t s,
                            const uint64_t* d_keys = nullptr, int64_t n_keys = 0,
                            bool count_only = false, int co_spread = 1, bool skip_empty = false,
                            bool codes = false, uint32_t part = 0, uint32_t n_parts = 0) {
  ReleaseGroup rg(s);             // the scratch buffers below: one release event
  const uint8_t* d_src = d_seq;   // the caller's buffer (the v1 fallback re-reads it)
  auto idx = std::make_unique<kmhg_index>();
  idx->stream = s;
  HIPC(hipGetDevice(&idx->device));
  idx->build_kind = ballot_ranks() ? KMHG_BUILD_PARTITIONED_BALLOT : KMHG_BUILD_PARTITIONED;
  idx->k = k;
  idx->L = L;
  const bool from_keys = d_seq == nullptr;
  const int64_t Nw = from_keys ? n_keys : L - k + 1;
  if (from_keys && Nw < 1) fail(KMHG_EINVAL, "empty key stream (internal error)");
  if (skip_empty && !(from_keys && count_only && k < 32))
    fail(KMHG_EINVAL, "padded key stream outside a count-only build (internal error)");
  // the partition kernels read the sequence as aligned 16-B words: copy an unaligned input
  DBuf<uint8_t> aligned_copy;
  if (!from_keys && (reinterpret_cast<uintptr_t>(d_seq) & 15) != 0) {
    aligned_copy.reset((size_t)L);
    aligned_copy.bind(s);
    HIPC(hipMemcpyAsync(aligned_copy.p, d_seq, (size_t)L, hipMemcpyDeviceToDevice, s));
    d_seq = aligned_copy.p;
  }
  const uint32_t ntiles = (uint32_t)((Nw + PTILE - 1) / PTILE);   // partition tiles
  // radix plan: fewest passes whose radix fits LDS.  Tiles of PTILE windows keep ~PTILE / R
  // elements per digit run: beyond ~300 digits the runs get too short for coalesced writes and
  // an extra pass is cheaper.
  uint32_t maxr = V2_MAXR_IL;
  const char* e = test_build_knob("KMHG_MAXR");   // testing knob: force more radix passes
  if (e && e[0])
    maxr = std::max<uint32_t>(2u, std::min<uint32_t>(maxr, (uint32_t)std::atoi(e)));
  auto plan = [&](uint32_t nbk, uint32_t& R) {
    for (uint32_t passes = 1; passes <= 4; ++passes) {
      R = (uint32_t)std::ceil(std::pow((double)nbk, 1.0 / passes) - 1e-9);
      while (std::pow((double)R, (double)passes) < (double)nbk) ++R;
      if (R <= maxr) return passes;
    }
    return 5u;
  };
  // group buckets: 1024 windows, one workgroup each.  (Wave buckets of 256 windows were
  // removed in round 4: group buckets halve the radix -- config 2 26.1 vs 24.8 Gbp/s -- and save
  // a pass from ~26 M windows -- config 3 26.3 vs 24.5.)
  // count-only builds: co_spread x more stream entries per group bucket -- a read batch's
  // distinct keys are a fraction of its key stream, so fewer buckets still fit their LDS
  // sub-tables (co_spread_for); one overflowing bucket fails the whole build (meta->overflow)
  // and sh_count_reads_device rebuilds at spread 1.  With co_spread = 0 the radix passes sort
  // by the bucket b1 among nb1 = 12 * ceil(Nw / (12 * V2_BW_WG)): the bucket among nb1 / s is
  // b1 / s exactly (floor(floor(h nb1 / 2^64) / s) = floor(h (nb1 / s) / 2^64)), so one sorted
  // stream serves every spread s in {1, 2, 3, 4}, and s is picked only before the bucket stage.
  const bool co_auto = count_only && co_spread == 0;
  int64_t bw_g = V2_BW_WG;
  if (count_only && !co_auto) bw_g *= std::max(1, std::min(8, co_spread));
  uint32_t nb_g =
      co_auto ? (uint32_t)(12 * std::max<int64_t>(1, (Nw + 12 * V2_BW_WG - 1) / (12 * V2_BW_WG)))
              : (uint32_t)std::max<int64_t>(1, (Nw + bw_g - 1) / bw_g);
  // Whole rounds of the bucket kernel: its workgroups take about equally long, so 4.77 rounds of
  // the device's resident workgroups (config 2: 9,766 buckets on 256 CUs x 8) cost 5; rounding
  // the bucket count up to whole rounds gives each bucket fewer windows instead (position builds
  // of 2-16 rounds; the parts of an owner-computes build split the same rounded table, so they
  // still assemble into the single-device table).  Only when the extra buckets are few (at most
  // an eighth more: a build just past a round boundary would otherwise nearly double its table
  // and halve its load).  The round is the building device's own (CUs x workgroups per CU).
  // KMHG_NB_ROUND=0 (test build) keeps ceil(windows / 1,024).
  if (!from_keys && !count_only) {
    const char* nre = test_build_knob("KMHG_NB_ROUND");
    if (!(nre && nre[0] == '0')) {
      const uint32_t wave_wg = bucket_round_of_current_device();
      if (wave_wg && nb_g > wave_wg && nb_g <= 16 * wave_wg) {
        const uint32_t rounded = (nb_g + wave_wg - 1) / wave_wg * wave_wg;
        if (rounded - nb_g <= nb_g / 8) nb_g = rounded;
      }
    }
  }
  uint32_t R = 0;
  uint32_t nb = nb_g;
  uint32_t passes = plan(nb_g, R);
  // owner-computes part (the reference's reader-pool partition,
  // src/kmer_reader.c:28-39): the whole build's geometry, of which this part keeps the buckets
  // [b0, b1) -- every window is encoded and hashed, only the part's keys are partitioned
  uint32_t b0 = 0, nbh = 0;
  if (n_parts >= 1) {           // n_parts = 0: a whole build
    if (from_keys || count_only) fail(KMHG_EINVAL, "part builds index sequences only");
    b0 = (uint32_t)((uint64_t)nb * part / n_parts);
    const uint32_t b1 = (uint32_t)((uint64_t)nb * (part + 1) / n_parts);
    nbh = nb;
    idx->is_part = true;
    if (b1 <= b0) {              // more parts than buckets: an empty part (nothing to build)
      idx->geom = Geom{0u, V2_CAPW, b0, nbh};
      idx->table.reset(1);
      idx->positions.reset(1);
      return idx.release();
    }
    nb = b1 - b0;
    passes = plan(nb, R);
  }
  if (passes > 4) fail(KMHG_EOVERFLOW, "sequence too long for the partitioned build");
  idx->geom = Geom{nb, V2_CAPW, b0, nbh};
  const Geom g = idx->geom;
  const uint64_t nhist = (uint64_t)R * ntiles;
  const uint32_t scan_tiles = tiles_for(nhist);
  // bucket-id streams (position builds that keep the code words): the radix passes carry
  // (bucket id, pos) -- 8 B per window instead of 12 -- the last pass positions only, and the
  // bucket kernel cuts each key from the code words.  The cut is a random 12-B read per window:
  // cheap while the code words (Nw / 4 bytes) stay in an XCD's 4 MB L2, a 128-B Infinity-Cache
  // line per window beyond.  Measured (A/B in one run): config 2 (10 M windows, 2.5 MB of code)
  // 30.1 -> 31.1 Gbp/s; config 3 (100 M, 25 MB) 28.5 -> 24.0 (bucket kernel 0.84 -> 2.0 ms).
  // So on up to BID_MAX_WINDOWS; KMHG_BUILD_BID=0 / 1 forces key / bucket-id streams.
  const bool bid = codes && !from_keys && !count_only && bid_streams_for(Nw);
  // position builds on key streams carry packed 12-B (key, pos) elements: a tile's digit run is
  // one contiguous write instead of a key piece and a position piece in two arrays
  // (tools/scatter_pattern.hip layout, profiles/r5a_scatter_layout.txt: radix 313 1.09 -> 0.87
  // ms per 100 M elements, radix 79 0.72 -> 0.61).  Built with -DKMHG_NO_AOS: SoA streams (A/B).
#ifdef KMHG_NO_AOS
  const bool aos = false;
#else
  const bool aos = !from_keys && !count_only && !bid;
#endif
  // Which streams are packed (stream p = pass p's output; -1 = a part build's dense stream):
  // the last one, which only the bucket kernel reads, always; an earlier one only at a radix
  // where the scatter's saving beats the 4 more bytes per element its histogram pass then reads.
  // Measured: config 3 (2 passes, radix 313) every stream packed 3.49 -> 3.21 ms per build
  // (scatters 0.94 + 1.03 -> 0.75 + 0.91 ms, histogram 0.27 -> 0.36); the 500 Mbp build (3
  // passes, radix 79) 18.2 -> 18.6 ms (histograms 1.9 -> 2.8 ms, scatters 11.2 -> 10.3), A/B
  // in one run (profiles/r5b_ab_aos_config3.log, r5c_ab_aos_config5.log).
  constexpr uint32_t AOS_MIN_RADIX = 160;
  // Pack8 (two-pass builds of small k: 2k <= 52): the first pass writes 8-B elements, key << sh
  // | the window's index inside its segment of 2^sh windows (sh = 64 - 2k), and the second pass
  // restores the position from the element's place in the stream (k_seg_bounds' table).  The
  // first stream's writes and the histogram pass's reads shrink from 12 to 8 B per window.
  // KMHG_PACK8=0 keeps the 12-B first stream (A/B, tests).
  const int sh8 = 64 - 2 * k;
  const uint64_t seg8 = sh8 >= 12 && sh8 < 64 ? (1ull << sh8) : 0;
  const uint32_t nseg8 = seg8 ? (uint32_t)(((uint64_t)Nw + seg8 - 1) / seg8) : 0;
  const char* p8e = test_build_knob("KMHG_PACK8");
  const bool pack8 = aos && passes == 2 && n_parts < 2 && seg8 && nseg8 <= 256 &&
                     !(p8e && p8e[0] == '0');
  // Digit streams (DS): each pass before the last also writes every output element's digit of
  // the next pass (u8 up to radix 256, else u16), and that pass's histogram reads 1-2 B per
  // element instead of the keys -- which also takes away the reason to leave the middle streams
  // unpacked.  The digit writes are short scattered runs (PTILE / R elements per tile and
  // digit); u8 digits pay once the streams outgrow the Infinity Cache, u16 digits (radix
  // 257-320: two-pass builds of ~66-100 M windows) did not.  Measured (A/B in one run,
  // profiles/r5y_ab_ds_*, r5y_ds_sizes_build_only.txt, k = 31 unless noted):
  //   u8: 500 Mbp (3 passes, radix 79) 18.37 -> 16.82 ms (u16 17.75; histograms 1.93 -> 0.48
  //     ms); 200 Mbp (3 passes, radix 59) 6.85 -> 6.23; 60 Mbp 1.773 -> 1.744; 40 Mbp
  //     1.115 -> 1.093; 30 Mbp 0.815 -> 0.804; but 20 Mbp 0.536 -> 0.549 and 16 Mbp
  //     0.433 -> 0.446 (in cache);
  //   u16: 100 Mbp (radix 317) 3.127 -> 3.149 ms; config 3 (k = 21, Pack8 first stream)
  //     2.81 -> 2.93 (histogram -0.11, first scatter +0.22 ms).
  // Sequence builds with positions on key streams without Pack8, radix <= 256, from
  // DS_MIN_WINDOWS windows; KMHG_DIGIT_STREAM=0 / 1 forces off / on, KMHG_DS_U8=0 u16 digits.
  // Bucket-id streams (u32 ids, in-cache sizes) can carry them too, but it is a wash: config 2
  // histogram 10.2 -> 6.7 us, first scatter +3-6 us, build 0.2076-0.2092 ms either way
  // (profiles/r5y_ab_ds_bid_config2.log).  KMHG_DS_BID=1 (or KMHG_DIGIT_STREAM=1) turns them on.
  constexpr int64_t DS_MIN_WINDOWS = 25'000'000;
  const char* dse = test_build_knob("KMHG_DIGIT_STREAM");
  const char* dbe = test_build_knob("KMHG_DS_BID");
  // (a part build's later streams hold ~1/n_parts of the windows)
  const int64_t ds_windows = n_parts >= 2 ? Nw / n_parts : Nw;
  const bool ds_keys = !bid && !from_keys && !count_only && passes >= 2 &&
                       (dse && dse[0] ? dse[0] == '1'
                                      : !pack8 && R <= 256 && ds_windows >= DS_MIN_WINDOWS);
  const bool ds_bids = bid && passes >= 2 &&
                       (dse && dse[0] ? dse[0] == '1' : R <= 256 && dbe && dbe[0] == '1');
  const bool ds_on = ds_keys || ds_bids;
  const char* dpe = test_build_knob("KMHG_DS_PACK");
  const bool ds_pack = ds_keys && !(dpe && dpe[0] == '0');
  auto packed = [&](int p) {
    return aos && (p + 1 == (int)passes || R >= AOS_MIN_RADIX || ds_pack);
  };
  bool any_unpacked = !aos;
  for (int p = -1; p + 1 < (int)passes; ++p) any_unpacked |= !packed(p) && !(pack8 && p == 0);
  const uint64_t kwords = bid ? 1 : aos ? ((uint64_t)(Nw + PTILE) * 3 + 1) / 2 : (uint64_t)(Nw + PTILE);
  DBuf<uint64_t> kA(kwords, s), kB(kwords, s);   // + pad
  // (Removed in round 4 after measurement, DESIGN.md §5: radix passes writing whole 128-B lines
  // through LDS write-combining buffers -- config 3 29.2 -> 25.0-28.7 Gbp/s, the 500 Mbp build
  // 18.1 -> 18.9-22.7 ms.)
  // bucket ids: pass p writes bA / bB alternately; the last pass writes none (the bucket starts
  // come from the histograms)
  // (bB first holds V_hist0's per-window ids, the first pass's input)
  DBuf<uint32_t> bA(bid && passes > 1 ? Nw + PTILE : 1, s);
  DBuf<uint32_t> bB(bid ? Nw + PTILE : 1, s);
  const bool no_pos = count_only;                        // keys only through the passes
  // (a part build's compacted windows land in kB / pB before they are packed: pB stays)
  const bool partc_pos = !from_keys && n_parts >= 2 && codes;
  DBuf<uint32_t> pA(no_pos || !any_unpacked ? 1 : Nw + PTILE, s),
      pB(no_pos || (!any_unpacked && !partc_pos) ? 1 : Nw + PTILE, s);
  const uint32_t pad = (uint32_t)Nw;
  DBuf<uint32_t> hist(nhist, s);
  DBuf<uint32_t> start((uint64_t)nb + 1, s);
  DBuf<uint32_t> segb(pack8 ? (uint64_t)R * (nseg8 + 1) : 1, s);
  // one digit buffer: pass p's histogram has read it before pass p rewrites it for pass p + 1
  // u8 digits at a radix <= 256 (KMHG_DS_U8=0: u16, A/B)
  const char* d8e = test_build_knob("KMHG_DS_U8");
  const bool ds8 = ds_on && R <= 256 && !(d8e && d8e[0] == '0');
  DBuf<uint16_t> dsb(ds_on ? ((uint64_t)Nw + PTILE + 8) / (ds8 ? 2 : 1) + 8 : 1, s);
  uint8_t* ds8p = ds8 ? reinterpret_cast<uint8_t*>(dsb.p) : nullptr;
  uint16_t* ds16p = ds8 ? nullptr : dsb.p;
  bool ds_ready = false;                                  // dsb holds the next pass's digits
  const Pack8 pk8{pack8 ? sh8 : 0, segb.p, nseg8, make_digit(1, R)};
  // scratch (zeroed in-kernel by V_hist0 / V_hist, no memset): [n_valid][meta][scan status]
  const size_t off_meta = 64, off_status = 128;
  const uint32_t n_status = scan_tiles + 1;               // look-back words + ticket
  const size_t scratch_bytes = off_status + (size_t)n_status * 8;
  DBuf<uint8_t> scratch(scratch_bytes, s);
  uint8_t* sc = scratch.p;
  uint32_t* n_valid = reinterpret_cast<uint32_t*>(sc);
  BuildMeta* meta = reinterpret_cast<BuildMeta*>(sc + off_meta);
  uint64_t* status = reinterpret_cast<uint64_t*>(sc + off_status);
  idx->rec = PinnedPool::get().take();                     // V_stats writes the totals here
  if (!co_auto) idx->table.reset(idx->slots());
  idx->positions.reset(no_pos ? 1 : Nw);
  idx->bstats.reset(nb);            // kept: a batch index's walk takes its row offsets from it
  // co_auto: HLL rows of the first histogram pass, V_hll's registers + ticket, its pinned record
  DBuf<uint32_t> hll_rows(co_auto ? (size_t)ntiles * (HLL_REGS / 4) : 1, s);
  DBuf<uint32_t> hll_regs(co_auto ? HLL_PART_WORDS : 1, s);
  PinnedRec hrec;
  if (co_auto) hrec = PinnedPool::get().take();

  // bucket starts straight from the histograms (V_bounds_lo), one level per pass p >= 1:
  // lo_save = pass 0's digit starts (saved by pass 1's V_hist), lvA / lvB = S_p of the passes
  // before the last (3+ passes), the last level writes `start`
  DBuf<uint32_t> lo_save(passes >= 2 ? R : 1, s);
  uint64_t r_top = 1;                                   // R^(passes - 1)
  for (uint32_t i = 1; i < passes; ++i) r_top *= R;
  DBuf<uint32_t> lvA(passes >= 3 ? r_top + 1 : 1, s), lvB(passes >= 4 ? r_top + 1 : 1, s);
  uint64_t *kin = kA.p, *kout = kB.p;
  uint32_t *pin = pA.p, *pout = pB.p;
  uint32_t div = 1;
  DiagBlock db{nullptr, nullptr, nullptr};
  // a part of 4+ (key streams): V_hist0 also writes the part's windows compacted per tile into
  // kB / pB (free until then) with their counts; a scan of the counts and one copy make them a
  // dense (key, position) stream of ~1/n_parts of the windows, and every radix pass runs over
  // that alone -- instead of encoding and hashing every window again in a first pass over all
  // of them.  It costs a copy and one more pass over the part's windows, so it pays from 4
  // parts on (one-GPU rehearsal, tools/part_step.py, per-rank step of 10 Mbp per part: 2 parts
  // 0.397 -> 0.467 ms, 4 parts 0.504 -> 0.495, 8 parts 0.749 -> 0.581).  KMHG_PART_COMPACT=0 / 1
  // forces the first pass over every window / the compaction (tests).
  const char* pce = test_build_knob("KMHG_PART_COMPACT");
  const bool partc = !from_keys && n_parts >= 2 && !bid && codes &&
                     (pce ? pce[0] == '1' : n_parts >= 4);
  DBuf<uint32_t> tcnt(partc ? ntiles : 1, s);
  if (from_keys) {   // pass 0 reads the caller's key stream in place (positions implicit)
    HIPC(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(n_valid), (int)Nw, 1, s));
    HIPC(hipMemsetAsync(meta, 0, sizeof(BuildMeta), s));
  } else {
    // a position index keeps its sequence's code words + window bits for the diagonal query
    // path (code words + N flags, 0.5 B per window with the first query's bits; V_hist0 writes them)
    if (codes) {
      idx->dcodes.reset(diag_block_words(Nw));
      db = idx->diag_block_of();
    }
    LAUNCH("k_v2_hist0", s,
           launch_v2_hist0(d_seq, L, k, Nw, g, make_digit(1, R), hist.p, ntiles, status,
                           n_status, meta, s, db.code, db.nbit, bid ? bB.p : nullptr,
                           partc ? kB.p : nullptr, partc ? pB.p : nullptr,
                           partc ? tcnt.p : nullptr));
    if (partc) {   // tile counts -> tile offsets, the part's window count -> n_valid
      LAUNCH("k_scan_u32", s, launch_scan_u32(tcnt.p, ntiles, status, n_valid, s));
    } else {
      LAUNCH("k_scan_u32", s, launch_scan_u32(hist.p, nhist, status, n_valid, s));
      if (bid) {
        const DigitOut ds0{ds16p, make_digit(R, R), ds8p};
        LAUNCH("k_v2_scatter_seq", s,
               launch_v2_scatter_bid0(bB.p, Nw, g, make_digit(1, R), hist.p, ntiles,
                                      passes == 1 ? nullptr : bA.p, pA.p, pad, s,
                                      ds_on ? &ds0 : nullptr));
        ds_ready = ds_on;
      } else {
        const DigitOut ds0{ds16p, make_digit(R, R), ds8p};
        LAUNCH("k_v2_scatter_seq", s,
               launch_v2_scatter_seq(d_seq, L, k, Nw, g, make_digit(1, R), hist.p, ntiles, kA.p,
                                     pA.p, pad, s, packed(0), pack8 ? &pk8 : nullptr,
                                     ds_on ? &ds0 : nullptr));
        ds_ready = ds_on;
        // the segment table, before pass 1's histogram overwrites pass 0's
        if (pack8)
          LAUNCH("k_seg_bounds", s,
                 launch_seg_bounds(hist.p, ntiles, R, nseg8, (uint32_t)(seg8 / PTILE), n_valid,
                                   segb.p, s));
      }
      div = R;
    }
  }
  uint32_t *bin = bA.p, *bout = bB.p;
  // the later passes' histogram layout: [digit][tile] over the tiles of their input.  A part
  // build keeps ~1/n_parts of the windows after pass 0, so it reads that count back and sizes
  // the later passes to it (a separate histogram, so pass 0's column 0 stays readable) instead
  // of walking every window's tile again -- one host round trip per part build.
  uint32_t* hp = hist.p;
  uint32_t C = ntiles, nst = n_status;
  uint64_t nh = nhist;
  DBuf<uint32_t> hist1;
  if (n_parts >= 2 && (passes > 1 || partc)) {
    uint32_t nv = 0;
    HIPC(hipMemcpyAsync(&nv, n_valid, 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    C = std::max<uint32_t>(1u, (uint32_t)(((uint64_t)nv + PTILE - 1) / PTILE));
    nh = (uint64_t)R * C;
    nst = tiles_for(nh) + 1;
    hist1.reset(nh);
    hist1.bind(s);
    hp = hist1.p;
    // pass 0's digit starts (its scanned column 0), which pass 1's V_hist saves otherwise
    if (!partc)
      HIPC(hipMemcpy2DAsync(lo_save.p, 4, hist.p, (size_t)ntiles * 4, 4, R,
                            hipMemcpyDeviceToDevice, s));
  }
  if (partc)   // the part's windows, dense in window order: every radix pass reads these
    LAUNCH("k_part_dense", s, launch_part_dense(kB.p, pB.p, tcnt.p, ntiles, n_valid, kA.p, pA.p,
                                                s, packed(-1)));
  // where pass 1 saves column 0: pass 0's histogram is hp's unless pass 0 was the one over
  // every window (its own layout, copied above)
  uint32_t* save1 = hp == hist.p || partc ? lo_save.p : nullptr;
  // each level of the bucket starts rides in its pass (BoundsFuse), except the last one of a
  // count-only build whose spread is chosen after the passes (co_auto); KMHG_FUSE_BOUNDS=0
  // (A/B) launches every level on its own
  const char* fbe = test_build_knob("KMHG_FUSE_BOUNDS");
  const bool fuse_on = !(fbe && fbe[0] == '0');
  auto level_of = [&](uint32_t p, const void* kprev, bool is_bid, uint32_t spread) {
    uint64_t dv = 1;                                    // R^p lower-digit values
    for (uint32_t i = 0; i < p; ++i) dv *= R;
    const bool last = p + 1 == passes;
    const uint32_t* lin = p == 1 ? lo_save.p : ((p - 1) % 2 ? lvA.p : lvB.p);
    uint32_t* lout = last ? start.p : (p % 2 ? lvA.p : lvB.p);
    const bool p8 = pack8 && p == 1;                    // the input is the packed 8-B stream
    BoundsFuse f{reinterpret_cast<const uint64_t*>(kprev), lin, lout,
                 make_digit((uint32_t)dv, R), (uint32_t)dv, spread,
                 is_bid ? 1 : p8 ? 3 : packed((int)p - 1) ? 2 : 0,
                 last ? g.nb : (uint32_t)(dv * R)};
    f.sh = p8 ? sh8 : 0;
    return f;
  };
  auto fused = [&](uint32_t p) { return p >= 1 && fuse_on && !(co_auto && p + 1 == passes); };
  auto launch_level = [&](const BoundsFuse& f) {
    const uint64_t* kp = f.bid ? nullptr : f.kprev;
    const uint32_t* bp = f.bid ? reinterpret_cast<const uint32_t*>(f.kprev) : nullptr;
    LAUNCH("k_v2_bounds", s, launch_v2_bounds_lo(kp, n_valid, g, f.Dlast, f.div, hp, C,
                                                 f.lo_start, f.spread, f.start, f.nlim, s, bp,
                                                 f.bid == 2, f.bid == 3 ? f.sh : 0));
  };
  for (uint32_t p = 1; bid && p < passes; ++p) {
    const Digit Dp = make_digit(div, R);
    const bool last = p + 1 == passes;
    if (ds_ready)
      LAUNCH("k_v2_hist", s,
             launch_v2_hist_digits(dsb.p, ds8, n_valid, g, Dp, hp, C, status, nst, s,
                                   p == 1 ? save1 : nullptr));
    else
      LAUNCH("k_v2_hist", s,
             launch_v2_hist_bid(bin, n_valid, g, Dp, hp, C, status, nst, s,
                                p == 1 ? save1 : nullptr));
    LAUNCH("k_scan_u32", s, launch_scan_u32(hp, nh, status, n_valid, s));
    const BoundsFuse lv = level_of(p, bin, true, 1u);
    const DigitOut dsn{ds16p, make_digit(div * R, R), ds8p};
    LAUNCH("k_v2_scatter", s,
           launch_v2_scatter_bid(bin, pin, n_valid, g, Dp, hp, C, last ? nullptr : bout,
                                 pout, pad, s, fused(p) ? &lv : nullptr,
                                 ds_on && !last ? &dsn : nullptr));
    ds_ready = ds_on && !last;
    if (!fused(p) && !last) launch_level(lv);
    std::swap(bin, bout);
    std::swap(pin, pout);
    div *= R;
  }
  for (uint32_t p = from_keys || partc ? 0 : 1; !bid && p < passes; ++p) {
    const Digit Dp = make_digit(div, R);
    const bool keys0 = from_keys && p == 0;
    const bool last = p + 1 == passes;
    const uint64_t* src = keys0 ? d_keys : kin;
    const bool hll = co_auto && p == 0;
    if (ds_ready)
      LAUNCH("k_v2_hist", s,
             launch_v2_hist_digits(dsb.p, ds8, n_valid, g, Dp, hp, C, status, nst, s,
                                   p == 1 ? save1 : nullptr));
    else
      LAUNCH("k_v2_hist", s,
             launch_v2_hist(src, n_valid, g, Dp, hp, C, status, nst, s,
                            hll ? hll_rows.p : nullptr, hll ? hll_regs.p : nullptr,
                            p == 1 ? save1 : nullptr, keys0 && skip_empty,
                            /*padded=*/!keys0, !keys0 && packed((int)p - 1),
                            pack8 && p == 1 ? sh8 : 0));
    LAUNCH("k_scan_u32", s, launch_scan_u32(hp, nh, status, n_valid, s));
    if (hll) {   // after the scan: the estimate travels with the valid key count
      LAUNCH("k_v2_hll", s, launch_v2_hll(hll_rows.p, ntiles, hll_regs.p,
                                          &hrec.meta->distinct_est, n_valid,
                                          &hrec.meta->n_positions, s));
      HIPC(hipEventRecord(hrec.ev, s));
    }
    if (keys0) {
      LAUNCH("k_v2_scatter", s,
             launch_v2_scatter_keys0(d_keys, (uint64_t)Nw, n_valid, g, Dp, hist.p, ntiles, kout,
                                     pout, pad, no_pos, skip_empty, s));
    } else {
      const BoundsFuse lv = level_of(p, kin, false, 1u);
      if (no_pos)
        LAUNCH("k_v2_scatter", s,
               launch_v2_scatter_nopos(kin, n_valid, g, Dp, hp, C, kout, pad, s,
                                       fused(p) ? &lv : nullptr));
      else {
        const DigitOut dsn{ds16p, make_digit(div * R, R), ds8p};
        LAUNCH("k_v2_scatter", s,
               launch_v2_scatter(kin, pin, n_valid, g, Dp, hp, C, kout, pout, pad, s,
                                 fused(p) ? &lv : nullptr, packed((int)p), packed((int)p - 1),
                                 pack8 && p == 1 ? &pk8 : nullptr,
                                 ds_on && !last ? &dsn : nullptr));
      }
      ds_ready = ds_on && !last;
      if (p >= 1 && !fused(p) && !last) launch_level(lv);
    }
    std::swap(kin, kout);
    std::swap(pin, pout);
    div *= R;
  }
  Geom gb = g;                     // the bucket stage's geometry
  if (co_auto) {
    // the estimate landed while the later radix passes were still queued on the device
    HIPC(hipEventSynchronize(hrec.ev));
    idx->co_est = hrec.meta->distinct_est;
    const uint64_t n_keys_valid = hrec.meta->n_positions;
    PinnedPool::get().give(hrec, false);
    idx->co_spread = co_spread_for(idx->co_est, n_keys_valid);
    gb = Geom{nb / (uint32_t)idx->co_spread, V2_CAPW};
    idx->geom = gb;
    idx->table.reset(idx->slots());
  }
  if (passes == 1) {
    // one pass (pass 0 reads chars or the caller's keys): the starts are the scanned column 0
    LAUNCH("k_v2_bounds", s,
           launch_v2_bounds_lo(nullptr, n_valid, g, make_digit(1, R), 1u, partc ? hp : hist.p,
                               partc ? C : ntiles, nullptr, g.nb / gb.nb, start.p, g.nb, s,
                               nullptr));
  } else if (!fused(passes - 1)) {
    // the last pass's input: kout / bout after the final swap
    launch_level(level_of(passes - 1, bid ? static_cast<const void*>(bout) : kout, bid,
                          g.nb / gb.nb));
  }
#ifdef KMHG_STAMPS
  static uint64_t* stamps = nullptr;
  if (!stamps) HIPC(hipMallocManaged(&stamps, sizeof(uint64_t) * 8 * (1u << 22)));
  HIPC(hipMemsetAsync(stamps, 0, sizeof(uint64_t) * 8 * nb, s));
  kmhg::set_stamp_buffer(stamps);
#endif
  // tests only: a corrupted stream or bound (KMHG_TEST_DISORDER=1|2|3) -> the bucket kernel's
  // checks -> v1 rebuild
  if (const char* td = test_build_knob("KMHG_TEST_DISORDER"))
    if (!no_pos && td[0] >= '1' && td[0] <= '3')
      launch_v2_test_disorder(aos ? reinterpret_cast<uint32_t*>(kin) + 2 : pin, start.p, n_valid,
                              td[0] - '0', s, aos ? 3u : 1u);
  // Build-time tags (round 6): a position build beyond the cache (key
  // streams, Nw > BID_MAX_WINDOWS) writes the diagonal query path's slot tags and repeated-key
  // bits itself, so the first seq.kmer.pos of a new index does not pay V_diag_prep (2.6 ms at
  // 500 Mbp, +70 % on the query).  In cache (config 2) the build is the headline and the
  // preparation stays with the first query (round-3 A/B: tags in the build +1-1.5 % there).
  // A part of an owner-computes build does the same for its own slots and keys (the owner-
  // routed query runs the diagonal path on it).  KMHG_BUILD_TAGS=0 / 1 (test build) forces
  // either on key streams.
  uint8_t* tg = nullptr;
  uint32_t* rep = nullptr;
  {
    const char* bte = test_build_knob("KMHG_BUILD_TAGS");
    const bool want = codes && !bid && !from_keys && !count_only &&
                      (bte ? bte[0] == '1' : Nw > BID_MAX_WINDOWS);
    if (want) {
      try {
        idx->ptag.reset(idx->slots() + 32);    // + the 32-B span the last probe group reads
        idx->ptag.bind(s);
        tg = idx->ptag.p;
        rep = db.uniq;
        HIPC(hipMemsetAsync(rep, 0, diag_uniq_words(Nw) * 4, s));
        // the side slot's tag (its key is the empty sentinel: 0) and the tail
        HIPC(hipMemsetAsync(tg + idx->slots() - 1, 0, 33, s));
      } catch (const Error& e) {               // no room for the tags: the first query makes them
        if (e.code != KMHG_ENOMEM) throw;
        (void)hipGetLastError();
        tg = nullptr;
        rep = nullptr;
      }
    }
  }
  LAUNCH("k_v2_bucket_wg", s,
         launch_v2_bucket_wg(kin, pin, start.p, gb, idx->table.p, idx->positions.p, idx->bstats.p,
                             meta, no_pos, s, n_valid, (uint32_t)Nw, bid ? db.code : nullptr, k,
                             aos, tg, rep));
  idx->tags_built = tg != nullptr;
  LAUNCH("k_v2_stats", s, launch_v2_stats(idx->bstats.p, gb.nb, n_valid, meta, idx->rec.meta, s));
  idx->bstats_nb = gb.nb;
  HIPC(hipEventRecord(idx->rec.ev, s));
#ifdef KMHG_STAMPS
  if (const char* f = std::getenv("KMHG_STAMP_FILE")) {
    HIPC(hipStreamSynchronize(s));
    if (FILE* fp = fopen(f, "wb")) { fwrite(stamps, 8, 8 * (size_t)nb, fp); fclose(fp); }
  }
#endif
  // no wait here: the build completes in stream order and finish_build() collects the totals
  idx->pending = true;
  idx->src = d_src;
  return idx.release();
}

// the tag filter of the diagonal query path (per call: tests switch it)
bool tags_on() {
  const char* e = test_build_knob("KMHG_QUERY_TAGS");
  return !(e && e[0] == '0');
}

// The LDS lane-order property the radix ranks rest on (kmhg_build_v2.hip), checked once per
// device before its first partitioned build: where lanes of one returning LDS add that hit the
// same counter are not served in lane order, every build takes the ballot-rank kernels.
// KMHG_TEST_BALLOT=1 (tests) forces them.
static std::atomic<int> g_lane_state[64];          // 0 unchecked, 1 lane order holds, 2 ballots
static std::mutex g_lane_mu;
// The check's stream and result buffer are made once per device and kept: no hipFree (which
// waits for the whole device, stalling work other streams have in flight) and only the check's
// own stream is synchronized.
static void lane_order_run(int blocks, uint64_t* bad, uint64_t* checked) {
  struct Probe {
    hipStream_t st = nullptr;
    unsigned long long* res = nullptr;
  };
  static Probe probes[64];                         // under g_lane_mu (callers hold it)
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  Probe& pr = probes[(unsigned)dev % 64];
  if (!pr.st) HIPC(hipStreamCreateWithFlags(&pr.st, hipStreamNonBlocking));
  if (!pr.res) HIPC(hipMalloc(&pr.res, 2 * sizeof(unsigned long long)));
  unsigned long long h[2] = {0, 0};
  hipError_t e = hipMemsetAsync(pr.res, 0, sizeof(h), pr.st);
  if (e == hipSuccess) {
    launch_lane_order_check(pr.res, pr.st, blocks);
    e = hipMemcpyAsync(h, pr.res, sizeof(h), hipMemcpyDeviceToHost, pr.st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(pr.st);
  hip_check(e, "LDS lane-order check");
  *bad = h[0];
  *checked = h[1];
}
bool lane_ballot() {
  if (const char* e = test_build_knob("KMHG_TEST_BALLOT"))
    if (e[0] == '1') return true;
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  std::atomic<int>& st = g_lane_state[(unsigned)dev % 64];
  int v = st.load(std::memory_order_acquire);
  if (v == 0) {
    std::lock_guard<std::mutex> lk(g_lane_mu);
    v = st.load(std::memory_order_relaxed);
    if (v == 0) {
      uint64_t bad = 0, chk = 0;
      lane_order_run(256, &bad, &chk);
      v = (bad == 0 && chk > 0) ? 1 : 2;
      st.store(v, std::memory_order_release);
    }
  }
  return v == 2;
}

int build_version() {   // read per build so tests can exercise the fallback (KMHG_BUILD=v1)
  const char* e = test_build_knob("KMHG_BUILD");
  return (e && std::string(e) == "v1") ? 1 : 2;
}

// Returns a possibly pending index (partitioned build); finish_build() completes it.
// codes: keep the sequence's code words for the diagonal query path (position indices; a
// count.kmers batch index has no use for them)
kmhg_index* build_device(const uint8_t* d_seq, int64_t L, int k, hipStream_t s, bool codes = true) {
  if (const char* e = test_build_knob("KMHG_DIAG_CODES"))   // tests / A/B: no code block
    if (e[0] == '0') codes = false;
  if (build_version() == 2)
    return build_device_v2(d_seq, L, k, s, nullptr, 0, false, 1, false, codes);
  return build_device_v1(d_seq, L, k, s);
}

// Wait for a pending build and collect its totals.  If a bucket's LDS sub-table overflowed
// (position builds: never observed -- distinct keys per bucket ~ Binomial with mean <= V2_BW;
// count-only builds do not come here), the index is rebuilt
// with the global-atomic build from the retained input.
void finish_build(kmhg_index* idx) {
  if (!idx->pending) return;
  HIPC(hipEventSynchronize(idx->rec.ev));
  const BuildMeta hm = *idx->rec.meta;
  PinnedPool::get().give(idx->rec, false);
  idx->rec = PinnedRec{};
  idx->pending = false;
  const uint8_t* src = idx->src;
  idx->src = nullptr;
  if (hm.overflow) {
    if (idx->is_part) fail(KMHG_EOVERFLOW, "a bucket of a part build overflowed its LDS table");
    std::unique_ptr<kmhg_index> v1(build_device_v1(src, idx->L, idx->k, idx->stream));
    idx->build_kind = KMHG_BUILD_GLOBAL;
    idx->tags_built = false;                     // the tags were the partitioned table's
    idx->bstats_nb = 0;                          // one global bucket: no per-bucket statistics
    idx->fallback = 1;                      // reported by kmhg_index_info (bench.py fails on it)
    idx->geom = v1->geom;
    idx->table.swap_with(v1->table);
    idx->positions.swap_with(v1->positions);
    idx->U = v1->U; idx->N = v1->N; idx->P = v1->P; idx->max_n = v1->max_n;
    v1->table.bind(idx->stream);
    v1->positions.bind(idx->stream);
    return;
  }
  idx->U = hm.n_kmers;
  idx->N = hm.n_positions;
  idx->P = hm.n_pairs;
  idx->max_n = hm.max_count;
}

// ---------------------------------------------------------------------------- query
// Windows [w0, w1) of the query (default: all L - kq + 1).  Rows come out ordered by window
// end, so shards of consecutive window ranges concatenate to the unsharded result.
kmhg_query* query_device(kmhg_index* idx, const uint8_t* d_seq, int64_t L, int kq, int64_t w0,
                         int64_t w1, hipStream_t s, bool part_query = false,
                         bool runs_mode = false) {
  ReleaseGroup rg(s);
  if (idx->canonical) fail(KMHG_EINVAL, "External pointer has incorrect tag");
  if (idx->is_part != part_query)
    fail(KMHG_EINVAL, idx->is_part ? "a part index must be assembled before it is queried"
                                   : "not a part of an owner-computes build");
  finish_build(idx);
  auto q = std::make_unique<kmhg_query>();
  q->device = idx->device;
  q->stream = s;
  idx->stream = s;
  const int64_t Nw = w1 - w0;
  if (Nw <= 0) return q.release();
  const bool aligned = (reinterpret_cast<uintptr_t>(d_seq) & 15) == 0;
  const uint32_t nt = tiles_for(Nw);
  // rows are written into a guessed capacity before the total is known (no host round trip
  // inside the query); a query with more rows than the guess -- heavy repeats -- is redone
  // by the two-pass path into an exact buffer
  uint64_t cap = (uint64_t)Nw + ((uint64_t)Nw >> 3) + 64;
  if (!runs_mode) q->rows.reset(cap);
  // probe / scan / emit.  (A one-pass probe + look-back + emit was measured slower and removed
  // in round 4: config 2 0.403 against 0.365 ms; re-measured round 3 with the diagonal path,
  // self query 94 -> 53 Gbp/s -- a tile that has probed waits for its predecessors' totals
  // while holding its CU slot, and the probe is occupancy / latency bound.)
  uint64_t H = 0;
  // diagonal path (k_query_probe): a position index queried at its own k
  const int64_t nA = idx->L - idx->k + 1;
  const char* de = test_build_knob("KMHG_QUERY_DIAG");
  // (a part query too: its anchors and verified windows count only where the part owns the key,
  // and its tags and repeated-key bits come from its own table, k_query_probe<..., PART>)
  const bool diag_ok = !(de && de[0] == '0') && kq == idx->k && idx->sources == 0 && nA > 0 &&
                       idx->U > 0 && idx->dcodes.p;
  bool diag = diag_ok;
  if (diag && !idx->ps_ready.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(idx->ps_mu);
    if (!idx->ps_ready.load(std::memory_order_relaxed) && !idx->ps_failed) {
      if (!idx->tags_built) {
        try {
          idx->ptag.reset(idx->slots() + 32);  // + the 32-B span the last probe group reads
        } catch (const Error& e) {             // no room for the tags: table probes only
          if (e.code != KMHG_ENOMEM) throw;
          idx->ps_failed = true;
          (void)hipGetLastError();
        }
      }
      if (idx->tags_built) {                   // the build wrote the tags and repeat bits
        idx->dcodes.bind(s);
        const DiagBlock db = idx->diag_block_of();
        LAUNCH("k_diag_valid", s, launch_diag_valid(db.nbit, idx->L, idx->k, db.uniq, true, s));
        HIPC(hipStreamSynchronize(s));
        idx->ps_ready.store(true, std::memory_order_release);
      } else if (!idx->ps_failed) {
        idx->ptag.bind(s);
        idx->dcodes.bind(s);
        const DiagBlock db = idx->diag_block_of();
        LAUNCH("k_diag_prep", s,
               launch_diag_prep(db.nbit, idx->L, idx->k, db.uniq, idx->table.p, idx->slots(),
                                idx->positions.p, idx->ptag.p, s));
        // once per index: later queries may run on other streams
        HIPC(hipStreamSynchronize(s));
        idx->ps_ready.store(true, std::memory_order_release);
      }
    }
  }
  diag = diag && idx->ps_ready.load(std::memory_order_acquire);

  DBuf<uint32_t> qrec(Nw, s);         // per window: 0, the one hit's position, or multi
  DBuf<uint2> qmulti(Nw, s);          // {count, first index}: written for multi-hit windows only
  // per-tile rows -> first row; then the long-scan scratch.  The row total goes straight into
  // pinned host memory (no copy launch before the host reads it).
  DBuf<uint64_t> tiles((size_t)nt + scan_u64_scratch(nt), s);
  uint64_t* tile_row0 = tiles.p;
  DBuf<uint32_t> elist((size_t)nt + 1, s);   // tiles with a multi-hit window; [nt] = their count
  PinnedRec hrec = PinnedPool::get().take();
  GiveBack give_back{hrec, s};
  uint64_t* total = &hrec.meta->n_kmers;
  LAUNCH("k_query_probe", s,
         launch_query_probe(d_seq, L, kq, idx->table.p, idx->geom, qrec.p, qmulti.p, w0, w1, aligned,
                            tile_row0, s, diag ? idx->diag_view() : DiagIdx{nullptr, nullptr, 0},
                            diag && tags_on() ? idx->ptag.p : nullptr, elist.p + nt));
  LAUNCH("k_scan_tiles_u64", s, launch_scan_u64(tile_row0, nt, total, tiles.p + nt, s));
  if (runs_mode) {
    // the rows as diagonal runs, made from the window records (k_qruns_*); rows written only
    // when runs would not be smaller (12 B per run against 8 B per row)
    DBuf<uint64_t> rtiles((size_t)nt + scan_u64_scratch(nt), s);
    PinnedRec hrec2 = PinnedPool::get().take();
    GiveBack give_back2{hrec2, s};
    uint64_t* n_runs = &hrec2.meta->n_kmers;
    LAUNCH("k_qruns_count", s, launch_qruns_count(qrec.p, qmulti.p, (uint64_t)Nw, rtiles.p, s));
    LAUNCH("k_scan_tiles_u64", s, launch_scan_u64(rtiles.p, nt, n_runs, rtiles.p + nt, s));
    HIPC(hipStreamSynchronize(s));
    H = __atomic_load_n(total, __ATOMIC_ACQUIRE);
    const uint64_t NR = __atomic_load_n(n_runs, __ATOMIC_ACQUIRE);
    q->H = (int64_t)H;
    if (H > (uint64_t)INT32_MAX) fail(KMHG_EOVERFLOW, "result has more than 2^31-1 rows");
    if (H && 3 * NR < 2 * H) {
      q->runs.reset(3 * NR);
      q->n_runs = (int64_t)NR;
      LAUNCH("k_qruns_emit", s,
             launch_qruns_emit(qrec.p, qmulti.p, idx->positions.p, (uint64_t)Nw, w0, kq,
                               tile_row0, rtiles.p, NR, q->runs.p, s));
      return q.release();
    }
    cap = std::max<uint64_t>(H, 1);              // the rows, into an exact buffer
    q->rows.reset(cap);
  }
  LAUNCH("k_query_emit", s,
         launch_query_emit(qrec.p, qmulti.p, Nw, w0, kq, idx->positions.p, tile_row0, q->rows.p, cap,
                           elist.p, elist.p + nt, true, s));
  HIPC(hipStreamSynchronize(s));
  H = __atomic_load_n(total, __ATOMIC_ACQUIRE);
  q->H = (int64_t)H;
  if (part_query) {              // the tile offsets stay with the query (the root's merge)
    tiles.bind(s);
    q->tile_off.swap_with(tiles);
    q->n_tiles = nt;
  }
  if (H <= cap) {
    rg.synced = true;                            // nothing queued behind the synchronize
    return q.release();
  }
  q->rows.bind(s);
  q->rows.reset(H);
  LAUNCH("k_query_emit", s,
         launch_query_emit(qrec.p, qmulti.p, Nw, w0, kq, idx->positions.p, tile_row0, q->rows.p, H,
                           elist.p, elist.p + nt, false, s));
  return q.release();
}

void prepare_readout(kmhg_index* idx, hipStream_t s);

// ---------------------------------------------------------------------------- kmer.pairs
// Rows (a, b) for the k-mers both indices hold, a's k-mers in a's kmer.pos row order
// (kmhg_join.hip).  Same two-phase shape as the query: probe + tile totals, one read-back, emit.
kmhg_query* pairs_device(kmhg_index* a, kmhg_index* b, hipStream_t s) {
  ReleaseGroup rg(s);
  if (a->canonical || b->canonical) fail(KMHG_EINVAL, "External pointer has incorrect tag");
  finish_build(a);
  finish_build(b);
  if (a->k != b->k) fail(KMHG_EINVAL, "the two indices must have the same k");
  if (a->device != b->device) fail(KMHG_EINVAL, "the two indices must be on the same device");
  prepare_readout(a, s);
  auto q = std::make_unique<kmhg_query>();
  q->device = a->device;
  q->stream = s;
  a->stream = s;
  b->stream = s;
  const uint32_t Ua = (uint32_t)a->U;
  if (Ua == 0 || b->U == 0) return q.release();
  const uint32_t nt = tiles_for(Ua);
  DBuf<uint4> jinfo(Ua, s);
  DBuf<uint64_t> tiles((size_t)nt + 1 + scan_u64_scratch(nt), s);
  LAUNCH("k_join_probe", s, launch_join_probe(a->canon.perm.p, Ua, a->table.p, b->table.p, b->geom,
                                              jinfo.p, tiles.p, s));
  LAUNCH("k_scan_tiles_u64", s, launch_scan_u64(tiles.p, nt, tiles.p + nt, tiles.p + nt + 1, s));
  uint64_t H = 0;
  HIPC(hipMemcpyAsync(&H, tiles.p + nt, sizeof(H), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  q->H = (int64_t)H;
  q->rows.reset(H);
  if (H)
    LAUNCH("k_join_emit", s, launch_join_emit(jinfo.p, Ua, a->positions.p, b->positions.p, tiles.p,
                                              q->rows.p, s));
  return q.release();
}

// ---------------------------------------------------------------------------- count.kmers
void prepare_canon(kmhg_index* idx, hipStream_t s);

// One count.kmers batch (a device-resident sequence) merged into the counts index `idx`
// (kmhg_count.hip): partitioned build of the batch -> its distinct keys in first-occurrence
// order -> probe / append into the count matrix -> table rebuilt for the grown key list.
struct Release {                   // a batch index dies in stream order
  kmhg_index* b; hipStream_t s;
  ~Release() { b->bind_all(s); }
};

void merge_batch(kmhg_index* idx, kmhg_index* B, uint32_t source, uint64_t base, hipStream_t s);

// Room for `need` rows in the count matrix (grown geometrically: repeated calls amortise the copy).
void reserve_rows(kmhg_index* idx, uint64_t need, hipStream_t s) {
  const uint32_t S = idx->sources;
  const uint64_t U0 = idx->U;
  if (need * S > (uint64_t)INT32_MAX)
    fail(KMHG_EOVERFLOW, "counts index larger than 2^31-1 counts (R vector limit)");
  if (need <= idx->rows_cap) return;
  const uint64_t cap = std::max<uint64_t>(need, idx->rows_cap * 2);
  const bool ord = !idx->canonical;               // count.kmers rows carry order keys
  DBuf<uint64_t> nk(cap), nr(ord ? cap : 0);
  DBuf<int32_t> nm(cap * S);
  if (U0) {
    HIPC(hipMemcpyAsync(nk.p, idx->ckeys.p, U0 * 8, hipMemcpyDeviceToDevice, s));
    HIPC(hipMemcpyAsync(nm.p, idx->positions.p, U0 * S * 4, hipMemcpyDeviceToDevice, s));
    if (ord) HIPC(hipMemcpyAsync(nr.p, idx->rord.p, U0 * 8, hipMemcpyDeviceToDevice, s));
  }
  idx->ckeys.bind(s);
  idx->positions.bind(s);
  idx->rord.bind(s);
  idx->ckeys.swap_with(nk);
  idx->positions.swap_with(nm);
  idx->rord.swap_with(nr);
  idx->rows_cap = cap;
}

// The first batch into an empty counts index or suffix hash: every key is new, the batch table
// becomes the counts table, and its occupied slots are compacted into rows in slot order in one
// pass (k_count_walk) -- no probe, append, table rebuild or C_fix.  count.kmers rows get their
// order keys (base + first position - 1); a suffix hash's rows are order-free.  Returns the
// rows written (B->U, exact, when the batch was built from a sequence).
uint64_t adopt_first_batch(kmhg_index* idx, kmhg_index* B, uint32_t source, uint64_t base,
                           hipStream_t s) {
  ReleaseGroup rg(s);
  const uint32_t S = idx->sources;
  const uint64_t Ub = B->U;
  reserve_rows(idx, Ub, s);
  const bool ord = !idx->canonical;
  const uint64_t ns = B->slots();
  idx->table.bind(s);
  idx->slot_row.bind(s);
  idx->row_slot.bind(s);
  idx->geom = B->geom;
  idx->table.swap_with(B->table);                  // B's release frees the old (empty) table
  idx->slot_row.reset(ns);
  idx->row_slot.reset(Ub);
  const int32_t* bpos = ord ? B->positions.p : nullptr;
  uint64_t* rord = ord ? idx->rord.p : nullptr;
  uint64_t n_new = Ub;
  const char* we = test_build_knob("KMHG_COUNT_WALK");   // "lb": the look-back walk (A/B, tests)
  if (B->bstats_nb == B->geom.nb && B->geom.nb > 0 && !(we && std::string(we) == "lb")) {
    // bucket-aligned tiles, row offsets from the bucket statistics: no look-back chain
    const uint32_t nt = count_walk_b_tiles(B->geom.nb);
    const uint32_t st = tiles_for(nt);
    DBuf<uint32_t> tc(nt + 2, s);                  // tile counts -> offsets; [nt] total, [nt+1] err
    DBuf<uint64_t> status((size_t)st + 1, s);
    HIPC(hipMemsetAsync(status.p, 0, ((size_t)st + 1) * 8, s));
    LAUNCH("k_walk_counts", s,
           launch_walk_counts(B->bstats.p, idx->table.p, idx->geom, tc.p, nt, tc.p + nt + 1, s));
    LAUNCH("k_scan_u32", s, launch_scan_u32(tc.p, nt, status.p, tc.p + nt, s));
    LAUNCH("k_count_walk_b", s,
           launch_count_walk_b(idx->table.p, idx->geom, tc.p, nt, S, source, idx->ckeys.p,
                               idx->positions.p, idx->slot_row.p, idx->row_slot.p, bpos, rord,
                               base, tc.p + nt + 1, s));   // tc: offsets, [nt] = total
    uint32_t h[2] = {0, 0};                        // rows written, consistency flag
    HIPC(hipMemcpyAsync(h, tc.p + nt, 8, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (h[1]) fail(KMHG_EDEVICE, "counts walk: bucket statistics disagree with the table (internal error)");
    n_new = h[0];
  } else {
    const uint64_t nw = count_walk_tiles(ns);
    DBuf<uint64_t> status(nw + 1, s);              // look-back words + the tile ticket
    HIPC(hipMemsetAsync(status.p, 0, (nw + 1) * 8, s));
    LAUNCH("k_count_walk", s,
           launch_count_walk(idx->table.p, ns, status.p,
                             reinterpret_cast<uint32_t*>(status.p + nw), S, source, idx->ckeys.p,
                             idx->positions.p, idx->slot_row.p, idx->row_slot.p, bpos, rord, base,
                             s));
    uint64_t last = 0;                             // the last tile's inclusive prefix
    HIPC(hipMemcpyAsync(&last, status.p + nw - 1, 8, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    n_new = last & ((1ull << 62) - 1);             // LB_MASK: payload of a status word
  }
  idx->U = n_new;
  idx->N = n_new * S;
  idx->P = n_new * ((uint64_t)S * (S - 1) / 2);
  idx->max_n = n_new ? S : 0;
  idx->kmer_count += n_new;
  idx->order_ready = !ord;
  idx->canon.ready = false;
  return n_new;
}

// Adopting a batch table keeps its size, set by the batch's windows / k-mer words; the rebuild
// sizes the table by the distinct keys (~1.5 slots per key).  A batch with heavy repetition
// (deep read coverage) would leave a sparse, oversized table, so adoption needs <= 6 slots per
// distinct key (<= 4x the rebuilt table); otherwise the general merge rebuilds a compact one.
// KMHG_COUNT_TABLE (tests): "adopt" adopts regardless of size, "rebuild" / "probe" never do.
bool adoptable(const kmhg_index* idx, const kmhg_index* B) {
  if (idx->U != 0 || B->u_upper) return false;   // a table sized by a key stream: rebuild
  if (const char* e = test_build_knob("KMHG_COUNT_TABLE")) return std::string(e) == "adopt";
  return B->slots() <= 6 * B->U;
}

void count_device(kmhg_index* idx, const uint8_t* d_seq, int64_t L, uint32_t source,
                  hipStream_t s) {
  ReleaseGroup rg(s);
  idx->stream = s;
  const int k = idx->k;
  if (L <= k) return;
  // the batch keeps its code words only to be eligible for bucket-id radix streams (<= 12 M
  // windows): a larger batch builds on key streams without them (no code block
  // allocated or written for a batch that is discarded after the merge); KMHG_COUNT_BID=0 (A/B)
  // builds every batch with key streams
  const char* cbe = test_build_knob("KMHG_COUNT_BID");
  const bool codes = !(cbe && cbe[0] == '0') && bid_streams_for(L - k + 1);
  std::unique_ptr<kmhg_index> B(build_device(d_seq, L, k, s, codes));
  Release rel{B.get(), s};
  finish_build(B.get());
  B->stream = s;
  if (!B->U) return;
  if (adoptable(idx, B.get()))
    adopt_first_batch(idx, B.get(), source, (uint64_t)idx->L, s);
  else
    merge_batch(idx, B.get(), source, (uint64_t)idx->L, s);
  idx->L += L;                     // the next batch's order keys start here
}

// Merge a batch index B (distinct keys with their counts in the slots) into the counts index,
// B's slots walked in slot order (empty slots skipped).  New keys get rows in that order;
// count.kmers rows get order keys base + first position - 1 (base = characters counted before
// the batch), so ensure_row_order can restore first-insertion order for a readout.
void merge_batch(kmhg_index* idx, kmhg_index* B, uint32_t source, uint64_t base, hipStream_t s) {
  ReleaseGroup rg(s);
  const int k = idx->k;
  const uint32_t S = idx->sources;
  const uint64_t Ub = B->U;
  const uint64_t U0 = idx->U;
  const bool ord = !idx->canonical;
  // KMHG_COUNT_TABLE (tests): "rebuild" / "probe" take the general merge even for the first batch
  const char* ct = test_build_knob("KMHG_COUNT_TABLE");
  if (adoptable(idx, B)) {         // first batch into an empty suffix hash
    adopt_first_batch(idx, B, source, base, s);
    return;
  }
  reserve_rows(idx, U0 + Ub, s);
  const uint64_t ni = B->slots();
  const uint32_t nt = tiles_for(ni);
  DBuf<uint32_t> rank(ni + 1, s);                 // flags -> ranks of the new keys; [ni] = total
  DBuf<uint64_t> status((size_t)nt + 1, s);
  HIPC(hipMemsetAsync(status.p, 0, ((size_t)nt + 1) * 8, s));
  LAUNCH("k_count_probe", s,
         launch_count_probe(nullptr, (uint32_t)ni, B->table.p, U0 ? idx->table.p : nullptr,
                            idx->geom, idx->slot_row.p, S, source, idx->positions.p, rank.p, s));
  LAUNCH("k_scan_u32", s, launch_scan_u32(rank.p, ni, status.p, rank.p + ni, s));
  LAUNCH("k_count_append", s,
         launch_count_append(nullptr, (uint32_t)ni, B->table.p, rank.p, rank.p + ni,
                             (uint32_t)U0, S, source, idx->ckeys.p, idx->positions.p,
                             ord ? B->positions.p : nullptr, ord ? idx->rord.p : nullptr, base,
                             s));
  uint32_t n_new = 0;
  HIPC(hipMemcpyAsync(&n_new, rank.p + ni, 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  const uint64_t U1 = U0 + n_new;
  // rebuild the table for U1 keys (aux of a source_n = 1 index carries the count itself, so
  // even a batch of known keys changes the slots): the partitioned build over the key list,
  // or global linear probing should a bucket overflow (never observed: a key list is distinct)
  idx->table.bind(s);
  idx->slot_row.bind(s);
  idx->row_slot.bind(s);
  // KMHG_COUNT_TABLE=probe: the fallback (tests)
  const bool probe_only = ct && std::string(ct) == "probe";
  std::unique_ptr<kmhg_index> K;
  bool ovf = true;
  if (!probe_only) {
    K.reset(build_device_v2(nullptr, 0, k, s, idx->ckeys.p, (int64_t)U1));
    HIPC(hipEventSynchronize(K->rec.ev));
    ovf = K->rec.meta->overflow != 0;
    PinnedPool::get().give(K->rec, false);
    K->rec = PinnedRec{};
    K->pending = false;
  }
  Release relk{K ? K.get() : B, s};
  idx->row_slot.reset(U1);
  if (!ovf) {
    idx->geom = K->geom;
    idx->table.swap_with(K->table);
    idx->slot_row.reset(idx->slots());
    LAUNCH("k_count_fix", s, launch_count_fix(idx->table.p, idx->slots(), S, idx->positions.p,
                                              idx->slot_row.p, idx->row_slot.p, s));
  } else {
    idx->geom = Geom{1u, (uint32_t)table_capacity((int64_t)U1)};
    idx->table.reset(idx->slots());
    idx->slot_row.reset(idx->slots());
    LAUNCH("k_table_init", s, launch_table_init(idx->table.p, idx->slots(), s));
    LAUNCH("k_count_insert", s,
           launch_count_insert(idx->ckeys.p, (uint32_t)U1, idx->table.p, idx->geom, S,
                               idx->positions.p, idx->slot_row.p, idx->row_slot.p, s));
  }
  idx->U = U1;
  idx->N = U1 * S;
  idx->P = U1 * ((uint64_t)S * (S - 1) / 2);
  idx->max_n = U1 ? S : 0;
  idx->kmer_count += n_new;
  if (ord && n_new) idx->order_ready = false;
  idx->canon.ready = false;
}

// First-insertion order of a count.kmers index's rows (the order of their order keys, rord):
// C_place puts each row's index at F[rord], C_rows compacts F in order into rorder (rank ->
// row).  The rows stay where they are: the readout arrays (k_count_canon) and the export take
// them through rorder.  Run when a readout first asks for rows after a batch.
void ensure_row_order(kmhg_index* idx, hipStream_t s) {
  if (idx->order_ready || idx->canonical || !idx->U) return;
  ReleaseGroup rg(s);
  const uint64_t U = idx->U;
  const int64_t n = idx->L;                       // every order key is < the characters counted
  // F takes 4 B per character ever counted into the pointer (idx->L over all batches), which
  // grows with the input, not with the rows: beyond 8 characters per row (many sources or
  // batches of mostly known k-mers) the rows are ordered by a radix sort of their U order keys
  // instead, O(U) scratch (advisor, round 4).  KMHG_ROW_ORDER_SORT=1 / 0 forces the sort / F
  // (tests: both give the same order).
  const char* rse = test_build_knob("KMHG_ROW_ORDER_SORT");
  const bool by_sort = rse ? rse[0] == '1' : (uint64_t)n > 8 * U;
  if (by_sort) {
    int bits = 1;
    while (bits < 64 && (1ull << bits) < (uint64_t)n) ++bits;
    size_t tb = 0;
    HIPC(rows_sort_temp_bytes((uint32_t)U, bits, &tb));
    DBuf<uint64_t> keys_out(U, s);
    DBuf<uint32_t> rows_in(U, s);
    DBuf<uint8_t> temp(std::max<size_t>(tb, 16), s);
    idx->rorder.bind(s);
    idx->rorder.reset(U);
    hipError_t sort_err = hipSuccess;
    LAUNCH("k_rows_sort", s, sort_err = launch_rows_sort(idx->rord.p, (uint32_t)U, bits,
                                                         keys_out.p, rows_in.p, idx->rorder.p,
                                                         temp.p, tb, s));
    HIPC(sort_err);                 // rorder is not valid unless the sort ran
    idx->order_ready = true;
    return;
  }
  DBuf<uint32_t> F((size_t)n, s);
  HIPC(hipMemsetAsync(F.p, 0xFF, (size_t)n * 4, s));
  LAUNCH("k_rows_place", s, launch_rows_place(idx->rord.p, (uint32_t)U, F.p, s));
  const uint64_t nt = ((uint64_t)n + TILE - 1) / TILE;
  DBuf<uint64_t> status(nt + 1, s);               // look-back words + the tile ticket
  HIPC(hipMemsetAsync(status.p, 0, (nt + 1) * 8, s));
  idx->rorder.bind(s);
  idx->rorder.reset(U);
  LAUNCH("k_rows_order", s,
         launch_rows_order(F.p, n, status.p, reinterpret_cast<uint32_t*>(status.p + nt),
                           idx->rorder.p, s));
  idx->order_ready = true;
}

// rorder of a counts index, or nullptr when its rows are already in order (a suffix hash)
const uint32_t* row_order_of(const kmhg_index* idx) {
  return idx->canonical ? nullptr : idx->rorder.p;
}

// ---------------------------------------------------------------------------- read counting
// count.kmers.fq.sh.rp / seq.kmer.depth.sh / kmer.spec.sh.n (kmhg_sh.hip).  The suffix_hash_n
// of the reference is a counts index of canonical k-mers (canonical = true, sources = counts_n).

// q_to_ll (src/Q_to_log_likelihood.h): -708 below '"', else log(1 - 10^(-(q-33)/10)) printed
// to 15 significant digits -- exactly the doubles the reference's table holds (checked against
// it by tests/golden/make_sh_golden.py), uploaded once per device.
const double* qll_device(hipStream_t s) {
  static std::mutex mu;
  static std::map<int, double*> tables;
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = tables.find(dev);
  if (it != tables.end()) return it->second;
  double h[256];
  for (int q = 0; q < 256; ++q) {
    if (q < 34) { h[q] = -708.0; continue; }
    char buf[64];
    snprintf(buf, sizeof buf, "%.15g", std::log(1.0 - std::pow(10.0, -(double)(q - 33) / 10.0)));
    h[q] = std::strtod(buf, nullptr);
  }
  double* d = static_cast<double*>(DevicePool::get().alloc(sizeof h));
  HIPC(hipMemcpyAsync(d, h, sizeof h, hipMemcpyHostToDevice, s));
  HIPC(hipStreamSynchronize(s));
  tables[dev] = d;
  return d;
}

double qll_host(int q) {   // the same table on the host (the iterator's threshold)
  if (q < 34) return -708.0;
  char buf[64];
  snprintf(buf, sizeof buf, "%.15g", std::log(1.0 - std::pow(10.0, -(double)(q - 33) / 10.0)));
  return std::strtod(buf, nullptr);
}

// The count-only partitioned build of a key stream at `spread` (0: from its HLL estimate),
// waited for.  `overflow`: a bucket's LDS sub-table filled up -- the table is unusable and the
// caller retries at spread 1 (the index still reports the spread and estimate it tried).
// `keys` is a padded stream (EMPTY_KEY entries skipped, k <= 31).
std::unique_ptr<kmhg_index> count_only_build(const uint64_t* keys, uint32_t total, int k,
                                             int spread, hipStream_t s, bool& overflow) {
  std::unique_ptr<kmhg_index> B(
      build_device_v2(nullptr, 0, k, s, keys, (int64_t)total, true, spread, true));
  HIPC(hipEventSynchronize(B->rec.ev));
  const BuildMeta hm = *B->rec.meta;
  PinnedPool::get().give(B->rec, false);
  B->rec = PinnedRec{};
  B->pending = false;
  B->stream = s;
  if (!B->co_spread) B->co_spread = spread;
  overflow = hm.overflow != 0;
  B->U = overflow ? 0 : hm.n_kmers;
  return B;
}

kmhg_index* new_sh_index(int k, int counts_n, hipStream_t s) {
  auto idx = std::make_unique<kmhg_index>();
  HIPC(hipGetDevice(&idx->device));
  idx->k = k;
  idx->sources = (uint32_t)counts_n;
  idx->canonical = true;
  idx->stream = s;
  idx->geom = Geom{1u, 8u};                      // an empty table: lookups before any count
  idx->table.reset(idx->slots());
  LAUNCH("k_table_init", s, launch_table_init(idx->table.p, idx->slots(), s));
  return idx.release();
}

// One batch of packed reads (device-resident) merged into the suffix hash: per-read upper
// bounds (R_ub) -> scan -> R_kmers emit, padded with EMPTY_KEY up to each read's bound ->
// partitioned build of the key stream, padding skipped (occurrence counts per distinct key) ->
// merge over the batch table's slots.  The padding (quality- or N-rejected windows) costs its
// 8 B per window in the build's first pass; the exact count pass it replaces re-walked every
// read and cost a second host round trip (reads leg: see DESIGN.md).
void sh_count_reads_device(kmhg_index* idx, const uint8_t* d_seq, const uint8_t* d_qual,
                           const int64_t* d_off, const uint8_t* d_hasq, uint32_t n_reads,
                           double mean_len, double min_ll, uint32_t source, hipStream_t s) {
  ReleaseGroup rg(s);
  idx->stream = s;
  if (!n_reads) return;
  const int k = idx->k;
  const double* qll = qll_device(s);
  DBuf<uint32_t> cnt((size_t)n_reads + 1, s);
  const uint32_t nt = tiles_for(n_reads);
  DBuf<uint64_t> status((size_t)nt + 2, s);        // scan look-back + ticket, then the span
  HIPC(hipMemsetAsync(status.p, 0, ((size_t)nt + 2) * 8, s));
  uint32_t* d_span = reinterpret_cast<uint32_t*>(status.p + nt + 1);
  LAUNCH("k_rk_span", s, launch_rk_span(d_off, n_reads, d_span, s));
  LAUNCH("k_read_ub", s, launch_read_ub(d_off, n_reads, k, cnt.p, s));
  LAUNCH("k_scan_u32", s, launch_scan_u32(cnt.p, n_reads, status.p, cnt.p + n_reads, s));
  // one round trip for the staging span and the stream length (pinned: the GiveBack returns it)
  PinnedRec hr = PinnedPool::get().take();
  GiveBack hr_back{hr, s};
  HIPC(hipMemcpyAsync(&hr.meta->n_pairs, d_span, 4, hipMemcpyDeviceToHost, s));
  HIPC(hipMemcpyAsync(&hr.meta->max_count, cnt.p + n_reads, 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  const uint32_t span = (uint32_t)__atomic_load_n(&hr.meta->n_pairs, __ATOMIC_ACQUIRE);
  const uint32_t total = __atomic_load_n(&hr.meta->max_count, __ATOMIC_ACQUIRE);
  const char* rkc = test_build_knob("KMHG_RK_CAP");   // A/B knob: LDS bytes per stream (16: global)
  const uint32_t cap = rkc ? (((uint32_t)std::atoi(rkc) + 15) & ~15u) : read_kmers_cap_span(span);
  (void)mean_len;
  if (!total) return;
  DBuf<uint64_t> keys(total, s);
  LAUNCH("k_read_kmers_emit", s,
         launch_read_kmers(d_seq, d_qual, d_off, d_hasq, n_reads, k, min_ll, qll, cap, cnt.p,
                           keys.p, s));
  // The count-only build gives each group bucket `spread` x V2_BW_WG stream entries, so that the
  // batch's distinct keys -- not its key stream -- fill the LDS sub-tables (bench, 3.7x
  // coverage: spread 1/2/3/4 -> 22.6/26.8/28.5/27.6 Gbp/s).  The spread comes from THIS
  // batch's HLL estimate of its distinct keys (build_device_v2, co_spread = 0).
  // KMHG_CO_GLOBAL=1 (tests): straight to the global fallback below
  const bool force_global = test_build_knob("KMHG_CO_GLOBAL") != nullptr;
  std::unique_ptr<kmhg_index> B;
  bool ovf = true;
  int path = 1;
  double est = 0.0;
  int spread = 0;
  if (!force_global) {
    B = count_only_build(keys.p, total, k, 0, s, ovf);
    est = B->co_est;
    spread = B->co_spread;
    if (ovf && spread > 1) {                     // a sub-table overflowed: spread 1 (mean 1024)
      path = 2;
      B->bind_all(s);
      B = count_only_build(keys.p, total, k, 1, s, ovf);
    }
  }
  if (ovf) {                                     // still overflowing: global find-or-insert
    path = 3;
    if (B) B->bind_all(s);
    B = std::make_unique<kmhg_index>();
    HIPC(hipGetDevice(&B->device));
    B->k = k;
    B->stream = s;
    B->geom = Geom{1u, (uint32_t)table_capacity((int64_t)total)};
    B->table.reset(B->slots());
    LAUNCH("k_table_init", s, launch_table_init(B->table.p, B->slots(), s));
    LAUNCH("k_key_count_insert", s,
           launch_key_count_insert(keys.p, total, B->table.p, B->geom, s));
    B->U = total;                                // an upper bound (row capacity only)
    B->u_upper = true;                           // sized by the stream: never adopted
  }
  Release rel{B.get(), s};
  idx->co_est = est;
  idx->co_spread = spread;
  idx->co_path = path;
  if (B->U == 0) return;                         // every window of the batch rejected
  merge_batch(idx, B.get(), source, 0, s);
}

// Host reads packed for the GPU: bases and qualities concatenated, read r = [off[r], off[r+1]).
struct ReadsHost {
  std::vector<uint8_t> seq, qual, hasq;
  std::vector<int64_t> off{0};
  int64_t records = 0;                           // records consumed, short ones included
  void clear() { seq.clear(); qual.clear(); hasq.clear(); off.assign(1, 0); }
  void add(const std::string& sq, const std::string& ql, bool hq) {
    seq.insert(seq.end(), sq.begin(), sq.end());
    if (hq) qual.insert(qual.end(), ql.begin(), ql.end());
    else qual.resize(seq.size(), 0);
    hasq.push_back(hq ? 1 : 0);
    off.push_back((int64_t)seq.size());
  }
  size_t n() const { return hasq.size(); }
};

// Largest base span of one device batch: every per-read window bound is <= its read length, so
// their u32 sum cannot wrap below this.
constexpr uint64_t SH_SPAN_MAX = (uint64_t)UINT32_MAX;

void sh_count_reads_host(kmhg_index* idx, const ReadsHost& r, double min_ll, uint32_t source,
                         hipStream_t s) {
  const size_t n = r.n();
  if (!n) return;
  if (n >= (size_t)UINT32_MAX) fail(KMHG_EOVERFLOW, "more than 2^32-1 reads in one batch");
  const size_t nb = r.seq.size();
  DBuf<uint8_t> dseq(nb + 16, s), dqual(nb + 16, s), dhq(n, s);
  DBuf<int64_t> doff(n + 1, s);
  HIPC(hipMemcpyAsync(dseq.p, r.seq.data(), nb, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(dqual.p, r.qual.data(), nb, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(dhq.p, r.hasq.data(), n, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(doff.p, r.off.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
  // the device pass sizes its key stream by per-read window bounds summed in u32: batches of
  // < SH_SPAN_MAX bases (offsets stay absolute, so a batch is a sub-range of the reads)
  for (size_t i0 = 0; i0 < n;) {
    size_t i1 = i0 + 1;
    while (i1 < n && (uint64_t)(r.off[i1 + 1] - r.off[i0]) < SH_SPAN_MAX) ++i1;
    const uint64_t span = (uint64_t)(r.off[i1] - r.off[i0]);
    if (span >= SH_SPAN_MAX) fail(KMHG_EOVERFLOW, "a read of 2^32 or more bases");
    sh_count_reads_device(idx, dseq.p, dqual.p, doff.p + i0, dhq.p + i0, (uint32_t)(i1 - i0),
                          (double)span / (double)(i1 - i0), min_ll, source, s);
    i0 = i1;
  }
  HIPC(hipStreamSynchronize(s));                 // the host arrays are reused
}

// kmer_reader_read's loop (src/kmer_reader.c:51-73): records up to max_reads, those longer
// than k kept, qualities used when the record has them.  Batches of SH_BATCH bases.
constexpr size_t SH_BATCH = (size_t)256 << 20;

int64_t read_fastx(const char* path, uint64_t max_reads, int k, ReadsHost& r,
                   const std::function<void(ReadsHost&)>& flush) {
  FastxReader rd(path);
  if (!rd.ok()) {   // gzopen failed: the reference's reader then reads nothing
    fprintf(stderr, "kmhg: unable to open %s: nothing counted\n", path);
    return 0;
  }
  std::string sq, ql;
  bool hq = false;
  uint64_t read_n = 0;
  int l;
  while ((l = rd.read(sq, ql, hq)) >= 0 && read_n < max_reads) {
    ++read_n;
    ++r.records;
    if (l <= k) continue;
    r.add(sq, ql, hq);
    if (r.seq.size() >= SH_BATCH && flush) { flush(r); r.clear(); }
  }
  return (int64_t)read_n;
}

void sh_depth_device(kmhg_index* idx, const uint8_t* d_seq, int64_t L, int k, int32_t* d_out,
                     hipStream_t s) {
  ReleaseGroup rg(s);
  idx->stream = s;
  const uint32_t S = idx->sources;
  if (L > 0)
    HIPC(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_out), (int)INT_MIN,
                           (size_t)L * S, s));
  if (L <= 0) return;
  const uint32_t nt = depth_tiles(L);
  DBuf<uint32_t> tcnt((size_t)nt + 1, s);
  const uint32_t ntt = tiles_for(nt);
  DBuf<uint64_t> status((size_t)ntt + 1, s);
  HIPC(hipMemsetAsync(status.p, 0, ((size_t)ntt + 1) * 8, s));
  LAUNCH("k_depth_seg_count", s, launch_depth_seg_count(d_seq, L, tcnt.p, s));
  LAUNCH("k_scan_u32", s, launch_scan_u32(tcnt.p, nt, status.p, tcnt.p + nt, s));
  uint32_t M = 0;
  HIPC(hipMemcpyAsync(&M, tcnt.p + nt, 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  DBuf<uint32_t> seg((size_t)2 * M + 2, s);
  DBuf<uint8_t> stale((size_t)M + 1, s);
  uint32_t* sstart = seg.p;
  uint32_t* send = seg.p + M + 1;
  if (M) LAUNCH("k_depth_seg_emit", s, launch_depth_seg_emit(d_seq, L, tcnt.p, sstart, send, s));
  LAUNCH("k_depth_modes", s,
         launch_depth_modes(d_seq, L, k, sstart, send, tcnt.p + nt, stale.p, idx->table.p,
                            idx->geom, S, idx->positions.p, d_out, s));
  if (M)
    LAUNCH("k_depth_probe", s,
           launch_depth_probe(d_seq, L, k, sstart, send, tcnt.p + nt, stale.p, idx->table.p,
                              idx->geom, S, idx->positions.p, d_out, s));
}

void check_sh(const kmhg_index* idx) {
  if (!idx || !idx->canonical)
    fail(KMHG_EINVAL, "unable to obtain suffix_hash_n from external pointer");
}

// ---------------------------------------------------------------------------- readout
void prepare_canon(kmhg_index* idx, hipStream_t s) {
  ReleaseGroup rg(s);
  idx->stream = s;
  Canon& c = idx->canon;
  if (c.ready) return;
  if (idx->sources) {            // counts index: rows in first-insertion order (ensure_row_order)
    ensure_row_order(idx, s);
    const uint32_t U = (uint32_t)idx->U, S = idx->sources;
    c.perm.reset(U);
    c.canon_off.reset(U + 1);
    c.pkeys.reset(S >= 2 ? U : 1);
    c.pair_off.reset(S >= 2 ? U : 1);
    c.rinfo.reset(U);
    LAUNCH("k_count_canon", s, launch_count_canon(row_order_of(idx), idx->row_slot.p,
                                                  idx->positions.p, U, S, c.perm.p,
                                                  c.canon_off.p, c.pkeys.p, c.pair_off.p,
                                                  c.rinfo.p, s));
    c.n_multi = S >= 2 ? U : 0;
    c.ready = true;
    return;
  }
  const int64_t L = idx->L;
  const uint32_t U = (uint32_t)idx->U;
  DBuf<uint2> F(L, s);
  HIPC(hipMemsetAsync(F.p, 0xFF, (size_t)L * 8, s));
  if (U) LAUNCH("k_read_first", s, launch_read_first(idx->table.p, idx->slots(), idx->positions.p,
                                                     F.p, s));
  const uint32_t nt = tiles_for(L);
  const size_t scratch_bytes = (size_t)nt * 24 + 64 + sizeof(ReadMeta);
  DBuf<uint8_t> scratch(scratch_bytes, s);
  HIPC(hipMemsetAsync(scratch.p, 0, scratch_bytes, s));
  uint64_t* st_a = reinterpret_cast<uint64_t*>(scratch.p);
  uint64_t* st_b = st_a + nt;
  uint64_t* st_c = st_b + nt;
  uint32_t* ticket = reinterpret_cast<uint32_t*>(scratch.p + (size_t)nt * 24);
  ReadMeta* rm = reinterpret_cast<ReadMeta*>(scratch.p + (size_t)nt * 24 + 64);
  c.perm.reset(U);
  c.canon_off.reset(U + 1);
  c.rinfo.reset(U);
  // keys with >= 2 positions: at most N/2
  c.pkeys.reset(idx->N / 2 + 1);
  c.pair_off.reset(idx->N / 2 + 1);
  LAUNCH("k_read_order", s,
         launch_read_order(F.p, L, idx->table.p, st_a, st_b, st_c, ticket, c.perm.p,
                           c.canon_off.p, c.pkeys.p, c.pair_off.p, c.rinfo.p, rm, s));
  ReadMeta h;
  HIPC(hipMemcpyAsync(&h, rm, sizeof(h), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (h.n_keys != idx->U || h.n_rows != idx->N || h.n_pairs != idx->P)
    fail(KMHG_EDEVICE, "readout order inconsistent with the index (internal error)");
  c.n_multi = h.n_multi;
  c.ready = true;
}

// Readout arrays for idx->row_order.  The first-occurrence arrays are built on the GPU
// (prepare_canon); the khash order relabels them: the keys go to the host once, the bucket
// order is replayed there (inherently sequential, ~0.1 us per key), and the permuted arrays
// come back.  The readout kernels then run unchanged.
void prepare_readout(kmhg_index* idx, hipStream_t s) {
  ReleaseGroup rg(s);
  finish_build(idx);
  Canon& c = idx->canon;
  if (c.ready && c.order == idx->row_order) return;
  if (c.ready && c.order != KMHG_ORDER_FIRST) c.ready = false;   // rebuild from first order
  prepare_canon(idx, s);
  c.order = KMHG_ORDER_FIRST;
  if (idx->row_order == KMHG_ORDER_FIRST) return;
  const uint32_t U = (uint32_t)idx->U;
  std::vector<uint64_t> keys(U);
  std::vector<uint32_t> perm(U);
  std::vector<uint2> info(U);
  if (U) {
    DBuf<uint64_t> dk(U, s);
    LAUNCH("k_gather_keys", s, launch_gather_keys(c.perm.p, U, idx->table.p, dk.p, s));
    HIPC(hipMemcpyAsync(keys.data(), dk.p, (size_t)U * 8, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(info.data(), c.rinfo.p, (size_t)U * 8, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(perm.data(), c.perm.p, (size_t)U * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
  }
  const std::vector<uint32_t> order = khash_bucket_order(keys);
  if (order.size() != U) fail(KMHG_EDEVICE, "khash order replay lost keys (internal error)");
  std::vector<uint32_t> perm_k(U), off_k(U + 1), pkeys;
  std::vector<uint2> info_k(U);
  std::vector<uint64_t> pair_off;
  uint64_t rows = 0, pairs = 0;
  for (uint32_t r = 0; r < U; ++r) {
    const uint32_t id = order[r];
    const uint64_t n = (uint64_t)info[id].x;
    perm_k[r] = perm[id];
    info_k[r] = info[id];
    off_k[r] = (uint32_t)rows;
    rows += n;
    if (n >= 2) {
      pkeys.push_back(r);
      pair_off.push_back(pairs);
      pairs += n * (n - 1) / 2;
    }
  }
  off_k[U] = (uint32_t)rows;
  if (rows != idx->N || pairs != idx->P || pkeys.size() != c.n_multi)
    fail(KMHG_EDEVICE, "khash readout order inconsistent with the index (internal error)");
  if (U) {
    HIPC(hipMemcpyAsync(c.perm.p, perm_k.data(), (size_t)U * 4, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(c.rinfo.p, info_k.data(), (size_t)U * 8, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(c.canon_off.p, off_k.data(), (size_t)(U + 1) * 4, hipMemcpyHostToDevice, s));
  }
  if (!pkeys.empty()) {
    HIPC(hipMemcpyAsync(c.pkeys.p, pkeys.data(), pkeys.size() * 4, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(c.pair_off.p, pair_off.data(), pair_off.size() * 8,
                        hipMemcpyHostToDevice, s));
  }
  HIPC(hipStreamSynchronize(s));   // host vectors die here
  c.order = KMHG_ORDER_KHASH;
}

void positions_sizes(kmhg_index* idx, uint32_t opt, int64_t* nk, int64_t* np, int64_t* npp,
                     int64_t* nc) {
  if (idx->canonical) fail(KMHG_EINVAL, "External pointer has incorrect tag");
  if (nk) *nk = (opt & KMHG_OPT_KMER) ? (int64_t)idx->U : 0;
  if (np) *np = (opt & KMHG_OPT_POS) ? (int64_t)idx->N : 0;
  if (npp) *npp = (opt & KMHG_OPT_PAIRS) ? (int64_t)idx->P : 0;
  if (nc) *nc = (opt & KMHG_OPT_COUNT) ? (int64_t)idx->U : 0;
}

void positions_device(kmhg_index* idx, uint32_t opt, char* kmers, int32_t* pos, int32_t* pairs,
                      int32_t* counts, hipStream_t s) {
  ReleaseGroup rg(s);
  if (idx->canonical) fail(KMHG_EINVAL, "External pointer has incorrect tag");
  if (idx->is_part) fail(KMHG_EINVAL, "a part index must be assembled before it is read");
  prepare_readout(idx, s);
  Canon& c = idx->canon;
  const uint32_t U = (uint32_t)idx->U;
  if ((opt & (KMHG_OPT_KMER | KMHG_OPT_COUNT)) && U)
    LAUNCH("k_read_keys", s,
           launch_read_keys(c.perm.p, c.rinfo.p, U, idx->table.p, idx->k,
                            (opt & KMHG_OPT_COUNT) ? counts : nullptr,
                            (opt & KMHG_OPT_KMER) ? kmers : nullptr, s));
  if ((opt & KMHG_OPT_POS) && idx->N) {
    DBuf<uint32_t> tile_key((size_t)read_pos_tiles(idx->N) + 1, s);
    LAUNCH("k_read_pos", s,
           launch_read_pos(c.rinfo.p, c.canon_off.p, U, idx->N, idx->positions.p, tile_key.p,
                           reinterpret_cast<int2*>(pos), s));
  }
  if ((opt & KMHG_OPT_PAIRS) && idx->P) {
    DBuf<uint32_t> tile_key((size_t)read_pairs_tiles(idx->P) + 1, s);
    LAUNCH("k_read_pairs", s,
           launch_read_pairs(c.pkeys.p, c.pair_off.p, (uint32_t)c.n_multi, idx->P, c.rinfo.p,
                             idx->positions.p, tile_key.p, pairs, s));
  }
}

// ------------------------------------------------------------------ multi-device seq.kmer.pos
// KMHG_DEVICES=d0,d1,... (SURVEY.md §5 "Config / flags"): the host-pointer seq.kmer.pos of the
// R API (.Call("sequence_kmer_positions"), src/kmer_hash.c:1151-1172) is split over these
// devices in one process, with the R signatures unchanged.  The index is replicated once per
// device by peer copies over xGMI (the image: table + positions + code block), the query's
// windows are cut into contiguous ranges (the multi-GPU shard unit of
// kmhg_query_run_device_range), each device receives only its range's slice of the host
// sequence (plus the neighbour chars the window rule reads) and queries it on its own host
// thread, and the rows stay in each device's HBM until kmhg_query_fill copies every part
// straight into the caller's buffer at its prefix offset.  Concatenation in range order is the
// unsharded row order.
void free_index(kmhg_index* idx);
void free_query(kmhg_query* q);

// the bucket holding the side slot's key ~0 (bucket_of(mix64(~0), nb), kmhg_device.h) on the host
uint32_t side_bucket_of(uint32_t nb) {
  return (uint32_t)(((unsigned __int128)mix64(EMPTY_KEY) * nb) >> 64);
}

std::vector<int> query_devices() {
  std::vector<int> out;
  const char* e = std::getenv("KMHG_DEVICES");
  if (!e || !*e) return out;
  int n = 0;
  HIPC(hipGetDeviceCount(&n));
  const std::string str(e);
  size_t a = 0;
  while (a <= str.size()) {
    size_t b = str.find(',', a);
    if (b == std::string::npos) b = str.size();
    const std::string tok = str.substr(a, b - a);
    char* end = nullptr;
    const long d = std::strtol(tok.c_str(), &end, 10);
    if (tok.empty() || *end || d < 0 || d >= n)
      fail(KMHG_EINVAL, "KMHG_DEVICES must list device ordinals (0.." + std::to_string(n - 1) +
                            "), got \"" + str + "\"");
    out.push_back((int)d);
    a = b + 1;
  }
  return out;
}

// A copy of `home` on device `dev`, by peer copies (hipMemcpyPeerAsync: xGMI between MI355X
// GPUs; a same-device copy when dev is home's own device).  Its diagonal-path bits and slot
// tags are derived by its own first query, as for an imported image.
kmhg_index* make_replica(kmhg_index* home, int dev) {
  auto r = std::make_unique<kmhg_index>();
  r->device = dev;
  r->k = home->k; r->L = home->L; r->geom = home->geom;
  r->U = home->U; r->N = home->N; r->P = home->P; r->max_n = home->max_n;
  r->kmer_count = home->kmer_count;
  r->row_order = home->row_order;
  DeviceGuard g(dev);
  hipStream_t s = lib_stream();
  r->stream = s;
  r->table.reset(home->slots());
  HIPC(hipMemcpyPeerAsync(r->table.p, dev, home->table.p, home->device,
                          home->slots() * sizeof(Slot), s));
  if (home->N) {
    r->positions.reset(home->N);
    HIPC(hipMemcpyPeerAsync(r->positions.p, dev, home->positions.p, home->device, home->N * 4,
                            s));
  }
  if (home->dcodes.p) {
    const uint64_t w = diag_block_words(home->L - home->k + 1);
    r->dcodes.reset(w);
    HIPC(hipMemcpyPeerAsync(r->dcodes.p, dev, home->dcodes.p, home->device, w * 8, s));
  }
  HIPC(hipStreamSynchronize(s));
  return r.release();
}

// The index's copy on device `dev` (one per device, shared by every query part that runs
// there; made on first use, freed with the index).
kmhg_index* replica_on(kmhg_index* home, int dev) {
  {
    std::lock_guard<std::mutex> lk(home->rep_mu);
    auto it = home->replicas.find(dev);
    if (it != home->replicas.end()) return it->second;
  }
  kmhg_index* r = make_replica(home, dev);          // outside the lock: devices copy in parallel
  std::lock_guard<std::mutex> lk(home->rep_mu);
  auto& slot = home->replicas[dev];
  if (slot) {                                       // another thread made it meanwhile
    free_index(r);
    return slot;
  }
  slot = r;
  return r;
}

kmhg_query* query_multi_device(kmhg_index* idx, const char* seq, int64_t L, int k,
                               const std::vector<int>& devs) {
  {
    DeviceGuard g(idx->device);
    finish_build(idx);
    if (idx->canonical) fail(KMHG_EINVAL, "External pointer has incorrect tag");
  }
  const int G = (int)devs.size();
  const int64_t Nw = L - k + 1;
  auto q = std::make_unique<kmhg_query>();
  q->device = idx->device;
  std::vector<kmhg_query*> parts(G, nullptr);
  std::vector<Error> errs(G, Error{KMHG_OK, ""});
  const bool poison = test_build_knob("KMHG_SLICE_POISON") != nullptr;   // tests: garbage outside
  // tests: parts after the first on the index's own device use a same-device replica, so the
  // copy path runs on a one-GPU box too
  const bool test_replica = test_build_knob("KMHG_TEST_REPLICA") != nullptr;
  auto run = [&](int i) {
    try {
      const int64_t w0 = Nw * i / G, w1 = Nw * (i + 1) / G;
      const bool home = devs[i] == idx->device && !(test_replica && i > 0);
      kmhg_index* use = home ? idx : replica_on(idx, devs[i]);
      DeviceGuard g(devs[i]);
      hipStream_t s = lib_stream();
      // a full-length buffer holding only chars [a, b): the window rule of windows [w0, w1)
      // reads chars [w0 - 1, w1 + k - 1); the tile stage's aligned loads and halo read a few
      // more around them, which feed only windows outside the range
      const int64_t a = std::max<int64_t>(0, (w0 & ~15ll) - 64);
      const int64_t b = std::min<int64_t>(L, w1 + k + 64);
      DBuf<uint8_t> d((size_t)L + 16, s);
      if (poison) HIPC(hipMemsetAsync(d.p, 'A', (size_t)L + 16, s));
      if (b > a) h2d_host(d.p + a, seq + a, (size_t)(b - a), s);
      parts[i] = query_device(use, d.p, L, k, w0, w1, s);
      HIPC(hipStreamSynchronize(s));
    } catch (const Error& e) {
      errs[i] = e;
    } catch (const std::bad_alloc&) {
      errs[i] = Error{KMHG_ENOMEM, "host allocation failed"};
    }
  };
  // one host thread per distinct device; the parts of one device run in order on its thread
  // (they share that device's stream and index copy)
  std::vector<int> uniq;
  for (int d : devs)
    if (std::find(uniq.begin(), uniq.end(), d) == uniq.end()) uniq.push_back(d);
  auto run_device = [&](int d) {
    for (int i = 0; i < G; ++i)
      if (devs[i] == d) run(i);
  };
  std::vector<std::thread> th;
  for (size_t u = 1; u < uniq.size(); ++u) th.emplace_back(run_device, uniq[u]);
  run_device(uniq[0]);
  for (auto& t : th) t.join();
  q->parts = parts;                                  // freed with q, also on the error path
  for (int i = 0; i < G; ++i)
    if (errs[i].code != KMHG_OK) {
      free_query(q.release());
      fail(errs[i].code, errs[i].msg);
    }
  int64_t off = 0;
  for (auto* p : parts) {
    q->part_off.push_back(off);
    off += p->H;
  }
  q->H = off;
  return q.release();
}

// The rows of a multi-device query on its home device (peer copies, once), for the readers
// that want one device buffer (kmhg_query_rows_device).
void gather_parts(kmhg_query* q) {
  if (q->parts.empty() || q->gathered) return;
  DeviceGuard g(q->device);
  hipStream_t s = lib_stream();
  q->rows.reset((size_t)std::max<int64_t>(q->H, 1));
  for (size_t i = 0; i < q->parts.size(); ++i)
    if (q->parts[i]->H)
      HIPC(hipMemcpyPeerAsync(q->rows.p + q->part_off[i], q->device, q->parts[i]->rows.p,
                              q->parts[i]->device, (size_t)q->parts[i]->H * 8, s));
  HIPC(hipStreamSynchronize(s));
  q->stream = s;
  q->gathered = true;
}

void free_query(kmhg_query* q) {
  if (!q) return;
  for (auto* p : q->parts) free_query(p);
  DeviceGuard g(q->device);
  // the caller keeps its stream alive until here (a multi-device query's own rows exist only
  // once gathered, on the library stream)
  if (q->parts.empty() || q->gathered) HIPC(hipStreamSynchronize(q->stream));
  q->rows.ordered = false;                 // its stream is idle: straight back to the pool
  delete q;
}

void free_index(kmhg_index* idx) {
  if (!idx) return;
  for (auto& kv : idx->replicas) free_index(kv.second);
  idx->replicas.clear();
  DeviceGuard g(idx->device);
  if (idx->pending) {                  // never used: no need to wait, the record is recycled
    PinnedPool::get().give(idx->rec, true);   // once the build's event has completed
    idx->pending = false;
  }
  // stream-ordered release: the buffers return to the pool once work queued on the index's
  // last stream has finished (queries on other streams are synchronised by their callers)
  ReleaseGroup rg(idx->stream);
  idx->bind_all(idx->stream);
  delete idx;
}

}  // namespace

bool kmhg::ballot_ranks() { return lane_ballot(); }

// ============================================================================ C-ABI
extern "C" {

const char* kmhg_last_error(void) { return g_err.c_str(); }
int kmhg_version(void) { return 1; }

int kmhg_build(const char* seq, size_t L, int k, int do_sort, kmhg_index** out) {
  (void)do_sort;
  return guarded([&] {
    if (!seq || !out) fail(KMHG_EINVAL, "null argument");
    // small or refused strings: the C length and the checks before anything touches the device
    if (L < H2D_SCAN_MIN || k < 1 || k > 32 || L >= (size_t)INT32_MAX) {
      L = effective_len(seq, L);
      check_build_args(L, k);
    }
    hipStream_t s = lib_stream();
    DBuf<uint8_t> d(L + 16, s);
    L = h2d_cstring(d.p, seq, L, s);
    check_build_args(L, k);
    std::unique_ptr<kmhg_index> idx(build_device(d.p, (int64_t)L, k, s));
    finish_build(idx.get());   // synchronous, like make_kmer_h_index (and d dies here)
    *out = idx.release();
  });
}

int kmhg_build_device(const void* d_seq, size_t L, int k, int do_sort, void* stream,
                      kmhg_index** out) {
  (void)do_sort;
  return guarded([&] {
    if (!d_seq || !out) fail(KMHG_EINVAL, "null argument");
    check_build_args(L, k);
    hipStream_t s = (hipStream_t)stream;   // caller stream; NULL = HIP null stream
    *out = build_device((const uint8_t*)d_seq, (int64_t)L, k, s);
  });
}

int kmhg_build_device_part(const void* d_seq, size_t L, int k, int part, int n_parts,
                           void* stream, kmhg_index** out) {
  return guarded([&] {
    if (!d_seq || !out) fail(KMHG_EINVAL, "null argument");
    check_build_args(L, k);
    if (n_parts < 1 || part < 0 || part >= n_parts) fail(KMHG_EINVAL, "part out of range");
    if (const char* e = test_build_knob("KMHG_BUILD"))
      if (std::string(e) == "v1") fail(KMHG_EINVAL, "part builds need the partitioned build");
    hipStream_t s = (hipStream_t)stream;
    *out = build_device_v2((const uint8_t*)d_seq, (int64_t)L, k, s, nullptr, 0, false, 1, false,
                           true, (uint32_t)part, (uint32_t)n_parts);
  });
}

int kmhg_part_info(kmhg_index* idx, int64_t info[10]) {
  return guarded([&] {
    if (!idx || !info) fail(KMHG_EINVAL, "null argument");
    if (!idx->is_part) fail(KMHG_EINVAL, "not a part index");
    DeviceGuard g(idx->device);
    finish_build(idx);
    const Geom& G = idx->geom;
    const uint32_t side_b = side_bucket_of(G.nbh);
    info[0] = G.b0;
    info[1] = G.nb;
    info[2] = G.nbh;
    info[3] = G.capb;
    info[4] = (int64_t)idx->N;
    info[5] = (int64_t)idx->U;
    info[6] = (int64_t)idx->P;
    info[7] = idx->max_n;
    info[8] = (G.nb && side_b >= G.b0 && side_b < G.b0 + G.nb) ? 1 : 0;
    info[9] = idx->dcodes.p ? (int64_t)(diag_block_words(idx->L - idx->k + 1) * 8) : 0;
  });
}

int kmhg_part_export(kmhg_index* idx, int64_t pos_base, void* d_table, void* d_side_slot,
                     void* d_positions, void* d_codes, void* stream) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    if (!idx->is_part) fail(KMHG_EINVAL, "not a part index");
    if (pos_base < 0 || pos_base + (int64_t)idx->N > (int64_t)UINT32_MAX)
      fail(KMHG_EINVAL, "position base out of range");
    DeviceGuard g(idx->device);
    finish_build(idx);
    hipStream_t s = (hipStream_t)stream;
    const uint64_t n = (uint64_t)idx->geom.nb * idx->geom.capb;
    if (d_table && n)
      LAUNCH("k_part_rebase", s,
             launch_part_rebase(idx->table.p, static_cast<Slot*>(d_table), n,
                                (uint32_t)pos_base, s));
    if (d_side_slot && idx->geom.nb)
      LAUNCH("k_part_rebase", s,
             launch_part_rebase(idx->table.p + n, static_cast<Slot*>(d_side_slot), 1,
                                (uint32_t)pos_base, s));
    if (d_positions && idx->N)
      HIPC(hipMemcpyAsync(d_positions, idx->positions.p, idx->N * 4, hipMemcpyDeviceToDevice, s));
    if (d_codes && idx->dcodes.p)
      HIPC(hipMemcpyAsync(d_codes, idx->dcodes.p, diag_block_words(idx->L - idx->k + 1) * 8,
                          hipMemcpyDeviceToDevice, s));
    HIPC(hipStreamSynchronize(s));
  });
}

int kmhg_free(kmhg_index* idx) {
  return guarded([&] { free_index(idx); });
}

// count.kmers: windows never span two sequences of the character vector, so a batch is the
// sequences joined by 'N'.  Alone, a sequence's final N-free run of exactly k chars yields no
// window (init_kmer reaches the string's end, src/kmer_hash.c:235-237); followed by the 'N' it
// would, so such a run is left out of the batch.
constexpr size_t COUNT_BATCH = (size_t)1 << 30;   // chars per build

kmhg_index* new_counts_index(int k, int source_n) {
  auto idx = std::make_unique<kmhg_index>();
  HIPC(hipGetDevice(&idx->device));
  idx->k = k;
  idx->sources = (uint32_t)source_n;
  idx->stream = lib_stream();
  return idx.release();
}

void check_count_args(int64_t n_seqs, int k, int source, int source_n, kmhg_index* c) {
  // count_kmers, src/kmer_hash.c:549-563 and 579-581 (same order, same texts)
  if (n_seqs < 1) fail(KMHG_EINVAL, "seq_r should be a character vector of length at least one");
  if (k < 1 || k > 32) fail(KMHG_EINVAL, "k must be a positive integer less than 1+MAX_K");
  if (source_n < 1 || source >= source_n)
    fail(KMHG_EINVAL, "source_n must be larger than 1 and larger than source");
  if (!c) return;
  if (!c->sources || c->canonical)
    fail(KMHG_EINVAL, "count.kmers needs a counts pointer (one made by count.kmers)");
  if (c->k != k)
    fail(KMHG_EINVAL, "mismatch between specified k and that given in the external pointer");
  if ((uint32_t)source_n != c->sources)
    fail(KMHG_EINVAL, "source_n differs from the source_n the counts pointer was made with");
}

int kmhg_count(kmhg_index** idx, const char* const* seqs, const size_t* lens, int64_t n_seqs,
               int k, int source, int source_n) {
  return guarded([&] {
    if (!idx || (n_seqs > 0 && (!seqs || !lens))) fail(KMHG_EINVAL, "null argument");
    check_count_args(n_seqs, k, source, source_n, *idx);
    std::unique_ptr<kmhg_index> fresh;
    kmhg_index* c = *idx;
    if (!c) {
      fresh.reset(new_counts_index(k, source_n));
      c = fresh.get();
    }
    DeviceGuard g(c->device);
    if (source >= 0) {   // negative: every insert fails its source check, nothing is counted
      hipStream_t s = lib_stream();
      std::vector<char> buf;
      auto flush = [&] {
        if (buf.empty()) return;
        if (buf.size() >= (size_t)INT32_MAX)
          fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1 (int positions)");
        DBuf<uint8_t> d(buf.size() + 16, s);
        HIPC(hipMemcpyAsync(d.p, buf.data(), buf.size(), hipMemcpyHostToDevice, s));
        count_device(c, d.p, (int64_t)buf.size(), (uint32_t)source, s);
        HIPC(hipStreamSynchronize(s));   // buf is reused
        buf.clear();
      };
      for (int64_t i = 0; i < n_seqs; ++i) {
        const char* q = seqs[i];
        if (!q) continue;
        size_t n = effective_len(q, lens[i]);
        if ((int64_t)n <= k) continue;                  // src/kmer_hash.c:583-584
        bool tail_k = LCN(q[n - k - 1]);                // final run of exactly k chars?
        for (size_t j = n - k; tail_k && j < n; ++j) tail_k = !LCN(q[j]);
        if (tail_k) n -= (size_t)k;
        if (!buf.empty() && buf.size() + n + 1 > COUNT_BATCH) flush();
        buf.insert(buf.end(), q, q + n);
        buf.push_back('N');
      }
      flush();
    }
    if (fresh) *idx = fresh.release();
  });
}

int kmhg_count_device(kmhg_index** idx, const void* d_seq, size_t L, int k, int source,
                      int source_n, void* stream) {
  return guarded([&] {
    if (!idx || (L && !d_seq)) fail(KMHG_EINVAL, "null argument");
    check_count_args(1, k, source, source_n, *idx);
    if (L >= (size_t)INT32_MAX) fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1 (int positions)");
    std::unique_ptr<kmhg_index> fresh;
    kmhg_index* c = *idx;
    if (!c) {
      fresh.reset(new_counts_index(k, source_n));
      c = fresh.get();
    }
    DeviceGuard g(c->device);
    if (source >= 0) count_device(c, (const uint8_t*)d_seq, (int64_t)L, (uint32_t)source,
                                  (hipStream_t)stream);
    if (fresh) *idx = fresh.release();
  });
}

// ---------------------------------------------------------------- suffix hash (read counting)
// count_kmers_fastq_sh_rp (src/kmer_hash.c:810-857): argument checks in the reference's order
// and with its texts; the remaining deviations are undefined-behaviour paths of the reference.
static void check_sh_params(const int32_t* p) {
  const int k = p[0];
  const uint32_t source_n = (uint32_t)p[6], source_i = (uint32_t)p[7];
  if (k < 1 || k > 32) fail(KMHG_EINVAL, "k must be a positive integer less than 1+MAX_K");
  if (source_n > 4 || source_n < 1) fail(KMHG_EINVAL, "Source_n must be in the range 1 - 4");
  if (source_i >= source_n) fail(KMHG_EINVAL, "source_i must be less than source_n");
  // k = 32: the reference's (1 << 2k) - 1 masks shift by 64 (undefined); prefix_bits > 2k with
  // k < 16 makes its suffix/prefix split underflow (src/kmer_reader.c:84-92)
  if (k == 32) fail(KMHG_EINVAL, "k must be at most 31 for the suffix hash");
  uint32_t pb = (uint32_t)p[1];
  if (pb > 36) pb = 36;
  if (2 * (uint32_t)k < 32 && pb > 2 * (uint32_t)k)
    fail(KMHG_EINVAL, "prefix_bits must not exceed 2k");
}

struct kmhg_reads {
  ReadsHost r;
};

// Into an existing suffix hash the reference checks k and source (src/kmer_reader.c:118-126):
// a mismatch prints a message and counts nothing.
static bool sh_accepts(const kmhg_index* sh, int k, uint32_t source) {
  if ((int)sh->k != k) {
    fprintf(stderr, "Incompatible arguments: k and total bit numbers do not add up\n");
    return false;
  }
  if (source >= sh->sources) {
    fprintf(stderr, "Value of source is too large\n");
    return false;
  }
  return true;
}

int kmhg_sh_count_fastq(kmhg_index** sh, const char* path, const int32_t params[8]) {
  return guarded([&] {
    if (!sh || !path || !params) fail(KMHG_EINVAL, "null argument");
    if (*sh) check_sh(*sh);
    check_sh_params(params);
    const int k = params[0];
    const double min_ll = qll_host((unsigned char)('!' + (unsigned char)params[2]));
    const uint64_t max_reads = (uint64_t)(int64_t)params[4];   // (size_t) of an int
    const uint32_t source = (uint32_t)params[7];
    hipStream_t s = lib_stream();
    std::unique_ptr<kmhg_index> fresh;
    kmhg_index* c = *sh;
    if (!c) {
      fresh.reset(new_sh_index(k, params[6], s));
      c = fresh.get();
    } else if (!sh_accepts(c, k, source)) {
      return;
    }
    DeviceGuard g(c->device);
    ReadsHost r;
    read_fastx(path, max_reads, k, r, [&](ReadsHost& b) {
      sh_count_reads_host(c, b, min_ll, source, s);
      c->L += (int64_t)b.seq.size();
    });
    sh_count_reads_host(c, r, min_ll, source, s);
    c->L += (int64_t)r.seq.size();
    if (fresh) *sh = fresh.release();
  });
}

int kmhg_fastx_read(const char* path, int64_t max_reads, int k, kmhg_reads** out) {
  return guarded([&] {
    if (!path || !out) fail(KMHG_EINVAL, "null argument");
    auto r = std::make_unique<kmhg_reads>();
    read_fastx(path, (uint64_t)max_reads, k, r->r, nullptr);
    *out = r.release();
  });
}

int kmhg_reads_info(const kmhg_reads* r, int64_t* n_records, int64_t* n_reads,
                    int64_t* n_bases) {
  return guarded([&] {
    if (!r) fail(KMHG_EINVAL, "null argument");
    if (n_records) *n_records = r->r.records;
    if (n_reads) *n_reads = (int64_t)r->r.n();
    if (n_bases) *n_bases = (int64_t)r->r.seq.size();
  });
}

int kmhg_reads_copy(const kmhg_reads* r, uint8_t* seq, uint8_t* qual, int64_t* offsets,
                    uint8_t* has_qual) {
  return guarded([&] {
    if (!r) fail(KMHG_EINVAL, "null argument");
    const ReadsHost& h = r->r;
    if (seq) memcpy(seq, h.seq.data(), h.seq.size());
    if (qual) memcpy(qual, h.qual.data(), h.qual.size());
    if (offsets) memcpy(offsets, h.off.data(), h.off.size() * 8);
    if (has_qual) memcpy(has_qual, h.hasq.data(), h.hasq.size());
  });
}

int kmhg_reads_free(kmhg_reads* r) {
  delete r;
  return KMHG_OK;
}

int kmhg_sh_count_reads(kmhg_index** sh, const kmhg_reads* r, const int32_t params[8]) {
  return guarded([&] {
    if (!sh || !r || !params) fail(KMHG_EINVAL, "null argument");
    if (*sh) check_sh(*sh);
    check_sh_params(params);
    const int k = params[0];
    const double min_ll = qll_host((unsigned char)('!' + (unsigned char)params[2]));
    const uint32_t source = (uint32_t)params[7];
    hipStream_t s = lib_stream();
    std::unique_ptr<kmhg_index> fresh;
    kmhg_index* c = *sh;
    if (!c) {
      fresh.reset(new_sh_index(k, params[6], s));
      c = fresh.get();
    } else if (!sh_accepts(c, k, source)) {
      return;
    }
    DeviceGuard g(c->device);
    // reads no longer than k were dropped when r was read with a smaller k
    ReadsHost keep;
    const ReadsHost* use = &r->r;
    bool all_long = true;
    for (size_t i = 0; i < r->r.n() && all_long; ++i)
      all_long = r->r.off[i + 1] - r->r.off[i] > k;
    if (!all_long) {
      for (size_t i = 0; i < r->r.n(); ++i) {
        const int64_t a = r->r.off[i], b = r->r.off[i + 1];
        if (b - a <= k) continue;
        keep.add(std::string((const char*)r->r.seq.data() + a, (size_t)(b - a)),
                 std::string((const char*)r->r.qual.data() + a, (size_t)(b - a)),
                 r->r.hasq[i] != 0);
      }
      use = &keep;
    }
    sh_count_reads_host(c, *use, min_ll, source, s);
    c->L += (int64_t)use->seq.size();
    if (fresh) *sh = fresh.release();
  });
}

int kmhg_sh_count_reads_device(kmhg_index** sh, const void* d_seq, const void* d_qual,
                               const int64_t* d_offsets, const uint8_t* d_has_qual,
                               int64_t n_reads, const int32_t params[8], void* stream) {
  return guarded([&] {
    if (!sh || !params || (n_reads > 0 && (!d_seq || !d_qual || !d_offsets || !d_has_qual)))
      fail(KMHG_EINVAL, "null argument");
    if (*sh) check_sh(*sh);
    check_sh_params(params);
    if (n_reads < 0 || n_reads >= (int64_t)UINT32_MAX) fail(KMHG_EINVAL, "bad read count");
    if ((reinterpret_cast<uintptr_t>(d_seq) | reinterpret_cast<uintptr_t>(d_qual)) & 15)
      fail(KMHG_EINVAL, "read bases and qualities must be 16-byte aligned");
    const int k = params[0];
    const double min_ll = qll_host((unsigned char)('!' + (unsigned char)params[2]));
    const uint32_t source = (uint32_t)params[7];
    hipStream_t s = (hipStream_t)stream;
    std::unique_ptr<kmhg_index> fresh;
    kmhg_index* c = *sh;
    if (!c) {
      fresh.reset(new_sh_index(k, params[6], s));
      c = fresh.get();
    } else if (!sh_accepts(c, k, source)) {
      return;
    }
    DeviceGuard g(c->device);
    // mean read length for the LDS staging size: the span of the whole batch (two int64 reads)
    double mean_len = 150;
    if (n_reads > 0) {
      int64_t ends[2] = {0, 0};
      HIPC(hipMemcpyAsync(&ends[0], d_offsets, 8, hipMemcpyDeviceToHost, s));
      HIPC(hipMemcpyAsync(&ends[1], d_offsets + n_reads, 8, hipMemcpyDeviceToHost, s));
      HIPC(hipStreamSynchronize(s));
      mean_len = (double)(ends[1] - ends[0]) / (double)n_reads;
      // the key stream is sized by per-read window bounds (each <= the read's length) summed in
      // u32: a batch spanning 2^32 or more bases could wrap that sum
      if (ends[1] < ends[0] || (uint64_t)(ends[1] - ends[0]) >= SH_SPAN_MAX)
        fail(KMHG_EINVAL, "a read batch must span fewer than 2^32 bases: split it");
    }
    sh_count_reads_device(c, (const uint8_t*)d_seq, (const uint8_t*)d_qual, d_offsets,
                          d_has_qual, (uint32_t)n_reads, mean_len, min_ll, source, s);
    if (fresh) *sh = fresh.release();
  });
}

// seq_kmer_depth_sh (src/kmer_hash.c:859-879) + seq_kmer_counts (src/kmer_reader.c:155-193)
static void check_depth(const kmhg_index* sh, int k) {
  check_sh(sh);
  if (k != sh->k) fail(KMHG_EINVAL, "Receieved error from seq_kmer_counts");
}

int kmhg_sh_depth(kmhg_index* sh, const char* seq, size_t L, int k, int32_t* counts) {
  return guarded([&] {
    check_depth(sh, k);
    if (L && (!seq || !counts)) fail(KMHG_EINVAL, "null argument");
    if (L >= (size_t)INT32_MAX) fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1");
    DeviceGuard g(sh->device);
    hipStream_t s = lib_stream();
    const size_t n = effective_len(seq, L);     // the walk ends at a NUL
    const size_t S = sh->sources;
    DBuf<uint8_t> d(n + 16, s);
    DBuf<int32_t> out(std::max<size_t>(L * S, 1), s);
    if (n) HIPC(hipMemcpyAsync(d.p, seq, n, hipMemcpyHostToDevice, s));
    sh_depth_device(sh, d.p, (int64_t)n, k, out.p, s);
    if (L > n)   // past a NUL: never written (NA)
      HIPC(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(out.p + n * S), (int)INT_MIN,
                             (L - n) * S, s));
    if (L) d2h_host(counts, out.p, L * S * 4, s);
    HIPC(hipStreamSynchronize(s));
  });
}

int kmhg_sh_depth_device(kmhg_index* sh, const void* d_seq, size_t L, int k, int32_t* d_counts,
                         void* stream) {
  return guarded([&] {
    check_depth(sh, k);
    if (L && (!d_seq || !d_counts)) fail(KMHG_EINVAL, "null argument");
    if (L >= (size_t)INT32_MAX) fail(KMHG_EOVERFLOW, "sequence longer than 2^31-1");
    DeviceGuard g(sh->device);
    sh_depth_device(sh, (const uint8_t*)d_seq, (int64_t)L, k, d_counts, (hipStream_t)stream);
  });
}

// kmer_spectrum_suffix_hash_n (src/kmer_hash.c:1010-1039) + sh_count_spectrum_nc
// (src/suffix_hash.c:338-421).  *status = 1, or the reference's negative code (counts zero).
int kmhg_sh_spectrum(kmhg_index* sh, int max_count, const int32_t* comb,
                     const int32_t* comb_inner, int comb_n, const int32_t* source_min,
                     int n_source_min, double* counts, int* status) {
  return guarded([&] {
    check_sh(sh);
    if (comb_n < 1) fail(KMHG_EINVAL, "comb_r should be an integer vector of length > 0");
    if (!comb || !comb_inner)
      fail(KMHG_EINVAL, "comb_inner_r should be an integer vector of the same length as comb_r");
    if (n_source_min != (int)sh->sources || !source_min)
      fail(KMHG_EINVAL, "source_min_r should be an integer vector of length sh->counts_n");
    if (max_count < 0) fail(KMHG_EINVAL, "max_count must be >= 0");   // reference: R alloc error
    if (!counts) fail(KMHG_EINVAL, "null argument");
    const uint32_t S = sh->sources;
    const size_t nbins = (size_t)(max_count + 1) * (size_t)comb_n * S;
    std::fill(counts, counts + nbins, 0.0);
    int st = 1;
    for (int i = 0; i < comb_n && st == 1; ++i) {
      if ((uint32_t)comb_inner[i] > 1) st = -3;
      else if ((uint32_t)comb[i] >= (1u << S)) st = -4;
    }
    if (status) *status = st;
    if (st != 1) {
      fprintf(stderr, "sh_count_spectrum_nc returned an error: %d\n", st);
      return;
    }
    DeviceGuard g(sh->device);
    hipStream_t s = lib_stream();
    finish_build(sh);
    if (!sh->U) return;
    std::vector<uint32_t> args((size_t)2 * comb_n + S);
    for (int i = 0; i < comb_n; ++i) {
      args[i] = (uint32_t)comb[i];
      args[comb_n + i] = (uint32_t)comb_inner[i];
    }
    for (uint32_t j = 0; j < S; ++j) args[2 * comb_n + j] = (uint32_t)source_min[j];
    DBuf<uint32_t> dargs(args.size(), s), bins(nbins, s);
    HIPC(hipMemcpyAsync(dargs.p, args.data(), args.size() * 4, hipMemcpyHostToDevice, s));
    HIPC(hipMemsetAsync(bins.p, 0, nbins * 4, s));
    LAUNCH("k_spectrum", s,
           launch_spectrum(sh->positions.p, sh->U, S, (uint32_t)max_count, dargs.p,
                           dargs.p + comb_n, (uint32_t)comb_n, dargs.p + 2 * comb_n, bins.p, s));
    std::vector<uint32_t> h(nbins);
    HIPC(hipMemcpyAsync(h.data(), bins.p, nbins * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (size_t i = 0; i < nbins; ++i) counts[i] = (double)h[i];
  });
}

// (key, counts) rows of a counts index in row order (tests, export)
int kmhg_counts_export(kmhg_index* idx, uint64_t* keys, int32_t* counts) {
  return guarded([&] {
    if (!idx || !idx->sources) fail(KMHG_EINVAL, "not a counts index");
    DeviceGuard g(idx->device);
    hipStream_t s = lib_stream();
    idx->stream = s;
    ReleaseGroup rg(s);
    ensure_row_order(idx, s);
    const uint64_t U = idx->U, S = idx->sources;
    const uint64_t* k = idx->ckeys.p;
    const int32_t* m = idx->positions.p;
    DBuf<uint64_t> gk;
    DBuf<int32_t> gm;
    if (U && row_order_of(idx) && (keys || counts)) {   // rows in first-insertion order
      gk.reset(U);
      gm.reset(U * S);
      gk.bind(s);
      gm.bind(s);
      LAUNCH("k_rows_gather", s, launch_rows_gather(row_order_of(idx), idx->ckeys.p,
                                                    idx->positions.p, (uint32_t)U, (uint32_t)S,
                                                    gk.p, gm.p, s));
      k = gk.p;
      m = gm.p;
    }
    if (U && keys) HIPC(hipMemcpyAsync(keys, k, U * 8, hipMemcpyDeviceToHost, s));
    if (U && counts) HIPC(hipMemcpyAsync(counts, m, U * S * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
  });
}

int kmhg_sh_last_batch(const kmhg_index* sh, double* distinct_est, int* spread, int* path) {
  return guarded([&] {
    if (!sh || !sh->canonical) fail(KMHG_EINVAL, "not a suffix hash");
    if (distinct_est) *distinct_est = sh->co_est;
    if (spread) *spread = sh->co_spread;
    if (path) *path = sh->co_path;
  });
}

int kmhg_index_wait(kmhg_index* idx) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    DeviceGuard g(idx->device);
    finish_build(idx);
  });
}

int kmhg_index_info(const kmhg_index* cidx, kmhg_info* info) {
  return guarded([&] {
    if (!cidx || !info) fail(KMHG_EINVAL, "null argument");
    kmhg_index* idx = const_cast<kmhg_index*>(cidx);   // completes a pending build
    DeviceGuard g(idx->device);
    finish_build(idx);
    info->k = idx->k;
    info->device = idx->device;
    info->seq_len = idx->L;
    info->n_kmers = (int64_t)idx->U;
    info->n_positions = (int64_t)idx->N;
    info->n_pairs = (int64_t)idx->P;
    info->max_count = idx->max_n;
    info->table_slots = (int64_t)idx->slots();
    info->device_bytes = (int64_t)(idx->table.bytes() + idx->positions.bytes() +
                                   idx->ckeys.bytes() + idx->slot_row.bytes() +
                                   idx->row_slot.bytes());
    info->sources = (int32_t)idx->sources;
    info->kind = idx->canonical ? 2 : (idx->sources ? 1 : 0);
    info->kmer_count = (int64_t)(idx->sources ? idx->kmer_count : idx->U);
    info->build = idx->build_kind;
    info->fallback = idx->fallback;
  });
}

int kmhg_set_row_order(kmhg_index* idx, int order) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    if (order != KMHG_ORDER_FIRST && order != KMHG_ORDER_KHASH) fail(KMHG_EINVAL, "unknown row order");
    idx->row_order = order;
  });
}

int kmhg_khash_order(const uint64_t* keys, int64_t n, uint32_t* order) {
  return guarded([&] {
    if (n < 0 || (n && (!keys || !order))) fail(KMHG_EINVAL, "null argument");
    const std::vector<uint64_t> k(keys, keys + n);
    const std::vector<uint32_t> o = khash_bucket_order(k);
    std::copy(o.begin(), o.end(), order);
  });
}

int kmhg_get_row_order(const kmhg_index* idx, int* order) {
  return guarded([&] {
    if (!idx || !order) fail(KMHG_EINVAL, "null argument");
    *order = idx->row_order;
  });
}

int kmhg_positions_size(kmhg_index* idx, uint32_t opt, int64_t* n_kmers, int64_t* n_pos_rows,
                        int64_t* n_pair_rows, int64_t* n_counts) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    DeviceGuard g(idx->device);
    finish_build(idx);
    positions_sizes(idx, opt, n_kmers, n_pos_rows, n_pair_rows, n_counts);
  });
}

int kmhg_positions_fill_device(kmhg_index* idx, uint32_t opt, char* d_kmers, int32_t* d_pos,
                               int32_t* d_pairs, int32_t* d_counts, void* stream) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    DeviceGuard g(idx->device);
    hipStream_t s = (hipStream_t)stream;   // caller stream; NULL = HIP null stream
    positions_device(idx, opt, d_kmers, d_pos, d_pairs, d_counts, s);
  });
}

// kmer.pos's pair rows into a host matrix (the R API's readout).  A pair row is {key label,
// position j, position q} for every j < q of a repeated key's list -- P rows from the lists'
// ~N positions (config 4: 686 M rows, 8.2 GB, from 40 M positions) -- so from HOST_PAIRS_MIN
// rows on, the lists and their keys' offsets cross PCIe (pkeys, pair_off, rinfo, positions:
// ~0.4 GB at config 4) and host threads write the rows, each from its stripe's first pair on
// (the pair t of a key with n positions: the largest j with j (2n - j - 1) / 2 <= t, as
// V_read_pairs).  KMHG_HOST_PAIRS=0 (test build): the rows are made on the device and copied.
constexpr uint64_t HOST_PAIRS_MIN = 1u << 22;           // rows (48 MB)
static void expand_pairs_host(const uint32_t* pk, const uint64_t* po, uint64_t M, const uint2* ri,
                              const int32_t* ps, uint64_t P, int32_t* out) {
  const int T = expand_threads(P * 12);
  const uint64_t stripe = (P + T - 1) / T;
  auto work = [=](uint64_t r0, uint64_t r1) {
    uint64_t m = (uint64_t)(std::upper_bound(po, po + M, r0) - po) - 1;
    uint64_t t = r0 - po[m], r = r0;
    while (r < r1) {
      const uint32_t c = pk[m];
      const uint64_t n = ri[c].x;
      const int32_t* lst = ps + (ri[c].y - n);
      auto S = [n](uint64_t x) { return x * (2 * n - x - 1) / 2; };
      uint64_t j = 0;
      if (t) {
        const double dn = 2.0 * (double)n - 1.0, disc = dn * dn - 8.0 * (double)t;
        j = (uint64_t)std::max(0.0, (dn - std::sqrt(std::max(disc, 0.0))) * 0.5);
        j = std::min<uint64_t>(j, n - 2);
        while (j > 0 && S(j) > t) --j;
        while (j + 1 <= n - 2 && S(j + 1) <= t) ++j;
      }
      uint64_t q = j + 1 + (t - S(j));
      const int32_t lab = (int32_t)(c + 1);
      for (; j + 1 < n && r < r1; ++j, q = j + 1) {
        const int32_t pj = lst[j];
        const uint64_t qe = std::min<uint64_t>(n, q + (r1 - r));
        int32_t* o = out + 3 * r;
        for (uint64_t x = q; x < qe; ++x, o += 3) {
          o[0] = lab;
          o[1] = pj;
          o[2] = lst[x];
        }
        r += qe - q;
      }
      ++m;
      t = 0;
    }
  };
  HostPool::get().run(T, [&](int i) {
    const uint64_t a = std::min(P, i * stripe), b = std::min(P, a + stripe);
    if (a < b) work(a, b);
  }, P * 12 >= HOST_BIG_BYTES);
}

static void pairs_to_host(kmhg_index* idx, int32_t* out, hipStream_t s) {
  Canon& c = idx->canon;                     // prepare_readout ran (positions_device)
  const uint64_t M = c.n_multi, U = idx->U, P = idx->P;
  std::unique_ptr<uint32_t[]> pk(new uint32_t[M]);
  std::unique_ptr<uint64_t[]> po(new uint64_t[M]);
  std::unique_ptr<uint2[]> ri(new uint2[U]);
  d2h_host(pk.get(), c.pkeys.p, M * 4, s);
  d2h_host(po.get(), c.pair_off.p, M * 8, s);
  d2h_host(ri.get(), c.rinfo.p, U * 8, s);
  uint64_t n_lists = 0;                      // the list entries in use: [0, max end)
  for (uint64_t m = 0; m < M; ++m) n_lists = std::max<uint64_t>(n_lists, ri[pk[m]].y);
  if (n_lists > idx->positions.n) fail(KMHG_EDEVICE, "pair lists beyond the positions");
  std::unique_ptr<int32_t[]> ps(new int32_t[std::max<uint64_t>(n_lists, 1)]);
  d2h_host(ps.get(), idx->positions.p, n_lists * 4, s);
  hint_huge_pages(out, P * 12);
  expand_pairs_host(pk.get(), po.get(), M, ri.get(), ps.get(), P, out);
}

int kmhg_positions_fill(kmhg_index* idx, uint32_t opt, char* kmers, int32_t* pos, int32_t* pairs,
                        int32_t* counts) {
  return guarded([&] {
    if (!idx) fail(KMHG_EINVAL, "null index");
    DeviceGuard g(idx->device);
    hipStream_t s = lib_stream();
    const size_t U = idx->U;
    const char* hpe = test_build_knob("KMHG_HOST_PAIRS");
    const bool host_pairs = (opt & KMHG_OPT_PAIRS) && pairs && idx->P >= HOST_PAIRS_MIN &&
                            idx->sources == 0 && !(hpe && hpe[0] == '0');   // position indices
    const uint32_t dopt = host_pairs ? opt & ~(uint32_t)KMHG_OPT_PAIRS : opt;
    DBuf<char> dk((opt & KMHG_OPT_KMER) ? U * (idx->k + 1) : 0, s);
    DBuf<int32_t> dp((opt & KMHG_OPT_POS) ? 2 * idx->N : 0, s);
    DBuf<int32_t> dpp((dopt & KMHG_OPT_PAIRS) ? 3 * idx->P : 0, s);
    DBuf<int32_t> dc((opt & KMHG_OPT_COUNT) ? U : 0, s);
    positions_device(idx, dopt, dk.p, dp.p, dpp.p, dc.p, s);
    if ((opt & KMHG_OPT_KMER) && U && kmers)
      d2h_host(kmers, dk.p, dk.bytes(), s);
    if ((opt & KMHG_OPT_POS) && idx->N && pos)
      d2h_host(pos, dp.p, dp.bytes(), s);
    if (host_pairs)
      pairs_to_host(idx, pairs, s);
    else if ((opt & KMHG_OPT_PAIRS) && idx->P && pairs)
      d2h_host(pairs, dpp.p, dpp.bytes(), s);
    if ((opt & KMHG_OPT_COUNT) && U && counts)
      d2h_host(counts, dc.p, dc.bytes(), s);
    HIPC(hipStreamSynchronize(s));
  });
}

int kmhg_pairs_run(kmhg_index* a, kmhg_index* b, kmhg_query** q, int64_t* n_rows) {
  return guarded([&] {
    if (!a || !b || !q) fail(KMHG_EINVAL, "null argument");
    DeviceGuard g(a->device);
    hipStream_t s = lib_stream();
    *q = pairs_device(a, b, s);
    HIPC(hipStreamSynchronize(s));
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_pairs_run_device(kmhg_index* a, kmhg_index* b, void* stream, kmhg_query** q,
                          int64_t* n_rows) {
  return guarded([&] {
    if (!a || !b || !q) fail(KMHG_EINVAL, "null argument");
    DeviceGuard g(a->device);
    *q = pairs_device(a, b, (hipStream_t)stream);
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_query_run(kmhg_index* idx, const char* seq, size_t L, int k, kmhg_query** q,
                   int64_t* n_rows) {
  return guarded([&] {
    if (!idx || !seq || !q) fail(KMHG_EINVAL, "null argument");
    const std::vector<int> devs = query_devices();
    if (devs.size() > 1 && idx->sources == 0) {   // position index over several devices
      L = effective_len(seq, L);
      check_query_args(L, k);
      *q = query_multi_device(idx, seq, (int64_t)L, k, devs);
      if (n_rows) *n_rows = (*q)->H;
      return;
    }
    if (L < H2D_SCAN_MIN || k < 1 || k > 31 || L >= (size_t)INT32_MAX) {
      L = effective_len(seq, L);             // (as kmhg_build)
      check_query_args(L, k);
    }
    DeviceGuard g(idx->device);
    hipStream_t s = lib_stream();
    DBuf<uint8_t> d(L + 16, s);
    L = h2d_cstring(d.p, seq, L, s);
    check_query_args(L, k);
    *q = query_device(idx, d.p, (int64_t)L, k, 0, (int64_t)L - k + 1, s);
    HIPC(hipStreamSynchronize(s));
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_query_run_device(kmhg_index* idx, const void* d_seq, size_t L, int k, void* stream,
                          kmhg_query** q, int64_t* n_rows) {
  return guarded([&] {
    if (!idx || !d_seq || !q) fail(KMHG_EINVAL, "null argument");
    check_query_args(L, k);
    DeviceGuard g(idx->device);
    hipStream_t s = (hipStream_t)stream;   // caller stream; NULL = HIP null stream
    *q = query_device(idx, (const uint8_t*)d_seq, (int64_t)L, k, 0, (int64_t)L - k + 1, s);
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_query_run_device_range(kmhg_index* idx, const void* d_seq, size_t L, int k,
                                int64_t w_begin, int64_t w_end, void* stream, kmhg_query** q,
                                int64_t* n_rows) {
  return guarded([&] {
    if (!idx || !d_seq || !q) fail(KMHG_EINVAL, "null argument");
    check_query_args(L, k);
    const int64_t Nw = (int64_t)L - k + 1;
    if (w_begin < 0 || w_end > Nw || w_begin > w_end) fail(KMHG_EINVAL, "window range out of bounds");
    DeviceGuard g(idx->device);
    hipStream_t s = (hipStream_t)stream;   // caller stream; NULL = HIP null stream
    *q = query_device(idx, (const uint8_t*)d_seq, (int64_t)L, k, w_begin, w_end, s);
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_query_run_device_range_runs(kmhg_index* idx, const void* d_seq, size_t L, int k,
                                     int64_t w_begin, int64_t w_end, void* stream,
                                     kmhg_query** q, int64_t* n_rows, int64_t* n_runs) {
  return guarded([&] {
    if (!idx || !d_seq || !q) fail(KMHG_EINVAL, "null argument");
    check_query_args(L, k);
    const int64_t Nw = (int64_t)L - k + 1;
    if (w_begin < 0 || w_end > Nw || w_begin > w_end) fail(KMHG_EINVAL, "window range out of bounds");
    DeviceGuard g(idx->device);
    hipStream_t s = (hipStream_t)stream;
    *q = query_device(idx, (const uint8_t*)d_seq, (int64_t)L, k, w_begin, w_end, s, false, true);
    if (n_rows) *n_rows = (*q)->H;
    if (n_runs) *n_runs = (*q)->n_runs;
  });
}

int kmhg_query_runs_device(kmhg_query* q, const int32_t** d_runs) {
  return guarded([&] {
    if (!q || !d_runs) fail(KMHG_EINVAL, "null argument");
    if (q->n_runs < 0) fail(KMHG_EINVAL, "the query holds rows, not runs");
    *d_runs = q->runs.p;
  });
}

int kmhg_query_run_device_part(kmhg_index* part, const void* d_seq, size_t L, int k,
                               void* stream, kmhg_query** q, int64_t* n_rows) {
  return guarded([&] {
    if (!part || !d_seq || !q) fail(KMHG_EINVAL, "null argument");
    check_query_args(L, k);
    DeviceGuard g(part->device);
    *q = query_device(part, (const uint8_t*)d_seq, (int64_t)L, k, 0, (int64_t)L - k + 1,
                      (hipStream_t)stream, true);
    if (n_rows) *n_rows = (*q)->H;
  });
}

int kmhg_query_tile_offsets(kmhg_query* q, uint64_t* d_out, int64_t* n_tiles, void* stream) {
  return guarded([&] {
    if (!q || !n_tiles) fail(KMHG_EINVAL, "null argument");
    if (!q->tile_off.p && q->H) fail(KMHG_EINVAL, "not a part query");
    *n_tiles = q->n_tiles;
    if (!d_out) return;
    DeviceGuard g(q->device);
    hipStream_t s = (hipStream_t)stream;
    if (q->n_tiles)
      HIPC(hipMemcpyAsync(d_out, q->tile_off.p, (size_t)q->n_tiles * 8, hipMemcpyDeviceToDevice, s));
    const uint64_t h = (uint64_t)q->H;            // [n_tiles] = the part's row total
    launch_fill_u64(d_out + q->n_tiles, h, s);
  });
}

int kmhg_merge_part_rows(const void* d_rows, const uint64_t* d_seg_base, const uint64_t* d_tile_off,
                         int n_parts, int64_t n_tiles, int k, int64_t w0, void* d_out,
                         void* stream) {
  return guarded([&] {
    if (n_parts < 1 || n_tiles < 0 || k < 1 || k > 32) fail(KMHG_EINVAL, "bad merge arguments");
    if (!n_tiles) return;
    if (!d_rows || !d_seg_base || !d_tile_off || !d_out) fail(KMHG_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    LAUNCH("k_merge_part_rows", s,
           launch_merge_part_rows(reinterpret_cast<const int2*>(d_rows), d_seg_base, d_tile_off,
                                  (uint32_t)n_parts, (uint32_t)n_tiles, k, w0,
                                  reinterpret_cast<int2*>(d_out), s));
    HIPC(hipGetLastError());
  });
}

int kmhg_seq_pack(const void* d_seq, int64_t L, uint32_t* d_code, uint16_t* d_nbit,
                  void* stream) {
  return guarded([&] {
    if (L < 0) fail(KMHG_EINVAL, "bad sequence length");
    if (!L) return;
    if (!d_seq || !d_code || !d_nbit) fail(KMHG_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    LAUNCH("k_seq_pack", s, launch_seq_pack(static_cast<const uint8_t*>(d_seq), L, d_code,
                                            d_nbit, s));
    HIPC(hipGetLastError());
  });
}

int kmhg_seq_unpack(const uint32_t* d_code, const uint16_t* d_nbit, int64_t word0, int64_t a,
                    int64_t b, void* d_seq, void* stream) {
  return guarded([&] {
    if (a < 0 || b < a || word0 < 0 || word0 > a / 16) fail(KMHG_EINVAL, "bad unpack range");
    if (b == a) return;
    if (!d_code || !d_nbit || !d_seq) fail(KMHG_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    LAUNCH("k_seq_unpack", s, launch_seq_unpack(d_code, d_nbit, (uint64_t)word0, a, b,
                                                static_cast<uint8_t*>(d_seq), s));
    HIPC(hipGetLastError());
  });
}

int kmhg_rows_runs(const void* d_rows, int64_t n_rows, void* d_runs, int64_t cap_runs,
                   int64_t* n_runs, void* stream) {
  return guarded([&] {
    if (n_rows < 0 || n_rows > INT32_MAX || !n_runs) fail(KMHG_EINVAL, "bad run arguments");
    *n_runs = 0;
    if (!n_rows) return;
    if (!d_rows) fail(KMHG_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    ReleaseGroup rg(s);
    const uint64_t nt = ((uint64_t)n_rows + TILE - 1) / TILE;
    DBuf<uint64_t> tiles(nt + scan_u64_scratch(nt), s);
    PinnedRec hrec = PinnedPool::get().take();
    GiveBack give_back{hrec, s};
    uint64_t* total = &hrec.meta->n_kmers;
    const int2* rows = reinterpret_cast<const int2*>(d_rows);
    LAUNCH("k_runs_count", s, launch_runs_count(rows, (uint64_t)n_rows, tiles.p, s));
    LAUNCH("k_scan_tiles_u64", s, launch_scan_u64(tiles.p, nt, total, tiles.p + nt, s));
    HIPC(hipStreamSynchronize(s));
    const uint64_t n = __atomic_load_n(total, __ATOMIC_ACQUIRE);
    *n_runs = (int64_t)n;
    if (d_runs && (int64_t)n <= cap_runs)
      LAUNCH("k_runs_emit", s, launch_runs_emit(rows, (uint64_t)n_rows, tiles.p,
                                                static_cast<int32_t*>(d_runs), s));
    HIPC(hipGetLastError());
  });
}

int kmhg_rows_to_host(const void* d_rows, int64_t n_rows, int32_t* rows, void* stream) {
  return guarded([&] {
    if (n_rows < 0) fail(KMHG_EINVAL, "bad row count");
    if (!n_rows) return;
    if (!d_rows || !rows) fail(KMHG_EINVAL, "null argument");
    rows_to_host(static_cast<const int2*>(d_rows), (uint64_t)n_rows, rows, (hipStream_t)stream);
  });
}

int kmhg_runs_expand(const void* d_runs, int64_t n_runs, int64_t n_rows, void* d_rows,
                     void* stream) {
  return guarded([&] {
    if (n_rows < 0 || n_rows > INT32_MAX || n_runs < 0 || n_runs > n_rows || (n_rows && !n_runs))
      fail(KMHG_EINVAL, "bad run arguments");
    if (!n_rows) return;
    if (!d_runs || !d_rows) fail(KMHG_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    ReleaseGroup rg(s);
    DBuf<uint32_t> cover(((uint64_t)n_rows + TILE - 1) / TILE, s);
    LAUNCH("k_runs_expand", s,
           launch_runs_expand(static_cast<const int32_t*>(d_runs), (uint64_t)n_runs,
                              (uint64_t)n_rows, cover.p, static_cast<int2*>(d_rows), s));
    HIPC(hipGetLastError());
  });
}

int kmhg_query_fill(kmhg_query* q, int32_t* rows) {
  return guarded([&] {
    if (!q) fail(KMHG_EINVAL, "null query");
    if (q->n_runs >= 0) fail(KMHG_EINVAL, "the query holds runs (kmhg_query_runs_device)");
    if (!q->H) return;
    if (!rows) fail(KMHG_EINVAL, "null output");
    if (!q->parts.empty() && !q->gathered) {   // every part straight into its rows, in parallel
      std::vector<Error> errs(q->parts.size(), Error{KMHG_OK, ""});
      auto copy = [&](size_t i) {
        try {
          kmhg_query* p = q->parts[i];
          if (!p->H) return;
          DeviceGuard g(p->device);
          rows_to_host(p->rows.p, (uint64_t)p->H, rows + 2 * q->part_off[i], lib_stream());
        } catch (const Error& e) {
          errs[i] = e;
        }
      };
      std::vector<std::thread> th;
      for (size_t i = 1; i < q->parts.size(); ++i) th.emplace_back(copy, i);
      copy(0);
      for (auto& t : th) t.join();
      for (auto& e : errs)
        if (e.code != KMHG_OK) fail(e.code, e.msg);
      return;
    }
    DeviceGuard g(q->device);
    hipStream_t s = lib_stream();
    rows_to_host(q->rows.p, (uint64_t)q->H, rows, s);
  });
}

int kmhg_query_rows_device(kmhg_query* q, const int32_t** d_rows) {
  return guarded([&] {
    if (!q || !d_rows) fail(KMHG_EINVAL, "null argument");
    if (q->n_runs >= 0) fail(KMHG_EINVAL, "the query holds runs (kmhg_query_runs_device)");
    gather_parts(q);
    *d_rows = reinterpret_cast<const int32_t*>(q->rows.p);
  });
}

int kmhg_query_copy_device(kmhg_query* q, void* d_dst, void* stream) {
  return guarded([&] {
    if (!q) fail(KMHG_EINVAL, "null query");
    if (q->n_runs >= 0) fail(KMHG_EINVAL, "the query holds runs (kmhg_query_runs_device)");
    if (!q->H) return;
    if (!d_dst) fail(KMHG_EINVAL, "null output");
    DeviceGuard g(q->device);
    hipStream_t s = (hipStream_t)stream;
    if (!q->parts.empty() && !q->gathered) {   // peer copies of the (finished) parts
      for (size_t i = 0; i < q->parts.size(); ++i)
        if (q->parts[i]->H)
          HIPC(hipMemcpyPeerAsync(static_cast<int2*>(d_dst) + q->part_off[i], q->device,
                                  q->parts[i]->rows.p, q->parts[i]->device,
                                  (size_t)q->parts[i]->H * 8, s));
      return;
    }
    if (s != q->stream) {   // order after the emit kernel queued on q->stream
      hipEvent_t ev;
      HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIPC(hipEventRecord(ev, q->stream));
      HIPC(hipStreamWaitEvent(s, ev, 0));
      HIPC(hipEventDestroy(ev));
    }
    HIPC(hipMemcpyAsync(d_dst, q->rows.p, (size_t)q->H * 8, hipMemcpyDeviceToDevice, s));
  });
}

int kmhg_query_free(kmhg_query* q) {
  return guarded([&] { free_query(q); });
}

int kmhg_image_sizes_get(const kmhg_index* cidx, kmhg_image_sizes* sz, int64_t header[8]) {
  return guarded([&] {
    if (!cidx || !sz || !header) fail(KMHG_EINVAL, "null argument");
    kmhg_index* idx = const_cast<kmhg_index*>(cidx);   // completes a pending build
    if (idx->sources) fail(KMHG_EINVAL, "index images hold position indices only");
    if (idx->is_part) fail(KMHG_EINVAL, "a part index is exported with kmhg_part_export");
    DeviceGuard g(idx->device);
    finish_build(idx);
    sz->table_bytes = (int64_t)(idx->slots() * sizeof(Slot));
    sz->positions_bytes = (int64_t)(idx->N * 4);
    sz->codes_bytes = idx->dcodes.p ? (int64_t)(diag_block_words(idx->L - idx->k + 1) * 8) : 0;
    header[0] = idx->k; header[1] = idx->L;
    header[2] = ((int64_t)idx->geom.nb << 32) | idx->geom.capb;
    header[3] = (int64_t)idx->U; header[4] = (int64_t)idx->N; header[5] = (int64_t)idx->P;
    header[6] = idx->max_n; header[7] = 0x6B6D6867;   // 'kmhg'
  });
}

int kmhg_image_export(const kmhg_index* cidx, void* d_table, void* d_positions, void* d_codes,
                      void* stream) {
  return guarded([&] {
    if (!cidx) fail(KMHG_EINVAL, "null index");
    kmhg_index* idx = const_cast<kmhg_index*>(cidx);
    if (idx->sources) fail(KMHG_EINVAL, "index images hold position indices only");
    DeviceGuard g(idx->device);
    finish_build(idx);
    hipStream_t s = (hipStream_t)stream;   // caller stream; NULL = HIP null stream
    if (d_table) HIPC(hipMemcpyAsync(d_table, idx->table.p, idx->slots() * sizeof(Slot),
                                     hipMemcpyDeviceToDevice, s));
    if (d_positions && idx->N)
      HIPC(hipMemcpyAsync(d_positions, idx->positions.p, idx->N * 4, hipMemcpyDeviceToDevice, s));
    if (d_codes && idx->dcodes.p)
      HIPC(hipMemcpyAsync(d_codes, idx->dcodes.p, diag_block_words(idx->L - idx->k + 1) * 8,
                          hipMemcpyDeviceToDevice, s));
    HIPC(hipStreamSynchronize(s));
  });
}

int kmhg_image_import(const int64_t header[8], const void* d_table, const void* d_positions,
                      const void* d_codes, void* stream, kmhg_index** out) {
  return guarded([&] {
    if (!header || !out || header[7] != 0x6B6D6867) fail(KMHG_EINVAL, "bad index image header");
    auto idx = std::make_unique<kmhg_index>();
    HIPC(hipGetDevice(&idx->device));
    hipStream_t s = (hipStream_t)stream;
    idx->k = (int)header[0]; idx->L = header[1];
    idx->geom = Geom{(uint32_t)((uint64_t)header[2] >> 32), (uint32_t)(header[2] & 0xFFFFFFFF)};
    idx->U = (uint64_t)header[3]; idx->N = (uint64_t)header[4]; idx->P = (uint64_t)header[5];
    idx->max_n = (uint32_t)header[6];
    idx->table.reset(idx->slots());
    idx->positions.reset(idx->N);
    if (!d_table || (idx->N && !d_positions)) fail(KMHG_EINVAL, "null image buffer");
    HIPC(hipMemcpyAsync(idx->table.p, d_table, idx->slots() * sizeof(Slot),
                        hipMemcpyDeviceToDevice, s));
    if (idx->N)
      HIPC(hipMemcpyAsync(idx->positions.p, d_positions, idx->N * 4, hipMemcpyDeviceToDevice, s));
    if (d_codes) {   // the diagonal query path's code block (its uniq bits are derived on first use)
      const uint64_t w = diag_block_words(idx->L - idx->k + 1);
      idx->dcodes.reset(w);
      HIPC(hipMemcpyAsync(idx->dcodes.p, d_codes, w * 8, hipMemcpyDeviceToDevice, s));
    }
    HIPC(hipStreamSynchronize(s));
    *out = idx.release();
  });
}

int kmhg_check_lds_lane_order(uint64_t* out_of_order, uint64_t* checked) {
  return guarded([&] {
    if (!out_of_order || !checked) fail(KMHG_EINVAL, "null result pointer");
    DBuf<unsigned long long> res(2, nullptr);
    HIPC(hipMemsetAsync(res.p, 0, 2 * sizeof(unsigned long long), nullptr));
    launch_lane_order_check(res.p, nullptr);
    unsigned long long h[2] = {0, 0};
    HIPC(hipMemcpy(h, res.p, sizeof(h), hipMemcpyDeviceToHost));
    *out_of_order = h[0];
    *checked = h[1];
  });
}

int kmhg_timing_enable(int on) {
  Timing::get().on = on != 0;
  return KMHG_OK;
}

int kmhg_timing_select(const char* kernel) {
  return guarded([&] { Timing::get().only = kernel ? kernel : ""; });
}

int kmhg_timing_reset(void) {
  return guarded([&] {
    Timing::get().collect();
    Timing::get().acc.clear();
  });
}

int kmhg_timing_report(char* buf, size_t cap) {
  return guarded([&] {
    Timing& t = Timing::get();
    t.collect();
    std::string js = "{";
    bool first = true;
    for (auto& kv : t.acc) {
      char tmp[256];
      snprintf(tmp, sizeof tmp, "%s\"%s\": [%lld, %.6f]", first ? "" : ", ", kv.first.c_str(),
               (long long)kv.second.first, kv.second.second);
      js += tmp;
      first = false;
    }
    js += "}";
    if (!buf || cap < js.size() + 1) fail(KMHG_EINVAL, "timing report buffer too small");
    memcpy(buf, js.c_str(), js.size() + 1);
  });
}

int kmhg_pool_trim(void) {
  return guarded([&] { DevicePool::get().trim(); });
}

int64_t kmhg_pool_cached_bytes(void) { return DevicePool::get().cached(); }

}  // extern "C"
