// Replay-mode host helper: torch's own CPU samplers run as parallel chunks, from C++.
//
// ParallelFrameDraws (replay.py) splits each draw of a replay frame -- the Exp(1) switch
// draws, the per-class normals, the resampling uniforms (gpmdm_pf.py:137-213) -- into chunks,
// each run by torch's sampler on a private generator placed exactly where the serial draw
// would stand at that chunk (gpmdm_rng_walk, torch_rng.cpp).  Run from Python threads, every
// chunk pays ~15 us of thread-pool and interpreter overhead under the GIL (the box's 16
// no-op tasks take ~220 us; tools/replay_draws_bench.py), which is more than a class's
// normals cost to draw: the frame's normals phase sat on the GPU's critical path at ~0.38 ms.
// Here one call runs all chunks of a draw on a pool of native threads with the GIL released
// (ctypes): the same samplers (Tensor::exponential_ / normal_ / uniform_ on a
// CPUGeneratorImpl), so the values are the Python chunks' bit for bit.  The pool's idle
// threads block (no spinning): torch's OpenMP pool spins after each region, and on a box
// whose cgroup grants 16 CPUs the spinning team ate the quota the frame's host thread and
// the HIP runtime needed (replay frame 6.9 -> 8.4 ms with at::parallel_for).
//
// Host code only (links libtorch_cpu); built by gpmdm_amd/build.py into
// gpmdm_amd/libgpmdm_replay.so and loaded by replay.py after torch.
#include <ATen/ATen.h>
#include <ATen/CPUGeneratorImpl.h>
#include <c10/core/InferenceMode.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int64_t kStateBytes = 5056;   // torch.Generator.get_state() of a CPU generator

enum Kind : int { kExponential = 0, kNormal = 1, kUniform = 2 };

thread_local std::string g_err;

void run_chunk(int kind, double* dst, int64_t a, int64_t b, const uint8_t* state) {
  // one generator per thread, re-placed per chunk (a fresh CPUGeneratorImpl seeds its
  // MT19937 first: ~3 us wasted per chunk)
  thread_local at::Generator gen = at::make_generator<at::CPUGeneratorImpl>();
  c10::InferenceMode no_autograd;       // plain buffers: skip the autograd dispatch layers
  const at::Tensor st = at::from_blob(const_cast<uint8_t*>(state), {kStateBytes}, at::TensorOptions().dtype(at::kByte));
  {
    std::lock_guard<std::mutex> lock(gen.mutex());
    gen.set_state(st);
  }
  at::Tensor seg = at::from_blob(dst + a, {b - a}, at::TensorOptions().dtype(at::kDouble));
  switch (kind) {
    case kExponential: seg.exponential_(1.0, gen); break;
    case kNormal: seg.normal_(0.0, 1.0, gen); break;
    default: seg.uniform_(0.0, 1.0, gen); break;
  }
}

// Worker threads that sleep between runs; the caller works on its run too.  One run at a
// time (run_mu); a worker joins a run only while it is current, and the caller waits for
// every worker that joined to leave before the run (on its stack) goes away.  warm(us) wakes
// the workers to poll for a run until the deadline (a frame's normals follow its switch by
// ~0.1 ms: woken then, the workers are running when the draw comes), then they sleep again.
class Pool {
 public:
  explicit Pool(int workers) {
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  int workers() const { return (int)th_.size(); }
  void run(int64_t n, const std::function<void(int64_t)>& f) {
    std::lock_guard<std::mutex> one(run_mu_);
    Run r{&f, n};
    {
      std::lock_guard<std::mutex> lk(mu_);
      cur_ = &r;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    work(r);
    std::unique_lock<std::mutex> lk(mu_);
    cur_ = nullptr;                     // no worker joins from here on
    done_.wait(lk, [&] { return r.active == 0; });
  }
  void warm(int64_t us) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      warm_until_.store(now_ns() + us * 1000, std::memory_order_relaxed);
      ++wgen_;
    }
    cv_.notify_all();
  }

 private:
  struct Run {
    const std::function<void(int64_t)>* fn;
    int64_t n;
    std::atomic<int64_t> next{0};
    int active = 0;                     // workers inside (guarded by mu_)
  };
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static void work(Run& r) {
    for (int64_t k = r.next.fetch_add(1); k < r.n; k = r.next.fetch_add(1)) (*r.fn)(k);
  }
  void loop() {
    uint64_t seen = 0, wseen = 0;
    for (;;) {
      // warm: poll for the next run until the deadline, then block
      while (gen_.load(std::memory_order_acquire) == seen && now_ns() < warm_until_.load(std::memory_order_relaxed))
        __builtin_ia32_pause();
      Run* r;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return (cur_ != nullptr && gen_.load() != seen) || wgen_ != wseen; });
        wseen = wgen_;
        if (cur_ == nullptr || gen_.load() == seen) continue;   // woken to warm up: poll
        seen = gen_.load();
        r = cur_;
        ++r->active;
      }
      work(*r);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--r->active == 0) done_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  Run* cur_ = nullptr;
  std::atomic<uint64_t> gen_{0};
  uint64_t wgen_ = 0;
  std::atomic<int64_t> warm_until_{0};
};

Pool* pool_for(int threads) {
  static std::mutex mu;
  static Pool* pool = nullptr;          // kept to the process's end (its threads sleep)
  std::lock_guard<std::mutex> lk(mu);
  const int workers = threads > 1 ? threads - 1 : 0;
  if (!pool || pool->workers() < workers) pool = new Pool(workers);   // (a smaller one is leaked)
  return pool;
}

}  // namespace

extern "C" {

// Fill dst[bounds[2k] : bounds[2k+1]) for k < n_chunks with torch's sampler `kind`
// (0 exponential_(1), 1 normal_(0, 1), 2 uniform_(0, 1)), chunk k drawn from a generator in
// the state states[k * 5056 ...], on `threads` threads (the caller's included).  The chunks
// run concurrently: they must not overlap.  Returns 0, or -1 with the message in
// gpmdm_replay_last_error().
int gpmdm_replay_draw_chunks(int kind, double* dst, const int64_t* bounds, const uint8_t* states,
                             int64_t n_chunks, int threads) {
  if (!dst || !bounds || !states || n_chunks < 0 || kind < 0 || kind > 2 || threads < 1) {
    g_err = "bad argument";
    return -1;
  }
  for (int64_t k = 0; k < n_chunks; ++k)
    if (bounds[2 * k] < 0 || bounds[2 * k + 1] < bounds[2 * k]) {
      g_err = "bad chunk bounds";
      return -1;
    }
  std::atomic<int> failed{0};
  std::string first_err;
  std::mutex err_mu;
  const std::function<void(int64_t)> task = [&](int64_t k) {
    try {
      run_chunk(kind, dst, bounds[2 * k], bounds[2 * k + 1], states + k * kStateBytes);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lock(err_mu);
      if (!failed.exchange(1)) first_err = e.what();
    }
  };
  try {
    if (n_chunks == 1 || threads == 1) {
      for (int64_t k = 0; k < n_chunks; ++k) task(k);
    } else {
      pool_for(threads)->run(n_chunks, task);
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  if (failed.load()) {
    g_err = first_err;
    return -1;
  }
  return 0;
}

// Wake the pool of `threads` threads to poll for work for the next `us` microseconds.
int gpmdm_replay_warm(int threads, int64_t us) {
  if (threads < 2 || us < 0 || us > 100000) return 0;
  try {
    pool_for(threads)->warm(us);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  return 0;
}

const char* gpmdm_replay_last_error(void) { return g_err.c_str(); }

}  // extern "C"
