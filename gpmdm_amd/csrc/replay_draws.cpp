// Replay-mode host helper: torch's own CPU samplers run as parallel chunks, from C++.
//
// ParallelFrameDraws (replay.py) splits each draw of a replay frame -- the Exp(1) switch
// draws, the per-class normals, the resampling uniforms (gpmdm_pf.py:137-213) -- into chunks,
// each run by torch's sampler on a private generator placed exactly where the serial draw
// would stand at that chunk (gpmdm_rng_walk, torch_rng.cpp).  Run from Python threads, every
// chunk pays ~15 us of thread-pool and interpreter overhead under the GIL (the box's 16
// no-op tasks take ~220 us; tools/replay_draws_bench.py), which is more than a class's
// normals cost to draw: the frame's normals phase sat on the GPU's critical path at ~0.38 ms.
// Here one call runs all chunks of a draw on torch's intra-op thread pool (at::parallel_for)
// with the GIL released (ctypes): the same samplers (Tensor::exponential_ / normal_ /
// uniform_ on a CPUGeneratorImpl), so the values are the Python chunks' bit for bit.
//
// Host code only (links libtorch_cpu); built by gpmdm_amd/build.py into
// gpmdm_amd/libgpmdm_replay.so and loaded by replay.py after torch.
#include <ATen/ATen.h>
#include <ATen/CPUGeneratorImpl.h>
#include <ATen/Parallel.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>

namespace {

constexpr int64_t kStateBytes = 5056;   // torch.Generator.get_state() of a CPU generator

enum Kind : int { kExponential = 0, kNormal = 1, kUniform = 2 };

thread_local std::string g_err;

void run_chunk(int kind, double* dst, int64_t a, int64_t b, const uint8_t* state) {
  at::Tensor st = at::empty({kStateBytes}, at::kByte);
  std::memcpy(st.data_ptr<uint8_t>(), state, kStateBytes);
  at::Generator gen = at::make_generator<at::CPUGeneratorImpl>();
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

}  // namespace

extern "C" {

// Fill dst[bounds[2k] : bounds[2k+1]) for k < n_chunks with torch's sampler `kind`
// (0 exponential_(1), 1 normal_(0, 1), 2 uniform_(0, 1)), chunk k drawn from a generator in
// the state states[k * 5056 ...].  Chunks may overlap only if the caller orders them so
// (they run concurrently: a later chunk overwriting an earlier one's values must be a
// separate call).  Returns 0, or -1 with the message in gpmdm_replay_last_error().
int gpmdm_replay_draw_chunks(int kind, double* dst, const int64_t* bounds, const uint8_t* states,
                             int64_t n_chunks) {
  if (!dst || !bounds || !states || n_chunks < 0 || kind < 0 || kind > 2) {
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
  try {
    at::parallel_for(0, n_chunks, 1, [&](int64_t k0, int64_t k1) {
      for (int64_t k = k0; k < k1; ++k) {
        try {
          run_chunk(kind, dst, bounds[2 * k], bounds[2 * k + 1], states + k * kStateBytes);
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> lock(err_mu);
          if (!failed.exchange(1)) first_err = e.what();
        }
      }
    });
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

// Threads of the pool the chunks run on (at::get_num_threads()).
int gpmdm_replay_threads(void) { return at::get_num_threads(); }

const char* gpmdm_replay_last_error(void) { return g_err.c_str(); }

}  // extern "C"
