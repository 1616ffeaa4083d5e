// Replay-mode host helper: positions of torch's CPU generator along its own stream.
//
// The reference draws every random number of a frame from torch's global CPU generator
// (gpmdm_pf.py:137-213): Exp(1) for the switch, per-class normals, uniforms for the
// resample.  torch's samplers are serial, ~13 ms per frame at P = 100k on one core -- twice
// the GPU frame.  They become parallel without changing a bit when each chunk of a draw runs
// torch's own sampler on a private generator placed exactly where the serial draw would have
// been when it reached that chunk.  This file computes those placements: torch's generator is
// an MT19937 (ATen MT19937RNGEngine.h) serialised by Generator.get_state() as
// CPUGeneratorImplState (5056 bytes: seed, left, seeded, next, state[624] as uint64, the
// double-normal cache, the float-normal cache).  A walk twists the MT state forward once over
// a stretch of the stream (every 624 outputs) and keeps the twisted blocks, so the state
// after any number of draws of that stretch is a copy of one block plus two counters.
//
// One random64 draw (uniform_real<double>, exponential, the normal fills) consumes two
// 32-bit outputs.  Host code only: no GPU.
#include <algorithm>
#include <cstdint>
#include <memory>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/gpmdm_hip.h"
#include "status.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
// CPUGeneratorImplState layout (torch.Generator.get_state(): 5056 bytes)
constexpr size_t kOffLeft = 8, kOffNext = 16, kOffState = 24;
static_assert(GPMDM_TORCH_GEN_STATE_BYTES == 5056, "torch CPU generator state size");

inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & kUpper) | (v & kLower)) >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
}

// ATen's mt19937::next_state (in place: p[i] = p[i + M] ^ twist(p[i], p[i + 1]) for
// i < N - M from old words; then from the words just written), out of place: o -> n.  The
// first loop reads old words only and the second depends on words N - M = 227 back, so both
// vectorise; the result is the in-place twist's word for word.
void next_state(const uint32_t* __restrict o, uint32_t* __restrict n) {
  for (int i = 0; i < kN - kM; ++i) n[i] = o[i + kM] ^ twist(o[i], o[i + 1]);
  for (int i = kN - kM; i < kN - 1; ++i) n[i] = n[i + kM - kN] ^ twist(o[i], o[i + 1]);
  n[kN - 1] = n[kM - 1] ^ twist(o[kN - 1], n[0]);
}

}  // namespace

struct gpmdm_rng_walk {
  std::vector<uint8_t> tmpl;        // the start state's bytes (seed, flags, normal caches)
  int32_t left0 = 0;
  uint32_t next0 = 0;
  std::vector<uint32_t> s0;         // MT words at the start
  std::unique_ptr<uint32_t[]> blocks;   // words after twist 1, 2, ... (kN each)
  long long n_blocks = 0, cap_blocks = 0;
  long long cap_outputs = 0;        // outputs covered
};

extern "C" {

// (Re)start a walk at `state` covering n_draws draws; the block buffer is kept when it is
// large enough (first touches of a fresh 5 MB buffer cost more than the twists).
static int walk_reset(gpmdm_rng_walk* w, const uint8_t* state, int64_t n_draws) {
  int32_t left;
  uint64_t next;
  std::memcpy(&left, state + kOffLeft, sizeof(left));
  std::memcpy(&next, state + kOffNext, sizeof(next));
  if (left < 1 || left > kN || next > (uint64_t)kN)
    return gpmdm::fail(GPMDM_E_INVALID, "not a torch CPU generator state (left / next out of range)");
  w->tmpl.assign(state, state + GPMDM_TORCH_GEN_STATE_BYTES);
  w->left0 = left;
  w->next0 = (uint32_t)next;
  w->s0.resize(kN);
  for (int i = 0; i < kN; ++i) {
    uint64_t v;
    std::memcpy(&v, state + kOffState + 8 * (size_t)i, sizeof(v));
    w->s0[i] = (uint32_t)v;
  }
  const long long outputs = 2 * (long long)n_draws;
  const long long before = w->left0 - 1;                 // outputs before the first twist
  const long long after = outputs > before ? outputs - before : 0;
  const long long nb = (after + kN - 1) / kN;
  if (!w->blocks || nb > w->cap_blocks) {
    w->blocks.reset(new (std::nothrow) uint32_t[(size_t)std::max<long long>(nb, 1) * kN]);
    w->cap_blocks = w->blocks ? std::max<long long>(nb, 1) : 0;
    if (!w->blocks) return gpmdm::fail(GPMDM_E_NOMEM, "rng walk blocks");
  }
  w->n_blocks = nb;
  const uint32_t* prev = w->s0.data();
  for (long long b = 0; b < nb; ++b) {
    uint32_t* cur = w->blocks.get() + (size_t)b * kN;
    next_state(prev, cur);
    prev = cur;
  }
  w->cap_outputs = before + nb * kN;
  return GPMDM_OK;
}

int gpmdm_rng_walk_create(const uint8_t* state, int64_t n_draws, gpmdm_rng_walk_t* out) {
  CHECK(state && out && n_draws >= 0 && n_draws < (1ll << 40), "bad argument");
  *out = nullptr;
  auto* w = new (std::nothrow) gpmdm_rng_walk();
  if (!w) return gpmdm::fail(GPMDM_E_NOMEM, "rng walk");
  const int rc = walk_reset(w, state, n_draws);
  if (rc) {
    delete w;
    return rc;
  }
  *out = w;
  return GPMDM_OK;
}

int gpmdm_rng_walk_reset(gpmdm_rng_walk_t w, const uint8_t* state, int64_t n_draws) {
  CHECK(w && state && n_draws >= 0 && n_draws < (1ll << 40), "bad argument");
  return walk_reset(w, state, n_draws);
}

// The generator state after `draws` random64 draws from the walk's start, with the
// normal-cache bytes of `cache_from` (NULL: the start state's) -- normal_fill, exponential_
// and uniform_ never touch those caches; the serial normal path of tensors under 16 values does.
int gpmdm_rng_walk_state(gpmdm_rng_walk_t w, int64_t draws, const uint8_t* cache_from, uint8_t* out) {
  CHECK(w && out && draws >= 0, "bad argument");
  const long long t = 2 * (long long)draws;
  CHECK(t <= w->cap_outputs, "draw offset beyond the walk");
  std::memcpy(out, cache_from ? cache_from : w->tmpl.data(), GPMDM_TORCH_GEN_STATE_BYTES);
  std::memcpy(out, w->tmpl.data(), kOffState);           // seed, left, seeded, next (left/next set below)
  const uint32_t* words;
  int32_t left;
  uint64_t next;
  const long long before = w->left0 - 1;
  if (t <= before) {
    words = w->s0.data();
    left = w->left0 - (int32_t)t;
    next = w->next0 + (uint64_t)t;
  } else {
    const long long tp = t - before;                     // outputs from the first twist on
    const long long b = (tp + kN - 1) / kN;              // twists done (>= 1)
    const long long j = tp - (b - 1) * kN;               // outputs taken from block b (1 .. kN)
    words = w->blocks.get() + (size_t)(b - 1) * kN;
    left = (int32_t)(kN + 1 - j);
    next = (uint64_t)j;
  }
  std::memcpy(out + kOffLeft, &left, sizeof(left));
  std::memcpy(out + kOffNext, &next, sizeof(next));
  for (int i = 0; i < kN; ++i) {
    const uint64_t v = words[i];
    std::memcpy(out + kOffState + 8 * (size_t)i, &v, sizeof(v));
  }
  return GPMDM_OK;
}

// gpmdm_rng_walk_state at n offsets, one state after the other in out (n x 5056 bytes).
int gpmdm_rng_walk_states(gpmdm_rng_walk_t w, int64_t n, const int64_t* draws, const uint8_t* cache_from,
                          uint8_t* out) {
  CHECK(w && out && draws && n >= 0, "bad argument");
  for (int64_t k = 0; k < n; ++k) TRY(gpmdm_rng_walk_state(w, draws[k], cache_from, out + k * GPMDM_TORCH_GEN_STATE_BYTES));
  return GPMDM_OK;
}

int gpmdm_rng_walk_destroy(gpmdm_rng_walk_t w) {
  delete w;
  return GPMDM_OK;
}

}  // extern "C"
