// CPU twin of kernels/rand_init.hip: the same (seed, stream, index) -> value function
// (atpu/rand.h), so host-built packs (fp32 oracle, HF-parity tests, CPU-only agents) hold
// exactly the weights a GPU-built pack holds. Threads split the range; each element is
// independent, so the result does not depend on the thread count.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "atpu/rand.h"
#include "atpu/runtime.h"

namespace atpu {

void rand_fill_host(void* dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0,
                    float scale1, int threads) {
  if (n <= 0) return;
  const uint64_t key = rnd::stream_key(seed, sid);
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const float f = (float)rnd::ih4(key, (uint64_t)i) * (i < n0 ? scale0 : scale1);
      if (f32) static_cast<float*>(dst)[i] = f;
      else static_cast<uint16_t*>(dst)[i] = rnd::f2bf_rne(f);
    }
  };
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 65536));
  if (threads <= 1) {
    work(0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(work, n * t / threads, n * (t + 1) / threads);
  for (auto& th : pool) th.join();
}

}  // namespace atpu
