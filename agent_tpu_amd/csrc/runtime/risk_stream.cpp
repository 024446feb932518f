// Streamed risk_accumulate over a CSV column (BASELINE config 5).
//
// The reference makes one pass over its input (ref ops/risk_accumulate.py:34-77). Round 3
// parsed a whole rank shard to host fp64 first (host memory grew with shard_size, and the
// parse, the copy and the reduce ran one after another). Here the shard goes through in
// chunks, three stages overlapped:
//
//   host threads                     copy stream                 compute stream
//   mmap'd record bytes -> pinned    hipMemcpyAsync -> HBM  -->  csv_parse_reduce (K13+K12)
//   slot i % 2 (+ record offsets)                                 reduce_stats_accumulate
//
// The GPU finds and parses the field itself (head_reduce.hip), so the host only copies raw
// record bytes: no per-value parse on the critical path. Records the device fast path cannot
// take come back as a row list and are parsed on the host (CsvTable::parse_double, the strtod
// path of extract_doubles): same values, same errors. Host memory is two pinned slots, and the
// consumed file pages are released behind the cursor, so the resident set does not grow with
// the shard.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "atpu/common.h"
#include "atpu/csv.h"
#include "atpu/kernels.h"
#include "atpu/risk_stream.h"

namespace atpu {

RiskStream::RiskStream(size_t slot_bytes, size_t slot_rows, int fb_cap)
    : slot_bytes_(std::max<size_t>(slot_bytes, 1 << 16)),
      slot_rows_(std::max<size_t>(slot_rows, 1024)),
      fb_cap_(std::max(fb_cap, 1)) {
  ATPU_CHECK(slot_bytes_ < (size_t(1) << 32), "risk stream: slot bytes must fit 32-bit record offsets");
  ATPU_HIP_CHECK(hipGetDevice(&dev_));
  for (auto& s : slots_) {
    ATPU_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_text), slot_bytes_, hipHostMallocDefault));
    ATPU_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.h_offs), (slot_rows_ + 1) * sizeof(uint32_t),
                                 hipHostMallocDefault));
    ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_text), slot_bytes_));
    ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_offs), (slot_rows_ + 1) * sizeof(uint32_t)));
    ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s.d_part), kCsvMaxBlocks * 4 * sizeof(double)));
    ATPU_HIP_CHECK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    ATPU_HIP_CHECK(hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming));
  }
  ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d_acc_), 4 * sizeof(double)));
  ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d_fb_count_), sizeof(int)));
  ATPU_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d_fb_rows_), size_t(fb_cap_) * sizeof(int64_t)));
}

RiskStream::~RiskStream() {
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(dev_);
  for (auto& s : slots_) {
    if (s.used) (void)hipEventSynchronize(s.consumed);
    (void)hipHostFree(s.h_text);
    (void)hipHostFree(s.h_offs);
    (void)hipFree(s.d_text);
    (void)hipFree(s.d_offs);
    (void)hipFree(s.d_part);
    (void)hipEventDestroy(s.copied);
    (void)hipEventDestroy(s.consumed);
  }
  (void)hipFree(d_acc_);
  (void)hipFree(d_fb_count_);
  (void)hipFree(d_fb_rows_);
  (void)hipSetDevice(cur);
}

namespace {

// copy [src, src + n) to dst on up to `threads` host threads (page faults of the mapped
// file and the memcpy both parallelise)
void parallel_copy(uint8_t* dst, const char* src, size_t n, int threads) {
  threads = std::max(1, std::min<int>(threads, static_cast<int>(n >> 22)));  // >= 4 MiB per thread
  if (threads == 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    const size_t lo = n * t / threads, hi = n * (t + 1) / threads;
    pool.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

RiskStream::Result RiskStream::run(const CsvTable& t, size_t start, size_t n, int col, hipStream_t copy,
                                   hipStream_t compute, int threads) {
  int cur = -1;
  ATPU_HIP_CHECK(hipGetDevice(&cur));
  ATPU_CHECK(cur == dev_, "risk stream: used on another device than it was built on");
  ATPU_CHECK(col >= 0, "risk stream: bad column");
  Result res;
  if (start > t.num_rows()) start = t.num_rows();
  const size_t end = start + std::min(n, t.num_rows() - start);
  ATPU_HIP_CHECK(hipMemsetAsync(d_fb_count_, 0, sizeof(int), compute));
  bool first = true;
  size_t a = start;
  while (a < end) {
    const uint64_t base = t.row_begin(a);
    size_t b = std::min(end, a + slot_rows_);
    if (t.row_end(b - 1) - base > slot_bytes_) {
      // largest b with its records' bytes within the slot
      size_t lo = a, hi = b;  // invariant: records [a, lo) fit, [a, hi) do not
      while (hi - lo > 1) {
        const size_t mid = lo + (hi - lo) / 2;
        if (t.row_end(mid - 1) - base <= slot_bytes_) lo = mid;
        else hi = mid;
      }
      b = lo;
      if (b == a) {  // one record larger than a slot: the host parses it
        res.host_rows.push_back(static_cast<int64_t>(a));
        a += 1;
        continue;
      }
    }
    const uint64_t nbytes = t.row_end(b - 1) - base;
    const int nr = static_cast<int>(b - a);
    Slot& s = slots_[res.chunks & 1];
    if (s.used) ATPU_HIP_CHECK(hipEventSynchronize(s.copied));  // its pinned buffers are free again
    parallel_copy(s.h_text, t.data() + base, nbytes, threads);
    for (int r = 0; r < nr; ++r) s.h_offs[r] = static_cast<uint32_t>(t.row_begin(a + r) - base);
    s.h_offs[nr] = static_cast<uint32_t>(nbytes);
    t.release_pages(base, base + nbytes);
    if (s.used) ATPU_HIP_CHECK(hipStreamWaitEvent(copy, s.consumed, 0));  // device buffers consumed
    ATPU_HIP_CHECK(hipMemcpyAsync(s.d_text, s.h_text, nbytes, hipMemcpyHostToDevice, copy));
    ATPU_HIP_CHECK(hipMemcpyAsync(s.d_offs, s.h_offs, (nr + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, copy));
    ATPU_HIP_CHECK(hipEventRecord(s.copied, copy));
    ATPU_HIP_CHECK(hipStreamWaitEvent(compute, s.copied, 0));
    const int blocks = csv_parse_blocks(nr);
    csv_parse_reduce(s.d_text, s.d_offs, nr, col, static_cast<int64_t>(a), s.d_part, blocks, d_fb_count_,
                     d_fb_rows_, fb_cap_, compute);
    reduce_stats_accumulate(s.d_part, blocks, d_acc_, first, compute);
    ATPU_HIP_CHECK(hipEventRecord(s.consumed, compute));
    s.used = true;
    first = false;
    res.chunks += 1;
    res.bytes += static_cast<int64_t>(nbytes);
    a = b;
  }
  if (!first) {
    double acc[4];
    int fb = 0;
    ATPU_HIP_CHECK(hipMemcpyAsync(acc, d_acc_, sizeof(acc), hipMemcpyDeviceToHost, compute));
    ATPU_HIP_CHECK(hipMemcpyAsync(&fb, d_fb_count_, sizeof(int), hipMemcpyDeviceToHost, compute));
    ATPU_HIP_CHECK(hipStreamSynchronize(compute));
    res.count = static_cast<int64_t>(acc[0]);
    res.sum = acc[1];
    res.min = acc[2];
    res.max = acc[3];
    res.fallback_total = fb;
    if (fb > 0) {
      const int k = std::min(fb, fb_cap_);
      std::vector<int64_t> rows(k);
      ATPU_HIP_CHECK(hipMemcpy(rows.data(), d_fb_rows_, k * sizeof(int64_t), hipMemcpyDeviceToHost));
      res.host_rows.insert(res.host_rows.end(), rows.begin(), rows.end());
    }
  }
  std::sort(res.host_rows.begin(), res.host_rows.end());
  res.overflow = res.fallback_total > fb_cap_;
  return res;
}

}  // namespace atpu
