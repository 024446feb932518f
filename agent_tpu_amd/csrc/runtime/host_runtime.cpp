// Host runtime: tokenizer twin, HIP device query, pinned double-buffer stager.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "atpu/common.h"
#include "atpu/runtime.h"

namespace atpu {

// ------------------------------------------------------------ tokenizer twin
namespace {
constexpr uint32_t kBasis = 2166136261u, kPrime = 16777619u;
constexpr int kPieceBytes = 24;
inline int cls_of(uint32_t c) {
  if (c == 0x20 || (c >= 0x09 && c <= 0x0D) || c < 0x20 || c == 0x7F) return 0;
  if ((c >= 0x21 && c <= 0x2F) || (c >= 0x3A && c <= 0x40) || (c >= 0x5B && c <= 0x60) || (c >= 0x7B && c <= 0x7E))
    return 1;
  return 2;
}
inline uint32_t step(uint32_t h, uint32_t c) {
  if (c >= 'A' && c <= 'Z') c += 32;
  return (h ^ c) * kPrime;
}
}  // namespace

namespace {
// Hash tokens of bytes [p, p+n) (the tokenize_host rules), at most cap; emit(id) per token.
template <typename Emit>
int tokenize_bytes(const uint8_t* p, int n, int cap, uint32_t mod, Emit emit) {
  const uint32_t cont = step(step(kBasis, '#'), '#');
  int nt = 0;
  for (int i = 0; i < n && nt < cap;) {
    const int c = cls_of(p[i]);
    if (c == 0) { ++i; continue; }
    if (c == 1) {
      emit(static_cast<int32_t>(1000u + step(kBasis, p[i]) % mod));
      ++nt;
      ++i;
      continue;
    }
    int j = i;
    while (j < n && cls_of(p[j]) == 2) ++j;
    for (int b0 = i, piece = 0; b0 < j && nt < cap; b0 += kPieceBytes, ++piece) {
      uint32_t h = piece == 0 ? kBasis : cont;
      for (int k = b0; k < std::min(j, b0 + kPieceBytes); ++k) h = step(h, p[k]);
      emit(static_cast<int32_t>(1000u + h % mod));
      ++nt;
    }
    i = j;
  }
  return nt;
}
}  // namespace

void tokenize_host(const uint8_t* text, const int32_t* offsets, int32_t* ids, int32_t* lens, int B, int S, int vocab,
                   int max_row_bytes) {
  if (S < 2 || vocab <= 1000) throw std::invalid_argument("tokenize_host: bad S/vocab");
  const uint32_t mod = static_cast<uint32_t>(vocab - 1000);
  for (int r = 0; r < B; ++r) {
    const int n = std::min(offsets[r + 1] - offsets[r], max_row_bytes);
    int32_t* out = ids + static_cast<size_t>(r) * S;
    int32_t* w = out + 1;
    const int nt = tokenize_bytes(text + offsets[r], n, S - 2, mod, [&](int32_t id) { *w++ = id; });
    out[0] = 101;
    out[1 + nt] = 102;
    for (int j = nt + 2; j < S; ++j) out[j] = 0;
    lens[r] = nt + 2;
  }
}

void word_maps_host(const uint8_t* text, const int64_t* offsets, int B, int vocab, int cap,
                    std::vector<int32_t>& ids, std::vector<int64_t>& word_of, std::vector<int64_t>& doc_off) {
  if (vocab <= 1000 || cap < 1) throw std::invalid_argument("word_maps_host: bad vocab/cap");
  const uint32_t mod = static_cast<uint32_t>(vocab - 1000);
  doc_off.assign(1, 0);
  std::vector<std::pair<int32_t, int64_t>> v;  // (token id, word index), word-major
  for (int r = 0; r < B; ++r) {
    const uint8_t* p = text + offsets[r];
    const int64_t n = offsets[r + 1] - offsets[r];
    v.clear();
    int64_t word = 0;
    for (int64_t a = 0; a <= n;) {  // words are separated by exactly one 0x20 (the caller joins str.split())
      int64_t b = a;
      while (b < n && p[b] != 0x20) ++b;
      if (b > a) {
        tokenize_bytes(p + a, static_cast<int>(b - a), cap, mod, [&](int32_t id) { v.emplace_back(id, word); });
        ++word;
      }
      a = b + 1;
    }
    std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (size_t k = 0; k < v.size(); ++k) {
      if (k > 0 && v[k].first == v[k - 1].first) continue;  // first word producing the id
      ids.push_back(v[k].first);
      word_of.push_back(v[k].second);
    }
    doc_off.push_back(static_cast<int64_t>(ids.size()));
  }
}

// -------------------------------------------------------------- device query
std::vector<DeviceInfo> device_query(int mem_of) {
  std::vector<DeviceInfo> out;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return out;
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (mem_of < 0) mem_of = cur;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
    DeviceInfo d{};
    d.index = i;
    d.name = prop.name;
    d.arch = prop.gcnArchName;
    d.total_bytes = prop.totalGlobalMem;
    d.cus = prop.multiProcessorCount;
    d.clock_khz = prop.clockRate;
    size_t fr = 0, tot = 0;
    d.free_bytes = 0;
    if (i == mem_of && hipSetDevice(i) == hipSuccess && hipMemGetInfo(&fr, &tot) == hipSuccess) d.free_bytes = fr;
    out.push_back(d);
  }
  (void)hipSetDevice(cur);
  return out;
}

// --------------------------------------------------------------- HostStager
HostStager::HostStager(int slots, size_t text_capacity, int max_rows)
    : slots_(slots), text_cap_(text_capacity), max_rows_(max_rows) {
  ATPU_CHECK(slots >= 1 && slots <= 8, "stager: 1..8 slots");
  for (auto& s : slots_) {
    ATPU_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.text), text_cap_, hipHostMallocDefault));
    ATPU_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.offsets), sizeof(int32_t) * (max_rows_ + 1),
                                 hipHostMallocDefault));
    ATPU_HIP_CHECK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    ATPU_HIP_CHECK(hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming));
    ATPU_HIP_CHECK(hipEventCreate(&s.t0));
    ATPU_HIP_CHECK(hipEventCreate(&s.t1));
  }
  thread_ = std::thread([this] { worker(); });
}

HostStager::~HostStager() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  for (auto& s : slots_) {
    if (s.copied) (void)hipEventSynchronize(s.copied), (void)hipEventDestroy(s.copied);
    if (s.consumed) (void)hipEventDestroy(s.consumed);
    if (s.t1) (void)hipEventSynchronize(s.t1);
    if (s.t0) (void)hipEventDestroy(s.t0);
    if (s.t1) (void)hipEventDestroy(s.t1);
    if (s.text) (void)hipHostFree(s.text);
    if (s.offsets) (void)hipHostFree(s.offsets);
  }
}

void HostStager::worker() {
  for (;;) {
    std::function<void()> job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
      if (stop_ && queue_.empty()) return;
      job = std::move(queue_.front());
      queue_.erase(queue_.begin());
    }
    job();
  }
}

void HostStager::submit(int slot, const CsvTable* table, size_t start, size_t n, int col, size_t max_bytes,
                        int threads) {
  ATPU_CHECK(slot >= 0 && slot < slots(), "stager: bad slot");
  ATPU_CHECK(n <= static_cast<size_t>(max_rows_), "stager: too many rows for slot");
  std::lock_guard<std::mutex> g(mu_);
  Slot& s = slots_[slot];
  ATPU_CHECK(!s.pending, "stager: slot already pending");
  s.pending = true;
  s.error.clear();
  queue_.push_back([this, slot, table, start, n, col, max_bytes, threads] {
    Slot& sl = slots_[slot];
    std::string err;
    int64_t rows = 0, bytes = 0;
    try {
      if (sl.has_copy) ATPU_HIP_CHECK(hipEventSynchronize(sl.copied));  // pinned buffer free again
      const size_t have = table->num_rows() > start ? table->num_rows() - start : 0;
      rows = static_cast<int64_t>(std::min(n, have));
      bytes = table->extract_column(start, rows, col, sl.text, text_cap_, sl.offsets, max_bytes, threads);
      if (bytes < 0) err = "stager: text capacity exceeded";
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> g2(mu_);
      sl.rows = rows;
      sl.bytes = bytes;
      sl.error = err;
      sl.pending = false;
    }
    cv_.notify_all();
  });
  cv_.notify_all();
}

std::pair<int64_t, int64_t> HostStager::wait(int slot) {
  ATPU_CHECK(slot >= 0 && slot < slots(), "stager: bad slot");
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return !slots_[slot].pending; });
  if (!slots_[slot].error.empty()) throw std::runtime_error(slots_[slot].error);
  return {slots_[slot].rows, slots_[slot].bytes};
}

std::pair<int64_t, int64_t> HostStager::upload(int slot, void* dev_text, size_t dev_text_cap, void* dev_offsets,
                                               hipStream_t copy_stream, hipStream_t compute_stream) {
  auto [rows, bytes] = wait(slot);
  Slot& s = slots_[slot];
  ATPU_CHECK(static_cast<size_t>(bytes) <= dev_text_cap, "stager: device text buffer too small");
  if (s.has_consume) ATPU_HIP_CHECK(hipStreamWaitEvent(copy_stream, s.consumed, 0));
  settle_timing(s);  // the previous pair of this slot completed before its pinned buffer was refilled
  ATPU_HIP_CHECK(hipEventRecord(s.t0, copy_stream));  // after the wait: times the copies only
  if (bytes > 0) ATPU_HIP_CHECK(hipMemcpyAsync(dev_text, s.text, bytes, hipMemcpyHostToDevice, copy_stream));
  ATPU_HIP_CHECK(
      hipMemcpyAsync(dev_offsets, s.offsets, sizeof(int32_t) * (rows + 1), hipMemcpyHostToDevice, copy_stream));
  ATPU_HIP_CHECK(hipEventRecord(s.t1, copy_stream));
  s.has_t = true;
  ATPU_HIP_CHECK(hipEventRecord(s.copied, copy_stream));
  s.has_copy = true;
  if (compute_stream != copy_stream) ATPU_HIP_CHECK(hipStreamWaitEvent(compute_stream, s.copied, 0));
  return {rows, bytes};
}

void HostStager::settle_timing(Slot& s) {
  if (!s.has_t) return;
  ATPU_HIP_CHECK(hipEventSynchronize(s.t1));
  float ms = 0.f;
  ATPU_HIP_CHECK(hipEventElapsedTime(&ms, s.t0, s.t1));
  h2d_ms_ += ms;
  h2d_n_ += 1;
  s.has_t = false;
}

std::pair<double, int64_t> HostStager::take_h2d_ms() {
  for (auto& s : slots_) settle_timing(s);
  std::pair<double, int64_t> out{h2d_ms_, h2d_n_};
  h2d_ms_ = 0.0;
  h2d_n_ = 0;
  return out;
}

void HostStager::release(int slot, hipStream_t compute_stream) {
  ATPU_CHECK(slot >= 0 && slot < slots(), "stager: bad slot");
  ATPU_HIP_CHECK(hipEventRecord(slots_[slot].consumed, compute_stream));
  slots_[slot].has_consume = true;
}

}  // namespace atpu
