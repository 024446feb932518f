// Host runtime pieces: tokenizer twin, device query, CSV -> pinned -> device
// staging pipeline.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "atpu/csv.h"

namespace atpu {

// Host twin of the K1 GPU tokenizer (identical output, see tokenize.hip).
void tokenize_host(const uint8_t* text, const int32_t* offsets, int32_t* ids, int32_t* lens, int B, int S, int vocab,
                   int max_row_bytes);
// Per document (words joined by single 0x20 bytes): its distinct hash-token ids, ascending,
// and the index of the first word producing each (at most cap tokens per word); doc_off[B+1]
// delimits each document's entries in ids / word_of (detokenization maps, runtime/summarize.py)
void word_maps_host(const uint8_t* text, const int64_t* offsets, int B, int vocab, int cap,
                    std::vector<int32_t>& ids, std::vector<int64_t>& word_of, std::vector<int64_t>& doc_off);

struct DeviceInfo {
  int index;
  std::string name;
  std::string arch;
  size_t total_bytes;
  size_t free_bytes;
  int cus;
  int clock_khz;
};
// Properties of every visible device; free HBM only for device ``mem_of`` (-1: the
// current device), so a DP rank never creates contexts on its peers' GPUs.
std::vector<DeviceInfo> device_query(int mem_of = -1);

// Classify top-k [n, k] -> JSON text. mode 0: reference-style rows
// [{"row":start+r,"topk":[{"index":i,"score":s},...]},...]; 1: [[index,...],...];
// 2: [[score,...],...]. Floats in the shortest round-trip form.
struct RiskStats {
  int64_t count;
  double sum, min, max;
};
// risk_accumulate over a Python list (see runtime/risk_parse.cpp); needs the GIL.
// mode 0 values, 1 items[field]. False = Python exception set.
bool risk_stats_pylist(struct _object* list, int mode, struct _object* field, RiskStats* st,
                       std::vector<double>* out);

std::string topk_json(int64_t start_row, const int32_t* idx, const float* score, int64_t n, int k, int mode);

// Double-buffered CSV column -> pinned host -> device pipeline.
//  submit(slot, ...)  : background thread extracts rows into slot's pinned
//                       buffer (after the slot's previous H2D has finished).
//  upload(slot, ...)  : waits for extraction, hipMemcpyAsync's text+offsets on
//                       the copy stream (after the compute stream released the
//                       slot's device buffers), and makes the compute stream
//                       wait for the copy.
//  release(slot, s)   : records on the compute stream that the device buffers
//                       of `slot` have been consumed.
class HostStager {
 public:
  HostStager(int slots, size_t text_capacity, int max_rows);
  ~HostStager();
  HostStager(const HostStager&) = delete;
  HostStager& operator=(const HostStager&) = delete;

  void submit(int slot, const CsvTable* table, size_t start, size_t n, int col, size_t max_bytes, int threads);
  // returns {rows, bytes}
  std::pair<int64_t, int64_t> upload(int slot, void* dev_text, size_t dev_text_cap, void* dev_offsets,
                                     hipStream_t copy_stream, hipStream_t compute_stream);
  void release(int slot, hipStream_t compute_stream);
  // Device time of the H2D copies (hipEvent pairs around each upload's memcpys, after its
  // wait for the slot's previous consumer), summed since the last call. Synchronizes on
  // the outstanding pairs. {milliseconds, copies}.
  std::pair<double, int64_t> take_h2d_ms();
  int slots() const { return static_cast<int>(slots_.size()); }
  size_t text_capacity() const { return text_cap_; }
  // host view of a slot's staged data (valid after upload/wait)
  const uint8_t* host_text(int slot) const { return slots_[slot].text; }
  const int32_t* host_offsets(int slot) const { return slots_[slot].offsets; }
  std::pair<int64_t, int64_t> wait(int slot);

 private:
  struct Slot {
    uint8_t* text = nullptr;
    int32_t* offsets = nullptr;
    hipEvent_t copied = nullptr;    // H2D done -> pinned buffer reusable
    hipEvent_t consumed = nullptr;  // compute done with device buffers
    hipEvent_t t0 = nullptr, t1 = nullptr;  // timing pair around the last upload's copies
    bool has_t = false;
    bool has_copy = false;
    bool has_consume = false;
    int64_t rows = 0, bytes = 0;
    bool pending = false;
    std::string error;
  };
  void worker();

  void settle_timing(Slot& s);
  std::vector<Slot> slots_;
  double h2d_ms_ = 0.0;
  int64_t h2d_n_ = 0;
  size_t text_cap_;
  int max_rows_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::function<void()>> queue_;
  bool stop_ = false;
  std::thread thread_;
};

// roctx ranges (MI355X_TRACE=1; no-ops otherwise), see runtime/trace.cpp
bool trace_enabled();
// CPU twin of rand_fill (kernels.h): the same values, on `threads` host threads
void rand_fill_host(void* dst, int64_t n, bool f32, uint64_t seed, uint64_t sid, float scale0, int64_t n0,
                    float scale1, int threads);

void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

}  // namespace atpu
