// Streamed CSV-column reduce for risk_accumulate (see runtime/risk_stream.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <vector>

#include "atpu/csv.h"

namespace atpu {

class RiskStream {
 public:
  // slot_bytes: record bytes per chunk (pinned + device, x2 slots); slot_rows: records per
  // chunk; fb_cap: device fast-path misses recorded per run (more -> Result::overflow)
  RiskStream(size_t slot_bytes, size_t slot_rows, int fb_cap);
  ~RiskStream();
  RiskStream(const RiskStream&) = delete;
  RiskStream& operator=(const RiskStream&) = delete;

  struct Result {
    // count / sum / min / max of the records the device parsed
    int64_t count = 0;
    double sum = 0.0, min = DBL_MAX, max = -DBL_MAX;
    // records the host must parse (device fast-path misses, records over a slot), ascending
    std::vector<int64_t> host_rows;
    int64_t fallback_total = 0;  // device misses (may exceed the recorded list)
    bool overflow = false;       // more misses than fb_cap: the caller re-parses the range on the host
    int64_t chunks = 0;
    int64_t bytes = 0;
  };
  // Field `col` of records [start, start+n) of `t`, streamed through the current device.
  // `copy` carries the H2D copies, `compute` the kernels; returns after `compute` drained.
  Result run(const CsvTable& t, size_t start, size_t n, int col, hipStream_t copy, hipStream_t compute,
             int threads);

  size_t slot_bytes() const { return slot_bytes_; }
  size_t slot_rows() const { return slot_rows_; }

 private:
  struct Slot {
    uint8_t* h_text = nullptr;
    uint32_t* h_offs = nullptr;
    uint8_t* d_text = nullptr;
    uint32_t* d_offs = nullptr;
    double* d_part = nullptr;
    hipEvent_t copied = nullptr;    // H2D done: the pinned buffers may be refilled
    hipEvent_t consumed = nullptr;  // kernels done: the device buffers may be overwritten
    bool used = false;
  };
  Slot slots_[2];
  double* d_acc_ = nullptr;
  int* d_fb_count_ = nullptr;
  int64_t* d_fb_rows_ = nullptr;
  size_t slot_bytes_, slot_rows_;
  int fb_cap_;
  int dev_ = 0;
};

}  // namespace atpu
