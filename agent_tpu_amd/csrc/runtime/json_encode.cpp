// Native JSON encoding of classify results (the per-row Python dicts of a
// node-sized shard ran below one GPU's engine rate). The reference returns one small
// top-k list per call (ref ops/map_classify_tpu.py:77-82); a DP map over the node
// returns 8 x 49k rows/s of them, so the rows are written straight from the int32 /
// fp32 top-k arrays. Floats use the shortest round-trip form (std::to_chars), the
// same values Python's json module emits for float(np.float32(x)).
#include <charconv>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "atpu/runtime.h"

namespace atpu {
namespace {

inline void put_int(std::string& o, int64_t v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof(b), v);
  o.append(b, r.ptr);
}

inline void put_float(std::string& o, float f) {
  const double v = static_cast<double>(f);
  if (!std::isfinite(v)) throw std::invalid_argument("topk json: non-finite score");
  char b[40];
  auto r = std::to_chars(b, b + sizeof(b), v);
  // Python writes integral floats as "1.0"; to_chars gives "1"
  bool has = false;
  for (char* p = b; p < r.ptr; ++p)
    if (*p == '.' || *p == 'e' || *p == 'n' || *p == 'i') has = true;
  o.append(b, r.ptr);
  if (!has) o.append(".0");
}

}  // namespace

std::string topk_json(int64_t start_row, const int32_t* idx, const float* score, int64_t n, int k, int mode) {
  if (n < 0 || k < 1) throw std::invalid_argument("topk json: bad shape");
  std::string o;
  o.reserve(static_cast<size_t>(n) * (mode == 0 ? 24 + 40 * k : 4 + 22 * k) + 2);
  o.push_back('[');
  for (int64_t r = 0; r < n; ++r) {
    if (r) o.push_back(',');
    const int32_t* ir = idx + r * k;
    const float* sr = score + r * k;
    if (mode == 0) {  // [{"row":R,"topk":[{"index":I,"score":S},...]},...]
      o.append("{\"row\":");
      put_int(o, start_row + r);
      o.append(",\"topk\":[");
      for (int j = 0; j < k; ++j) {
        if (j) o.push_back(',');
        o.append("{\"index\":");
        put_int(o, ir[j]);
        o.append(",\"score\":");
        put_float(o, sr[j]);
        o.push_back('}');
      }
      o.append("]}");
    } else {  // columns: [[I,...],...] (mode 1) or [[S,...],...] (mode 2)
      o.push_back('[');
      for (int j = 0; j < k; ++j) {
        if (j) o.push_back(',');
        if (mode == 1) put_int(o, ir[j]);
        else put_float(o, sr[j]);
      }
      o.push_back(']');
    }
  }
  o.push_back(']');
  return o;
}

}  // namespace atpu
