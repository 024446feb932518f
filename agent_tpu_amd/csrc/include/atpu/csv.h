// Memory-mapped CSV table with a byte-offset record index.
//
// Replaces the reference's O(start_row) csv.DictReader scan
// (/root/reference/ops/csv_shard.py:9-26): the index is built once per file and
// any row range is then served in O(rows). Record/field semantics follow
// CPython's _csv module (excel dialect: ',' delimiter, '"' quote, doublequote,
// non-strict) so shard outputs are byte-identical to the reference.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace atpu {

class CsvTable {
 public:
  explicit CsvTable(const std::string& path);
  ~CsvTable();
  CsvTable(const CsvTable&) = delete;
  CsvTable& operator=(const CsvTable&) = delete;

  const std::string& path() const { return path_; }
  uint64_t file_size() const { return size_; }
  int64_t mtime_ns() const { return mtime_ns_; }
  // number of non-blank data records after the header
  size_t num_rows() const { return starts_.size(); }
  // true when the row index came from the on-disk cache (ATPU_CSV_INDEX_DIR)
  bool index_from_cache() const { return index_from_cache_; }
  const std::vector<std::string>& header() const { return header_; }
  int column_index(const std::string& name) const;

  // Parse data record `row` into its fields.
  void parse_row(size_t row, std::vector<std::string>& fields) const;

  // Parse field `col` of rows [start, start+n) as doubles (Python float()
  // syntax minus '_' separators; surrounding whitespace ignored). Throws
  // std::invalid_argument naming the first bad value.
  void extract_doubles(size_t start, size_t n, int col, double* out, int threads) const;

  // Field `col` of data record `row` as a double, exactly as extract_doubles parses it
  // (same std::invalid_argument on a bad value). The streamed risk reduce's host fallback.
  double parse_double(size_t row, int col) const;

  // Raw bytes of the mapped file and the byte range of data record `row` (its start and
  // the start of the next record, or the file end): the streamed risk reduce ships these
  // bytes to the GPU, which parses the field itself (K13).
  const char* data() const { return data_; }
  uint64_t row_begin(size_t row) const { return starts_[row]; }
  uint64_t row_end(size_t row) const { return row + 1 < starts_.size() ? starts_[row + 1] : size_; }
  // Drop this process's mapping of the pages inside [begin, end) (page-aligned inward):
  // a streamed pass over a large shard keeps its resident set bounded (the pages stay in
  // the page cache; a later access faults them back in).
  void release_pages(uint64_t begin, uint64_t end) const;

  // Pack field `col` of rows [start, start+n) into `out` (capacity `cap`
  // bytes) with int32 offsets[n+1]; each value truncated to `max_bytes`.
  // Work is split over `threads` host threads. Returns bytes written, or -1
  // if `cap` is too small.
  int64_t extract_column(size_t start, size_t n, int col, uint8_t* out, size_t cap,
                         int32_t* offsets, size_t max_bytes, int threads) const;

 private:
  // Parse one record beginning at byte `pos`; returns the byte index just past
  // the record terminator(s). If `fields` is null only the boundary is found.
  size_t parse_record(size_t pos, std::vector<std::string>* fields) const;
  // Extract only field `col` of the record starting at `pos` into `out`.
  void parse_field(size_t pos, int col, std::string& out, size_t max_bytes) const;
  void build_index();
  // persisted row index: <ATPU_CSV_INDEX_DIR>/<hash>.rowidx,
  // valid for the same (path, size, mtime)
  bool load_index_cache(const std::string& file);
  void save_index_cache(const std::string& file) const;
  bool index_from_cache_ = false;

  std::string path_;
  const char* data_ = nullptr;
  uint64_t size_ = 0;
  int64_t mtime_ns_ = 0;
  int fd_ = -1;
  std::vector<std::string> header_;
  std::vector<uint64_t> starts_;
};

}  // namespace atpu
