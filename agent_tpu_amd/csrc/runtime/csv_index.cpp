// CsvTable: mmap + record index + excel-dialect field parser.
// See include/atpu/csv.h for the contract; parity target is the reference's
// csv.DictReader use in /root/reference/ops/csv_shard.py:17-24.
#include "atpu/csv.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace atpu {

namespace {

inline bool is_eol(char c) { return c == '\n' || c == '\r'; }

// Per-field parser states (CPython _csv.c names, minus the escapechar states
// the excel dialect never enters).
enum class St { kStartField, kInField, kInQuoted, kQuoteInQuoted };

}  // namespace

CsvTable::CsvTable(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
  struct stat st {};
  if (::fstat(fd_, &st) != 0) {
    ::close(fd_);
    throw std::runtime_error("cannot stat " + path);
  }
  size_ = static_cast<uint64_t>(st.st_size);
  mtime_ns_ = static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
  if (size_ > 0) {
    void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) {
      ::close(fd_);
      throw std::runtime_error("mmap failed for " + path);
    }
    ::madvise(p, size_, MADV_SEQUENTIAL);
    data_ = static_cast<const char*>(p);
  }
  const char* dir = std::getenv("ATPU_CSV_INDEX_DIR");
  std::string cache;
  if (dir && *dir) {
    uint64_t h = 1469598103934665603ULL;  // FNV-1a of the path
    for (unsigned char c : path_) h = (h ^ c) * 1099511628211ULL;
    char name[40];
    std::snprintf(name, sizeof(name), "/%016llx.rowidx", static_cast<unsigned long long>(h));
    cache = std::string(dir) + name;
  }
  if (cache.empty() || !load_index_cache(cache)) {
    build_index();
    if (!cache.empty()) save_index_cache(cache);
  }
  if (data_) ::madvise(const_cast<char*>(data_), size_, MADV_RANDOM);
}

CsvTable::~CsvTable() {
  if (data_) ::munmap(const_cast<char*>(data_), size_);
  if (fd_ >= 0) ::close(fd_);
}

int CsvTable::column_index(const std::string& name) const {
  // csv.DictReader's dict(zip(...)) keeps the LAST duplicate key
  for (int i = static_cast<int>(header_.size()) - 1; i >= 0; --i)
    if (header_[i] == name) return i;
  return -1;
}

size_t CsvTable::parse_record(size_t pos, std::vector<std::string>* fields) const {
  std::string cur;
  St st = St::kStartField;
  size_t i = pos;
  auto save = [&] {
    if (fields) fields->push_back(cur);
    cur.clear();
  };
  for (; i < size_; ++i) {
    const char c = data_[i];
    switch (st) {
      case St::kStartField:
        if (is_eol(c)) { save(); return i + 1; }
        if (c == '"') { st = St::kInQuoted; break; }
        if (c == ',') { save(); break; }
        if (fields) cur.push_back(c);
        st = St::kInField;
        break;
      case St::kInField:
        if (is_eol(c)) { save(); return i + 1; }
        if (c == ',') { save(); st = St::kStartField; break; }
        if (fields) cur.push_back(c);
        break;
      case St::kInQuoted:
        if (c == '"') { st = St::kQuoteInQuoted; break; }
        if (fields) cur.push_back(c);
        break;
      case St::kQuoteInQuoted:
        if (c == '"') { if (fields) cur.push_back('"'); st = St::kInQuoted; break; }
        if (c == ',') { save(); st = St::kStartField; break; }
        if (is_eol(c)) { save(); return i + 1; }
        if (fields) cur.push_back(c);
        st = St::kInField;  // non-strict: text after a closing quote is kept
        break;
    }
  }
  save();  // end of data acts as the last line's EOL
  return i;
}

void CsvTable::parse_field(size_t pos, int col, std::string& out, size_t max_bytes) const {
  out.clear();
  int field = 0;
  St st = St::kStartField;
  auto push = [&](char c) {
    if (field == col && out.size() < max_bytes) out.push_back(c);
  };
  for (size_t i = pos; i < size_; ++i) {
    const char c = data_[i];
    switch (st) {
      case St::kStartField:
        if (is_eol(c)) return;
        if (c == '"') { st = St::kInQuoted; break; }
        if (c == ',') { if (field++ == col) return; break; }
        push(c);
        st = St::kInField;
        break;
      case St::kInField:
        if (is_eol(c)) return;
        if (c == ',') { if (field++ == col) return; st = St::kStartField; break; }
        push(c);
        break;
      case St::kInQuoted:
        if (c == '"') { st = St::kQuoteInQuoted; break; }
        push(c);
        break;
      case St::kQuoteInQuoted:
        if (c == '"') { push('"'); st = St::kInQuoted; break; }
        if (c == ',') { if (field++ == col) return; st = St::kStartField; break; }
        if (is_eol(c)) return;
        push(c);
        st = St::kInField;
        break;
    }
  }
}

namespace {
constexpr char kIdxMagic[8] = {'A', 'T', 'P', 'U', 'I', 'D', 'X', '1'};
}

bool CsvTable::load_index_cache(const std::string& file) {
  FILE* f = std::fopen(file.c_str(), "rb");
  if (!f) return false;
  char magic[8];
  uint64_t size = 0, plen = 0, n = 0;
  int64_t mtime = 0;
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kIdxMagic, 8) == 0 &&
            std::fread(&size, 8, 1, f) == 1 && std::fread(&mtime, 8, 1, f) == 1 && std::fread(&plen, 8, 1, f) == 1 &&
            size == size_ && mtime == mtime_ns_ && plen == path_.size() && plen < (1u << 20);
  if (ok) {
    std::string p(plen, '\0');
    ok = std::fread(&p[0], 1, plen, f) == plen && p == path_ && std::fread(&n, 8, 1, f) == 1 && n <= size_;
    if (ok) {
      starts_.resize(n);
      ok = n == 0 || std::fread(starts_.data(), 8, n, f) == n;
      for (size_t i = 0; ok && i < n; ++i) ok = starts_[i] < size_ && (i == 0 || starts_[i] > starts_[i - 1]);
    }
  }
  std::fclose(f);
  if (!ok) {
    starts_.clear();
    return false;
  }
  header_.clear();
  if (size_ > 0) parse_record(0, &header_);
  index_from_cache_ = true;
  return true;
}

void CsvTable::save_index_cache(const std::string& file) const {
  const std::string tmp = file + ".tmp" + std::to_string(::getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;  // best effort: an unwritable cache dir only costs the rebuild
  const uint64_t size = size_, plen = path_.size(), n = starts_.size();
  const int64_t mtime = mtime_ns_;
  bool ok = std::fwrite(kIdxMagic, 1, 8, f) == 8 && std::fwrite(&size, 8, 1, f) == 1 &&
            std::fwrite(&mtime, 8, 1, f) == 1 && std::fwrite(&plen, 8, 1, f) == 1 &&
            std::fwrite(path_.data(), 1, plen, f) == plen && std::fwrite(&n, 8, 1, f) == 1 &&
            (n == 0 || std::fwrite(starts_.data(), 8, n, f) == n);
  ok = (std::fclose(f) == 0) && ok;
  if (ok)
    std::rename(tmp.c_str(), file.c_str());
  else
    std::remove(tmp.c_str());
}

void CsvTable::build_index() {
  size_t pos = 0;
  if (size_ == 0) return;
  if (is_eol(data_[0])) {
    pos = 1;  // first line is blank: DictReader's fieldnames become []
  } else {
    pos = parse_record(0, &header_);
  }
  starts_.reserve(size_ / 64 + 16);
  // Boundary-only scan: a quote opens a quoted field only at field start; in
  // an unquoted field (or after a closing quote) quotes are literal.
  while (pos < size_) {
    while (pos < size_ && is_eol(data_[pos])) ++pos;  // blank records: skipped
    if (pos >= size_) break;
    starts_.push_back(pos);
    size_t i = pos;
    bool field_start = true;
    bool done = false;
    while (i < size_ && !done) {
      if (field_start && data_[i] == '"') {
        ++i;
        for (;;) {
          const void* q = std::memchr(data_ + i, '"', size_ - i);
          if (!q) { i = size_; break; }
          i = static_cast<size_t>(static_cast<const char*>(q) - data_) + 1;
          if (i < size_ && data_[i] == '"') { ++i; continue; }  // "" escape
          break;
        }
      }
      field_start = false;
      while (i < size_) {
        const char c = data_[i];
        if (c == ',') { field_start = true; ++i; break; }
        if (is_eol(c)) { ++i; done = true; break; }
        ++i;
      }
    }
    pos = i;
  }
}

void CsvTable::parse_row(size_t row, std::vector<std::string>& fields) const {
  if (row >= starts_.size()) throw std::out_of_range("row out of range");
  fields.clear();
  parse_record(starts_[row], &fields);
}

int64_t CsvTable::extract_column(size_t start, size_t n, int col, uint8_t* out, size_t cap,
                                 int32_t* offsets, size_t max_bytes, int threads) const {
  if (start > starts_.size()) start = starts_.size();
  n = std::min(n, starts_.size() - start);
  threads = std::max(1, std::min<int>(threads, static_cast<int>((n + 255) / 256)));
  std::vector<std::string> blobs(threads);
  std::vector<std::vector<int32_t>> lens(threads);
  auto work = [&](int t) {
    const size_t lo = start + n * t / threads, hi = start + n * (t + 1) / threads;
    std::string field;
    auto& blob = blobs[t];
    auto& ln = lens[t];
    ln.reserve(hi - lo);
    for (size_t r = lo; r < hi; ++r) {
      if (col >= 0) parse_field(starts_[r], col, field, max_bytes);
      else field.clear();
      blob += field;
      ln.push_back(static_cast<int32_t>(field.size()));
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
  }
  size_t total = 0;
  for (auto& b : blobs) total += b.size();
  if (total > cap) return -1;
  size_t off = 0, row = 0;
  offsets[0] = 0;
  for (int t = 0; t < threads; ++t) {
    std::memcpy(out + off, blobs[t].data(), blobs[t].size());
    for (int32_t len : lens[t]) {
      off += static_cast<size_t>(len);
      offsets[++row] = static_cast<int32_t>(off);
    }
  }
  return static_cast<int64_t>(total);
}

namespace {

// Python float() syntax minus '_' separators, surrounding whitespace ignored; false on a bad value
bool field_to_double(const std::string& field, double* out) {
  size_t b = 0, e = field.size();
  while (b < e && std::isspace(static_cast<unsigned char>(field[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(field[e - 1]))) --e;
  const std::string v = field.substr(b, e - b);
  char* end = nullptr;
  const double d = v.empty() ? 0.0 : std::strtod(v.c_str(), &end);
  if (v.empty() || end != v.c_str() + v.size()) return false;
  *out = d;
  return true;
}

}  // namespace

double CsvTable::parse_double(size_t row, int col) const {
  if (row >= starts_.size()) throw std::out_of_range("row out of range");
  std::string field;
  parse_field(starts_[row], col, field, 4096);
  double d = 0.0;
  if (!field_to_double(field, &d)) throw std::invalid_argument("could not convert string to float: '" + field + "'");
  return d;
}

void CsvTable::release_pages(uint64_t begin, uint64_t end) const {
  if (!data_ || end <= begin) return;
  const uint64_t pg = static_cast<uint64_t>(::sysconf(_SC_PAGESIZE));
  const uint64_t b = (begin + pg - 1) / pg * pg, e = std::min(end, size_) / pg * pg;
  if (e > b) ::madvise(const_cast<char*>(data_) + b, e - b, MADV_DONTNEED);
}

void CsvTable::extract_doubles(size_t start, size_t n, int col, double* out, int threads) const {
  if (start > starts_.size()) start = starts_.size();
  n = std::min(n, starts_.size() - start);
  threads = std::max(1, std::min<int>(threads, static_cast<int>((n + 4095) / 4096)));
  std::vector<std::string> errors(threads);
  auto work = [&](int t) {
    const size_t lo = start + n * t / threads, hi = start + n * (t + 1) / threads;
    std::string field;
    for (size_t r = lo; r < hi; ++r) {
      parse_field(starts_[r], col, field, 4096);
      if (!field_to_double(field, &out[r - start])) {
        errors[t] = "could not convert string to float: '" + field + "'";
        return;
      }
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
  }
  for (const auto& e : errors)
    if (!e.empty()) throw std::invalid_argument(e);
}

}  // namespace atpu
