// Host-code sanitizer harness: drives the C++ CSV row index
// and the host tokenizer — the native code that parses untrusted input — over
// adversarial inputs, built with -fsanitize=address,undefined on the host
// side only (GPU ASan / xnack+ are not available on this pool). Any memory
// error aborts with a sanitizer report; exit 0 means clean.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <exception>
#include <random>
#include <string>
#include <vector>

#include "atpu/csv.h"
#include "atpu/runtime.h"

using atpu::CsvTable;

static std::string write_tmp(const std::string& body, int idx) {
  char path[256];
  std::snprintf(path, sizeof(path), "/tmp/atpu_san_%d_%d.csv", (int)getpid(), idx);
  FILE* f = std::fopen(path, "wb");
  if (!f) std::abort();
  std::fwrite(body.data(), 1, body.size(), f);
  std::fclose(f);
  return path;
}

static std::string random_csv(std::mt19937& rng) {
  static const char* atoms[] = {"a", "bc", ",", "\"", "\"\"", "\n", "\r\n", " ", "1.5", "-3e2", "x y", "\xc3\xa9",
                                "\"q,\"", "", "\r", "nan", "\t"};
  std::uniform_int_distribution<int> pick(0, (int)(sizeof(atoms) / sizeof(atoms[0])) - 1), len(0, 400);
  std::string s = "id,text,risk\n";
  const int n = len(rng);
  for (int i = 0; i < n; ++i) s += atoms[pick(rng)];
  return s;
}

static void exercise_table(const std::string& path);

static void exercise(const std::string& path) {
  try {
    exercise_table(path);
  } catch (const std::exception&) {  // malformed input may be rejected, never corrupt memory
  }
}

static void exercise_table(const std::string& path) {
  CsvTable t(path);
  std::vector<std::string> fields;
  const size_t rows = t.num_rows();
  for (size_t r = 0; r < rows; ++r) t.parse_row(r, fields);
  const int ncol = (int)t.header().size();
  for (int col = 0; col < std::max(ncol, 1); ++col) {
    for (size_t start : {size_t(0), rows / 2, rows}) {
      const size_t n = rows - start;
      std::vector<uint8_t> buf(64);
      std::vector<int32_t> offs(n + 1);
      t.extract_column(start, n, col, buf.data(), buf.size(), offs.data(), 16, 2);  // tiny cap: truncation
      std::vector<double> vals(n);
      try {
        t.extract_doubles(start, n, col, vals.data(), 2);
      } catch (const std::exception&) {  // non-numeric field: the documented ValueError path
      }
    }
  }
  t.column_index("text");
  t.column_index("missing");
}

int main() {
  std::mt19937 rng(1234);
  std::vector<std::string> fixed = {
      "", "id,text,risk", "id,text,risk\n", "id,text,risk\n\n\n1,a,2\n", "id,text\n1,\"unterminated\n",
      "id,text\n1,\"a\"\"b\"\n2,\"multi\nline\"\n3,last-no-newline", "\xef\xbb\xbfid,text\r\n1,crlf\r\n",
      std::string("id,text\n1,") + std::string(100000, 'z') + "\n", "a,b,c\n1\n1,2,3,4,5\n,,\n"};
  int idx = 0;
  for (const auto& body : fixed) {
    const std::string p = write_tmp(body, idx++);
    exercise(p);
    exercise(p);  // second open reads the persisted row index when ATPU_CSV_INDEX_DIR is set
    std::remove(p.c_str());
  }
  for (int it = 0; it < 300; ++it) {
    const std::string p = write_tmp(random_csv(rng), idx++);
    exercise(p);
    std::remove(p.c_str());
  }
  // host tokenizer over random bytes (UTF-8 fragments, long rows, short windows)
  std::uniform_int_distribution<int> byte(0, 255), rl(0, 3000);
  for (int it = 0; it < 200; ++it) {
    const int B = 1 + it % 7;
    std::vector<uint8_t> text;
    std::vector<int32_t> offs{0};
    for (int b = 0; b < B; ++b) {
      const int n = rl(rng);
      for (int i = 0; i < n; ++i) text.push_back((uint8_t)byte(rng));
      offs.push_back((int32_t)text.size());
    }
    const int S = 2 + it % 130;
    std::vector<int32_t> ids(B * S), lens(B);
    atpu::tokenize_host(text.data(), offs.data(), ids.data(), lens.data(), B, S, 30522, 1 + it * 17);
  }
  std::printf("host sanitizer harness: clean\n");
  return 0;
}
