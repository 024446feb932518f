// roctx ranges for rocprofv3 --marker-trace.
//
// Enabled by MI355X_TRACE=1 (read once). The roctx library of
// rocprofiler-sdk is dlopen'ed on first use so the module has no link-time
// dependency on it and costs one branch per call when tracing is off.
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "atpu/runtime.h"

namespace atpu {
namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();
using MarkFn = void (*)(const char*);

struct Roctx {
  bool enabled = false;
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = std::getenv("MI355X_TRACE");
    if (!env || (std::strcmp(env, "1") != 0 && std::strcmp(env, "true") != 0)) return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      r.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
      r.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
      r.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
      if (r.push && r.pop) {
        r.enabled = true;
        return;
      }
    }
  });
  return r;
}

}  // namespace

bool trace_enabled() { return roctx().enabled; }

void trace_push(const char* name) {
  const Roctx& r = roctx();
  if (r.enabled) r.push(name);
}

void trace_pop() {
  const Roctx& r = roctx();
  if (r.enabled) r.pop();
}

void trace_mark(const char* name) {
  const Roctx& r = roctx();
  if (r.enabled && r.mark) r.mark(name);
}

}  // namespace atpu
