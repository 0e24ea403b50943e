// roctx ranges from native code without a link-time dependency: the roctx
// library is resolved once with dlopen (rocprofiler-sdk's, then the legacy
// roctracer one); without it the ranges are no-ops.  The ranges show up in
// `rocprofv3 --marker-trace` next to the kernels they enclose.
#pragma once

#include <dlfcn.h>
#include <cstdlib>
#include <cstring>

namespace dmp {
namespace trace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* off = std::getenv("DMP_DISABLE_ROCTX");
    if (off && std::strcmp(off, "1") == 0) return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "libroctx64.so.4", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
      if (!h) h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (push && pop) return;
      push = nullptr;
      pop = nullptr;
    }
  }
};

inline const Roctx& roctx() {
  static Roctx r;
  return r;
}

// RAII range: `dmp::trace::Range r("ddp.bucket");`
class Range {
 public:
  explicit Range(const char* name) : on_(roctx().push != nullptr) {
    if (on_) roctx().push(name);
  }
  ~Range() {
    if (on_) roctx().pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace dmp
