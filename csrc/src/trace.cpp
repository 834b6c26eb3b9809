// roctx ranges, loaded lazily (see anx/trace.hpp).
#include "anx/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace anx {

namespace {
using PushFn = int (*)(const char*);
using PopFn = int (*)();
struct Roctx {
  PushFn push = nullptr;
  PopFn pop = nullptr;
};
const Roctx& lib() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("ANX_ROCTX");
    if (e && e[0] == '0') return;
    for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                             "libroctx64.so"}) {
      void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      auto push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
      auto pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
      if (push && pop) {
        r.push = push;
        r.pop = pop;
        return;
      }
    }
  });
  return r;
}
}  // namespace

bool roctx_enabled() { return lib().push != nullptr; }
void roctx_push(const char* name) {
  if (lib().push) lib().push(name);
}
void roctx_pop() {
  if (lib().pop) lib().pop();
}

}  // namespace anx
