// roctx phase ranges via dlopen (see trace.hpp).
#include "heat/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace heat {
namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();

struct Roctx {
  PushFn push = nullptr;
  PopFn pop = nullptr;
  Roctx() {
    const char* e = std::getenv("HEAT_ROCTX");
    if (e && e[0] == '0') return;
    // rocprofv3 (rocprofiler-sdk) intercepts the SDK's roctx library; the
    // legacy roctracer libroctx64 is only a fallback (its ranges are not
    // seen by rocprofv3 --marker-trace).
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libroctx64.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};

Roctx& roctx() {
  static Roctx r;
  return r;
}

}  // namespace

void trace_push(const char* name) {
  auto& r = roctx();
  if (r.push) r.push(name);
}

void trace_pop() {
  auto& r = roctx();
  if (r.pop) r.pop();
}

}  // namespace heat
