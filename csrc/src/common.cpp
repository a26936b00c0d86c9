// Error helpers (HIP-free so host-only builds such as the sanitizer self-test
// can link them).
#include "heat/common.hpp"

#include <cstdarg>
#include <cstring>

namespace heat {

void throw_error(const char* file, int line, const std::string& msg) {
  const char* base = std::strrchr(file, '/');
  throw Error(strprintf("%s:%d: %s", base ? base + 1 : file, line, msg.c_str()));
}

std::string strprintf(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return buf;
}

}  // namespace heat
