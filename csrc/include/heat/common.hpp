// Common definitions for the MI355X-native heat-diffusion engine.
//
// Error handling replaces the reference's total absence of return-code checks
// (cuda/cuda_heat.cu:178-242, mpi/mpi_heat_improved_persistent_stat.c:48-308):
// every HIP / RCCL / socket call goes through a checking macro that throws
// heat::Error with file:line, and the C API converts it into an error string.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace heat {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] void throw_error(const char* file, int line, const std::string& msg);

std::string strprintf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }
inline int64_t round_down(int64_t a, int64_t b) { return (a / b) * b; }

}  // namespace heat

#define HEAT_CHECK(cond, ...)                                                  \
  do {                                                                         \
    if (!(cond))                                                               \
      ::heat::throw_error(__FILE__, __LINE__,                                  \
                          std::string("check failed: " #cond ": ") +           \
                              ::heat::strprintf(__VA_ARGS__));                 \
  } while (0)

#define HIP_CHECK(expr)                                                        \
  do {                                                                         \
    hipError_t e__ = (expr);                                                   \
    if (e__ != hipSuccess)                                                     \
      ::heat::throw_error(__FILE__, __LINE__,                                  \
                          std::string(#expr " -> ") + hipGetErrorString(e__)); \
  } while (0)
