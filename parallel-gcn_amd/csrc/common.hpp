// parallel-gcn_amd/csrc/common.hpp -- shared helpers for the HIP kernels and host runtime.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/pgcn.h"

namespace pgcn {

// Error handling: the reference exits on error under DEBUG_CUDA (include/utils.cuh:25-40);
// here every HIP call is checked and surfaces as an exception in C++ and as a status code
// at the C ABI.
struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string &msg) : std::runtime_error(msg), status(s) {}
};

#define PGCN_HIP(expr)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      throw ::pgcn::Error((int)e_, std::string(#expr) + " -> " + hipGetErrorString(e_) + \
                                       " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

#define PGCN_CHECK(cond, status, msg)                         \
  do {                                                        \
    if (!(cond)) throw ::pgcn::Error((status), (msg));        \
  } while (0)

// Status translation for the C ABI.
template <class F>
int guarded(F &&f) {
  try {
    f();
    return PGCN_OK;
  } catch (const Error &e) {
    fprintf(stderr, "[pgcn] %s\n", e.what());
    return e.status;
  } catch (const std::bad_alloc &) {
    return PGCN_E_NOMEM;
  } catch (const std::exception &e) {
    fprintf(stderr, "[pgcn] %s\n", e.what());
    return PGCN_E_INVALID;
  }
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline long long ceil_div(long long a, long long b) { return (a + b - 1) / b; }

constexpr int kWave = 64;   // CDNA wavefront
constexpr int kCUs = 256;   // MI355X compute units (8 XCDs x 32)

}  // namespace pgcn
