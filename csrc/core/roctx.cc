#include "roctx.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>
#include <cstring>

namespace sca::trace {

bool roctx_on() {
  static const bool on = [] {
    const char* v = std::getenv("SCA_ROCTX");
    return v && std::strcmp(v, "0") != 0 && *v;
  }();
  return on;
}

uint64_t range_start(const char* message) { return uint64_t(roctxRangeStartA(message)); }

void range_stop(uint64_t id) { roctxRangeStop(roctx_range_id_t(id)); }

}  // namespace sca::trace
