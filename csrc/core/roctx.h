// roctx ranges: with SCA_ROCTX=1 the engine opens one range per
// request and per node call, and every GPU micro-batch opens one from launch to
// completion, so `rocprofv3 --marker-trace --kernel-trace` shows the inference
// graph next to the kernels it launched.  Ranges are started / stopped by id
// (roctxRangeStartA / roctxRangeStop): a node call starts on one thread and
// finishes on another (continuations), which push/pop ranges cannot express.
#pragma once

#include <cstdint>

namespace sca::trace {

bool roctx_on();  // SCA_ROCTX=1, read once
uint64_t range_start(const char* message);
void range_stop(uint64_t id);

}  // namespace sca::trace
