// Sampling CPU profiler for the serving process (the reference
// profiles its JVM engine with YourKit / JVisualVM, testing/profiling/engine/
// README.md:3-30; here the engine is native, so it samples itself).
//
// Per-thread CPU-time timers (threads alive at start()) deliver SIGPROF
// every 1/hz seconds of each thread's CPU time to that thread; the handler stores that thread's program counter
// into a preallocated array (async-signal-safe: one atomic increment, one
// store).  stop() returns each sample as (module path, offset in module) for
// offline symbolisation (llvm-symbolizer), so hidden-visibility functions of
// the extension resolve through its .symtab.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace sca::prof {

bool start(int hz, size_t max_samples = size_t(1) << 21);
// (module, offset) -> samples, most frequent first; empty module = unknown.
std::vector<std::pair<std::pair<std::string, uint64_t>, uint64_t>> stop();

}  // namespace sca::prof
