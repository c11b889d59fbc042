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

struct Loc {
  std::string module;  // empty: unknown
  uint64_t offset = 0; // in module (or the raw address)
};
struct Sample {
  std::vector<Loc> frames;  // [0] = interrupted PC, then callers (depth > 1)
  uint64_t count = 0;
};
struct Profile {
  int depth = 1;
  std::vector<Sample> samples;  // distinct stacks, most frequent first
};

// depth > 1 also records depth - 1 callers through the DWARF unwinder.
bool start(int hz, size_t max_samples = size_t(1) << 20, int depth = 1);
Profile stop();

}  // namespace sca::prof
