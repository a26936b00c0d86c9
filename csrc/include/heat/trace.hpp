// roctx phase ranges (reference: Paraver traces of scatter / steady state /
// gather / Allreduce, Heat.pdf p.8-11).  libroctx64 is loaded
// lazily with dlopen so the engine has no hard dependency on it; when no
// profiler is attached the calls are near-free.  rocprofv3 --marker-trace
// records them.  Disable with HEAT_ROCTX=0.
#pragma once

namespace heat {

void trace_push(const char* name);
void trace_pop();

struct TraceRange {
  explicit TraceRange(const char* name) { trace_push(name); }
  ~TraceRange() { trace_pop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace heat
