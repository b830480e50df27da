// trace.h — the reference's timer sections (timer.h:342-413 MyScope over
// dealii::TimerOutput, the section names of operator_ns.cc, multigrid.cc,
// solver_l.cc) as roctx ranges and, when timing is on, a per-section tally
// of host wall time and of the GPU time between two events on the section's
// stream (gls_timer_* in include/gls_op.h).
//
// Off (the default; GLS_TIMING=1 in the environment or gls_timer_enable
// turns it on), a section is one roctx push / pop pair: a no-op unless a
// tool (rocprofv3 --marker-trace) is attached.  On, each section also takes
// two pooled events; their elapsed times are collected when the tally is
// read, so timing adds no host synchronisation to the calls it measures.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace gls
{
bool timing_enabled();

class Section
{
public:
  Section(const char *name, hipStream_t s);
  Section(const std::string &name, hipStream_t s)
    : Section(name.c_str(), s)
  {}
  ~Section();
  Section(const Section &)            = delete;
  Section &operator=(const Section &) = delete;

private:
  int         entry = -1; // tally entry, -1: timing off
  int64_t     gen    = 0;
  hipStream_t stream = nullptr;
  hipEvent_t  e0     = nullptr;
  double      t0     = 0.0;
};
} // namespace gls
