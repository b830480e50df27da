// trace.cc — timer sections (trace.h) and the gls_timer_* C ABI: the
// reference's TimerOutput wall-time statistics (timer.h:194-338,
// print_wall_time_statistics) for the sections this library runs.
#include "trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gls_op.h"
#include "common.h"

namespace gls
{
namespace
{
struct Entry
{
  std::string name;
  int64_t     calls   = 0;
  double      host_ms = 0.0;
  double      gpu_ms  = 0.0;
  int64_t     gpu_n   = 0; // calls with a GPU time
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
};

struct Tally
{
  std::mutex                 mu;
  bool                       on = false;
  std::vector<Entry>         entries;
  std::map<std::string, int> index;
  std::vector<hipEvent_t>    pool; // events of the current device (one-GPU processes)
  int64_t                    gen = 0; // gls_timer_reset count (sections open across a reset drop out)

  Tally()
  {
    const char *e = std::getenv("GLS_TIMING");
    on            = e && e[0] == '1';
  }
  hipEvent_t
  take()
  {
    if (!pool.empty())
      {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
      }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess)
      {
        (void)hipGetLastError();
        return nullptr;
      }
    return e;
  }
  // elapsed times of an entry's pending event pairs (waits for them)
  void
  collect(Entry &en)
  {
    for (auto &p : en.pending)
      {
        float ms = 0.f;
        if (hipEventSynchronize(p.second) == hipSuccess &&
            hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess)
          {
            en.gpu_ms += ms;
            ++en.gpu_n;
          }
        else
          (void)hipGetLastError();
        pool.push_back(p.first);
        pool.push_back(p.second);
      }
    en.pending.clear();
  }
};

Tally &
tally()
{
  static Tally t;
  return t;
}

double
now_ms()
{
  return std::chrono::duration<double, std::milli>(
           std::chrono::steady_clock::now().time_since_epoch())
    .count();
}
} // namespace

bool
timing_enabled()
{
  return tally().on;
}

Section::Section(const char *name, hipStream_t s)
{
  roctxRangePushA(name);
  Tally &t = tally();
  if (!t.on)
    return;
  std::lock_guard<std::mutex> lk(t.mu);
  auto it = t.index.find(name);
  if (it == t.index.end())
    {
      it = t.index.emplace(name, (int)t.entries.size()).first;
      t.entries.push_back(Entry{});
      t.entries.back().name = name;
    }
  entry  = it->second;
  gen    = t.gen;
  stream = s;
  e0     = t.take();
  if (e0 && hipEventRecord(e0, s) != hipSuccess)
    {
      (void)hipGetLastError();
      t.pool.push_back(e0);
      e0 = nullptr;
    }
  t0 = now_ms();
}

Section::~Section()
{
  if (entry >= 0)
    {
      Tally                      &t = tally();
      std::lock_guard<std::mutex> lk(t.mu);
      if (gen != t.gen)
        {
          if (e0)
            t.pool.push_back(e0);
          roctxRangePop();
          return;
        }
      Entry &en = t.entries[(size_t)entry];
      ++en.calls;
      en.host_ms += now_ms() - t0;
      if (e0)
        {
          hipEvent_t e1 = t.take();
          if (e1 && hipEventRecord(e1, stream) == hipSuccess)
            en.pending.emplace_back(e0, e1);
          else
            {
              (void)hipGetLastError();
              t.pool.push_back(e0);
              if (e1)
                t.pool.push_back(e1);
            }
          // bounded memory: a long timed run collects as it goes
          if (en.pending.size() >= 4096)
            t.collect(en);
        }
    }
  roctxRangePop();
}
} // namespace gls

extern "C" {

glsStatus
gls_timer_enable(int on, int *was_on)
{
  GLS_TRY
  gls::Tally                 &t = gls::tally();
  std::lock_guard<std::mutex> lk(t.mu);
  if (was_on)
    *was_on = t.on ? 1 : 0;
  t.on = on != 0;
  GLS_CATCH
}

glsStatus
gls_timer_reset(void)
{
  GLS_TRY
  gls::Tally                 &t = gls::tally();
  std::lock_guard<std::mutex> lk(t.mu);
  for (auto &en : t.entries)
    t.collect(en); // (returns their events to the pool)
  t.entries.clear();
  t.index.clear();
  ++t.gen;
  GLS_CATCH
}

// caller-opened sections (the reference's MyScope around its own code:
// newton::solve, richardson::solve, direct::solve, solver_nl.cc / solver_l.cc)
glsStatus
gls_timer_begin(const char *name, void *stream, void **token)
{
  GLS_TRY
  if (!name || !token)
    throw std::runtime_error("gls_timer_begin: null argument");
  *token = new gls::Section(name, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_timer_end(void *token)
{
  GLS_TRY
  if (!token)
    throw std::runtime_error("gls_timer_end: null token");
  delete static_cast<gls::Section *>(token);
  GLS_CATCH
}

int64_t
gls_timer_n_sections(void)
{
  gls::Tally                 &t = gls::tally();
  std::lock_guard<std::mutex> lk(t.mu);
  return (int64_t)t.entries.size();
}

glsStatus
gls_timer_section(int64_t i, char *name, int64_t name_len, int64_t *calls, double *host_ms,
                  double *gpu_ms)
{
  GLS_TRY
  gls::Tally                 &t = gls::tally();
  std::lock_guard<std::mutex> lk(t.mu);
  if (i < 0 || i >= (int64_t)t.entries.size())
    throw std::runtime_error("gls_timer_section: index out of range");
  gls::Entry &en = t.entries[(size_t)i];
  t.collect(en);
  if (name && name_len > 0)
    {
      std::strncpy(name, en.name.c_str(), (size_t)name_len - 1);
      name[name_len - 1] = '\0';
    }
  if (calls)
    *calls = en.calls;
  if (host_ms)
    *host_ms = en.host_ms;
  if (gpu_ms)
    *gpu_ms = en.gpu_n > 0 ? en.gpu_ms : -1.0;
  GLS_CATCH
}

int64_t
gls_timer_report(char *buf, int64_t len)
{
  std::string out;
  {
    gls::Tally                 &t = gls::tally();
    std::lock_guard<std::mutex> lk(t.mu);
    char line[512];
    std::snprintf(line, sizeof line, "%-56s %10s %14s %14s %14s\n", "section", "calls",
                  "host ms", "GPU ms", "GPU ms/call");
    out += line;
    for (auto &en : t.entries)
      {
        t.collect(en);
        std::snprintf(line, sizeof line, "%-56s %10lld %14.3f %14.3f %14.5f\n", en.name.c_str(),
                      (long long)en.calls, en.host_ms, en.gpu_ms,
                      en.gpu_n > 0 ? en.gpu_ms / (double)en.gpu_n : 0.0);
        out += line;
      }
  }
  if (buf && len > 0)
    {
      std::strncpy(buf, out.c_str(), (size_t)len - 1);
      buf[len - 1] = '\0';
    }
  return (int64_t)out.size() + 1;
}

} // extern "C"
