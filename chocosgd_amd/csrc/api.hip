// Library-wide C-ABI plumbing: per-thread error text, version, profiling hooks.
#include "choco_common.h"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <unordered_map>
#include <mutex>
#include <string>
#include <vector>

namespace choco {

static thread_local char g_err[1024] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CHOCO_ERR_HIP, "launch of %s failed: %s", what, hipGetErrorString(e));
  return CHOCO_OK;
}

// ---------------------------------------------------------------- profiling
struct PendingEv {
  std::string name;
  hipEvent_t a, b;
  bool closed;
};
static std::atomic<bool> g_prof_on{false};
static std::mutex g_prof_mu;
static std::vector<PendingEv> g_pending;
static std::map<std::string, std::pair<double, int64_t>> g_acc;
static std::vector<std::string> g_filter;  // only these kernel names are timed (empty = all)
static std::vector<hipEvent_t> g_free_ev;  // events are reused: no create/destroy per launch

static thread_local ProfArm g_armed{nullptr, nullptr};
// launches per kernel name, counted whether or not timing is on (choco_launch_count: the
// bench's warm-hit rates; names are the string literals of the call sites)
static std::mutex g_cnt_mu;
static std::unordered_map<const char*, int64_t> g_launches;

void profile_begin(const char* name, hipStream_t) {
  g_armed = ProfArm{nullptr, nullptr};
  {
    std::lock_guard<std::mutex> g(g_cnt_mu);
    ++g_launches[name];
  }
  if (!g_prof_on.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> g(g_prof_mu);
  if (!g_filter.empty() && std::find(g_filter.begin(), g_filter.end(), std::string(name)) == g_filter.end()) return;
  PendingEv p{name, nullptr, nullptr, false};  // closed once a launch takes the pair
  for (hipEvent_t* e : {&p.a, &p.b}) {
    if (!g_free_ev.empty()) {
      *e = g_free_ev.back();
      g_free_ev.pop_back();
    } else if (hipEventCreate(e) != hipSuccess) {
      return;
    }
  }
  g_armed = ProfArm{p.a, p.b};
  g_pending.push_back(p);
}

void profile_end(const char*, hipStream_t) { g_armed = ProfArm{nullptr, nullptr}; }

ProfArm profile_take() {
  const ProfArm r = g_armed;
  g_armed = ProfArm{nullptr, nullptr};
  if (r.a) {  // the launch records this pair: only now may it be read (events are reused)
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (auto it = g_pending.rbegin(); it != g_pending.rend(); ++it)
      if (it->a == r.a) {
        it->closed = true;
        break;
      }
  }
  return r;
}

static void profile_drain_locked() {
  for (auto& p : g_pending) {
    if (p.closed) {
      float ms = 0.f;
      // (an armed pair that never reached a launch is not closed: skipped)
      if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        auto& e = g_acc[p.name];
        e.first += ms;
        e.second += 1;
      }
    }
    g_free_ev.push_back(p.a);
    g_free_ev.push_back(p.b);
  }
  g_pending.clear();
}

}  // namespace choco

using namespace choco;

CHOCO_API int choco_version(void) { return 1; }

CHOCO_API int choco_last_error(char* buf, size_t len) {
  size_t n = strlen(g_err);
  if (buf && len) {
    size_t c = n < len - 1 ? n : len - 1;
    memcpy(buf, g_err, c);
    buf[c] = 0;
  }
  return (int)n;
}

CHOCO_API int choco_profile_enable(int32_t on) {
  g_prof_on.store(on != 0);
  return CHOCO_OK;
}

CHOCO_API int choco_profile_filter(const char* names) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_filter.clear();
  std::string all = names ? names : "";
  size_t p = 0;
  while (p <= all.size()) {
    const size_t q = std::min(all.find(',', p), all.size());
    if (q > p) g_filter.push_back(all.substr(p, q - p));
    p = q + 1;
  }
  return CHOCO_OK;
}

CHOCO_API int choco_profile_read(const char* name, double* total_ms, int64_t* count) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  profile_drain_locked();
  auto it = g_acc.find(name ? name : "");
  if (total_ms) *total_ms = it == g_acc.end() ? 0.0 : it->second.first;
  if (count) *count = it == g_acc.end() ? 0 : it->second.second;
  return CHOCO_OK;
}

CHOCO_API int64_t choco_launch_count(const char* name) {
  std::lock_guard<std::mutex> g(g_cnt_mu);
  int64_t n = 0;
  for (const auto& e : g_launches)
    if (name && strcmp(e.first, name) == 0) n += e.second;
  return n;
}

CHOCO_API int choco_profile_reset(void) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  profile_drain_locked();
  g_acc.clear();
  return CHOCO_OK;
}
