// Failure detector of a multi-process job: a host thread per rank that turns
// a collective which never completes (a stalled or dead peer, an RCCL
// asynchronous error, a launcher's SIGTERM after a peer failed) into a
// diagnosed exit instead of a silent hang.
//
// The reference gets this from its launcher (KungFu's kungfu-run stops the
// job when a peer exits: "exit on error: <k> tasks failed",
// tcb/slurm-2810438.out:133-137) and from TF's collective timeouts; with our
// own RCCL communicator (csrc/comm.hip) nothing else watches a collective,
// because torch's ProcessGroupNCCL watchdog is not in the picture.
//
// Model: the Python step loop beats a heartbeat (phase name, step, allowed
// seconds) before every step and every host wait; the thread wakes every
// poll interval and fires when
//   * the heartbeat's deadline passed (the rank is stuck in that phase),
//   * ncclCommGetAsyncError reports an error on a registered communicator,
//   * SIGTERM arrived (installed only while the watchdog runs).
// Firing aborts every registered communicator (ncclCommAbort, which also
// releases a host thread blocked on the stuck collective's stream), writes
// ONE JSON line {"status": "comm_error", ...} (rank 0 on stdout, the others
// on stderr), and _exit()s with a non-zero code.  Non-zero ranks wait a
// short grace first, so rank 0's line is written before a fail-fast
// launcher tears the job down.  Dry-run mode (tests) records the firing
// instead of exiting, and a test hook replaces ncclCommAbort.
#include "common.h"

#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" int kfb_rccl_destroy(void* comm, int abort);
extern "C" int kfb_rccl_async_error(void* comm);
extern "C" const char* kfb_rccl_error_string(int code);

namespace {

typedef int (*abort_fn_t)(void*);

struct Watchdog {
  std::mutex mu;
  std::vector<void*> comms;
  std::string phase = "startup";
  long step = -1;
  double deadline = 0.0;  // steady-clock seconds; 0: disarmed
  double timeout = 300.0;
  double armed_for = 0.0;
  double poll = 0.25;
  double grace = 2.0;
  int rank = 0;
  int exit_code = 3;
  int dry_run = 0;
  abort_fn_t abort_hook = nullptr;
  std::atomic<int> running{0};
  std::atomic<int> alive{0};  // the thread is inside loop()
  std::atomic<int> fired{0};
  std::atomic<int> aborts{0};
  std::string report;
  struct sigaction old_term;
  bool term_installed = false;
};

// never destroyed: the (detached) thread may still be polling while the
// process runs its exit handlers
Watchdog& g_wd = *new Watchdog;
volatile sig_atomic_t g_term_signal = 0;

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void on_term(int sig) { g_term_signal = sig; }

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if ((unsigned char)c < 0x20) {
      o += ' ';
    } else {
      o += c;
    }
  }
  return o;
}

// Caller holds g_wd.mu.
void fire_locked(const char* kind, const std::string& reason) {
  Watchdog& w = g_wd;
  if (w.fired.exchange(1)) return;
  for (void* c : w.comms) {
    if (w.abort_hook)
      w.abort_hook(c);
    else
      kfb_rccl_destroy(c, 1);
    w.aborts.fetch_add(1);
  }
  w.comms.clear();
  char buf[2048];
  snprintf(buf, sizeof(buf),
           "{\"status\": \"comm_error\", \"kind\": \"%s\", \"rank\": %d, \"step\": %ld, "
           "\"phase\": \"%s\", \"timeout_s\": %.1f, \"reason\": \"%s\", "
           "\"communicators_aborted\": %d}\n",
           kind, w.rank, w.step, json_escape(w.phase).c_str(), w.armed_for,
           json_escape(reason).c_str(), w.aborts.load());
  w.report = buf;
  w.deadline = 0.0;
  const int fd = w.rank == 0 ? 1 : 2;
  ssize_t off = 0, n = (ssize_t)strlen(buf);
  while (off < n) {
    const ssize_t k = write(fd, buf + off, n - off);
    if (k <= 0) break;
    off += k;
  }
  if (w.dry_run) return;
  if (w.rank != 0) usleep((useconds_t)(w.grace * 1e6));
  _exit(w.exit_code);
}

void loop() {
  Watchdog& w = g_wd;
  while (w.running.load()) {
    usleep((useconds_t)(w.poll * 1e6));
    std::lock_guard<std::mutex> lk(w.mu);
    if (!w.running.load() || w.fired.load()) continue;
    if (g_term_signal) {
      fire_locked("terminated", "signal " + std::to_string((int)g_term_signal) +
                                    " from the launcher (a peer failed or the job timed out)");
      continue;
    }
    // (with the test hook the handles are not real communicators)
    for (void* c : w.comms) {
      if (w.abort_hook) break;
      const int rc = kfb_rccl_async_error(c);
      // 1007: ncclInProgress (a non-blocking operation still running)
      if (rc != 0 && rc != 1007) {
        const char* m = kfb_rccl_error_string(rc);
        fire_locked("rccl_async_error", std::string("RCCL asynchronous error ") +
                                            std::to_string(rc) + ": " + (m ? m : "?"));
        break;
      }
    }
    if (!w.fired.load() && w.deadline > 0.0 && now_s() > w.deadline) {
      char r[256];
      snprintf(r, sizeof(r), "no progress for %.1f s (a peer stalled or a collective hung)",
               w.armed_for);
      fire_locked("deadline", r);
    }
  }
  w.alive.store(0);
}

}  // namespace

// Starts (or reconfigures) the watchdog.  timeout_s: the default allowance
// of a heartbeat; poll_s: wake-up interval; dry_run: record instead of exit.
KFB_API int kfb_watchdog_start(int rank, double timeout_s, double poll_s, int exit_code,
                               int dry_run, int handle_sigterm) {
  Watchdog& w = g_wd;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    w.rank = rank;
    w.timeout = timeout_s > 0 ? timeout_s : 300.0;
    w.poll = poll_s > 0 ? poll_s : 0.25;
    w.exit_code = exit_code;
    w.dry_run = dry_run;
    w.fired.store(0);
    w.aborts.store(0);
    w.report.clear();
    w.deadline = 0.0;
    w.phase = "startup";
    w.step = -1;
    g_term_signal = 0;
    if (handle_sigterm && !w.term_installed) {
      struct sigaction sa;
      memset(&sa, 0, sizeof(sa));
      sa.sa_handler = on_term;
      sigemptyset(&sa.sa_mask);
      if (sigaction(SIGTERM, &sa, &w.old_term) == 0) w.term_installed = true;
    }
  }
  if (!w.running.load()) {
    while (w.alive.load()) usleep(1000);  // a stopped thread still draining
    w.running.store(1);
    w.alive.store(1);
    std::thread(loop).detach();
  }
  return 0;
}

// Heartbeat: the rank entered ``phase`` (of ``step``); it must beat again
// within ``timeout_s`` seconds (<= 0: the default).  A negative step keeps
// the previous one.
KFB_API int kfb_watchdog_beat(const char* phase, long step, double timeout_s) {
  Watchdog& w = g_wd;
  std::lock_guard<std::mutex> lk(w.mu);
  if (phase) w.phase = phase;
  if (step >= 0) w.step = step;
  w.armed_for = timeout_s > 0 ? timeout_s : w.timeout;
  w.deadline = now_s() + w.armed_for;
  return w.fired.load();
}

// No deadline until the next beat (a phase with no collective in it).
KFB_API int kfb_watchdog_pause() {
  std::lock_guard<std::mutex> lk(g_wd.mu);
  g_wd.deadline = 0.0;
  return 0;
}

KFB_API int kfb_watchdog_add_comm(void* comm) {
  std::lock_guard<std::mutex> lk(g_wd.mu);
  if (comm) g_wd.comms.push_back(comm);
  return (int)g_wd.comms.size();
}

KFB_API int kfb_watchdog_remove_comm(void* comm) {
  std::lock_guard<std::mutex> lk(g_wd.mu);
  auto& v = g_wd.comms;
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i] == comm) {
      v.erase(v.begin() + i);
      return 1;
    }
  return 0;
}

// Test hook: called with each communicator instead of ncclCommAbort.
KFB_API int kfb_watchdog_set_abort_hook(void* fn) {
  std::lock_guard<std::mutex> lk(g_wd.mu);
  g_wd.abort_hook = (abort_fn_t)fn;
  return 0;
}

// 1 once fired; the JSON line written (if any) is copied into out.
KFB_API int kfb_watchdog_fired(char* out, int n) {
  std::lock_guard<std::mutex> lk(g_wd.mu);
  if (out && n > 0) {
    strncpy(out, g_wd.report.c_str(), (size_t)n - 1);
    out[n - 1] = 0;
  }
  return g_wd.fired.load();
}

KFB_API int kfb_watchdog_aborts() { return g_wd.aborts.load(); }

KFB_API int kfb_watchdog_stop() {
  Watchdog& w = g_wd;
  w.running.store(0);
  std::lock_guard<std::mutex> lk(w.mu);
  w.comms.clear();
  w.deadline = 0.0;
  if (w.term_installed) {
    sigaction(SIGTERM, &w.old_term, nullptr);
    w.term_installed = false;
  }
  return 0;
}
