// Progress watchdog for multi-GPU jobs (ABI 34).
//
// A collective that one rank never joins leaves its peers waiting forever:
// inside a replayed HIP graph RCCL's own watchdog does not see the captured
// collectives (torch does not track work issued during a capture), and a host
// thread blocked in a stream or event wait never returns to Python.  This
// thread does not need the interpreter: the caller arms it with a timeout and
// reports progress (gsplat_hip_watchdog_beat, with a one-line state such as
// "rank 3 step 27 timed replay"); when no beat arrives within the timeout it
// prints the last state to stderr, optionally writes a fallback text to a file
// descriptor (the bench's result line of a phase that already completed), and
// ends the process with _exit -- no exec, no unwinding through a thread that
// is stuck in a HIP call.
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>

namespace gs {
namespace {

struct Watchdog {
  std::mutex mu;
  std::condition_variable cv;
  std::thread th;
  bool armed = false, stop = false, started = false;
  double timeout_s = 0.0;
  int exit_code = 3;
  std::chrono::steady_clock::time_point deadline;
  std::string state, tag;
  int fb_fd = -1;
  int fb_exit = -1;
  std::string fallback;

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    while (!stop) {
      if (!armed) {
        cv.wait(lk);
        continue;
      }
      if (cv.wait_until(lk, deadline) == std::cv_status::timeout && armed && !stop &&
          std::chrono::steady_clock::now() >= deadline) {
        fprintf(stderr,
                "[gsplat_hip watchdog] %s: no progress for %.0f s; last state: %s -- "
                "ending the process (status %d)\n",
                tag.c_str(), timeout_s, state.c_str(), fb_fd >= 0 ? fb_exit : exit_code);
        fflush(stderr);
        int code = exit_code;
        if (fb_fd >= 0) {
          const char *p = fallback.data();
          size_t left = fallback.size();
          while (left > 0) {
            const ssize_t w = write(fb_fd, p, left);
            if (w <= 0) break;
            p += w;
            left -= (size_t)w;
          }
          code = fb_exit;
        }
        _exit(code);
      }
    }
  }
};

Watchdog &wd() {
  static Watchdog *w = new Watchdog();  // never destroyed: its thread may outlive exit paths
  return *w;
}

}  // namespace
}  // namespace gs

// Arm (or re-arm) with a timeout in seconds; `tag` names the process in the
// message ("rank 3"); `exit_code` is the status on expiry (non-zero).
extern "C" int gsplat_hip_watchdog_arm(double timeout_s, const char *tag, int exit_code) {
  if (!(timeout_s > 0.0)) return 1;
  gs::Watchdog &w = gs::wd();
  std::lock_guard<std::mutex> lk(w.mu);
  if (!w.started) {
    w.th = std::thread([&w] { w.run(); });
    w.th.detach();
    w.started = true;
  }
  w.timeout_s = timeout_s;
  w.exit_code = exit_code != 0 ? exit_code : 3;
  w.tag = tag ? tag : "";
  w.armed = true;
  w.deadline = std::chrono::steady_clock::now() +
               std::chrono::microseconds((int64_t)(timeout_s * 1e6));
  w.cv.notify_all();
  return 0;
}

// Progress: restart the timeout and record the state printed on expiry.
extern "C" int gsplat_hip_watchdog_beat(const char *state) {
  gs::Watchdog &w = gs::wd();
  std::lock_guard<std::mutex> lk(w.mu);
  w.state = state ? state : "";
  w.deadline = std::chrono::steady_clock::now() +
               std::chrono::microseconds((int64_t)(w.timeout_s * 1e6));
  w.cv.notify_all();
  return 0;
}

// On expiry also write `text` to `fd` and end with `exit_code` (fd < 0:
// clear).  For a phase after the job's main result: that result is still
// delivered when the later phase hangs.
extern "C" int gsplat_hip_watchdog_set_fallback(int fd, const char *text, int exit_code) {
  gs::Watchdog &w = gs::wd();
  std::lock_guard<std::mutex> lk(w.mu);
  w.fb_fd = fd;
  w.fallback = (fd >= 0 && text) ? text : "";
  w.fb_exit = exit_code;
  return 0;
}

extern "C" int gsplat_hip_watchdog_disarm(void) {
  gs::Watchdog &w = gs::wd();
  std::lock_guard<std::mutex> lk(w.mu);
  w.armed = false;
  w.cv.notify_all();
  return 0;
}
