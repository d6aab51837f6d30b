// group_sync.h — the host threading of a multi-device context (icp_group.cpp): one persistent
// driver thread per member and the in-process all-gather of the host transport. Plain C++ (no
// HIP), so the CPU sanitizer builds (csrc/Makefile asan / tsan, tests/test_sanitize.py) exercise
// exactly this code with N threads.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace icp {

// A persistent driver thread: runs one posted job at a time.
class Driver {
 public:
  Driver() : th_([this] { loop(); }) {}
  ~Driver() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = std::move(f);
      busy_ = true;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return !busy_; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    while (true) {
      cv_.wait(g, [this] { return quit_ || (busy_ && job_); });
      if (quit_) return;
      auto f = std::move(job_);
      job_ = nullptr;
      g.unlock();
      f();
      g.lock();
      busy_ = false;
      cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::function<void()> job_;
  bool busy_ = false, quit_ = false;
  std::thread th_;  // last: started once the members above exist
};

// In-process all-gather of one record per member (the host transport): members deposit their
// record, the last arrival publishes the generation, everyone copies the gathered array. Two
// buffers alternate by generation: exchange k+2 can only start after every member has finished
// copying exchange k (it had to arrive at k+1 first).
struct LocalExchange {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<double> buf[2];
  const std::atomic<int>* abort = nullptr;

  int gather(int rank, const double* local, int count, double* gathered) {
    std::unique_lock<std::mutex> g(m);
    std::vector<double>& b = buf[gen & 1];
    if (b.size() < (size_t)n * count) b.resize((size_t)n * count);
    std::memcpy(b.data() + (size_t)rank * count, local, sizeof(double) * count);
    const uint64_t my = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(g, [&] { return gen != my || (abort && abort->load()); });
      if (gen == my) return 1;  // a peer member failed
    }
    std::memcpy(gathered, b.data(), sizeof(double) * (size_t)n * count);
    return 0;
  }
  void wake() {
    std::lock_guard<std::mutex> g(m);
    cv.notify_all();
  }
  // before a job: an exchange abandoned by a failed job (some members arrived, then gave up)
  // must not count towards the next one
  void reset() {
    std::lock_guard<std::mutex> g(m);
    arrived = 0;
  }
};

struct ExchangeSlot {
  LocalExchange* x;
  int rank;
};

inline int local_exchange(void* user, const double* local, int32_t count, double* gathered) {
  auto* s = static_cast<ExchangeSlot*>(user);
  return s->x->gather(s->rank, local, count, gathered);
}

}  // namespace icp
