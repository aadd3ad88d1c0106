// Core of the native token prefetcher (no Python dependency): used by the pybind11 module prefetch.cpp
// and by the sanitizer harness prefetch_check.cpp. See prefetch.cpp for the design notes.
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace kop_native {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

class TokenPrefetcher {
 public:
  TokenPrefetcher(const std::string& path, int itemsize, int64_t batch, int64_t window, uint64_t seed,
                  int depth, int threads)
      : itemsize_(itemsize), batch_(batch), window_(window), seed_(seed), depth_(depth) {
    if (itemsize != 2 && itemsize != 4) throw std::invalid_argument("itemsize must be 2 (uint16) or 4 (uint32)");
    if (batch <= 0 || window <= 1 || depth <= 0 || threads <= 0) throw std::invalid_argument("bad prefetch shape");
    fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path);
    struct stat st {};
    if (::fstat(fd_, &st) != 0) throw std::runtime_error("cannot stat " + path);
    bytes_ = static_cast<size_t>(st.st_size);
    ntok_ = static_cast<int64_t>(bytes_ / itemsize_);
    if (ntok_ <= window_) throw std::invalid_argument(path + ": fewer tokens than one window");
    base_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
    ::madvise(base_, bytes_, MADV_RANDOM);
    slots_.resize(depth_);
    for (int i = 0; i < depth_; ++i) {
      slots_[i].data.resize(static_cast<size_t>(batch_ * window_));
      slots_[i].index = -1;
    }
    for (int t = 0; t < threads; ++t) workers_.emplace_back([this] { work(); });
  }

  ~TokenPrefetcher() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    cv_ready_.notify_all();
    for (auto& t : workers_) t.join();
    if (base_ && base_ != MAP_FAILED) ::munmap(base_, bytes_);
    if (fd_ >= 0) ::close(fd_);
  }

  // Next batch [batch * window] int64, row-major; blocks until it is ready. The buffer is handed out
  // (moved), the slot gets a fresh one.
  std::vector<int64_t> next() {
    std::vector<int64_t> out;
    {
      std::unique_lock<std::mutex> lk(mu_);
      const int64_t want = consumed_;
      Slot& s = slots_[want % depth_];
      cv_ready_.wait(lk, [&] { return stop_ || (s.index == want && s.ready); });
      if (stop_) throw std::runtime_error("prefetcher stopped");
      out.swap(s.data);
      s.data.resize(static_cast<size_t>(batch_ * window_));
      s.ready = false;
      s.index = -1;
      ++consumed_;
    }
    cv_work_.notify_all();
    return out;
  }
  int64_t batch() const { return batch_; }
  int64_t window() const { return window_; }

  // Drop the next n batches without materialising them (resume at a step boundary).
  void skip(int64_t n) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& s : slots_) {
      s.index = -1;
      s.ready = false;
    }
    consumed_ += n;
    issued_ = consumed_;
    cv_work_.notify_all();
  }

  int64_t num_tokens() const { return ntok_; }
  int64_t position() const { return consumed_; }

  // The exact window starts of batch i (tests check determinism against numpy with these).
  std::vector<int64_t> starts(int64_t i) const {
    std::vector<int64_t> s(batch_);
    const uint64_t span = static_cast<uint64_t>(ntok_ - window_ + 1);
    for (int64_t r = 0; r < batch_; ++r)
      s[r] = static_cast<int64_t>(splitmix64(seed_ ^ splitmix64(static_cast<uint64_t>(i) * 0x100000001B3ull + r)) % span);
    return s;
  }

 private:
  struct Slot {
    std::vector<int64_t> data;
    int64_t index = -1;
    bool ready = false;
    bool busy = false;
  };

  void fill(int64_t i, std::vector<int64_t>& dst) const {
    auto st = starts(i);
    for (int64_t r = 0; r < batch_; ++r) {
      int64_t* o = dst.data() + r * window_;
      if (itemsize_ == 2) {
        const uint16_t* src = static_cast<const uint16_t*>(base_) + st[r];
        for (int64_t k = 0; k < window_; ++k) o[k] = src[k];
      } else {
        const uint32_t* src = static_cast<const uint32_t*>(base_) + st[r];
        for (int64_t k = 0; k < window_; ++k) o[k] = src[k];
      }
    }
  }

  void work() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_work_.wait(lk, [&] {
        return stop_ || (issued_ < consumed_ + depth_ && !slots_[issued_ % depth_].busy &&
                         slots_[issued_ % depth_].index == -1);
      });
      if (stop_) return;
      const int64_t i = issued_++;
      Slot& s = slots_[i % depth_];
      s.busy = true;
      s.index = i;
      std::vector<int64_t> buf;
      buf.swap(s.data);
      lk.unlock();
      fill(i, buf);
      lk.lock();
      s.data.swap(buf);
      s.busy = false;
      if (s.index == i) {
        s.ready = true;
        cv_ready_.notify_all();
      }
    }
  }

  int fd_ = -1;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  int64_t ntok_ = 0;
  const int itemsize_;
  const int64_t batch_, window_;
  const uint64_t seed_;
  const int depth_;
  std::vector<Slot> slots_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_ready_;
  int64_t issued_ = 0, consumed_ = 0;
  bool stop_ = false;
};

}  // namespace kop_native
