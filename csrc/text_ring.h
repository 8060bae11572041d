// mxstream — text file reader into pinned host slots (SURVEY.md F-src / K18: host reader ->
// pinned ring -> async H2D -> device parse). Core without Python (csrc/reader.cpp binds it; the
// ThreadSanitizer harness csrc/tests/tsan_main.cpp drives it from several threads).
//
// A background thread cuts the byte range [lo, hi) of a file into newline-aligned chunks of at
// most `chunk` bytes and reads each one with `threads` parallel pread()s straight into one of the
// caller's slots (page-locked buffers, so the H2D copy is one DMA). It also counts the chunk's
// lines, so the consumer never scans the text on the host. Slots cycle: the consumer takes a
// filled slot with next(), uploads it, and release()s it once its copy has completed; the
// reader stays up to (slots - 1) chunks ahead (bounded memory, back-pressure on a slow
// consumer).
#pragma once
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "thread_pool.h"

namespace mxs {

struct Ready {
  int slot;
  int64_t nbytes;
  int64_t nlines;
  int64_t end_off;   // file offset just past the chunk (relative to lo)
  intptr_t ptr = 0;  // mapped mode: the chunk's first byte inside the file mapping
};

// Mapped mode (TextRingCore(MappedTag, ...)): no slot buffers and no copy on the host. The file
// is mmapped once; a chunk is "read" by counting its newlines with the parallel readers straight
// from the mapping -- which also faults its pages into the process page table -- and is handed
// out as a pointer into the mapping. The caller page-locks the mapping (hipHostRegister,
// read-only) and the copy engine reads the page cache directly: one DMA, no CPU memcpy (the
// pread path copies every byte once on the host). Slots are virtual: they only bound how far
// the reader runs ahead of the consumer.
struct MappedTag {};

class TextRingCore {
 public:
  TextRingCore(const std::string& path, int64_t lo, int64_t hi,
               std::vector<std::pair<intptr_t, int64_t>> slots, int64_t chunk, int threads)
      : lo_(lo), hi_(hi), chunk_(chunk), threads_(std::max(1, std::min(threads, 64))) {
    // Validate before opening: a throwing constructor never runs the destructor (no fd leak).
    if (slots.size() < 2) throw std::invalid_argument("TextFileRing needs at least 2 slots");
    if (lo < 0 || hi < lo) throw std::invalid_argument("bad byte range");
    for (auto& s : slots) {
      if (s.second < chunk) throw std::invalid_argument("slot smaller than the chunk size");
      slots_.push_back({reinterpret_cast<char*>(s.first), s.second});
      free_.push_back((int)slots_.size() - 1);
    }
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    // persistent readers: starting `threads` threads per chunk cost ~1 ms per 48 MB chunk
    if (threads_ > 1) pool_.reset(new WorkerPool(threads_ - 1));
  }
  // count_lines = false: no pass over the bytes on the host (nlines = -1: the consumer counts
  // on the device); only the last page of each chunk is read (its cut at the last newline).
  TextRingCore(MappedTag, const std::string& path, int64_t lo, int64_t hi, int nslots,
               int64_t chunk, int threads, bool count_lines = true)
      : lo_(lo), hi_(hi), chunk_(chunk), threads_(std::max(1, std::min(threads, 64))),
        count_(count_lines) {
    if (nslots < 2) throw std::invalid_argument("TextFileRing needs at least 2 slots");
    if (lo < 0 || hi < lo) throw std::invalid_argument("bad byte range");
    if (chunk <= 0) throw std::invalid_argument("bad chunk size");
    for (int i = 0; i < nslots; ++i) {
      slots_.push_back({nullptr, chunk});
      free_.push_back(i);
    }
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat stt;
    if (::fstat(fd_, &stt) != 0 || stt.st_size < hi) {
      ::close(fd_);
      fd_ = -1;
      throw std::invalid_argument("byte range past the end of " + path);
    }
    map_len_ = (size_t)stt.st_size;
    if (map_len_) {
      void* m = ::mmap(nullptr, map_len_, PROT_READ, MAP_SHARED, fd_, 0);
      if (m == MAP_FAILED) {
        ::close(fd_);
        fd_ = -1;
        throw std::runtime_error("cannot map " + path + ": " + std::strerror(errno));
      }
      map_ = static_cast<char*>(m);
      (void)::madvise(map_, map_len_, MADV_SEQUENTIAL);
    }
    if (threads_ > 1) pool_.reset(new WorkerPool(threads_ - 1));
  }
  ~TextRingCore() {
    close();
    if (map_) ::munmap(map_, map_len_);
  }
  // Mapped mode: the whole file's mapping (base, bytes); (0, 0) otherwise.
  intptr_t map_base() const { return reinterpret_cast<intptr_t>(map_); }
  int64_t map_bytes() const { return (int64_t)map_len_; }
  // Mapped mode: the reader thread hands every `seg` bytes of the mapping (page-aligned file
  // offsets k * seg) to fn(address, bytes) -- the binding page-locks them -- before it hands out
  // a chunk that touches them, so the page-locking runs segment by segment beside the stream
  // instead of once for the whole file before the first chunk. fn returns 0 or an error code.
  // Set before start().
  void on_segments(int64_t seg, std::function<int(intptr_t, int64_t)> fn) {
    if (seg <= 0 || seg % 4096) throw std::invalid_argument("segment size must be whole pages");
    seg_ = seg;
    seg_fn_ = std::move(fn);
    seg_done_ = lo_ / seg * seg;
  }
  int64_t segment_bytes() const { return seg_; }

  void start() {
    if (!th_.joinable()) th_ = std::thread([this] { run(); });
  }

  // Waits up to timeout_ms for a filled slot. Returns false when none is ready (then *eof tells
  // whether every chunk has been handed out); throws the reader's error.
  bool next(int timeout_ms, Ready* r, bool* eof) {
    std::string err;
    bool got = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      // system_clock deadline: pthread_cond_timedwait, which ThreadSanitizer intercepts
    // (steady_clock waits use pthread_cond_clockwait, invisible to GCC 11's TSan).
    cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms),
                   [&] { return !ready_.empty() || done_; });
      if (!ready_.empty()) {
        *r = ready_.front();
        ready_.pop_front();
        got = true;
      }
      *eof = done_ && ready_.empty() && !got;
      err = err_;
    }
    if (!err.empty()) throw std::runtime_error(err);
    return got;
  }

  void release(int slot) {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= (int)slots_.size()) throw std::invalid_argument("bad slot");
    free_.push_back(slot);
    cv_.notify_all();
  }

  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      cv_.notify_all();
    }
    if (th_.joinable()) th_.join();
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
  }

 private:
  struct Slot {
    char* p;
    int64_t cap;
  };

  void touch_pages(const char* p, int64_t len) {
    const int T = (int)std::min<int64_t>(threads_, std::max<int64_t>(1, len >> 22));
    auto piece = [&](int t) {
      const int64_t a = (len * t / T) & ~(int64_t)4095, b = len * (t + 1) / T;
      unsigned s = 0;
      for (int64_t o = a; o < b; o += 4096) s += (unsigned char)((volatile const char*)p)[o];
      touched_.fetch_add(s, std::memory_order_relaxed);  // keeps the reads
    };
    if (T == 1 || !pool_) {
      for (int t = 0; t < T; ++t) piece(t);
    } else {
      pool_->run(T, piece);
    }
  }
  std::atomic<unsigned> touched_{0};

  // Mapped mode: the newlines of [off, off + len) counted from the mapping by the parallel
  // readers (the first touch of each page happens here, off the consumer's thread).
  void count_mapped(int64_t off, int64_t len, int64_t* newlines) {
    const int T = (int)std::min<int64_t>(threads_, std::max<int64_t>(1, len >> 20));
    std::vector<int64_t> cnt((size_t)T, 0);
    const char* src = map_ + off;
    auto piece = [&](int t) {
      const int64_t a = len * t / T, b = len * (t + 1) / T;
      cnt[(size_t)t] = std::count(src + a, src + b, '\n');
    };
    if (T == 1 || !pool_) {
      for (int t = 0; t < T; ++t) piece(t);
    } else {
      pool_->run(T, piece);
    }
    int64_t k = 0;
    for (int64_t x : cnt) k += x;
    *newlines = k;
  }

  bool read_range(char* dst, int64_t off, int64_t len, int64_t* newlines) {
    // `threads_` contiguous pieces read in parallel (page cache -> pinned memory copies); each
    // piece's newlines are counted right after its read, while the bytes are still in cache
    // (a separate counting pass re-read the whole chunk from memory).
    const int T = (int)std::min<int64_t>(threads_, std::max<int64_t>(1, len >> 20));
    std::atomic<bool> ok{true};
    std::vector<int64_t> cnt((size_t)T, 0);
    auto piece = [&](int t) {
      const int64_t a = len * t / T, b = len * (t + 1) / T;
      int64_t pos = a;
      while (pos < b) {
        const ssize_t r = ::pread(fd_, dst + pos, (size_t)(b - pos), (off_t)(off + pos));
        if (r <= 0) {
          if (r < 0 && errno == EINTR) continue;
          ok = false;
          return;
        }
        pos += r;
      }
      cnt[(size_t)t] = std::count(dst + a, dst + b, '\n');
    };
    if (T == 1 || !pool_) {
      for (int t = 0; t < T; ++t) piece(t);
    } else {
      pool_->run(T, piece);
    }
    int64_t k = 0;
    for (int64_t x : cnt) k += x;
    *newlines = k;
    return ok;
  }

  void run() {
    int64_t off = lo_;
    std::string err;
    while (off < hi_) {
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !free_.empty(); });
        if (stop_) return;
        slot = free_.front();
        free_.pop_front();
      }
      const int64_t want = std::min(chunk_, hi_ - off);
      int64_t nl_read = 0;
      const char* dst;
      if (map_ && seg_fn_) {
        bool seg_ok = true;
        while (seg_done_ < off + want && seg_done_ < (int64_t)map_len_) {
          const int64_t len = std::min<int64_t>(seg_, (int64_t)map_len_ - seg_done_);
          // Fault the segment's pages into the page table first (parallel page-stride reads):
          // page-locking resident pages takes microseconds, while page-locking absent ones
          // faults them in under the runtime's lock, stalling every HIP call of the consumer.
          touch_pages(map_ + seg_done_, len);
          const int rc = seg_fn_(reinterpret_cast<intptr_t>(map_ + seg_done_), len);
          if (rc) {
            err = "page-locking the file mapping failed (error " + std::to_string(rc) + ")";
            seg_ok = false;
            break;
          }
          seg_done_ += seg_;
        }
        if (!seg_ok) break;
      }
      if (map_) {
        dst = map_ + off;
        if (count_) count_mapped(off, want, &nl_read);
      } else {
        char* buf = slots_[slot].p;
        dst = buf;
        if (!read_range(buf, off, want, &nl_read)) {
          err = "read failed at offset " + std::to_string(off);
          break;
        }
      }
      int64_t used = want;
      if (off + want < hi_) {
        const char* nl = static_cast<const char*>(memrchr(dst, '\n', (size_t)want));
        if (!nl) {
          err = "a line is longer than the ingest chunk (" + std::to_string(chunk_) + " bytes)";
          break;
        }
        used = nl - dst + 1;
      }
      // (the bytes past `used` hold no newline: used ends at the chunk's last one)
      const int64_t nl = (map_ && !count_) ? -1
                         : nl_read + (used > 0 && dst[used - 1] != '\n' ? 1 : 0);
      const intptr_t ptr = map_ ? reinterpret_cast<intptr_t>(dst) : 0;
      off += used;
      std::lock_guard<std::mutex> g(mu_);
      ready_.push_back({slot, used, nl, off - lo_, ptr});
      cv_.notify_all();
    }
    std::lock_guard<std::mutex> g(mu_);
    err_ = err;
    done_ = true;
    cv_.notify_all();
  }

  int fd_ = -1;
  char* map_ = nullptr;
  size_t map_len_ = 0;
  int64_t lo_, hi_, chunk_;
  int threads_;
  bool count_ = true;
  int64_t seg_ = 0, seg_done_ = 0;
  std::function<int(intptr_t, int64_t)> seg_fn_;
  std::unique_ptr<WorkerPool> pool_;
  std::vector<Slot> slots_;
  std::deque<int> free_;
  std::deque<Ready> ready_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false, stop_ = false;
  std::string err_;
  std::thread th_;
};

}  // namespace mxs
