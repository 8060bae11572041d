// mxstream — key-group indexed keyed-state files (restore at a different
// parallelism reads only the owned key-group range). Core without Python: csrc/runtime.cpp binds
// it (the checkpoint writer runs it on a worker thread), csrc/tests/tsan_main.cpp runs concurrent
// writers under ThreadSanitizer.
// Layout: "MXSKG001" | u64 header_len | header (UTF-8 JSON) | u32 kg_lo | u32 kg_hi |
//         u64 offsets[kg_hi - kg_lo + 2] (row offsets) | columns (each nrows * itemsize, kg-sorted)
//
// The window snapshot sorts its rows by key group on the device (runtime/window_state.py), so the
// usual input is already in file order: the columns then go to the file as they are. Otherwise a
// stable counting sort gives the row permutation and the gather runs in slices on several
// threads. Either way the columns are written with positioned writes of 16 MB pieces from up to
// 8 threads (one ofstream and a per-row memcpy gather took 0.5-0.9 s for 290 MB at 10M keys,
// profiles/r6_ckpt_breakdown.json).
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mxs {

namespace kgf {

inline void pwrite_all(int fd, const char* p, size_t n, uint64_t off) {
  while (n) {
    const ssize_t w = ::pwrite(fd, p, n, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("checkpoint write failed: ") + std::strerror(errno));
    }
    p += w;
    n -= (size_t)w;
    off += (uint64_t)w;
  }
}

// Rows [r0, r1) of a column gathered through perm into dst.
inline void gather(char* dst, const char* src, size_t isz, const uint64_t* perm, size_t r0,
                   size_t r1) {
  switch (isz) {
    case 1:
      for (size_t i = r0; i < r1; ++i) dst[i - r0] = src[perm[i]];
      break;
    case 4:
      for (size_t i = r0; i < r1; ++i)
        std::memcpy(dst + (i - r0) * 4, src + perm[i] * 4, 4);
      break;
    case 8:
      for (size_t i = r0; i < r1; ++i)
        std::memcpy(dst + (i - r0) * 8, src + perm[i] * 8, 8);
      break;
    default:
      for (size_t i = r0; i < r1; ++i) std::memcpy(dst + (i - r0) * isz, src + perm[i] * isz, isz);
  }
}

}  // namespace kgf

// Rows with key group kgp[i] (in [kg_lo, kg_hi]); each column is (data, itemsize) of n rows.
// Written to path.inprogress, then renamed: a crash never leaves a partial file behind.
inline void write_kg_columns(const std::string& path, const std::string& header, uint32_t kg_lo,
                             uint32_t kg_hi, const int32_t* kgp, size_t n,
                             const std::vector<std::pair<const char*, size_t>>& cols,
                             int threads = 8, size_t piece_bytes = (size_t)16 << 20) {
  const uint32_t ngroups = kg_hi - kg_lo + 1;
  std::vector<uint64_t> off(ngroups + 1, 0);
  bool sorted = true;
  for (size_t i = 0; i < n; ++i) {
    const int32_t g = kgp[i];
    if (g < (int32_t)kg_lo || g > (int32_t)kg_hi) throw std::invalid_argument("row key group outside file range");
    off[g - kg_lo + 1]++;
    if (i && g < kgp[i - 1]) sorted = false;
  }
  for (uint32_t g = 0; g < ngroups; ++g) off[g + 1] += off[g];
  std::vector<uint64_t> perm;
  if (!sorted) {
    perm.resize(n);
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    for (size_t i = 0; i < n; ++i) perm[cur[kgp[i] - kg_lo]++] = i;  // stable counting sort
  }

  // File image: preamble, then every column at a known offset.
  std::string pre;
  pre.append("MXSKG001", 8);
  const uint64_t hl = header.size();
  pre.append((const char*)&hl, 8);
  pre.append(header);
  pre.append((const char*)&kg_lo, 4);
  pre.append((const char*)&kg_hi, 4);
  pre.append((const char*)off.data(), off.size() * 8);
  std::vector<uint64_t> col_off(cols.size());
  uint64_t end = pre.size();
  for (size_t c = 0; c < cols.size(); ++c) {
    col_off[c] = end;
    end += (uint64_t)n * cols[c].second;
  }

  const std::string tmp = path + ".inprogress";
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("cannot open " + tmp + ": " + std::strerror(errno));
  try {
    kgf::pwrite_all(fd, pre.data(), pre.size(), 0);
    // Pieces of <= piece_bytes (16 MB) of one column each; workers take them in order.
    const size_t kPiece = std::max<size_t>(1, piece_bytes);
    struct Piece {
      size_t col, r0, r1;
    };
    std::vector<Piece> pieces;
    for (size_t c = 0; c < cols.size(); ++c) {
      const size_t rows = std::max<size_t>(1, kPiece / cols[c].second);
      for (size_t r = 0; r < n; r += rows) pieces.push_back({c, r, std::min(n, r + rows)});
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    std::string err;
    auto work = [&]() {
      std::vector<char> buf;
      try {
        for (;;) {
          const size_t k = next.fetch_add(1);
          if (k >= pieces.size() || failed.load()) return;
          const Piece& p = pieces[k];
          const char* src = cols[p.col].first;
          const size_t isz = cols[p.col].second;
          const char* data;
          if (sorted) {
            data = src + p.r0 * isz;
          } else {
            buf.resize((p.r1 - p.r0) * isz);
            kgf::gather(buf.data(), src, isz, perm.data(), p.r0, p.r1);
            data = buf.data();
          }
          kgf::pwrite_all(fd, data, (p.r1 - p.r0) * isz, col_off[p.col] + p.r0 * isz);
        }
      } catch (const std::exception& e) {
        if (!failed.exchange(true)) err = e.what();
      }
    };
    const size_t nt = std::min<size_t>((size_t)std::max(1, threads), pieces.size());
    if (nt <= 1) {
      work();
    } else {
      std::vector<std::thread> th;
      for (size_t t = 0; t + 1 < nt; ++t) th.emplace_back(work);
      work();
      for (auto& x : th) x.join();
    }
    if (failed.load()) throw std::runtime_error(err + " (" + tmp + ")");
  } catch (...) {
    ::close(fd);
    std::remove(tmp.c_str());
    throw;
  }
  if (::close(fd) != 0) throw std::runtime_error("write failed: " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed: " + path);
}

}  // namespace mxs
