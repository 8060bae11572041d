// mxstream — key-group indexed keyed-state files (restore at a different
// parallelism reads only the owned key-group range). Core without Python: csrc/runtime.cpp binds
// it (the checkpoint writer runs it on a worker thread), csrc/tests/tsan_main.cpp runs concurrent
// writers under ThreadSanitizer.
// Layout: "MXSKG001" | u64 header_len | header (UTF-8 JSON) | u32 kg_lo | u32 kg_hi |
//         u64 offsets[kg_hi - kg_lo + 2] (row offsets) | columns (each nrows * itemsize, kg-sorted)
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mxs {

// Rows with key group kgp[i] (in [kg_lo, kg_hi]); each column is (data, itemsize) of n rows.
// Written to path.inprogress, then renamed: a crash never leaves a partial file behind.
inline void write_kg_columns(const std::string& path, const std::string& header, uint32_t kg_lo,
                             uint32_t kg_hi, const int32_t* kgp, size_t n,
                             const std::vector<std::pair<const char*, size_t>>& cols) {
  const uint32_t ngroups = kg_hi - kg_lo + 1;
  std::vector<uint64_t> off(ngroups + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    const int32_t g = kgp[i];
    if (g < (int32_t)kg_lo || g > (int32_t)kg_hi) throw std::invalid_argument("row key group outside file range");
    off[g - kg_lo + 1]++;
  }
  for (uint32_t g = 0; g < ngroups; ++g) off[g + 1] += off[g];
  std::vector<uint64_t> perm(n);
  {
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    for (size_t i = 0; i < n; ++i) perm[cur[kgp[i] - kg_lo]++] = i;  // stable counting sort
  }
  const std::string tmp = path + ".inprogress";
  std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
  if (!f) throw std::runtime_error("cannot open " + tmp);
  f.write("MXSKG001", 8);
  const uint64_t hl = header.size();
  f.write((const char*)&hl, 8);
  f.write(header.data(), (std::streamsize)hl);
  f.write((const char*)&kg_lo, 4);
  f.write((const char*)&kg_hi, 4);
  f.write((const char*)off.data(), (std::streamsize)(off.size() * 8));
  std::vector<char> tmpbuf;
  for (const auto& [src, isz] : cols) {
    tmpbuf.resize(n * isz);
    for (size_t i = 0; i < n; ++i) std::memcpy(&tmpbuf[i * isz], src + perm[i] * isz, isz);
    f.write(tmpbuf.data(), (std::streamsize)tmpbuf.size());
  }
  f.flush();
  if (!f) throw std::runtime_error("write failed: " + tmp);
  f.close();
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed: " + path);
}

}  // namespace mxs
