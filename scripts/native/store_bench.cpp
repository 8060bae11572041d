// Host session store phases on the box's CPUs (no GPU): the spill worker's insert phases
// (insert_hot, build_cold, index_cold, publish_cold, expire) for evictions of D rows of drifting
// dense keys, and the promote path's indexed extract of ~80K revisited keys.
//   g++ -O3 -std=c++17 -pthread -Icsrc scripts/native/store_bench.cpp -o /tmp/store_bench
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>

#include "session_store.h"
using namespace mxs::sess;
using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}
int main(int argc, char** argv) {
  const int64_t D = argc > 2 ? atoll(argv[2]) : 300000;
  SessionCore c(5000, 30000, 0);
  c.max_threads_ = argc > 1 ? atoi(argv[1]) : 16;
  std::mt19937_64 rng(1);
  std::vector<int64_t> rows(400000 * 8), moved(400000);
  double t[6] = {0};
  int nsteps = 0;
  for (int i = 0; i < 30; ++i) {
    std::vector<int64_t> k(D), s(D), e(D), a(D), n(D, 4), f(D, 1);
    std::iota(k.begin(), k.end(), i * D);
    std::shuffle(k.begin(), k.end(), rng);
    for (int64_t j = 0; j < D; ++j) {
      s[j] = i * 2000 + k[j] % 2000;
      e[j] = s[j] + 5000;
      a[j] = k[j] % 97;
    }
    SessionCore::ColdPlan p;
    auto t0 = clk::now();
    c.insert_hot(k.data(), s.data(), e.data(), a.data(), n.data(), f.data(), D, true, p);
    auto t1 = clk::now();
    c.build_cold_parallel(k.data(), s.data(), e.data(), a.data(), n.data(), D, p);
    auto t2 = clk::now();
    c.index_cold(p);
    auto t3 = clk::now();
    c.publish_cold(p);
    std::vector<int64_t> rel;
    c.expire_cold(i * 2000 - 40000, rel);
    auto t4 = clk::now();
    std::vector<int64_t> want;
    if (i >= 12) {
      for (int j = 0; j < 90000; ++j) want.push_back((i - 10) * D + (int64_t)(rng() % D));
      std::sort(want.begin(), want.end());
      want.erase(std::unique(want.begin(), want.end()), want.end());
    }
    auto t5 = clk::now();
    if (!want.empty())
      c.extract_rows_into(want.data(), want.size(), i * 2000, 4, 5000, rows.data(), 400000,
                          moved.data(), 400000);
    auto t6 = clk::now();
    if (i >= 12) {
      t[0] += ms(t0, t1);
      t[1] += ms(t1, t2);
      t[2] += ms(t2, t3);
      t[3] += ms(t3, t4);
      t[4] += ms(t5, t6);
      ++nsteps;
    }
  }
  printf("{\"threads\": %d, \"rows_per_eviction\": %ld, \"ms\": {\"insert_hot\": %.3f, "
         "\"build_cold\": %.3f, \"index_cold\": %.3f, \"publish_expire\": %.3f, "
         "\"extract_rows_into\": %.3f}, \"cold_rows\": %zu}\n",
         c.max_threads_, (long)D, t[0] / nsteps, t[1] / nsteps, t[2] / nsteps, t[3] / nsteps,
         t[4] / nsteps, c.num_cold_rows());
}
