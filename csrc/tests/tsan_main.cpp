// mxstream — ThreadSanitizer harness of the threaded host code. Built by
// `python -m mxstream.build --tsan` with -fsanitize=thread and run by tests/test_debug.py. It
// drives, with real threads, every host component that runs concurrently in the engine:
//   1. the pinned-slot text file reader (csrc/text_ring.h): background reader + parallel pread
//      workers + a consumer taking and releasing slots;
//   2. the socket source (csrc/socket_reader.h): reader thread + polling consumer, and a close()
//      from a third thread while the reader is blocked in recv();
//   3. the session store's spill-worker hand-off (csrc/session_store.h): rows inserted on a worker
//      thread (session_operator.py _evict) while the main thread works on its own store, joined
//      before the main thread uses the store again; two stores on two threads;
//   4. concurrent key-group checkpoint writers (csrc/kg_file.h: the async checkpoint's worker
//      writes while another rank's / operator's writer runs).
// Exit code 0 and no "ThreadSanitizer" report = pass.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

#include "kg_file.h"
#include "session_store.h"
#include "socket_reader.h"
#include "text_ring.h"
#include "window_tier.h"

using namespace mxs;

static int fail(const std::string& what) {
  std::fprintf(stderr, "tsan_main: %s\n", what.c_str());
  return 1;
}

static std::string tmp_path(const char* name) {
  const char* d = std::getenv("TMPDIR");
  return std::string(d ? d : "/tmp") + "/mxs_tsan_" + std::to_string(getpid()) + "_" + name;
}

static int test_text_ring() {
  const std::string path = tmp_path("ring.txt");
  std::string all;
  for (int i = 0; i < 60000; ++i)
    all += "2019-08-28T10:00:" + std::to_string(i % 60) + " ch" + std::to_string(i % 977) +
           ".example.com " + std::to_string(i * 37 % 100000) + "\n";
  {
    std::ofstream f(path, std::ios::binary);
    f << all;
  }
  const int64_t chunk = 64 << 10;
  std::vector<std::vector<char>> bufs(3, std::vector<char>(chunk));
  std::vector<std::pair<intptr_t, int64_t>> slots;
  for (auto& b : bufs) slots.push_back({(intptr_t)b.data(), chunk});
  TextRingCore ring(path, 0, (int64_t)all.size(), slots, chunk, 4);
  ring.start();
  std::string got;
  int64_t lines = 0;
  std::atomic<bool> ok{true};
  std::thread consumer([&] {
    for (;;) {
      Ready r{-1, 0, 0, 0};
      bool eof = false;
      if (!ring.next(200, &r, &eof)) {
        if (eof) return;
        continue;
      }
      got.append(bufs[r.slot].data(), (size_t)r.nbytes);
      lines += r.nlines;
      ring.release(r.slot);
    }
  });
  consumer.join();
  ring.close();
  std::remove(path.c_str());
  if (!ok || got != all) return fail("text ring: bytes differ");
  if (lines != 60000) return fail("text ring: line count " + std::to_string(lines));
  return 0;
}

static int listen_any(int* port) {
  const int s = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  if (bind(s, (sockaddr*)&a, sizeof(a)) != 0 || listen(s, 1) != 0) return -1;
  socklen_t len = sizeof(a);
  getsockname(s, (sockaddr*)&a, &len);
  *port = ntohs(a.sin_port);
  return s;
}

static int test_socket() {
  int port = 0;
  const int ls = listen_any(&port);
  if (ls < 0) return fail("socket: listen");
  const int n = 5000;
  std::thread server([&] {
    const int c = accept(ls, nullptr, nullptr);
    std::string payload;
    for (int i = 0; i < n; ++i) payload += "line-" + std::to_string(i) + "\r\n";
    for (size_t i = 0; i < payload.size(); i += 1000) {
      const size_t m = std::min<size_t>(1000, payload.size() - i);
      if (send(c, payload.data() + i, m, 0) < 0) break;
    }
    ::close(c);
    ::close(ls);
  });
  SocketReaderCore src("127.0.0.1", port, "\n", 0, 100);
  src.start();
  int seen = 0;
  for (;;) {
    std::string joined, err;
    size_t k = 0;
    bool eof = false;
    src.poll(700, 50, &joined, &k, &eof, &err);
    if (!err.empty()) return fail("socket: " + err);
    size_t pos = 0;
    for (size_t i = 0; i < k; ++i) {
      const size_t e = joined.find('\n', pos);
      if (joined.substr(pos, e - pos) != "line-" + std::to_string(seen)) return fail("socket: line");
      ++seen;
      pos = e + 1;
    }
    if (eof) break;
  }
  server.join();
  src.close();
  if (seen != n) return fail("socket: " + std::to_string(seen) + " lines");

  // close() from another thread while the reader blocks in recv() on a silent connection.
  int port2 = 0;
  const int ls2 = listen_any(&port2);
  std::atomic<bool> stop{false};
  std::thread silent([&] {
    const int c = accept(ls2, nullptr, nullptr);
    (void)!send(c, "x\n", 2, 0);
    while (!stop) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    ::close(c);
    ::close(ls2);
  });
  SocketReaderCore src2("127.0.0.1", port2, "\n", 0, 100);
  src2.start();
  std::string j, e;
  size_t k = 0;
  bool eof = false;
  while (k == 0) src2.poll(10, 50, &j, &k, &eof, &e);
  std::thread closer([&] { src2.close(); });
  closer.join();
  stop = true;
  silent.join();

  // Back-pressure: a 64-line queue, a slow consumer -- the reader blocks, nothing is lost, and a
  // close() while the reader waits for space returns.
  int port3 = 0;
  const int ls3 = listen_any(&port3);
  const int n3 = 20000;
  std::thread fast([&] {
    const int c = accept(ls3, nullptr, nullptr);
    std::string payload;
    for (int i = 0; i < n3; ++i) payload += std::to_string(i) + "\n";
    for (size_t i = 0; i < payload.size(); i += 4096) {
      const size_t m = std::min<size_t>(4096, payload.size() - i);
      if (send(c, payload.data() + i, m, 0) < 0) break;
    }
    ::close(c);
    ::close(ls3);
  });
  SocketReaderCore src3("127.0.0.1", port3, "\n", 0, 100, 64);
  src3.start();
  int got3 = 0;
  for (;;) {
    std::string joined, err;
    size_t k3 = 0;
    bool eof3 = false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    src3.poll(50, 50, &joined, &k3, &eof3, &err);
    got3 += (int)k3;
    if (eof3) break;
  }
  fast.join();
  src3.close();
  if (got3 != n3) return fail("socket back-pressure: " + std::to_string(got3) + " lines");
  if (src3.blocked() == 0) return fail("socket back-pressure: the reader never waited");
  return 0;
}

static int test_session_spill_worker() {
  sess::SessionCore main_store(5000, 30000, AGG_SUM_I64), other(5000, 0, AGG_COUNT);
  const int64_t n = 20000;
  std::vector<int64_t> k(n), s(n), e(n), a(n), c(n), f(n), t(n), v(n);
  for (int64_t i = 0; i < n; ++i) {
    k[i] = i;
    s[i] = 1000 * (i % 50);
    e[i] = s[i] + 5000;
    a[i] = i % 13;
    c[i] = 1 + i % 3;
    f[i] = (i % 4 == 0) ? 1 : 0;  // some fired-and-unmodified rows go to a cold chunk
    t[i] = 100000 + (i * 7) % 9000;
    v[i] = i % 100;
  }
  // The spill worker inserts evicted rows while the main thread folds into another store.
  std::thread worker([&] { main_store.insert(k.data(), s.data(), e.data(), a.data(), c.data(),
                                             f.data(), n, true); });
  const int64_t late_other = other.process(k.data(), t.data(), v.data(), n, 0);
  worker.join();  // session_operator.py _join_spill(): before the store is used again
  const int64_t late = main_store.process(k.data(), t.data(), v.data(), n, 90000);
  sess::SessionCore::FireOut o, o2;
  ExprProg empty{};
  main_store.fire(INT64_MAX, empty, empty, o);
  std::thread t2([&] { other.fire(INT64_MAX, empty, empty, o2); });
  t2.join();
  if (late_other != 0 || late < 0 || o.okey.empty() || o2.okey.empty())
    return fail("session store: unexpected result");
  return 0;
}

static int test_kg_writers() {
  const size_t n = 50000;
  std::vector<int32_t> kg(n);
  std::vector<int64_t> col(n);
  for (size_t i = 0; i < n; ++i) {
    kg[i] = (int32_t)((i * 2654435761u) % 128);
    col[i] = (int64_t)i;
  }
  std::vector<std::thread> th;
  std::vector<std::string> paths;
  for (int w = 0; w < 4; ++w) paths.push_back(tmp_path(("kg" + std::to_string(w)).c_str()));
  // kg-sorted copy: the writer's no-permutation path
  std::vector<int32_t> kgs(kg);
  std::vector<int64_t> cols_s(n);
  {
    std::vector<size_t> ord(n);
    for (size_t i = 0; i < n; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return kg[a] < kg[b]; });
    for (size_t i = 0; i < n; ++i) {
      kgs[i] = kg[ord[i]];
      cols_s[i] = col[ord[i]];
    }
  }
  // Writers 0/1: unsorted input (threaded gather), writers 2/3: sorted input; 64 KB pieces so
  // each file is written by the writer's own pool of 4 threads.
  for (int w = 0; w < 4; ++w)
    th.emplace_back([&, w] {
      const bool srt = w >= 2;
      write_kg_columns(paths[w], "{\"rank\": " + std::to_string(w % 2) + "}", 0, 127,
                       srt ? kgs.data() : kg.data(), n,
                       {{(const char*)(srt ? cols_s.data() : col.data()), 8},
                        {(const char*)(srt ? kgs.data() : kg.data()), 4}},
                       4, (size_t)64 << 10);
    });
  for (auto& x : th) x.join();
  std::vector<std::string> body;
  for (auto& p : paths) {
    std::ifstream f(p, std::ios::binary);
    std::string b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() < 8 || std::memcmp(b.data(), "MXSKG001", 8) != 0) return fail("kg file: " + p);
    body.push_back(std::move(b));
    std::remove(p.c_str());
  }
  // sorted and unsorted input of the same rows give the same file
  if (body[0] != body[2] || body[1] != body[3]) return fail("kg file: sorted != unsorted input");
  return 0;
}

// The host window tier's threaded firing: radix-partitioned merge (threads scatter rows into
// partition buffers, then aggregate partitions) and the threaded epilogue, checked against the
// single-threaded sums.
static int test_window_tier_threads() {
  mxs::WindowTierCore t(mxs::AGG_SUM_I64);
  const size_t n = 300000;
  std::vector<uint64_t> key(n);
  std::vector<int64_t> pane(n), acc(n), cnt(n, 1);
  std::vector<uint8_t> dirty(n, 0);
  int64_t expect = 0;
  for (size_t i = 0; i < n; ++i) {
    key[i] = (i * 2654435761u) % 90000;
    pane[i] = (int64_t)(i % 6);
    acc[i] = (int64_t)(i % 97);
    if (pane[i] >= 1 && pane[i] <= 4) expect += acc[i];
  }
  t.absorb(key.data(), pane.data(), acc.data(), cnt.data(), dirty.data(), n / 2);
  t.absorb(key.data() + n / 2, pane.data() + n / 2, acc.data() + n / 2, cnt.data() + n / 2,
           dirty.data() + n / 2, n - n / 2);
  std::vector<uint64_t> dk(1000), k, ok;
  std::vector<int64_t> da(1000, 1), dc(1000, 1), a, c, oraw;
  std::vector<double> ov;
  std::vector<int32_t> oc;
  for (size_t i = 0; i < dk.size(); ++i) dk[i] = 100000 + i;  // keys only the device holds
  t.merge_fire(1, 4, dk.data(), da.data(), dc.data(), dk.size(), false, &k, &a, &c);
  mxs::ExprProg none;
  std::memset(&none, 0, sizeof(none));
  t.epilogue(k, a, c, none, none, 0, 1, &ok, &ov, &oraw, &oc);
  int64_t got = 0;
  for (int64_t x : oraw) got += x;
  if (got != expect + (int64_t)dk.size()) return fail("window tier: threaded merge sum");
  return 0;
}

int main() {
  if (int rc = test_window_tier_threads()) return rc;
  if (int rc = test_text_ring()) return rc;
  if (int rc = test_socket()) return rc;
  if (int rc = test_session_spill_worker()) return rc;
  if (int rc = test_kg_writers()) return rc;
  std::printf("tsan_main ok\n");
  return 0;
}
