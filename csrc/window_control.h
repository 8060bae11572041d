// mxstream — the host control state of a keyed event-/processing-time window operator: Flink 1.8
// window arithmetic (TimeWindow.getWindowStartWithOffset with Java's truncated remainder,
// SlidingEventTimeWindows' assignment of an element to size/slide windows) and the bookkeeping
// that drives firing, late re-firing and purging of the pane ring. ONE implementation shared by
// the Python-bound operator (runtime/window_operator.py KeyedWindowOperator, through the
// pybind class WindowControl) and the C ABI pipeline (csrc/pipeline.cpp WindowPipeline).
//
// Reference semantics: chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:46
// (timeWindow(5 min, 5 s)), chapter3/README.md:209-228 (allowed lateness: a late element
// re-fires its window until maxTimestamp + lateness <= watermark, then the window is cleaned).
//
// State (host only, identical on every rank):
//   nfs        smallest window start not yet evaluated (every window starting before it is
//              due and has fired);
//   [min_live, max_seen]  the live pane range (oldest unpurged pane, newest pane with data).
// Panes are gcd(size, slide) long; pane p covers [offset + p * pane, offset + (p + 1) * pane).
#ifndef MXS_WINDOW_CONTROL_H_
#define MXS_WINDOW_CONTROL_H_

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <stdexcept>
#include <vector>

namespace mxs {

class WindowControl {
 public:
  using i128 = __int128;
  static constexpr int64_t kMin = INT64_MIN, kMax = INT64_MAX;

  WindowControl(int64_t size, int64_t slide, int64_t offset, int64_t lateness)
      : size_(size), slide_(slide), offset_(offset), late_(lateness) {
    if (size <= 0 || slide <= 0) throw std::invalid_argument("window size and slide must be positive");
    if (lateness < 0) throw std::invalid_argument("negative allowed lateness");
    pane_ = std::gcd(size, slide);
    ppw_ = size / pane_;
  }

  int64_t size() const { return size_; }
  int64_t slide() const { return slide_; }
  int64_t offset() const { return offset_; }
  int64_t lateness() const { return late_; }
  int64_t pane() const { return pane_; }
  int64_t panes_per_window() const { return ppw_; }

  // ---- window arithmetic ------------------------------------------------------------------
  static int64_t clamp64(i128 v) { return v > kMax ? kMax : v < kMin ? kMin : (int64_t)v; }
  static i128 fdiv(i128 a, i128 b) {  // floor division
    i128 q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
  }
  static i128 java_rem(i128 a, i128 b) {  // Java's % on long: sign of the dividend
    const i128 r = (a < 0 ? -a : a) % (b < 0 ? -b : b);
    return a < 0 ? -r : r;
  }
  int64_t pane_of(i128 t) const { return clamp64(fdiv(t - offset_, pane_)); }
  int64_t pane_start(i128 p) const { return clamp64((i128)offset_ + p * pane_); }
  // TimeWindow.getWindowStartWithOffset(t, offset, slide)
  i128 last_start128(i128 t) const { return t - java_rem(t - offset_ + slide_, slide_); }
  int64_t last_start(i128 t) const { return clamp64(last_start128(t)); }
  // First window start whose window [s, s + size) contains t.
  int64_t first_start_containing(i128 t) const {
    const i128 ls = last_start128(t);
    return clamp64(ls - fdiv(ls - (t - size_ + 1), slide_) * slide_);
  }
  // Smallest window start >= t.
  int64_t align_up(i128 t) const {
    const i128 ls = last_start128(t);
    return clamp64(ls >= t ? ls : ls + slide_);
  }
  // Newest pane of the newest window already evaluated (kMin: none).
  int64_t fired_hi() const {
    if (!has_nfs_) return kMin;
    return pane_of((i128)nfs_ - slide_ + size_ - 1);
  }
  // Smallest window start whose cleanup time (maxTs + lateness) is after wm: elements of older
  // windows only are late (dropped). Processing time: nothing is late.
  int64_t late_ts(int64_t wm, bool event_time = true) const {
    if (wm == kMin || !event_time) return kMin;
    return align_up((i128)wm - size_ - late_ + 2);
  }
  // The step's base pane when a watermark exists (every non-late element has
  // ts >= wm - size - lateness + 1); kMin otherwise (the caller takes the batch minimum).
  int64_t pane_base_from_wm(int64_t wm) const {
    if (wm == kMin) return kMin;
    return pane_of((i128)wm - size_ - late_ + 1);
  }

  // ---- bookkeeping ------------------------------------------------------------------------
  bool has_nfs() const { return has_nfs_; }
  bool has_live() const { return has_live_; }
  int64_t nfs() const { return nfs_; }
  int64_t min_live() const { return min_live_; }
  int64_t max_seen() const { return max_seen_; }
  void set_nfs(bool has, int64_t v) {
    has_nfs_ = has;
    nfs_ = has ? v : 0;
  }
  void set_live(bool has, int64_t lo, int64_t hi) {
    has_live_ = has;
    min_live_ = has ? lo : 0;
    max_seen_ = has ? hi : 0;
  }

  // A settled step's data panes [gmin, gmax] (absolute): the live range grows to hold them and
  // the fire cursor moves back to the first not-yet-due window that contains new data. Returns
  // the number of consecutive panes the ring must hold (the caller grows it first when larger)
  // -- call commit_live() after growing.
  int64_t live_span_with(int64_t gmin, int64_t gmax) const {
    const int64_t lo = has_live_ ? std::min(min_live_, gmin) : gmin;
    const int64_t hi = has_live_ ? std::max(max_seen_, gmax) : gmax;
    return clamp64((i128)hi - lo + 1);
  }
  void observe(int64_t gmin, int64_t gmax, int64_t old_wm) {
    const int64_t lo = has_live_ ? std::min(min_live_, gmin) : gmin;
    const int64_t hi = has_live_ ? std::max(max_seen_, gmax) : gmax;
    min_live_ = lo;
    max_seen_ = hi;
    has_live_ = true;
    // Invariant: every window starting before nfs is due and has been evaluated. New data can
    // belong to not-yet-due windows before the cursor (older but not late): lower the cursor
    // to the first such window. Due windows that receive data (lateness) re-fire instead.
    int64_t cand = first_start_containing(pane_start(gmin));
    if (old_wm > kMin) cand = std::max(cand, align_up((i128)old_wm - size_ + 2));
    nfs_ = has_nfs_ ? std::min(nfs_, cand) : cand;
    has_nfs_ = true;
  }

  // Window [s, s + size) overlaps the live pane range.
  bool overlaps_live(int64_t s) const {
    if (!has_live_) return false;
    const int64_t p0 = pane_of(s), p1 = clamp64((i128)p0 + ppw_ - 1);
    return !(p1 < min_live_ || p0 > max_seen_);
  }
  // Pane range [p0, p1] of window s clipped to the live range (p1 < p0: no live pane).
  std::pair<int64_t, int64_t> window_panes(int64_t s) const {
    const int64_t p = pane_of(s);
    return {std::max(p, min_live_), std::min(clamp64((i128)p + ppw_ - 1), max_seen_)};
  }

  // Windows the watermark makes due (maxTimestamp <= wm), oldest first, skipping windows that
  // hold no live pane; the cursor moves past them (and jumps over data-free stretches).
  std::vector<int64_t> take_due(int64_t wm) {
    std::vector<int64_t> due;
    if (!has_nfs_ || !has_live_) return due;
    i128 s = nfs_;
    const int64_t first_live = first_start_containing(pane_start(min_live_));
    if (s < first_live) s = first_live;
    const i128 last_data_start = last_start128((i128)pane_start((i128)max_seen_ + 1) - 1);
    while (s + size_ - 1 <= wm) {
      if (s > last_data_start) {
        // No window beyond the newest pane holds data: jump to the first window that can.
        const i128 a = align_up((i128)wm - size_ + 2);
        s = s > a ? s : a;
        break;
      }
      if (overlaps_live((int64_t)s)) due.push_back((int64_t)s);
      s += slide_;
    }
    nfs_ = clamp64(s);
    return due;
  }
  // Upper bound of the windows a settled step will fire or re-fire (latency-bounded firing):
  // re-firings of data panes [gmin, min(gmax, fired_hi)] plus first firings up to new_wm.
  int64_t due_count(bool has_data, int64_t gmin, int64_t gmax, int64_t fhi, bool has_new_wm,
                    int64_t new_wm) const {
    int64_t n = 0;
    if (has_data && gmin <= fhi && has_nfs_) {
      const i128 s0 = first_start_containing(pane_start(gmin));
      const i128 s1 = std::min<i128>((i128)nfs_ - slide_,
                                     last_start128(pane_start(std::min(gmax, fhi))));
      if (s1 >= s0) n += clamp64((s1 - s0) / slide_ + 1);
    }
    if (has_new_wm && has_nfs_) {
      const i128 last = (i128)new_wm - size_ + 1;  // windows with start <= last are due
      if (last >= nfs_) n += clamp64((last - nfs_) / slide_ + 1);
    }
    return n;
  }
  // Windows to re-fire after late-but-allowed data landed in panes [pmin, pmax] (already
  // evaluated windows not cleaned at the step's old watermark).
  std::vector<int64_t> refire_windows(int64_t pmin, int64_t pmax, int64_t old_wm) const {
    std::vector<int64_t> out;
    if (!has_nfs_) return out;
    i128 s = first_start_containing(pane_start(pmin));
    const i128 end_s = std::min<i128>((i128)nfs_ - slide_, last_start128(pane_start(pmax)));
    for (; s <= end_s; s += slide_)
      if (s + size_ - 1 + late_ > old_wm) out.push_back((int64_t)s);
    return out;
  }
  // Purge after watermark wm: panes [from, stop) are to be zeroed (at most `ring` of them, the
  // oldest are already gone); the live range starts at keep_from afterwards. Returns
  // {keep_from, from, stop}; from >= stop: nothing to zero.
  struct Purge {
    int64_t keep_from, from, stop;
  };
  Purge purge_range(int64_t wm, int64_t ring) const {
    Purge r{kMin, 0, 0};
    if (!has_live_) return r;
    if (wm == kMax) {
      r.keep_from = clamp64((i128)max_seen_ + 1);
    } else {
      // Earliest window that is not cleaned: s + size - 1 + lateness > wm.
      r.keep_from = pane_of(align_up((i128)wm - size_ - late_ + 2));
    }
    r.from = min_live_;
    r.stop = std::min(r.keep_from, clamp64((i128)max_seen_ + 1));
    if ((i128)r.stop - r.from > ring) r.from = clamp64((i128)r.stop - ring);
    return r;
  }
  void commit_purge(int64_t keep_from) {
    if (!has_live_ || keep_from <= min_live_) return;
    min_live_ = keep_from;
    if (min_live_ > max_seen_) {
      has_live_ = false;
      min_live_ = max_seen_ = 0;
    }
  }

 private:
  int64_t size_, slide_, offset_, late_, pane_, ppw_;
  int64_t nfs_ = 0, min_live_ = 0, max_seen_ = 0;
  bool has_nfs_ = false, has_live_ = false;
};

}  // namespace mxs

#endif  // MXS_WINDOW_CONTROL_H_
