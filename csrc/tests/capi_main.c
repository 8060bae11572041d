/* mxstream — C ABI smoke/golden test (built and run by tests/test_capi.py).
 *
 * Replays the chapter3 README stream of BandwidthMonitorWithEventTime (chapter3/README.md:285-289:
 * 5-min / 5-s sliding event-time windows, 1-min out-of-orderness bound, one record per
 * micro-batch) through the C ABI and checks the firings SURVEY.md Appendix A.4 derives: 12
 * windows of sum 10000, 12 of 10100 and 36 of 10200 before end of input, the 09:01 record dropped
 * as late, and the Mbps map of the reference (sum * 8.0 / 60 / 1024 / 1024).
 * Usage: capi_main <device: 0 = host twins, 1 = HIP device>
 */
#include <stdio.h>
#include <stdlib.h>

#include "mxs_c.h"

#define T0 1566957600000LL /* 2019-08-28T10:00:00+08:00 in epoch ms */

int main(int argc, char** argv) {
  mxs_window_config cfg;
  mxs_window_config_default(&cfg);
  cfg.size_ms = 5 * 60 * 1000;
  cfg.slide_ms = 5 * 1000;
  cfg.ooo_bound_ms = 60 * 1000;
  cfg.agg = MXS_AGG_SUM_I64;
  cfg.device = argc > 1 ? atoi(argv[1]) : 0;
  cfg.max_keys = 1024;
  mxs_pipeline* p = mxs_pipeline_create(&cfg);
  if (!p) {
    fprintf(stderr, "create failed: %s\n", mxs_last_error());
    return 2;
  }
  const int64_t ts[5] = {T0, T0 + 60000, T0 + 120000, T0 - 59 * 60000, T0 + 360000};
  const int64_t val[5] = {10000, 100, 100, 100, 100};
  const uint64_t key = 1; /* dictionary id of "www.163.com" */
  int n10000 = 0, n10100 = 0, n10200 = 0, other = 0;
  mxs_window_result r[256];
  for (int i = 0; i < 5; ++i) {
    if (mxs_pipeline_process(p, &key, &ts[i], &val[i], 1) != 0) {
      fprintf(stderr, "process failed: %s\n", mxs_last_error());
      return 3;
    }
    int64_t n;
    while ((n = mxs_pipeline_take_results(p, r, 256)) > 0)
      for (int64_t j = 0; j < n; ++j) {
        if (r[j].key != key || r[j].window_end - r[j].window_start != cfg.size_ms) ++other;
        else if (r[j].raw == 10000) ++n10000;
        else if (r[j].raw == 10100) ++n10100;
        else if (r[j].raw == 10200) ++n10200;
        else ++other;
      }
  }
  const double mbps = 10000 * 8.0 / 60 / 1024 / 1024;
  printf("fired: %d x 10000 (%.19g Mbps), %d x 10100, %d x 10200, other %d; late dropped %lld\n",
         n10000, mbps, n10100, n10200, other, (long long)mxs_pipeline_late_dropped(p));
  int ok = n10000 == 12 && n10100 == 12 && n10200 == 36 && other == 0 &&
           mxs_pipeline_late_dropped(p) == 1;
  /* End of input: MAX watermark fires the 72 windows still open (sums 10200 .. 100). */
  if (mxs_pipeline_finish(p) != 0) return 4;
  const int64_t rest = mxs_pipeline_num_results(p);
  printf("after finish: %lld more windows, watermark %lld\n", (long long)rest,
         (long long)mxs_pipeline_watermark(p));
  ok = ok && rest == 72;
  mxs_pipeline_destroy(p);
  printf("%s\n", ok ? "capi ok" : "capi MISMATCH");
  return ok ? 0 : 1;
}
