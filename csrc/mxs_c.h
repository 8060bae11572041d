/* mxstream — C ABI of the native keyed-window pipeline (csrc/pipeline.cpp).
 *
 * The surface a non-Python host binds to (a JNI layer for the DataStream-style Java API of
 * BASELINE.json, or a C/C++ service): one pipeline = one rank's keyed event-time tumbling /
 * sliding window with allowed lateness and a bounded-out-of-orderness watermark — the
 * reference's BandwidthMonitorWithEventTime shape (chapter3/src/main/java/me/zjy/
 * BandwidthMonitorWithEventTime.java:30-55) — running the gfx950 kernels (device = 1) or their
 * C++ twins (device = 0). Built as build/lib/libmxstream.so by `python -m mxstream.build --capi`.
 *
 * Threading: a pipeline is single-threaded (one caller at a time); distinct pipelines are
 * independent. Errors: functions return < 0 and mxs_last_error() describes the failure.
 */
#ifndef MXS_C_H_
#define MXS_C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MXS_API __attribute__((visibility("default")))

/* Aggregates (same numbering as the engine's AggKind). */
enum { MXS_AGG_SUM_I64 = 0, MXS_AGG_SUM_F64 = 1, MXS_AGG_MIN_I64 = 2, MXS_AGG_MAX_I64 = 3,
       MXS_AGG_MIN_F64 = 4, MXS_AGG_MAX_F64 = 5, MXS_AGG_COUNT = 6, MXS_AGG_AVG_F64 = 7,
       MXS_AGG_AVG_I64 = 8 };

typedef struct mxs_window_config {
  int64_t size_ms;          /* window size */
  int64_t slide_ms;         /* == size_ms for tumbling windows */
  int64_t offset_ms;        /* window offset (0 = epoch aligned) */
  int64_t lateness_ms;      /* allowed lateness (late-but-allowed data re-fires) */
  int64_t ooo_bound_ms;     /* BoundedOutOfOrdernessTimestampExtractor bound */
  int32_t agg;              /* MXS_AGG_* */
  int32_t device;           /* 0 = C++ twins on the host, 1 = HIP device */
  int32_t device_index;     /* HIP device ordinal when device == 1 */
  int32_t max_parallelism;  /* Flink key groups (128) */
  int64_t max_keys;         /* keyed state sizing */
  int64_t batch_capacity;   /* events per process() call (grows on demand) */
} mxs_window_config;

typedef struct mxs_window_result {
  int64_t window_start;
  int64_t window_end;
  uint64_t key;
  double value;             /* aggregate result (avg = sum / count; f64 aggregates as double) */
  int64_t raw;              /* raw accumulator: exact integer sum / f64 bit pattern */
  uint32_t count;           /* elements in the window */
  int32_t refire;           /* 1: re-firing caused by late-but-allowed data */
} mxs_window_result;

typedef struct mxs_pipeline mxs_pipeline;

MXS_API void mxs_window_config_default(mxs_window_config* cfg);
MXS_API mxs_pipeline* mxs_pipeline_create(const mxs_window_config* cfg);
MXS_API void mxs_pipeline_destroy(mxs_pipeline* p);
/* One micro-batch of host arrays (keys, event timestamps in ms, int64 values / f64 bit
 * patterns). Fires every window the advanced watermark allows; results queue up until taken. */
MXS_API int mxs_pipeline_process(mxs_pipeline* p, const uint64_t* keys, const int64_t* ts,
                                 const int64_t* vals, int64_t n);
/* End of input: Long.MAX_VALUE watermark fires every remaining window. */
MXS_API int mxs_pipeline_finish(mxs_pipeline* p);
MXS_API int64_t mxs_pipeline_num_results(const mxs_pipeline* p);
/* Moves up to `cap` queued results into `out`; returns how many were written. */
MXS_API int64_t mxs_pipeline_take_results(mxs_pipeline* p, mxs_window_result* out, int64_t cap);
MXS_API int64_t mxs_pipeline_watermark(const mxs_pipeline* p);
MXS_API int64_t mxs_pipeline_late_dropped(const mxs_pipeline* p);
MXS_API int64_t mxs_pipeline_records_in(const mxs_pipeline* p);
/* ---- keyed rolling aggregates and tumbling count windows ------------------------------------
 * keyBy(k).sum/min/max(v) with one output row per input record (StreamGroupedReduce,
 * chapter2/src/main/java/me/zjy/ComputeCpuMax.java:26), or keyBy(k).countWindow(n) with an
 * incremental aggregate (one row per completed window; count_window = n > 0). One rank; the
 * gfx950 kernels (device = 1: table lookup -> radix sort -> per-key ordered / segmented wave
 * scan) or their C++ twins (device = 0). Rows come out in input order of the emitting records. */
typedef struct mxs_rolling_config {
  int32_t agg;              /* MXS_AGG_* (avg only with count windows) */
  int32_t device;           /* 0 = C++ twins, 1 = HIP device */
  int32_t device_index;
  int32_t reserved;
  int64_t max_keys;         /* keyed state sizing */
  int64_t batch_capacity;   /* events per process() call (grows on demand) */
  int64_t count_window;     /* 0: rolling aggregate; n > 0: tumbling count windows of n */
} mxs_rolling_config;

typedef struct mxs_rolling_row {
  uint64_t key;
  int64_t raw;              /* aggregate: integer / f64 bit pattern (avg: the sum); count: n */
  int64_t index;            /* position of the emitting record in its process() batch */
} mxs_rolling_row;

typedef struct mxs_rolling mxs_rolling;

MXS_API void mxs_rolling_config_default(mxs_rolling_config* cfg);
MXS_API mxs_rolling* mxs_rolling_create(const mxs_rolling_config* cfg);
MXS_API void mxs_rolling_destroy(mxs_rolling* r);
/* One micro-batch (host arrays: keys, int64 values / f64 bit patterns); rows queue up. */
MXS_API int mxs_rolling_process(mxs_rolling* r, const uint64_t* keys, const int64_t* vals,
                                int64_t n);
MXS_API int64_t mxs_rolling_num_rows(const mxs_rolling* r);
MXS_API int64_t mxs_rolling_take_rows(mxs_rolling* r, mxs_rolling_row* out, int64_t cap);

/* ---- keyed event-time session windows --------------------------------------------------------
 * keyBy(k).window(EventTimeSessionWindows.withGap(gap)) with an incremental aggregate, allowed
 * lateness (late-but-allowed elements merge into fired sessions and re-fire them) and a
 * bounded-out-of-orderness watermark (chapter3/README.md:412-428). Host C++ session store (the
 * CPU engine and host-DRAM tier of the GPU session operator, csrc/session_store.h). */
typedef struct mxs_session_config {
  int64_t gap_ms;           /* session gap */
  int64_t lateness_ms;      /* allowed lateness */
  int64_t ooo_bound_ms;     /* BoundedOutOfOrdernessTimestampExtractor bound */
  int32_t agg;              /* MXS_AGG_* */
  int32_t reserved;
} mxs_session_config;

typedef struct mxs_session_result {
  uint64_t key;
  int64_t start;            /* session [start, end) */
  int64_t end;
  double value;             /* aggregate result */
  int64_t raw;              /* raw accumulator */
  uint32_t count;           /* elements in the session */
  int32_t refire;           /* 1: re-firing caused by late-but-allowed data */
} mxs_session_result;

typedef struct mxs_session mxs_session;

MXS_API void mxs_session_config_default(mxs_session_config* cfg);
MXS_API mxs_session* mxs_session_create(const mxs_session_config* cfg);
MXS_API void mxs_session_destroy(mxs_session* s);
/* One micro-batch (keys, event timestamps in ms, int64 values / f64 bit patterns). Elements are
 * checked for lateness against the watermark before the batch; then the watermark advances
 * (max ts - bound) and every session it passes fires. Results queue up until taken. */
MXS_API int mxs_session_process(mxs_session* s, const uint64_t* keys, const int64_t* ts,
                                const int64_t* vals, int64_t n);
MXS_API int mxs_session_finish(mxs_session* s);
MXS_API int64_t mxs_session_num_results(const mxs_session* s);
MXS_API int64_t mxs_session_take_results(mxs_session* s, mxs_session_result* out, int64_t cap);
MXS_API int64_t mxs_session_watermark(const mxs_session* s);
MXS_API int64_t mxs_session_late_dropped(const mxs_session* s);

MXS_API const char* mxs_last_error(void);
MXS_API const char* mxs_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MXS_C_H_ */
