"""mxstream — an MI355X-native stateful stream-processing engine.

A from-scratch re-design (not a port) of the capabilities of the
`monitor-systam-flink-quickstart` Flink tutorial: threshold alerts, keyed state, event-time
tumbling/sliding windows with watermarks, allowed lateness, session windows and checkpoints —
executed as micro-batches by gfx950 HIP kernels (LDS-resident hash sub-tables, fused window
firing) with the keyBy shuffle as an RCCL all-to-all over xGMI, one process per GPU.

Entry points:
  mxstream.api           Flink-style DataStream API (StreamExecutionEnvironment, keyBy, ...)
  mxstream.runtime       native-backed operators (KeyedWindowOperator, ...)
  mxstream.parallel      torch.distributed / RCCL communication
  mxstream.models        the reference's pipelines and the BASELINE benchmark configs
"""
__version__ = "0.1.0"
