"""flink_amd — MI355X-native keyed event-time window aggregation (drop-in for Flink's
WindowOperator on the keyBy().window(...).aggregate/reduce path).

The compute path is libgpuwin.so (hand-written gfx950 HIP kernels behind the C ABI in
include/gpuwin.h); this package is its host-side mirror of the reference interface.
"""
from .windowing import (  # noqa: F401
    MAX_WATERMARK, DataStream, Duration, EventTimeSessionWindows, EventTimeTrigger, GpuWindowOperator,
    KeyedStream, PurgingTrigger, SlidingEventTimeWindows, StreamExecutionEnvironment, StreamRecord,
    TumblingEventTimeWindows, Watermark, WindowedStream, assign_to_key_group,
    compute_default_max_parallelism, compute_key_group_range_for_operator_index,
    compute_operator_index_for_key_group, java_hash, java_string_hash,
)
from ._native import GpuWinError, NativeLibraryError  # noqa: F401

__all__ = [n for n in dir() if not n.startswith("_")]
