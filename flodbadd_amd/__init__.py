"""flodbadd_amd -- MI355X (gfx950) packet-parse + flow-classification path for flodbadd.

Drop-in for the reference's per-frame `parse_packet_pcap` + `process_parsed_packet`
(src/packets.rs:202-802, called from src/capture.rs:1036-1061): a C ABI
(include/flodbadd_gpu.h, libflodbadd_gpu.so) over hand-written HIP kernels, plus this thin
Python host mirror used by the tests and the bench.
"""
from . import _native
from ._native import (DNS_OUT_DTYPE, FB_CLASS_DNS, FB_CLASS_DROP, FB_CLASS_FILTERED, FB_CLASS_SESSION,
                      FLOW_REC_DTYPE, PKT_OUT_DTYPE, STATS_DTYPE, FbError, NativeLibraryMissing, gpu_lib)
from .sessions import Protocol, Session, SessionFilter, SessionInfo, SessionPacketData, SessionStats
from .queue import DeviceSegBatch, SegQueue

__all__ = ["_native", "DeviceSegBatch", "SegQueue", "gpu_lib", "FbError", "NativeLibraryMissing", "PKT_OUT_DTYPE", "DNS_OUT_DTYPE",
           "STATS_DTYPE", "FLOW_REC_DTYPE", "FB_CLASS_SESSION", "FB_CLASS_DNS", "FB_CLASS_DROP",
           "FB_CLASS_FILTERED", "Protocol", "Session", "SessionFilter", "SessionInfo", "SessionPacketData",
           "SessionStats"]


def FlodbaddGpuCapture(*args, **kwargs):  # lazy import keeps `import flodbadd_amd` light
    from .capture import FlodbaddGpuCapture as _C
    return _C(*args, **kwargs)
