"""One batch per call without a launch per call: the resident queue-fed parse (fb_seg_queue_*,
DESIGN §3.7) for a Python capture loop.

    cap = FlodbaddGpuCapture(0)
    batches = [DeviceSegBatch(frames, offsets) for ...]   # device buffers first: hipFree waits for
    with SegQueue(cap, depth=8) as q:                      # the queue's kernel while it lives
        t = q.submit(batches[0])
        ...
        q.wait(t)
        records, dns, classes, stats = batches[0].result()

The outputs are exactly FlodbaddGpuCapture.process_frames_seg's parse half
(fb_parse_classify_seg_dev): records compacted per 64-frame segment, DNS side records, classes and
PACKET_STATS.  One queue per device at a time.  There is no CPU fallback: the HIP library must load.
"""
import ctypes as C

import numpy as np

from . import _native as N


class DeviceSegBatch:
    """Device buffers of one frame batch (frames, offsets) and of its segmented outputs, with the
    fb_seg_batch descriptor the queue takes.  `load` re-fills it with another batch that fits."""

    def __init__(self, frames, offsets, with_classes=True, max_frames=None, max_bytes=None):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = len(offsets) - 1
        self.cap_frames = max(int(max_frames or n), 1)
        self.cap_bytes = max(int(max_bytes or frames.nbytes), 1)
        nseg = (self.cap_frames + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES
        self._fr = N.DeviceBuffer(self.cap_bytes)
        self._of = N.DeviceBuffer(4 * (self.cap_frames + 1))
        self._out = N.DeviceBuffer(nseg * N.SEG_BYTES)
        self._seg = N.DeviceBuffer(nseg * 4)
        self._cls = N.DeviceBuffer(self.cap_frames) if with_classes else None
        self._st = N.DeviceBuffer(N.STATS_DTYPE.itemsize)
        self.desc = np.zeros(1, dtype=N.SEG_BATCH_DTYPE)
        self.load(frames, offsets)

    def load(self, frames, offsets):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        n = len(offsets) - 1
        if n > self.cap_frames or frames.nbytes > self.cap_bytes:
            raise ValueError("batch of %d frames / %d bytes exceeds this buffer set (%d / %d)"
                             % (n, frames.nbytes, self.cap_frames, self.cap_bytes))
        if frames.nbytes:
            self._fr.upload(frames)
        self._of.upload(offsets)
        self.n, self.frames_bytes = n, frames.nbytes
        self.desc[0] = (self._fr.ptr.value, frames.nbytes, self._of.ptr.value, n, 0, self._out.ptr.value,
                        self._seg.ptr.value, self._cls.ptr.value if self._cls else 0, self._st.ptr.value)
        return self

    def fill_outputs(self, byte=0xA5, stats_byte=0xEE):
        """Overwrite the output buffers (copies from the host: while a queue lives its kernel holds
        the CUs a fill kernel would need) -- the tests check that nothing outside a segment's records
        is written."""
        self._out.upload(np.full(self._out.nbytes, byte, dtype=np.uint8))
        self._st.upload(np.full(self._st.nbytes, stats_byte, dtype=np.uint8))

    def raw(self):
        """(segment bytes, per-segment counts, classes or None, stats) as the device holds them."""
        n, nseg = self.n, max((self.n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES, 1)
        raw = self._out.download(np.zeros(nseg * N.SEG_BYTES, dtype=np.uint8))
        seg = self._seg.download(np.zeros(nseg, dtype=np.uint32))[: (n + N.FB_SEG_FRAMES - 1) // N.FB_SEG_FRAMES]
        cls = self._cls.download(np.zeros(max(n, 1), dtype=np.uint8))[:n] if self._cls else None
        st = self._st.download(np.zeros(1, dtype=N.STATS_DTYPE))
        return raw, seg, cls, st

    def update_table(self, capture, stream=None):
        """Apply this (completed) batch's SESSION records to `capture`'s session table
        (fb_flow_update_seg_dev on `stream`, asynchronous) -- beside a queue created shared."""
        N.check(N.gpu_lib().fb_flow_update_seg_dev(capture.ctx, self._out.ptr, self._seg.ptr, self.n, self._st.ptr,
                                                   stream))

    def result(self):
        """(SESSION records in packet order, DNS records, classes or None, stats)."""
        raw, seg, cls, st = self.raw()
        out, dns = N.seg_unpack(raw, seg)
        return out, dns, cls, st

    def free(self):
        for b in (self._fr, self._of, self._out, self._seg, self._cls, self._st):
            if b is not None:
                b.free()


class SegQueue:
    """fb_seg_queue_* over a FlodbaddGpuCapture's context (its filter, service table, LAN prefixes
    and own IPs as they are at creation)."""

    def __init__(self, capture, depth=8, idle_ms=0, shared=False):
        """shared: FB_QUEUE_SHARED -- one workgroup on each of an eighth of the CUs, leaving the rest to the context's table
        update kernels beside the resident parse (a loop applying each completed batch to the table)."""
        self._lib = N.gpu_lib()
        q = self._lib.fb_seg_queue_create_ex(capture.ctx, int(depth), int(idle_ms),
                                             N.FB_QUEUE_SHARED if shared else 0)
        if not q:
            raise N.FbError(N.FB_ERR_INVAL, self._lib.fb_last_error().decode(errors="replace"))
        self._q = C.c_void_p(q)
        self._live = {}  # ticket -> batch (kept alive until its ticket is waited for)

    def submit(self, batch):
        """Hand `batch` (a DeviceSegBatch) to the running kernel; returns its ticket.  Blocks only
        while `depth` batches are in flight."""
        t = C.c_uint64()
        N.check(self._lib.fb_seg_queue_submit(self._q, N.ptr(batch.desc), C.byref(t)))
        self._live[t.value] = batch
        return t.value

    def set_limit(self, limit):
        """Lower the queue's submission limit (fb_seg_queue_set_limit): the submit past it fails with
        FB_ERR_INVAL, as the one past FB_QUEUE_MAX_SUBMISSIONS does."""
        N.check(self._lib.fb_seg_queue_set_limit(self._q, int(limit)))

    def done(self, ticket):
        rc = self._lib.fb_seg_queue_query(self._q, int(ticket))
        if rc < 0:
            N.check(rc)
        if rc == N.FB_OK:
            self._live.pop(ticket, None)
        return rc == N.FB_OK

    def wait(self, ticket):
        N.check(self._lib.fb_seg_queue_wait(self._q, int(ticket)))
        self._live.pop(ticket, None)

    def close(self):
        if self._q:
            rc = self._lib.fb_seg_queue_destroy(self._q)
            self._q = None
            self._live.clear()
            N.check(rc)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
