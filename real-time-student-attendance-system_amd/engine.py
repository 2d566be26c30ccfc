"""Device-resident batches and the device-side driver used by the benchmark,
the GPU parity tests and the sharded runner.

Inputs of the hot path are kept resident in HBM (``DeviceBatch``: packed id
bytes + u32 offsets + u32 key slots), generated on the GPU by the
counter-based generator, so a timed step is one K1 launch over a batch that
is already on the device.
"""
from __future__ import annotations

import ctypes as C
import gc

import numpy as np

from ._lib import Context, GenParams, SKE_MEM_DEVICE
from . import synthetic

PASS_KINDS = 9  # SKE_PASS_KINDS (include/sketch.h)


class _no_gc:
    """Collect cyclic garbage now, then keep the collector off until exit
    (around a stream capture: see SketchEngine.capture)."""

    def __enter__(self):
        gc.collect()
        self.was = gc.isenabled()
        gc.disable()

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


class DeviceBuffer:
    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        p = C.c_void_p()
        ctx.call("ske_device_alloc", int(max(nbytes, 16)), C.byref(p))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    def free(self):
        if self.ptr:
            self.ctx.call("ske_device_free", C.c_void_p(self.ptr))
            self.ptr = None

    def to_host(self, dtype, count) -> np.ndarray:
        out = np.zeros(count, dtype)
        if out.nbytes:
            self.ctx.call("ske_memcpy", out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr),
                          out.nbytes, 1)
        return out

    def from_host(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        if a.nbytes:
            self.ctx.call("ske_memcpy", C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p),
                          a.nbytes, 0)


class SweBatch(C.Structure):
    """ske_swipe_batch (include/sketch.h)."""
    _fields_ = [("slot", C.c_void_p), ("bytes", C.c_void_p), ("offs", C.c_void_p),
                ("width", C.c_uint32), ("n", C.c_uint64), ("out_valid", C.c_void_p)]


class DeviceBatch:
    """Packed swipes resident on the device."""

    def __init__(self, ctx: Context, n: int, width: int):
        self.ctx, self.n, self.width = ctx, int(n), int(width)
        self.bytes = DeviceBuffer(ctx, self.n * width + 64)
        self.offs = DeviceBuffer(ctx, (self.n + 1) * 4)
        self.slot = DeviceBuffer(ctx, self.n * 4 + 16)

    @classmethod
    def from_host(cls, ctx: Context, buf: np.ndarray, offs: np.ndarray, slot: np.ndarray):
        b = cls.__new__(cls)
        b.ctx, b.n, b.width = ctx, len(offs) - 1, 0
        b.bytes = DeviceBuffer(ctx, buf.nbytes + 64)
        b.offs = DeviceBuffer(ctx, offs.nbytes)
        b.slot = DeviceBuffer(ctx, max(slot.nbytes, 16))
        b.bytes.from_host(np.ascontiguousarray(buf, np.uint8))
        b.offs.from_host(np.ascontiguousarray(offs, np.uint32))
        b.slot.from_host(np.ascontiguousarray(slot, np.uint32))
        return b

    def to_host(self):
        offs = self.offs.to_host(np.uint32, self.n + 1)
        buf = self.bytes.to_host(np.uint8, int(offs[-1]))
        slot = self.slot.to_host(np.uint32, self.n)
        return buf, offs, slot

    def free(self):
        for b in (self.bytes, self.offs, self.slot):
            b.free()


class Graph:
    """An executable HIP graph of recorded sketch calls (ske_capture_end)."""

    def __init__(self, ctx: Context, ptr: int):
        self.ctx, self.ptr = ctx, ptr

    def launch(self):
        self.ctx.call("ske_graph_launch", C.c_void_p(self.ptr))

    def free(self):
        if self.ptr:
            self.ctx.call("ske_graph_free", C.c_void_p(self.ptr))
            self.ptr = None


class SketchEngine:
    """Device-pointer driver over one libsketch context."""

    def __init__(self, device: int = 0, ctx: Context | None = None):
        self.ctx = ctx if ctx is not None else Context(device)
        self._cdf_bufs = []

    # ---- Bloom
    def reserve(self, fid: int, error: float, capacity: int, expansion: int = 2,
                nonscaling: bool = False):
        self.ctx.call("ske_bf_reserve", fid, float(error), int(capacity), int(expansion),
                      1 if nonscaling else 0)

    def gen_params(self, w: synthetic.Workload, seed=None, slot_base=0,
                   cdf: np.ndarray | None = None) -> GenParams:
        """Generator parameters; `cdf` (u32, n_keys entries) overrides the
        workload's own key distribution (e.g. a rank's share of the keys)."""
        if cdf is None:
            cdf = synthetic.key_cdf(w)
        dev = None
        if cdf is not None:
            buf = DeviceBuffer(self.ctx, cdf.nbytes)
            buf.from_host(cdf)
            self._cdf_bufs.append(buf)
            dev = buf.ptr
        return synthetic.gen_params(w, seed=seed, slot_base=slot_base, key_cdf_dev=dev)

    def members_batch(self, p: GenParams, start: int, n: int) -> DeviceBatch:
        width = self.ctx.lib.ske_gen_id_width(C.byref(p))
        b = DeviceBatch(self.ctx, n, width)
        self.ctx.call("ske_gen_members", C.byref(p), int(start), int(n), C.c_void_p(b.bytes.ptr),
                      C.c_void_p(b.offs.ptr))
        return b

    def preload(self, fid: int, p: GenParams, n: int, chunk: int = 1 << 24,
                replies: bool = False) -> np.ndarray | None:
        """BF.MADD of the first n members (data_generator.py:57-63 scaled)."""
        outs = []
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            b = self.members_batch(p, s, m)
            out = DeviceBuffer(self.ctx, m) if replies else None
            self.ctx.call("ske_bf_madd", fid, C.c_void_p(b.bytes.ptr), C.c_void_p(b.offs.ptr), m,
                          C.c_void_p(out.ptr) if out else None, SKE_MEM_DEVICE)
            if out:
                outs.append(out.to_host(np.int8, m))
                out.free()
            b.free()
        return np.concatenate(outs) if replies else None

    def swipe_batch(self, p: GenParams, start: int, n: int) -> DeviceBatch:
        width = self.ctx.lib.ske_gen_id_width(C.byref(p))
        b = DeviceBatch(self.ctx, n, width)
        self.ctx.call("ske_gen_swipes", C.byref(p), int(start), int(n), C.c_void_p(b.bytes.ptr),
                      C.c_void_p(b.offs.ptr), C.c_void_p(b.slot.ptr))
        return b

    # ---- hot path
    def hll_reserve(self, nslots: int):
        self.ctx.call("ske_hll_reserve", int(nslots))

    def swipes(self, fid: int, b: DeviceBatch, out: DeviceBuffer | None = None):
        self.ctx.call("ske_swipes", fid, C.c_void_p(b.slot.ptr), C.c_void_p(b.bytes.ptr),
                      C.c_void_p(b.offs.ptr), b.n, C.c_void_p(out.ptr) if out else None,
                      SKE_MEM_DEVICE)

    def swipes_async(self, fid: int, b: DeviceBatch, out: DeviceBuffer | None = None):
        self.ctx.call("ske_swipes_async", fid, C.c_void_p(b.slot.ptr), C.c_void_p(b.bytes.ptr),
                      C.c_void_p(b.offs.ptr), b.n, C.c_void_p(out.ptr) if out else None)

    def swipes_fixed(self, fid: int, b: DeviceBatch, out: DeviceBuffer | None = None):
        """K1 over a fixed-width batch (ids at bytes + i*width, no offsets)."""
        assert b.width > 0
        self.ctx.call("ske_swipes_fixed", fid, C.c_void_p(b.slot.ptr), C.c_void_p(b.bytes.ptr),
                      b.width, b.n, C.c_void_p(out.ptr) if out else None, SKE_MEM_DEVICE)

    def swipes_fixed_async(self, fid: int, b: DeviceBatch, out: DeviceBuffer | None = None):
        self.ctx.call("ske_swipes_fixed_async", fid, C.c_void_p(b.slot.ptr),
                      C.c_void_p(b.bytes.ptr), b.width, b.n, C.c_void_p(out.ptr) if out else None)

    @staticmethod
    def many_args(batches, outs=None, fixed: bool = False):
        """The ske_swipe_batch array of a many-batch call, built once: a
        caller that replays the same batches (a serving loop over resident
        buffers, the benchmark) passes it as `prepared` and skips the
        per-call Python marshalling."""
        outs = outs if outs is not None else [None] * len(batches)
        arr = (SweBatch * len(batches))()
        for a, b, o in zip(arr, batches, outs):
            a.slot, a.bytes = b.slot.ptr, b.bytes.ptr
            a.offs = None if fixed else b.offs.ptr
            a.width = b.width if fixed else 0
            a.n = b.n
            a.out_valid = o.ptr if o is not None else None
        return arr

    def swipes_many_async(self, fid: int, batches, outs=None, branches: int = 0,
                          fixed: bool = False, prepared=None):
        """Enqueue K1 over several resident batches in one native call
        (ske_swipes_many_async): batch j on branch j mod `branches` (0: 16),
        forked from and joined back into the context stream; with several
        branches two launches share the chip, half the CUs each.  `fixed`:
        read the ids as fixed-width (as swipes_fixed_async).  `prepared`: the
        many_args() array of these batches."""
        arr = prepared if prepared is not None else self.many_args(batches, outs, fixed)
        self.ctx.call("ske_swipes_many_async", fid, C.cast(arr, C.c_void_p), len(arr), branches)

    def swipes_stats(self, fid: int, b: DeviceBatch) -> tuple[int, int]:
        probes, nvalid = C.c_uint64(), C.c_uint64()
        self.ctx.call("ske_swipes_stats", fid, C.c_void_p(b.bytes.ptr), C.c_void_p(b.offs.ptr),
                      b.n, C.byref(probes), C.byref(nvalid))
        return probes.value, nvalid.value

    def variant(self, fid: int) -> int:
        return self.ctx.lib.ske_swipes_variant(self.ctx.ptr, fid)

    def set_option(self, name: str, value: int):
        self.ctx.call("ske_set_option", name.encode(), int(value))

    def pass_times(self, reset: bool = True) -> list[tuple[float, int]]:
        """(summed ms, kernel count) per K1 pass kind, from the HIP event
        pairs the library records around each kernel while the option
        "pass_timing" is on: [single-kernel K1, partitioned A, B, C (or the
        segmented C1), segmented level-2 sort, segmented window apply, and a
        host-fed call's H2D copies, D2H copies, whole call]."""
        ms = (C.c_double * PASS_KINDS)()
        cnt = (C.c_uint64 * PASS_KINDS)()
        self.ctx.call("ske_pass_times", ms, cnt, 1 if reset else 0)
        return [(ms[i], cnt[i]) for i in range(PASS_KINDS)]

    def set_stream(self, stream_ptr: int | None):
        self.ctx.call("ske_set_stream", C.c_void_p(stream_ptr) if stream_ptr else None)

    def get_stream(self) -> int | None:
        """The stream calls enqueue on now (None: the context's own stream)."""
        p = C.c_void_p()
        self.ctx.call("ske_get_stream", C.byref(p))
        return p.value

    def sync(self):
        """Wait for the context stream; raises SKE_ERANGE (SketchLibError)
        when an enqueued K1 met a valid swipe whose slot is outside the slab."""
        self.ctx.call("ske_sync")

    def check_errors(self):
        self.ctx.call("ske_check_errors")

    # ---- HIP graphs: record enqueue-only calls once, replay many times
    def capture(self, fn) -> "Graph":
        """Record the device work `fn()` enqueues on the context stream (only
        *_async calls) into an uploaded executable graph.

        Python's cyclic garbage collector is run before and held off during
        the recording: a collection inside it could finalise an unreachable
        Context or device buffer (ske_close / hipFree / hipStreamSynchronize),
        which a thread-local stream capture forbids -- the capture would be
        invalidated and this recording fail."""
        with _no_gc():
            self.ctx.call("ske_capture_begin")
            try:
                fn()
            except BaseException:
                # end the capture (the stream must leave capture mode) and drop
                # the partial graph; the recording call's error is the one raised
                g = C.c_void_p()
                if self.ctx.lib.ske_capture_end(self.ctx.ptr, C.byref(g)) == 0 and g.value:
                    self.ctx.lib.ske_graph_free(self.ctx.ptr, g)
                raise
            g = C.c_void_p()
            self.ctx.call("ske_capture_end", C.byref(g))
        return Graph(self.ctx, g.value)

    def capture_branched(self, steps, main, side) -> "Graph":
        """Record `steps` (callables, each enqueuing one *_async call) into one
        graph of 1 + len(side) independent branches: step j on branch
        j mod (1 + len(side)), forked from and joined back into `main` (torch
        streams).  On replay, launches of different branches overlap; with the
        "k1_grid" option at half the CUs two K1 launches share the chip.  The
        context stream is `main` afterwards."""
        import torch
        streams = [main] + list(side)
        fork = torch.cuda.Event()
        joins = [torch.cuda.Event() for _ in side]

        def record():
            fork.record(main)
            for s_ in side:
                s_.wait_event(fork)
            for j, fn in enumerate(steps):
                self.set_stream(streams[j % len(streams)].cuda_stream)
                fn()
            for s_, ev in zip(side, joins):
                ev.record(s_)
                main.wait_event(ev)
            self.set_stream(main.cuda_stream)

        self.set_stream(main.cuda_stream)
        return self.capture(record)

    # ---- HLL reads
    def registers(self, slot: int) -> np.ndarray:
        out = np.zeros(16384, np.uint8)
        self.ctx.call("ske_hll_export_raw", int(slot), out.ctypes.data_as(C.c_void_p))
        return out

    def registers_all(self, nslots: int) -> np.ndarray:
        p, nb = C.c_void_p(), C.c_uint64()
        self.ctx.call("ske_hll_slab", C.byref(p), C.byref(nb))
        out = np.zeros((nslots, 16384), np.uint8)
        assert nslots * 16384 <= nb.value
        self.ctx.call("ske_memcpy", out.ctypes.data_as(C.c_void_p), p, out.nbytes, 1)
        return out

    def pfcount_each(self, slots) -> np.ndarray:
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        out = np.zeros(s.size, np.uint64)
        if s.size:
            self.ctx.call("ske_hll_pfcount_each", s.ctypes.data_as(C.c_void_p), s.size,
                          out.ctypes.data_as(C.c_void_p), 0)
        return out

    def bloom_bits(self, fid: int, link: int, nbytes: int) -> np.ndarray:
        out = np.zeros(nbytes, np.uint8)
        self.ctx.call("ske_bf_export_link", fid, link, out.ctypes.data_as(C.c_void_p), nbytes)
        return out
