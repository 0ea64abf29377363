"""``HipEngine``: one GPU's share of the Lloyd iteration, driven through the
C-ABI of ``include/kmeans_amd.h``.

The engine owns one ``km_ctx`` (rows resident in HBM, centroids, statistics
buffer, stream).  ``kmeans.LloydRunner`` drives it with the same sequence of
calls as the reference's ``fit`` loop (kmeans_spark.py:266-318).  When the
process is one rank of a multi-GPU job the statistics buffer is a torch
tensor bound into the context and the context enqueues on a dedicated torch
stream, so the RCCL all-reduce is stream-ordered between ``assign_stats`` and
``update`` without host synchronisation.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib

_PD = ctypes.POINTER(ctypes.c_double)
_PF = ctypes.POINTER(ctypes.c_float)
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI64 = ctypes.POINTER(ctypes.c_int64)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class HipEngine:
    """A GPU context holding this rank's rows (no CPU fallback: raises if the
    HIP extension or a gfx950 device is unavailable)."""

    def __init__(self, device: int = 0, distributed: bool = False):
        self.lib = _lib.load()
        n = _lib.device_count()
        if n <= 0:
            raise _lib.KmError("no HIP device visible: the MI355X path needs a gfx950 GPU")
        self.device = device
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.km_create(device, ctypes.byref(ctx)), "km_create")
        self.ctx = ctx
        self.n = 0
        self.d = 0
        self.k = 0
        self._stats_t = None
        self._tstream = None
        self._coll_ev = None        # [(start, end)] HIP events around each collective while timed
        self.distributed = distributed
        if distributed:
            import torch
            self._torch = torch
            self._tstream = torch.cuda.Stream(device=f"cuda:{device}")
            _lib.check(self.lib.km_set_stream(self.ctx, ctypes.c_void_p(self._tstream.cuda_stream)), "km_set_stream")

    # -- lifetime --------------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            self.lib.km_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc, what):
        return _lib.check(rc, what)

    # -- data ------------------------------------------------------------------
    def load_host(self, rows: np.ndarray) -> int:
        """Copy this rank's rows (float32 [n][d]) into HBM once (rdd.cache(), L256)."""
        rows = np.ascontiguousarray(rows, dtype=np.float32)
        if rows.ndim != 2:
            raise ValueError("rows must be a 2-D array")
        n, d = rows.shape
        self._c(self.lib.km_load_begin(self.ctx, n, d), "km_load_begin")
        if n:
            self._c(self.lib.km_load_rows(self.ctx, 0, _ptr(rows, _PF), n), "km_load_rows")
        self.n, self.d = n, d
        return n

    def load_blobs(self, n: int, d: int, global_row0: int, n_centers: int, box: float = 10.0, std: float = 1.0,
                   seed: int = 0) -> int:
        self._c(self.lib.km_generate_blobs(self.ctx, n, d, global_row0, n_centers, box, std, seed),
                "km_generate_blobs")
        self.n, self.d = n, d
        return n

    def sum_x(self) -> np.ndarray:
        out = np.zeros(self.d, dtype=np.float64)
        self._c(self.lib.km_sum_x(self.ctx, _ptr(out, _PD)), "km_sum_x")
        return out

    def set_sse(self, enable: bool) -> None:
        """compute_sse: residuals of every row summed into the stats buffer's
        SSE slot during assign_stats (kmeans_spark.py:278-286)."""
        self._c(self.lib.km_set_sse(self.ctx, 1 if enable else 0), "km_set_sse")

    def set_screen(self, mode: int) -> None:
        """Screening kernel of the fused path (-1 auto; 0 fp16x3; 1 fp16x3 +
        per-key bounds; 2 / 3 the fast fp16 screen, diagnostic library only;
        4 k_s1, one fp16 MFMA per product with in-kernel fp32 re-scoring and
        delta statistics, where the geometry has it).  A cost choice only:
        results are exact in every mode (tests pin each one)."""
        self._c(self.lib.km_set_screen(self.ctx, int(mode)), "km_set_screen")

    def screen(self) -> int:
        """The screen the next fused launch uses (0..4)."""
        m = ctypes.c_int32()
        self._c(self.lib.km_get_screen(self.ctx, ctypes.byref(m)), "km_get_screen")
        return m.value

    # -- centroids / iteration -------------------------------------------------
    def set_centroids(self, C: np.ndarray) -> None:
        C = np.ascontiguousarray(C, dtype=np.float64)
        k, d = C.shape
        self._c(self.lib.km_set_centroids(self.ctx, _ptr(C, _PD), k, d), "km_set_centroids")
        if self.distributed and (self._stats_t is None or k != self.k):
            torch = self._torch
            self._stats_t = torch.zeros(k * (d + 1) + 1, dtype=torch.float64, device=f"cuda:{self.device}")
            torch.cuda.synchronize(self.device)
            self._c(self.lib.km_bind_stats_buffer(self.ctx, ctypes.c_void_p(self._stats_t.data_ptr())),
                    "km_bind_stats_buffer")
        self.k = k

    def get_centroids(self, which: int = 0) -> np.ndarray:
        out = np.empty((self.k, self.d), dtype=np.float64)
        self._c(self.lib.km_get_centroids(self.ctx, which, _ptr(out, _PD)), "km_get_centroids")
        return out

    def assign_stats(self) -> None:
        self._c(self.lib.km_assign_stats(self.ctx), "km_assign_stats")

    def run_collective(self, fn, tensor=None) -> None:
        """Run ``fn(stats_tensor, async_op=True)`` (an in-place all-reduce)
        ordered on this context's HIP stream, with no host synchronisation.

        Ordering (torch ProcessGroupNCCL = RCCL here): the collective runs on
        the process group's own stream, which first waits on the CURRENT
        stream -- made ``self._tstream``, the wrapper of the engine's stream,
        so the all-reduce reads the statistics only after km_assign_stats
        wrote them; ``work.wait()`` then "lets the current stream wait for the
        NCCL to finish" (torch/include/torch/csrc/distributed/c10d/
        ProcessGroupNCCL.hpp:289-317 and WorkNCCL::wait/synchronize,
        :355-371: a stream-level wait, not a host block), so km_update /
        km_update_async enqueued next on the engine stream read the summed
        buffer.  gloo (CPU tensors) completes inside wait()."""
        with self._torch.cuda.stream(self._tstream):
            if self._coll_ev is not None:
                e0 = self._torch.cuda.Event(enable_timing=True)
                e1 = self._torch.cuda.Event(enable_timing=True)
                e0.record(self._tstream)
            work = fn(self._stats_t if tensor is None else tensor, async_op=True)
            if work is not None:
                work.wait()
            if self._coll_ev is not None:
                e1.record(self._tstream)
                self._coll_ev.append((e0, e1))

    def time_collectives(self, enable: bool) -> None:
        """Record HIP events on the engine stream around each collective
        (from the statistics being ready to the summed buffer being usable by
        the next kernel); read with ``collective_ms``."""
        self._coll_ev = [] if enable else None

    def collective_ms(self) -> Tuple[float, int]:
        """(total ms, collectives) recorded since ``time_collectives(True)``."""
        evs = self._coll_ev or []
        if evs:
            self._torch.cuda.synchronize(self.device)
        return sum(a.elapsed_time(b) for a, b in evs), len(evs)

    def update(self) -> Tuple[_lib.KmStatus, np.ndarray]:
        st = _lib.KmStatus()
        counts = np.zeros(self.k, dtype=np.int64)
        self._c(self.lib.km_update(self.ctx, ctypes.byref(st), _ptr(counts, _PI64)), "km_update")
        return st, counts

    # -- batches of iterations with one host sync (km_batch_*) -------------------
    def batch_begin(self) -> None:
        self._c(self.lib.km_batch_begin(self.ctx), "km_batch_begin")

    def update_async(self, tol: float, empty_seed: int = 0) -> None:
        self._c(self.lib.km_update_async(self.ctx, float(tol), int(empty_seed)), "km_update_async")

    def set_layout(self, sizes, row0: int, device_repair: int) -> None:
        """The dataset's takeSample partition layout; device_repair moves the
        empty-cluster repair onto the GPU: 1 = one rank holding every row,
        2 = rows spread over ranks (the caller all-reduces the repair rows,
        ``repair_exchange``)."""
        sizes = np.ascontiguousarray(sizes, dtype=np.int64)
        self._c(self.lib.km_set_layout(self.ctx, _ptr(sizes, _PI64), len(sizes), int(row0), int(device_repair)),
                "km_set_layout")
        self._rep_mode = int(device_repair)
        self._rep_t = None

    def repair_state(self) -> Tuple[bool, bool]:
        """(armed, waiting): the next km_update_async may enqueue a device
        repair / the last one left its iteration to repair_apply_async."""
        a, w = ctypes.c_int32(), ctypes.c_int32()
        self._c(self.lib.km_repair_state(self.ctx, ctypes.byref(a), ctypes.byref(w)), "km_repair_state")
        return bool(a.value), bool(w.value)

    def repair_bind(self) -> None:
        """Layout mode 2: a torch tensor as the repair-row buffer (the one the
        process group all-reduces); call before enqueueing the iterations."""
        if self._rep_t is None or self._rep_t.numel() != self.k * self.d:
            torch = self._torch
            self._rep_t = torch.zeros(self.k * self.d, dtype=torch.float64, device=f"cuda:{self.device}")
            torch.cuda.synchronize(self.device)
            self._c(self.lib.km_bind_repair_buffer(self.ctx, ctypes.c_void_p(self._rep_t.data_ptr())),
                    "km_bind_repair_buffer")

    def repair_exchange(self, allreduce) -> None:
        """Layout mode 2: sum the ranks' picked replacement rows (each holds
        its own, zeros elsewhere) on this context's stream, then finish the
        iteration on the device (km_repair_apply_async)."""
        self.run_collective(allreduce, self._rep_t)
        self._c(self.lib.km_repair_apply_async(self.ctx), "km_repair_apply_async")

    def batch_end(self, m: int):
        """Sync once; [(status, counts)] of the iterations of the batch that ran
        (the rest were no-ops after the device stopped it)."""
        st = (_lib.KmStatus * max(m, 1))()
        counts = np.zeros((max(m, 1), self.k), dtype=np.int64)
        n = ctypes.c_int32(0)
        self._c(self.lib.km_batch_end(self.ctx, st, _ptr(counts, _PI64), ctypes.byref(n)), "km_batch_end")
        return [(st[i], counts[i]) for i in range(n.value)]

    def replace_rows(self, ids, rows: np.ndarray) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        rows = np.ascontiguousarray(rows, dtype=np.float64).reshape(len(ids), self.d)
        if len(ids):
            self._c(self.lib.km_replace_rows(self.ctx, _ptr(ids, _PI32), _ptr(rows, _PD), len(ids)),
                    "km_replace_rows")

    def commit(self) -> None:
        self._c(self.lib.km_commit(self.ctx), "km_commit")

    def gather_rows(self, local_idx) -> np.ndarray:
        idx = np.ascontiguousarray(local_idx, dtype=np.int64)
        out = np.empty((len(idx), self.d), dtype=np.float64)
        if len(idx):
            self._c(self.lib.km_gather_rows(self.ctx, _ptr(idx, _PI64), len(idx), _ptr(out, _PD)),
                    "km_gather_rows")
        return out

    def bernoulli(self, seeds, sizes, bases, fraction: float) -> Optional[np.ndarray]:
        """takeSample's Bernoulli pass on this GPU (km_bernoulli_sample): the
        picks (global row indices, partitions in the given order), or None when
        the device pass cannot hold them (the caller samples on the host)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        sizes = np.ascontiguousarray(sizes, dtype=np.int64)
        bases = np.ascontiguousarray(bases, dtype=np.int64)
        cap = int(4.0 * fraction * float(sizes.sum())) + 64 * max(len(sizes), 1)
        out = np.empty(cap, dtype=np.int64)
        n = ctypes.c_int64(0)
        rc = self.lib.km_bernoulli_sample(self.ctx, seeds.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                          _ptr(sizes, _PI64), _ptr(bases, _PI64), len(sizes), float(fraction),
                                          _ptr(out, _PI64), cap, ctypes.byref(n))
        if rc == -1:  # KM_ERR_ARG: more picks than the device pass holds
            return None
        self._c(rc, "km_bernoulli_sample")
        return out[:n.value].copy()

    def predict(self) -> np.ndarray:
        out = np.empty(self.n, dtype=np.int32)
        self._c(self.lib.km_predict(self.ctx, _ptr(out, _PI32)), "km_predict")
        return out

    def predict_device(self) -> None:
        """km_predict with the labels left in HBM (no host copy)."""
        self._c(self.lib.km_predict(self.ctx, None), "km_predict")

    def labels(self) -> np.ndarray:
        out = np.empty(self.n, dtype=np.int32)
        self._c(self.lib.km_labels(self.ctx, _ptr(out, _PI32)), "km_labels")
        return out

    def sync(self) -> None:
        self._c(self.lib.km_sync(self.ctx), "km_sync")

    def info(self) -> dict:
        inf = _lib.KmInfo()
        self._c(self.lib.km_info_get(self.ctx, ctypes.byref(inf)), "km_info_get")
        return {f: getattr(inf, f) for f, _ in inf._fields_}

    # -- profiling ---------------------------------------------------------------
    _PHASES = {"assign": 0, "resolve": 1, "stats": 2, "update": 3, "prep": 4}   # KM_K_* (kmeans_amd.h)

    def profile(self, enable: bool = True, phases=None, every: int = 1) -> None:
        """Time launches with HIP events: every phase, or only ``phases``
        (names of ``_PHASES``), one launch in ``every`` of each.  Each timed
        launch costs a few microseconds of stream time, so a timed region
        records only the phases it reports."""
        mask = 0
        if enable:
            mask = -1 if phases is None else sum(1 << self._PHASES[p] for p in phases)
        self._c(self.lib.km_profile_every(self.ctx, int(every)), "km_profile_every")
        self._c(self.lib.km_profile(self.ctx, mask), "km_profile")

    def prof_read(self, kind: str) -> Tuple[float, int]:
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        self._c(self.lib.km_prof_read(self.ctx, _lib.KERNEL_KINDS[kind], ctypes.byref(ms), ctypes.byref(n)),
                "km_prof_read")
        return ms.value, n.value


def make_engine(comm, device: Optional[int] = None) -> HipEngine:
    """One engine per rank on GPU ``LOCAL_RANK`` (taken modulo the visible
    devices, so several ranks can share one GPU when rehearsing)."""
    if device is None:
        n = _lib.device_count()
        dev = comm.local_rank % n if n > 0 else comm.local_rank
    else:
        dev = device
    return HipEngine(dev, distributed=comm.world > 1)
