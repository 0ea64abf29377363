"""TEST-ONLY engine: the HipEngine interface computed on the CPU by the oracle.

Used by the ``-m "not gpu"`` tests to exercise the product's host logic
(KMeans driver, data placement, takeSample policy, empty-cluster repair,
logging, the multi-rank all-reduce path over ``gloo``) without a GPU.  It is
injected through ``KMeans._engine_factory``; the product never imports it.
Arithmetic mirrors the device path: float32 rows, float64 statistics, the
SSE as the sum of every row's float64 residual to its pre-update centroid
(an extra slot of the all-reduced statistics buffer).
"""
import numpy as np

from oracle import kmeans_oracle as orc


class _Status:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class OracleEngine:
    def __init__(self, comm):
        self.distributed = comm.world > 1
        self.n = self.d = self.k = 0
        self.sse = False
        self._stats_t = None

    # data -------------------------------------------------------------------
    def load_host(self, rows):
        self.X = np.asarray(rows, dtype=np.float32).astype(np.float64)
        self.n, self.d = self.X.shape if self.X.ndim == 2 else (0, 0)
        return self.n

    def sum_x(self):
        return self.X.sum(axis=0) if self.n else np.zeros(self.d)

    def set_sse(self, enable):
        self.sse = bool(enable)

    # iteration --------------------------------------------------------------------
    def set_centroids(self, C):
        self.cur = np.array(C, dtype=np.float64)
        self.k = len(self.cur)
        self.new = self.cur.copy()

    def get_centroids(self, which=0):
        return (self.new if which else self.cur).copy()

    # batches (mirror of km_batch_begin / km_update_async / km_batch_end) --------------
    def batch_begin(self):
        self._batching, self._stopped, self._slots = True, False, []

    def update_async(self, tol, empty_seed=0):
        if self._stopped:
            return
        st, counts = self.update()
        stop = 3 if st.nonfinite else (2 if st.n_empty else (1 if st.max_shift < tol else 0))
        st.stop_reason = stop
        self._slots.append((self.cur.copy(), self.new.copy(), st, counts))
        self._stopped = bool(stop)
        self.cur = self.new.copy()                      # speculative commit

    def batch_end(self, m):
        if self._slots:                                 # state after the last iteration that ran
            self.cur, self.new = self._slots[-1][0].copy(), self._slots[-1][1].copy()
        self._batching = self._stopped = False
        return [(st, counts) for _, _, st, counts in self._slots]

    def assign_stats(self):
        if getattr(self, "_stopped", False):            # a stopped batch: no-op
            return
        import torch
        S = np.zeros(self.k * (self.d + 1) + 1)
        T = S[:-1].reshape(self.k, self.d + 1)
        if self.n:
            self._labels = orc.assign(self.X, self.cur)[0]
            np.add.at(T[:, :self.d], self._labels, self.X)
            np.add.at(T[:, self.d], self._labels, 1.0)
            if self.sse:
                S[-1] = float(((self.X - self.cur[self._labels]) ** 2).sum())
        else:
            self._labels = np.zeros(0, dtype=np.int64)
        self._stats_t = torch.from_numpy(S)

    def run_collective(self, fn):
        fn(self._stats_t)

    def update(self):
        flat = self._stats_t.numpy()
        S = flat[:-1].reshape(self.k, self.d + 1)
        cnt = S[:, self.d]
        old = self.cur
        new = np.where(cnt[:, None] > 0, S[:, :self.d] / np.where(cnt > 0, cnt, 1)[:, None], old)
        self.new = new
        shift = np.sqrt(((new - old) ** 2).sum(axis=1))
        st = _Status(sse=float(flat[-1]), max_shift=float(shift.max()), n_empty=int((cnt == 0).sum()),
                     nonfinite=int(not np.all(np.isfinite(new))), q_rerank=0, q_full=0, ran=1,
                     stop_reason=0)
        return st, cnt.astype(np.int64)

    def replace_rows(self, ids, rows):
        self.new[np.asarray(ids)] = np.asarray(rows).reshape(len(ids), self.d)

    def commit(self):
        self.cur = self.new.copy()

    def gather_rows(self, idx):
        return self.X[np.asarray(idx, dtype=np.int64)]

    def predict(self):
        return orc.assign(self.X, self.cur)[0].astype(np.int32) if self.n else np.zeros(0, np.int32)

    def labels(self):
        return self._labels.astype(np.int32)

    def info(self):
        return {"n": self.n, "d": self.d, "k": self.k, "path": 0}


class DeviceRepairEngine(OracleEngine):
    """The OracleEngine with the device's empty-cluster repair protocol
    (km_set_layout / km_repair_state / km_repair_buffer /
    km_repair_apply_async): in a batch that is "armed" the update repairs
    empties itself by the takeSample policy (kmeans_spark.py:191-204) instead
    of stopping the batch; with rows spread over ranks (mode 2) every rank
    picks the same global rows, writes the ones it holds into the repair
    buffer (zeros elsewhere), the caller all-reduces that buffer
    (repair_exchange) and the apply step finishes the iteration.  Arming as on
    the device: armed after new centroids, disarmed by a batch without
    empties."""

    def set_layout(self, sizes, row0, mode):
        self.layout, self.row0, self.rep_mode = [int(v) for v in sizes], int(row0), int(mode)
        self.armed, self.waiting, self._rep_t, self._pending = bool(mode), False, None, None

    def set_centroids(self, C):
        super().set_centroids(C)
        self.armed = bool(getattr(self, "rep_mode", 0))

    def replace_rows(self, ids, rows):
        super().replace_rows(ids, rows)
        self.armed = bool(self.rep_mode)

    def repair_bind(self):
        import torch
        if self._rep_t is None or self._rep_t.numel() != self.k * self.d:
            self._rep_t = torch.zeros(self.k * self.d, dtype=torch.float64)

    def repair_state(self):
        return bool(self.rep_mode) and self.armed, self.waiting

    def update_async(self, tol, empty_seed=0):
        if self._stopped:
            return
        st, counts = self.update()
        st.repaired = 0
        repair = bool(self.rep_mode) and self.armed
        if repair and st.n_empty and not st.nonfinite and st.n_empty < sum(self.layout):
            empty = [j for j in range(self.k) if counts[j] == 0]
            gidx = orc.take_sample_indices(self.layout, len(empty), int(empty_seed))
            buf = np.zeros(self.k * self.d)
            for i, g in enumerate(gidx):
                if self.row0 <= g < self.row0 + self.n:
                    buf[i * self.d:(i + 1) * self.d] = self.X[g - self.row0]
            self._pending = (st, counts, empty, len(gidx), tol)
            if self.rep_mode == 2:
                self.repair_bind()
                self._rep_t.copy_(__import__("torch").from_numpy(buf))
                self.waiting = True
                return
            self._apply(buf)
            return
        stop = 3 if st.nonfinite else (2 if st.n_empty else (1 if st.max_shift < tol else 0))
        self._finish(st, counts, stop)

    def repair_exchange(self, allreduce):
        allreduce(self._rep_t)
        self.waiting = False
        self._apply(self._rep_t.numpy())

    def _apply(self, buf):
        st, counts, empty, num, tol = self._pending
        rows = np.asarray(buf).reshape(self.k, self.d)[:num]
        old = self.cur
        for i in range(num):
            self.new[empty[i]] = rows[i]
        shift = np.sqrt(((self.new - old) ** 2).sum(axis=1))
        st.max_shift = float(shift.max())
        st.nonfinite = int(not np.all(np.isfinite(self.new)))
        st.repaired = 1
        self._finish(st, counts, 3 if st.nonfinite else (1 if st.max_shift < tol else 0))

    def _finish(self, st, counts, stop):
        st.stop_reason = stop
        self._slots.append((self.cur.copy(), self.new.copy(), st, counts))
        self._stopped = bool(stop)
        self.cur = self.new.copy()                      # speculative commit

    def batch_end(self, m):
        out = super().batch_end(m)
        if getattr(self, "rep_mode", 0):
            self.armed = any(st.n_empty for st, _ in out)
        return out


def factory(comm):
    return OracleEngine(comm)


def factory_device_repair(comm):
    return DeviceRepairEngine(comm)
