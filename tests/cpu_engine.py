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


def factory(comm):
    return OracleEngine(comm)
