"""Benchmark of the Lloyd-iteration hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

A "step" is one Lloyd iteration of ``KMeans.fit`` (assign -> partial stats ->
RCCL all-reduce -> update -> commit, kmeans_spark.py:266-318) over the
workload's rows, which were generated in HBM before timing; steps are
enqueued in batches with one host synchronisation per batch, as ``fit`` runs
them (``LloydRunner.run``).  Default workload
= the metric's configuration, N=100M rows, d=64, k=256 (fits one MI355X: 25.6
GB); the N rows are split over the ranks (strong scaling).  Rank 0 prints one
JSON line with ``roofline`` (dominant kernel, HIP-event timed on its stream)
and ``cpu_baseline`` (the oracle's per-point restatement of the reference
closures, timed on this host on a bounded sample, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Lloyd iters/sec + points/sec, N=100M d=64 k=256, 1–8 GPUs; % of roofline"
CONFIGS = {
    # name: (N_total, d, k, n_centers)
    "c3": (100_000_000, 64, 256, 256),
    "c2": (10_000_000, 16, 8, 8),
    "c4": (1_000_000_000, 32, 1024, 1024),
    "c5": (50_000_000, 128, 4096, 4096),
    "c3_small": (4_000_000, 64, 256, 256),
    "c3_shard8": (12_500_000, 64, 256, 256),   # one GPU's share of c3 at 8 GPUs (overhead check)
    # c5 with poor seeds (BASELINE.json configs[4]): 3 data rows + 4093 far
    # points, so the first step replaces 4093 empty clusters (on the device)
    "c5_poor": (50_000_000, 128, 4096, 4096),
    # rows wider than 256 features (k_assign_wide; not a BASELINE config)
    "w784": (4_000_000, 784, 256, 256),
}
POOR_SEEDS = {"c5_poor"}
SSE_CONFIGS = {"c4"}  # BASELINE.json configs[3]: "... compute_sse=True"
HBM_PEAK_GBS = 8000.0                 # MI355X spec (MI355X_MICROARCH.md)
F16_DENSE_TFLOPS = 2516.6             # dense f16/bf16 MFMA peak (MI355X_MICROARCH.md)
F16X3_EFFECTIVE_TFLOPS = F16_DENSE_TFLOPS / 3.0  # fp16x3 split: 3 MFMAs per product


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--screen", type=int, default=-1, choices=[-1, 0, 1, 2, 3, 4, 5],
                   help="fused-path screen (km_set_screen): -1 the runtime's choice (4 = k_s1 where the "
                        "geometry has it), 0/1 fp16x3 k_fused16 with full statistics every iteration "
                        "(2, 3: diagnostic library only)")
    p.add_argument("--sse", type=int, default=None, choices=[0, 1],
                   help="compute_sse (kmeans_spark.py:38); default: on for c4, whose BASELINE config "
                        "(configs[3]) states compute_sse=True, off elsewhere (the reference default)")
    p.add_argument("--predict", type=int, default=0, metavar="P",
                   help="after the fit steps, time P predict passes (km_predict, labels left in HBM; "
                        "kmeans_spark.py:321-352) and add a 'predict' object to the line")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work per worker")
    p.add_argument("--no-first-iter", action="store_true", help="skip the first-iterations timing (first_iter)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="per-launch HBM bytes from a rocprofv3 --pmc pass (optional)")
    return p.parse_args()


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        dev = local % max(torch.cuda.device_count(), 1)   # == local on a full node
        torch.cuda.set_device(dev)
        backend = os.environ.get("KM_DIST_BACKEND", "nccl")  # nccl == RCCL; gloo only to rehearse on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def usable_cpus():
    """os.cpu_count(), capped by this process's CPU
    affinity and cgroup quota: on the GPU box os.cpu_count() reports the whole
    host while a job gets a share of it."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(d, k, n_total, seconds):
    """The reference closure restated (oracle, per-point np.linalg.norm +
    argmin + reduceByKey combine; kmeans_spark.py:147-173) on a bounded
    sample, one process per usable CPU, like Spark local[*].  Cross-checked
    against the reference's own closures by scripts/check_cpu_baseline.py
    (within 10 %, profiles/r2_cpu_baseline_check.txt)."""
    from multiprocessing import get_context
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_baseline as cb
    workers = usable_cpus()
    # calibrate points per worker for ~`seconds` of work
    rate = cb.calibrate(d, k)
    per = int(max(2000, min(400_000, rate * seconds)))
    with get_context("spawn").Pool(workers) as pool:
        # the workers generate their partitions, then start their passes
        # together; the rate is timed over the passes only (first start to
        # last end on the shared monotonic clock), not over process spawn,
        # imports or data generation
        # (spawn + numpy import + a partition of <= 400k rows: a few seconds;
        # a late worker starts at once and its lag counts against the rate)
        start_at = time.monotonic() + 6.0 + per * d * 2e-8
        res = pool.starmap(cb.run_partition, [(d, k, per, w, start_at) for w in range(workers)])
    dt = max(r[2] for r in res) - min(r[1] for r in res)
    pts = sum(r[0] for r in res)
    pps = pts / dt
    return {"value": pps / n_total, "unit": f"Lloyd it/s (extrapolated to N={n_total:,})", "cores": workers,
            "kind": "port", "points_per_sec": pps, "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"{workers} workers x {per} points, d={d}, k={k}, one assign+combine pass each "
                      f"(oracle/cpu_baseline.py restating kmeans_spark.py:147-173), passes started together and "
                      f"timed first start to last end (no spawn/import/data generation); it/s = points/s / N"}


def main():
    args = parse()
    world, rank, local = init_dist(args)
    import kmeans_amd
    from kmeans_amd.comm import Communicator

    N, d, k, centers = CONFIGS[args.config]
    sse = bool(args.sse) if args.sse is not None else args.config in SSE_CONFIGS
    comm = Communicator()
    km = kmeans_amd.KMeans(k=k, max_iter=10 ** 9, tolerance=1e-300, seed=42, compute_sse=sse)
    km.verbose = False
    data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=centers, box=10.0, std=1.0, seed=2024)
    run = km._make_runner(data, comm)
    C0 = km._initialize_centroids(run)          # takeSample policy (L72), outside the timed region
    if args.config in POOR_SEEDS:
        C0 = np.vstack([C0[:3], np.full((k - 3, d), 100.0) + np.arange(k - 3)[:, None]])
    eng = run.engine
    eng.set_screen(args.screen)
    eng.set_sse(sse)
    eng.set_centroids(C0)
    km.sse_history = []

    log = None  # silent run: the loop skips formatting its log lines (kmeans.LloydRunner.iteration)

    import torch
    # iterations run in batches with one host sync each (LloydRunner.run: the
    # device records every iteration and would stop a batch on convergence,
    # empty clusters or NaN; tolerance 1e-300 never converges)
    run.run(km, log, args.warmup)
    eng.sync()
    comm.barrier()
    torch.cuda.synchronize()
    # events only around the dominant kernel inside the timed region (each
    # record costs a few us of stream time); the other phases' durations come
    # from two untimed steps after it
    # (one launch in 4 on the sub-millisecond steps of c1/c2, where each timed
    # launch's ~6 us of stream time would be 4% of the step)
    eng.profile(True, phases=("assign", "stats"), every=4 if args.config in ("c1", "c2") else 1)
    ran0 = run.iterations_ran
    if world > 1:
        run.host_ms = {}   # host wall time per call kind (LloydRunner.run): where a multi-rank step goes
    t0 = time.perf_counter()
    run.run(km, log, args.warmup + args.steps, first=args.warmup)
    eng.sync()
    torch.cuda.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    host_ms, run.host_ms = run.host_ms, None
    # iterations the device actually ran in the timed region: a batch stops
    # early only on convergence (max_shift < 1e-300, i.e. an exact fixed
    # point), empties or NaN; the rate counts what ran, never args.steps
    ran = run.iterations_ran - ran0
    eng.profile(True, phases=("resolve", "update", "prep"), every=1)
    if world > 1:
        eng.time_collectives(True)   # HIP events around each all-reduce, engine stream
    run.run(km, log, args.warmup + args.steps + 2, first=args.warmup + args.steps)
    eng.sync()
    eng.profile(False)
    coll = eng.collective_ms() if world > 1 else None
    eng.time_collectives(False)
    dt = float(comm.allreduce_np(np.array([t1 - t0])).max()) if world == 1 else None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([t1 - t0], dtype=torch.float64,
                         device=f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    kern = {name: eng.prof_read(name) for name in ("assign", "resolve", "stats", "update", "prep")}
    info = eng.info()
    screen = eng.screen() if info["path"] == 2 else None
    n_local = info["n"]
    flops_launch = 2.0 * n_local * k * d                 # algorithmic distance contraction
    bytes_stats = n_local * (d * 4 + 4)                  # X once + labels
    bytes_assign = n_local * (d * 4 + 4)
    dom = max(("assign", "stats"), key=lambda kk: kern[kk][0])
    ms_dom, launches = kern[dom]
    avg_s = (ms_dom / max(launches, 1)) / 1e3
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            te = tj.get(args.config) if "config" not in tj else (tj if tj["config"] == args.config else None)
            if te is not None and te.get("kernel", "assign") == dom:
                # measured on one GPU holding all N rows; a rank's launch covers n_local
                traffic = te.get("bytes_per_launch") * n_local / N
        except Exception:
            traffic = None
    if info["path"] == 2 and dom == "assign" and screen in (2, 3):
        # fast screen: NX fp16 MFMAs per product (2516.6 TF dense) -- at c3 the
        # MFMA time is 1.3 ms (NX = 1) against 3.2 ms of HBM, so HBM bounds it
        nx = 1 if screen == 2 else 2
        t_mfma = flops_launch * nx / (F16_DENSE_TFLOPS * 1e12)
        bytes_fast = n_local * (d * 4 + 8)               # X once + row norm + label
        t_hbm = bytes_fast / (HBM_PEAK_GBS * 1e9)
        kname = f"k_fused1 (fast fp16 screen, {nx} row part{'s' if nx > 1 else ''}, pairwise bound + f64 sums)"
        if t_hbm >= t_mfma:
            ach = bytes_fast / avg_s / 1e9
            roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                    "traffic": traffic, "kernel": kname,
                    "bytes_note": "N*(d*4+8) per launch (rows once + row norm + label); the MFMA time at "
                                  f"{nx} fp16 MFMA(s) per product is {t_mfma * 1e3:.2f} ms vs {t_hbm * 1e3:.2f} ms HBM",
                    "tflops": flops_launch / avg_s / 1e12}
        else:
            ach = flops_launch * nx / avg_s / 1e12
            roof = {"bound": "mfma", "achieved": ach, "peak": F16_DENSE_TFLOPS, "unit": "TFLOP/s",
                    "frac": ach / F16_DENSE_TFLOPS, "traffic": traffic, "kernel": kname,
                    "peak_note": f"dense f16 MFMA 2516.6 TF; achieved = {nx}*2*n*k*d per launch / avg launch time"}
    elif info["path"] == 2 and dom == "assign" and screen == 4:
        # k_s1 (km_screen1.hip): one fp16 MFMA per product (1.3 ms of MFMA at
        # c3 against 3.2 ms of HBM at the spec peak), candidates re-scored in
        # fp32; delta statistics on the fused geometries (c3), labels only
        # before the statistics pass on the unfused ones (c4)
        t_mfma = flops_launch / (F16_DENSE_TFLOPS * 1e12)
        b_alg = n_local * d * 4
        t_hbm = b_alg / (HBM_PEAK_GBS * 1e9)
        kname = ("k_s1 (one fp16 MFMA per product, fp32 re-score of candidates, delta statistics)"
                 if info["fused_stats"] else
                 "k_s1 (one fp16 MFMA per product, fp32 re-score of candidates; labels, statistics in a second pass)")
        note = (f"MFMA time at one fp16 MFMA per product {t_mfma * 1e3:.2f} ms vs {t_hbm * 1e3:.2f} ms HBM at 8 TB/s; "
                "the kernel also reads the row-norm bound (and, with delta statistics, the previous label): 4-8 B per row")
        if t_hbm >= t_mfma:
            ach = b_alg / avg_s / 1e9
            roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                    "traffic": traffic, "kernel": kname,
                    "bytes_note": "algorithmic N*d*4 per launch (X read once, SURVEY 8d); " + note,
                    "tflops": flops_launch / avg_s / 1e12,
                    "tflops_frac_f16_dense": flops_launch / avg_s / 1e12 / F16_DENSE_TFLOPS}
        else:
            ach = flops_launch / avg_s / 1e12
            roof = {"bound": "mfma", "achieved": ach, "peak": F16_DENSE_TFLOPS, "unit": "TFLOP/s",
                    "frac": ach / F16_DENSE_TFLOPS, "traffic": traffic, "kernel": kname,
                    "peak_note": "dense f16 MFMA 2516.6 TF, one MFMA per product; achieved = 2*n*k*d per launch / "
                                 "avg launch time; " + note,
                    "hbm_gbs": b_alg / avg_s / 1e9}
    elif info["path"] == 2 and dom == "assign" and screen == 5:
        # KM_SCREEN_ONE: k_assign_mfma16 with one fp16 MFMA per product
        ach = flops_launch / avg_s / 1e12
        roof = {"bound": "mfma", "achieved": ach, "peak": F16_DENSE_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / F16_DENSE_TFLOPS, "traffic": traffic,
                "kernel": "k_assign_mfma16 (one fp16 MFMA per product on 16x16x32, one-part bound)",
                "peak_note": "dense f16 MFMA 2516.6 TF, one MFMA per product; achieved = 2*n*k*d per launch / "
                             "avg launch time (HIP events, engine stream)",
                "hbm_gbs": n_local * d * 4 / avg_s / 1e9}
    elif info["path"] == 2 and dom == "assign":
        ach = flops_launch / avg_s / 1e12
        # the fused screen runs on v_mfma_f32_16x16x32_f16 where dp is a
        # multiple of 32 (k_fused16), else on 32x32x16 (k_fused)
        kname = (("k_fused16 (fp16x3 screen on 16x16x32 MFMA + f64 sums)" if info["dp"] % 32 == 0 else
                  "k_fused (fp16x3 screen on 32x32x16 MFMA + f64 sums)") if info["fused_stats"] else
                 "k_assign_wide (fp16x3 screen, feature chunks)" if info["dp"] > 256 else
                 "k_assign_mfma16 (fp16x3 screen on 16x16x32 MFMA)" if info["dp"] % 32 == 0 else
                 "k_assign_mfma (fp16x3 screen on 32x32x16 MFMA)")
        roof = {"bound": "mfma", "achieved": ach, "peak": F16X3_EFFECTIVE_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / F16X3_EFFECTIVE_TFLOPS, "traffic": traffic, "kernel": kname,
                "peak_note": "dense f16 MFMA 2516.6 TF / 3 (fp16x3 split: 3 MFMAs per product); "
                             "achieved = 2*n*k*d per launch / avg launch time (HIP events, engine stream)",
                "hbm_gbs": n_local * d * 4 / avg_s / 1e9}
    else:
        b = bytes_stats if dom == "stats" else bytes_assign
        ach = b / avg_s / 1e9
        roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": traffic, "kernel": "k_stats" if dom == "stats" else "k_assign_small",
                "bytes_note": "N*(d*4+4) per launch (rows once + labels)"}
    kernel_ms = {kk: (v[0] / max(v[1], 1)) for kk, v in kern.items()}
    if kern["update"][1] == 0 and kern["assign"][1] > 0:
        # the single-rank small path folds the update into the assign launch
        # (k_assign_small's last workgroup): one launch carries both
        kernel_ms["assign+update (folded)"] = kernel_ms.pop("assign")
        kernel_ms.pop("update")
    if coll is not None:
        kernel_ms["allreduce"] = coll[0] / max(coll[1], 1)
    pred = None
    if args.predict > 0:
        # predict (kmeans_spark.py:321-352): one assignment pass with no
        # statistics; labels stay in HBM (the LabelsRDD the caller collects)
        eng.profile(True, phases=("assign", "resolve"), every=1)
        eng.predict_device()                    # one untimed pass
        eng.prof_read("assign"), eng.prof_read("resolve")
        comm.barrier()
        tp0 = time.perf_counter()
        for _ in range(args.predict):
            eng.predict_device()                # synchronises per pass
        tp1 = time.perf_counter()
        pa, pr = eng.prof_read("assign"), eng.prof_read("resolve")
        eng.profile(False)
        ms_a = pa[0] / max(pa[1], 1)
        ms_w = (tp1 - tp0) / args.predict * 1e3
        pred = {"passes": args.predict, "ms_per_pass": ms_w, "kernel_ms": {"assign": ms_a, "resolve": pr[0] / max(pr[1], 1)},
                "gb_s": n_local * d * 4 / (ms_a / 1e3) / 1e9, "points_per_sec": n_local / (ms_w / 1e3),
                "kernel": ("k_assign_small (labels only)" if info["path"] == 1 else
                           "k_s1 (labels only)" if screen == 4 else
                           "k_fused16 / k_fused (no statistics)" if info["fused_stats"] else
                           "k_assign_wide" if info["dp"] > 256 else
                           "k_assign_mfma16" if info["dp"] % 32 == 0 else "k_assign_mfma"),
                "note": "ms_per_pass: host wall time per km_predict (launch + sync, labels left in HBM); "
                        "gb_s: rows read once (N*d*4) / HIP-event time of the assign launch"}

    # the iterations after new centroids (kmeans_spark.py:266-318 from the
    # start of a fit): the first runs the full-statistics screen (and, on the
    # k_s1 geometries, colours the chains), the second is the first delta
    # pass; steady state (ms_per_step) excludes both.  Host wall time of each
    # with its own sync, after the same set_centroids a fit makes
    first_iter = None
    if not args.no_first_iter:
        eng.set_centroids(C0)
        first_iter = {}
        for i in range(2):
            comm.barrier()
            tf0 = time.perf_counter()
            run.run(km, log, i + 1, first=i)
            eng.sync()
            tf1 = time.perf_counter()
            first_iter[f"iter{i + 1}_ms"] = (tf1 - tf0) * 1e3
        first_iter["note"] = ("host wall time per iteration with a sync, after set_centroids(C0): iter1 = full "
                              "statistics pass (first screen after new centroids), iter2 = the first pass of the "
                              "steady-state path (k_s1 with delta statistics on the c3 class)")
    if rank == 0:
        it_s = ran / dt
        out = {
            "metric": METRIC, "value": it_s, "unit": "Lloyd it/s", "n_gpus": world, "steps": args.steps,
            "steps_ran": ran, "warmup": args.warmup, "ms_per_step": dt / max(ran, 1) * 1e3,
            "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic Gaussian blobs generated in HBM (centers U(-10,10), std 1)",
            "config": {"workload": f"{args.config}: N={N} d={d} k={k}" + (", compute_sse=True" if sse else ""),
                       "N": N, "d": d, "k": k, "compute_sse": sse,
                       "parallelism": f"dp{world} (rows sharded, one RCCL all-reduce of k*(d+1) f64 per step)"},
            "points_per_sec": N * it_s, "roofline": roof, "kernel_avg_ms": kernel_ms,
            "resolve": {"q_rerank": run.last["q_rerank"], "q_full": run.last["q_full"]} if run.last else None,
            "empty_repairs_on_device": run.device_repairs,
            "screen": screen,
            "first_iter": first_iter,
            "host_ms_per_step": ({kk: v / max(ran, 1) for kk, v in host_ms.items()} if host_ms else None),
            "predict": pred,
            "arith": ("fp16 MFMA screen (balanced image, pairwise bound)" if screen in (2, 3) else
                      "one fp16 MFMA per product, candidates re-scored in fp32 with a rigorous bound" +
                      (", float64 delta statistics" if info["fused_stats"] else "") if screen == 4 else
                      "one fp16 MFMA per product with a rigorous one-part bound" if screen == 5 else
                      "fp16x3 MFMA screen with a rigorous bound") +
                     ", float64 exact re-rank of ambiguous points, float64 partial sums",
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(d, k, N, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
