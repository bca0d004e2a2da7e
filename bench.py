#!/usr/bin/env python3
"""bench.py — SpMM throughput on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workload (config.workload): ogbn-products-shaped synthetic power-law CSR (2,449,029 x 2,449,029,
123,718,280 nnz) x dense N=128 fp32 — the config BASELINE.json's north-star target is quoted on
(configs[2]); it fits one GPU.  A "step" is one SpMM over that matrix with inputs resident in HBM:
  N=1   oneflow_spmm.spmm(...) (op layer -> C-ABI -> plan/main/reduce HIP kernels)
  N>1   1-D row split over N ranks (BalancedSplitter rows): exchange of the Split(0) dense
        shards (RCCL all-gather, or the halo rows only; the fastest kept at setup) + local SpMM
        (strong scaling: the same matrix is divided across ranks).  config.parallelism names the
        exchange that ran; 2-D grids are measured but only reported (extra.grid_best).
value = 2*nnz*N FLOPs per step (whole job) / max-over-ranks step time, in GFLOP/s.

Extra objects: `roofline` (dominant kernel spmm_main, HIP events on its stream, algorithmic
gather-model bytes) and `cpu_baseline` (the operator's kCPU kernel, SURVEY.md §8d
row a2, on the host cores this process may use, plus a 1-thread run; rank 0 at N=1 only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config products] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "of-spmm_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
HBM_MEASURED_GBS = 6300.0  # the guide's measured HBM copy rate; above it the rate is "effective"
METRIC = "SpMM effective GFLOP/s + achieved HBM GB/s vs roofline, 1/2/4/8 MI355X"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


class PhaseWatch:
    """Per-rank phase log and deadline.  Every rank prints each phase it
    enters, with its elapsed time, to stderr; a watchdog thread ends a rank whose phase outlives
    its limit: it names the phase, aborts the native RCCL communicator (so peers blocked on this
    rank fail rather than hang) and exits with EXIT_STALL.  A rank that has touched the GPU only
    ever exits; it is never re-exec'd."""

    EXIT_STALL = 75

    def __init__(self, rank: int, world: int, scale: float = 1.0):
        import threading
        self.rank, self.world, self.scale = rank, world, scale
        self.t0 = time.monotonic()
        self.name, self.started, self.deadline = "start", self.t0, None
        self.on_abort = []  # callables run before the exit (communicator abort)
        self._lock = threading.Lock()
        threading.Thread(target=self._watch, name="phase-watch", daemon=True).start()

    def phase(self, name: str, limit_s: float | None = None):
        now = time.monotonic()
        limit = None if limit_s is None else limit_s * self.scale
        with self._lock:
            self.name, self.started = name, now
            self.deadline = None if limit is None else now + limit
        print(f"[rank {self.rank}/{self.world}] {now - self.t0:8.1f} s  phase: {name}"
              + (f" (limit {limit:.0f} s)" if limit is not None else ""), file=sys.stderr, flush=True)

    def _watch(self):
        while True:
            time.sleep(0.25)
            with self._lock:
                name, started, deadline = self.name, self.started, self.deadline
            if deadline is None or time.monotonic() <= deadline:
                continue
            print(f"[rank {self.rank}/{self.world}] STALLED: phase '{name}' still running after "
                  f"{time.monotonic() - started:.0f} s (limit {deadline - started:.0f} s); aborting "
                  f"the communicator and exiting {self.EXIT_STALL}", file=sys.stderr, flush=True)
            for f in self.on_abort:
                try:
                    f()
                except Exception as e:  # noqa: BLE001 -- exiting anyway
                    print(f"[rank {self.rank}] abort hook failed: {e!r}", file=sys.stderr, flush=True)
            os._exit(self.EXIT_STALL)


def alg_bytes(rows: int, nnz: int, n: int, s_v: int, s_i: int = 4) -> int:
    """Gather model: row_ptr once, col/val once, one B row per nonzero, C once."""
    return s_i * (rows + 1) + (s_i + s_v) * nnz + s_v * nnz * n + s_v * rows * n


def host_cpu() -> dict:
    """nproc and the CPU model of this host (recorded with every CPU number)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None  # cgroup v2 CPU quota of this process, in CPUs (None = unlimited / unknown)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "model": model, "affinity": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


class Mark:
    """A point on the launch stream: a HIP event (GPU), or the host clock after the work issued
    so far has finished (the CPU rehearsal, where every call is synchronous)."""

    def __init__(self, on_gpu: bool):
        self.on_gpu = on_gpu
        self.ev = torch.cuda.Event(enable_timing=True) if on_gpu else None
        self.t = 0.0

    def record(self):
        if self.on_gpu:
            self.ev.record()
        else:
            self.t = time.perf_counter()

    def ms_to(self, later: "Mark") -> float:
        return self.ev.elapsed_time(later.ev) if self.on_gpu else (later.t - self.t) * 1e3


def _claim_stdout():
    """Route fd 1 to stderr for the whole run (RCCL and the HIP runtime print banners on stdout)
    and return a writer on the real stdout for the one JSON line of the bench contract."""
    real = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    return os.fdopen(real, "w")


def _spawn_ranks_if_needed(gpus: int, deadline_s: float):
    """`python bench.py --gpus N` without a launcher: start the N ranks here (the environment
    contract of oneflow.distributed.launch, python/oneflow/distributed/launch.py:103-140) and exit
    with their status.  Runs before anything touches the GPU; the package is not imported (its
    native library stays unloaded in this parent)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ofx_launch", os.path.join(ROOT, "of-spmm_amd", "oneflow_spmm", "launch.py"))
    launch = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(launch)
    log(f"[bench] --gpus {gpus} without a launcher: spawning {gpus} local ranks "
        f"(deadline {deadline_s:.0f} s)")
    sys.exit(launch.spawn_local_ranks(gpus, [os.path.abspath(__file__), *sys.argv[1:]],
                                      timeout=deadline_s))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="products")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="host threads for input generation and the secondary CPU numbers")
    ap.add_argument("--cpu-baseline-threads", type=int, default=0,
                    help="threads of the cpu_baseline (default: the cores this process may use, "
                         "min(nproc, affinity, cgroup quota); never more)")
    ap.add_argument("--variant", type=int, default=0, help="force a kernel variant (VEC*100+LPR)")
    ap.add_argument("--comm", choices=["rccl", "rccl-p2p", "rccl-pull"], default=None,
                    help="all-gather schedule for N>1 (default: measured at setup, faster kept)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="column blocks for gather/SpMM overlap at N>1 (default: measured)")
    ap.add_argument("--exchange", default="auto",
                    help="B exchange for N>1: auto | any | allgather | halo | nsplit | grid<R>x<C>"
                         "[/s<S>].  auto (default): the fastest 1-D row-split exchange measured at "
                         "setup (all-gather or halo, the north star's partition); the 2-D grids "
                         "are measured too but only reported (extra.grid_best).  any: the fastest "
                         "of all, grids included")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend at N>1; gloo is a rehearsal of the multi-rank code "
                         "path on fewer GPUs (ranks share devices, bytes are host-staged: not a "
                         "performance number)")
    ap.add_argument("--force-rowsplit", action="store_true",
                    help="run the N>1 code path (RCCL all-gather + local SpMM) even with one rank")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: rehearse the N>1 path on host tensors with the kCPU kernel (needs "
                         "--backend gloo; not a performance number)")
    ap.add_argument("--deadline", type=float, default=1800.0,
                    help="seconds the whole multi-rank run may take when bench.py spawns its ranks; "
                         "past it the ranks are terminated and the exit status is 124")
    ap.add_argument("--phase-timeout-scale", type=float,
                    default=float(os.environ.get("OFX_PHASE_TIMEOUT_SCALE", "1")),
                    help="multiplies every per-rank phase limit (N>1: a rank stalled in a phase "
                         "past its limit names it and exits 75)")
    ap.add_argument("--stall-test", default=os.environ.get("OFX_BENCH_STALL", ""),
                    help="tests only: 'rank:phase' makes that rank sleep in that phase; "
                         "'rank:exchange' makes it never join its first exchange of B; "
                         "'0:native-tune' fails the first tune as if every native exchange had")
    ap.add_argument("--exchange-deadline", type=float,
                    default=float(os.environ.get("OFX_EXCHANGE_DEADLINE", "120")),
                    help="N>1, set-up / tune / warmup: seconds an exchange of B may take to "
                         "complete before the rank aborts its communicator and exits 76 naming it "
                         "(0 = off; the timed steps never wait: exchanges stay asynchronous)")
    ap.add_argument("--tune-budget", type=float, default=120.0,
                    help="seconds of exchange-candidate timing at setup (N>1); the candidates run "
                         "in order of their modelled time, the rest are skipped")
    args = ap.parse_args()
    _spawn_ranks_if_needed(args.gpus, args.deadline)
    out_stream = _claim_stdout()

    t_wall0 = time.time()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)
    rehearsal = args.backend == "gloo"
    on_gpu = args.device == "cuda"
    if not on_gpu and not rehearsal:
        log("[bench] error: --device cpu is a rehearsal of the multi-rank path: use --backend gloo")
        sys.exit(2)
    if on_gpu:
        dev_index = local_rank % torch.cuda.device_count() if rehearsal else local_rank
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    red_dev = "cpu" if rehearsal else device  # where the timing reductions run

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
    rowsplit = world > 1 or args.force_rowsplit
    watch = PhaseWatch(rank, world, args.phase_timeout_scale) if rowsplit else None
    global _WATCH
    _WATCH = watch
    stall_rank, _, stall_phase = args.stall_test.partition(":")

    def enter_phase(name, limit_s):
        if watch is None:
            return
        watch.phase(name, limit_s)
        if (stall_phase and stall_phase != "native-tune" and int(stall_rank) == rank
                and name.startswith(stall_phase)):
            time.sleep(1e6)  # the watchdog ends this rank
    enter_phase("process group init", 300)
    if rowsplit:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29571")
            os.environ.setdefault("RANK", "0")
        if rehearsal:
            dist.init_process_group("gloo", world_size=world, rank=rank)
        else:
            dist.init_process_group("nccl", device_id=device, world_size=world, rank=rank)
        if dist.get_world_size() != args.gpus and not (args.force_rowsplit and args.gpus == 1):
            log(f"[bench] error: {dist.get_world_size()} ranks joined, --gpus {args.gpus}")
            sys.exit(2)

    import oneflow_spmm as fs
    from oneflow_spmm import ops, synth
    from oneflow_spmm.distributed import RowSplitSpmm

    cfg = {**synth.CONFIGS, **synth.EXTRA_CONFIGS}[args.config]
    m, k, nnz, n, dt = cfg["m"], cfg["k"], cfg["nnz"], cfg["n"], cfg["dtype"]
    s_v = torch.empty(0, dtype=dt).element_size()
    threads = args.cpu_threads

    # ---- inputs (this rank's rows only), resident in HBM before timing -------------------------
    enter_phase("inputs", 900)
    t0 = time.time()
    rp_full = synth.row_ptr(m, k, nnz)
    lo, hi = fs._C.balanced_range(m, world, rank)
    rows = hi - lo
    cols = synth.columns(m, k, rp_full, lo, hi, threads=threads)
    j0, j1 = int(rp_full[lo]), int(rp_full[hi])
    nnz_local = j1 - j0
    vals = synth.values(j0, j1, dt)
    local_rp = torch.from_numpy((rp_full[lo:hi + 1] - rp_full[lo]).astype(np.int32))
    d_rp = local_rp.to(device)
    d_ci = torch.from_numpy(cols).to(device)
    d_v = vals.to(device)
    out = torch.empty((rows, n), dtype=dt, device=device)
    log(f"[bench] inputs for rank {rank}: rows {rows} nnz {nnz_local} built in {time.time() - t0:.1f}s")

    events = [Mark(on_gpu) for _ in range(3)]
    opts = ops.make_options(variant=args.variant) if args.variant else None
    if not rowsplit:
        d_b = synth.dense(0, k, n, dt, device=device)
        if opts is None:
            def step():
                fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out)
        else:
            kern = ops.SpmmCsrKernel(m, k, n, nnz, torch.int32, dt, device, opts)

            def step():
                kern(d_rp, d_ci, d_v, d_b, out)
    else:
        pinned_sub = int(args.exchange.split("/s")[1]) if "/s" in args.exchange else 1
        auto = args.exchange in ("auto", "any")
        full = None
        if auto or args.exchange.startswith(("nsplit", "grid")):
            # the grid / column-split candidates need the whole CSR on every rank
            f_ci = torch.from_numpy(synth.columns(m, k, rp_full, threads=threads)).to(device)
            full = (torch.from_numpy(rp_full.astype(np.int32)).to(device), f_ci,
                    synth.values(0, nnz, dt).to(device))

        def build_rs(comm):
            enter_phase("communicator init", 400)
            try:
                r = RowSplitSpmm(m, k, n, nnz_local, dt, torch.int32, device, comm=comm)
            except fs.OfxError as e:  # own RCCL communicator refused: torch.distributed's (also RCCL)
                log(f"[bench] native RCCL communicator unavailable ({e}); using torch.distributed")
                r = RowSplitSpmm(m, k, n, nnz_local, dt, torch.int32, device, comm="torch")
            watch.on_abort.append(r.abort)
            # set-up, tune and warmup await every exchange (a peer that never joins ends this rank
            # with the exchange named); the timed steps do not
            r.set_exchange_deadline(args.exchange_deadline)
            if stall_phase == "exchange" and int(stall_rank) == rank:
                # tests only: this rank never joins its first exchange of B (its peers' deadline fires)
                r.gather_block = lambda *a, **kw: time.sleep(1e6)
            enter_phase("bind (shards, remap, plans, halo and grid layouts)", 900)
            klo, khi = r.k_range
            r.load_shard(synth.dense(klo, khi, n, dt, device=device))
            r.bind(d_rp, d_ci, d_v, halo=auto or args.exchange == "halo", full_csr=full,
                   grid_subs=tuple(sorted({1, 2, pinned_sub})))
            return r

        rs = build_rs("torch" if rehearsal else "auto")
        # exchange: all-gather (ring / point-to-point) x pipeline depth (column blocks gathered
        # while the previous block computes), or halo-only rows; measured here, untimed, the
        # fastest 1-D row-split candidate kept (every candidate gives the same bytes)
        comm_times, tune_s, comm_fallback = {}, None, None
        if args.comm or args.pipeline or not auto:
            rs.exchange = args.exchange if not auto else "allgather"
            if rs.exchange not in ("allgather", "halo") and rs.exchange not in rs.grids:
                raise SystemExit(f"--exchange {rs.exchange}: not available (grids: {list(rs.grids)})")
            rs.comm_kind = args.comm or rs.comm_kind
            rs.set_pipeline(args.pipeline or 1)
            if rs.exchange == "halo":  # column blocks of the halo exchange
                rs.set_pipeline(1)
                rs.set_halo_pipeline(args.pipeline or 1)
        else:
            t_tune = time.time()

            def tune():
                return rs.tune(out, force=args.force_rowsplit, budget_s=args.tune_budget, log=log,
                               on_candidate=lambda nm: enter_phase(f"tune: {nm}", 180),
                               rowsplit_only=args.exchange == "auto")
            # tests only (--stall-test <rank>:native-tune): the first tune fails as if every native
            # candidate had, so the gloo rehearsal walks the rebuild below
            fake_fail = stall_phase == "native-tune"
            try:
                if fake_fail:
                    raise RuntimeError("RowSplitSpmm.tune: every exchange failed: (test)")
                comm_times = tune()
            except RuntimeError as e:
                # every candidate on the native communicator failed (on every rank alike: tune's
                # times are max-reduced): the same exchanges over torch.distributed's RCCL group
                if ((rs.comm_kind == "torch" and not fake_fail)
                        or not str(e).startswith("RowSplitSpmm.tune:")):
                    raise
                comm_fallback = str(e)[:400]
                log(f"[bench] {comm_fallback}; rebuilding the exchange on torch.distributed")
                watch.on_abort.remove(rs.abort)
                try:
                    rs.close()
                except Exception as ce:  # noqa: BLE001 -- an aborted communicator may refuse
                    log(f"[bench] closing the native communicator: {ce}")
                rs = build_rs("torch")
                comm_times = tune()
            tune_s = time.time() - t_tune
            log("[bench] exchange candidates (ms, max over ranks; model-predicted): " +
                ", ".join(f"{kk} {vv:.3f} ({rs.tune_report[kk]['predicted_ms']:.3f})"
                          for kk, vv in sorted(comm_times.items(), key=lambda x: x[1])))
        setup_s = time.time() - t0
        log(f"[bench] exchange kept: {rs.exchange} / {rs.comm_kind} / pipeline "
            f"{rs.halo_chunks if rs.exchange == 'halo' else rs.chunks}")

        def step():
            rs.step(out)

    # ---- warmup + timed region -----------------------------------------------------------------
    enter_phase("warmup", 300)
    for _ in range(args.warmup):
        step()
    sync()
    if rowsplit:
        dist.barrier()
    sync()
    if rowsplit:
        rs.set_exchange_deadline(0)  # asynchronous exchanges in the timed region
    enter_phase("timed steps", 600)
    ev_start, ev_end = Mark(on_gpu), Mark(on_gpu)
    t_start = time.perf_counter()
    ev_start.record()
    for _ in range(args.steps):
        step()
    ev_end.record()
    if rowsplit:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t_start
    if rowsplit:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    flops = 2.0 * nnz * n
    value = flops * args.steps / elapsed / 1e9

    enter_phase("phase timing and report", 600)
    # ---- dominant-kernel timing: events on the launch stream around the SpMM launches ---------
    # N=1: the op call (plan + main + reduce; main dominates).  N>1: the local SpMM after the
    # gather.  Measured over a separate short run so the timed region above has no extra events.
    sync()
    spmm_ms, gather_ms = [], []
    for _ in range(max(args.steps, 5)):
        if not rowsplit:
            events[1].record()
            step()
            events[2].record()
        else:
            events[0].record()
            rs.gather_phase()
            events[1].record()
            rs.compute_phase(out)
            events[2].record()
        sync()
        spmm_ms.append(events[1].ms_to(events[2]))
        if rowsplit:
            gather_ms.append(events[0].ms_to(events[1]))
    kern_ms_separate = float(np.mean(spmm_ms))
    kern_ms = kern_ms_separate
    if not rowsplit:
        # N=1: the op's launches are the only work on the launch stream, so the HIP events that
        # bracket the timed region on that stream give the average op duration directly
        kern_ms = ev_start.ms_to(ev_end) / args.steps
    gather_mean = float(np.mean(gather_ms)) if gather_ms else 0.0
    phase = {"spmm_ms_max": kern_ms, "gather_ms_max": gather_mean}
    if rowsplit and world > 1:
        t = torch.tensor([kern_ms, gather_mean], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        phase = {"spmm_ms_max": float(t[0]), "gather_ms_max": float(t[1])}
    # cold-cache SpMM: a 512 MB scratch write evicts the 256 MB Infinity Cache
    # and the L2s before each launch; median of 5.  The timed region above is the warm number.
    cold = []
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=device) if on_gpu else None
    for i in range(5 if on_gpu else 0):
        scratch.fill_(i)
        if not rowsplit:
            events[1].record()
            step()
            events[2].record()
        else:
            events[1].record()
            rs.compute_phase(out)
            events[2].record()
        sync()
        cold.append(events[1].ms_to(events[2]))
    del scratch
    cold_ms = float(np.median(cold)) if cold else float("nan")
    # N=1, reported beside the value (never the value): the same op with attr static_csr, whose
    # kernel state keeps the work-list plan across calls (a GNN's constant graph)
    static_ms = None
    if not rowsplit and on_gpu and opts is None:
        fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out, static_csr=True)  # plans once
        sync()
        e0, e1 = Mark(on_gpu), Mark(on_gpu)
        e0.record()
        for _ in range(args.steps):
            fs.spmm(d_rp, d_ci, d_v, m, k, d_b, out=out, static_csr=True)
        e1.record()
        sync()
        static_ms = e0.ms_to(e1) / args.steps
        fs._C.static_plans(release=True)
    bytes_launch = alg_bytes(rows, nnz_local, n, s_v)
    if rowsplit and rs.exchange in rs.grids:  # the grid's SpMM: its row group x N/C columns
        gp = rs.grids[rs.exchange]
        bytes_launch = gp.sub * alg_bytes(gp.ghi - gp.glo, int(rp_full[gp.ghi] - rp_full[gp.glo]),
                                          gp.w, s_v)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9

    # HBM-side traffic of the dominant kernel per launch from the committed rocprofv3 PMC summary
    # of this same workload (scripts/profile.sh + scripts/rocprof_summary.py; beyond-L2 bytes =
    # 128 B x TCC_EA0_RDREQ_128B (== 2 x FETCH_SIZE on gfx950) + WRITE_SIZE).
    traffic, traffic_src = None, None
    prof = os.path.join(ROOT, "profiles", f"{args.config}_rocprof.json")
    if not rowsplit and os.path.exists(prof):
        pj = json.load(open(prof))
        t = pj.get("traffic", {}).get("beyond_l2_bytes_per_launch")
        if t:
            traffic, traffic_src = float(t), os.path.relpath(prof, ROOT)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16",
                  torch.float64: "f64"}[dt],
        "data": "synthetic (deterministic Chung-Lu power-law CSR, gamma 2.5; dataset-shaped)",
        "config": {"workload": f"{args.config}: CSR {m}x{k}, {nnz} nnz x dense N={n}",
                   "m": m, "k": k, "nnz": nnz, "n": n, "index": "int32",
                   # built from the exchange tune() kept (or the one pinned), never a constant
                   "parallelism": "single GPU" if not rowsplit else
                   (f"REHEARSAL with gloo on {torch.cuda.device_count() if on_gpu else 0} GPU(s), "
                    f"host-staged bytes, not a performance number: {rs.describe()}")
                   if rehearsal else rs.describe()},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_unit": "bytes per launch (beyond L2: Infinity Cache + HBM)",
                     "traffic_source": traffic_src,
                     # the algorithmic (gather-model) rate can exceed what HBM alone delivers when
                     # hot B rows are served by the 256 MB Infinity Cache
                     "model": ("effective (gather model; beyond-L2 traffic includes Infinity-Cache "
                               "hits)" if achieved > HBM_MEASURED_GBS else "gather model"),
                     "kernel": "spmm_main_kernel (+plan/reduce, timed together; HIP events "
                               "on the launch stream around the timed region at N=1)",
                     "alg_bytes_per_launch": bytes_launch, "kernel_ms": round(kern_ms, 4)},
    }
    result["extra"] = {"kernel_ms_events_separate_run": round(kern_ms_separate, 4),
                       "kernel_ms_cold_median": round(cold_ms, 4) if cold else None,
                       "static_csr_ms_per_step": round(static_ms, 4) if static_ms else None,
                       "static_csr_gflops": round(flops / (static_ms * 1e-3) / 1e9, 2)
                       if static_ms else None,
                       "gbs_cold": round(bytes_launch / (cold_ms * 1e-3) / 1e9, 1) if cold else None}
    if rowsplit:
        nz = torch.tensor([nnz_local, nnz_local], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(nz[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(nz[1:], op=dist.ReduceOp.SUM)
        comm_size = rs.comm_size()
        g2d = getattr(rs, "tune_best_2d", None)
        result["extra"].update({
            "ranks_seen": dist.get_world_size(),
            "rccl_comm_ranks": comm_size[0] if comm_size else None,
            # ranks of the communicator the kept exchange ran on (RCCL's, or the torch group's)
            "exchange_comm_ranks": comm_size[0] if comm_size and rs.comm_kind != "torch"
            else dist.get_world_size(rs.group),
            "exchange_is_rowsplit": rs.is_rowsplit_exchange(rs.exchange),
            # the fastest 2-D partition measured by tune(): reported, never the value (a grid needs
            # the whole CSR on every rank and is not the north star's 1-D row split)
            "grid_best": ({"exchange": g2d[0], "ms": round(g2d[1], 4),
                           "gflops": round(flops / (g2d[1] * 1e-3) / 1e9, 2)} if g2d else None),
            "allgather_ms_rank0": round(gather_mean, 4),
            "spmm_ms_rank0": round(kern_ms, 4),
            "allgather_ms_max": round(phase["gather_ms_max"], 4),
            "spmm_ms_max": round(phase["spmm_ms_max"], 4),
            # SpMM phase alone with the gathered B resident (SURVEY.md §8e reports it separately)
            "spmm_phase_gflops_aggregate": round(flops / (phase["spmm_ms_max"] * 1e-3) / 1e9, 2),
            # B bytes this rank receives in the exchange phase / its time
            "allgather_gbs_per_rank": round(((rs.halo.halo_rows * n if rs.exchange == "halo" else
                                              rs.grids[rs.exchange].exchange_rows()[0]
                                              if rs.exchange in rs.grids
                                              else (rs.k_padded - rs.pad) * n) * s_v) /
                                            (phase["gather_ms_max"] * 1e-3) / 1e9, 2)
            if phase["gather_ms_max"] > 0 else None,
            "rows_rank0": rows, "nnz_rank0": nnz_local,
            "exchange": rs.exchange, "allgather_schedule": rs.comm_kind,
            "pipeline_blocks": rs.halo_chunks if rs.exchange == "halo" else rs.chunks,
            "halo_rows_received": rs.halo.halo_rows if rs.halo is not None else None,
            "remote_rows_total": (rs.k - (rs.k_range[1] - rs.k_range[0])),
            "allgather_tune_ms": {kk: (round(vv, 4) if np.isfinite(vv) else None)
                                  for kk, vv in comm_times.items()},
            # the north star's configuration (plain row split + one all-gather of B), always
            # measured by tune() whichever exchange wins: ms per step and its aggregate rate
            "rowsplit_allgather_p1": ({"ms": round(comm_times[ag1], 4),
                                       "gflops": round(flops / (comm_times[ag1] * 1e-3) / 1e9, 2)}
                                      if (ag1 := f"{'torch' if rs.comm_kind == 'torch' else 'rccl'}/p1") in comm_times
                                      and np.isfinite(comm_times[ag1]) else None),
            "tune_errors": getattr(rs, "tune_errors", {}) or None,
            # every native-RCCL candidate failed and the exchange was rebuilt on torch.distributed
            "comm_fallback": comm_fallback,
            # every candidate: model time (xGMI assumption), the model refitted to
            # the first measurement, the measured time (max over ranks) and whether it ran
            "tune_candidates": getattr(rs, "tune_report", {}) or None,
            "tune_rate_fit_gbs": round(rs.tune_rate_fit / 1e9, 2)
            if getattr(rs, "tune_rate_fit", None) else None,
            "tune_seconds": round(tune_s, 2) if tune_s is not None else None,
            "setup_seconds": round(setup_s, 2),
            "nnz_per_rank_max_over_mean": round(float(nz[0]) / (float(nz[1]) / world), 4)})
        # memory of the run: peak device memory (torch's allocator, this process) and peak host
        # RSS per rank, max and sum over ranks
        import resource
        peak = torch.tensor([torch.cuda.max_memory_allocated(device) / 1e9 if on_gpu else 0.0,
                             resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6],
                            dtype=torch.float64, device=red_dev)
        peak_sum = peak.clone()
        if world > 1:
            dist.all_reduce(peak, op=dist.ReduceOp.MAX)
            dist.all_reduce(peak_sum, op=dist.ReduceOp.SUM)
        result["extra"]["memory_gb"] = {
            "device_peak_max_rank": round(float(peak[0]), 2),
            "device_peak_sum": round(float(peak_sum[0]), 2),
            "host_rss_peak_max_rank": round(float(peak[1]), 2),
            "host_rss_peak_sum": round(float(peak_sum[1]), 2)}
        result["extra"]["wall_seconds_to_line"] = round(time.time() - t_wall0, 1)

    # ---- CPU baseline (rank 0, N=1 only): the operator's own kCPU kernel ------
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle
        # bounded sample: the first rows holding <= 130M nonzeros (all of products; rows are
        # randomly permuted, so a leading block is representative), B whole on the host
        r_s = m if nnz <= 130_000_000 else int(np.searchsorted(rp_full, 130_000_000, side="right")) - 1
        nnz_s = int(rp_full[r_s])
        flops_s = 2.0 * nnz_s * n
        what = "full workload" if r_s == m else f"rows [0,{r_s}) = {nnz_s} nnz"
        h_b = synth.dense(0, k, n, dt)
        h_rp = torch.from_numpy(rp_full.astype(np.int32))
        h_ci = torch.from_numpy(cols)
        h_out = torch.empty((r_s, n), dtype=dt)
        # the cores this process may use: min(nproc, affinity, cgroup quota).  On the GPU box a
        # 16-CPU quota sits on a 256-core host; more threads than the quota only add throttling
        # (round 2 measured 256 threads at a third of the 16-thread rate), so none are used.
        hc = host_cpu()
        usable = min(x for x in (hc["nproc"] or 1, hc["affinity"],
                                 int(np.ceil(hc["cgroup_cpu_quota"])) if hc["cgroup_cpu_quota"]
                                 else None) if x)
        nt_cpu = min(args.cpu_baseline_threads or usable, usable)

        def time_a2(nt, row_end, budget_s, max_reps):
            kw = dict(out=h_out[:row_end], row_end=row_end, num_threads=nt)
            ops.spmm_csr_cpu(h_rp, h_ci, vals, h_b, m, k, **kw)  # warm-up (page-in)
            reps_, t_ = 0, 0.0
            while t_ < budget_s and reps_ < max_reps:
                t1 = time.perf_counter()
                ops.spmm_csr_cpu(h_rp, h_ci, vals, h_b, m, k, **kw)
                t_ += time.perf_counter() - t1
                reps_ += 1
            return 2.0 * float(rp_full[row_end]) * n * reps_ / t_ / 1e9, reps_, t_

        cpu_gflops, reps, t_cpu = time_a2(nt_cpu, r_s, 6.0, 5)
        bitexact = bool(torch.equal(h_out.view(torch.uint8), out[:r_s].cpu().view(torch.uint8)))
        # one thread (OneFlow's default CPU_THREADING_RUNTIME=SEQ, CMakeLists.txt:54, and the
        # launcher's OMP_NUM_THREADS=1, launch.py:117-118) on the first rows holding ~1/16 of the
        # sample's nonzeros
        r1 = int(np.searchsorted(rp_full[: r_s + 1], rp_full[r_s] // 16))
        g1, reps1, t1s = time_a2(1, r1, 4.0, 2)
        result["cpu_baseline"] = {
            "value": round(cpu_gflops, 3), "unit": "GFLOP/s", "cores": nt_cpu, "kind": "port",
            "implementation": "ofx_spmm_csr_cpu: the operator's DeviceType::kCPU kernel (SURVEY.md "
                              "§8a row a2; OpenMP row-parallel, the reference's gather -> mul -> "
                              "segment-sum order, same hub schedule as the GPU)",
            "host": {**hc, "usable_cores": usable},
            "sample": f"{what} x{reps} runs ({t_cpu:.1f} s), {nt_cpu} OpenMP threads = the cores "
                      f"this process may use ({hc['nproc']} host cores, affinity {hc['affinity']}, "
                      f"cgroup quota {hc['cgroup_cpu_quota']}); same inputs and schedule as the GPU",
            "bitexact_vs_gpu": bitexact,
            "one_thread": {"value": round(g1, 3), "unit": "GFLOP/s", "cores": 1,
                           "sample": f"rows [0,{r1}) = {int(rp_full[r1])} nnz x{reps1} runs "
                                     f"({t1s:.1f} s)"}}
        # the oracle's C restatement (test infrastructure; the checker, timed for reference only)
        rp_np = rp_full[: r_s + 1]
        ci_np = cols[:nnz_s].astype(np.int64)
        v_np = vals.numpy() if dt != torch.bfloat16 else vals.view(torch.int16).numpy().view(np.uint16)
        v_np = v_np[:nnz_s]
        b_np = h_b.numpy() if dt != torch.bfloat16 else h_b.view(torch.int16).numpy().view(np.uint16)
        oracle.spmm(rp_np, ci_np, v_np, b_np, dtype=result["dtype"], nthreads=nt_cpu,
                    row_end=min(r_s, 100000))
        t1 = time.perf_counter()
        oracle.spmm(rp_np, ci_np, v_np, b_np, dtype=result["dtype"], nthreads=nt_cpu)
        t_o = time.perf_counter() - t1
        result["extra"]["cpu_oracle"] = {
            "value": round(flops_s / t_o / 1e9, 3), "unit": "GFLOP/s", "cores": nt_cpu,
            "sample": f"{what}, one run ({t_o:.1f} s), oracle/spmm_oracle.c (the tests' checker)"}
        del ci_np, b_np, h_rp, h_ci, h_b, h_out
        # BASELINE configs[0]: the Cora-shaped problem on the OneFlow CPU op path (plumbing)
        cc = synth.CONFIGS["cora"]
        c_rp, c_ci, c_v = synth.csr(cc["m"], cc["k"], cc["nnz"], threads=threads)
        c_b = synth.dense(0, cc["k"], cc["n"], cc["dtype"])
        cora = {}
        for nt in (1, threads):
            fs.spmm_csr(c_rp, c_ci, c_v, cc["m"], cc["k"], c_b, num_threads=nt)
            ts = []
            for _ in range(50):
                t1 = time.perf_counter()
                fs.spmm_csr(c_rp, c_ci, c_v, cc["m"], cc["k"], c_b, num_threads=nt)
                ts.append(time.perf_counter() - t1)
            cora[f"ms_{nt}_threads"] = round(float(np.median(ts)) * 1e3, 4)
        result["extra"]["cora_cpu_op_path"] = cora
    if rank == 0:
        print(json.dumps(result), file=out_stream, flush=True)
    if rowsplit:
        enter_phase("shutdown", 120)
        rs.close()
        dist.destroy_process_group()
        if watch is not None:
            watch.phase("done")


_WATCH = None
EXIT_EXCHANGE = 76


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # noqa: BLE001
        if type(e).__name__ != "ExchangeTimeout":
            raise
        # an exchange of B did not complete (the RCCL path aborted its communicator already): name
        # the phase and the exchange, run the abort hooks, exit -- never re-exec a GPU process
        w = _WATCH
        where = f"phase '{w.name}'" if w is not None else "setup"
        print(f"[rank {os.environ.get('RANK', '0')}/{os.environ.get('WORLD_SIZE', '1')}] EXCHANGE "
              f"STALLED in {where}: {e}; exiting {EXIT_EXCHANGE}", file=sys.stderr, flush=True)
        for f in (w.on_abort if w is not None else []):
            try:
                f()
            except Exception as ee:  # noqa: BLE001 -- exiting anyway
                print(f"abort hook failed: {ee!r}", file=sys.stderr, flush=True)
        os._exit(EXIT_EXCHANGE)
