"""Benchmark: scan-pair registrations/s (8k-pt clouds, 20 ICP iterations) at 1..N GPUs.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

With ``--gpus N > 1`` and no ``WORLD_SIZE`` in the environment, bench.py starts
``torch.distributed.run`` with N ranks as a CHILD process (before anything here touches the GPU) and
exits with its status; the driver's own ``torch.distributed.run`` launch lands directly in the rank
code.

Workload (BASELINE.json configs[2]/[3]): every rank registers its own batch of
1024 independent synthetic radar scan pairs (8192 source / 8192 target points, pair i seeded
1000 + i, rank r owns pairs [1024 r, 1024 (r + 1))), 20 ICP iterations exactly (PCL defaults
otherwise; the |ΔMSE| early stop disabled so every pair does the same work) plus the fitness pass.
A step = one device-resident batch registration + the all-gather of the 96-B result structs over
RCCL.  Inputs are resident in HBM before timing.  value = pairs registered by all ranks / max-over-
ranks wall time.  The results checked (status, iterations, pairs of every rank and both pair groups
against the oracle) are the TIMED run's, copied before any diagnostic rerun.

Beside the headline: ``incl_upload`` (the same steps with each batch's H2D upload from pinned host
memory inside the timed region, overlapped with the previous batch on a copy stream), ``gather``
(the all-gather timed alone), ``roofline`` (the kernel with the larger share of the single-group
step, the batched update since round 4, with the batched search beside it as ``nn_kernel``: SURVEY
§8(d)'s algorithmic bytes over the library's HIP events on the launch stream; ``traffic`` from the
committed PMC passes of the same library build, matched by sha256), ``c1`` / ``c2`` / ``c5`` (BASELINE.json's single-pair configs:
2k/2k PCL defaults, 8k/8k 20 iterations, and the 8k-scan-vs-65k-map registration, one pair per call,
each with its own roofline, oracle check and single-core CPU baseline) and ``cpu_baseline`` (the
oracle — the C restatement of the reference CPU path — on one pinned core, with median / p90 per
pair, and on all the process's cores, both running the node's two fitness passes,
``iterative_closest_point.cpp:516,:520``).

``--dry-run`` exercises the launcher, the sharding and the gather on CPU (gloo, no GPU, no
registration): every rank fills its result rows with their global pair index, and rank 0 checks the
gathered order (tests/test_bench_launcher.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "icp-4dradar_amd"))

PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector (= f32 MFMA) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
FLOP_PER_PAIR_EVAL = 8     # 3 sub + 3 mul + 2 add (FLANN L2_Simple); compare/select not counted
FLOP_PER_BOX_TEST = 11     # 6 sub + 3 mul + 2 add (point-to-box lower bound); max/compare not counted


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=1024, help="pairs per GPU")
    ap.add_argument("--points", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="single-core CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--cpu-all-seconds", type=float, default=8.0, help="all-cores CPU-baseline budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-upload", action="store_true", help="skip the incl-upload figure")
    ap.add_argument("--configs", default="C1,C2,C5", help="single-pair configs reported beside the headline "
                                                          "(rank 0, N=1): C1, C2, C5; '' for none")
    ap.add_argument("--no-c5", action="store_true", help="drop C5 from --configs")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 headline (profiling the single-pair configs)")
    ap.add_argument("--config-cpu-seconds", type=float, default=3.0, help="CPU-baseline budget per single-pair config")
    ap.add_argument("--check", type=int, default=8, help="pairs of the timed run checked against the oracle "
                                                         "(N=1; with N>1 two per rank)")
    ap.add_argument("--gather", choices=("icp4r", "torch"), default="icp4r",
                    help="N>1: the results' all-gather through the library's RCCL communicator "
                         "(icp4r_gather_results, include/icp4r/icp4r_multi.h) or torch.distributed's")
    ap.add_argument("--dry-run", action="store_true", help="launcher/shard/gather only, gloo on CPU (tests)")
    ap.add_argument("--plan", action="append", default=[], metavar="NAME=VALUE",
                    help="plan option for the library context (icp4r_set_plan_option; A/B runs, DESIGN.md §6)")
    ap.add_argument("--plan-from-env", action="store_true",
                    help="(tools) also take plan options from ICP4R_<NAME> environment variables")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    """N ranks through torch.distributed.run, as a child process (never exec from here)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def _env_rank():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def user_plan(args) -> dict:
    """The plan options of this run: --plan NAME=VALUE (and, for the A/B tools, ICP4R_<NAME>
    variables with --plan-from-env).  The library itself reads no environment."""
    import icp4r

    out = icp4r.env_plan() if args.plan_from_env else {}
    for kv in args.plan:
        k, v = kv.split("=", 1)
        out[k.strip()] = int(v)
    return out


def _metric():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        return json.load(f)["metric"]


# ------------------------------------------------------------------------------------------ dry run
def run_dry(args) -> int:
    import torch
    import torch.distributed as dist

    from icp4r import RESULT_DTYPE
    from icp4r import dist as idist

    world, rank, _ = _env_rank()
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    P = args.pairs
    mine = idist.shard(rank, world, P)
    rows = np.zeros(P, RESULT_DTYPE)
    rows["reserved"] = np.arange(mine.start, mine.stop, dtype=np.int32)
    rows["iterations"] = args.iters
    local = torch.from_numpy(rows.view(np.uint8).reshape(P, 96).copy())
    t0 = time.perf_counter()
    allr = idist.gather_results(local, world)
    elapsed = time.perf_counter() - t0
    res = np.frombuffer(allr.numpy().tobytes(), dtype=RESULT_DTYPE)
    order_ok = bool(len(res) == world * P and (res["reserved"] == np.arange(world * P)).all())
    if rank == 0:
        print(json.dumps({"metric": _metric(), "dry_run": True, "n_gpus": world, "pairs_per_gpu": P,
                          "gathered_pairs": int(len(res)), "gather_order_ok": order_ok,
                          "gather_ms": elapsed * 1e3}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if order_ok else 1


# ------------------------------------------------------------------------------------------ inputs
def make_shard(first: int, count: int, n: int):
    from icp4r import synth

    src = np.empty((count, n, 4), np.float32)
    tgt = np.empty((count, n, 4), np.float32)
    for k in range(count):
        p = synth.make_pair(first + k, n)
        src[k] = p.src_xyzi()
        tgt[k] = p.tgt_xyzi()
    return src, tgt


def _pose_err(T, To):
    T = np.asarray(T, np.float64)
    To = np.asarray(To, np.float64)
    M = T[:3, :3].T @ To[:3, :3]
    dr = float(np.arctan2(np.linalg.norm([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]]) / 2,
                          (np.trace(M) - 1) / 2))
    return float(np.abs(T[:3, 3] - To[:3, 3]).max()), dr


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------------------------------ CPU baseline
def cpu_baseline(src, tgt, iters: int, budget_s: float, all_budget_s: float) -> dict:
    """The oracle (C restatement of PCL 1.8.1 ICP, -O2) per pair as the node calls it: align, then
    getFitnessScore twice (`iterative_closest_point.cpp:514,:516,:520`; the oracle's align computes
    the first).  Single core (the calling thread pinned to one CPU) with per-pair median / p90, and
    all the process's cores (a thread pool; the oracle's ctypes calls release the GIL)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    import oracle  # checker / CPU baseline only

    kw = dict(numerics=oracle.NUM_F32, max_iterations=iters, mse_threshold_absolute=-1.0,
              transformation_epsilon=-1.0)

    def one(k):
        t0 = time.perf_counter()
        o = oracle.align(src[k], tgt[k], **kw)
        oracle.fitness(src[k], tgt[k], o["T"])  # the node's second getFitnessScore (:520)
        return time.perf_counter() - t0

    allowed = sorted(os.sched_getaffinity(0))
    # the box's CPU share for one GPU is 16 threads (OMP_NUM_THREADS there); never more than allowed
    threads = max(1, min(len(allowed), int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))
    # all cores first: pool threads inherit the (full) affinity of the thread that creates them
    n_all, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while (time.perf_counter() - t0) < all_budget_s and n_all < len(src):
            chunk = list(range(n_all, min(len(src), n_all + threads)))
            list(ex.map(one, chunk))
            n_all += len(chunk)
    dt_all = time.perf_counter() - t0
    # one pinned core
    core = allowed[0]
    os.sched_setaffinity(0, {core})
    try:
        one(0)  # warm-up
        per, t0 = [], time.perf_counter()
        while len(per) < len(src) and (time.perf_counter() - t0) < budget_s:
            per.append(one(len(per)))
        dt = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, set(allowed))
    per_ms = np.array(per) * 1e3
    cpu = _cpu_model()
    return {"value": len(per) / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "per_pair_ms_median": float(np.median(per_ms)), "per_pair_ms_p90": float(np.percentile(per_ms, 90)),
            "fitness_passes": 2,
            "sample": f"{len(per)} pairs of the benchmark workload ({src.shape[1]}/{tgt.shape[1]} pts, {iters} iters "
                      f"+ 2 getFitnessScore passes as the node calls them), oracle/icp_oracle.c: FLANN-style kd-tree "
                      f"NN + float Umeyama, -O2, 1 thread pinned to CPU {core}, {dt:.1f} s on {cpu} "
                      f"(nproc={os.cpu_count()}, {len(allowed)} CPUs allowed)",
            "all_cores": {"value": n_all / dt_all, "unit": "pairs/s", "cores": threads,
                          "sample": f"{n_all} pairs on a {threads}-thread pool over {dt_all:.1f} s (the box's CPU "
                                    f"share for one GPU)"}}


# ------------------------------------------------------------------------------------------ single pairs
LIB = os.path.join(ROOT, "icp-4dradar_amd", "icp4r", "_lib", "libicp4r.so")
PMC_PATH = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def library_sha256() -> str | None:
    """Hash of the library this run loads: a committed PMC figure is used only for the very build it
    was measured on (profiles/pmc_traffic.json records the hash of the build tools/profile_round.sh
    profiled); after any rebuild `traffic` is null until the profile is re-taken."""
    import hashlib

    try:
        with open(os.environ.get("ICP4R_LIBRARY", LIB), "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def pmc_traffic(config: str, kernel: str, sha: str | None):
    """(HBM bytes per launch of `kernel` in `config` from the committed FETCH_SIZE (x2, gfx950) +
    WRITE_SIZE passes, or None, and a note saying why)."""
    try:
        with open(PMC_PATH) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    if sha and pmc.get("library_sha256") == sha:
        same = "same library build"
    else:
        # the library differs: the row still holds when the ICP kernels' sources, their launch code,
        # headers and build flags are the ones profiled (a rebuild after a GICP / map / ego change)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from srchash import icp_sources_sha256

        src = icp_sources_sha256()
        if not src or pmc.get("icp_sources_sha256") != src:
            return None, "profiles/pmc_traffic.json was measured on another build of the ICP kernels (sha256 differs)"
        same = "same ICP kernel sources and build flags (library sha256 differs elsewhere)"
    row = pmc.get("configs", {}).get(config, {}).get(kernel)
    if not row or "hbm_bytes_per_launch" not in row:
        return None, f"no PMC row for {kernel} in {config}"
    return row["hbm_bytes_per_launch"], f"profiles/pmc_traffic.json ({pmc.get('tag')}), {same}"


# The sequential float folds of the PCL-numerics update (Eigen's rowwise().sum() and
# the cross-covariance, in correspondence order) are one dependent add chain per sum: two passes of n
# dependent adds per iteration.  Measured cost per dependent add with the fold's LDS prefetch:
# 6.4-6.7 cycles (tools/experiments/chain_bench.hip) at the 2.4 GHz max clock.
CHAIN_CYCLES_PER_ADD = 6.4
CLOCK_GHZ = 2.4


def sigma_panels(n: int, max_kc: int = 680) -> dict:
    """Eigen 3.3's GEMM panels of umeyama's sigma for |C| = n (icp4r_math.hpp sigma_kc, default host
    facts: L1d 32 KiB, gebp mr 8 -> max_kc 680)."""
    if n < 48 or n <= max_kc:
        kc = n
    else:
        r = n % max_kc
        kc = max_kc if r == 0 else max_kc - 8 * ((max_kc - 1 - r) // (8 * (n // max_kc + 1)))
    return {"kc": kc, "panels": -(-n // kc) if kc else 0}


def update_chain_floor_ms(n: int) -> float:
    """Dependent-add floor of one PCL-numerics update: pass A's n-long centroid chains, then pass B's
    panel chains (kc long, all panels at once) and the panel adds into sigma."""
    sp = sigma_panels(n)
    return (n + sp["kc"] + sp["panels"]) * CHAIN_CYCLES_PER_ADD / (CLOCK_GHZ * 1e6)


def single_pair_cpu(src, tgt, oparams: dict, budget_s: float, fitness_passes: int) -> dict:
    """The oracle on one pinned core, the node's call: align (+ its getFitnessScore) and, for the
    icp4radar node, the second getFitnessScore (`iterative_closest_point.cpp:516,:520`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only

    allowed = sorted(os.sched_getaffinity(0))
    core = allowed[0]
    os.sched_setaffinity(0, {core})
    try:
        o = oracle.align(src, tgt, **oparams)  # warm-up
        per, t0 = [], time.perf_counter()
        while (time.perf_counter() - t0) < budget_s and len(per) < 2000:
            t1 = time.perf_counter()
            o = oracle.align(src, tgt, **oparams)
            if fitness_passes > 1:
                oracle.fitness(src, tgt, o["T"])
            per.append(time.perf_counter() - t1)
        dt = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, set(allowed))
    per_ms = np.array(per) * 1e3
    return {"value": len(per) / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "per_pair_ms_median": float(np.median(per_ms)), "per_pair_ms_p90": float(np.percentile(per_ms, 90)),
            "fitness_passes": fitness_passes,
            "sample": f"the same pair registered {len(per)} times ({len(src)}/{len(tgt)} pts) by oracle/icp_oracle.c "
                      f"(FLANN-style kd-tree NN + float Umeyama, -O2), 1 thread pinned to CPU {core}, {dt:.1f} s on "
                      f"{_cpu_model()}"}


def single_pair_measure(ctx, name: str, workload: str, src, tgt, params, oparams: dict, sha: str | None,
                        reps: int, cpu_budget_s: float | None, fitness_passes: int, check: bool,
                        hbm_formula: bool = False) -> dict:
    """One pair per call (`iterative_closest_point.cpp:510-521` is one pair per frame; C5 the node's
    scan-to-map call, `radar_odometry.cpp:386-411`), synchronous icp4r_align from host buffers.
    value = registrations/s of the device time (HIP events around the whole launch sequence);
    wall = the synchronous call incl. both clouds' PCIe upload and the result download.
    roofline: the NN search kernel (nn_tile_kernel), FP32 VALU work counted on the device (evaluations
    x 8 + box tests x 11 FLOP) over its average launch time (HIP events on its stream); for C5 also
    priced against HBM with SURVEY §8(d)'s hash-grid byte formula.  The update's bound is the
    sequential float fold chain (2 x n dependent adds per iteration), reported as `chain_floor_ms`."""
    import icp4r

    n, m = len(src), len(tgt)
    r, _ = ctx.align(src, tgt, params)  # warm-up
    ctx.reset_timers()
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r, _ = ctx.align(src, tgt, params)
        walls.append(time.perf_counter() - t0)
    dev_ms, calls = ctx.batch_time_ms()
    # per-kernel figures from the same registration repeated with per-kernel events (they cost device
    # time between kernels, so the timed calls above ran without them)
    ctx.set_kernel_timing(True)
    try:
        ctx.reset_timers()
        for _ in range(max(reps // 4, 3)):
            r, _ = ctx.align(src, tgt, params)
        nn_ms, nn_launches = ctx.kernel_time_ms()
        upd_ms, upd_launches = ctx.stage_time_ms(icp4r.STAGE_UPDATE)
        _, kcalls = ctx.batch_time_ms()
        st = ctx.nn_stats()
    finally:
        ctx.set_kernel_timing(False)
    calls = kcalls  # (per-registration launch counts below are over the timing calls)
    evals = st["evaluations"] / max(nn_launches, 1)
    tests = st["box_tests"] / max(nn_launches, 1)
    plan = icp4r.plan(1, n, m, ctx=ctx)
    iters = int(r.iterations)
    if plan["solo"]:
        return _solo_measure(ctx, r, name, workload, src, tgt, params, oparams, walls, dev_ms, calls, nn_ms,
                             nn_launches, st, plan, cpu_budget_s, fitness_passes, check, sha)
    kernel = "nn_tile_kernel" if plan["pruned"] and not plan["lds"] else "nn_kernel"
    flops = evals * FLOP_PER_PAIR_EVAL + tests * FLOP_PER_BOX_TEST
    tflops = flops / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0
    traffic, traffic_note = pmc_traffic(name, kernel, sha)
    roof = {"bound": "valu", "kernel": kernel, "achieved": tflops, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": tflops / PEAK_FP32_TFLOPS, "traffic": traffic, "traffic_source": traffic_note,
            "library_sha256": sha, "avg_launch_ms": nn_ms, "launches_per_registration": nn_launches / max(calls, 1),
            "evaluations_per_launch": evals, "box_tests_per_launch": tests, "flop_per_launch": flops,
            "evaluated_fraction_of_brute_force": evals / (n * m)}
    if traffic is not None and nn_ms > 0:
        roof["traffic_gbs"] = traffic / (nn_ms * 1e-3) / 1e9
    if hbm_formula:
        # SURVEY §8(d) hash-grid formula per NN launch: queries in (16 B) + key out (8 B) + 16 B per
        # examined target (sum_q K_q) + 24 B per box tested (lo/hi xyz) — every examination priced as a
        # fresh read.  nn_tile_kernel stages each target tile in LDS once per workgroup and re-reads it
        # from there, so these are candidate bytes, not HBM traffic: the HBM fraction is `hbm_counter`
        # (the FETCH / WRITE counters of this build), this one is labelled as what it is.
        b = n * (16 + 8) + 16 * evals + 24 * tests
        a = b / (nn_ms * 1e-3) / 1e9 if nn_ms > 0 else 0.0
        roof["candidate_bytes_lds_reused"] = {"bytes_per_launch": b, "rate_gbs": a,
                                              "note": "SURVEY 8(d) hash-grid formula; LDS re-reads, not HBM"}
    if traffic is not None and nn_ms > 0:
        roof["hbm_counter"] = {"achieved": traffic / (nn_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                               "frac": traffic / (nn_ms * 1e-3) / 1e9 / PEAK_HBM_GBS}
    floor_ms = update_chain_floor_ms(n)
    ukernel = ("fold_update_held_kernel" if plan.get("held_update") else "fold_update_wide_kernel") if plan.get("wide_update") \
        else "fold_update_kernel"
    update = {"bound": "latency", "kernel": ukernel,
              "achieved": floor_ms, "peak": upd_ms, "unit": "ms",
              "frac": floor_ms / upd_ms if upd_ms > 0 else None, "chain_floor_ms": floor_ms, "avg_launch_ms": upd_ms,
              "launches_per_registration": upd_launches / max(calls, 1),
              "share_of_device_time": upd_ms * upd_launches / max(calls, 1) / dev_ms if dev_ms > 0 else None,
              "sigma_panels": sigma_panels(n),
              "note": "PCL's summation order: pass A's n-long sequential centroid chains, then pass B's "
                      "sigma chains of one Eigen GEMM panel (kc) each plus the panel adds; achieved / peak = "
                      "that dependent-add floor / the launch's time (DESIGN.md §5)"}
    upd_traffic, upd_note = pmc_traffic(name, update["kernel"], sha)
    update["traffic"], update["traffic_source"] = upd_traffic, upd_note
    roof["share_of_device_time"] = nn_ms * nn_launches / max(calls, 1) / dev_ms if dev_ms > 0 else None
    # `roofline` prices the kernel with the larger share of the registration's device time (the top row
    # of profiles/<round>/kernel_stats_<config>.csv), the other one sits beside it
    nn_first = (roof["share_of_device_time"] or 0) >= (update["share_of_device_time"] or 0)
    out = {"workload": workload, "value": 1e3 / dev_ms if dev_ms > 0 else None, "unit": "pairs/s",
           "registration_device_ms": dev_ms, "registration_wall_ms_incl_pcie": 1e3 * float(np.median(walls)),
           "status": int(r.status), "iterations": iters, "plan": plan,
           "roofline": roof if nn_first else update,
           ("update_kernel" if nn_first else "nn_kernel"): update if nn_first else roof,
           "nn_plus_update_share_of_device_time": (nn_ms * nn_launches + upd_ms * upd_launches) / max(calls, 1) / dev_ms
           if dev_ms > 0 else None}
    _check_and_cpu(ctx, out, r, src, tgt, params, oparams, cpu_budget_s, fitness_passes, check)
    return out


def _check_and_cpu(ctx, out: dict, r, src, tgt, params, oparams: dict, cpu_budget_s, fitness_passes: int, check: bool):
    if check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # checker only: the registration above was timed without it

        o = oracle.align(src, tgt, aligned=True, **oparams)
        r2, al = ctx.align(src, tgt, params, want_aligned=True)  # (untimed: the aligned cloud too)
        out["bit_exact_vs_oracle"] = bool((r.matrix() == o["T"]).all() and r.fitness == o["fitness"] and
                                          int(r.iterations) == o["iterations"] and bytes(r2) == bytes(r) and
                                          (al[:, :3].view(np.uint32) == o["aligned"][:, :3].view(np.uint32)).all())
    if cpu_budget_s:
        cpu = single_pair_cpu(src, tgt, oparams, cpu_budget_s, fitness_passes)
        out["cpu_baseline"] = cpu
        out["speedup_vs_cpu"] = out["value"] / cpu["value"] if out["value"] else None


def _solo_measure(ctx, r, name, workload, src, tgt, params, oparams, walls, dev_ms, calls, solo_ms, solo_launches, st,
                  plan, cpu_budget_s, fitness_passes, check, sha) -> dict:
    """The solo plan (solo_kernel: every ICP iteration and the fitness pass of the pair in one
    1024-thread workgroup, after init_kernel and index_kernel).  Its bound is latency: the
    registration is a dependent chain — per iteration the cached-neighbour test, the search of the
    misses, then PCL's sequential float folds (2 x n dependent adds: pass A's centroids before pass B's
    cross-covariance) and the serial 3x3 solve; the fitness pass ends in a sequential double sum of n
    terms.  `chain_floor_ms` is those fold chains alone at the dependent-add latency measured for
    them (CHAIN_CYCLES_PER_ADD, tools/experiments/chain_bench.hip); frac = floor / kernel time.  The
    FP32 VALU figures of the search beside it are the device-counted evaluations and box tests of the
    whole registration over the kernel time."""
    n, m = len(src), len(tgt)
    iters = int(r.iterations)
    per = max(solo_launches, 1)
    evals = st["evaluations"] / per
    tests = st["box_tests"] / per
    flops = evals * FLOP_PER_PAIR_EVAL + tests * FLOP_PER_BOX_TEST
    floor_ms = iters * update_chain_floor_ms(n) + n * CHAIN_CYCLES_PER_ADD / (CLOCK_GHZ * 1e6)
    tflops = flops / (solo_ms * 1e-3) / 1e12 if solo_ms > 0 else 0.0
    roof = {"bound": "latency", "kernel": "solo_kernel", "achieved": floor_ms, "peak": solo_ms, "unit": "ms",
            "frac": floor_ms / solo_ms if solo_ms > 0 else None, "chain_floor_ms": floor_ms,
            "avg_launch_ms": solo_ms, "launches_per_registration": solo_launches / max(calls, 1),
            "kernel_share_of_device_time": solo_ms * solo_launches / max(calls, 1) / dev_ms if dev_ms > 0 else None,
            "valu": {"achieved": tflops, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": tflops / PEAK_FP32_TFLOPS,
                     "evaluations_per_registration": evals, "box_tests_per_registration": tests,
                     "evaluated_fraction_of_brute_force": evals / (n * m * (iters + 1))},
            "cache_hit_rate": st["cache_hits"] / st["cache_tested"] if st["cache_tested"] else None,
            "traffic": None, "traffic_source": None, "library_sha256": sha,
            "note": "achieved / peak here = the fold-chain floor / the kernel's time (latency-bound: PCL's "
                    "sequential summation order); see DESIGN.md §5 solo_kernel"}
    # HBM bytes of the launch (the whole registration) from the PMC passes of this build, beside its
    # algorithmic floor: every source and target point read once (16 B each) and the result row
    roof["traffic"], roof["traffic_source"] = pmc_traffic(name, "solo_kernel", sha)
    roof["algorithmic_bytes"] = 16 * (n + m) + 96
    out = {"workload": workload, "value": 1e3 / dev_ms if dev_ms > 0 else None, "unit": "pairs/s",
           "registration_device_ms": dev_ms, "registration_wall_ms_incl_pcie": 1e3 * float(np.median(walls)),
           "status": int(r.status), "iterations": iters, "plan": plan, "roofline": roof}
    _check_and_cpu(ctx, out, r, src, tgt, params, oparams, cpu_budget_s, fitness_passes, check)
    return out


def single_pair_configs(ctx, which: list[str], sha, cpu_s: float | None, check: bool) -> dict:
    """C1, C2, C5 of BASELINE.json: one pair per call on one GPU."""
    import icp4r
    from icp4r import synth

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # parameters of the checker / CPU baseline only

    fixed = dict(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    out = {}
    if "C1" in which:  # the reference-default CPU config: PCL defaults (10 iterations, early stops live)
        p = synth.make_pair(0, 2048)
        out["c1"] = single_pair_measure(
            ctx, "C1", "C1: 1 pair, 2048/2048-pt scans, PCL defaults (10 iterations max, early stops live) + fitness",
            p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(), {"numerics": oracle.NUM_F32}, sha, reps=50,
            cpu_budget_s=cpu_s, fitness_passes=2, check=check)
    if "C2" in which:  # single 8k pair, 20 iterations
        p = synth.make_pair(1, 8192)
        out["c2"] = single_pair_measure(
            ctx, "C2", "C2: 1 pair, 8192/8192-pt scans, 20 ICP iterations (fixed) + fitness",
            p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(**fixed), dict(numerics=oracle.NUM_F32, **fixed), sha,
            reps=20, cpu_budget_s=cpu_s, fitness_passes=2, check=check)
    if "C5" in which:  # 8k scan vs the 65,540-pt map of 10 accumulated scans (radar_odometry.cpp:386-411)
        p = synth.make_map_pair(0)
        out["c5"] = single_pair_measure(
            ctx, "C5", "C5: 8192-pt scan vs 65540-pt map (10 accumulated scans), 20 iterations (fixed) + fitness",
            p.src_xyzi(), p.tgt_xyzi(), icp4r.default_params(**fixed), dict(numerics=oracle.NUM_F32, **fixed), sha,
            reps=10, cpu_budget_s=cpu_s, fitness_passes=1, check=check, hbm_formula=True)
    return out


# ------------------------------------------------------------------------------------------ GPU run
def run_gpu(args) -> int:
    import torch
    import torch.distributed as dist

    world, rank, local = _env_rank()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
        rank = dist.get_rank()
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import icp4r
    from icp4r import dist as idist

    sha = library_sha256()
    which = [c for c in args.configs.split(",") if c and not (args.no_c5 and c == "C5")]
    opts = user_plan(args)
    if args.no_c3:  # the single-pair configs alone (tools/profile_round.sh profiles them this way)
        ctx = icp4r.Context(dev.index, plan=opts)
        out = single_pair_configs(ctx, which, sha, None if args.no_cpu else args.config_cpu_seconds, args.check > 0)
        ctx.close()
        if rank == 0:
            print(json.dumps({"metric": _metric(), "configs_only": True, "library_sha256": sha, **out}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    n = args.points
    P = args.pairs
    first = idist.shard(rank, world, P).start
    src_h, tgt_h = make_shard(first, P, n)
    src = torch.from_numpy(src_h.reshape(-1, 4)).to(dev)
    tgt = torch.from_numpy(tgt_h.reshape(-1, 4)).to(dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * n
    cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
    results = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
    gathered = torch.zeros((world * P, 96), dtype=torch.uint8, device=dev)

    ctx = icp4r.Context(dev.index, plan=opts)
    # fixed work: 20 iterations for every pair (the |ΔMSE| and exact-identity stops disabled)
    params = icp4r.default_params(max_iterations=args.iters, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)

    def mk_batch(s, t):
        return icp4r.Batch(src=s.data_ptr(), tgt=t.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                           tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), guess=None, aligned=None, npairs=P,
                           max_src_n=n, max_tgt_n=n)

    batch = mk_batch(src, tgt)
    stream = torch.cuda.current_stream(dev).cuda_stream

    comm = None
    if world > 1 and args.gather == "icp4r":
        # the library's own RCCL communicator (one rank per GPU); rank 0's id reaches the others over the
        # torch.distributed store
        uid = [icp4r.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = icp4r.Comm(ctx, world, rank, uid[0])

    def gather():
        if world > 1:
            if comm is not None:  # icp4r_gather_results: ncclAllGather of the device-written rows
                comm.gather(results.data_ptr(), world * P, gathered.data_ptr(), stream)
            else:
                idist.gather_results(results, world, out=gathered)

    def step():
        ctx.align_batch_device(batch, params, results.data_ptr(), stream)
        gather()

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.reset_timers()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    batch_ms, _ = ctx.batch_time_ms()
    # the TIMED run's results (every step writes the same rows; copied before any rerun below)
    timed = (gathered if world > 1 else results).cpu().numpy().copy()

    # the all-gather alone
    gather_ms = None
    if world > 1:
        barrier_sync()
        tg = time.perf_counter()
        for _ in range(10):
            gather()
        barrier_sync()
        gather_ms = max_over_ranks((time.perf_counter() - tg) / 10 * 1e3)

    # incl-upload: the same steps with each batch uploaded from pinned host memory inside the timed
    # region; batch k+1's upload (copy stream) overlaps batch k's registration (compute stream)
    upload = None
    if not args.no_upload:
        src_pin = torch.from_numpy(src_h.reshape(-1, 4)).pin_memory()
        tgt_pin = torch.from_numpy(tgt_h.reshape(-1, 4)).pin_memory()
        slots = [(torch.empty_like(src), torch.empty_like(tgt)) for _ in range(2)]
        slot_batches = [mk_batch(s, t) for s, t in slots]
        copy_stream = torch.cuda.Stream(dev)
        comp = torch.cuda.current_stream(dev)
        uploaded = [torch.cuda.Event() for _ in range(2)]
        freed = [torch.cuda.Event() for _ in range(2)]
        for e in freed:
            e.record(comp)

        def upload_step(k):
            sl = k % 2
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_event(freed[sl])
                slots[sl][0].copy_(src_pin, non_blocking=True)
                slots[sl][1].copy_(tgt_pin, non_blocking=True)
                uploaded[sl].record(copy_stream)
            comp.wait_event(uploaded[sl])
            ctx.align_batch_device(slot_batches[sl], params, results.data_ptr(), stream)
            gather()
            freed[sl].record(comp)

        # untimed warmup of this leg too: the copy stream's first transfers and both slots' first
        # registrations carry one-time costs (queue creation, first touch) that are not per batch
        for k in range(max(args.warmup, 1) * 2):
            upload_step(k)
        barrier_sync()
        tu = time.perf_counter()
        for k in range(args.steps):
            upload_step(k)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        up_elapsed = max_over_ranks(time.perf_counter() - tu)
        # the upload alone (H2D rate)
        torch.cuda.synchronize(dev)
        th = time.perf_counter()
        for _ in range(3):
            slots[0][0].copy_(src_pin, non_blocking=True)
            slots[0][1].copy_(tgt_pin, non_blocking=True)
        torch.cuda.synchronize(dev)
        h2d_s = (time.perf_counter() - th) / 3
        nbytes = src_pin.numel() * 4 + tgt_pin.numel() * 4
        same = bool((results.cpu().numpy() == timed[rank * P:(rank + 1) * P] if world > 1 else
                     results.cpu().numpy() == timed).all())
        upload = {"value": world * P * args.steps / up_elapsed, "unit": "pairs/s",
                  "ms_per_step": up_elapsed / args.steps * 1e3, "h2d_bytes_per_step": nbytes,
                  "h2d_ms_alone": h2d_s * 1e3, "h2d_gbs": nbytes / h2d_s / 1e9, "results_equal_resident": same,
                  "note": "H2D of each batch's clouds (pinned host -> HBM) inside the timed region, double-buffered: "
                          "batch k+1 uploads on a copy stream while batch k registers"}
        del slots, slot_batches, src_pin, tgt_pin

    # Kernel-level measurements (roofline, test and update kernels): the timed steps run the batch as
    # pair groups on several streams (icp4r run_pairs, plan option groups), where one group's kernels
    # overlap another's and a launch time is not one kernel's; so the same steps are repeated once
    # more with a single group, outside the timed region, and the per-kernel numbers come from that
    # run (tools/profile_round.sh profiles the single-group configuration, so rocprof's averages
    # match these).
    # (per-kernel events only here: each event record between two kernels costs device time, so the
    # timed steps above run without them — icp4r_set_kernel_timing)
    groups_prev, _ = ctx.get_plan_option("groups")
    ctx.set_plan_option("groups", 1)
    try:
        ctx.set_kernel_timing(True)
        ctx.reset_timers()
        for _ in range(min(args.steps, 5)):
            ctx.align_batch_device(batch, params, results.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        group1_batch_ms, _ = ctx.batch_time_ms()
    finally:
        ctx.set_kernel_timing(False)
        ctx.set_plan_option("groups", groups_prev)
    single_group_equal = bool((results.cpu().numpy() == (timed[rank * P:(rank + 1) * P] if world > 1 else timed)).all())
    nn_ms, nn_launches = ctx.kernel_time_ms()  # the NN launches (the batched search); the update below
    test_ms, test_launches = ctx.stage_time_ms(icp4r.STAGE_NN_TEST)
    upd_ms, upd_launches = ctx.stage_time_ms(icp4r.STAGE_UPDATE)
    st = ctx.nn_stats()  # work the NN kernels performed in the single-group steps
    evals, tests = st["evaluations"], st["box_tests"]
    plan = icp4r.plan(P, n, n, ctx=ctx)
    kernel = "nn_lds_kernel" if plan["lds"] else "nn_pruned_kernel" if plan["pruned"] else "nn_kernel"

    # the single-pair configs C1, C2, C5 (rank 0 at N=1: one GPU each; their CPU baselines too)
    configs = {}
    if rank == 0 and world == 1 and which:
        configs = single_pair_configs(ctx, which, sha, None if args.no_cpu else args.config_cpu_seconds,
                                      args.check > 0)

    # checks on the TIMED results: statuses, iteration counts, and pairs of every rank / both pair
    # groups against the oracle (rank 0 regenerates those pairs' inputs from their seeds)
    res = np.frombuffer(timed.tobytes(), dtype=icp4r.RESULT_DTYPE)
    status_ok = bool((res["status"] == 0).all())
    iters_ok = bool((res["iterations"] == args.iters).all())
    diag = {"status_nonzero": int((res["status"] != 0).sum()), "iter_min": int(res["iterations"].min()),
            "iter_max": int(res["iterations"].max()), "conv_states": sorted(set(int(v) for v in res["convergence_state"])),
            "single_group_rerun_equal": single_group_equal}
    ok = status_ok and iters_ok and single_group_equal
    check = []
    if rank == 0 and args.check > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        from icp4r import synth

        if world == 1:
            k = min(args.check, P)
            picks = sorted(set(np.linspace(0, P - 1, k).round().astype(int).tolist()) | {P // 2 - 1, P // 2} & set(range(P)))
        else:
            picks = sorted({r * P + j for r in range(world) for j in (0, P - 1)})
        for g in picks:
            p = synth.make_pair(g, n)
            o = oracle.align(p.src_xyzi(), p.tgt_xyzi(), numerics=oracle.NUM_F32, max_iterations=args.iters,
                             mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
            T = res[g]["T"].reshape(4, 4).T
            dt, dr = _pose_err(T, o["T"])
            check.append({"pair": int(g), "rank": int(g // P), "group": int((g % P) >= P // 2), "dt_m": dt, "dr_rad": dr,
                          "bit_exact": bool((T == o["T"]).all() and res[g]["fitness"] == o["fitness"])})
        ok = ok and all(c["dt_m"] <= 1e-4 and c["dr_rad"] <= 1e-4 for c in check)
    ok = ok and all(c.get("bit_exact_vs_oracle", True) and c["status"] == 0 for c in configs.values())

    total_pairs = world * P * args.steps
    value = total_pairs / elapsed
    # the search kernel's own work: every evaluation except the test kernel's one per hit
    evals_per_launch = (evals - st["cache_hits"]) / max(nn_launches, 1)
    tests_per_launch = tests / max(nn_launches, 1)
    flops_per_launch = evals_per_launch * FLOP_PER_PAIR_EVAL + tests_per_launch * FLOP_PER_BOX_TEST
    achieved_tflops = flops_per_launch / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0
    brute_equiv_tflops = P * n * n * FLOP_PER_PAIR_EVAL / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0

    # cached-neighbour test kernel (HBM-bound; by default only the fitness pass's test runs here, the
    # iteration passes' tests are fused into fold_update_kernel's tail): per tested query X (16, .w =
    # L) + nn_t (16) read, per hit its key (8) written; in an iteration pass (ICP4R_FUSE_TEST=0) also
    # U (4) read, X (16) + U (4) written.
    cache_test = None
    t_own = st["cache_tested"] - st["tested_in_update"]
    h_own = st["cache_hits"] - st["hits_in_update"]
    if test_launches:
        tb = (t_own * 32 + h_own * 8) / test_launches
        cache_test = {"kernel": "nn_cache_test_kernel", "bound": "hbm", "avg_launch_ms": test_ms,
                      "launches": test_launches, "bytes_per_launch": tb,
                      "achieved": tb / (test_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                      "frac": tb / (test_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                      "hit_rate": st["cache_hits"] / max(st["cache_tested"], 1),
                      "tests_fused_into_update": st["tested_in_update"]}
    # The two kernels that share the C3 step, each priced against HBM on SURVEY §8(d)'s algorithmic
    # bytes: every cloud read once per ICP pass, 16 B per point — 16 * (N + M) * pairs per launch (each
    # launch is one pass over the batch) — with the PMC counter bytes of the same kernel, shape and
    # library build beside them (`traffic`; profiles/pmc_traffic.json).  `roofline` is the one with
    # the larger share of the single-group step's device time (the top row of
    # profiles/<round>/kernel_stats_C3.csv); the other sits beside it.
    alg_bytes = 16 * (n + n) * P
    default_shape = (P, n, args.iters) == (1024, 8192, 20)

    def hbm_roof(kname: str, avg_ms: float, launches: int) -> dict:
        tr, tr_note = (pmc_traffic("C3", kname, sha) if default_shape
                       else (None, "profiles cover the default C3 shape only"))
        ach = alg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        return {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": ach / PEAK_HBM_GBS, "algorithmic_bytes_per_launch": alg_bytes,
                "traffic": tr, "traffic_source": tr_note,
                "traffic_gbs": tr / (avg_ms * 1e-3) / 1e9 if tr and avg_ms > 0 else None,
                "traffic_over_algorithmic": tr / alg_bytes if tr else None,
                "library_sha256": sha, "avg_launch_ms": avg_ms, "launches": launches,
                "share_of_device_time": avg_ms * launches / max(min(args.steps, 5), 1) / group1_batch_ms
                if group1_batch_ms > 0 else None}

    # fold_update_kernel: PCL's sequential float folds (pass A centroids, pass B sigma panels), the solve,
    # and the next pass's cached-neighbour test fused into its tail.  Per tested point it reads X (16 B,
    # .w = L), nn_t (16) and U (4) and writes X and U: `one_read_bytes` counts X and nn_t once plus the
    # test's U / writes; the counters show the passes' re-reads.
    update = hbm_roof("fold_update_kernel", upd_ms, upd_launches)
    update["cache_hit_rate"] = st["cache_hits"] / max(st["cache_tested"], 1)
    if upd_launches and upd_ms > 0:
        ub = (P * n * 32 * upd_launches + st["tested_in_update"] * 24) / upd_launches
        update["one_read_bytes"] = {"bytes_per_launch": ub, "achieved": ub / (upd_ms * 1e-3) / 1e9,
                                    "frac": ub / (upd_ms * 1e-3) / 1e9 / PEAK_HBM_GBS}
    # the batched search: HBM on the same §8(d) bytes, and its FP32 VALU work counted on the device
    search = hbm_roof(kernel, nn_ms, nn_launches)
    search["valu"] = {
        "achieved": achieved_tflops, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": achieved_tflops / PEAK_FP32_TFLOPS, "flop_per_launch": flops_per_launch,
        "evaluations_per_launch": evals_per_launch, "box_tests_per_launch": tests_per_launch,
        "evaluated_fraction_of_brute_force": evals_per_launch / (P * n * n),
        "brute_force_equivalent_tflops": brute_equiv_tflops,
        "note": "distance evaluations x 8 FLOP (3 sub, 3 mul, 2 add) + point-to-box tests x 11 FLOP of the "
                "exact pruned search (queries the cached-neighbour test could not resolve), counted on the "
                "device; compare/select/ballot/LDS not counted. brute_force_equivalent_tflops = n*m*8 per "
                "pass / search time: exact pruning, so SURVEY 8(d)'s FLOP roofline does not bound it"}
    update_first = (update["share_of_device_time"] or 0) >= (search["share_of_device_time"] or 0)
    roofline, beside = (update, search) if update_first else (search, update)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(src_h, tgt_h, args.iters, args.cpu_seconds, args.cpu_all_seconds)
        line = {
            "metric": _metric(),
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded 4D-radar scan pairs, SURVEY.md App. B)",
            "config": {
                "workload": f"C3/C4: {P} independent pairs per GPU, {n}/{n}-pt scans, {args.iters} ICP iterations "
                            f"(fixed) + fitness pass, exact NN ({'kd-block pruned' if plan['pruned'] else 'brute force'}), "
                            f"PCL numerics (bit-exact float restatement)",
                "nn_plan": plan,
                "pairs_per_gpu": P, "points": n, "iterations": args.iters,
                "parallelism": f"pairs sharded over {world} rank(s), RCCL all-gather of results" if world > 1
                else "1 GPU",
            },
            "roofline": roofline,
            ("nn_kernel" if update_first else "update_kernel"): beside,
            "incl_upload": upload,
            "gather": {"ms": gather_ms, "bytes": world * P * 96,
                       "via": "icp4r_gather_results (library RCCL communicator, ncclAllGather)" if comm is not None
                       else "torch.distributed all_gather_into_tensor (RCCL)"} if world > 1 else None,
            "cache_test_kernel": cache_test,
            **configs,
            "cpu_baseline": cpu,
            "speedup_vs_cpu": (value / cpu["value"]) if cpu else None,
            "batch_device_ms": batch_ms,
            "parity_ok": ok,
            "parity_check": check,
            "result_diag": diag,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.check()
        comm.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        return launch(args, argv)  # nothing above has touched the GPU
    if args.dry_run:
        return run_dry(args)
    return run_gpu(args)


if __name__ == "__main__":
    sys.exit(main())
