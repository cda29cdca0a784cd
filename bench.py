#!/usr/bin/env python3
"""Benchmark: batched ALIP-MPC-CBF solves/sec on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg1|cfg2|cfg3|cfg4|cfg5] [--batch B] ...

One "step" = one fused interior-point solve of a batch of B independent NLP instances whose inputs are
already resident in HBM (one launch of solve_kernel through the C ABI on the current HIP stream).
Default workload = BASELINE configs[1] ("cfg2"): B = 4096 random ALIP initial states per GPU, N = 3,
5 circular obstacles, fp64.  For N > 1 GPUs (torchrun, one process per GPU, RCCL) every rank solves its
own shard (instances are generated from (seed, global index), so every GPU count solves the same instances
with the same program) and each step ends with one RCCL gather of the
per-instance outputs to rank 0 — the path has no other exchange.
The other BASELINE configs are presets (not the driver's default line):
  cfg1  B = 1, N = 3, no obstacles, sig_step (the reference's own CPU-runnable case: single-solve latency)
  cfg3  B = 65,536 per GPU, N = 5, 5 circles + 5 ellipses, fp64 (weak scaling)
  cfg4  262,144 instances in total sharded over the GPUs, N = 3, 5 circles, fp64 (strong scaling)
  cfg5  1,048,576 randomized scenes in total (one obstacle field each), N = 3, fp32 solve kernels;
        also reports the feasible fraction (solutions re-evaluated by the fp64 reference callbacks, no
        active row violated by more than 1e-4; counts all-reduced over ranks)

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for the roofline / cpu_baseline fields).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))

# per-IP-iteration algorithmic work of one instance: KKT GEMM J^T Sigma J (2 m n^2) +
# Cholesky and two triangular solves (n^3/3 + 2 n^2) + NLP evaluation (rollout, f, grad, c, J)
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 matrix / vector peak (AMD spec; MI355X_MICROARCH.md lists no FP64 row)
FP32_PEAK_TFLOPS = 157.3     # MI355X FP32 matrix = vector peak (MI355X_MICROARCH.md)

# BASELINE.json configs: (instances, per_gpu?, horizon, circles, ellipses, precision, distinct fields).
# program: the device program (cfg.program, include/alipmpc.h) — "wave" (one instance per wavefront: the
# latency-bound small batches: cfg1, cfg2; cfg3, whose N = 5 ellipse shape the lane program does not cover), "lane"
# (one instance per lane: the 10^5+-instance configs cfg4 / cfg5).  A property of the config, never of the shard
# size: every GPU count runs the same program on the same instances, so the outputs do not depend on world size.
CONFIGS = {
    "cfg1": dict(batch=1, per_gpu=True, horizon=3, circles=0, ellipses=0, fp32=False, variant="sig_step",
                 program="wave"),
    "cfg2": dict(batch=4096, per_gpu=True, horizon=3, circles=5, ellipses=0, fp32=False, program="wave"),
    "cfg3": dict(batch=65536, per_gpu=True, horizon=5, circles=5, ellipses=5, fp32=False, program="wave"),
    "cfg4": dict(batch=262144, per_gpu=False, horizon=3, circles=5, ellipses=0, fp32=False, program="lane"),
    "cfg5": dict(batch=1048576, per_gpu=False, horizon=3, circles=5, ellipses=0, fp32=True, program="lane"),
}
HBM_PEAK_GBS = 8000.0
# scene blocks: instance g of a config's global batch is instance g % BLOCK of block g // BLOCK, generated from
# (seed * 1000 + g // BLOCK) — so a shard [lo, hi) holds the same instances whatever the world size (SURVEY 8e:
# scenes from (seed, global index)).  Per-GPU (weak-scaling) configs use blocks of the per-rank batch: rank r's shard
# is block r (the seed recipe of rounds 1-2, seed * 1000 + rank).
BLOCK = {"cfg4": 32768, "cfg5": 32768}


def flops_per_iter(n, m, N, nobs):
    kkt = 2 * m * n * n
    chol = n ** 3 / 3 + 2 * n * n
    nlp = 2 * (2 * N * 3 * n + N * nobs * 3 * n + N * 4 * n + N * 6 * n) + 50 * N
    return kkt + chol + nlp


def solve_rows(N, rps, modi):
    """Constraint rows of the solve layout (f_en split into two rows for modi)."""
    return N * (rps + (1 if modi else 0))


def scene_block(config, k, size, seed, n_cir, n_elp, N):
    """Block k of a config's global instance sequence (SURVEY 8d distribution; seed * 1000 + k)."""
    from alipmpc import scenes
    s = seed * 1000 + k
    if config == "cfg2":
        return scenes.make_batch(size, seed=s, n_cir=n_cir, N=N)
    # vectorised generator: one obstacle field per instance (cfg3: 4096 fields shared within a block)
    return scenes.make_batch_vec(size, seed=s, n_cir=n_cir, n_elp=n_elp, N=N, fields=4096 if config == "cfg3" else None)


def global_inputs(config, lo, hi, block, seed, n_cir, n_elp, N):
    """Instances [lo, hi) of the global batch: the blocks they overlap, generated from (seed, block index) and
    sliced, so the same global index always holds the same instance.  ALIPMPC_SCENE_CACHE=<dir> keeps the arrays
    between runs of one profiling session (tools/gpu_run.sh prof: cfg5 takes ~45 s to generate)."""
    cache = os.environ.get("ALIPMPC_SCENE_CACHE")
    if cache:
        fn = os.path.join(cache, f"{config}_{lo}_{hi}_{block}_{seed}_{n_cir}_{n_elp}_{N}.npz")
        if os.path.exists(fn):
            with np.load(fn) as z:
                return {k: z[k] for k in z.files}
    parts = []
    for k in range(lo // block, (hi - 1) // block + 1):
        bt = scene_block(config, k, block, seed, n_cir, n_elp, N)
        a, b = max(lo, k * block) - k * block, min(hi, (k + 1) * block) - k * block
        parts.append({key: v[a:b] for key, v in bt.items() if v is not None})
    out = {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}
    if cache:
        os.makedirs(cache, exist_ok=True)
        np.savez(fn, **out)
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (default: the config's)")
    ap.add_argument("--variant", default=None, choices=["modi", "sig_step"], help="default: the config's (modi)")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--obstacles", type=int, default=None, help="circles per instance")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="threads for the all-cores CPU baseline (the GPU box allots 16)")
    ap.add_argument("--sweep-batch", type=int, default=65536, help="instances for the Jacobian-sweep roofline")
    ap.add_argument("--program", default=None, choices=["wave", "lane"], help="default: the config's")
    ap.add_argument("--restoration", default="ipopt", choices=["ipopt", "substitute"],
                    help="cfg.restoration: IPOPT's restoration phase (default, the reference's) or the r1-r5 substitute")
    ap.add_argument("--closed-loop-steps", type=int, default=1,
                    help="walking steps of the per-tick closed-loop figure (f_cyc = 40 solves each; 0 = skip)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import alipmpc
    from alipmpc import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank if world > 1 else 0)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a visible MI355X (torch.cuda.is_available() is False)")

    preset = CONFIGS[args.config]
    args.variant = args.variant or preset.get("variant", "modi")
    variant = {"modi": alipmpc.VARIANT_MODI, "sig_step": alipmpc.VARIANT_SIG_STEP}[args.variant]
    N = args.horizon or preset["horizon"]
    n_cir = preset["circles"] if args.obstacles is None else args.obstacles
    n_elp = preset["ellipses"]
    fp32 = preset["fp32"]
    if args.batch is not None:
        B = args.batch
    elif preset["per_gpu"]:
        B = preset["batch"]
    else:   # a fixed total sharded over the ranks (contiguous shards, sizes differ by at most one)
        from alipmpc import sharding
        lo, hi = sharding.shard_range(preset["batch"], rank, world)
        B = hi - lo
    prec = {"precision": alipmpc.PREC_FP32} if fp32 else {}
    program = args.program or preset.get("program", "wave")
    prec["program"] = alipmpc.PROGRAM_LANE if program == "lane" else alipmpc.PROGRAM_WAVE
    prec["restoration"] = alipmpc.RESTORATION_SUBSTITUTE if args.restoration == "substitute" else alipmpc.RESTORATION_IPOPT
    cfg = alipmpc.default_cfg(variant, N, nc_max=n_cir, ne_max=n_elp, **prec)
    solver = alipmpc.Solver(cfg, device=dev.index)
    weak = preset["per_gpu"] or args.batch is not None
    if weak:     # rank r's shard = block r of the global sequence
        block, lo = B, rank * B
    else:
        block, lo = BLOCK[args.config], sharding_lo(preset["batch"], rank, world)
    batch = global_inputs(args.config, lo, lo + B, block, args.seed, n_cir, n_elp, N)
    n = solver.n
    inp = {
        "x0": torch.from_numpy(batch["x0"]).to(dev),
        "goal": torch.from_numpy(batch["goal"]).to(dev),
        "leg": torch.from_numpy(batch["leg"].astype(np.int8)).to(dev),
        "cir": torch.from_numpy(batch["cir"]).to(dev),
        "nc": torch.from_numpy(batch["nc"].astype(np.int32)).to(dev),
        "u0": torch.from_numpy(batch["u0"]).to(dev),
    }
    if n_elp:
        inp["elp"] = torch.from_numpy(batch["elp"]).to(dev)
        inp["ne"] = torch.from_numpy(batch["ne"].astype(np.int32)).to(dev)
    out = {
        "u": torch.empty((B, n), dtype=torch.float64, device=dev),
        "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
        "x_pred": torch.empty((B, N, 5), dtype=torch.float64, device=dev),
        "status": torch.empty((B,), dtype=torch.int32, device=dev),
        "iters": torch.empty((B,), dtype=torch.int32, device=dev),
    }
    # one gather of the per-instance outputs (u, foot, status, iters packed as fp64 rows) to rank 0 per
    # step: sharding.gather_to_root (the collective the gloo tests cover), padded to the largest shard
    stream = torch.cuda.current_stream(dev)
    solve = lambda: solver.solve_device(inp, out, stream=stream)  # noqa: E731
    step = make_step(solve, out, n, B_total_of(preset, args, B, world), rank, world, stream)
    elapsed, ev = timed_loop(step, args.warmup, args.steps, world, dev)
    K = args.steps
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    status = out["status"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    # lane program + IPOPT's restoration phase: instances whose line search failed are solved by the fp64 wave program
    try:
        handoffs = solver.lane_handoffs(stream) if program == "lane" else 0
    except (AttributeError, RuntimeError):
        handoffs = None
    B_total = B_total_of(preset, args, B, world)
    total_solves = B_total * K
    value = total_solves / elapsed
    # roofline of the dominant kernel (solve_kernel): algorithmic FP64 flops per launch / launch time
    try:
        slots = solver.solve_slots()
    except (AttributeError, RuntimeError):
        slots = None
    kname = solver.solve_program()
    try:
        launches, team = solver.solve_launches(B)
    except (AttributeError, RuntimeError):
        launches, team = 1, 1
    m = solve_rows(N, solver.rps, variant == alipmpc.VARIANT_MODI)
    fpi = flops_per_iter(n, m, N, n_cir + n_elp)
    # the lane program's KKT system is fp64 in both precisions; its bound is vector issue (FP64 VALU peak =
    # the FP64 matrix peak on MI355X); the wave program's KKT GEMM runs on MFMA in the solve precision
    peak = FP32_PEAK_TFLOPS if (fp32 and program == "wave") else FP64_PEAK_TFLOPS
    launch_flops = fpi * float(iters.sum())
    achieved = launch_flops / (kernel_ms * 1e-3) / 1e12
    # counter-derived fields of the dominant kernel from the committed rocprofv3 passes of this config
    # (tools/roofline.py writes profiles/solve_kernel_counters.json from profiles/r2/<config>/): HBM traffic and
    # the issue / MFMA shares that say which bound the kernel actually sits against
    bid = alipmpc.build_id()
    prof = counter_record(f"{kname}|B={B}", bid)
    traffic = prof.get("hbm_bytes_per_launch")

    # quality beside the rate (every config): solves/s counts every instance, so report how many of them
    # converged and how many returned plans are feasible for the reference constraints
    feas = feasible_fraction(alipmpc, solver, cfg, inp, out, dev, world, dist)

    # the wave program's binding resource is the per-iteration dependency chain of its slowest instances (MFMA busy
    # ~0.05, VALU issue ~0.5): the critical instance's iteration time alone on its SIMD, live, against the issue floor
    lat = latency_probe(solver, inp, out, iters, prof, dev) if (rank == 0 and program == "wave") else None
    sweep = jacobian_sweep(alipmpc, scenes, variant, args, dev) if (rank == 0 and args.sweep_batch > 0) else None
    cl = closed_loop_rate(solver, inp, out, args.closed_loop_steps, dev) \
        if (rank == 0 and args.closed_loop_steps > 0) else None

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, batch, args.cpu_seconds, workload=args.config)
        # the same C restatement with OpenMP over the host cores this job may use (batches that give
        # every thread at least one 64-instance chunk)
        if B >= 64 * args.cpu_threads:
            cpu_mt = cpu_baseline(cfg, batch, args.cpu_seconds / 2, threads=args.cpu_threads, workload=args.config)

    if rank == 0:
        line = {
            "metric": "MPC solves/sec (batched scenarios), N=3 horizon 5-obstacle, 1->8 MI355X",
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if preset["per_gpu"] or args.batch is not None else "strong",
            "vs_baseline": None,
            "dtype": "f32" if fp32 else "f64",
            "data": f"synthetic (rand_obs distribution, SURVEY 8d), instances generated from (seed, global index) in "
                    f"blocks of {block}",
            "config": {
                "workload": f"{args.config}: {B_total} ALIP initial states ({B} on rank 0), N={N} horizon, "
                            f"{n_cir} circles + {n_elp} ellipses, variant={args.variant}, "
                            f"{'fp32' if fp32 else 'fp64'}, interior point (tol {cfg.tol:g}, max_iter {cfg.max_iter} "
                            f"= the reference's IPOPT cap)",
                "batch_per_gpu": B, "global_batch": B_total, "horizon": N, "obstacles": n_cir + n_elp,
                "variant": args.variant, "parallelism": f"shard{world}" if world > 1 else "single",
                "restoration": "ipopt" if cfg.restoration == alipmpc.RESTORATION_IPOPT else "substitute",
                "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
                "resident_slots": slots,
                "program": program,
                "launch": ("persistent work queue, one instance per lane" +
                           (f"; {handoffs} instances with a failed line search handed to the fp64 wave program's "
                            f"restoration-capable work queue (IPOPT's restoration phase)" if handoffs else "")
                           if program == "lane" else
                           ("split launch: phase 1 one wavefront per instance up to the iteration cut, phase 2 "
                            "resumes the unfinished instances" + (" (trial-cut ones on 4-wave teams)" if team > 1 else
                                                                  " one wavefront each"))
                           if launches == 2 else
                           "one wavefront per instance (B <= resident slots, no queue)" if slots and B <= slots else
                           "persistent work queue, one instance per wavefront"),
                "launches_per_solve": launches + (1 if handoffs else 0),
                "lane_handoffs": handoffs if program == "lane" else None,
                "build_id": bid,
            },
            "roofline": {
                "kernel": kname,
                # the binding resource from the counters of this build: MFMA busy (wave program ~0.05, never the bound),
                # vector issue (>= half of the SIMD issue slots: cfg3's queue of 65,536 instances, the lane program) or
                # else the latency chain of the slowest instances (cfg2, cfg1; see "latency")
                "bound": bound_label(program, prof),
                "latency": lat,
                "achieved": achieved,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                # fp32 configs: both fractions (the lane program's fp32 build keeps its KKT system in fp64)
                "frac_fp64_peak": achieved / FP64_PEAK_TFLOPS if fp32 else None,
                "frac_fp32_peak": achieved / FP32_PEAK_TFLOPS if fp32 else None,
                "traffic": traffic,
                "valu_issue_frac": prof.get("valu_issue_frac"),
                "active_issue_frac": prof.get("active_issue_frac"),
                "mfma_busy_share": prof.get("mfma_busy_share"),
                "insts_per_iter": prof.get("insts_per_iter"),
                "counters": ("profiles/solve_kernel_counters.json (tools/roofline.py), build " + bid) if prof else None,
                "kernel_ms": kernel_ms,
                "flops_per_iter": fpi,
                "iters_per_launch": int(iters.sum()),
            },
            "cpu_baseline": cpu,
            "cpu_baseline_allcores": cpu_mt,
            "jacobian_sweep": sweep,
            "closed_loop": cl,
            "feasible": feas,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def sharding_lo(total, rank, world):
    from alipmpc import sharding
    return sharding.shard_range(total, rank, world)[0]


def B_total_of(preset, args, B, world):
    """Instances in the whole job: per-GPU configs (weak scaling) B x world; fixed totals (strong) the
    config's batch."""
    return B * world if (preset["per_gpu"] or args.batch is not None) else preset["batch"]


def pack_outputs(out, n):
    """Per-instance outputs as fp64 rows [u (n) | foot (3) | status | iters] (the gathered record)."""
    import torch
    return torch.cat([out["u"].reshape(-1, n), out["foot"], out["status"].to(torch.float64).reshape(-1, 1),
                      out["iters"].to(torch.float64).reshape(-1, 1)], dim=1)


def make_step(solve, out, n, B_total, rank, world, stream=None):
    """One bench step: the solve launch (bracketed by the given HIP event pair, recorded on the launch
    stream), then at N > 1 one gather of the packed outputs to rank 0 with alipmpc.sharding.gather_to_root
    (contiguous shards of B_total, padded to the largest).  step(ev) returns the gathered
    [B_total, n + 5] tensor on rank 0 (None on the other ranks and at N = 1)."""
    from alipmpc import sharding

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        solve()
        if ev is not None:
            ev[1].record(stream)
        if world == 1:
            return None
        return sharding.gather_to_root(pack_outputs(out, n), B_total, rank, world)
    return step


def timed_loop(step, warmup, K, world, dev):
    """W untimed steps, then K timed steps bracketed by barrier + synchronize on both sides; returns the
    max-over-ranks wall time and the per-launch HIP event pairs (none on a CPU device: the gloo tests
    drive this loop with a stub solver)."""
    import torch
    import torch.distributed as dist
    gpu = torch.device(dev).type == "cuda"
    sync = (lambda: torch.cuda.synchronize(dev)) if gpu else (lambda: None)  # noqa: E731
    for _ in range(warmup):
        step()
    sync()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if gpu else None
          for _ in range(K)]
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(K):
        step(ev[k])
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, ev


def counter_record(key, bid):
    """The committed rocprofv3 counter record of kernel|B (profiles/solve_kernel_counters.json, tools/roofline.py) —
    only when it was measured on this very build (same alipmpc_build_id); otherwise none, never a stale one."""
    tp = os.path.join(ROOT, "profiles", "solve_kernel_counters.json")
    try:
        with open(tp) as fh:
            rec = json.load(fh).get(key, {})
    except (OSError, ValueError):
        return {}
    return rec if rec.get("build_id") == bid else {}


CLOCK_GHZ = 2.4   # MI355X max engine clock (MI355X_MICROARCH.md); cycle figures below are at this clock
ISSUE_CYC = 4     # one wave alone issues at most one instruction per 4 cycles (MI355X_MICROARCH.md: s_nop / v_fma 4)


def bound_label(program, prof):
    """Roofline bound of the solve kernel: "mfma" when the matrix cores are busy >= half the SIMD cycles, "valu" when
    vector issue takes >= half the issue slots (and, without counters, for the lane program, whose fp64 KKT algebra runs
    on the vector ALUs), else "latency" (the wave program's dependency chains)."""
    mfma, valu = prof.get("mfma_busy_share"), prof.get("valu_issue_frac")
    if mfma is not None and mfma >= 0.5:
        return "mfma"
    if (valu is not None and valu >= 0.5) or (valu is None and program == "lane"):
        return "valu"
    return "latency"


def latency_probe(solver, inp, out, iters, prof, dev, copies=64, reps=5):
    """The critical instance's interior-point iteration time with its SIMD to itself: the batch's instance with the
    most iterations, solved as `copies` identical instances (one wave each, one per SIMD), mean launch time over reps
    launches / its iterations -> cycles per iteration at CLOCK_GHZ.  Against the instruction-issue floor of one wave
    (insts_per_iter x ISSUE_CYC, from the build's committed counter record): frac = floor / measured."""
    import torch
    b = int(np.argmax(iters))
    sub = {k: v[b:b + 1].repeat((copies,) + (1,) * (v.dim() - 1)).contiguous() for k, v in inp.items()}
    o = {k: torch.empty((copies,) + tuple(v.shape[1:]), dtype=v.dtype, device=dev) for k, v in out.items()}
    st = torch.cuda.current_stream(dev)
    ms = []
    for r in range(reps + 2):
        solver.solve_device(sub, o, stream=st)
        torch.cuda.synchronize(dev)
        if r >= 2:
            ms.append(solver.last_kernel_ms())
    it = int(o["iters"][0].item())
    cyc = float(np.mean(ms)) * 1e-3 * CLOCK_GHZ * 1e9 / max(it, 1)
    ipi = prof.get("insts_per_iter")
    floor = ipi * ISSUE_CYC if ipi else None
    return {"instance_iters": it, "launch_ms": float(np.mean(ms)), "cycles_per_iter": cyc, "clock_ghz": CLOCK_GHZ,
            "issue_floor_cycles": floor, "frac": (floor / cyc) if floor else None,
            "note": "critical instance alone on its SIMD; floor = counter insts_per_iter x 4 cycles (one wave's issue)"}


def jacobian_sweep(alipmpc, scenes, variant, args, dev, reps=20):
    """HBM roofline of the unfused Jacobian sweep (the eval hook: f, grad f, c, J of the reference
    callbacks at given u; sweep_kernel at N = 3 with circle slots) on cfg2-shaped instances (N = 3, 5 circles)
    whatever --config is.
    Algorithmic bytes per instance = 8(n + 8 + 3 n_c + 5 n_e) read + 8(1 + n + m + m n) written (n = 5N,
    m = padded rows)."""
    import torch
    cfg = alipmpc.default_cfg(variant, 3, nc_max=5, ne_max=0)
    Bs = args.sweep_batch
    s = alipmpc.Solver(cfg, device=dev.index)
    bt = scenes.make_batch_vec(Bs, seed=args.seed * 1000 + 7, n_cir=cfg.nc_max, N=cfg.N, fields=4096)
    n, m = 5 * cfg.N, cfg.N * s.rps
    inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
           "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(bt["cir"]).to(dev),
           "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev), "u": torch.from_numpy(bt["u0"]).to(dev)}
    out = {"f": torch.empty(Bs, dtype=torch.float64, device=dev),
           "grad": torch.empty((Bs, n), dtype=torch.float64, device=dev),
           "c": torch.empty((Bs, m), dtype=torch.float64, device=dev),
           "J": torch.empty((Bs, m, n), dtype=torch.float64, device=dev)}
    st = torch.cuda.current_stream(dev)
    for _ in range(2):
        s.eval_device(inp, out, stream=st)
    # back-to-back launches (no host sync, no event in between) between one HIP event pair on the launch stream:
    # mean launch duration = elapsed / reps.  An event pair around every launch adds the dispatch gap of a 65 us
    # kernel (profiles/r2/sweep: rocprofv3 trace 0.0649 ms/launch vs 0.076 ms per-launch events)
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the host enqueues all launches while the stream is held by a spin kernel (one Python + C-ABI call takes about
    # as long as one 65 us launch: without the hold, the GPU would wait on the host between launches)
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(2e7))
    a.record(st)
    for _ in range(reps):
        s.eval_device(inp, out, stream=st)
    b.record(st)
    torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / reps
    per = 8 * (n + 8 + 3 * cfg.nc_max) + 8 * (1 + n + m + m * n)
    gbs = Bs * per / (ms * 1e-3) / 1e9
    # the eval hook at N = 3 (32 instances per wave, 2 waves per workgroup)
    kern = f"sweep_kernel<{cfg.nc_max},{'true' if variant == alipmpc.VARIANT_MODI else 'false'},32,2>"
    # HBM traffic per launch from the committed PMC passes of the same kernel and batch (tools/roofline.py --sweep)
    traffic = counter_record(f"{kern}|B={Bs}", alipmpc.build_id()).get("hbm_bytes_per_launch")
    return {"kernel": kern, "bound": "hbm", "batch": Bs, "bytes_per_instance": per,
            "kernel_ms": ms, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "traffic": traffic, "evals_per_s": Bs / (ms * 1e-3)}


def closed_loop_rate(solver, inp, out, steps, dev, f_cyc=40):
    """the reference driver's receding horizon at its control rate (alipmpc_closed_loop_batch:
    f_cyc solves per walking step, each one tick closer to touchdown, warm-started from the previous plan) on
    this rank's episodes.  Start: the bench instances' x0 with the stance on the first foothold the timed solve
    planned (the consistent touchdown pair).  Rate = episode-ticks solved / (HIP-event time of the whole loop
    on the launch stream: the per-tick projection, solve and update launches)."""
    import torch
    B = inp["x0"].shape[0]
    st = torch.cuda.current_stream(dev)
    cin = {"x0": inp["x0"], "foot0": out["foot"][:, 0:2].contiguous(), "goal": inp["goal"], "leg": inp["leg"],
           "cir": inp["cir"], "nc": inp["nc"]}
    if "elp" in inp:
        cin["elp"], cin["ne"] = inp["elp"], inp["ne"]
    co = {"status": torch.empty((B, steps, f_cyc), dtype=torch.int32, device=dev),
          "iters": torch.empty((B, steps, f_cyc), dtype=torch.int32, device=dev),
          "steps_to_goal": torch.empty((B,), dtype=torch.int32, device=dev)}
    solver.closed_loop_device(cin, co, steps, f_cyc=f_cyc, stream=st)
    torch.cuda.synchronize(dev)
    solver.closed_loop_device(cin, co, steps, f_cyc=f_cyc, stream=st)
    torch.cuda.synchronize(dev)
    ms = solver.last_kernel_ms()
    status = co["status"].cpu().numpy()
    ran = status != -10
    ticks = int(ran.sum())
    return {"episodes": B, "steps": steps, "f_cyc": f_cyc, "ticks": ticks, "ms": ms,
            "solves_per_s": ticks / (ms * 1e-3), "mean_iters": float(co["iters"].cpu().numpy()[ran].mean()),
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status[ran], return_counts=True))},
            "program": solver.solve_program()}


def feasible_fraction(alipmpc, solver, cfg, inp, out, dev, world, dist, chunk=65536):
    """Share of instances whose returned u, evaluated by the fp64 eval kernel (the reference callbacks),
    violates no active constraint row by more than 1e-4 (the reference analogue is status != 2,
    86.6 % in its logs), and the shares with status 0 or 1 / status 0.  Counts are summed over ranks."""
    import torch
    c64 = alipmpc.default_cfg(cfg.variant, cfg.N, nc_max=cfg.nc_max, ne_max=cfg.ne_max)
    ev = alipmpc.Solver(c64, device=dev.index)
    B = inp["x0"].shape[0]
    m = ev.m_max
    feas = 0
    for i0 in range(0, B, chunk):
        i1 = min(B, i0 + chunk)
        sub = {k: v[i0:i1] for k, v in inp.items() if k != "u0"}
        sub["u"] = out["u"][i0:i1]
        o = {"c": torch.empty((i1 - i0, m), dtype=torch.float64, device=dev),
             "cl": torch.empty((i1 - i0, m), dtype=torch.float64, device=dev),
             "cu": torch.empty((i1 - i0, m), dtype=torch.float64, device=dev),
             "row_active": torch.empty((i1 - i0, m), dtype=torch.int8, device=dev)}
        ev.eval_device(sub, o)
        v = torch.clamp(torch.maximum(o["cl"] - o["c"], o["c"] - o["cu"]), min=0.0)
        v = torch.where(o["row_active"] != 0, v, torch.zeros_like(v))
        feas += int((v.amax(dim=1) <= 1e-4).sum().item())
    return quality_counts(feas, out["status"], dev, world)


def quality_counts(feas, status, dev, world):
    """Feasible / converged (status 0 or 1) / solved (status 0) shares over the whole job: per-rank counts
    summed with one all-reduce."""
    import torch
    import torch.distributed as dist
    conv = int(((status == 0) | (status == 1)).sum().item())
    solved = int((status == 0).sum().item())
    cnt = torch.tensor([feas, conv, solved, status.numel()], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(cnt)
    feas, conv, solved, tot = (float(x) for x in cnt.tolist())
    return {"feasible_fraction": feas / tot, "converged_fraction": conv / tot, "solved_fraction": solved / tot,
            "instances": int(tot),
            "check": "fp64 reference callbacks at the returned u, max active-row violation <= 1e-4"}


def cpu_baseline(cfg, batch, seconds, threads=1, workload="cfg2"):
    """C restatement (oracle/liboracle.so) of the same algorithm (fp64), bounded sample of the same
    workload, timed on this host (1 thread, or OpenMP over `threads`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as C
    co = C.default_cfg(cfg.variant, cfg.N, nc_max=cfg.nc_max, ne_max=cfg.ne_max)
    co.restoration = cfg.restoration
    B = batch["x0"].shape[0]
    ne_max = cfg.ne_max
    elp = batch["elp"] if ne_max else None
    ne = batch["ne"] if ne_max else None
    done = 0
    t0 = time.perf_counter()
    chunk = 64 * threads
    while time.perf_counter() - t0 < seconds:
        i0 = done % B
        i1 = min(i0 + chunk, B)
        C.solve_batch(co, batch["x0"][i0:i1], batch["goal"][i0:i1], batch["leg"][i0:i1], batch["cir"][i0:i1],
                      batch["nc"][i0:i1], elp[i0:i1] if ne_max else np.zeros((i1 - i0, 0, 5)),
                      ne[i0:i1] if ne_max else np.zeros(i1 - i0), batch["u0"][i0:i1],
                      nthreads=threads)
        done += i1 - i0
    dt = time.perf_counter() - t0
    prec = " (fp64: the GPU line runs fp32)" if cfg.precision == 1 else ""
    return {"value": done / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{done} instances of the {workload} workload (first {min(done, B)} of the GPU batch, cycled), "
                      f"C oracle oracle/alipmpc_oracle.c, same interior-point algorithm{prec}, {threads} thread(s), "
                      f"{dt:.1f} s"}


if __name__ == "__main__":
    main()
