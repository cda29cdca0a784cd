#!/usr/bin/env python3
"""Benchmark: batched ALIP-MPC-CBF solves/sec on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--variant modi] [--horizon 3]

One "step" = one fused interior-point solve of a batch of B independent NLP instances whose inputs are
already resident in HBM (one launch of solve_kernel through the C ABI on the current HIP stream).
Default workload = BASELINE configs[1] ("cfg2"): B = 4096 random ALIP initial states per GPU, N = 3,
5 circular obstacles, fp64.  For N > 1 GPUs (torchrun, one process per GPU, RCCL) every rank solves its
own 4096-instance shard (weak scaling; scenes are generated from (seed, rank)) and each step ends with
one RCCL gather of the per-instance outputs to rank 0 — the path has no other exchange.

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
HBM_PEAK_GBS = 8000.0


def flops_per_iter(n, m, N, nobs):
    kkt = 2 * m * n * n
    chol = n ** 3 / 3 + 2 * n * n
    nlp = 2 * (2 * N * 3 * n + N * nobs * 3 * n + N * 4 * n + N * 6 * n) + 50 * N
    return kkt + chol + nlp


def solve_kernel_name(N, rps, modi):
    """The solve_kernel<N, KSM> instance the library dispatches (csrc/alipmpc.hip: ksm_of): constraint rows
    in the solve layout (f_en split into two rows for modi) + N objective rows, in 4-row J-layout steps."""
    m = N * (rps + (1 if modi else 0))
    rows = ((m + 3) // 4) * 4 + 4 * ((N + 3) // 4)
    ksm = next(k for k in (8, 10, 12, 16, 24, 32, 48) if rows <= 4 * k)
    return f"solve_kernel<{N},{ksm}>", m


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--variant", default="modi", choices=["modi", "sig_step"])
    ap.add_argument("--horizon", type=int, default=3)
    ap.add_argument("--obstacles", type=int, default=5)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="threads for the all-cores CPU baseline (the GPU box allots 16)")
    ap.add_argument("--sweep-batch", type=int, default=65536, help="instances for the Jacobian-sweep roofline")
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

    variant = {"modi": alipmpc.VARIANT_MODI, "sig_step": alipmpc.VARIANT_SIG_STEP}[args.variant]
    N = args.horizon
    cfg = alipmpc.default_cfg(variant, N, nc_max=args.obstacles, ne_max=0)
    solver = alipmpc.Solver(cfg, device=dev.index)
    B = args.batch
    batch = scenes.make_batch(B, seed=args.seed * 1000 + rank, n_cir=args.obstacles, N=N)
    n = solver.n
    inp = {
        "x0": torch.from_numpy(batch["x0"]).to(dev),
        "goal": torch.from_numpy(batch["goal"]).to(dev),
        "leg": torch.from_numpy(batch["leg"].astype(np.int8)).to(dev),
        "cir": torch.from_numpy(batch["cir"]).to(dev),
        "nc": torch.from_numpy(batch["nc"].astype(np.int32)).to(dev),
        "u0": torch.from_numpy(batch["u0"]).to(dev),
    }
    out = {
        "u": torch.empty((B, n), dtype=torch.float64, device=dev),
        "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
        "x_pred": torch.empty((B, N, 5), dtype=torch.float64, device=dev),
        "status": torch.empty((B,), dtype=torch.int32, device=dev),
        "iters": torch.empty((B,), dtype=torch.int32, device=dev),
    }
    # one gather of per-instance outputs (u, foot, status, iters packed as fp64 rows) to rank 0
    pack_w = n + 3 + 2
    packed = torch.empty((B, pack_w), dtype=torch.float64, device=dev)
    gathered = [torch.empty_like(packed) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream(dev)

    def step():
        solver.solve_device(inp, out, stream=stream)
        if world > 1:
            packed[:, :n] = out["u"]
            packed[:, n:n + 3] = out["foot"]
            packed[:, n + 3] = out["status"].to(torch.float64)
            packed[:, n + 4] = out["iters"].to(torch.float64)
            dist.gather(packed, gathered, dst=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        ev[k][0].record(stream)
        solver.solve_device(inp, out, stream=stream)
        ev[k][1].record(stream)
        if world > 1:
            packed[:, :n] = out["u"]
            packed[:, n:n + 3] = out["foot"]
            packed[:, n + 3] = out["status"].to(torch.float64)
            packed[:, n + 4] = out["iters"].to(torch.float64)
            dist.gather(packed, gathered, dst=0)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    status = out["status"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    total_solves = world * B * K
    value = total_solves / elapsed
    # roofline of the dominant kernel (solve_kernel): algorithmic FP64 flops per launch / launch time
    kname, m = solve_kernel_name(N, solver.rps, variant == alipmpc.VARIANT_MODI)
    fpi = flops_per_iter(n, m, N, args.obstacles)
    launch_flops = fpi * float(iters.sum())
    achieved = launch_flops / (kernel_ms * 1e-3) / 1e12
    traffic = None
    tp = os.path.join(ROOT, "profiles", "solve_kernel_traffic.json")
    if os.path.exists(tp):
        try:
            with open(tp) as fh:
                tj = json.load(fh)
            if tj.get("B") == B and tj.get("N") == N:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    sweep = jacobian_sweep(alipmpc, scenes, cfg, args, dev) if (rank == 0 and args.sweep_batch > 0) else None

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, batch, args.cpu_seconds)
        # the same C restatement with OpenMP over the host cores this job may use
        cpu_mt = cpu_baseline(cfg, batch, args.cpu_seconds / 2, threads=args.cpu_threads)

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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (rand_obs distribution, SURVEY 8d), generated per rank from (seed, rank)",
            "config": {
                "workload": f"cfg2: B={B} ALIP initial states per GPU, N={N} horizon, {args.obstacles} circles, "
                            f"variant={args.variant}, fp64, interior point (tol 1e-8, max_iter {cfg.max_iter} = the "
                            f"reference's IPOPT cap)",
                "batch_per_gpu": B, "global_batch": B * world, "horizon": N, "obstacles": args.obstacles,
                "variant": args.variant, "parallelism": f"shard{world}" if world > 1 else "single",
                "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
            },
            "roofline": {
                "kernel": kname,
                "bound": "mfma",
                "achieved": achieved,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "kernel_ms": kernel_ms,
                "flops_per_iter": fpi,
                "iters_per_launch": int(iters.sum()),
            },
            "cpu_baseline": cpu,
            "cpu_baseline_allcores": cpu_mt,
            "jacobian_sweep": sweep,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def jacobian_sweep(alipmpc, scenes, cfg, args, dev, reps=10):
    """HBM roofline of the unfused Jacobian sweep (eval_kernel: f, grad f, c, J of the
    reference callbacks at given u).  Algorithmic bytes per instance = 8(n + 8 + 3 n_c + 5 n_e) read +
    8(1 + n + m + m n) written (n = 5N, m = padded rows)."""
    import torch
    Bs = args.sweep_batch
    s = alipmpc.Solver(cfg, device=dev.index)
    bt = scenes.make_batch(Bs, seed=args.seed * 1000 + 7, n_cir=cfg.nc_max, N=cfg.N, scenes_per_batch=4096)
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
    # back-to-back launches (no host sync in between) so the launch latency overlaps the previous kernel;
    # per-launch HIP events on the launch stream
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(st)
        s.eval_device(inp, out, stream=st)
        b.record(st)
    torch.cuda.synchronize(dev)
    ms = float(np.mean([a.elapsed_time(b) for a, b in evs[1:]]))
    per = 8 * (n + 8 + 3 * cfg.nc_max) + 8 * (1 + n + m + m * n)
    gbs = Bs * per / (ms * 1e-3) / 1e9
    return {"kernel": f"eval_kernel<{cfg.N}>", "bound": "hbm", "batch": Bs, "bytes_per_instance": per,
            "kernel_ms": ms, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "evals_per_s": Bs / (ms * 1e-3)}


def cpu_baseline(cfg, batch, seconds, threads=1):
    """C restatement (oracle/liboracle.so) of the same algorithm, bounded sample of the same workload,
    timed on this host (1 thread, or OpenMP over `threads`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as C
    co = C.default_cfg(cfg.variant, cfg.N, nc_max=cfg.nc_max, ne_max=0)
    B = batch["x0"].shape[0]
    done = 0
    t0 = time.perf_counter()
    chunk = 64 * threads
    while time.perf_counter() - t0 < seconds:
        i0 = done % B
        i1 = min(i0 + chunk, B)
        C.solve_batch(co, batch["x0"][i0:i1], batch["goal"][i0:i1], batch["leg"][i0:i1], batch["cir"][i0:i1],
                      batch["nc"][i0:i1], np.zeros((i1 - i0, 0, 5)), np.zeros(i1 - i0), batch["u0"][i0:i1],
                      nthreads=threads)
        done += i1 - i0
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{done} instances of the cfg2 workload (first {min(done, B)} of the GPU batch, cycled), "
                      f"C oracle oracle/alipmpc_oracle.c, same interior-point algorithm, {threads} thread(s), "
                      f"{dt:.1f} s"}


if __name__ == "__main__":
    main()
