"""Dev A/B: cfg2-shaped solve launch time of several library builds on the same box (one process each).
  python tools/ab_solve.py path/to/libA.so path/to/libB.so ...  [env AB_B=4096 AB_REPS=30]"""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--one":
    os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, sys.argv[2])
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    import torch
    import alipmpc
    from alipmpc import scenes
    B, reps = int(os.environ.get("AB_B", "4096")), int(os.environ.get("AB_REPS", "30"))
    s = alipmpc.Solver(alipmpc.default_cfg(0, nc_max=5, ne_max=0, restoration=int(os.environ.get("AB_REST", "0"))))
    bt = scenes.make_batch(B, seed=0, n_cir=5)
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev), "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev), "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    st = torch.cuda.current_stream()
    ms = []
    for r in range(reps + 3):
        s.solve_device(inp, out, stream=st)
        ms.append(s.last_kernel_ms())
    ms = np.array(ms[3:])
    import hashlib
    hsh = hashlib.md5(out["u"].cpu().numpy().tobytes() + out["status"].cpu().numpy().tobytes() +
                      out["iters"].cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"{sys.argv[2]}: median {np.median(ms):.4f} ms  min {ms.min():.4f}  iters {out['iters'].float().mean().item():.3f}"
          f"  outputs {hsh}", flush=True)
else:
    for rnd in range(2):
        for lib in sys.argv[1:]:
            subprocess.check_call([sys.executable, __file__, "--one", lib])
