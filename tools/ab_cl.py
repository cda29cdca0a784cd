"""Dev A/B: cold cfg2 solve launch time AND the closed loop's per-tick rate (one walking step, f_cyc = 40) of several
library builds on the same box, one process each, with a hash of every output (variants that must not change the
arithmetic print the same hashes).
  python tools/ab_cl.py devlib/libA.so devlib/libB.so ...   [env AB_B=4096 AB_REPS=30 AB_N=3 AB_NE=0]"""
import hashlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(spec):
    # spec = path[:NAME=VALUE,...]: the library and environment settings of one variant
    lib, _, env = spec.partition(":")
    for kv in filter(None, env.split(",")):
        k, _, v = kv.partition("=")
        os.environ[k] = v
    os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, lib)
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    sys.path.insert(0, ROOT)
    import torch
    import alipmpc
    import bench
    B, reps = int(os.environ.get("AB_B", "4096")), int(os.environ.get("AB_REPS", "30"))
    N, ne = int(os.environ.get("AB_N", "3")), int(os.environ.get("AB_NE", "0"))
    cfgname = "cfg2" if (N == 3 and ne == 0) else "cfg3"
    bt = bench.global_inputs(cfgname, 0, B, B, 0, 5, ne, N)
    s = alipmpc.Solver(alipmpc.default_cfg(0, N, nc_max=5, ne_max=ne))
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    if "ne" in inp:
        inp["ne"] = inp["ne"].to(torch.int32)
    out = {"u": torch.empty((B, 5 * N), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "x_pred": torch.empty((B, N, 5), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev), "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    st = torch.cuda.current_stream()
    ms = []
    for _ in range(reps + 3):
        s.solve_device(inp, out, stream=st)
        ms.append(s.last_kernel_ms())
    ms = np.array(ms[3:])
    h = hashlib.md5(b"".join(out[k].cpu().numpy().tobytes() for k in ("u", "status", "iters"))).hexdigest()[:10]
    line = f"{spec}: cold median {np.median(ms):.4f} ms min {ms.min():.4f} iters {out['iters'].float().mean().item():.3f} [{h}]"
    if os.environ.get("AB_CL", "1") == "1":
        cin = {"x0": inp["x0"], "foot0": out["foot"][:, 0:2].contiguous(), "goal": inp["goal"], "leg": inp["leg"],
               "cir": inp["cir"], "nc": inp["nc"]}
        if "elp" in inp:
            cin["elp"], cin["ne"] = inp["elp"], inp["ne"]
        F = 40
        co = {"status": torch.empty((B, 1, F), dtype=torch.int32, device=dev),
              "iters": torch.empty((B, 1, F), dtype=torch.int32, device=dev),
              "foot": torch.empty((B, 1, 3), dtype=torch.float64, device=dev)}
        cms = []
        for _ in range(3):
            s.closed_loop_device(cin, co, 1, f_cyc=F, stream=st)
            cms.append(s.last_kernel_ms())
        hc = hashlib.md5(b"".join(co[k].cpu().numpy().tobytes() for k in ("status", "iters", "foot"))).hexdigest()[:10]
        cl = min(cms[1:])
        line += f" | closed loop {cl:.2f} ms = {cl / F:.3f} ms/tick, {B * F / cl * 1e3 / 1e6:.2f} M tick-solves/s [{hc}]"
    print(line, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one(sys.argv[2])
    else:
        for rnd in range(2):
            for lib in sys.argv[1:]:
                subprocess.check_call([sys.executable, __file__, "--one", lib], timeout=300)
