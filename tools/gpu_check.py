"""Dev script: quick GPU-vs-oracle comparison (run on the GPU box via gpurun)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import alipmpc
from alipmpc import scenes
import oracle as C

def main():
    alipmpc.load()
    # eval parity on the callback goldens
    for name, var in [("modi", 0), ("sig_step", 1)]:
        g = np.load(os.path.join(ROOT, f"tests/golden/g1_callbacks_{name}.npz"))
        cfg = alipmpc.default_cfg(var, select_obs=0, detour=0)
        s = alipmpc.Solver(cfg)
        B = len(g["f"])
        o = s.eval(g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
        ef = np.max(np.abs(o["f"] - g["f"]) / (1 + np.abs(g["f"])))
        eg = np.max(np.abs(o["grad"] - g["grad"]) / (1 + np.abs(g["grad"])))
        ec = eJ = 0
        for t in range(B):
            act = o["row_active"][t].astype(bool); m = g["m"][t]
            assert act.sum() == m, (t, act.sum(), m)
            ec = max(ec, np.max(np.abs(o["c"][t][act] - g["c"][t][:m])))
            eJ = max(eJ, np.max(np.abs(o["J"][t][act] - g["J"][t][:m])))
        print(f"eval {name}: f {ef:.2e} grad {eg:.2e} c {ec:.2e} J {eJ:.2e}", flush=True)
    # solve parity on sup_learn rows
    d = np.load(os.path.join(ROOT, "tests/golden/g3_sup_learn.npz"))
    B = len(d["leg"])
    cfg = alipmpc.default_cfg(0, nc_max=6, ne_max=0)
    s = alipmpc.Solver(cfg)
    cir = np.tile(d["cir_safe"], (B, 1, 1))
    t0 = time.time()
    o = s.solve(d["x_nex"], [10, 10], d["leg"], cir, np.full(B, 6), u0=d["u0"])
    print(f"gpu solve sup_learn B={B}: {time.time()-t0:.3f}s kernel {s.last_kernel_ms():.3f} ms", flush=True)
    co = C.default_cfg(0, nc_max=6, ne_max=0)
    r = C.solve_batch(co, d["x_nex"], [10, 10], d["leg"], cir, np.full(B, 6), np.zeros((B, 0, 5)), np.zeros(B), d["u0"], nthreads=8)
    ok = d["ok_ref"].astype(bool)
    eg = np.max(np.abs(o["foot"][:, :2] - d["foot_logged"]), axis=1)
    eo = np.max(np.abs(o["foot"] - r["foot"]), axis=1)
    print("gpu status", np.unique(o["status"], return_counts=True), "iters mean", o["iters"].mean())
    print("oracle status", np.unique(r["status"], return_counts=True), "iters mean", r["iters"].mean())
    print(f"gpu vs logged on ok rows: {(eg[ok] < 1e-4).sum()}/{ok.sum()}  ; gpu vs oracle foot <1e-6: {(eo < 1e-6).sum()}/{B}, same status {(o['status']==r['status']).sum()}")
    both0 = (o["status"] == 0) & (r["status"] == 0)
    print(f"  both converged {both0.sum()}, max foot diff there {eo[both0].max():.2e}, frac <1e-6 {(eo[both0]<1e-6).mean():.4f}")
    # synthetic batch timing
    for B in [4096, 16384]:
        bt = scenes.make_batch(B, seed=0, n_cir=5)
        cfg = alipmpc.default_cfg(0, nc_max=5, ne_max=0)
        s = alipmpc.Solver(cfg)
        for rep in range(3):
            o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
            print(f"B={B} kernel {s.last_kernel_ms():.3f} ms -> {B/s.last_kernel_ms()*1e3:.3e} solves/s; status {np.unique(o['status'], return_counts=True)} iters {o['iters'].mean():.1f}", flush=True)
    bt = scenes.make_batch(1024, seed=0, n_cir=5)
    co = C.default_cfg(0, nc_max=5, ne_max=0)
    r = C.solve_batch(co, bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], np.zeros((1024, 0, 5)), np.zeros(1024), bt["u0"], nthreads=8)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    eo = np.max(np.abs(o["foot"] - r["foot"]), axis=1)
    both0 = (o["status"] == 0) & (r["status"] == 0)
    print(f"synthetic 1024: gpu vs oracle <1e-6 {(eo<1e-6).sum()}, both conv {both0.sum()}, frac<1e-6 there {(eo[both0]<1e-6).mean():.4f}")

if __name__ == "__main__":
    main()
