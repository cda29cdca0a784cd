"""Dev: outputs of the two launch forms (work queue: B > slots; one wave per instance: chunks) per library build, as
hashes (fp32 cfg5 shape by default), to see which form a change altered."""
import hashlib, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--one":
    lib, prec = sys.argv[2], int(sys.argv[3])
    os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, lib)
    os.environ["ALIPMPC_SPLIT_IT"] = "0"
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    import alipmpc
    from alipmpc import scenes
    kw = dict(nc_max=5, ne_max=0)
    if prec:
        kw["precision"] = alipmpc.PREC_FP32
    s = alipmpc.Solver(alipmpc.default_cfg(0, 3, **kw))
    slots = s.solve_slots()
    B = slots + slots // 2 + 5
    bt = scenes.make_batch_vec(B, seed=600 + prec, n_cir=5, N=3)
    args = lambda i, j: (bt["x0"][i:j], bt["goal"][i:j], bt["leg"][i:j], bt["cir"][i:j], bt["nc"][i:j])  # noqa
    big = s.solve(*args(0, B), u0=bt["u0"])
    ch = slots // 2
    parts = [s.solve(*args(i, i + ch), u0=bt["u0"][i:i + ch]) for i in range(0, B, ch)]
    small = {k: np.concatenate([p[k] for p in parts]) for k in big}
    h = lambda o: hashlib.md5(b"".join(o[k].tobytes() for k in ("u", "status", "iters"))).hexdigest()[:10]  # noqa
    d = np.any(big["u"] != small["u"], axis=1)
    print(f"{lib} prec {prec}: queue form {h(big)}  one-wave form {h(small)}  differing instances {int(d.sum())}/{B}")
else:
    for prec in (1, 0):
        for lib in sys.argv[1:]:
            subprocess.check_call([sys.executable, __file__, "--one", lib, str(prec)], timeout=300)
