"""GPU parity tests: the HIP kernels behind libalipmpc.so, called through the C ABI, against the reference
goldens (tests/golden) and the oracle (oracle/) on the same seeded inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-12


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b)))) if a.size else 0.0


def _oracle_solve(coracle, cfg_kw, bt, nthreads=8):
    cfg = coracle.default_cfg(**cfg_kw)
    return coracle.solve_batch(cfg, bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt.get("elp"),
                               bt.get("ne"), bt["u0"], nthreads=nthreads)


def _compare(out, ref, min_conv=0.8, min_agree=0.97, min_status=0.97):
    """Parity on the foothold p_list[0] and the predicted states where both solves converged (the NLP is
    nonconvex: rounding-level differences can steer a few instances into another basin)."""
    both = (out["status"] == 0) & (ref["status"] == 0)
    assert both.mean() >= min_conv, both.mean()
    scale = np.maximum(1.0, np.abs(ref["foot"]))
    ok = np.all(np.abs(out["foot"] - ref["foot"]) <= 1e-4 * scale, axis=1)
    okx = np.all(np.abs(out["x_pred"] - ref["x_pred"]).reshape(len(ok), -1) <= 1e-4 * np.maximum(1.0, np.abs(ref["x_pred"]).reshape(len(ok), -1)), axis=1)
    agree = (ok & okx)[both].mean()
    assert agree >= min_agree, agree
    same_status = (out["status"] == ref["status"]).mean()
    assert same_status >= min_status, same_status
    return agree


@pytest.mark.parametrize("name,variant", [("modi", 0), ("sig_step", 1)])
def test_eval_matches_reference_callbacks(gpu_lib, golden, name, variant):
    g = golden(f"g1_callbacks_{name}")
    cfg = gpu_lib.default_cfg(variant, select_obs=0, detour=0)
    s = gpu_lib.Solver(cfg)
    B = len(g["f"])
    o = s.eval(g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
    assert rel(o["f"], g["f"]) < REL
    assert rel(o["grad"], g["grad"]) < REL
    for t in range(B):
        act = o["row_active"][t].astype(bool)
        m = g["m"][t]
        assert act.sum() == m
        assert rel(o["c"][t][act], g["c"][t][:m]) < REL
        assert rel(o["J"][t][act], g["J"][t][:m]) < REL
        assert np.all(o["c"][t][~act] == 0) and np.all(o["J"][t][~act] == 0)


def test_eval_horizon5(gpu_lib, golden, coracle):
    g = golden("g1_callbacks_modi_n5")
    B = len(g["f"])
    cfg = gpu_lib.default_cfg(0, 5, nc_max=10, ne_max=10, select_obs=0, detour=0)
    s = gpu_lib.Solver(cfg)
    o = s.eval(g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
    assert rel(o["f"], g["f"]) < REL
    cc = coracle.default_cfg(0, 5, nc_max=10, ne_max=10, select_obs=0, detour=0)
    r = coracle.eval_batch(cc, g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
    assert rel(o["grad"], r["grad"]) < REL
    assert rel(o["J"], r["J"]) < REL
    for t in range(B):
        act = o["row_active"][t].astype(bool)
        assert rel(o["c"][t][act], g["c"][t][:g["m"][t]]) < REL


@pytest.mark.parametrize("name,variant", [("modi", 0), ("sig_step", 1)])
def test_setup_matches_reference(gpu_lib, golden, name, variant):
    g = golden(f"g2_setup_{name}")
    B = len(g["m"])
    cfg = gpu_lib.default_cfg(variant)
    s = gpu_lib.Solver(cfg)
    o = s.eval(g["x0"], g["goal"], g["leg"], g["cir"], g["nc"], g["elp"], g["ne"], np.tile(g["x0"], (1, 3)))
    for t in range(B):
        act = o["row_active"][t].astype(bool)
        m = g["m"][t]
        assert act.sum() == m
        assert np.array_equal(o["cl"][t][act], g["cl"][t][:m])
        assert np.array_equal(o["cu"][t][act], g["cu"][t][:m])
        assert np.allclose(o["goal_eff"][t], g["goal_eff"][t], rtol=0, atol=1e-14)
        assert np.all(np.isneginf(o["cl"][t][~act])) and np.all(np.isposinf(o["cu"][t][~act]))


def test_solve_sup_learn_recorded_cyipopt(gpu_lib, golden, coracle):
    # solution parity: run to convergence (max_iter 100 instead of the reference's cap of 30)
    d = golden("g3_sup_learn")
    B = len(d["leg"])
    cfg = gpu_lib.default_cfg(0, nc_max=6, ne_max=0, max_iter=100)
    s = gpu_lib.Solver(cfg)
    cir = np.tile(d["cir_safe"], (B, 1, 1))
    o = s.solve(d["x_nex"], [10, 10], d["leg"], cir, np.full(B, 6), u0=d["u0"])
    ok = d["ok_ref"].astype(bool)
    err = np.max(np.abs(o["foot"][:, :2] - d["foot_logged"]), axis=1)
    assert (err[ok] < 1e-4).sum() >= int(0.97 * ok.sum())
    bt = dict(x0=d["x_nex"], goal=np.tile([10.0, 10.0], (B, 1)), leg=d["leg"], cir=cir, nc=np.full(B, 6),
              u0=d["u0"])
    ref = _oracle_solve(coracle, dict(variant=0, nc_max=6, ne_max=0, max_iter=100), bt)
    _compare(o, ref)


def _artifact(name, obj):
    """Write a small JSON record of a test's measured numbers under $ALIPMPC_TEST_ARTIFACTS (if set)."""
    import json
    import os
    d = os.environ.get("ALIPMPC_TEST_ARTIFACTS")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "w") as fh:
            json.dump(obj, fh, indent=1)


def test_sup_learn_basin_misses_objectives(gpu_lib, golden):
    """The converged rows the GPU solves into another local minimum than the reference re-solve (SLSQP on the
    reference callbacks, u_ref): the reference objective f (LIP_Prob.objective, MPC_LIP_modi.py:430-444) at both
    solutions, recorded, and the GPU's minimum is feasible."""
    d = golden("g3_sup_learn")
    B = len(d["leg"])
    cfg = gpu_lib.default_cfg(0, nc_max=6, ne_max=0, max_iter=100)
    s = gpu_lib.Solver(cfg)
    cir = np.tile(d["cir_safe"], (B, 1, 1))
    o = s.solve(d["x_nex"], [10, 10], d["leg"], cir, np.full(B, 6), u0=d["u0"])
    ok = d["ok_ref"].astype(bool)
    err = np.max(np.abs(o["foot"][:, :2] - d["foot_logged"]), axis=1)
    miss = np.nonzero(ok & (err >= 1e-4))[0]
    rows = []
    if miss.size:
        ev = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=6, ne_max=0))
        args = (d["x_nex"][miss], [10, 10], d["leg"][miss], cir[miss], np.full(miss.size, 6))
        eg = ev.eval(*args, u=o["u"][miss])
        er = ev.eval(*args, u=d["u_ref"][miss])
        for j, i in enumerate(miss):
            act = eg["row_active"][j].astype(bool)
            vg = float(np.max(np.maximum(0, np.maximum(eg["cl"][j] - eg["c"][j], eg["c"][j] - eg["cu"][j]))[act]))
            rows.append({"row": int(i), "status_gpu": int(o["status"][i]), "f_gpu": float(eg["f"][j]),
                         "f_ref": float(er["f"][j]), "viol_gpu": vg, "foot_err": float(err[i])})
    _artifact("sup_learn_basin_misses.json", {"pinned_rows": int(ok.sum()), "misses": rows})
    assert len(miss) <= int(0.03 * ok.sum())
    for r in rows:
        assert r["status_gpu"] != 0 or r["viol_gpu"] <= 1e-6


@pytest.mark.parametrize("max_iter", [30, 100])
def test_sup_learn_warm_start_chain(gpu_lib, golden, coracle, max_iter):
    """The 640 recorded cyipopt calls run as the chain the reference ran them in: one episode (80 walking steps x 8
    ticks), every call warm-started from the previous call's plan, unshifted (logger_iml.py:333-342: guess =
    ravel(mpc_state_tar), the previous gen_control_test's x_mpc_tar = the GPU's u_out; [x_nex] x 3 on the first
    call).  Checked against the same chain through the C oracle (same interior point) and against the recorded
    cyipopt footholds (the count reproduced to <= 1e-4 is recorded).  r6: with IPOPT's restoration phase (the default,
    cfg.restoration) the chain reproduces 532 / 538 of the 640 calls at max_iter 30 / 100, the oracle the same
    (profiles/r6/resto); the rounds-1-5 substitute reproduced 479 — the bar is 520."""
    d = golden("g3_sup_learn")
    n = len(d["leg"])
    cs = d["cir_safe"]
    goal = np.array([[10.0, 10.0]])
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=6, ne_max=0, max_iter=max_iter))
    cc = coracle.default_cfg(0, 3, nc_max=6, ne_max=0)
    cc.max_iter = max_iter
    fg, fo = np.zeros((n, 3)), np.zeros((n, 3))
    sg, so = np.zeros(n, np.int32), np.zeros(n, np.int32)
    ug = uo = d["u0"][0]
    for i in range(n):
        a = (d["x_nex"][i:i + 1], goal, d["leg"][i:i + 1], cs[None], np.array([6]))
        og = s.solve(*a, u0=ug[None])
        oo = coracle.solve_batch(cc, *a, np.zeros((1, 0, 5)), np.zeros(1), uo[None])
        fg[i], fo[i], sg[i], so[i] = og["foot"][0], oo["foot"][0], og["status"][0], oo["status"][0]
        ug, uo = og["u"][0], oo["u"][0]
    eg = np.max(np.abs(fg[:, :2] - d["foot_logged"]), axis=1)
    eo = np.max(np.abs(fo[:, :2] - d["foot_logged"]), axis=1)
    both = (sg == 0) & (so == 0)
    agree = np.max(np.abs(fg - fo), axis=1) <= 1e-4
    rec = {"max_iter": max_iter, "rows": n, "gpu_reproduces_cyipopt_1e-4": int((eg <= 1e-4).sum()),
           "oracle_reproduces_cyipopt_1e-4": int((eo <= 1e-4).sum()),
           "gpu_reproduces_cyipopt_1e-6": int((eg <= 1e-6).sum()),
           "gpu_vs_oracle_chain_agree_converged": float(agree[both].mean()),
           "status_gpu": {str(k): int(v) for k, v in zip(*np.unique(sg, return_counts=True))}}
    _artifact(f"sup_learn_chain_{max_iter}.json", rec)
    assert agree[both].mean() >= 0.97, rec
    assert (sg == so).mean() >= 0.95, rec
    assert (eg <= 1e-4).sum() >= 520, rec


@pytest.mark.parametrize("variant,name", [(0, "modi"), (1, "sig_step")])
def test_solve_synthetic_scipy_goldens(gpu_lib, golden, variant, name):
    d = golden(f"g3_synthetic_{name}")
    good = (d["agree"] < 1e-8) & (d["viol"] < 1e-8)
    cfg = gpu_lib.default_cfg(variant, nc_max=6, ne_max=6, max_iter=100)   # to convergence
    s = gpu_lib.Solver(cfg)
    o = s.solve(d["x0"], d["goal"], d["leg"], d["cir"], d["nc"], d["elp"], d["ne"], u0=d["u0"])
    err = np.max(np.abs(o["foot"] - d["foot_ref"]), axis=1)
    assert np.all(err[good] < 1e-4), err[good].max()


def test_solve_cfg2_batch_vs_oracle(gpu_lib, coracle):
    from alipmpc import scenes
    bt = scenes.make_batch(2048, seed=11, n_cir=5)
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=5, ne_max=0))
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    ref = _oracle_solve(coracle, dict(variant=0, nc_max=5, ne_max=0), bt)
    _compare(o, ref)
    # u is the canonical u_k = x_{k+1}; foot and states are consistent with the ALIP step map
    assert np.allclose(o["u"].reshape(-1, 3, 5), o["x_pred"], rtol=0, atol=0)


@pytest.mark.parametrize("prec", [0, 1])
def test_max_slots_n6_every_launch_form(gpu_lib, coracle, prec):
    """alipmpc_create either rejects a shape (EINVAL: N * rows_per_step > 128; EUNSUPPORTED: a
    workspace beyond the CU's 160 KB of LDS, or an fp32 / lane hand-off whose fp64 workspace does not fit) or every
    launch of it succeeds.  N = 6 (the horizon limit) at the largest obstacle-slot count create accepts, half circles and
    half ellipses: the one-wave split form (B below the resident slots), the work queue (B above them) and one
    closed-loop tick must all launch, return finite iterates and valid statuses, and agree with the C oracle's statuses
    on the instances compared (fp64: >= 90 %; fp32: the instance solved at all).  (r5a's N = 6 `EHIP invalid argument`
    was a launch of the team-capable build whose workspaces exceeded 160 KB at N = 6 — DESIGN.md §3.1.)"""
    from alipmpc import scenes
    N = 6
    kw = {"precision": gpu_lib.PREC_FP32} if prec else {}
    found = None
    for tot in range(24, 0, -1):
        nc, ne = (tot + 1) // 2, tot // 2
        try:
            s = gpu_lib.Solver(gpu_lib.default_cfg(0, N, nc_max=nc, ne_max=ne, **kw))
        except RuntimeError as e:
            assert "EINVAL" in str(e) or "EUNSUPPORTED" in str(e), str(e)
            continue
        found = (nc, ne, s)
        break
    assert found is not None
    nc, ne, s = found
    assert nc + ne >= 8, (nc, ne)   # (the largest accepted shape is not a degenerate one)
    slots = s.solve_slots()
    valid = {0, 1, 2, -1, -2, -3, -13}
    for B in (64, slots + 64):
        bt = scenes.make_batch(B, seed=61 + B % 7, n_cir=nc, n_elp=ne, N=N)
        o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u0=bt["u0"])
        assert np.isfinite(o["u"]).all() and set(np.unique(o["status"])) <= valid, (B, np.unique(o["status"]))
        if B == 64:
            co = coracle.default_cfg(0, N, nc_max=nc, ne_max=ne)
            if prec:
                co.tol, co.acceptable_tol = s.cfg.tol, s.cfg.acceptable_tol
            ref = coracle.solve_batch(co, bt["x0"][:32], bt["goal"][:32], bt["leg"][:32], bt["cir"][:32], bt["nc"][:32],
                                      bt["elp"][:32], bt["ne"][:32], bt["u0"][:32])
            agree = np.mean(o["status"][:32] == ref["status"])
            print(f"N=6 nc={nc} ne={ne} prec={prec}: status agreement {agree:.3f}")
            assert agree >= (0.9 if not prec else 0.75), agree
    foot0 = o["foot"][:64, 0:2].copy()
    cl = s.closed_loop(bt["x0"][:64], foot0, bt["goal"][:64], bt["leg"][:64].astype(np.int8), bt["cir"][:64],
                       bt["nc"][:64], bt["elp"][:64], bt["ne"][:64], steps=1, f_cyc=2)
    assert set(np.unique(cl["status"])) <= valid | {gpu_lib.ROLLOUT_DONE}


# (N <= 3 with more than 16 obstacle slots: the Hessian blocks' second slot per lane, hess_blocks_lanes; no obstacle
# slots at N <= 3: the 4-row-step J layout, solve_kernel<N, 4, ...>)
@pytest.mark.parametrize("variant,N,n_cir,n_elp", [(1, 3, 4, 0), (0, 3, 3, 3), (0, 5, 5, 5), (0, 1, 2, 0),
                                                   (0, 4, 5, 0), (0, 6, 3, 0), (0, 3, 12, 8), (1, 2, 14, 6),
                                                   (1, 3, 0, 0), (0, 2, 0, 0)])
def test_solve_variants_vs_oracle(gpu_lib, coracle, variant, N, n_cir, n_elp):
    from alipmpc import scenes
    bt = scenes.make_batch(256, seed=100 + N + n_elp, n_cir=n_cir, n_elp=n_elp, N=N)
    cfg = gpu_lib.default_cfg(variant, N, nc_max=n_cir, ne_max=n_elp)
    s = gpu_lib.Solver(cfg)
    if n_cir + n_elp == 0:
        assert s.solve_program().startswith(f"solve_kernel<{N},4,"), s.solve_program()
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u0=bt["u0"])
    ref = _oracle_solve(coracle, dict(variant=variant, N=N, nc_max=n_cir, ne_max=n_elp), bt)
    _compare(o, ref, min_conv=0.5, min_agree=0.95, min_status=0.9)


def test_edge_cases(gpu_lib, coracle):
    from alipmpc import scenes
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=5, ne_max=0))
    bt = scenes.make_batch(8, seed=3, n_cir=5)
    # empty batch is a no-op
    o = s.solve(bt["x0"][:0], bt["goal"][:0], bt["leg"][:0], bt["cir"][:0], bt["nc"][:0], u0=bt["u0"][:0])
    assert o["u"].shape == (0, 15)
    # ragged obstacle counts, including none, and obstacles all outside the 4 m detection range
    nc = np.array([0, 1, 2, 3, 4, 5, 5, 5], np.int32)
    cir = bt["cir"].copy()
    cir[6, :, :2] += 50.0
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], cir, nc, u0=bt["u0"])
    ref = coracle.solve_batch(coracle.default_cfg(0, nc_max=5, ne_max=0), bt["x0"], bt["goal"], bt["leg"], cir, nc,
                              None, None, bt["u0"])
    both = (o["status"] == 0) & (ref["status"] == 0)
    assert both.sum() >= 6
    assert np.all(np.abs(o["foot"] - ref["foot"])[both] <= 1e-4 * np.maximum(1.0, np.abs(ref["foot"][both])))
    # B = 1
    o1 = s.solve(bt["x0"][:1], bt["goal"][:1], bt["leg"][:1], cir[:1], nc[:1], u0=bt["u0"][:1])
    assert np.array_equal(o1["foot"][0], o["foot"][0])
    # a CoM velocity the step-to-step model cannot bring into the body-velocity bounds with a leg of at
    # most 0.3 m is infeasible: status 2 (the reference's "fail"), the iterate is still returned
    x0 = bt["x0"][:1].copy()
    x0[0, 2:4] = [3.0, 3.0]
    o2 = s.solve(x0, bt["goal"][:1], bt["leg"][:1], cir[:1], nc[:1], u0=np.tile(x0, (1, 3)))
    assert o2["status"][0] == 2 and np.all(np.isfinite(o2["u"]))
    # max slot counts: 8 circles + 8 ellipses (m = 3 * 21 rows)
    bt16 = scenes.make_batch(64, seed=5, n_cir=8, n_elp=8)
    s16 = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=8, ne_max=8))
    o16 = s16.solve(bt16["x0"], bt16["goal"], bt16["leg"], bt16["cir"], bt16["nc"], bt16["elp"], bt16["ne"],
                    u0=bt16["u0"])
    ref16 = _oracle_solve(coracle, dict(variant=0, nc_max=8, ne_max=8), bt16)
    _compare(o16, ref16, min_conv=0.5, min_agree=0.9, min_status=0.9)


def test_invalid_arguments_raise(gpu_lib):
    with pytest.raises(RuntimeError):
        gpu_lib.Solver(gpu_lib.default_cfg(0, 7))            # horizon above the kernel limit
    with pytest.raises(RuntimeError):
        gpu_lib.Solver(gpu_lib.default_cfg(0, 3, nc_max=20, ne_max=20))


def test_device_pointer_mode_and_determinism(gpu_lib):
    import torch
    from alipmpc import scenes
    B = 1024
    bt = scenes.make_batch(B, seed=21, n_cir=5)
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=5, ne_max=0))
    host = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    s.solve_device(inp, out)
    torch.cuda.synchronize()
    assert np.array_equal(out["foot"].cpu().numpy(), host["foot"])
    assert np.array_equal(out["status"].cpu().numpy(), host["status"])
    host2 = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    assert np.array_equal(host2["u"], host["u"]) and np.array_equal(host2["iters"], host["iters"])


def test_full_size_properties_cfg3(gpu_lib):
    """BASELINE configs[2] size (B = 65536, N = 5, 5 circles + 5 ellipses): size-independent properties of
    every returned plan — finite outputs, valid statuses, the ALIP step map between foot, u and states,
    and, for converged instances, feasibility of the reference constraints at the returned u (evaluated by
    the eval kernel) within the solver tolerance."""
    from alipmpc import scenes
    B = 65536
    bt = scenes.make_batch(B, seed=33, n_cir=5, n_elp=5, N=5, scenes_per_batch=512)
    cfg = gpu_lib.default_cfg(0, 5, nc_max=5, ne_max=5)
    s = gpu_lib.Solver(cfg)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u0=bt["u0"])
    assert np.all(np.isfinite(o["u"])) and np.all(np.isfinite(o["foot"]))
    assert set(np.unique(o["status"]).tolist()) <= {-3, -1, 0, 1, 2}
    assert (o["status"] == 0).mean() > 0.7
    assert np.array_equal(o["u"].reshape(B, 5, 5), o["x_pred"])
    ev = s.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], o["u"], want_J=False)
    conv = o["status"] == 0
    act = ev["row_active"].astype(bool)
    viol = np.maximum(ev["cl"] - ev["c"], ev["c"] - ev["cu"])
    viol[~act] = 0
    assert np.max(viol[conv]) < 1e-6
    # foot = p_0 = W (u_1 - A x0) is exactly the step map the eval kernel sees: x_1 = A x0 + B p_0
    import alipmpc.planner as pl
    beta = np.sqrt(9.81)
    A, Bm = pl._alip_matrices(beta, 0.4, 0.4)
    x1 = bt["x0"] @ A.T + o["foot"] @ Bm.T
    assert np.max(np.abs(x1 - o["x_pred"][:, 0])) < 1e-12


# ---------------------------------------------------------------- DD variant (MPC_DD_sig_step.py)
def _dd_batch(B, seed, n_cir=5, N=3):
    from alipmpc import scenes
    bt = scenes.make_batch(B, seed=seed, n_cir=n_cir, N=N)
    rng = np.random.default_rng(seed + 17)
    x0 = np.stack([bt["x0"][:, 0], bt["x0"][:, 1], bt["x0"][:, 4]], 1)
    last_u = np.stack([rng.uniform(0.45, 0.75, B), rng.uniform(-0.15, 0.15, B)], 1)
    return dict(x0=x0, goal=bt["goal"], cir=bt["cir"], nc=bt["nc"], last_u=last_u, u0=np.tile(last_u, (1, N)))


def test_dd_eval_matches_reference_callbacks(gpu_lib, golden):
    g = golden("g1_callbacks_dd")
    s = gpu_lib.Solver(gpu_lib.default_cfg(2))
    o = s.eval(g["x0"], g["goal"], None, g["cir"], g["nc"], g["elp"], g["ne"], g["u"], last_u=g["last_u"])
    assert rel(o["f"], g["f"]) < REL
    assert rel(o["grad"], g["grad"]) < REL
    for t in range(len(g["f"])):
        act = o["row_active"][t].astype(bool)
        assert act.sum() == g["m"][t]
        assert rel(o["c"][t][act], g["c"][t][:g["m"][t]]) < REL
        assert rel(o["J"][t][act], g["J"][t][:g["m"][t]]) < REL


def test_dd_solve_matches_scipy_goldens(gpu_lib, golden, coracle):
    d = golden("g3_synthetic_dd")
    good = (d["agree"] < 1e-6) & (d["viol"] < 1e-8)
    s = gpu_lib.Solver(gpu_lib.default_cfg(2, nc_max=6, ne_max=6, max_iter=100))   # to convergence
    o = s.solve(d["x0"], d["goal"], None, d["cir"], d["nc"], d["elp"], d["ne"], u0=d["u0"], last_u=d["last_u"])
    err = np.max(np.abs(o["u"] - d["u_ref"]), axis=1)
    assert np.all(err[good] < 1e-4), err[good].max()
    cc = coracle.default_cfg(2, nc_max=6, ne_max=6, max_iter=100)
    r = coracle.solve_batch_dd(cc, d["x0"], d["goal"], d["cir"], d["nc"], d["elp"], d["ne"], d["u0"], d["last_u"])
    assert (o["status"] == r["status"]).mean() >= 0.95
    both = (o["status"] == 0) & (r["status"] == 0)
    assert (np.max(np.abs(o["u"] - r["u"]), axis=1)[both] < 1e-6).mean() >= 0.95
    assert np.allclose(o["foot"][:, :2], o["u"][:, :2]) and np.all(o["foot"][:, 2] == 0)


@pytest.mark.parametrize("N", [3, 5])
def test_dd_batch_vs_oracle(gpu_lib, coracle, N):
    bt = _dd_batch(512, seed=40 + N, N=N)
    s = gpu_lib.Solver(gpu_lib.default_cfg(2, N, nc_max=5, ne_max=0))
    o = s.solve(bt["x0"], bt["goal"], None, bt["cir"], bt["nc"], u0=bt["u0"], last_u=bt["last_u"])
    cc = coracle.default_cfg(2, N, nc_max=5, ne_max=0)
    r = coracle.solve_batch_dd(cc, bt["x0"], bt["goal"], bt["cir"], bt["nc"], None, None, bt["u0"], bt["last_u"],
                               nthreads=8)
    assert (o["status"] == r["status"]).mean() >= 0.95
    both = (o["status"] == 0) & (r["status"] == 0)
    assert both.mean() >= 0.5
    ok = np.max(np.abs(o["u"] - r["u"]), axis=1) < 1e-4
    assert ok[both].mean() >= 0.97
    okx = np.max(np.abs(o["x_pred"] - r["x_pred"]).reshape(len(ok), -1), axis=1) < 1e-4
    assert okx[both].mean() >= 0.97


def test_planner_dropins_match_batched_solver(gpu_lib, golden):
    """ALIP_plan/planner.py drop-ins (MPCCBF / MPCCBFSigStep / MPCCBFDD) return the reference tuples and the
    same solution as one batched launch."""
    import alipmpc.planner as pl
    d = golden("g3_sup_learn")
    cir = d["cir_safe"]
    mp = pl.MPCCBF([[10, 10]], cir, cir, [], [], [-0.5, 10.5])
    idx = [0, 7, 33]
    batch = mp.solve_batch(d["x_nex"][idx], d["leg"][idx], d["u0"][idx])
    for j, i in enumerate(idx):
        xs, p0, hd, c2g, feasi, pos_det = mp.gen_control_test(d["x_nex"][i], d["leg"][i], d["u0"][i])
        assert feasi == batch["status"][j]
        assert np.max(np.abs(p0 - batch["foot"][j])) < 1e-12
        assert len(xs) == 3 and len(hd) == 3 and pos_det.shape[1] == 2
        assert np.max(np.abs(np.array(xs) - batch["x_pred"][j])) < 1e-12
    ss = pl.MPCCBFSigStep([[10, 10]], cir, cir, [-0.5, 10.5])
    out = ss.gen_control_test(d["x_nex"][0], d["leg"][0], None)
    assert len(out) == 4 and out[1].shape == (3,)
    bt = _dd_batch(4, seed=5)
    dd = pl.MPCCBFDD([[10, 10]], bt["cir"][0][:bt["nc"][0]], bt["cir"][0][:bt["nc"][0]], [], [], [-0.5, 10.5])
    db = dd.solve_batch(bt["x0"][:1], bt["u0"][:1], bt["last_u"][:1])
    states, heading, control, c2g, fesi = dd.gen_dd_control(bt["x0"][0], bt["u0"][0], bt["last_u"][0])
    assert fesi == db["status"][0] and len(states) == 4 and len(control) == 3
    assert np.max(np.abs(np.array(states[1:]) - db["x_pred"][0])) < 1e-12
    assert np.max(np.abs(np.ravel(control) - db["u"][0])) < 1e-15


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_rollout_matches_oracle(gpu_lib, coracle, variant):
    """alipmpc_rollout_batch (S solve launches + plant-update kernels on one stream) against the oracle's
    closed loop on the same seeded episodes: whole trajectories (footholds, touchdown states, statuses,
    steps to goal) agree on the large majority of episodes (a rounding-level difference can switch a
    nonconvex solve into another basin and the episode then diverges)."""
    from alipmpc import scenes
    dd = variant == 2
    N, B, S = 3, 128, 6
    bt = scenes.make_batch(B, seed=91 + variant, n_cir=5, N=N)
    if dd:
        x0 = bt["x0"][:, [0, 1, 4]].copy()
        u0 = np.tile([0.6, 0.0], (B, N))
        lu = np.tile([0.6, 0.0], (B, 1))
    else:
        x0, lu = bt["x0"].copy(), None
    x0[:16, 0:2] = bt["goal"][:16] - np.array([0.3, 0.2])
    if not dd:
        u0 = np.tile(x0, (1, N))
    cfg = gpu_lib.default_cfg(variant, N, nc_max=5, ne_max=0)
    s = gpu_lib.Solver(cfg)
    o = s.rollout(x0, bt["goal"], None if dd else bt["leg"], bt["cir"], bt["nc"], u0=u0, last_u=lu, steps=S)
    ref = coracle.rollout_batch(coracle.default_cfg(variant, N, nc_max=5, ne_max=0), x0, bt["goal"], bt["leg"],
                                bt["cir"], bt["nc"], None, None, u0, lu, steps=S, nthreads=8)
    same_status = (o["status"] == ref["status"]).all(1)
    fo = np.nan_to_num(o["foot"], nan=1e9)
    fr = np.nan_to_num(ref["foot"], nan=1e9)
    same_path = (np.abs(fo - fr) <= 1e-4 * np.maximum(1.0, np.abs(fr))).all((1, 2)) & \
        (np.abs(o["x"] - ref["x"]) <= 1e-4 * np.maximum(1.0, np.abs(ref["x"]))).all((1, 2))
    agree = (same_status & same_path).mean()
    assert agree >= 0.85, agree
    assert (o["steps_to_goal"] == ref["steps_to_goal"]).mean() >= 0.9
    assert (o["steps_to_goal"][:16] > 0).sum() >= 8
    # retired instances are not solved again
    for b in np.nonzero(o["steps_to_goal"] > 0)[0]:
        assert (o["status"][b, o["steps_to_goal"][b]:] == gpu_lib.ROLLOUT_DONE).all()
    # device-pointer path gives the same trajectories
    import torch
    dev = torch.device("cuda", 0)
    inp = {"x0": torch.from_numpy(x0).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
           "cir": torch.from_numpy(bt["cir"]).to(dev), "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev),
           "u0": torch.from_numpy(u0).to(dev)}
    if dd:
        inp["last_u"] = torch.from_numpy(lu).to(dev)
    else:
        inp["leg"] = torch.from_numpy(bt["leg"].astype(np.int8)).to(dev)
    out = {"foot": torch.empty((B, S, 3), dtype=torch.float64, device=dev),
           "x": torch.empty((B, S + 1, x0.shape[1]), dtype=torch.float64, device=dev),
           "status": torch.empty((B, S), dtype=torch.int32, device=dev),
           "steps_to_goal": torch.empty((B,), dtype=torch.int32, device=dev)}
    s.rollout_device(inp, out, S)
    torch.cuda.synchronize()
    assert np.array_equal(out["status"].cpu().numpy(), o["status"])
    assert np.array_equal(np.nan_to_num(out["foot"].cpu().numpy(), nan=7.0), np.nan_to_num(o["foot"], nan=7.0))
    assert np.array_equal(out["steps_to_goal"].cpu().numpy(), o["steps_to_goal"])


def _violation(ev):
    v = np.maximum(np.maximum(ev["cl"] - ev["c"], ev["c"] - ev["cu"]), 0.0)
    v[~ev["row_active"].astype(bool)] = 0.0
    return v.max(axis=1)


@pytest.mark.parametrize("N,n_cir,n_elp,max_iter,min_conv,min_agree,feas_margin",
                         [(3, 5, 0, 30, 0.75, 0.98, 0.01), (5, 5, 5, 100, 0.5, 0.95, 0.06)])
def test_fp32_solve_vs_oracle(gpu_lib, coracle, N, n_cir, n_elp, max_iter, min_conv, min_agree, feas_margin):
    """cfg.precision = fp32 (BASELINE cfg5): the solve kernel in fp32 arithmetic (default fp32 tolerances:
    1e-4 at N = 3, 3e-4 at N = 5) against the fp64 C oracle on the same seeded batch.  Tolerance for fp32:
    foothold within 1e-3 (abs, |foot| ~ 1-10 m) on >= min_agree of the instances both converge on; the
    solution, evaluated by the fp64 reference callbacks, violates no constraint by more than 1e-4 on about as
    many instances as the fp64 oracle's does (N = 5: more fp32 solves stop at the iteration cap)."""
    from alipmpc import scenes
    B = 512
    bt = scenes.make_batch(B, seed=41 + N, n_cir=n_cir, n_elp=n_elp, N=N)
    cfg = gpu_lib.default_cfg(0, N, nc_max=n_cir, ne_max=n_elp, precision=gpu_lib.PREC_FP32, max_iter=max_iter)
    assert cfg.tol == (gpu_lib.FP32_TOL if N <= 3 else gpu_lib.FP32_TOL_LONG)
    s = gpu_lib.Solver(cfg)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u0=bt["u0"])
    ref = _oracle_solve(coracle, dict(variant=0, N=N, nc_max=n_cir, ne_max=n_elp, max_iter=max_iter), bt)
    both = (o["status"] == 0) & (ref["status"] == 0)
    counts = lambda st: dict(zip(*np.unique(st, return_counts=True)))  # noqa: E731
    assert both.mean() >= min_conv, (both.mean(), counts(o["status"]), counts(ref["status"]))
    err = np.abs(o["foot"] - ref["foot"]).max(axis=1)
    assert np.mean(err[both] <= 1e-3) >= min_agree, np.mean(err[both] <= 1e-3)
    s64 = gpu_lib.Solver(gpu_lib.default_cfg(0, N, nc_max=n_cir, ne_max=n_elp))
    feas32 = _violation(s64.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"],
                                 u=o["u"], want_J=False)) <= 1e-4
    feas64 = _violation(s64.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"],
                                 u=ref["u"], want_J=False)) <= 1e-4
    assert feas32.mean() >= feas64.mean() - feas_margin, (feas32.mean(), feas64.mean())
    # infeasibility verdicts agree with fp64 (status 2 <=> 2) on nearly all instances
    assert ((o["status"] == 2) == (ref["status"] == 2)).mean() >= 0.97


def test_fp32_dd_unsupported(gpu_lib):
    cfg = gpu_lib.default_cfg(gpu_lib.VARIANT_DD, 3, precision=gpu_lib.PREC_FP32)
    with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
        gpu_lib.Solver(cfg)


@pytest.mark.parametrize("variant,N", [(0, 3), (1, 3), (0, 5)])
def test_trace_batch_matches_plan_traces(gpu_lib, variant, N):
    """alipmpc_trace_batch (trace_kernel) against the numpy restatement of gen_control_test's pos_det
    (planner.plan_traces = xk_track_det per planned step, pinned to the reference by g4_aux), on solve
    outputs; host and device pointer paths."""
    from alipmpc import planner, scenes
    bt = scenes.make_batch(200, seed=61 + N, n_cir=5, N=N)
    cfg = gpu_lib.default_cfg(variant, N, nc_max=5, ne_max=0)
    s = gpu_lib.Solver(cfg)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    tr = s.trace(bt["x0"], o["u"])
    assert tr.shape == (200, N, 42, 2)
    k = planner.alip_constants()
    ref = planner.plan_traces(k["beta"], 0.4, k["A"], k["W"], k["M_A"], k["M_B"], bt["x0"], o["u"])
    assert np.max(np.abs(tr - ref)) < 1e-12
    import torch
    dev = torch.device("cuda", 0)
    td = torch.empty((200, N, 42, 2), dtype=torch.float64, device=dev)
    s.trace_device(torch.from_numpy(bt["x0"]).to(dev), torch.from_numpy(o["u"]).to(dev), td)
    torch.cuda.synchronize()
    assert np.array_equal(td.cpu().numpy(), tr)
    with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
        gpu_lib.Solver(gpu_lib.default_cfg(gpu_lib.VARIANT_DD, 3)).trace(bt["x0"], np.zeros((200, 6)))


def test_rollout_plans_and_data_log(gpu_lib, coracle, tmp_path):
    """rollout u_traj (the plan of every step) is consistent with the executed steps, and data_log episode
    logs built from the GPU rollout + GPU traces equal those built with the numpy traces."""
    from alipmpc import datalog, planner, scenes
    B, S = 64, 6
    bt = scenes.make_batch(B, seed=77, n_cir=5)
    x0 = bt["x0"].copy()
    x0[:8, 0:2] = bt["goal"][:8] - np.array([0.4, 0.3])
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, 3, nc_max=5, ne_max=0))
    r = s.rollout(x0, bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)), steps=S)
    act = r["status"] != gpu_lib.ROLLOUT_DONE
    assert np.array_equal(r["u"][:, :, 0:5][act], r["x"][:, 1:][act])      # x^(t+1) = plan's x_1
    assert np.isnan(r["u"][~act]).all()
    assert np.isfinite(r["u"][act]).all()
    k = planner.alip_constants()
    for b in (0, 1, 9, 20):
        lg = datalog.episode_logs(r, b, s.trace, cir=bt["cir"][b])
        ln = datalog.episode_logs(r, b, lambda xs, us: planner.plan_traces(k["beta"], 0.4, k["A"], k["W"],
                                                                         k["M_A"], k["M_B"], xs, us),
                                  cir=bt["cir"][b])
        for name in datalog.NAMES:
            a, c = lg[name], ln[name]
            if isinstance(c, list):
                assert len(a) == len(c) and all(np.max(np.abs(x - y), initial=0) < 1e-12 for x, y in zip(a, c))
            else:
                assert np.max(np.abs(np.asarray(a) - np.asarray(c)), initial=0) < 1e-12, name
        datalog.write_data_log(str(tmp_path / f"LIP_gpu{b}_"), lg)
    assert (r["steps_to_goal"][:8] > 0).sum() >= 2


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("N", [1, 2, 4, 6])
def test_fp32_all_horizons_agree_with_fp64(gpu_lib, variant, N):
    """Every compiled fp32 instantiation (horizons 1..6, both LIP variants, GJ and Cholesky solve paths)
    runs and lands where the fp64 kernel lands on most instances (foothold within 1e-3 where both
    converge)."""
    from alipmpc import scenes
    n_cir = 4 if variant == 1 else 5
    bt = scenes.make_batch(128, seed=300 + N + 10 * variant, n_cir=n_cir, N=N)
    kw = dict(nc_max=n_cir, ne_max=0, max_iter=100)
    o64 = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, **kw)).solve(
        bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    o32 = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, precision=gpu_lib.PREC_FP32, **kw)).solve(
        bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    # a factorisation the regularisation cannot rescue ends that instance with status -3 and its last
    # (finite) iterate, as IPOPT's Error_In_Step_Computation does
    assert np.isfinite(o32["u"]).all() and np.isfinite(o32["foot"]).all()
    assert np.isin(o32["status"], [0, 1, 2, -1, -3]).all()
    assert np.mean(o32["status"] == -3) <= 0.05
    both = (o64["status"] == 0) & (o32["status"] == 0)
    assert both.mean() >= 0.4, (both.mean(), np.unique(o32["status"], return_counts=True))
    err = np.abs(o32["foot"] - o64["foot"]).max(axis=1)
    assert np.mean(err[both] <= 1e-3) >= 0.9, np.mean(err[both] <= 1e-3)


WQ_CASES = [  # (variant, N, circles, ellipses, precision): cfg2/cfg4's kernel, cfg5's (fp32), cfg3's (N = 5)
    (0, 3, 5, 0, 0), (0, 3, 5, 0, 1), (0, 5, 5, 5, 0)]


@pytest.mark.parametrize("variant,N,n_cir,n_elp,prec", WQ_CASES)
def test_work_queue_batch_independence(gpu_lib, variant, N, n_cir, n_elp, prec):
    """Every LIP solve launch is the persistent work-queue program (at most the resident workgroups).
    An instance's result must not depend on the batch it is solved in: the same instances solved as one
    batch larger than the resident slots and in chunks of half the slots are bit-identical (status, iters,
    u, foot, x_pred); every instance is solved exactly once (NaN-filled device outputs); the queue counters
    reset between launches (a second launch reproduces the first bit for bit).  A closed-loop rollout
    (retired instances skipped through the queue) matches its chunked counterpart bit for bit too."""
    import torch
    from alipmpc import scenes
    kw = dict(nc_max=n_cir, ne_max=n_elp)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, **kw))
    slots = s.solve_slots()
    assert slots >= 1024 and slots % 4 == 0, slots
    B = slots + slots // 2 + 37
    bt = scenes.make_batch_vec(B, seed=71 + N + prec, n_cir=n_cir, n_elp=n_elp, N=N)
    args = lambda i0, i1: (bt["x0"][i0:i1], bt["goal"][i0:i1], bt["leg"][i0:i1], bt["cir"][i0:i1],  # noqa: E731
                           bt["nc"][i0:i1], None if bt["elp"] is None else bt["elp"][i0:i1],
                           None if bt["ne"] is None else bt["ne"][i0:i1])
    big = s.solve(*args(0, B), u0=bt["u0"])
    ch = slots // 2
    parts = [s.solve(*args(i, i + ch), u0=bt["u0"][i:i + ch]) for i in range(0, B, ch)]
    small = {k: np.concatenate([p[k] for p in parts]) for k in big}
    for k in big:
        assert np.array_equal(big[k], small[k]), k
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    if "ne" in inp:
        inp["ne"] = inp["ne"].to(torch.int32)
    n = 5 * N
    runs = []
    for _ in range(2):
        out = {"u": torch.full((B, n), float("nan"), dtype=torch.float64, device=dev),
               "foot": torch.full((B, 3), float("nan"), dtype=torch.float64, device=dev),
               "x_pred": torch.full((B, N, 5), float("nan"), dtype=torch.float64, device=dev),
               "status": torch.full((B,), -99, dtype=torch.int32, device=dev),
               "iters": torch.full((B,), -99, dtype=torch.int32, device=dev)}
        s.solve_device(inp, out)
        torch.cuda.synchronize()
        runs.append({k: v.cpu().numpy() for k, v in out.items()})
        assert np.isfinite(runs[-1]["u"]).all() and (runs[-1]["status"] != -99).all()
    for k in runs[0]:
        assert np.array_equal(runs[0][k], runs[1][k]), k
        assert np.array_equal(runs[0][k], big[k]), k
    if N != 3 or prec:
        return
    # rollout: queue launch with retired instances vs the same instances in slot-sized chunks
    S = 6
    u0 = np.tile(bt["x0"], (1, 3))
    r_big = s.rollout(*args(0, B), u0=u0, steps=S)
    r_parts = [s.rollout(*args(i, i + ch), u0=u0[i:i + ch], steps=S) for i in range(0, B, ch)]
    r_small = {k: np.concatenate([p[k] for p in r_parts]) for k in r_big}
    for k in r_big:
        assert np.array_equal(np.nan_to_num(r_big[k], nan=7.0), np.nan_to_num(r_small[k], nan=7.0)), k


BENCH_KERNELS = [  # the program each BASELINE bench number comes from (bench.CONFIGS), at B > resident slots; the
    # wave-program rows of the N = 3 shapes are kept as separate cases
    ("cfg5", 0, 3, 5, 0, 1, "lane"), ("cfg4", 0, 3, 5, 0, 0, "lane"), ("cfg3", 0, 5, 5, 5, 0, "wave"),
    ("cfg5", 0, 3, 5, 0, 1, "wave"), ("cfg4", 0, 3, 5, 0, 0, "wave")]


@pytest.mark.parametrize("name,variant,N,n_cir,n_elp,prec,program", BENCH_KERNELS)
def test_bench_kernels_beyond_resident_slots_vs_oracle(gpu_lib, coracle, name, variant, N, n_cir, n_elp, prec,
                                                       program):
    """The solve program and scene generator bench.py measures for cfg3 / cfg4 / cfg5 (bench.CONFIGS: the lane
    program for cfg4 / cfg5, the wave program for cfg3; bench.global_inputs), at a batch above the program's resident
    slots (the persistent work queue cycles every wave / lane through several instances), against the fp64 C oracle
    on a fixed random subset of 2,048 instances.  Bars: fp64 as test_solve_variants_vs_oracle (cfg3) /
    test_solve_cfg2_batch_vs_oracle (cfg4); fp32 as test_fp32_solve_vs_oracle (foothold within 1e-3 where both
    converge)."""
    import bench
    if program == "lane":
        assert bench.CONFIGS[name]["program"] == "lane"
    kw = dict(nc_max=n_cir, ne_max=n_elp,
              program=gpu_lib.PROGRAM_LANE if program == "lane" else gpu_lib.PROGRAM_WAVE)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, **kw))
    assert s.solve_program().startswith("lane_kernel" if program == "lane" else "solve_kernel")
    slots = s.solve_slots()
    B = slots + slots // 8 + 123
    block = 65536 if name == "cfg3" else bench.BLOCK[name]
    bt = bench.global_inputs(name, 0, B, block, 5, n_cir, n_elp, N)
    bt.setdefault("elp", None)
    bt.setdefault("ne", None)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u0=bt["u0"])
    idx = np.sort(np.random.default_rng(9).choice(B, 2048, replace=False))
    sub = {k: (None if v is None else v[idx]) for k, v in bt.items()}
    osub = {k: v[idx] for k, v in o.items()}
    ref = _oracle_solve(coracle, dict(variant=variant, N=N, nc_max=n_cir, ne_max=n_elp), sub)
    if prec:
        both = (osub["status"] == 0) & (ref["status"] == 0)
        assert both.mean() >= 0.75, both.mean()
        err = np.abs(osub["foot"] - ref["foot"]).max(axis=1)
        assert np.mean(err[both] <= 1e-3) >= 0.98, np.mean(err[both] <= 1e-3)
        assert ((osub["status"] == 2) == (ref["status"] == 2)).mean() >= 0.97
    elif N == 5:
        _compare(osub, ref, min_conv=0.5, min_agree=0.95, min_status=0.9)
    else:
        _compare(osub, ref)


def test_unconverged_iterates_track_oracle(gpu_lib, coracle):
    """The reference uses the iterate as its plan whatever IPOPT's status (main_sim_mpc.py:117-121), so
    instances that end with status 2 (infeasible) or -1 (iteration cap) are compared too: the GPU runs
    the oracle's algorithm, and its last iterate lands near the oracle's on most such instances (their
    trajectories are not contracting, so rounding-level differences can grow on a few of them)."""
    from alipmpc import scenes
    bt = scenes.make_batch(4096, seed=0, n_cir=5)
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, nc_max=5, ne_max=0))
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    ref = _oracle_solve(coracle, dict(variant=0, nc_max=5, ne_max=0), bt)
    unc = (ref["status"] == 2) | (ref["status"] == -1)
    assert unc.sum() >= 100
    assert (o["status"][unc] == ref["status"][unc]).mean() >= 0.9
    err = np.abs(o["foot"] - ref["foot"]).max(axis=1)[unc]
    _artifact("unconverged_iterates.json",
              {"instances": int(unc.sum()), "status_agree": float((o["status"][unc] == ref["status"][unc]).mean()),
               "foot_le_1e-4": float(np.mean(err <= 1e-4)), "foot_le_1e-6": float(np.mean(err <= 1e-6)),
               "foot_le_1e-9": float(np.mean(err <= 1e-9)), "foot_median": float(np.median(err))})
    # (measured on MI355X, profiles/r3/parity: 99.8 % within 1e-4, 99.4 % within 1e-6, median 3e-15)
    assert np.mean(err <= 1e-4 * np.maximum(1.0, np.abs(ref["foot"][unc]).max(axis=1))) >= 0.95, \
        np.mean(err <= 1e-4)
    assert np.mean(err <= 1e-6) >= 0.9, np.mean(err <= 1e-6)
    assert np.isfinite(o["u"]).all()


@pytest.mark.parametrize("variant,prec", [(1, 0), (1, 1), (0, 0)])
def test_factorisation_failure_returns_last_iterate(gpu_lib, coracle, variant, prec):
    """IPOPT's Error_In_Step_Computation path (status -3): a non-finite obstacle (kept because obstacle
    selection is off) makes the KKT matrix non-finite, so the inertia correction cannot regularise it at
    the first iteration.  The instance must stop with status -3 after 0 iterations, as the C oracle does,
    returning the iterate from before the failing iteration bit for bit (= the max_iter = 0 output); the
    other instances of the batch are unaffected.  fp32 (cfg.restoration = IPOPT): the fp32 program's line search
    fails on the non-finite step first and hands the instance to the fp64 program (include/alipmpc.h), so the
    iterate is the fp64 program's max_iter = 0 output."""
    from alipmpc import scenes
    bt = scenes.make_batch(4, seed=3, n_cir=4)
    cir = bt["cir"].copy()
    cir[1, 0, :] = [np.nan, 1.0, 0.5]
    kw = dict(nc_max=4, ne_max=0, select_obs=0)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, **kw))
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], cir, bt["nc"], u0=bt["u0"])
    assert o["status"][1] == -3 and o["iters"][1] == 0
    if prec:
        assert s.lane_handoffs() >= 1
        kw.pop("precision")
    s0 = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, max_iter=0, **kw))
    o0 = s0.solve(bt["x0"], bt["goal"], bt["leg"], cir, bt["nc"], u0=bt["u0"])
    assert np.array_equal(o["u"][1], o0["u"][1]) and np.array_equal(o["foot"][1], o0["foot"][1])
    assert np.isfinite(o["u"][1]).all()
    ref = coracle.solve_batch(coracle.default_cfg(variant, 3, nc_max=4, ne_max=0, select_obs=0), bt["x0"],
                              bt["goal"], bt["leg"], cir, bt["nc"], None, None, bt["u0"])
    assert ref["status"][1] == -3 and ref["iters"][1] == 0
    ok = np.array([0, 2, 3])
    assert (o["status"][ok] != -3).all()


def test_solve_horizon5_scipy_goldens(gpu_lib, golden):
    """BASELINE cfg3 shape (N = 5, 5 circles + 5 ellipses) solutions pinned to the reference NLP:
    SLSQP and trust-constr on the reference objective/constraints (g3_synthetic_modi_n5); to convergence
    (max_iter 100), foothold within 1e-4 on every row both scipy methods agree on."""
    d = golden("g3_synthetic_modi_n5")
    good = (d["agree"] < 1e-8) & (d["viol"] < 1e-8)
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, 5, nc_max=5, ne_max=5, max_iter=100))
    o = s.solve(d["x0"], d["goal"], d["leg"], d["cir"], d["nc"], d["elp"], d["ne"], u0=d["u0"])
    err = np.max(np.abs(o["foot"] - d["foot_ref"]), axis=1)
    assert good.sum() >= 30
    assert np.all(err[good] < 1e-4), err[good].max()
    s32 = gpu_lib.Solver(gpu_lib.default_cfg(0, 5, nc_max=5, ne_max=5, max_iter=100,
                                             precision=gpu_lib.PREC_FP32))
    o32 = s32.solve(d["x0"], d["goal"], d["leg"], d["cir"], d["nc"], d["elp"], d["ne"], u0=d["u0"])
    err32 = np.max(np.abs(o32["foot"] - d["foot_ref"]), axis=1)
    assert np.mean(err32[good] < 1e-3) >= 0.9


def test_cfg1_sig_step_no_obstacles(gpu_lib, golden):
    """BASELINE cfg1 (MPC_LIP_sig_step.py as-is: B = 1, N = 3, no obstacles) through the planner drop-in
    MPCCBFSigStep.gen_control_test (warm start None -> [x0, x0, x0], the reference's own rule), one scene at
    a time, against SLSQP / trust-constr on the reference (g3_synthetic_sig_step_nobs): foothold within
    1e-4 at the reference's cap of 20 iterations on every row both scipy methods agree on; the batched
    launch gives the same plans."""
    import alipmpc.planner as pl
    d = golden("g3_synthetic_sig_step_nobs")
    good = np.nonzero((d["agree"] < 1e-8) & (d["viol"] < 1e-8))[0]
    assert len(good) >= 30
    errs, feet = [], []
    for i in good:
        ss = pl.MPCCBFSigStep([list(d["goal"][i])], [], [], [-0.5, 10.5])
        xs, p0, hd, c2g = ss.gen_control_test(d["x0"][i], d["leg"][i], None)
        errs.append(np.max(np.abs(np.ravel(p0) - d["foot_ref"][i])))
        feet.append(np.ravel(p0))
    assert max(errs) < 1e-4, max(errs)
    s = gpu_lib.Solver(gpu_lib.default_cfg(1, 3, nc_max=0, ne_max=0))
    B = len(good)
    o = s.solve(d["x0"][good], d["goal"][good], d["leg"][good], np.zeros((B, 0, 3)), np.zeros(B, np.int32),
                u0=d["u0"][good])
    assert np.max(np.abs(o["foot"] - np.array(feet))) < 1e-12   # planner: p0 = W(u_1 - A x0) on the host


# ---------------------------------------------------------------- lane program (cfg.program = PROGRAM_LANE)
LANE_CASES = [  # (variant, circles, precision): cfg2/cfg4 shape fp64, sup_learn slots, sig_step, cfg5 (fp32)
    (0, 5, 0), (0, 6, 0), (1, 4, 0), (1, 0, 0), (0, 5, 1)]


@pytest.mark.parametrize("variant,n_cir,prec", LANE_CASES)
def test_lane_program_vs_oracle(gpu_lib, coracle, variant, n_cir, prec):
    """The lane program (one interior-point instance per lane, csrc/lane_solve.inc) against the C oracle on
    a seeded batch: fp64 runs the oracle's algorithm (statuses equal on >= 99 % of the instances, footholds
    and states within 1e-4 where both converge — SURVEY 8d's bar); fp32 with test_fp32_solve_vs_oracle's
    bars (footholds within 1e-3 where both converge, infeasibility verdicts equal on >= 97 %)."""
    from alipmpc import scenes
    B = 4096
    bt = scenes.make_batch(B, seed=800 + n_cir + 10 * variant + 100 * prec, n_cir=n_cir)
    kw = dict(nc_max=n_cir, ne_max=0, program=gpu_lib.PROGRAM_LANE)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, **kw))
    assert s.solve_program().startswith("lane_kernel<3,")
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    ref = _oracle_solve(coracle, dict(variant=variant, nc_max=n_cir, ne_max=0), bt)
    assert np.isfinite(o["u"]).all()
    if prec:
        both = (o["status"] == 0) & (ref["status"] == 0)
        assert both.mean() >= 0.75, both.mean()
        err = np.abs(o["foot"] - ref["foot"]).max(axis=1)
        assert np.mean(err[both] <= 1e-3) >= 0.98, np.mean(err[both] <= 1e-3)
        assert ((o["status"] == 2) == (ref["status"] == 2)).mean() >= 0.97
    else:
        _compare(o, ref, min_conv=0.8, min_agree=0.99, min_status=0.99)
    assert np.allclose(o["u"].reshape(-1, 3, 5), o["x_pred"], rtol=0, atol=0)


@pytest.mark.parametrize("prec", [0, 1])
def test_lane_program_batch_independence(gpu_lib, prec):
    """The lane program's result for an instance does not depend on the batch: one batch above the resident
    lane slots and the same instances in chunks of half the slots are bit-identical; NaN-filled device
    outputs are all written (every instance solved once) and a second launch reproduces the first (the
    queue counters reset)."""
    import torch
    from alipmpc import scenes
    kw = dict(nc_max=5, ne_max=0, program=gpu_lib.PROGRAM_LANE)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, 3, **kw))
    slots = s.solve_slots()
    assert slots >= 16384 and slots % 32 == 0, slots
    B = slots + slots // 2 + 37
    bt = scenes.make_batch_vec(B, seed=91 + prec, n_cir=5, N=3)
    big = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    ch = slots // 2
    parts = [s.solve(bt["x0"][i:i + ch], bt["goal"][i:i + ch], bt["leg"][i:i + ch], bt["cir"][i:i + ch],
                     bt["nc"][i:i + ch], u0=bt["u0"][i:i + ch]) for i in range(0, B, ch)]
    for k in big:
        assert np.array_equal(big[k], np.concatenate([p[k] for p in parts])), k
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    for _ in range(2):
        out = {"u": torch.full((B, 15), float("nan"), dtype=torch.float64, device=dev),
               "foot": torch.full((B, 3), float("nan"), dtype=torch.float64, device=dev),
               "x_pred": torch.full((B, 3, 5), float("nan"), dtype=torch.float64, device=dev),
               "status": torch.full((B,), -99, dtype=torch.int32, device=dev),
               "iters": torch.full((B,), -99, dtype=torch.int32, device=dev)}
        s.solve_device(inp, out)
        torch.cuda.synchronize()
        got = {k: v.cpu().numpy() for k, v in out.items()}
        for k in got:
            assert np.array_equal(got[k], big[k]), k


@pytest.mark.parametrize("variant,prec", [(0, 0), (1, 0), (0, 1)])
def test_lane_program_factorisation_failure(gpu_lib, coracle, variant, prec):
    """Error_In_Step_Computation on the lane program: a non-finite obstacle (obstacle selection off) makes the
    KKT matrix unfactorisable at the first iteration -> status -3 after 0 iterations with the iterate from
    before the failing iteration (= the max_iter = 0 output, bit for bit), as the C oracle; the other lanes
    of the wave are unaffected."""
    from alipmpc import scenes
    bt = scenes.make_batch(4, seed=3, n_cir=4)
    cir = bt["cir"].copy()
    cir[1, 0, :] = [np.nan, 1.0, 0.5]
    kw = dict(nc_max=4, ne_max=0, select_obs=0, program=gpu_lib.PROGRAM_LANE)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    o = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, **kw)).solve(bt["x0"], bt["goal"], bt["leg"], cir, bt["nc"],
                                                                    u0=bt["u0"])
    assert o["status"][1] == -3 and o["iters"][1] == 0
    o0 = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, max_iter=0, **kw)).solve(bt["x0"], bt["goal"], bt["leg"], cir,
                                                                                bt["nc"], u0=bt["u0"])
    assert np.array_equal(o["u"][1], o0["u"][1]) and np.array_equal(o["foot"][1], o0["foot"][1])
    assert np.isfinite(o["u"][1]).all()
    assert (o["status"][[0, 2, 3]] != -3).all()


@pytest.mark.parametrize("variant", [0, 1])
def test_lane_program_rollout_vs_oracle(gpu_lib, coracle, variant):
    """Closed-loop rollouts (retired instances skipped through the lane work queue) on the lane program against
    the oracle's closed loop, with test_rollout_matches_oracle's bars."""
    from alipmpc import scenes
    N, B, S = 3, 256, 6
    bt = scenes.make_batch(B, seed=191 + variant, n_cir=5, N=N)
    x0 = bt["x0"].copy()
    x0[:16, 0:2] = bt["goal"][:16] - np.array([0.3, 0.2])
    u0 = np.tile(x0, (1, N))
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, nc_max=5, ne_max=0, program=gpu_lib.PROGRAM_LANE))
    o = s.rollout(x0, bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=u0, steps=S)
    ref = coracle.rollout_batch(coracle.default_cfg(variant, N, nc_max=5, ne_max=0), x0, bt["goal"], bt["leg"],
                                bt["cir"], bt["nc"], None, None, u0, None, steps=S, nthreads=8)
    same_status = (o["status"] == ref["status"]).all(1)
    fo, fr = np.nan_to_num(o["foot"], nan=1e9), np.nan_to_num(ref["foot"], nan=1e9)
    same_path = (np.abs(fo - fr) <= 1e-4 * np.maximum(1.0, np.abs(fr))).all((1, 2))
    assert (same_status & same_path).mean() >= 0.85
    assert (o["steps_to_goal"] == ref["steps_to_goal"]).mean() >= 0.9
    for b in np.nonzero(o["steps_to_goal"] > 0)[0]:
        assert (o["status"][b, o["steps_to_goal"][b]:] == gpu_lib.ROLLOUT_DONE).all()


def test_lane_program_unsupported_shapes(gpu_lib):
    """The lane program serves N = 3 with circles only (<= 6 slots): other shapes are refused at create."""
    for kw in (dict(N=5), dict(ne_max=2), dict(nc_max=8)):
        N = kw.pop("N", 3)
        cfg = gpu_lib.default_cfg(0, N, **{"nc_max": 5, "ne_max": 0, **kw}, program=gpu_lib.PROGRAM_LANE)
        with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
            gpu_lib.Solver(cfg)
    with pytest.raises(RuntimeError, match="EUNSUPPORTED"):
        gpu_lib.Solver(gpu_lib.default_cfg(gpu_lib.VARIANT_DD, 3, nc_max=5, ne_max=0, program=gpu_lib.PROGRAM_LANE))


# ---------------------------------------------------------------- closed loop at the control rate
def _cl_first_departure(o, ref, thr=1e-6):
    """Per episode, the first tick (flattened step * f_cyc + tick) at which the closed loop leaves the oracle's path:
    the controller command (a function of the tick's plan) differs by more than thr, or the status or the iteration
    count differs; B x 1 array, S * f_cyc where it never does."""
    B = o["status"].shape[0]
    st_o, st_r = o["status"].reshape(B, -1), ref["status"].reshape(B, -1)
    it_o, it_r = o["iters"].reshape(B, -1), ref["iters"].reshape(B, -1)
    ad = np.nan_to_num(np.abs(o["action"] - ref["action"]).max(-1), nan=np.inf).reshape(B, -1)
    both_nan = (np.isnan(o["action"]).all(-1) & np.isnan(ref["action"]).all(-1)).reshape(B, -1)
    diff = ((ad > thr) & ~both_nan) | (st_o != st_r) | (it_o != it_r)
    first = np.where(diff.any(1), np.argmax(diff, 1), diff.shape[1])
    return first, ad


def _cl_drift_table(o, ref, F, tol=1e-4):
    """Where each drifting episode leaves the oracle: for every step whose touchdown foothold
    converged on both sides but differs by more than tol, the episode's first departure tick (_cl_first_departure) with
    both sides' status and iteration count at that tick and at the tick before."""
    B, S = o["foot"].shape[:2]
    err = np.abs(o["foot"] - ref["foot"]).max(-1)
    conv = (o["status"][:, :, -1] == 0) & (ref["status"][:, :, -1] == 0)
    st_o, st_r = o["status"].reshape(B, -1), ref["status"].reshape(B, -1)
    it_o, it_r = o["iters"].reshape(B, -1), ref["iters"].reshape(B, -1)
    first, ad = _cl_first_departure(o, ref)
    rows = []
    for b, s in zip(*np.nonzero(conv & (err > tol))):
        t = int(first[b]) if first[b] < S * F else -1
        row = {"episode": int(b), "step": int(s), "foot_err": float(err[b, s]), "first_tick": t,
               "first_step_tick": [t // F, t % F] if t >= 0 else None}
        if t >= 0:
            row.update(gpu=[int(st_o[b, t]), int(it_o[b, t])], oracle=[int(st_r[b, t]), int(it_r[b, t])],
                       action_err=float(ad[b, t]),
                       prev_gpu=[int(st_o[b, t - 1]), int(it_o[b, t - 1])] if t > 0 else None,
                       prev_oracle=[int(st_r[b, t - 1]), int(it_r[b, t - 1])] if t > 0 else None)
            # the tick's own solve converged on both sides in the same number of iterations, yet the plans differ by
            # more than 1e-6: a kernel / oracle discrepancy rather than a drift after an unconverged iterate
            row["converged_same_path"] = bool(st_o[b, t] == 0 and st_r[b, t] == 0 and it_o[b, t] == it_r[b, t])
        rows.append(row)
    return rows


def _self_drift(tag):
    """The oracle loop's own sensitivity for a closed-loop case (tools/self_drift.py, profiles/r6/parity/self_drift.json):
    per statistic the smallest value over its fp64 perturbation rows (one ulp at the start, one ulp at every solve, the
    tolerance at every solve) — the floor a GPU-vs-oracle bar is set against."""
    import json
    import os
    fn = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r6", "parity",
                      "self_drift.json")
    with open(fn) as fh:
        cases = json.load(fh)["cases"]
    rows = [cases[k] for k in (tag, tag + "_jitter", tag + "_toljitter") if k in cases]
    return {k: min(r[k] for r in rows) for k in ("status_agree", "iters_within_1", "steps_to_goal_agree", "foot_le_1e-3",
                                                  "foot_le_1e-4")}


@pytest.mark.parametrize("variant,kick,program,prec", [(0, 0.0, 0, 0), (0, 0.05, 0, 0), (1, 0.05, 0, 0), (0, 0.05, 1, 0),
                                                       (0, 0.05, 1, 1)])
def test_closed_loop_matches_oracle(gpu_lib, coracle, variant, kick, program, prec):
    """alipmpc_closed_loop_batch (f_cyc = 40 solves per walking step, heading tube + avg_hd at each touchdown,
    get_next_states projection at rest_t = T - i T / 40, warm start from the previous plan, stance switch and
    close-to-goal stop as main_sim_mpc.py:65-135) against oracle.closed_loop_batch on the same seeded episodes:
    per-tick statuses, iteration counts, steps to the goal and converged touchdown footholds agree on the large
    majority of ticks / steps (each tick warm-starts from the previous plan, so a rounding-level difference can
    change an iteration count or move an unconverged iterate, and the episode then drifts)."""
    from alipmpc import scenes
    B, S, F = 48, 4, 40
    bt = scenes.make_batch(B, seed=520 + variant + int(kick * 100), n_cir=5)
    x0 = bt["x0"].copy()
    x0[:12, 0:2] = bt["goal"][:12] - (np.array([1.0, 0.8]) if variant == 1 else np.array([0.6, 0.5]))
    leg = bt["leg"].astype(np.int8)
    # a consistent start: x0 is the state as the stance switches onto the first planned foothold of a solve from
    # x0 (the MPC's x_1 = flow of x0 about u_0 over T), leg the parity that solve was posed with
    co = coracle.default_cfg(variant, 3, nc_max=5, ne_max=0)
    foot0 = coracle.solve_batch(co, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None,
                                np.tile(x0, (1, 3)))["foot"][:, 0:2]
    kw = dict(precision=gpu_lib.PREC_FP32) if prec else {}
    cfg = gpu_lib.default_cfg(variant, 3, nc_max=5, ne_max=0, program=program, **kw)
    o = gpu_lib.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F,
                                        kick=kick, seed=7)
    if prec:   # the fp32 program against the oracle at its own tolerances (a fair comparator)
        co = coracle.default_cfg(variant, 3, nc_max=5, ne_max=0, tol=cfg.tol, acceptable_tol=cfg.acceptable_tol)
    ref = coracle.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, kick=kick,
                                    seed=7)
    assert o["status"].shape == (B, S, F)
    err = np.abs(o["foot"] - ref["foot"]).max(-1)
    conv = (o["status"][:, :, -1] == 0) & (ref["status"][:, :, -1] == 0)
    drift = _cl_drift_table(o, ref, F)
    tag = f"{variant}_{kick}_{program}" + ("_fp32" if prec else "")
    _artifact(f"closed_loop_{tag}.json",
              {"converged_steps": int(conv.sum()), "foot_le_1e-3": float((err[conv] <= 1e-3).mean()),
               "foot_le_1e-4": float((err[conv] <= 1e-4).mean()), "foot_le_1e-6": float((err[conv] <= 1e-6).mean()),
               "foot_median": float(np.median(err[conv])), "status_agree": float((o["status"] == ref["status"]).mean()),
               "iters_within_1": float((np.abs(o["iters"] - ref["iters"]) <= 1).mean()),
               "steps_to_goal_agree": float((o["steps_to_goal"] == ref["steps_to_goal"]).mean()),
               "status_m3": [int((o["status"] == -3).sum()), int((ref["status"] == -3).sum())]})
    _artifact(f"closed_loop_drift_{tag}.json", drift)
    # Error_In_Step_Computation no more often than the oracle's loop
    assert (o["status"] == -3).sum() <= (ref["status"] == -3).sum()
    if prec:
        # fp32 lane program (BASELINE cfg5) against the oracle at the same tolerances (1e-4 / 1e-3): iteration counts
        # and unconverged iterates still differ with the precision; test_fp32_solve_vs_oracle's foothold bar on the
        # converged touchdowns
        assert (o["steps_to_goal"] == ref["steps_to_goal"]).mean() >= 0.85
        assert conv.sum() >= 0.3 * B * S
        # (both sides stop anywhere inside the 1e-4 tolerance ball and warm-start the next tick from there — the
        # iteration counts differ on ~18 % of the ticks — so the touchdowns of 4 chained steps drift apart: r5 measured
        # 0.79-0.82 within 1e-3 against the same-tolerance oracle's loop, a statistic of the loop's sensitivity more
        # than of the kernel.  The kernel's own bar is the same-inputs form: every solve both sides converge on lands
        # within 1e-3 of the oracle's, test_closed_loop_same_inputs_match_oracle.)
        assert (err[conv] <= 1e-3).mean() >= 0.75 and np.median(err[conv]) <= 1e-4, (err[conv] <= 1e-3).mean()
        np.testing.assert_allclose(o["hd"][:, 0], ref["hd"][:, 0], rtol=0, atol=1e-12)
        np.testing.assert_allclose(o["x"][:, 0], x0, rtol=0, atol=0)
        assert np.array_equal(np.isnan(o["action"]).all(-1), o["status"] == gpu_lib.ROLLOUT_DONE)
        return
    # Each statistic against the oracle loop's OWN sensitivity (r6): the same episodes through the
    # oracle twice, the second perturbed by rounding-size amounts (one ulp at the start, one ulp / the tolerance at
    # every solve: tools/self_drift.py, profiles/r6/parity/self_drift.json); two loops that differ only by rounding
    # drift apart that much, so the GPU-vs-oracle bar is that figure minus 0.03.
    sd = _self_drift(tag)
    gstat = {"status_agree": (o["status"] == ref["status"]).mean(),
             "iters_within_1": (np.abs(o["iters"] - ref["iters"]) <= 1).mean(),
             "steps_to_goal_agree": (o["steps_to_goal"] == ref["steps_to_goal"]).mean(),
             "foot_le_1e-3": (err[conv] <= 1e-3).mean(), "foot_le_1e-4": (err[conv] <= 1e-4).mean()}
    for k, v in gstat.items():
        assert v >= sd[k] - 0.03, (k, v, sd[k])
    assert conv.sum() >= 0.4 * B * S
    assert np.median(err[conv]) <= 1e-6
    # every drift starts at an unconverged solve (iteration cap / infeasible: the returned iterate is path-dependent)
    # or where the iteration count differs (a warm start on the tolerance boundary), never inside a converged solve
    # that took the same iterations (r4 measurement: profiles/r4/parity/closed_loop_drift_*.json)
    assert not any(r.get("converged_same_path") for r in drift), [r for r in drift if r.get("converged_same_path")]
    # and the steps reached on the oracle's own path (no departure up to the touchdown tick) match it
    first, _ = _cl_first_departure(o, ref)
    on_path = (first[:, None] > np.arange(S)[None, :] * F + F - 1) & conv
    assert on_path.sum() >= 0.5 * conv.sum() and (err[on_path] <= 1e-6).all(), (on_path.sum(), err[on_path].max())
    # the first step's heading inputs depend on the initial state alone
    np.testing.assert_allclose(o["hd"][:, 0], ref["hd"][:, 0], rtol=0, atol=1e-12)
    np.testing.assert_allclose(o["x"][:, 0], x0, rtol=0, atol=0)
    # controller commands (gen_nex_foot_input + gen_tsc_control per tick): NaN exactly after the stops, and
    # equal to the oracle's on the steps both loops entered from the same touchdown state with the same turn
    # input, at ticks where this and the previous solve took the same path (status, iteration count)
    assert np.array_equal(np.isnan(o["action"]).all(-1), o["status"] == gpu_lib.ROLLOUT_DONE)
    S_, F_ = o["status"].shape[1:]
    step_ok = (np.abs(o["x"][:, :S_] - ref["x"][:, :S_]).max(-1) <= 1e-9) & (np.abs(o["hd"] - ref["hd"]).max(-1) <= 1e-9)
    st_same = (o["status"] == ref["status"]) & (o["iters"] == ref["iters"]) & (o["status"] >= 0)
    prev = np.concatenate([np.ones((B, S_, 1), bool), st_same[:, :, :-1]], axis=2)
    same = st_same & prev & step_ok[:, :, None]
    aerr = np.abs(o["action"] - ref["action"]).max(-1)[same]
    assert same.mean() >= 0.4, same.mean()
    assert (aerr <= 1e-6).mean() >= 0.95 and np.median(aerr) <= 1e-9, ((aerr <= 1e-6).mean(), np.median(aerr))
    assert (o["steps_to_goal"][:12] > 0).sum() >= 4
    done = o["status"] == gpu_lib.ROLLOUT_DONE
    for b in np.nonzero(o["steps_to_goal"] > 0)[0]:
        assert done[b, o["steps_to_goal"][b]:].all() and not done[b, :o["steps_to_goal"][b]].any()


@pytest.mark.parametrize("program,prec", [(1, 1), (1, 0), (0, 0)])
def test_closed_loop_step_failures_vs_oracle(gpu_lib, coracle, program, prec):
    """Error_In_Step_Computation (status -3) in the closed loop no more often than in the oracle's loop (VERDICT r3
    item 1): 4096 episodes x 1 walking step (40 ticks) of cfg5's scene distribution, a quarter of them started
    within a metre of the goal, stance on the first foothold the same program plans from x0 (bench.py's
    closed_loop_rate start).  The r3 lane loop logged -3 on 0.14 % (fp32) / 0.005 % (fp64) of the ticks: plans whose
    last state sat exactly on the goal, where the target heading's derivatives are 0 / 0;
    each such plan warm-started the next tick at the same point, so the episode stayed at -3."""
    from alipmpc import scenes
    B, F = 4096, 40
    bt = scenes.make_batch_vec(B, seed=4242, n_cir=5, N=3)
    rng = np.random.default_rng(4243)
    x0 = bt["x0"].copy()
    near = np.arange(B) % 4 == 0
    ang = rng.uniform(np.pi, 1.5 * np.pi, near.sum())
    rad = rng.uniform(0.2, 1.0, near.sum())
    x0[near, 0:2] = bt["goal"][near] + np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
    leg = bt["leg"].astype(np.int8)
    kw = dict(nc_max=5, ne_max=0, program=program)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, 3, **kw))
    foot0 = s.solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2].copy()
    o = s.closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=F)
    ref = coracle.closed_loop_batch(coracle.default_cfg(0, 3, nc_max=5, ne_max=0), x0, foot0, bt["goal"], leg,
                                    bt["cir"], bt["nc"], steps=1, f_cyc=F, nthreads=16)
    # the comparator at the program's own tolerances (fp32: tol 1e-4 / acceptable 1e-3), so that precision effects
    # are told from tolerance effects
    c = s.cfg
    same = coracle.closed_loop_batch(coracle.default_cfg(0, 3, nc_max=5, ne_max=0, tol=c.tol,
                                                         acceptable_tol=c.acceptable_tol), x0, foot0, bt["goal"], leg,
                                     bt["cir"], bt["nc"], steps=1, f_cyc=F, nthreads=16) if prec else ref
    cnt = lambda st: {str(k): int(v) for k, v in zip(*np.unique(st[st != -10], return_counts=True))}  # noqa: E731
    _artifact(f"closed_loop_m3_{program}_{prec}.json", {"episodes": B, "ticks": int((o["status"] != -10).sum()),
                                                        "gpu": cnt(o["status"]), "oracle": cnt(ref["status"]),
                                                        "oracle_same_tol": cnt(same["status"])})
    # (fp32, r5: the goal-frame fp32 lane build had logged -3 on 0.03 % of the ticks — iterates converging onto the goal,
    # where a goal-frame |g - p| kept shrinking to ~1e-150 and the heading term's curvature 1 / |g - p|^4 overflowed the
    # KKT matrix; the objective's goal differences are now taken in map coordinates, as the oracle rounds them: none)
    assert (o["status"] == -3).sum() <= (same["status"] == -3).sum(), (cnt(o["status"]), cnt(same["status"]))
    # iteration-cap stops and converged ticks as the same-tolerance oracle's (r4's fp32 loop: 3x the cap stops, 74 %
    # vs 91 % converged — the fp32 heading error near the goal)
    ran = o["status"] != -10
    n_cap, n_cap_ref = (o["status"] == -1).sum(), (same["status"] == -1).sum()
    assert n_cap <= 1.25 * n_cap_ref + 20, (cnt(o["status"]), cnt(same["status"]))
    assert (o["status"][ran] == 0).mean() >= (same["status"][ran] == 0).mean() - 0.03, (cnt(o["status"]),
                                                                                        cnt(same["status"]))
    # the episodes near the goal reach it: the singular region is exercised
    assert (o["steps_to_goal"][near] > 0).sum() > 0


@pytest.mark.parametrize("N,nc,ne,variant", [(3, 5, 0, 0), (3, 5, 0, 1), (6, 5, 5, 0), (2, 20, 0, 0), (1, 4, 20, 1)])
def test_eval_batch_vs_oracle(gpu_lib, coracle, N, nc, ne, variant):
    """The Jacobian sweep (eval_kernel, 16 lanes per instance, grid-stride) on a ragged batch of seeded random
    scenes against the C oracle's reference callbacks (select_obs and detour on): every output of every
    instance, including > 16 obstacle slots (select_obs / detour in two 16-slot passes)."""
    from alipmpc import scenes
    B = 5003
    bt = scenes.make_batch_vec(B, seed=17 + N, n_cir=nc, n_elp=ne, N=N)
    # the generator mixes part of the circles into ellipses: trim / pad (shifted copies) to exactly nc, ne slots
    for key, cnt, want, d in (("cir", "nc", nc, 3), ("elp", "ne", ne, 5)):
        if want == 0:
            continue
        a = bt[key][:, :want]
        while a.shape[1] < want:
            extra = min(a.shape[1], want - a.shape[1])
            a = np.concatenate([a, a[:, :extra] + np.r_[0.7, -0.6, np.zeros(d - 2)]], axis=1)
        bt[key] = np.ascontiguousarray(a)
        bt[cnt] = np.clip(bt[cnt] + want, 0, want).astype(np.int32)
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, nc_max=nc, ne_max=ne))
    u = bt["u0"] + 0.05 * np.random.default_rng(3).standard_normal(bt["u0"].shape)
    o = s.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt.get("elp"), bt.get("ne"), u)
    r = coracle.eval_batch(coracle.default_cfg(variant, N, nc_max=nc, ne_max=ne), bt["x0"], bt["goal"], bt["leg"],
                           bt["cir"], bt["nc"], bt.get("elp"), bt.get("ne"), u)
    assert rel(o["f"], r["f"]) < 1e-11
    assert rel(o["grad"], r["grad"]) < 1e-11
    assert np.array_equal(o["row_active"], r["row_active"])
    assert rel(o["c"], r["c"]) < 1e-11 and rel(o["J"], r["J"]) < 1e-11
    assert np.array_equal(o["cl"], r["cl"]) and np.array_equal(o["cu"], r["cu"])


def test_nominal_gait_matches_reference_helpers(gpu_lib):
    """alipmpc_nominal_gait_batch against the planner's restatement of alip_des_vel / cal_foot_with_veldes
    (MPC_LIP_modi.py:181-194; pinned to the reference by tests/test_oracle.py's g4 goldens): both legs, a given
    target velocity, host and device pointers."""
    import torch
    from alipmpc import planner as pl
    rng = np.random.default_rng(11)
    B = 1000
    x = rng.normal(size=(B, 5)) * np.array([3.0, 3.0, 0.5, 0.5, 1.0])
    leg = np.where(rng.random(B) < 0.5, -1, 1).astype(np.int8)
    mp = pl.MPCCBF([[10, 10]], [], [], [], [], [-0.5, 10.5])
    s = gpu_lib.Solver(gpu_lib.default_cfg(0))
    vd, foot = s.nominal_gait(x, leg, vx_max=0.6)
    for b in range(0, B, 7):
        v_ref = mp.alip_des_vel(0.6, int(leg[b]))
        np.testing.assert_allclose(vd[b], v_ref, rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(foot[b], mp.cal_foot_with_veldes(x[b], v_ref), rtol=1e-12, atol=1e-12)
    tgt = rng.normal(size=(B, 2)) * 0.3
    vd2, foot2 = s.nominal_gait(x, vel_des=tgt)
    assert np.array_equal(vd2, tgt)
    for b in range(0, B, 11):
        np.testing.assert_allclose(foot2[b], mp.cal_foot_with_veldes(x[b], tgt[b]), rtol=1e-12, atol=1e-12)
    # device pointers on the current stream give the same bits
    dev = torch.device("cuda", 0)
    xt, lt = torch.from_numpy(x).to(dev), torch.from_numpy(leg).to(dev)
    vt, ft = torch.empty((B, 2), dtype=torch.float64, device=dev), torch.empty((B, 2), dtype=torch.float64, device=dev)
    from alipmpc._lib import _ptr
    rc = s._L.alipmpc_nominal_gait_batch(s._h, B, 0.6, _ptr(xt), _ptr(lt), None, _ptr(vt), _ptr(ft),
                                         gpu_lib._lib._stream_arg(torch.cuda.current_stream()))
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(ft.cpu().numpy(), foot) and np.array_equal(vt.cpu().numpy(), vd)


@pytest.mark.parametrize("variant,nc,B", [(0, 5, 5003), (1, 5, 4099), (0, 0, 1000), (0, 3, 777), (1, 6, 2048), (0, 6, 65)])
def test_sweep_kernel_bit_identical_to_group_eval(gpu_lib, variant, nc, B, monkeypatch):
    """The eval hook's sweep kernel (N = 3, circle slots: lane-per-instance set-up + wave-cooperative J stores)
    against eval_kernel (16 lanes per instance; ALIPMPC_EVAL_KERNEL=group) on a ragged batch with select_obs /
    detour on: the same bits for f, grad f, goal, bounds and activity, rounding-level agreement for c and J
    (fma contraction); both are pinned to the reference callbacks by the tests above.
    Also: a partial output set through device pointers (the bench's f / grad / c / J) writes the same J."""
    import torch
    from alipmpc import scenes
    bt = scenes.make_batch_vec(B, seed=23 + nc, n_cir=max(nc, 1), N=3)
    cir = np.ascontiguousarray(bt["cir"][:, :nc]) if nc else np.zeros((B, 0, 3))
    rng = np.random.default_rng(5)
    ncnt = np.where(rng.random(B) < 0.3, rng.integers(0, nc + 1, B), np.clip(bt["nc"], 0, nc)).astype(np.int32)
    u = bt["u0"] + 0.05 * rng.standard_normal(bt["u0"].shape)
    cfg = gpu_lib.default_cfg(variant, 3, nc_max=nc, ne_max=0)
    outs = []
    for kern in ("sweep", "group"):
        if kern == "group":
            monkeypatch.setenv("ALIPMPC_EVAL_KERNEL", "group")
        s = gpu_lib.Solver(cfg)
        outs.append(s.eval(bt["x0"], bt["goal"], bt["leg"], cir, ncnt, None, None, u))
    a, g = outs
    for k in ("f", "grad", "goal_eff", "row_active", "cl", "cu"):
        assert np.array_equal(a[k], g[k]), k
    # row values and J rows: the same formulas, but the compiler's fma contraction of a row's arithmetic may differ
    # between the two kernels (rounding level)
    for k in ("c", "J"):
        assert np.max(np.abs(a[k] - g[k]) / np.maximum(1.0, np.abs(g[k]))) <= 1e-14, k
        assert np.array_equal(a[k] == 0, g[k] == 0), k
    monkeypatch.delenv("ALIPMPC_EVAL_KERNEL")
    s = gpu_lib.Solver(cfg)
    dev = torch.device("cuda", 0)
    inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
           "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(cir).to(dev),
           "nc": torch.from_numpy(ncnt).to(dev), "u": torch.from_numpy(u).to(dev)}
    J = torch.full((B, s.m_max, 15), np.nan, dtype=torch.float64, device=dev)
    s.eval_device(inp, {"J": J})
    torch.cuda.synchronize()
    assert np.array_equal(J.cpu().numpy(), a["J"])


@pytest.mark.parametrize("variant,nc,B", [(0, 5, 5003), (1, 3, 4161), (0, 0, 97)])
def test_sweep_kernel_launch_shapes_bit_identical(gpu_lib, variant, nc, B, monkeypatch):
    """The sweep kernel's launch shapes (32 instances per wave x 2 waves per workgroup, the default; 64 x 1,
    ALIPMPC_SWEEP_SHAPE=641) hand instances to lanes differently but run the same per-instance arithmetic: every
    output bit-equal, on ragged batches (B not a multiple of either chunk) with select_obs / detour on."""
    from alipmpc import scenes
    bt = scenes.make_batch_vec(B, seed=41 + nc, n_cir=max(nc, 1), N=3)
    cir = np.ascontiguousarray(bt["cir"][:, :nc]) if nc else np.zeros((B, 0, 3))
    ncnt = np.clip(bt["nc"], 0, nc).astype(np.int32)
    u = bt["u0"] + 0.05 * np.random.default_rng(9).standard_normal(bt["u0"].shape)
    cfg = gpu_lib.default_cfg(variant, 3, nc_max=nc, ne_max=0)
    outs = []
    for shape in (None, "641"):
        if shape:
            monkeypatch.setenv("ALIPMPC_SWEEP_SHAPE", shape)
        outs.append(gpu_lib.Solver(cfg).eval(bt["x0"], bt["goal"], bt["leg"], cir, ncnt, None, None, u))
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("program,variant,N,n_cir,n_elp", [
    ("wave", 0, 3, 5, 0), ("wave", 1, 3, 5, 0), ("wave", 0, 5, 5, 5), ("wave", 2, 3, 5, 0),
    ("lane", 0, 3, 5, 0), ("lane", 1, 3, 5, 0)])
@pytest.mark.parametrize("max_iter", [1, 3])
def test_first_iterates_pin_solve_callbacks(gpu_lib, coracle, program, variant, N, n_cir, n_elp, max_iter):
    """The solve programs evaluate the NLP with their own row code (wave: row_value / row_coef; lane: row_eval /
    eval_point; DD: its rollout rows), separate from the eval kernels the g1 goldens pin.  Their first
    interior-point iterates are a direct check of those callbacks: the Newton step at the reference's warm start
    is a function of f, grad f, c, J (and the Hessian) there, so u after 1 and 3 iterations must equal the C
    oracle's (whose callbacks are pinned to the reference, tests/test_oracle.py) to rounding on nearly every
    instance (Gauss-Jordan vs Cholesky and fma contraction are the only differences)."""
    from alipmpc import scenes
    B = 512
    kw = dict(nc_max=n_cir, ne_max=n_elp, max_iter=max_iter)
    if program == "lane":
        kw["program"] = gpu_lib.PROGRAM_LANE
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, **kw))
    if variant == 2:   # DD (MPC_DD_sig_step.py): unicycle states, warm start = the last command repeated
        bt = _dd_batch(B, seed=71 + N, n_cir=n_cir, N=N)
        o = s.solve(bt["x0"], bt["goal"], None, bt["cir"], bt["nc"], u0=bt["u0"], last_u=bt["last_u"])
        cc = coracle.default_cfg(2, N, nc_max=n_cir, ne_max=n_elp, max_iter=max_iter)
        ref = coracle.solve_batch_dd(cc, bt["x0"], bt["goal"], bt["cir"], bt["nc"], None, None, bt["u0"],
                                     bt["last_u"], nthreads=8)
    else:
        bt = scenes.make_batch_vec(B, seed=71 + N + 3 * variant, n_cir=n_cir, n_elp=n_elp, N=N)
        o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt.get("elp"), bt.get("ne"), u0=bt["u0"])
        ref = _oracle_solve(coracle, dict(variant=variant, N=N, nc_max=n_cir, ne_max=n_elp, max_iter=max_iter), bt)
    assert np.array_equal(o["iters"] <= max_iter, np.ones(B, bool))
    scale = np.maximum(1.0, np.abs(ref["u"]))
    err = (np.abs(o["u"] - ref["u"]) / scale).max(axis=1)
    assert np.mean(err <= 1e-8) >= 0.99, (np.mean(err <= 1e-8), np.median(err))
    assert np.median(err) <= 1e-11, np.median(err)
    assert (o["status"] == ref["status"]).mean() >= 0.99


@pytest.mark.parametrize("variant,kick,B", [(0, 0.0, 3000), (1, 0.05, 3000), (0, 0.0, 5000)])
def test_closed_loop_launch_order_bit_identical(gpu_lib, variant, kick, B, monkeypatch):
    """The closed loop can launch each tick's solves longest-first (opt-in ALIPMPC_CL_ORDER=1: by the last tick's iteration counts; a counting
    sort whose ties fall in any order).  The order changes when and on which SIMD an instance runs, never its
    arithmetic: every output equals the identity-order loop's (ALIPMPC_CL_ORDER=0) bit for bit, on a batch above
    one wave per SIMD's worth of instances with stops, kicks and infeasible scenes.  B = 5000 is above the 4096
    resident slots: the work-queue launch with the order and inactive (stopped) episodes."""
    from alipmpc import scenes
    S, F = 2, 40
    bt = scenes.make_batch(B, seed=610 + variant, n_cir=5)
    x0 = bt["x0"].copy()
    x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
    leg = bt["leg"].astype(np.int8)
    cfg = gpu_lib.default_cfg(variant, 3, nc_max=5, ne_max=0)
    s0 = gpu_lib.Solver(cfg)
    foot0 = s0.solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
    outs = []
    for order in ("1", "0"):
        monkeypatch.setenv("ALIPMPC_CL_ORDER", order)
        outs.append(gpu_lib.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F,
                                                    kick=kick, seed=3))
    a, b = outs
    assert (a["status"] == 2).sum() > 0 and (a["steps_to_goal"] > 0).sum() > 0
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("variant,N,n_cir,n_elp,prec,B", [(0, 3, 5, 0, 0, 4000), (1, 3, 5, 0, 0, 3000),
                                                          (0, 5, 5, 5, 0, 1500), (0, 3, 5, 0, 1, 4000)])
def test_split_launch_bit_identical(gpu_lib, variant, N, n_cir, n_elp, prec, B, monkeypatch):
    """A batch that fits the resident slots runs as a split launch (phase 1 up to ALIPMPC_SPLIT_IT iterations, the
    loop state of the unfinished instances to records, phase 2 resumes them one wave each).  The record holds the
    exact loop state, so every output equals the one-phase launch's (ALIPMPC_SPLIT_IT=0) bit for bit, whatever the
    cut — including cuts inside restorations, at the iteration cap's edge and in fp32."""
    from alipmpc import scenes
    bt = scenes.make_batch_vec(B, seed=900 + N + variant + 7 * prec, n_cir=n_cir, n_elp=n_elp, N=N)
    kw = dict(nc_max=n_cir, ne_max=n_elp)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    cfg = gpu_lib.default_cfg(variant, N, **kw)
    outs = {}
    for k in ("0", "1", "7", "16", str(cfg.max_iter - 1)):
        # phase 2 one wave per instance, and with team records (ALIPMPC_SPLIT_TR: an instance at that many
        # line-search trials is cut early and resumes on a team, the workgroup's 4 waves in lockstep, consecutive
        # trials per round)
        for tr in (("0", "3", "12") if k != "0" else (("0", "12") if not prec else ("0",))):
            monkeypatch.setenv("ALIPMPC_SPLIT_IT", k)
            monkeypatch.setenv("ALIPMPC_SPLIT_TR", tr)
            s = gpu_lib.Solver(cfg)
            assert s.solve_slots() >= B
            outs[k + "/" + tr] = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt.get("elp"),
                                         bt.get("ne"), u0=bt["u0"])
    ref = outs.pop("0/0")
    assert (ref["iters"] > 16).sum() > 0 and (ref["status"] == 2).sum() > 0
    for k, o in outs.items():
        for key in ref:
            assert np.array_equal(o[key], ref[key]), (k, key)


def test_split_launch_graph_capture_keeps_its_records(gpu_lib):
    """A split-launch solve captured into a HIP graph (torch.cuda.CUDAGraph) at B = 1000, an eager B = 4000 solve on
    the capture stream afterwards, then the graph replayed on that stream: the replay's outputs equal an eager B = 1000
    solve's bit for bit.  (Each stream's record buffer is sized once for the resident slots and kept until destroy,
    include/alipmpc.h; r3 re-allocated it for the larger batch and the replay wrote into freed memory — ADVICE r3.)"""
    import torch
    from alipmpc import scenes
    s = gpu_lib.Solver(gpu_lib.default_cfg(0, 3, nc_max=5, ne_max=0))
    assert s.solve_launches(1000)[0] == 2 and s.solve_launches(4000)[0] == 2
    dev = torch.device("cuda", 0)

    def inputs(B, seed):
        bt = scenes.make_batch_vec(B, seed=seed, n_cir=5, N=3)
        d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
        d["leg"] = d["leg"].to(torch.int8)
        d["nc"] = d["nc"].to(torch.int32)
        return d

    def outputs(B):
        f = lambda *sh: torch.full(sh, float("nan"), dtype=torch.float64, device=dev)  # noqa: E731
        return {"u": f(B, 15), "foot": f(B, 3), "x_pred": f(B, 3, 5),
                "status": torch.full((B,), -99, dtype=torch.int32, device=dev),
                "iters": torch.full((B,), -99, dtype=torch.int32, device=dev)}
    small, big = inputs(1000, 61), inputs(4000, 62)
    ref = outputs(1000)
    s.solve_device(small, ref)
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    og = outputs(1000)
    with torch.cuda.stream(st):
        s.solve_device(small, og)       # the capture stream's first solve: allocates its record buffer
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        s.solve_device(small, og)
    ob = outputs(4000)
    with torch.cuda.stream(st):
        s.solve_device(big, ob)         # a larger batch on the capture stream
        for v in og.values():
            v.fill_(-7)
        g.replay()
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(og[k], ref[k]), k
    assert (ob["status"] != -99).all()


@pytest.mark.parametrize("variant,kick,B,prec", [(0, 0.0, 3000, 0), (1, 0.05, 3000, 0), (0, 0.0, 4096, 1)])
def test_closed_loop_split_team_bit_identical(gpu_lib, variant, kick, B, prec, monkeypatch):
    """The closed loop's per-tick solves run as split launches (ALIPMPC_CL_SPLIT_IT: phase-1 cap, then the
    unfinished instances resume from their records; ALIPMPC_CL_SPLIT_TR: an instance at that many line-search trials
    is cut early and resumes as a team of 4 waves that evaluates consecutive trials in one round), with the episodes
    in groups on streams of their own or not.  Every output equals the one-phase, one-group loop's bit for bit."""
    from alipmpc import scenes
    S, F = 2, 40
    bt = scenes.make_batch(B, seed=710 + variant + 3 * prec, n_cir=5)
    x0 = bt["x0"].copy()
    x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
    leg = bt["leg"].astype(np.int8)
    kw = dict(nc_max=5, ne_max=0)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    cfg = gpu_lib.default_cfg(variant, 3, **kw)
    s0 = gpu_lib.Solver(cfg)
    foot0 = s0.solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
    outs = {}
    # (ALIPMPC_CL_GROUPS: contiguous episode groups whose ticks run on streams of their own)
    for cut, tr, grp in (("0", "0", "1"), ("16", "40", "4"), ("3", "0", "3"), ("8", "5", "1"), ("0", "0", "4")):
        monkeypatch.setenv("ALIPMPC_CL_SPLIT_IT", cut)
        monkeypatch.setenv("ALIPMPC_CL_SPLIT_TR", tr)
        monkeypatch.setenv("ALIPMPC_CL_GROUPS", grp)
        outs[cut + "/" + tr + "/" + grp] = gpu_lib.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"],
                                                                           bt["nc"], steps=S, f_cyc=F, kick=kick,
                                                                           seed=3)
    ref = outs.pop("0/0/1")
    assert (ref["status"] == 2).sum() > 0 and (ref["steps_to_goal"] > 0).sum() > 0
    for name, o in outs.items():
        for k in ref:
            assert np.array_equal(o[k], ref[k], equal_nan=True), (name, k)


@pytest.mark.parametrize("program,prec,B", [(1, 1, 6000), (1, 0, 3000), (0, 0, 5000)])
def test_closed_loop_groups_bit_identical(gpu_lib, program, prec, B, monkeypatch):
    """Episode groups that do not divide the ring of work-queue pairs (ALIPMPC_CL_GROUPS = 3, 5, 7) on the programs
    that take instances from the work queue every tick: the lane program, and the wave program on a batch above its
    resident slots.  Each group owns a counter pair, so a group running ticks ahead of another never lands on a pair
    still in use; every output equals the one-group loop's bit for bit."""
    from alipmpc import scenes
    S, F = 2, 40
    bt = scenes.make_batch(B, seed=820 + program + 3 * prec, n_cir=5)
    x0 = bt["x0"].copy()
    x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
    leg = bt["leg"].astype(np.int8)
    kw = dict(nc_max=5, ne_max=0, program=program)
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    cfg = gpu_lib.default_cfg(0, 3, **kw)
    s0 = gpu_lib.Solver(cfg)
    if program == 0:
        assert s0.solve_slots() < B
    foot0 = s0.solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
    outs = {}
    for grp in ("1", "3", "5", "7"):
        monkeypatch.setenv("ALIPMPC_CL_GROUPS", grp)
        outs[grp] = gpu_lib.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F,
                                                    kick=0.05, seed=5)
    ref = outs.pop("1")
    assert (ref["status"] == 2).sum() > 0 and (ref["steps_to_goal"] > 0).sum() > 0
    for name, o in outs.items():
        for k in ref:
            assert np.array_equal(o[k], ref[k], equal_nan=True), (name, k)


@pytest.mark.parametrize("variant,program,prec", [(0, 0, 0), (1, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1), (1, 1, 1),
                                                  (2, 0, 0)])
def test_goal_singular_abort_matches_oracle(gpu_lib, coracle, variant, program, prec):
    """cfg.goal_singular = ABORT: an instance starting ON the goal (x0 = goal, zero warm start: every
    planned state exactly at the goal) ends as the reference's NaN gradient makes IPOPT end it — status -13
    (Invalid_Number_Detected) at iteration 0 with the starting iterate — in every program, precision and variant,
    as in the C oracle (tests/test_oracle.py::test_goal_singular_abort_semantics); the default (ZERO) solves on
    there, and ordinary instances in the same batch are unaffected by the switch (bit-identical outputs)."""
    from alipmpc import scenes
    dd = variant == 2
    N, B = 3, 64
    n = 6 if dd else 15
    bt = _dd_batch(B, seed=930, n_cir=3) if dd else scenes.make_batch(B, seed=930 + variant, n_cir=3)
    x0, goal = bt["x0"].copy(), bt["goal"].copy()
    x0[:8] = 0.0
    goal[:8] = 0.0
    u0 = bt["u0"].copy() if dd else np.tile(x0, (1, N))
    u0[:8] = 0.0
    kw = dict(nc_max=3, ne_max=0)
    if program:
        kw["program"] = gpu_lib.PROGRAM_LANE
    if prec:
        kw["precision"] = gpu_lib.PREC_FP32
    outs = {}
    for gs in (gpu_lib.GOAL_SINGULAR_ZERO, gpu_lib.GOAL_SINGULAR_ABORT):
        s = gpu_lib.Solver(gpu_lib.default_cfg(variant, N, goal_singular=gs, **kw))
        if dd:
            outs[gs] = s.solve(x0, goal, None, bt["cir"], bt["nc"], u0=u0, last_u=bt["last_u"])
        else:
            outs[gs] = s.solve(x0, goal, bt["leg"], bt["cir"], bt["nc"], u0=u0)
    a, z = outs[gpu_lib.GOAL_SINGULAR_ABORT], outs[gpu_lib.GOAL_SINGULAR_ZERO]
    assert (a["status"][:8] == gpu_lib.INVALID_NUMBER_DETECTED).all() and (a["iters"][:8] == 0).all()
    assert np.array_equal(a["u"][:8], np.zeros((8, n)))
    assert (z["status"][:8] != gpu_lib.INVALID_NUMBER_DETECTED).all() and (z["iters"][:8] > 0).all()
    for k in a:
        assert np.array_equal(a[k][8:], z[k][8:], equal_nan=True), k
    co = coracle.default_cfg(variant, N, nc_max=3, ne_max=0, goal_singular=gpu_lib.GOAL_SINGULAR_ABORT)
    if dd:
        r = coracle.solve_batch_dd(co, x0[:8], goal[:8], bt["cir"][:8], bt["nc"][:8], None, None, u0[:8],
                                   bt["last_u"][:8])
    else:
        r = coracle.solve_batch(co, x0[:8], goal[:8], bt["leg"][:8], bt["cir"][:8], bt["nc"][:8], None, None, u0[:8])
    assert np.array_equal(r["status"], a["status"][:8]) and np.array_equal(r["u"], a["u"][:8])


@pytest.mark.parametrize("variant,kick,program,prec", [(0, 0.0, 0, 0), (1, 0.05, 0, 0), (0, 0.05, 1, 0), (0, 0.05, 1, 1)])
def test_closed_loop_same_inputs_match_oracle(gpu_lib, coracle, variant, kick, program, prec):
    """The closed loop of test_closed_loop_matches_oracle driven from the host (oracle.closed_loop_batch's driver),
    every tick's solve sent to the program AND to the C oracle (at the program's tolerances) on the same inputs: the
    kernel's own agreement with the oracle, with no drift of two loops in it.  fp64: the same status on >= 99.5 % of
    the solves, iteration counts within one on >= 99.9 %, footholds within 1e-6 on >= 99.5 % of the solves that
    converged in the same iterations on both sides.  fp32 (against the oracle at tol 1e-4): statuses on >= 97 %,
    footholds within 1e-3 on >= 99 % of the solves both converged."""
    from alipmpc import scenes
    B, S, F = 48, 4, 40
    bt = scenes.make_batch(B, seed=520 + variant + int(kick * 100), n_cir=5)
    x0 = bt["x0"].copy()
    x0[:12, 0:2] = bt["goal"][:12] - (np.array([1.0, 0.8]) if variant == 1 else np.array([0.6, 0.5]))
    leg = bt["leg"].astype(np.int8)
    co = coracle.default_cfg(variant, 3, nc_max=5, ne_max=0)
    foot0 = coracle.solve_batch(co, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None,
                                np.tile(x0, (1, 3)))["foot"][:, 0:2]
    kw = dict(precision=gpu_lib.PREC_FP32) if prec else {}
    s = gpu_lib.Solver(gpu_lib.default_cfg(variant, 3, nc_max=5, ne_max=0, program=program, **kw))
    cc = coracle.default_cfg(variant, 3, nc_max=5, ne_max=0, tol=s.cfg.tol, acceptable_tol=s.cfg.acceptable_tol)
    orig = coracle.solve_batch
    rec = {k: [] for k in ("gst", "git", "ost", "oit", "ferr")}

    def solve(cfg, x0_, goal, leg_, cir, nc, elp, ne, u0, nthreads=1):
        r = s.solve(x0_, goal, leg_, cir, nc, u0=u0)
        ro = orig(cc, x0_, goal, leg_, cir, nc, None, None, u0, nthreads=8)
        for k, v in (("gst", r["status"]), ("git", r["iters"]), ("ost", ro["status"]), ("oit", ro["iters"]),
                     ("ferr", np.abs(r["foot"] - ro["foot"]).max(-1))):
            rec[k].append(v)
        return ro
    coracle.solve_batch = solve
    try:
        coracle.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, kick=kick,
                                  seed=7)
    finally:
        coracle.solve_batch = orig
    R = {k: np.concatenate(v) for k, v in rec.items()}
    same_st = R["gst"] == R["ost"]
    it1 = np.abs(R["git"] - R["oit"]) <= 1
    conv = (R["gst"] == 0) & (R["ost"] == 0)
    same_path = conv & (R["git"] == R["oit"])
    tag = f"{variant}_{kick}_{program}_{prec}"
    _artifact(f"closed_loop_same_inputs_{tag}.json",
              {"solves": int(len(same_st)), "status_agree": float(same_st.mean()), "iters_within_1": float(it1.mean()),
               "both_converged": int(conv.sum()), "foot_le_1e-6_same_iters": float((R["ferr"][same_path] <= 1e-6).mean()),
               "foot_le_1e-3_converged": float((R["ferr"][conv] <= 1e-3).mean()),
               "status_pairs": {f"{g}/{o}": int(((R["gst"] == g) & (R["ost"] == o)).sum())
                                for g, o in sorted(set(zip(R["gst"].tolist(), R["ost"].tolist())))}})
    if prec:
        assert same_st.mean() >= 0.97, same_st.mean()
        assert (R["ferr"][conv] <= 1e-3).mean() >= 0.99, (R["ferr"][conv] <= 1e-3).mean()
    else:
        assert same_st.mean() >= 0.995, same_st.mean()
        assert it1.mean() >= 0.999, it1.mean()
        assert (R["ferr"][same_path] <= 1e-6).mean() >= 0.995, (R["ferr"][same_path] <= 1e-6).mean()
