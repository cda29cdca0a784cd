"""Synthetic scenario batches — the distribution of the reference's random obstacle fields.

Obstacles follow rand_obs.random_circle / random_obs (rand_obs.py:31-72): centres ~ U[0, 8.5]^2 rounded
to 0.01, radii ~ U[0.35, 1.0] rounded to 0.01, rejected when any pair is closer than r1 + r2 + 2*0.8
(the seed circles (10,10,0.3) and (0,0,1.0) take part in the rejection and are dropped afterwards);
in 'mix' scenes every second obstacle becomes an ellipse [xc, yc, a=r, b~U[a/2,a], phi=deg(U{0..180})].
Obstacles are inflated by safe_dis = 0.4 as the driver does (main_sim_mpc.py:11,14).
Initial states: position ~ U[0,10]^2 outside every inflated obstacle by 0.2, heading towards the goal
(10, 10) + N(0, 0.2), body velocity vx ~ U[0.45, 0.75], vy = -leg * U[0.17, 0.33] rotated to world,
leg ~ U{-1, +1}, warm start u0 = [x0]*N (logger_mpc.py:327-328).
Unlike the reference's unbounded rejection loop, placement gives up after `max_tries` draws per obstacle
and relaxes the spacing rule (needed for 10-obstacle scenes, which rarely fit the reference's rule).
"""
import numpy as np

SAFE_DIS = 0.4
GOAL = (10.0, 10.0)


def random_circles(rng, num, margin=8.5, radius=1.0, safe_dis=0.8, max_tries=2000):
    placed = [(10.0, 10.0, 0.3), (0.0, 0.0, 1.0)]
    tries = 0
    spacing = safe_dis
    while len(placed) < num + 2:
        x = round(margin * rng.random(), 2)
        y = round(margin * rng.random(), 2)
        r = round((radius - 0.35) * rng.random() + 0.35, 2)
        ok = all((x - c[0]) ** 2 + (y - c[1]) ** 2 - (r + c[2] + 2 * spacing) ** 2 >= 0 for c in placed)
        if ok:
            placed.append((x, y, r))
            tries = 0
        else:
            tries += 1
            if tries > max_tries:
                spacing *= 0.5
                tries = 0
    return np.array(placed[2:], dtype=np.float64)


def to_mix(rng, cir):
    cl, el = [], []
    for i, c in enumerate(cir):
        if i % 2 == 0:
            cl.append(c)
        else:
            a = c[2]
            b = round((a / 2) * rng.random() + a / 2, 2)
            phi = round(int(rng.integers(0, 181)) * np.pi / 180, 2)
            el.append([c[0], c[1], a, b, phi])
    return np.array(cl, np.float64).reshape(-1, 3), np.array(el, np.float64).reshape(-1, 5)


def sample_state(rng, cir_safe, elp_safe, goal=GOAL, clearance=0.2):
    while True:
        pos = rng.uniform(0.0, 10.0, 2)
        ok = np.hypot(pos[0] - goal[0], pos[1] - goal[1]) > 0.5
        for c in cir_safe:
            ok &= np.hypot(*(pos - c[:2])) >= c[2] + clearance
        for e in elp_safe:
            ok &= np.hypot(*(pos - e[:2])) >= max(e[2], e[3]) + clearance
        if ok:
            break
    leg = int(rng.choice([-1, 1]))
    th = np.arctan2(goal[1] - pos[1], goal[0] - pos[0]) + rng.normal(0.0, 0.2)
    vbx = rng.uniform(0.45, 0.75)
    vby = -leg * rng.uniform(0.17, 0.33)
    c, s = np.cos(th), np.sin(th)
    return np.array([pos[0], pos[1], c * vbx - s * vby, s * vbx + c * vby, th]), leg


def make_batch(B, seed=0, n_cir=5, n_elp=0, N=3, nc_max=None, ne_max=None, scenes_per_batch=None,
               in_range=False):
    """Build a batch of B instances.  n_elp > 0 uses 'mix' scenes with n_cir + n_elp obstacles.
    scenes_per_batch: number of distinct obstacle fields (instances cycle over them; default B).
    in_range: place every obstacle within the 4 m detection range of x0 (fixed m for timing)."""
    rng = np.random.default_rng(seed)
    nc_max = n_cir if nc_max is None else nc_max
    ne_max = n_elp if ne_max is None else ne_max
    S = B if scenes_per_batch is None else scenes_per_batch
    x0 = np.zeros((B, 5))
    leg = np.zeros(B, np.int8)
    cir = np.zeros((B, nc_max, 3))
    elp = np.zeros((B, max(ne_max, 0), 5))
    nc = np.zeros(B, np.int32)
    ne = np.zeros(B, np.int32)
    scenes = []
    for _ in range(S):
        tot = n_cir + n_elp
        c = random_circles(rng, tot)
        if n_elp > 0:
            cc, ee = to_mix(rng, c)
        else:
            cc, ee = c, np.zeros((0, 5))
        cs = cc + np.array([0, 0, SAFE_DIS]) if len(cc) else cc
        es = ee + np.array([0, 0, SAFE_DIS, SAFE_DIS, 0]) if len(ee) else ee
        scenes.append((cs, es))
    for b in range(B):
        cs, es = scenes[b % S]
        st, lg = sample_state(rng, cs, es)
        if in_range:
            # shift the scene so its centroid sits ~2 m ahead of the robot
            cen = np.mean(np.concatenate([cs[:, :2], es[:, :2]]) if len(es) else cs[:, :2], axis=0)
            d = st[:2] + 2.0 * np.array([np.cos(st[4]), np.sin(st[4])]) - cen
            cs = cs.copy(); cs[:, :2] += d
            es = es.copy()
            if len(es):
                es[:, :2] += d
        x0[b] = st
        leg[b] = lg
        nc[b] = min(len(cs), nc_max)
        ne[b] = min(len(es), ne_max)
        cir[b, :nc[b]] = np.asarray(cs, float).reshape(-1, 3)[:nc[b]]
        if ne_max:
            elp[b, :ne[b]] = np.asarray(es, float).reshape(-1, 5)[:ne[b]]
    u0 = np.tile(x0, (1, N))
    goal = np.tile(np.array(GOAL), (B, 1))
    return dict(x0=x0, goal=goal, leg=leg, cir=cir, nc=nc, elp=elp if ne_max else None, ne=ne if ne_max else None,
                u0=u0)


def make_batch_vec(B, seed=0, n_cir=5, n_elp=0, N=3, fields=None, max_rounds=4000):
    """Same distribution as make_batch, vectorised over instances, with `fields` distinct obstacle fields
    (default: one PER INSTANCE — the Monte-Carlo sweep of BASELINE cfg5, 1M randomized scenes; instance b
    uses field b % fields).  Every round draws candidates for each unfinished field and accepts the first
    one that passes the same spacing rule (halved after 2000 consecutive rejections, as random_circles);
    initial states are rejection-sampled per instance the same way.  Not stream-identical to make_batch
    (different draw order), distribution-identical."""
    rng = np.random.default_rng(seed)
    tot = n_cir + n_elp
    K = tot + 2
    F = B if fields is None else max(1, min(int(fields), B))
    B_inst, B = B, F
    obs = np.zeros((B, K, 3))
    obs[:, 0] = (10.0, 10.0, 0.3)
    obs[:, 1] = (0.0, 0.0, 1.0)
    cnt = np.full(B, 2)
    spacing = np.full(B, 0.8)
    tries = np.zeros(B, np.int64)
    C = 32   # candidates per field and round; the first acceptable one is taken (= sequential rejection)
    for _ in range(max_rounds * max(tot, 1)):
        todo = np.nonzero(cnt < K)[0]
        if todo.size == 0:
            break
        x = np.round(8.5 * rng.random((todo.size, C)), 2)
        y = np.round(8.5 * rng.random((todo.size, C)), 2)
        r = np.round(0.65 * rng.random((todo.size, C)) + 0.35, 2)
        o = obs[todo]
        slot = np.arange(K)[None, None, :] < cnt[todo, None, None]
        d = (x[:, :, None] - o[:, None, :, 0]) ** 2 + (y[:, :, None] - o[:, None, :, 1]) ** 2 - \
            (r[:, :, None] + o[:, None, :, 2] + 2 * spacing[todo, None, None]) ** 2
        okc = np.all((d >= 0) | ~slot, axis=2)                  # (todo, C)
        first = np.argmax(okc, axis=1)
        anyok = okc[np.arange(todo.size), first]
        # the 2000-rejection relaxation applies within the candidate sequence too
        nrej = np.where(anyok, first, C)
        over = tries[todo] + nrej > 2000
        ok = anyok & ~over
        acc = todo[ok]
        obs[acc, cnt[acc]] = np.stack([x[ok, first[ok]], y[ok, first[ok]], r[ok, first[ok]]], axis=1)
        cnt[acc] += 1
        tries[acc] = 0
        rej = todo[~ok]
        tries[rej] += np.minimum(nrej[~ok], 2001 - tries[rej])
        relax = rej[tries[rej] > 2000]
        spacing[relax] *= 0.5
        tries[relax] = 0
    assert np.all(cnt == K), "obstacle placement did not finish"
    obs = obs[:, 2:]
    if n_elp > 0:   # to_mix: every second obstacle becomes an ellipse
        ci = np.arange(0, tot, 2)
        ei = np.arange(1, tot, 2)
        cir = obs[:, ci]
        a = obs[:, ei, 2]
        b = np.round((a / 2) * rng.random(a.shape) + a / 2, 2)
        phi = np.round(rng.integers(0, 181, a.shape) * np.pi / 180, 2)
        elp = np.concatenate([obs[:, ei, :2], a[..., None], b[..., None], phi[..., None]], axis=2)
        elp = elp + np.array([0, 0, SAFE_DIS, SAFE_DIS, 0])
    else:
        cir, elp = obs, np.zeros((B, 0, 5))
    cir = cir + np.array([0, 0, SAFE_DIS])
    if B_inst != F:   # instance b -> field b % F
        idx = np.arange(B_inst) % F
        cir, elp, B = cir[idx], elp[idx], B_inst
    # initial states outside every inflated obstacle (+0.2) and > 0.5 from the goal
    pos = np.zeros((B, 2))
    todo = np.arange(B)
    while todo.size:
        p = rng.uniform(0.0, 10.0, (todo.size, 2))
        ok = np.hypot(p[:, 0] - GOAL[0], p[:, 1] - GOAL[1]) > 0.5
        ok &= np.all(np.hypot(p[:, None, 0] - cir[todo, :, 0], p[:, None, 1] - cir[todo, :, 1]) >=
                     cir[todo, :, 2] + 0.2, axis=1)
        if elp.shape[1]:
            ok &= np.all(np.hypot(p[:, None, 0] - elp[todo, :, 0], p[:, None, 1] - elp[todo, :, 1]) >=
                         np.maximum(elp[todo, :, 2], elp[todo, :, 3]) + 0.2, axis=1)
        pos[todo[ok]] = p[ok]
        todo = todo[~ok]
    leg = rng.choice(np.array([-1, 1], np.int8), B)
    th = np.arctan2(GOAL[1] - pos[:, 1], GOAL[0] - pos[:, 0]) + rng.normal(0.0, 0.2, B)
    vbx = rng.uniform(0.45, 0.75, B)
    vby = -leg * rng.uniform(0.17, 0.33, B)
    c, s = np.cos(th), np.sin(th)
    x0 = np.stack([pos[:, 0], pos[:, 1], c * vbx - s * vby, s * vbx + c * vby, th], axis=1)
    return dict(x0=x0, goal=np.tile(np.array(GOAL), (B, 1)), leg=leg,
                cir=np.ascontiguousarray(cir), nc=np.full(B, cir.shape[1], np.int32),
                elp=np.ascontiguousarray(elp) if n_elp else None,
                ne=np.full(B, elp.shape[1], np.int32) if n_elp else None,
                u0=np.tile(x0, (1, N)))
