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
        cir[b, :nc[b]] = cs[:nc[b]]
        if ne_max:
            elp[b, :ne[b]] = es[:ne[b]]
    u0 = np.tile(x0, (1, N))
    goal = np.tile(np.array(GOAL), (B, 1))
    return dict(x0=x0, goal=goal, leg=leg, cir=cir, nc=nc, elp=elp if ne_max else None, ne=ne if ne_max else None,
                u0=u0)
