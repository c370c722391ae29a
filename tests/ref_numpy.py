"""Second, independent restatement of the reference path in numpy float32 (test-only).

Used to cross-check the C oracle (oracle/rps_oracle.c) before the oracle is trusted as the
GPU checker.  numpy float32 arithmetic rounds every operation and never contracts a*b+c,
and np.sqrt / division are correctly rounded, so agreement with the C oracle is bitwise.
Every function cites the WGSL line it restates (assets/compute_shader.wgsl).
"""
import math

import numpy as np

F = np.float32
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Random123 Philox4x32-10 on uint32 arrays / scalars."""
    c0, c1, c2, c3 = (np.asarray(v, np.uint64) for v in (c0, c1, c2, c3))
    k0, k1 = int(k0), int(k1)
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
    return [v.astype(np.uint32) for v in (c0, c1, c2, c3)]


def u01(w):
    return (np.asarray(w, np.uint32) >> np.uint32(8)).astype(F) * F(1.0 / 16777216.0)


SIN_C = [F(-2.50521083854417188e-08), F(2.75573192239858907e-06), F(-1.98412698412698413e-04),
         F(8.33333333333333333e-03), F(-1.66666666666666667e-01)]
COS_C = [F(2.08767569878680990e-09), F(-2.75573192239858907e-07), F(2.48015873015873016e-05),
         F(-1.38888888888888889e-03), F(4.16666666666666667e-02), F(-0.5)]


def sincos_turns(u):
    u = np.asarray(u, F)
    u4 = u * F(4.0)
    q = u4.astype(np.int32)
    f = u4 - q.astype(F)
    th = f * F(1.57079632679489662)
    t2 = th * th
    sp = np.full_like(t2, SIN_C[0])
    for c in SIN_C[1:]:
        sp = sp * t2 + c
    s = th + (th * t2) * sp
    cp = np.full_like(t2, COS_C[0])
    for c in COS_C[1:]:
        cp = cp * t2 + c
    c = F(1.0) + t2 * cp
    q &= 3
    co = np.select([q == 0, q == 1, q == 2], [c, -s, -c], s)
    so = np.select([q == 0, q == 1, q == 2], [s, c, -s], -c)
    return co.astype(F), so.astype(F)


LOG_C = [F(1 / 15), F(1 / 13), F(1 / 11), F(1 / 9), F(1 / 7), F(1 / 5), F(1 / 3)]


def log_unit(u):
    """ln(u), u in (0, 1]: exponent split by bit operations + the atanh series (the oracle's
    orc_log_unit, the device's log_unit)."""
    u = np.asarray(u, F)
    b = u.view(np.uint32)
    e = ((b >> np.uint32(23)) & np.uint32(255)).astype(np.int32) - 127
    m = ((b & np.uint32(0x007FFFFF)) | np.uint32(0x3F800000)).view(F)
    big = m > F(1.41421356)
    m = np.where(big, m * F(0.5), m).astype(F)
    e = np.where(big, e + 1, e)
    s = (m - F(1.0)) / (m + F(1.0))
    s2 = s * s
    p = np.full_like(s2, LOG_C[0])
    for c in LOG_C[1:]:
        p = p * s2 + c
    t = s + s
    lnm = t + t * (s2 * p)
    ef = e.astype(F)
    return (ef * F(6.93145751953125e-01) + (ef * F(1.42860682030941723e-06) + lnm)).astype(F)


def init_scatter(bounds, seed, n, id_offset=0, global_count=None):
    """x, y of the seeded initial scatter (src/main.rs:191-205; the oracle's orc_init_scatter):
    x linear in the global id, y = Box-Muller normal from Philox with the fixed-op log."""
    global_count = global_count or (id_offset + n)
    x_min, x_max, y_min, y_max = (F(v) for v in bounds)
    g = np.arange(id_offset, id_offset + n, dtype=np.uint64)
    t = g.astype(F) / F(global_count)
    x = x_min + t * (x_max - x_min)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    ones = np.full(n, 0xFFFFFFFF, np.uint32)
    w = philox4x32_10(g.astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32), ones, ones, k0, k1)
    u1 = ((np.asarray(w[0], np.uint32) >> np.uint32(8)) + np.uint32(1)).astype(F) * F(1.0 / 16777216.0)
    c, _ = sincos_turns(u01(w[1]))
    with np.errstate(invalid="ignore"):
        z = np.sqrt(F(-2.0) * log_unit(u1)) * c
    yc = (y_min + y_max) / F(2.0)
    sd = (y_max - y_min) * F(0.125)
    y = yc + z * sd
    y = np.where(y < y_min, y_min, y)
    y = np.where(y > y_max, y_max, y).astype(F)
    return x.astype(F), y


def attractor_positions(ext, active_step):
    dt = float(F(ext["dt"]))
    t = float(active_step) * dt
    out = []
    for a in ext["attractors"]:
        ang = float(F(a["angular_velocity"])) * t + float(F(a["phase"]))
        px = F(float(F(a["center"][0])) + float(F(a["orbit_radius"])) * math.cos(ang))
        py = F(float(F(a["center"][1])) + float(F(a["orbit_radius"])) * math.sin(ang))
        s = F(a["softening"])
        out.append((px, py, F(a["strength"]), s * s))
    return out


def inv_sqrt(r2):
    """bit-level guess 0x5f375a86 - (bits >> 1), three f32 Newton steps."""
    r2 = np.asarray(r2, F)
    y = (np.uint32(0x5f375a86) - (r2.view(np.uint32) >> np.uint32(1))).astype(np.uint32).view(F)
    h = F(0.5) * r2
    for _ in range(3):
        t = h * y
        t = t * y
        t = F(1.5) - t
        y = y * t
    return y


def attract(atts, x, y):
    sx = np.zeros_like(x)
    sy = np.zeros_like(y)
    for px, py, st, e2 in atts:
        dx = px - x
        dy = py - y
        r2 = (dx * dx + dy * dy) + e2
        inv = inv_sqrt(r2)
        s = st * ((inv * inv) * inv)
        sx = sx + dx * s
        sy = sy + dy * s
    return sx, sy


def wall(bounds, damp, x, y, vx, vy):
    """check_screen_bounds, wgsl:69-99."""
    x_min, x_max, y_min, y_max = (F(b) for b in bounds)
    damp = F(damp)
    lo = x <= x_min
    hi = (~lo) & (x >= x_max)
    x = np.where(lo, x_min, np.where(hi, x_max, x))
    vx = np.where(lo, np.abs(vx) * damp, np.where(hi, -np.abs(vx) * damp, vx))
    lo = y <= y_min
    hi = (~lo) & (y >= y_max)
    y = np.where(lo, y_min, np.where(hi, y_max, y))
    vy = np.where(lo, np.abs(vy) * damp, np.where(hi, -np.abs(vy) * damp, vy))
    return x.astype(F), y.astype(F), vx.astype(F), vy.astype(F)


def life_steps(life, dt):
    """clamp(ceil(L / dt), 1, 65535) in f32, vectorised."""
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.ceil(np.asarray(life, F) / F(dt)).astype(F)
    out = np.where(q >= F(65535.0), F(65535.0), q)
    out = np.where(q >= F(1.0), out, F(1.0))  # NaN and q < 1 -> 1
    return out.astype(np.uint32)


def exp_from_life(life, clock, dt):
    return ((np.uint32(clock & 0xFFFFFFFF) + life_steps(life, dt) - np.uint32(1)) & np.uint32(0xFFFF)).astype(np.uint16)


def life_from_exp(exp, clock, dt):
    left = (exp.astype(np.uint32) - np.uint32(clock & 0xFFFF)) & np.uint32(0xFFFF)
    return ((left + np.uint32(1)).astype(F) * F(dt)).astype(F)


def stream_step(cfg, ext, soa, active_step, id_offset=0, clock=None):
    """One active stream step; cfg/ext are plain dicts (see tests/test_oracle_semantics.py).
    clock: the step's lifetime clock (default active_step); soa["exp"] (u16) is the lifetime
    state, created from soa["life"] at `clock` when absent."""
    clock = active_step if clock is None else clock
    dt = F(cfg["dt"])
    g = F(cfg["gravity"])
    x, y, vx, vy = (soa[k].copy() for k in ("x", "y", "vx", "vy"))
    atts = attractor_positions(dict(ext, dt=cfg["dt"]), active_step) if ext.get("attractors") else []
    drag = F(ext.get("drag", 0.0))
    drag_f = F(1.0) - drag * dt
    if ext.get("integrator", 0) == 0:
        vx = vx + F(0.0) * dt  # apply_gravity, wgsl:397-400
        vy = vy + (-g) * dt
        if atts:
            ax, ay = attract(atts, x, y)
            vx = vx + ax * dt
            vy = vy + ay * dt
        if drag != 0:
            vx = vx * drag_f
            vy = vy * drag_f
        x = x + vx * dt  # update_particle_positions, wgsl:392-395
        y = y + vy * dt
    else:
        half_dt2 = (F(0.5) * dt) * dt
        half_dt = F(0.5) * dt
        ax0, ay0 = attract(atts, x, y)
        ay0 = ay0 + (-g)
        x1 = (x + vx * dt) + ax0 * half_dt2
        y1 = (y + vy * dt) + ay0 * half_dt2
        ax1, ay1 = attract(atts, x1, y1)
        ay1 = ay1 + (-g)
        vx = vx + (ax0 + ax1) * half_dt
        vy = vy + (ay0 + ay1) * half_dt
        if drag != 0:
            vx = vx * drag_f
            vy = vy * drag_f
        x, y = x1, y1
    x, y, vx, vy = wall(cfg["bounds"], cfg["damping"], x, y, vx, vy)
    out = dict(x=x, y=y, vx=vx, vy=vy)
    if ext.get("lifetime"):
        exp = soa.get("exp")
        exp = exp_from_life(soa["life"], clock, dt) if exp is None else exp.copy()
        re = exp == np.uint16(clock & 0xFFFF)
        idx = np.nonzero(re)[0]
        if len(idx):
            gid = np.uint64(id_offset) + idx.astype(np.uint64)
            seed = int(ext["seed"])
            w = philox4x32_10(gid & MASK, gid >> np.uint64(32), np.uint64(active_step & 0xFFFFFFFF),
                              np.uint64(active_step >> 32), seed & 0xFFFFFFFF, seed >> 32)
            em = ext["emitter"]
            r = F(em["radius"]) * np.sqrt(u01(w[0]))
            c, s = sincos_turns(u01(w[1]))
            x[idx] = F(em["center"][0]) + r * c
            y[idx] = F(em["center"][1]) + r * s
            smin, smax = F(em["speed"][0]), F(em["speed"][1])
            spd = smin + u01(w[3]) * (smax - smin)
            vx[idx] = spd * c
            vy[idx] = spd * s
            lmin, lmax = F(ext["lifetime"][0]), F(ext["lifetime"][1])
            steps = life_steps(lmin + u01(w[2]) * (lmax - lmin), dt)
            exp[idx] = ((np.uint32(clock & 0xFFFFFFFF) + steps) & np.uint32(0xFFFF)).astype(np.uint16)
        out["exp"] = exp
        out["life"] = life_from_exp(exp, clock + 1, dt)
    return out


# ------------------------------------------------------------------------------------
# SPH (pure-Python loops; small N only)
# ------------------------------------------------------------------------------------
def hash_cell(cx, cy):
    return ((cx & 0xFFFFFFFF) * 15823 + (cy & 0xFFFFFFFF) * 9737333) & 0xFFFFFFFF


def f32_to_i32(v):
    v = float(v)
    if v != v:
        return 0
    if v >= 2147483520.0:
        return 2147483647
    if v <= -2147483648.0:
        return -2147483648
    return int(v)  # truncation toward zero


def bitonic_passes(P):
    """(group_width, flip) for each pass of src/particle_buffers.rs:108-138."""
    S = P.bit_length() - 1
    out = []
    for stage in range(S):
        for step in range(stage + 1):
            out.append((1 << (stage - step), step == 0))
    return out


def bitonic_pairs(P, gw, flip):
    gh = 2 * gw - 1
    for i in range(P // 2):
        h = i & (gw - 1)
        left = h + (gh + 1) * (i // gw)
        right = left + (gh - 2 * h if flip else (gh + 1) // 2)
        yield left, right


GRID_OFFSETS = [(-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 0), (0, 1), (1, -1), (1, 0), (1, 1)]


def sph_step(cfg, soa, lookup, active):
    """bin -> sort -> offsets (-> pre -> sim if active) on python lists / float32 arrays.
    lookup: list of [key, idx] of length P (persistent, zero-initialised)."""
    n = len(soa["x"])
    N = cfg["n"]
    r = F(cfg["radius"])
    x_max, y_max = F(cfg["bounds"][1]), F(cfg["bounds"][3])
    offsets = [0xFFFFFFFF] * n
    for i in range(n):  # wgsl:455-468
        cx = f32_to_i32((soa["x"][i] + x_max) / r)
        cy = f32_to_i32((soa["y"][i] + y_max) / r)
        lookup[i] = [hash_cell(cx, cy) % N, i]
    P = len(lookup)
    for gw, flip in bitonic_passes(P):  # wgsl:470-505
        for l, rr in bitonic_pairs(P, gw, flip):
            if lookup[l][0] > lookup[rr][0]:
                lookup[l], lookup[rr] = lookup[rr], lookup[l]
    for i in range(n):  # wgsl:507-525
        prev = lookup[i - 1][0] if i > 0 else 0xFFFFFFFF
        if lookup[i][0] != prev:
            offsets[lookup[i][0]] = i
    if not active:
        return offsets, None, None
    dt = F(cfg["dt"])
    vx = soa["vx"] + F(0.0) * dt
    vy = soa["vy"] + (-F(cfg["gravity"])) * dt
    px = soa["x"] + vx * dt
    py = soa["y"] + vy * dt
    r2 = r * r

    def neighbours(i):
        cx = f32_to_i32((px[i] + x_max) / r)
        cy = f32_to_i32((py[i] + y_max) / r)
        for ox, oy in GRID_OFFSETS:
            key = hash_cell(cx + ox, cy + oy) % N
            j = offsets[key]
            while j < N:
                if lookup[j][0] != key:
                    break
                yield lookup[j][1]
                j += 1

    dn, ndn, vn = F(cfg["norms"][0]), F(cfg["norms"][1]), F(cfg["norms"][2])
    dens = np.zeros((n, 2), F)
    for i in range(n):  # wgsl:207-254
        d = F(0)
        nd = F(0)
        for oi in neighbours(i):
            dx = px[i] - px[oi]
            dy = py[i] - py[oi]
            sq = dx * dx + dy * dy
            if sq > r2:
                continue
            dist = np.sqrt(sq)
            if dist >= r:
                k1 = k2 = F(0)
            else:
                v = r - dist
                k1 = (dn * v) * v
                k2 = ((ndn * v) * v) * v
            d = d + k1
            nd = nd + k2
        dens[i] = (d, nd)
    td, pm, nm = F(cfg["target_density"]), F(cfg["pressure_mult"]), F(cfg["near_mult"])
    nx, ny, nvx, nvy = soa["x"].copy(), soa["y"].copy(), vx.copy(), vy.copy()
    for i in range(n):  # wgsl:435-453
        rho, rhon = dens[i]
        Pp = (rho - td) * pm
        Pn = rhon * nm
        fx = F(0)
        fy = F(0)
        for oi in neighbours(i):
            if oi == i:
                continue
            dx = px[oi] - px[i]
            dy = py[oi] - py[i]
            sq = dx * dx + dy * dy
            if sq > r2:
                continue
            dist = np.sqrt(sq)
            if dist > F(0.0001):
                dirx, diry = dx / dist, dy / dist
            else:
                dirx, diry = F(0), F(1)
            rj, rnj = dens[oi]
            Pj = (rj - td) * pm
            Pnj = rnj * nm
            pt = (Pp / (rho * rho)) + (Pj / (rj * rj))
            npt = (Pn / (rho * rho)) + (Pnj / (rj * rnj))
            if dist >= r:
                dk = ndk = F(0)
            else:
                v = r - dist
                dk = (F(-2.0) * dn) * v
                ndk = ((F(-3.0) * ndn) * v) * v
            fx = fx + (dirx * pt) * dk
            fy = fy + (diry * pt) * dk
            fx = fx + (dirx * npt) * ndk
            fy = fy + (diry * npt) * ndk
        qx = vx[i] + fx * dt
        qy = vy[i] + fy * dt
        wx = F(0)
        wy = F(0)
        for oi in neighbours(i):
            if oi == i:
                continue
            dx = px[i] - px[oi]
            dy = py[i] - py[oi]
            sq = dx * dx + dy * dy
            if sq > r2:
                continue
            dist = np.sqrt(sq)
            if dist >= r:
                k = F(0)
            else:
                v = r * r - dist * dist
                k = ((vn * v) * v) * v
            wx = wx + (vx[oi] - qx) * k
            wy = wy + (vy[oi] - qy) * k
        qx = qx + (wx * F(cfg["visc_strength"])) * dt
        qy = qy + (wy * F(cfg["visc_strength"])) * dt
        ox = soa["x"][i] + qx * dt
        oy = soa["y"][i] + qy * dt
        a, b, c, d2 = wall(cfg["bounds"], cfg["damping"], np.array([ox], F), np.array([oy], F),
                           np.array([qx], F), np.array([qy], F))
        nx[i], ny[i], nvx[i], nvy[i] = a[0], b[0], c[0], d2[0]
    soa.update(x=nx, y=ny, vx=nvx, vy=nvy)
    pred = np.stack([px, py], axis=1).astype(F)
    return offsets, dens, pred
