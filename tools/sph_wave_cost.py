"""Per-wave scan cost of the SPH density / sim passes at a given size (diagnosis of the
non-power-of-two slowdown, VERDICT r03 "What's weak" 4).

Runs the bench's SPH workload for F frames on the GPU through rps_amd, reads the frame's
lookup and predicted positions (rps_read_debug), and recomputes on the host, for every slot t
of the P-slot work mapping (64 consecutive slots per wave): the entries of its particle's nine
runs (the reference's scan, wgsl:223-254), how many are within the radius, and whether the
slot owns its particle (lowest slot holding it; repeats return at once).  A wave costs the
longest scan among its live lanes, so the sum over waves of that maximum, against the sum of
the lanes' own costs, is how much of the kernel the long scans serialise.

    python tools/sph_wave_cost.py FRAMES N [N ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rust-particle-system_amd", "python"))
import numpy as np  # noqa: E402
import rps_amd as rps  # noqa: E402


def f2i(v):
    """i32(f32): truncation, saturating, NaN -> 0 (WGSL conversion, wgsl:121-130)."""
    v = np.asarray(v, np.float64)
    out = np.where(np.isnan(v), 0.0, np.clip(np.trunc(v), -2147483648.0, 2147483647.0))
    return out.astype(np.int64).astype(np.int32)


def keys_of(cx, cy, n):
    h = (cx.astype(np.uint32).astype(np.uint64) * 15823 + cy.astype(np.uint32).astype(np.uint64) * 9737333) & 0xFFFFFFFF
    return (h % n).astype(np.int64)


OFFS = [(-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 0), (0, 1), (1, -1), (1, 0), (1, 1)]


def analyse(n, frames):
    scale = max(1.0, (n / 50000) ** 0.5)
    cfg = rps.default_particle_config(n, screen_bounds=rps.screen_bounds_for(1920.0 * scale, 1080.0 * scale))
    parts = rps.setup_particles_scatter(cfg, n, seed=1)
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload(parts)
        ctx.step(frames)
        ctx.sync()
        lk = ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP).reshape(-1, 2)
        pred = ctx.read_debug(rps.DEBUG_PREDICTED).reshape(-1, 2)
    P = lk.shape[0]
    keys, idx = lk[:, 0].astype(np.int64), lk[:, 1].astype(np.int64)
    kn = keys[:n]
    r = np.float32(cfg.smoothing_radius)
    sb = list(cfg.screen_bounds)
    px, py = pred[idx, 0], pred[idx, 1]  # slot t's particle's predicted position
    cx = f2i((px + np.float32(sb[1])) / r)
    cy = f2i((py + np.float32(sb[3])) / r)
    total = np.zeros(P, np.int64)
    within = np.zeros(P, np.int64)
    BIG = 1 << 40
    first_nan = np.full(P, BIG, np.int64)  # flat index of the first entry whose d^2 is NaN
    within_before_nan = np.zeros(P, np.int64)
    r2 = np.float32(r * r)
    for ox, oy in OFFS:
        k = keys_of((cx + ox).astype(np.int32), (cy + oy).astype(np.int32), n)
        s = np.searchsorted(kn, k, "left")
        e = np.searchsorted(kn, k, "right")
        ln = e - s
        # within-radius entries of this run, slot by slot (runs are short except key 0's)
        rep = np.repeat(np.arange(P), ln)
        first = np.cumsum(ln) - ln  # flat index of each slot's first entry
        loc = np.arange(ln.sum()) - np.repeat(first, ln)  # entry's index within its run
        ent = np.repeat(s, ln) + loc
        q = pred[idx[ent]]
        dx = q[:, 0] - px[rep]
        dy = q[:, 1] - py[rep]
        sq = dx * dx + dy * dy
        win = ~(sq > r2)
        flat = total[rep] + loc
        isn = np.isnan(sq)
        fn = np.full(P, BIG, np.int64)
        np.minimum.at(fn, rep[isn], flat[isn])
        first_nan = np.minimum(first_nan, fn)
        within += np.bincount(rep, weights=win.astype(np.float64), minlength=P).astype(np.int64)
        wb = win & (flat < first_nan[rep])
        within_before_nan += np.bincount(rep, weights=wb.astype(np.float64), minlength=P).astype(np.int64)
        total += ln
    owner = np.full(n, P, np.int64)
    np.minimum.at(owner, idx, np.arange(P))
    live_sim = owner[idx] == np.arange(P)
    live_den = live_sim | (np.arange(P) < n)
    nan = int(np.isnan(pred[:, 0]).sum())
    stop = np.minimum(total, first_nan + 1)  # a scan stops at its first NaN entry
    own_fin = np.isfinite(px) & np.isfinite(py)
    den_cost = np.where(own_fin, stop, total)  # own non-finite positions scan everything
    sim_cost = np.where(total <= 128, within_before_nan, stop)  # masked lanes pay their set bits
    out = {"n": n, "P": P, "frames": frames, "nan": nan, "key0_run": int((kn == 0).sum()),
           "own_nonfinite_slots": int((~own_fin).sum())}
    for name, cost, live in (("density_full", total, live_den), ("density", den_cost, live_den),
                             ("density_allstop", stop, live_den), ("sim_nostop", np.where(total <= 128, within, total), live_sim),
                             ("sim", sim_cost, live_sim)):
        c = np.where(live, cost, 0).reshape(-1, 64)
        lanes = live.reshape(-1, 64).sum(1)
        wmax = c.max(1)
        out[name] = {"lane_sum": int(c.sum()), "wave_max_sum": int(wmax.sum()),
                     "efficiency": float(c.sum() / max(1, wmax.sum() * 64)),
                     "live_lanes_per_wave": float(lanes.mean()),
                     "waves_over_128": int((wmax > 128).sum()), "max_wave": int(wmax.max()),
                     "top_waves": [int(v) for v in np.sort(wmax)[-8:]],
                     "cost_in_top_1pct_waves": float(np.sort(wmax)[-max(1, len(wmax) // 100):].sum() / wmax.sum())}
    out["lanes_over_128"] = int(((total > 128) & live_sim).sum())
    long_ = (total > 128) & own_fin  # the long-scan queue (rps_kernels.hip kLongScan)
    out["long_queue_density"] = int((long_ & live_den).sum())
    out["long_queue_sim_owners"] = int((long_ & live_sim).sum())
    short_sim = np.where(live_sim & ~long_, sim_cost, 0).reshape(-1, 64).max(1)
    short_den = np.where(live_den & ~long_, den_cost, 0).reshape(-1, 64).max(1)
    out["short_wave_max"] = {"sim_max": int(short_sim.max()), "sim_p99": float(np.percentile(short_sim, 99)),
                             "sim_mean": float(short_sim.mean()), "den_max": int(short_den.max()),
                             "den_p99": float(np.percentile(short_den, 99)), "den_mean": float(short_den.mean())}
    # the longest sim lanes: what they scan
    top = np.argsort(np.where(live_sim, sim_cost, -1))[-6:]
    out["top_sim_lanes"] = [{"slot": int(t), "particle": int(idx[t]), "cost": int(sim_cost[t]), "total": int(total[t]),
                             "first_nan": int(min(first_nan[t], BIG - 1)), "within": int(within[t]),
                             "own_finite": bool(own_fin[t]), "cell": [int(cx[t]), int(cy[t])],
                             "runs": [int(np.searchsorted(kn, kk, "right") - np.searchsorted(kn, kk, "left"))
                                      for kk in (keys_of(np.int32(cx[t] + ox), np.int32(cy[t] + oy), n) for ox, oy in OFFS)],
                             "keys": [int(keys_of(np.int32(cx[t] + ox), np.int32(cy[t] + oy), n)) for ox, oy in OFFS]}
                            for t in top]
    k0 = np.nonzero(kn == 0)[0]
    k0fin = np.isfinite(pred[idx[k0], 0])
    out["key0_finite_positions"] = [int(v) for v in np.nonzero(k0fin)[0][:20]]
    return out


if __name__ == "__main__":
    import json

    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    for n in [int(a) for a in sys.argv[2:]] or [50000, 65536]:
        print(json.dumps(analyse(n, frames)), flush=True)
