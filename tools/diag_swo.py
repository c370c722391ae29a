"""Diagnostic: SPH with and without the spatial work order vs the oracle, hex of mismatches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rust-particle-system_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
import rps_amd as rps  # noqa: E402
from helpers import copy_soa  # noqa: E402


def blob(n, seed, spread):
    g = np.random.default_rng(seed)
    return dict(x=np.clip(g.normal(0, spread, n), -955, 955).astype(np.float32),
                y=np.clip(g.normal(0, spread * 0.6, n), -535, 535).astype(np.float32),
                vx=g.normal(0, 30, n).astype(np.float32), vy=g.normal(0, 30, n).astype(np.float32))


def run(swo, n, frames, soa, cfg):
    os.environ["RPS_SPH_SWO"] = swo
    out = []
    with rps.Context(n, rps.MODE_SPH) as ctx:
        ctx.set_config(cfg, rps.make_ext(shader_delay=0))
        ctx.upload_soa(soa)
        for f in range(frames):
            ctx.step(1)
            out.append(dict(pred=ctx.read_debug(rps.DEBUG_PREDICTED).copy(), dens=ctx.read_debug(rps.DEBUG_DENSITIES).copy(),
                            lookup=ctx.read_debug(rps.DEBUG_SPATIAL_LOOKUP).copy(), **ctx.download_soa()))
    return out


n = 50000
cfg = rps.default_particle_config(n, gravity=100.0)
soa = blob(n, n + 1, max(20.0, np.sqrt(n) * 1.2))
a = run("0", n, 3, soa, cfg)
b = a
st = orc.SphState(n)
ref = copy_soa(soa)
for f in range(3):
    st.grid(cfg, ref)
    st.pre(cfg, ref)
    o = dict(pred=st.pred.copy(), dens=st.dens.copy())
    st.sim(cfg, ref)
    o.update(copy_soa(ref))
    for k in ("pred", "dens", "x", "y", "vx", "vy"):
        ia = a[f][k].view(np.uint32).reshape(-1)
        ib = b[f][k].view(np.uint32).reshape(-1)
        io = o[k].view(np.uint32).reshape(-1)
        bad_ab = np.nonzero(ia != ib)[0]
        bad_ao = np.nonzero(ia != io)[0]
        print(f"frame {f} {k}: off!=on {len(bad_ab)}  off!=oracle {len(bad_ao)}  nan(off) {np.isnan(a[f][k]).sum()}")
        for j in list(bad_ab[:4]) + list(bad_ao[:4]):
            print(f"   idx {j}: off {ia[j]:08x} on {ib[j]:08x} oracle {io[j]:08x}")
        if k == "dens" and len(bad_ao):
            la = a[f]["lookup"].reshape(-1, 2)
            for j in bad_ao[:4]:
                i = j // 2
                slots = np.nonzero(la[:, 1] == i)[0]
                print(f"   particle {i}: slots {slots[:10]} keys {la[slots, 0][:10]} pred {a[f]['pred'][i]} "
                      f"oracle slots {np.nonzero(st.lookup.reshape(-1, 2)[:, 1] == i)[0][:10]}")
    la = a[f]["lookup"].reshape(-1, 2)
    print("lookup equal:", np.array_equal(la, b[f]["lookup"].reshape(-1, 2)))
    # slots referencing the first mismatching particle
    bad = np.nonzero(a[f]["dens"].view(np.uint32).reshape(-1) != b[f]["dens"].view(np.uint32).reshape(-1))[0]
    if len(bad):
        i = bad[0] // 2
        slots = np.nonzero(la[:, 1] == i)[0]
        print(f"   particle {i}: slots {slots[:10]} (N={n}) keys {la[slots, 0][:10]}")
