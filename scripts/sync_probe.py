"""Where the fixed cost of a timed region goes (GPU box; one JSON object).

  python scripts/sync_probe.py [auto|spin|yield|blocking]

sets the HIP host-wait mode (hipSetDeviceFlags, before torch creates the
context), then measures on the headline operator:
  sync_idle_us      torch.cuda.synchronize() with nothing in flight
  one_vmult         wall (enqueue + synchronize) vs events of a single vmult
  region            bench.py's pattern after a 200 ms settle: W warm-up,
                    synchronize, opening event, clock, K vmults, closing
                    event, synchronize, clock (wall vs events per step)
"""
import ctypes as C
import json
import os
import sys
import time

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}
MODE = sys.argv[1] if len(sys.argv) > 1 else "auto"
if MODE != "auto":
    hip = C.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(C.c_uint(FLAGS[MODE]))
    if rc != 0:
        raise SystemExit(f"hipSetDeviceFlags({MODE}) failed: {rc}")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

K, W = 20, 5


def main():
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    mesh = d.mesh(d.n_refinements)
    vel, p, slip = d.boundary_descriptor()
    cm = mesh.constraint_mask(vel, p, slip)
    params, w = d.operator_parameters(2.5e-4)
    u = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
    op = glsamd.NavierStokesOperator(mesh, cm, "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u)
    if params["order"] > 0:
        op.set_previous_solution(gi.history(u, params["order"]), w)
    src = op._dev(gi.src_vector(mesh.n_dofs))
    dst = op.initialize_dof_vector()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        for _ in range(20):
            op.vmult(dst, src)
        torch.cuda.synchronize()
    out = {"mode": MODE}
    t = []
    for _ in range(200):
        a = time.perf_counter()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - a)
    out["sync_idle_us"] = float(np.median(t)) * 1e6
    wall, evt = [], []
    for _ in range(50):
        e0, e1 = ev(), ev()
        e0.record()
        torch.cuda.synchronize()
        a = time.perf_counter()
        op.vmult(dst, src)
        e1.record()
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - a)
        evt.append(e0.elapsed_time(e1) * 1e-3)
    out["one_vmult"] = {"wall_us": float(np.median(wall)) * 1e6,
                        "events_us": float(np.median(evt)) * 1e6}
    reg = []
    for _ in range(8):
        for _ in range(W):
            op.vmult(dst, src)
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record()
        a = time.perf_counter()
        for _ in range(K):
            op.vmult(dst, src)
        e1.record()
        torch.cuda.synchronize()
        el = time.perf_counter() - a
        reg.append({"wall_us_per_step": round(el * 1e6 / K, 2),
                    "events_us_per_step": round(e0.elapsed_time(e1) * 1e3 / K, 2)})
    out["region"] = reg
    print(json.dumps(out))


if __name__ == "__main__":
    main()
