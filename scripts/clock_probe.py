"""Does the headline vmult run slower right after the GPU has been idle?
(GPU box; prints one JSON object.)

  chain_after_idle   30 regions of K vmults back to back, one event pair per
                     region and no host sync between them, started after
                     `idle_s` of GPU idleness: per-step time of each region
  bench_pattern      bench.py's pattern after `idle_s` idle: W warm-up vmults,
                     synchronize, K timed (events), repeated `reps` times
  bench_settled      the same with `settle_ms` of back-to-back vmults before
                     the warm-up
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import glsamd  # noqa: E402
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402

K, W, IDLE_S, REPS, SETTLE_MS = 20, 5, 3.0, 4, 100.0


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
    for _ in range(10):
        op.vmult(dst, src)
    torch.cuda.synchronize()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    out = {"K": K, "W": W, "idle_s": IDLE_S, "settle_ms": SETTLE_MS}
    time.sleep(IDLE_S)
    evs = [ev() for _ in range(31)]
    evs[0].record()
    for r in range(30):
        for _ in range(K):
            op.vmult(dst, src)
        evs[r + 1].record()
    torch.cuda.synchronize()
    out["chain_after_idle_us_per_step"] = [round(evs[r].elapsed_time(evs[r + 1]) * 1e3 / K, 2)
                                           for r in range(30)]

    def pattern(settle, settle_ms=SETTLE_MS):
        res = []
        for _ in range(REPS):
            time.sleep(IDLE_S)
            if settle:
                t0 = time.perf_counter()
                n = 0
                while (time.perf_counter() - t0) * 1e3 < settle_ms:
                    for _ in range(20):
                        op.vmult(dst, src)
                    n += 20
                    torch.cuda.synchronize()
            for _ in range(W):
                op.vmult(dst, src)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0, e1 = ev(), ev()
            e0.record()
            for _ in range(K):
                op.vmult(dst, src)
            e1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            res.append({"wall_us_per_step": round(wall * 1e3 / K, 2),
                        "events_us_per_step": round(e0.elapsed_time(e1) * 1e3 / K, 2)})
        return res

    if len(sys.argv) > 1:
        # settle lengths to compare: bench's pattern after each
        for ms in (float(x) for x in sys.argv[1].split(",")):
            out[f"bench_settled_{int(ms)}ms"] = pattern(ms > 0, ms)
    else:
        out["bench_pattern"] = pattern(False)
        out["bench_settled"] = pattern(True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
