#!/usr/bin/env python3
"""Diagnostic: per-wave phase timeline of k_brick from a GLS_STAMPS build.

GLS_AMD_LIB=dealii-ns-gls_amd/lib/var/stamps.so python scripts/timeline.py [--nref 2]
Prints, over all waves of one vmult: the mean duration of every phase, the
spread of wave start/end times, and the per-CU concurrency."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-ns-gls_amd", "python"))
import glsinputs as gi  # noqa: E402
import glsmesh as gm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nref", type=int, default=2)
    ap.add_argument("--brick", default=None)
    ap.add_argument("--out", default="gpurun_out/timeline.json")
    args = ap.parse_args()
    import torch
    import glsamd
    d = gm.read_deck(os.path.join(gm.DECK_DIR, "input_hoffmann_3D_Re3900.json"))
    mesh = d.mesh(args.nref)
    vel, p, slip = d.boundary_descriptor()
    cmask = mesh.constraint_mask(vel, p, slip)
    params, weights = d.operator_parameters(2.5e-4)
    brick = tuple(int(x) for x in args.brick.split(",")) if args.brick else None
    op = glsamd.NavierStokesOperator(mesh, cmask, "f64", brick=brick)
    op.set_parameters(**params)
    u_star = gi.linearization_point(mesh.n_nodes, mesh.dim, d.u_max)
    op.set_linearization_point(u_star)
    op.set_previous_solution(gi.history(u_star, params["order"]), weights)
    src = op._dev(gi.src_vector(mesh.n_dofs))
    dst = op.initialize_dof_vector()
    for _ in range(10):
        op.vmult(dst, src)
    torch.cuda.synchronize()
    op.vmult(dst, src)
    torch.cuda.synchronize()
    L = glsamd.lib()
    L.gls_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
    n = 16384 * 4 * 8
    buf = np.zeros(n, dtype=np.uint64)
    rc = L.gls_debug_stamps(buf.ctypes.data, buf.nbytes)
    assert rc == 0, L.gls_last_error()
    nb = op.n_cells // 16 if brick is None else op.n_cells // int(np.prod(brick))
    st = buf.reshape(-1, 4, 8)[:nb].astype(np.float64)
    t0 = st[:, :, 0][st[:, :, 0] > 0].min()
    t = np.where(st > 0, (st - t0) * 10.0 / 1000.0, np.nan)  # us (100 MHz clock)
    names = {0: "top", 1: "prologue done", 2: "r0 evaluate done", 3: "r0 physics done",
             4: "r1 evaluate done", 5: "r1 physics done", 6: "rounds done", 7: "written"}
    res = {"n_bricks": int(nb), "phases_us": {}}
    order = [0, 1, 2, 3, 4, 5, 6, 7]
    for a, b in zip(order[:-1], order[1:]):
        dd = t[:, :, b] - t[:, :, a]
        res["phases_us"][f"{names[a]} -> {names[b]}"] = [float(np.nanmean(dd)),
                                                         float(np.nanpercentile(dd, 90))]
    life = t[:, 0, 7] - t[:, 0, 0]
    res["brick_top_to_rounds_done_us"] = [float(np.nanmean(life)), float(np.nanmin(life)),
                                          float(np.nanmax(life))]
    starts = t[:, 0, 0]
    res["start_quantiles_us"] = [float(np.nanpercentile(starts, q)) for q in (0, 10, 25, 50, 75, 90, 100)]
    ends = t[:, 0, 7]
    res["end_quantiles_us"] = [float(np.nanpercentile(ends, q)) for q in (0, 10, 25, 50, 75, 90, 100)]
    grid = np.linspace(0, np.nanmax(ends), 40)
    conc = [int(np.sum((starts <= g) & (ends > g))) for g in grid]
    res["active_bricks_over_time"] = [[round(float(g), 2), c] for g, c in zip(grid, conc)]
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
